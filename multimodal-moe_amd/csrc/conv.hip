// Implicit-GEMM convolutions of the RT-DETR body on the bf16 MFMA (gfx950):
// padding (KS - 1) / 2, KS in {1, 3}, stride 1 or (KS = 3) 2, NHWC
// (channels_last) activations and [Cout][KS][KS][Cin] (channels_last) weights.  They replace
// MIOpen for the convolutions that dominate the training step (SURVEY.md 8(f)
// row 1: "the backbone ... dominate images/sec"; the HybridEncoder's
// RepVGG 3x3 / 1x1 pairs and the ResNet 3x3 / 1x1 layers): the reference
// engine trains them inside RTDETR.train (src/models/vision/rtdetr.py:82-94).
//
//   conv_fwd_kernel    Y[p, n] = sum_{tap, c} X[nbr(p, tap), c] W[n, tap, c]
//                      GEMM M = pixels (B H W), N = Cout, K = KS^2 Cin.  The A
//                      tile's rows are the 64-channel slices of each pixel's
//                      neighbour for the K-tile's tap, fetched by LDS-DMA with a
//                      per-row source address (a padding neighbour reads a zero
//                      row), so no im2col buffer exists.  The data gradient
//                      is the same GEMM over dY with W'[c][tap][n] =
//                      W[n][KS^2-1-tap][c]: large problems write W' once
//                      (conv_weight_flip_kernel, K-contiguous image), small
//                      ones read it in place from W as an MN-contiguous
//                      operand image (template flag BT; no extra launch).
//                      Stride 2: the forward's neighbour of output pixel
//                      (y, x) is input (2y + dy, 2x + dx); the data gradient
//                      of input pixel (y, x) for tap (dy, dx) reads dY at
//                      ((y + dy) / 2, (x + dx) / 2) when both are even, else
//                      the zero row -- or, per parity class of the dX pixel
//                      (one launch each, template flag PH), only its 1, 2, 2
//                      or 4 valid taps: the zero-row form's sums without its
//                      4x MFMA work (no scatter, no atomics either way).
//   conv_wgrad_kernel  dW[n, tap, c] = sum_p dY[p, n] X[nbr(p, tap), c]
//                      GEMM M = Cout, N = KS^2 Cin, K = pixels, split over S
//                      slices of the pixels (fp32 partials) and summed in a
//                      fixed order by conv_wgrad_reduce_kernel (deterministic).
// Tiles 128 x 128 x 64, 4 waves (2 x 2), an S-deep LDS-DMA ring (one
// global_load_lds_dwordx4 per lane per 1 KiB, counted vmcnt waits, raw
// s_barrier), K-contiguous operand images (fwd) or MN-contiguous ones read by
// ds_read_b64_tr_b16 (wgrad), v_mfma_f32_16x16x32_bf16.
#include <algorithm>

#include "mfma_lds.h"
#include "moe_common.h"
#include "prof.h"

namespace moe {

// weight-gradient tile: 128 x 128, 64 on a side with 64 channels
static int wg_bm(int N) { return N % 128 == 0 ? 128 : 64; }
static int wg_bn(int C) { return C % 128 == 0 ? 128 : 64; }
// rtdetr_conv_set_tuning knobs (measurement / A-B; 0 or -1 = automatic)
static int g_conv_bm = 0;          // "conv_bm": forward tile rows 64, 128 or 256
static int g_conv_big = 0;         // "conv_big": 1 = the 8-wave 256 x 128 forward / data-gradient tile
static int g_conv_wg_stages = 0;   // "conv_wg_stages": weight-gradient ring depth 2..4
static int g_conv_wg_splits = 0;   // "conv_wg_splits": weight-gradient pixel slices
static int g_conv_dgrad_flip = -1; // "conv_dgrad_flip": 1 = always write W', 0 = always read in place
static int g_conv_dgrad_phase = 1; // "conv_dgrad_phase": 0 = stride-2 data gradient over all 9 taps (zero rows; A/B)
static int g_conv_areg = 0;        // "conv_areg": 1 = forward / data-gradient A operand in registers (AR)
static int g_conv_halo = -1;       // "conv_halo": 3x3 stride-1 forward / data gradient on conv3x3_halo_kernel:
                                   // 0 = never, 1 = BM 256 (8 waves), 2 = BM 128 (4 waves) where eligible,
                                   // -1 = automatic
static int g_conv_8ph = -1;        // "conv_8ph": the 256 x 256 eight-phase kernel (conv_8ph_kernel): 0 never,
                                   // 1 wherever it applies, -1 automatic (3x3, >= 256 tiles)
static int g_conv_k32 = -1;        // "conv_k32": 1-3 = forward / data-gradient 32-deep K-tiles, ring depth 2-4;
                                   // 0 = never; -1 = automatic (k32_auto)

struct ConvArgs {
  const uint16_t* x;     // [B Hs Ws, C] (fwd: X; dgrad: dY)
  const uint16_t* w;     // [N][KS][KS][C] (fwd: W; dgrad: W')
  uint16_t* y;           // [B H W, N]
  const uint16_t* zero;  // >= 256 zero bytes (padding rows)
  int B, H, W, C, N;     // H, W: this GEMM's output pixels (fwd: Y, dgrad: dX)
  int P;                 // B H W
  int mt_n;              // M tiles
  int Hs, Ws;            // the source image x (fwd: X, dgrad: dY)
  int st, sh;            // neighbour of (y, x) for tap (dy, dx): ((st y + dy) >> sh, (st x + dx) >> sh), valid
                         // only when sh == 0 or both are even (fwd: st = stride, sh = 0; dgrad: st = 1,
                         // sh = stride / 2)
  // fused epilogue on the bf16 result v (each NULL / 0 = off), in this order:
  //   v = act( (v + resid[p][n]) + bias[n] ),  then v = 0 where mask[p][n] <= 0
  // (the arithmetic of rtdetr_bias_act_nhwc / rtdetr_add_bias_relu_nhwc and of
  // a ReLU backward on the data gradient, so fused and separate agree bitwise);
  // resid_post (the evaluation forward's folded RepVgg block + CSP shortcut):
  //   v = bf16( bf16(act(v + bias[n])) + resid[p][n] )  -- torch's SiLU then add
  const float* bias;
  const uint16_t* resid;
  const uint16_t* mask;
  int relu;              // act: 0 none, 1 ReLU, 2 SiLU
  // PH (stride-2 data gradient by parity class): this launch's output pixels
  // are dX's (b, 2a + ry, 2c + rx), a < H, c < W; dX is [B, Hd, Wd]; the
  // class's taps are ky' in {1} (ry = 0) or {0, 2} (ry = 1) (kx' likewise),
  // reading dY at (a + (ky' == 2), c + (kx' == 2))
  int ry, rx, Hd, Wd;
  // forward only (rtdetr_conv_fwd_stats): per-tile column sums of the stored
  // bf16 output and of its square, stats[(m0 / BM) * 2 + {0, 1}][n] (the
  // partial layout of the BatchNorm statistics, csrc/bnact.hip)
  float* stats;
  int resid_post;        // resid added after the activation (see above)
  // output rows (and resid rows) of image b at b yS + yoff + pixel when yS > 0
  // (forward only: the evaluation forward's input projections write their level
  // of the decoder memory [B, S, N] in place); 0 = dense [B H W, N]
  long long yS, yoff;
};

// Wait until K-tile kt's DMA has landed for this wave: up to min(S - 2, newer)
// younger tiles (GW instructions each) may stay in flight.
template <int S, int GW>
__device__ __forceinline__ void wait_ring(int newer) {
  if constexpr (S >= 4) {
    if (newer >= 2) wait_vm<2 * GW>();
    else if (newer == 1) wait_vm<GW>();
    else wait_vm<0>();
  } else if constexpr (S == 3) {
    if (newer >= 1) wait_vm<GW>();
    else wait_vm<0>();
  } else {
    wait_vm<0>();
  }
}

__device__ __forceinline__ void dma16(const uint16_t* src, char* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

// s_waitcnt vmcnt(n) for a run-time n (0..15; a larger n waits for 15, which
// is only stricter), as the builtin so the compiler's waitcnt pass sees it
template <int N>
__device__ __forceinline__ void vm_wait_b() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x70 | 0xF00);
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void vm_wait_dyn(int n) {
  switch (n < 0 ? 0 : (n > 15 ? 15 : n)) {
    case 0: vm_wait_b<0>(); break;
    case 1: vm_wait_b<1>(); break;
    case 2: vm_wait_b<2>(); break;
    case 3: vm_wait_b<3>(); break;
    case 4: vm_wait_b<4>(); break;
    case 5: vm_wait_b<5>(); break;
    case 6: vm_wait_b<6>(); break;
    case 7: vm_wait_b<7>(); break;
    case 8: vm_wait_b<8>(); break;
    case 9: vm_wait_b<9>(); break;
    case 10: vm_wait_b<10>(); break;
    case 11: vm_wait_b<11>(); break;
    case 12: vm_wait_b<12>(); break;
    case 13: vm_wait_b<13>(); break;
    case 14: vm_wait_b<14>(); break;
    default: vm_wait_b<15>(); break;
  }
}

// Epilogue of the implicit-GEMM convolutions (conv_fwd_kernel and
// conv3x3_halo_kernel): the fused bias / residual / activation / ReLU-mask
// operations and the BatchNorm statistics of ConvArgs, on the accumulator tile
// of WGM x WGN waves (wave (wm, wn) owns rows wm BM/WGM + 16 i and columns
// wn BN/WGN + 16 j).  PRE_OK: the epilogue operands may be loaded up front.
// EXT: the evaluation forward's extensions (SiLU, the residual after the
// activation, output rows at an image stride -- rtdetr_conv_fwd_act); a
// compile-time switch, so that the training kernels keep their register budget
// (the run-time branches cost the 32-deep tiles a workgroup per CU).
template <int BM, int BN, int WGM, int WGN, bool PH, bool PRE_OK, bool EXT = false>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, f32x4 (&acc)[BM / (16 * WGM)][BN / (16 * WGN)],
                                              char* smem, int m0, int n0, int tid, int lane, int wm, int wn) {
  constexpr int NTH = 64 * WGM * WGN;
  constexpr int CPR = BN / 8;
  constexpr int TM = BM / (16 * WGM), TN = BN / (16 * WGN);
  const int HW = a.H * a.W;
  // Epilogue through LDS: lane holds Y[m0 + wm BM/2 + 16 i + (lane & 15)][n0 + wn 64 + 16 j + 4 (lane >> 4) + 0..3];
  // the tile goes to a row-major [BM][BN] bf16 image (16-B chunk c of row r at chunk c ^ (r % CPR):
  // conflict-free 8-B writes and 16-B reads), then out as whole 256-B rows of 16-B stores
  // (register-direct 8-B stores at a row stride run at about half that rate).  The fused
  // epilogue's operands (same 16-B chunks as the stores) are loaded first, behind the image.
  constexpr int RPP = NTH / CPR;  // rows per store pass
  // epilogue operands loaded up front (else per store pass: registers; the
  // 32-deep variant keeps its register budget for 4 waves per SIMD)
  constexpr bool PRE = BM / RPP <= 16 && PRE_OK;
  constexpr int NPRE = PRE ? BM / RPP : 1;
  const int ec = tid % CPR;
  uint4 eres[NPRE], emask[NPRE];
  // global output row of GEMM row p (PH: the class pixel's dX row)
  auto grow = [&](int p) -> size_t {
    if constexpr (PH) {
      const int b = p / HW, rem = p - b * HW, ya = rem / a.W, xc = rem - ya * a.W;
      return ((size_t)b * a.Hd + 2 * ya + a.ry) * a.Wd + 2 * xc + a.rx;
    } else if constexpr (EXT) {
      if (a.yS == 0) return (size_t)p;
      const int b = p / HW;  // rows of image b start at b yS + yoff (a level block of [B, S, N])
      return (size_t)b * a.yS + a.yoff + (p - b * HW);
    } else {
      return (size_t)p;
    }
  };
  const bool ecol = n0 + ec * 8 < a.N;  // this thread's 8 output columns exist
  if (PRE && ecol && (a.resid != nullptr || a.mask != nullptr)) {
#pragma unroll
    for (int k = 0; k < NPRE; ++k) {
      const int p = m0 + tid / CPR + RPP * k;
      const size_t g = grow(p < a.P ? p : 0) * a.N + n0 + ec * 8;
      if (a.resid != nullptr) eres[k] = *reinterpret_cast<const uint4*>(a.resid + g);
      if (a.mask != nullptr) emask[k] = *reinterpret_cast<const uint4*>(a.mask + g);
    }
  }
  float eb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (a.bias != nullptr && ecol) {
    const float4 b0 = *reinterpret_cast<const float4*>(a.bias + n0 + ec * 8);
    const float4 b1 = *reinterpret_cast<const float4*>(a.bias + n0 + ec * 8 + 4);
    eb[0] = b0.x; eb[1] = b0.y; eb[2] = b0.z; eb[3] = b0.w;
    eb[4] = b1.x; eb[5] = b1.y; eb[6] = b1.z; eb[7] = b1.w;
  }
  const bool efloat = a.resid != nullptr || a.bias != nullptr || a.relu;
  float st_s[8], st_q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) st_s[e] = st_q[e] = 0.f;
  __syncthreads();  // every wave is done reading the ring
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = wm * (BM / WGM) + 16 * i + (lane & 15);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wn * (BN / WGN) + 16 * j + 4 * (lane >> 4);
      uint2 v;
      v.x = pack2bf(acc[i][j][0], acc[i][j][1]);
      v.y = pack2bf(acc[i][j][2], acc[i][j][3]);
      *reinterpret_cast<uint2*>(smem + r * (BN * 2) + (((col >> 3) ^ (r % CPR)) << 4) + (col & 7) * 2) = v;
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < BM / RPP; ++k) {
    const int r = tid / CPR + RPP * k, c = ec;
    const int p = m0 + r;
    if (p < a.P && ecol) {
      uint4 v = *reinterpret_cast<const uint4*>(smem + r * (BN * 2) + ((c ^ (r % CPR)) << 4));
      uint4 er, em;
      if constexpr (PRE) {
        er = eres[k];
        em = emask[k];
      } else {
        const size_t g = grow(p) * a.N + n0 + ec * 8;
        if (a.resid != nullptr) er = *reinterpret_cast<const uint4*>(a.resid + g);
        if (a.mask != nullptr) em = *reinterpret_cast<const uint4*>(a.mask + g);
      }
      if (efloat) {
        float f[8];
        unpack8(v, f);
        if (a.resid != nullptr && !(EXT && a.resid_post)) {
          float q[8];
          unpack8(er, q);
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] += q[e];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] += eb[e];
        if (!EXT || a.relu == 1) {
          if (a.relu) {
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] = fmaxf(f[e], 0.f);
          }
        } else if (a.relu == 2) {
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = f[e] / (1.f + __expf(-f[e]));
        }
        v = pack8(f);
        if constexpr (EXT) {
          if (a.resid != nullptr && a.resid_post) {
            float q[8];
            unpack8(v, f);
            unpack8(er, q);
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] += q[e];
            v = pack8(f);
          }
        }
      }
      if (a.mask != nullptr) {  // keep where the mask element is > 0 (bf16: sign clear, not zero)
        const uint32_t mw[4] = {em.x, em.y, em.z, em.w};
        uint32_t vw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t lo = mw[q] & 0xffffu, hi = mw[q] >> 16;
          const uint32_t keep_lo = ((lo & 0x8000u) || lo == 0) ? 0u : 0xffffu;
          const uint32_t keep_hi = ((hi & 0x8000u) || hi == 0) ? 0u : 0xffff0000u;
          vw[q] &= keep_lo | keep_hi;
        }
        v = make_uint4(vw[0], vw[1], vw[2], vw[3]);
      }
      *reinterpret_cast<uint4*>(a.y + grow(p) * a.N + n0 + c * 8) = v;
      if constexpr (!PH) {
        if (a.stats != nullptr) {  // BatchNorm statistics of the stored values
          float f[8];
          unpack8(v, f);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            st_s[e] += f[e];
            st_q[e] = fmaf(f[e], f[e], st_q[e]);
          }
        }
      }
    }
  }
  if constexpr (!PH) {
    if (a.stats != nullptr) {  // the RPP row groups' sums added in row order
      __syncthreads();  // every thread is done reading the output image
      float* red = reinterpret_cast<float*>(smem);  // [2][RPP][BN]
      const int rg = tid / CPR;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[rg * BN + ec * 8 + e] = st_s[e];
        red[(RPP + rg) * BN + ec * 8 + e] = st_q[e];
      }
      __syncthreads();
      for (int c = tid; c < BN; c += NTH) {
        float s1 = 0.f, s2 = 0.f;
        for (int r = 0; r < RPP; ++r) {
          s1 += red[r * BN + c];
          s2 += red[(RPP + r) * BN + c];
        }
        float* pp = a.stats + (size_t)(m0 / BM) * 2 * a.N + n0 + c;
        pp[0] = s1;
        pp[a.N] = s2;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// forward / data gradient
// ---------------------------------------------------------------------------
// WGM x WGN waves (2 x 2: 256 threads; the big tiles 256 x 128 / 256 x 256
// run 4 x 2 / 2 x 4 = 8 waves, 512 threads, two per SIMD): wave (wm, wn)
// computes rows wm BM/WGM .. and columns wn BN/WGN .. of the tile.
// AR (the A operand in registers): each wave loads its own A fragments --
// rows wm BM/WGM + 16 i + (lane & 15), 16 B of k per lane, straight from the
// pixel's neighbour row -- with plain vector loads into a two-deep register
// buffer, and only B goes through the LDS-DMA ring.  The conv's K-tile needs
// (BM + BN) x 128 B per workgroup through the LDS-DMA fill path, the bound of
// the 128 x 128 tile (~46 GB/s per CU against a measured LDS-DMA fill ceiling
// of ~70-90 GB/s per CU, MI355X_MICROARCH.md ldsdma-fill); with A on the
// vector-load path the ring carries half the bytes and the LDS serves B's
// fragment reads only.  One K-tile in flight (S = 2).
// KT: K-tile depth, 64 (128-B operand rows, 2 MFMA k-steps per barrier) or
// 32 (64-B rows, one k-step: half the ring bytes per stage, so more
// workgroups per CU at the same depth -- "conv_k32"); the 32-deep
// K-contiguous image swizzles chunk c of row r to c ^ ((r >> 2) & 3).
template <int KS, int S, int BM, int BN, bool BT, bool PH = false, int WGM = 2, int WGN = 2, bool AR = false,
          int KT = 64, bool EXT = false>
__global__ __launch_bounds__(64 * WGM * WGN) void conv_fwd_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  static_assert(BN == 64 || BN == 128 || BN == 256, "output-channel tile: 64, 128 or 256");
  static_assert(!AR || S == 2, "AR: one K-tile in flight");
  static_assert(KT == 64 || (KT == 32 && !AR), "K-tile 64, or 32 without AR");
  constexpr int NW = WGM * WGN, NTH = 64 * NW;
  constexpr int RB = KT * 2;              // bytes per operand row of a K-contiguous K-tile image
  constexpr int CH = KT / 8;              // 16-B chunks per such row
  constexpr int RPI = 1024 / RB;          // rows per DMA instruction (64 lanes x 16 B)
  constexpr int TILE = (AR ? BN : BM + BN) * RB;  // bytes of one ring stage
  constexpr int CPR = BN / 8;            // 16-B chunks per output row of the tile
  constexpr int TM = BM / (16 * WGM), TN = BN / (16 * WGN);  // 16 x 16 blocks per wave
  constexpr int AP = BM / (RPI * NW), BP = BN / (RPI * NW);   // DMA instructions per wave per K-tile (A, B)
  static_assert(AP >= 1 && BP >= 1 && AP * RPI * NW == BM && BP * RPI * NW == BN, "tile / wave split");
  auto kswz = [](int r) { return KT == 64 ? ((r >> 1) & 7) : ((r >> 2) & 3); };
  constexpr int GW = (AR ? 0 : AP) + BP;  // DMA instructions per wave per K-tile
  constexpr int PAD = (KS - 1) / 2;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  // XCD-aware map: the N tiles of one M tile run on one XCD (they share the A panel);
  // a partial last N tile (N % BN, forward only: the stem's 32-channel layers) reads
  // zero weight rows and stores only its valid columns
  const int NT = (a.N + BN - 1) / BN;
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int nt = slot % NT;
  const int mt = (slot / NT) * 8 + xcd;
  if (mt >= a.mt_n) return;
  const int m0 = mt * BM, n0 = nt * BN;
  const int cpt = a.C / KT;        // K-tiles per tap
  const int nty = PH ? 1 + a.ry : KS, ntx = PH ? 1 + a.rx : KS;  // taps per axis
  const int nk = nty * ntx * cpt;
  const int HW = a.H * a.W, HWs = a.Hs * a.Ws;
  // this lane's A rows (one per DMA instruction j): pixel, coordinates, source chunk
  int py[AP], px[AP], pb[AP], ach[AP];
  bool pv[AP];
#pragma unroll
  for (int j = 0; j < AP; ++j) {
    const int r = (wave + NW * j) * RPI + lane / CH;
    const int p = m0 + r;
    pv[j] = p < a.P;
    const int pp = pv[j] ? p : 0;
    pb[j] = pp / HW;
    const int rem = pp - pb[j] * HW;
    py[j] = rem / a.W;
    px[j] = rem - py[j] * a.W;
    ach[j] = ((lane % CH) ^ kswz(r)) * 8;
  }
  // B rows.  Forward: K-contiguous [BN][64] image of W[n][tap][c0..c0+63].
  // BT (data gradient, a.w = the ORIGINAL weight [a.C][KS][KS][a.N]): the
  // operand is W'[n][tap][k] = W[k][KS^2-1-tap][n], read as an MN-contiguous
  // [64 k-rows][BN] image (k-row = one of W's output channels, BN contiguous
  // input channels; ds_read_b64_tr_b16 fragments) -- no transposed copy of W.
  const uint16_t* wrow[BP];
  bool bv[BP];  // this lane's weight row exists (n0 + r < N)
#pragma unroll
  for (int j = 0; j < BP; ++j) {
    if constexpr (BT) {  // CPR lanes per k-row
      const int kr = (wave + NW * j) * (64 / CPR) + lane / CPR;
      wrow[j] = a.w + (size_t)kr * (KS * KS * a.N) + n0 + ((lane % CPR) ^ mimg_swz<BN>(kr)) * 8;
      bv[j] = true;
    } else {
      const int r = (wave + NW * j) * RPI + lane / CH;
      bv[j] = n0 + r < a.N;
      wrow[j] = bv[j] ? a.w + (size_t)(n0 + r) * (KS * KS * a.C) + ((lane % CH) ^ kswz(r)) * 8
                      : a.zero + ((lane % CH) ^ kswz(r)) * 8;
    }
  }
  // K-tile kt -> (input-channel offset c0, weight tap, neighbour offset dy, dx)
  auto tapinfo = [&](int kt, int& c0, int& tap, int& dy, int& dx) {
    const int t = kt / cpt;
    c0 = (kt - t * cpt) * KT;
    if constexpr (PH) {  // class tap (ty, tx) -> flipped-weight tap and dY offset (0 or +1 per axis)
      const int ty = t / ntx, tx = t - ty * ntx;
      const int ky = a.ry ? 2 * ty : 1, kx = a.rx ? 2 * tx : 1;
      tap = ky * KS + kx;
      dy = ky == 2;
      dx = kx == 2;
    } else {
      tap = t;
      dy = tap / KS - PAD;
      dx = tap % KS - PAD;
    }
  };
  auto issue = [&](int kt) {
    char* buf = smem + (kt % S) * TILE;
    int c0, tap, dy, dx;
    tapinfo(kt, c0, tap, dy, dx);
#pragma unroll
    for (int j = 0; j < (AR ? 0 : AP); ++j) {
      int yy = py[j] * a.st + dy, xx = px[j] * a.st + dx;
      bool ok = pv[j] && !(((yy | xx) & a.sh));  // sh = 1: both even
      yy >>= a.sh;
      xx >>= a.sh;
      ok = ok && yy >= 0 && yy < a.Hs && xx >= 0 && xx < a.Ws;
      const uint16_t* src = ok ? a.x + ((size_t)(pb[j] * HWs + yy * a.Ws + xx)) * a.C + c0 + ach[j] : a.zero + ach[j];
      dma16(src, buf + (wave + NW * j) * 1024);
    }
    constexpr int BOFF = AR ? 0 : BM * RB;  // the B image's offset in the stage
#pragma unroll
    for (int j = 0; j < BP; ++j) {
      if constexpr (BT) dma16(wrow[j] + (size_t)c0 * (KS * KS * a.N) + (KS * KS - 1 - tap) * a.N,
                              buf + BOFF + (wave + NW * j) * 1024);
      else dma16(bv[j] ? wrow[j] + tap * a.C + c0 : wrow[j], buf + BOFF + (wave + NW * j) * 1024);
    }
  };
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (AR) {
    // this lane's A rows (one per 16-row block i): pixel coordinates
    int qy[TM], qx[TM], qb[TM];
    bool qv[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int p = m0 + wm * (BM / WGM) + 16 * i + (lane & 15);
      qv[i] = p < a.P;
      const int pp = qv[i] ? p : 0;
      qb[i] = pp / HW;
      const int rem = pp - qb[i] * HW;
      qy[i] = rem / a.W;
      qx[i] = rem - qy[i] * a.W;
    }
    const int kch = (lane >> 4) * 8;  // this lane's 8 k of each 32-k step
    auto load_a = [&](int kt, bf16x8 (&dst)[TM][2]) {
      int c0, tap, dy, dx;
      tapinfo(kt, c0, tap, dy, dx);
      (void)tap;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        int yy = qy[i] * a.st + dy, xx = qx[i] * a.st + dx;
        bool ok = qv[i] && !(((yy | xx) & a.sh));
        yy >>= a.sh;
        xx >>= a.sh;
        ok = ok && yy >= 0 && yy < a.Hs && xx >= 0 && xx < a.Ws;
        const uint16_t* src = ok ? a.x + ((size_t)(qb[i] * HWs + yy * a.Ws + xx)) * a.C + c0 + kch : a.zero + kch;
        dst[i][0] = *reinterpret_cast<const bf16x8*>(src);
        dst[i][1] = *reinterpret_cast<const bf16x8*>(src + 32);
      }
    };
    auto compute = [&](const char* bbuf, const bf16x8 (&af)[TM][2]) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 bfr[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = read_frag<BN, !BT>(bbuf, wn * (BN / WGN) + 16 * j, ks, lane);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i][ks], acc[i][j], 0, 0, 0);
      }
    };
    // s_waitcnt vmcnt(0) as a builtin (the compiler's waitcnt pass sees it)
    auto drain = [] {
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_waitcnt(0x70 | 0xF00);
      asm volatile("" ::: "memory");
    };
    bf16x8 A0[TM][2], A1[TM][2];
    if (nk > 0) {
      issue(0);
      load_a(0, A0);
    }
    for (int kt = 0; kt < nk; kt += 2) {
      drain();  // B DMA and A loads of tile kt have landed (this wave)
      __builtin_amdgcn_s_barrier();  // ... for every wave; slot (kt + 1) % 2 is free
      if (kt + 1 < nk) {
        issue(kt + 1);
        load_a(kt + 1, A1);
      }
      compute(smem + (kt % 2) * TILE, A0);
      if (kt + 1 < nk) {
        drain();
        __builtin_amdgcn_s_barrier();
        if (kt + 2 < nk) {
          issue(kt + 2);
          load_a(kt + 2, A0);
        }
        compute(smem + ((kt + 1) % 2) * TILE, A1);
      }
    }
  } else {
#pragma unroll
    for (int s = 0; s < S - 1; ++s)
      if (s < nk) issue(s);
    for (int kt = 0; kt < nk; ++kt) {
      wait_ring<S, GW>(nk - 1 - kt);
      __builtin_amdgcn_s_barrier();  // every wave's DMA of tile kt has landed
      if (kt + S - 1 < nk) issue(kt + S - 1);  // refills the slot consumed in iteration kt - 1
      const char* cur = smem + (kt % S) * TILE;
      if constexpr (KT == 64) {
        compute_tile_w<BM, BN, WGM, WGN, true, !BT>(cur, cur + BM * 128, acc, lane, wm, wn);
      } else {  // one 32-deep k-step
        auto rd32 = [&](const char* img, int row_base) {
          const int r = row_base + (lane & 15), c = lane >> 4;
          return *reinterpret_cast<const bf16x8*>(img + r * 64 + ((c ^ ((r >> 2) & 3)) << 4));
        };
        const char* bimg = cur + BM * 64;
        bf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = rd32(cur, wm * (BM / WGM) + 16 * i);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (BT) bfr[j] = read_frag<BN, false>(bimg, wn * (BN / WGN) + 16 * j, 0, lane);
          else bfr[j] = rd32(bimg, wn * (BN / WGN) + 16 * j);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      }
    }
  }
  conv_epilogue<BM, BN, WGM, WGN, PH, KT == 64, EXT>(a, acc, smem, m0, n0, tid, lane, wm, wn);
}

// ---------------------------------------------------------------------------
// 3x3 stride-1 convolutions with a halo-staged A operand (round 6)
// ---------------------------------------------------------------------------
// conv_fwd_kernel stages, for every (tap, 64-channel slice) K-tile, the BM
// neighbour rows of its output pixels: 9 x BM rows per slice, each through a
// per-row computed LDS-DMA source (tap offsets, bounds) -- the issue cost of
// those DMAs and their address arithmetic, not the bytes, left the MFMA pipe
// busy 0.33 of the time (r05 PMC).  Here the M-tile is BM consecutive output
// pixels in raster order, and for each 64-channel slice three halo groups are
// staged once:
//   group g (dy = g - 1): pixels m0 + dy W - 1 .. m0 + dy W + BM  (BM + 2 rows)
// as plain contiguous rows (a row outside [0, P) reads the zero row).  Tap
// (dy, dx)'s A fragment for output row r is halo row r + dx + 1 of group
// dy + 1; a lane whose pixel has no such neighbour (y + dy or x + dx outside
// the image -- which includes every row that wrapped into another image row
// or image) reads a zero row of LDS instead.  So a slice costs 3 (BM + 2) A
// rows instead of 9 BM, with no per-tap address work, and the B operand (the
// weight K-tile of the tap) streams through a BS-deep ring as before.
// Schedule, per K-step kt = (slice cs, tap t), t = 3 g + (dx + 1):
//   wait (this wave's B(kt) and halo(g, cs) landed) -> barrier ->
//   issue B(kt + BS - 1); at t = 3 the group-0 halo of slice cs + 1, at t = 6
//   group 1 of cs + 1, at t = 0 group 2 of cs (each group's previous contents
//   were last read before this barrier) -> MFMA on (cs, t).
// Each group reload has six K-steps to land.  The per-wave vmcnt waits are
// counted at run time from the wave's own issue sequence.
// BM x BN tile, WGM x WGN waves of 64 x 64; the same K order for every output
// (slice-major, tap-minor) and the shared epilogue (conv_epilogue).
template <int BM, int BN, int WGM, int WGN, int BS>
__global__ __launch_bounds__(64 * WGM * WGN) void conv3x3_halo_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NW = WGM * WGN;
  constexpr int HR = BM + 2;                      // halo rows per group
  constexpr int GI = (HR + 7) / 8;                // 1-KiB DMA instructions per group (8 rows each)
  constexpr int GS = GI * 1024;                   // group stride (bytes)
  constexpr int HALO = 3 * GS;
  constexpr int BT_BYTES = BN * 128;              // one B K-tile image
  constexpr int BP = BN / (8 * NW);               // B DMA instructions per wave per K-step
  constexpr int ZOFF = HALO + BS * BT_BYTES;      // the 128-B zero row
  constexpr int TM = BM / (16 * WGM), TN = BN / (16 * WGN);
  static_assert(BP >= 1 && BP * 8 * NW == BN, "B tile / wave split");
  static_assert(BM / WGM == 64 && BN / WGN == 64, "64 x 64 wave tiles");
  static_assert(ZOFF + 128 <= 160 * 1024 && BM * BN * 2 <= ZOFF, "LDS budget");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  const int NT = a.N / BN;
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int nt = slot % NT;
  const int mt = (slot / NT) * 8 + xcd;
  if (mt >= a.mt_n) return;
  const int m0 = mt * BM, n0 = nt * BN;
  const int ncs = a.C / 64;
  const int nk = 9 * ncs;
  const int HW = a.H * a.W;
  if (tid < 8) *reinterpret_cast<uint4*>(smem + ZOFF + tid * 16) = make_uint4(0, 0, 0, 0);
  // tap validity of this lane's output rows (bit t: tap t = 3 (dy + 1) + dx + 1 has its neighbour)
  uint32_t tv[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int p = m0 + wm * 64 + 16 * i + (lane & 15);
    const int rem = p % HW, y = rem / a.W, x = rem - y * a.W;
    const uint32_t ym = y > 0, yp = y < a.H - 1, xm = x > 0, xp = x < a.W - 1;
    const uint32_t rows[3] = {ym, 1u, yp}, cols[3] = {xm, 1u, xp};
    uint32_t m = 0;
#pragma unroll
    for (int t = 0; t < 9; ++t) m |= (rows[t / 3] & cols[t % 3]) << t;
    tv[i] = m;
  }
  // halo group g of slice cs: GI instructions j = wave + NW u (rows 8 j .. 8 j + 7)
  const int hc = (GI - wave + NW - 1) / NW;  // this wave's instructions per group
  auto issue_halo = [&](int g, int cs) {
    const long long q0 = (long long)m0 + (long long)(g - 1) * a.W - 1;
    char* gbase = smem + g * GS;
    for (int j = wave; j < GI; j += NW) {
      const int hr = 8 * j + (lane >> 3);
      const int c = (lane & 7) ^ ((hr >> 1) & 7);
      const long long q = q0 + hr;
      const bool ok = hr < HR && q >= 0 && q < a.P;
      const uint16_t* src = ok ? a.x + (size_t)q * a.C + cs * 64 + c * 8 : a.zero + c * 8;
      dma16(src, gbase + j * 1024);
    }
  };
  // B K-tile kt = (cs, t): W[n0 + r][t][cs 64 ..], rows 8 j .. 8 j + 7 for j = wave + NW b
  auto issue_b = [&](int kt) {
    const int cs = kt / 9, t = kt - cs * 9;
    char* bbase = smem + HALO + (kt % BS) * BT_BYTES;
#pragma unroll
    for (int b = 0; b < BP; ++b) {
      const int j = wave + NW * b;
      const int r = 8 * j + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      dma16(a.w + (size_t)(n0 + r) * (9 * a.C) + t * a.C + cs * 64 + c * 8, bbase + j * 1024);
    }
  };
  // per-wave issue bookkeeping (scalars, constant indices only): cumulative DMA
  // instruction count after the B tiles kt .. kt + BS - 2 (bq[]) and after the
  // latest issue of each halo group (h0, h1, h2)
  static_assert(BS >= 2 && BS <= 4, "B ring depth");
  int cnt = 0;
  int bq[BS - 1];
  issue_halo(0, 0);
  cnt += hc;
  int h0 = cnt;
  issue_halo(1, 0);
  cnt += hc;
  int h1 = cnt;
  issue_halo(2, 0);
  cnt += hc;
  int h2 = cnt;
#pragma unroll
  for (int s = 0; s < BS - 1; ++s) {
    if (s < nk) {
      issue_b(s);
      cnt += BP;
    }
    bq[s] = cnt;
  }
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int zrow = ZOFF;
  for (int kt = 0; kt < nk; ++kt) {
    const int cs = kt / 9, t = kt - cs * 9, g = t / 3, dx = t - 3 * g - 1;
    vm_wait_dyn(cnt - max(bq[0], g == 0 ? h0 : (g == 1 ? h1 : h2)));
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (kt + BS - 1 < nk) {
      issue_b(kt + BS - 1);
      cnt += BP;
    }
#pragma unroll
    for (int s = 0; s + 1 < BS - 1; ++s) bq[s] = bq[s + 1];
    bq[BS - 2] = cnt;
    if (t == 3 && cs + 1 < ncs) {
      issue_halo(0, cs + 1);
      cnt += hc;
      h0 = cnt;
    } else if (t == 6 && cs + 1 < ncs) {
      issue_halo(1, cs + 1);
      cnt += hc;
      h1 = cnt;
    } else if (t == 0 && cs > 0) {
      issue_halo(2, cs);
      cnt += hc;
      h2 = cnt;
    }
    const char* gbase = smem + g * GS;
    const char* bimg = smem + HALO + (kt % BS) * BT_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[TM], bfr[TN];
      const int c = ks * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int h = wm * 64 + 16 * i + (lane & 15) + dx + 1;
        const int off = ((tv[i] >> t) & 1) ? (int)(gbase - smem) + h * 128 + ((c ^ ((h >> 1) & 7)) << 4)
                                            : zrow + (c << 4);
        af[i] = *reinterpret_cast<const bf16x8*>(smem + off);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = read_frag<BN, true>(bimg, wn * 64 + 16 * j, ks, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
  }
  vm_wait_b<0>();  // (nothing is in flight here; the epilogue reuses the halo LDS)
  conv_epilogue<BM, BN, WGM, WGN, false, true>(a, acc, smem, m0, n0, tid, lane, wm, wn);
}

// ---------------------------------------------------------------------------
// 256 x 256 tiles in 8 phases (round 6)
// ---------------------------------------------------------------------------
// The 2-barrier-per-K-tile structure of conv_fwd_kernel (and of the halo
// kernel above, which cut the A staging ~2.5x and ran no faster) sits at the
// ~750 TFLOP/s ceiling cdna_hip_programming.md section 5 describes for that
// structure; its 256 x 256 eight-phase schedule is the way past it.  Here:
// 8 waves as 2 (M) x 4 (N), 128 x 64 outputs per wave (acc 8 x 4 blocks),
// 64-deep K-tiles double-buffered in LDS (A [256][64] + B [256][64] = 64 KiB
// per buffer), each K-tile computed in 4 phases -- one 64 x 32 quadrant of the
// wave tile per phase, 16 MFMA -- in the order (0,0) (0,1) (1,1) (1,0), so a
// phase reads 8 A fragments, 4 B fragments, or both.  The staging unit is the
// half-tile: H0 = A rows {0..63, 128..191} (both wave rows' first quarters),
// H1 = A rows {64..127, 192..255}, H2 = B rows (output channels) {64 c + 0..31},
// H3 = {64 c + 32..63}; 16 KiB, two LDS-DMA instructions per wave each.  A
// half-tile is re-staged (for the K-tile two ahead, same buffer) in the phase
// after its last read: H0 in phase 1, H3 in 2, H1 in 3, H2 in 4 (phases 0-3
// compute the even buffer, 4-7 the odd one: the odd buffer's half-tiles go out
// in phases 5, 6, 7 and 0).  Three half-tiles stay in flight across the
// barriers: vmcnt(6) at phases 3 and 7 retires the other buffer, whose reads
// start one phase later.  Phase body: fragment reads -> half-tile issue ->
// [wait] -> barrier -> lgkmcnt(0) -> setprio(1), 16 MFMA, setprio(0) ->
// barrier.  A rows are gathered per tap like conv_fwd_kernel's (any
// KS / stride / dgrad geometry of ConvArgs, PH excluded); every output's K loop
// runs in conv_fwd_kernel's order (tap-major, channel slice minor, k-steps of
// 32 in order), so the two kernels agree bit for bit.
template <int KS>
__global__ __launch_bounds__(512, 1) void conv_8ph_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BM = 256, BN = 256, NW = 8;
  constexpr int IMG = 256 * 128;  // one [256][64] bf16 operand image
  constexpr int BUF = 2 * IMG;    // A + B of one K-tile
  constexpr int PAD = (KS - 1) / 2;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int NT = a.N / BN;
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int nt = slot % NT;
  const int mt = (slot / NT) * 8 + xcd;
  if (mt >= a.mt_n) return;
  const int m0 = mt * BM, n0 = nt * BN;
  const int cpt = a.C / 64;
  const int nk = KS * KS * cpt;
  const int HW = a.H * a.W, HWs = a.Hs * a.Ws;
  // A staging: half h, instruction u (0, 1): half-rows 8 j .. 8 j + 7, j = wave + 8 u;
  // lane's half-row hr = 8 j + lane / 8 -> tile row r = (hr & 63) + 128 (hr >> 6) + 64 h
  int py[2][2], px[2][2], pb[2][2], ach[2][2];
  bool pv[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int hr = 8 * (wave + 8 * u) + (lane >> 3);
      const int r = (hr & 63) + 128 * (hr >> 6) + 64 * h;
      const int p = m0 + r;
      pv[h][u] = p < a.P;
      const int pp = pv[h][u] ? p : 0;
      pb[h][u] = pp / HW;
      const int rem = pp - pb[h][u] * HW;
      py[h][u] = rem / a.W;
      px[h][u] = rem - py[h][u] * a.W;
      ach[h][u] = ((lane & 7) ^ ((r >> 1) & 7)) * 8;
    }
  auto tapinfo = [&](int kt, int& c0, int& tap, int& dy, int& dx) __attribute__((always_inline)) {
    const int t = kt / cpt;
    c0 = (kt - t * cpt) * 64;
    tap = t;
    dy = t / KS - PAD;
    dx = t % KS - PAD;
  };
  auto issue_a = [&](int h, int kt) __attribute__((always_inline)) {
    char* img = smem + (kt & 1) * BUF;
    int c0, tap, dy, dx;
    tapinfo(kt, c0, tap, dy, dx);
    (void)tap;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int hr0 = 8 * (wave + 8 * u);
      const int r0 = (hr0 & 63) + 128 * (hr0 >> 6) + 64 * h;
      int yy = py[h][u] * a.st + dy, xx = px[h][u] * a.st + dx;
      bool ok = pv[h][u] && !(((yy | xx) & a.sh));
      yy >>= a.sh;
      xx >>= a.sh;
      ok = ok && yy >= 0 && yy < a.Hs && xx >= 0 && xx < a.Ws;
      const uint16_t* src = ok ? a.x + ((size_t)(pb[h][u] * HWs + yy * a.Ws + xx)) * a.C + c0 + ach[h][u]
                               : a.zero + ach[h][u];
      dma16(src, img + r0 * 128);
    }
  };
  // B staging: half h (H2 = 0, H3 = 1): half-row hr -> channel row n = 64 (hr >> 5) + (hr & 31) + 32 h
  auto issue_b = [&](int h, int kt) __attribute__((always_inline)) {
    char* img = smem + (kt & 1) * BUF + IMG;
    int c0, tap, dy, dx;
    tapinfo(kt, c0, tap, dy, dx);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int hr0 = 8 * (wave + 8 * u);
      const int hr = hr0 + (lane >> 3);
      const int n = 64 * (hr >> 5) + (hr & 31) + 32 * h;
      const int n0r = 64 * (hr0 >> 5) + (hr0 & 31) + 32 * h;
      const int c = (lane & 7) ^ ((n >> 1) & 7);
      dma16(a.w + (size_t)(n0 + n) * (KS * KS * a.C) + tap * a.C + c0 + c * 8, img + n0r * 128);
    }
  };
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[4][2], bfr[2][2];
  // fragment addresses: the K-contiguous image's swizzle (r >> 1) & 7 depends only on lane & 15 for
  // 16-aligned row blocks, so every fragment of a k-step is one per-lane base + a constant offset
  // (ds_read_b128's immediate): two bases per operand instead of one address register per fragment
  const int fr = lane & 15, fc = lane >> 4;
  const int abase0 = kimg_off(wr * 128 + fr, fc), abase1 = kimg_off(wr * 128 + fr, 4 + fc);
  const int bbase0 = IMG + kimg_off(wc * 64 + fr, fc), bbase1 = IMG + kimg_off(wc * 64 + fr, 4 + fc);
  auto read_a = [&](int kt, int qa) __attribute__((always_inline)) {
    const char* img = smem + (kt & 1) * BUF;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      af[i][0] = *reinterpret_cast<const bf16x8*>(img + abase0 + (qa * 64 + 16 * i) * 128);
      af[i][1] = *reinterpret_cast<const bf16x8*>(img + abase1 + (qa * 64 + 16 * i) * 128);
    }
  };
  auto read_b = [&](int kt, int qb) __attribute__((always_inline)) {
    const char* img = smem + (kt & 1) * BUF;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      bfr[j][0] = *reinterpret_cast<const bf16x8*>(img + bbase0 + (qb * 32 + 16 * j) * 128);
      bfr[j][1] = *reinterpret_cast<const bf16x8*>(img + bbase1 + (qb * 32 + 16 * j) * 128);
    }
  };
  auto mfma = [&](int qa, int qb) __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[qa * 4 + i][qb * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j][ks], af[i][ks], acc[qa * 4 + i][qb * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto bar = []() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // prologue: K-tile 0 (even buffer) whole, K-tile 1's H0, H3, H1 (its H2 goes out in phase 0);
  // nk is even (ph8_ok), so every loop trip computes two whole K-tiles and has one exit
  issue_a(0, 0);
  issue_b(1, 0);
  issue_a(1, 0);
  issue_b(0, 0);
  issue_a(0, 1);
  issue_b(1, 1);
  issue_a(1, 1);
  vm_wait_b<6>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  bar();
  for (int kt = 0; kt < nk; kt += 2) {
    const bool nx0 = kt + 2 < nk;  // (then kt + 3 < nk as well)
    // phase 0: quadrant (0,0) of the even tile
    read_a(kt, 0);
    read_b(kt, 0);
    issue_b(0, kt + 1);
    bar();
    mfma(0, 0);
    bar();
    // phase 1: (0,1)
    read_b(kt, 1);
    if (nx0) issue_a(0, kt + 2);
    bar();
    mfma(0, 1);
    bar();
    // phase 2: (1,1)
    read_a(kt, 1);
    if (nx0) issue_b(1, kt + 2);
    bar();
    mfma(1, 1);
    bar();
    // phase 3: (1,0); retire the odd tile
    read_b(kt, 0);
    if (nx0) {
      issue_a(1, kt + 2);
      vm_wait_b<6>();
    } else {
      vm_wait_b<0>();
    }
    bar();
    mfma(1, 0);
    bar();
    // phases 4-7: the odd tile kt + 1
    read_a(kt + 1, 0);
    read_b(kt + 1, 0);
    if (nx0) issue_b(0, kt + 2);
    bar();
    mfma(0, 0);
    bar();
    read_b(kt + 1, 1);
    if (nx0) issue_a(0, kt + 3);
    bar();
    mfma(0, 1);
    bar();
    read_a(kt + 1, 1);
    if (nx0) issue_b(1, kt + 3);
    bar();
    mfma(1, 1);
    bar();
    read_b(kt + 1, 0);
    if (nx0) {
      issue_a(1, kt + 3);
      vm_wait_b<6>();
    } else {
      vm_wait_b<0>();
    }
    bar();
    mfma(1, 0);
    bar();
  }
  vm_wait_b<0>();
  conv_epilogue<BM, BN, 2, 4, false, false, true>(a, acc, smem, m0, n0, tid, lane, wr, wc);
}

// The ResNet-D stem's first convolution (3 -> 32 channels, 3x3, stride 2,
// pad 1, the frozen BatchNorm folded: bias + ReLU) -- 3 input channels are too
// shallow for the implicit GEMM's K-tiles (MIOpen ran it at ~110 us plus a
// bias + ReLU pass).  One thread per output pixel computes all NO outputs on
// the vector ALU: its 9 CI input values loaded first (independent loads in
// flight), the weights fp32 [9 CI][NO] read with uniform addresses (scalar
// loads into SGPRs, operands of packed fp32 FMAs: two output channels per
// v_pk_fma_f32; weights staged in LDS instead cost a waited ds_read per two
// FMAs), fp32 sums + bias, ReLU, one rounding, 16-B stores of the NHWC row.
template <int NO, int CI>
__global__ __launch_bounds__(256) void conv_direct_kernel(const uint16_t* __restrict__ x, const float* __restrict__ wf,
                                                          const float* __restrict__ bias, uint16_t* __restrict__ y,
                                                          int B, int H, int W, int Ho, int Wo, int st, int relu) {
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  const long long P = (long long)B * Ho * Wo;
  const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  const int HWo = Ho * Wo;
  const int b = (int)(p / HWo), rem = (int)(p - (long long)b * HWo), yo = rem / Wo, xo = rem - yo * Wo;
  // all 9 CI input loads issued first (one latency, not nine); the tap loop
  // kept rolled (unrolled, the compiler hoists all 9 CI NO weight loads and
  // spills SGPRs) over a shifting register window: tap t reads raw[0 .. CI)
  // and moves the rest down
  uint16_t raw[9 * CI];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int yy = yo * st + t / 3 - 1, xx = xo * st + t % 3 - 1;
    const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
    const uint16_t* src = x + (((size_t)b * H + (ok ? yy : 0)) * W + (ok ? xx : 0)) * CI;
#pragma unroll
    for (int c = 0; c < CI; ++c) raw[t * CI + c] = ok ? src[c] : (uint16_t)0;
  }
  f32x2 acc[NO / 2];
#pragma unroll
  for (int n = 0; n < NO / 2; ++n) acc[n] = f32x2{0.f, 0.f};
#pragma unroll 1
  for (int t = 0; t < 9; ++t) {
    const float* wt = wf + (size_t)t * CI * NO;
#pragma unroll
    for (int c = 0; c < CI; ++c) {
      const float v = bf2f(raw[c]);
      const f32x2 vv = f32x2{v, v};
#pragma unroll
      for (int n = 0; n < NO; n += 2)
        acc[n / 2] = __builtin_elementwise_fma(vv, f32x2{wt[c * NO + n], wt[c * NO + n + 1]}, acc[n / 2]);
    }
#pragma unroll
    for (int i = 0; i < 8 * CI; ++i) raw[i] = raw[i + CI];
  }
  uint4* out = reinterpret_cast<uint4*>(y + (size_t)p * NO);
#pragma unroll
  for (int n = 0; n < NO; n += 8) {
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float t = acc[(n + j) / 2][(n + j) % 2] + (bias ? bias[n + j] : 0.f);
      o[j] = relu ? fmaxf(t, 0.f) : t;
    }
    out[n / 8] = pack8(o);
  }
}

// W'[c][tap][n] = W[n][KS^2-1-tap][c]: the data gradient's K-contiguous
// weight.  One workgroup transposes a 64 x 64 (n, c) block of one tap through
// LDS: 128-B row reads along c, 128-B row writes along n.
__global__ __launch_bounds__(256) void conv_weight_flip_kernel(const uint16_t* __restrict__ w,
                                                               uint16_t* __restrict__ wt, int N, int C, int KS) {
  __shared__ uint16_t t[64][66];
  const int c0 = blockIdx.x * 64, n0 = blockIdx.y * 64, tap = blockIdx.z, T = KS * KS;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int n = ty + 4 * r;
    t[n][tx] = w[((size_t)(n0 + n) * T + (T - 1 - tap)) * C + c0 + tx];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int c = ty + 4 * r;
    wt[((size_t)(c0 + c) * T + tap) * N + n0 + tx] = t[tx][c];
  }
}

// Every registered convolution weight of a step flipped in ONE launch (the
// data gradients then read their W' from persistent buffers): descriptor i
// owns blocks [block0_i, block0_{i+1}), one 64 x 64 (n, c) block of one tap
// each, as conv_weight_flip_kernel.
struct FlipDesc {
  const uint16_t* w;
  uint16_t* wt;
  int N, C, KS, block0;
};

__global__ __launch_bounds__(256) void conv_weight_flip_multi_kernel(const FlipDesc* __restrict__ d, int n) {
  __shared__ uint16_t t[64][66];
  int i = 0;
  while (i + 1 < n && d[i + 1].block0 <= (int)blockIdx.x) ++i;  // (n is small: a uniform scan)
  const uint16_t* w = d[i].w;
  uint16_t* wt = d[i].wt;
  const int N = d[i].N, C = d[i].C, T = d[i].KS * d[i].KS;
  const int cb = C / 64, nbk = N / 64;
  const int local = blockIdx.x - d[i].block0;
  const int tap = local / (cb * nbk), rem = local - tap * cb * nbk;
  const int n0 = (rem / cb) * 64, c0 = (rem - (rem / cb) * cb) * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int nn = ty + 4 * r;
    t[nn][tx] = w[((size_t)(n0 + nn) * T + (T - 1 - tap)) * C + c0 + tx];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int c = ty + 4 * r;
    wt[((size_t)(c0 + c) * T + tap) * N + n0 + tx] = t[tx][c];
  }
}

// ---------------------------------------------------------------------------
// weight gradient
// ---------------------------------------------------------------------------
struct ConvWgArgs {
  const uint16_t* dy;    // [P][N], P = B Ho Wo
  const uint16_t* x;     // [B H W][C]
  float* part;           // [S][N][KS KS C]
  const uint16_t* zero;
  int B, H, W, C, N, P;
  int nsplit, kt_per;    // pixel K-tiles per slice
  int Ho, Wo, st;        // output pixels (dY) and the stride: x neighbour (st y + dy, st x + dx)
};

// Tile WBM (output channels) x WBN (tap-major input channels of one tap):
// 128 x 128, or 64 on a side with 64 channels (ResNet stage 1).
template <int KS, int S, int WBM, int WBN>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(ConvWgArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TM = WBM / 32, TN = WBN / 32;
  constexpr int TILE = (WBM + WBN) * 128;  // bytes of one ring stage
  // DMA: LA (LB) lanes per 2 WBM- (WBN-) byte k-row, NA (NB) instructions per wave per K-tile
  constexpr int LA = WBM / 8, LB = WBN / 8, NA = LA / 4, NB = LB / 4;
  constexpr int GW = NA + NB;
  constexpr int PAD = (KS - 1) / 2;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int NN = KS * KS * a.C;      // GEMM N
  const int MT = a.N / WBM, NT = NN / WBN;
  // work units u = split * tiles + tile, a contiguous run of ceil(units / 8)
  // per XCD: the tiles of one pixel slice share an XCD (its dY and X rows
  // stream through that L2 once; slices of one tile spread over XCDs made
  // every XCD read all rows) and every XCD gets the same number of units
  const int tiles = MT * NT;
  const int units = tiles * a.nsplit, per_xcd = (units + 7) / 8;
  const int local = blockIdx.x >> 3;
  const int u = (blockIdx.x & 7) * per_xcd + local;
  if (local >= per_xcd || u >= units) return;
  const int tile = u % tiles, split = u / tiles;
  const int mt = tile % MT, nt = tile / MT;
  const int m0 = mt * WBM, nn0 = nt * WBN;
  const int tap = nn0 / a.C, c0 = nn0 - tap * a.C;
  const int dy_ = tap / KS - PAD, dx_ = tap % KS - PAD;
  const int ktot = (a.P + 63) / 64;
  const int kt0 = split * a.kt_per;
  const int nk = max(0, min(a.kt_per, ktot - kt0));
  const int HWo = a.Ho * a.Wo, HW = a.H * a.W;
  // A (dY) k-row of this lane in instruction j: (wave + 4 j) (64 / LA) + lane / LA; its pixel
  // advances by 64 per K-tile.  B (X) k-rows likewise, with the pixel's (y, x) kept and
  // advanced incrementally (no divisions in the loop) for the neighbour's bounds.
  int cha[NA], pa[NA], chb[NB], pb[NB], pi[NB], py[NB], px[NB];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int kr = (wave + 4 * j) * (64 / LA) + lane / LA;
    cha[j] = ((lane % LA) ^ mimg_swz<WBM>(kr)) * 8;
    pa[j] = kt0 * 64 + kr;
  }
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int kr = (wave + 4 * j) * (64 / LB) + lane / LB;
    chb[j] = ((lane % LB) ^ mimg_swz<WBN>(kr)) * 8;
    const int p = kt0 * 64 + kr;
    pb[j] = p;
    const int q = p < a.P ? p : 0;
    pi[j] = q / HWo;
    const int rem = q - pi[j] * HWo;
    py[j] = rem / a.Wo;
    px[j] = rem - py[j] * a.Wo;
  }
  auto issue = [&](int kt) {
    char* buf = smem + (kt % S) * TILE;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int p = pa[j];
      dma16(p < a.P ? a.dy + (size_t)p * a.N + m0 + cha[j] : a.zero + cha[j], buf + (wave + 4 * j) * 1024);
      pa[j] = p + 64;
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int p = pb[j];
      const int yy = py[j] * a.st + dy_, xx = px[j] * a.st + dx_;
      const bool ok = p < a.P && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W;
      const long long nb = (long long)pi[j] * HW + (long long)yy * a.W + xx;  // the neighbour's flat pixel index
      dma16(ok ? a.x + (size_t)nb * a.C + c0 + chb[j] : a.zero + chb[j], buf + WBM * 128 + (wave + 4 * j) * 1024);
      // next K-tile: 64 output pixels on (row-major within the image; images are contiguous)
      pb[j] = p + 64;
      int x = px[j] + 64, y = py[j], im = pi[j];
      while (x >= a.Wo) {
        x -= a.Wo;
        if (++y == a.Ho) {
          y = 0;
          ++im;
        }
      }
      px[j] = x;
      py[j] = y;
      pi[j] = im;
    }
  };
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float csum[TM];
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) issue(s);
  for (int kt = 0; kt < nk; ++kt) {
    wait_ring<S, GW>(nk - 1 - kt);
    __builtin_amdgcn_s_barrier();
    if (kt + S - 1 < nk) issue(kt + S - 1);
    const char* cur = smem + (kt % S) * TILE;
    compute_tile<WBM, WBN, false, false, false>(cur, cur + WBM * 128, acc, csum, lane, wm, wn);
  }
  // lane holds dW[m0 + wm WBM/2 + 16 i + (lane & 15)][nn0 + wn WBN/2 + 16 j + 4 (lane >> 4) + 0..3]
  float* out = a.part + (size_t)split * a.N * NN;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm * (WBM / 2) + 16 * i + (lane & 15);
    float* row = out + (size_t)m * NN + nn0 + wn * (WBN / 2) + 4 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < TN; ++j)
      *reinterpret_cast<float4*>(row + 16 * j) = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
  }
}

// dW = sum of the slices' fp32 partials in a fixed order, written as bf16 or
// fp32.  A workgroup owns 16 float4 columns; its 16 thread groups sum the
// slices k = group (mod 16) in increasing k, then group 0 adds the 16 sums in
// group order (a weight with few output tiles is cut into up to 256 slices;
// this keeps the sum spread over the chip and short per thread).
__device__ __forceinline__ void wgrad_reduce_body(const float* __restrict__ part, int nsplit, long long n,
                                                  void* __restrict__ dw, int out_bf16, long long blk,
                                                  float4 (&red)[15][16]) {
  const int col = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const long long i = (blk * 16ll + col) * 4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n) {
    for (int k = grp; k < nsplit; k += 16) {
      const float4 v = *reinterpret_cast<const float4*>(part + (size_t)k * n + i);
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
  }
  if (grp) red[grp - 1][col] = s;
  __syncthreads();
  if (grp || i >= n) return;
#pragma unroll
  for (int g = 0; g < 15; ++g) {
    const float4 v = red[g][col];
    s.x += v.x;
    s.y += v.y;
    s.z += v.z;
    s.w += v.w;
  }
  if (out_bf16) {
    uint2 o;
    o.x = pack2bf(s.x, s.y);
    o.y = pack2bf(s.z, s.w);
    *reinterpret_cast<uint2*>(static_cast<uint16_t*>(dw) + i) = o;
  } else {
    *reinterpret_cast<float4*>(static_cast<float*>(dw) + i) = s;
  }
}

__global__ __launch_bounds__(256) void conv_wgrad_reduce_kernel(const float* __restrict__ part, int nsplit,
                                                                long long n, void* __restrict__ dw, int out_bf16) {
  __shared__ float4 red[15][16];
  wgrad_reduce_body(part, nsplit, n, dw, out_bf16, blockIdx.x, red);
}

// The slice sums of up to kWgRedBatch weight gradients in ONE launch (round 6:
// the training step defers every convolution's reduction to the end of the
// backward, src/rtdetr_moe/conv.py deferred_wgrads): descriptor q owns blocks
// [base[q], base[q + 1]); each block runs conv_wgrad_reduce_kernel's body, so
// every dW is bitwise what its own reduction launch writes.  The table
// travels as the kernel argument (no host-to-device copy inside a capture).
constexpr int kWgRedBatch = 48;
struct WgRedBatch {
  const float* part[kWgRedBatch];
  void* dw[kWgRedBatch];
  long long n[kWgRedBatch];
  int nsplit[kWgRedBatch];
  int base[kWgRedBatch + 1];
  int count, out_bf16;
};

__global__ __launch_bounds__(256) void conv_wgrad_reduce_batch_kernel(WgRedBatch b) {
  __shared__ float4 red[15][16];
  const int bid = blockIdx.x;
  int lo = 0, hi = b.count - 1;  // the last q with base[q] <= bid (uniform binary search)
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (b.base[mid] <= bid) lo = mid;
    else hi = mid - 1;
  }
  wgrad_reduce_body(b.part[lo], b.nsplit[lo], b.n[lo], b.dw[lo], b.out_bf16, bid - b.base[lo], red);
}

// (per device; a failure is reported through moe_last_error and the launch
// that follows fails its check_launch)
template <auto FN>
static void allow_lds_once(size_t bytes) {
  static unsigned long long done = 0;
  (void)allow_dyn_lds(reinterpret_cast<const void*>(FN), (int)bytes, &done, "conv: dynamic LDS");
}

// output size of a padding (KS - 1) / 2 convolution
static int conv_out(int n, int KS, int stride) { return (n + 2 * ((KS - 1) / 2) - KS) / stride + 1; }

static int conv_check(const void* const* ptrs, int np, int B, int H, int W, int C, int N, int KS, int stride,
                      const char* what, int cmul = 64) {
  if (KS != 1 && KS != 3) return fail(std::string(what) + ": kernel size must be 1 or 3");
  if (stride != 1 && !(stride == 2 && KS == 3)) return fail(std::string(what) + ": stride must be 1 (or 2 with KS 3)");
  if (B < 0 || H <= 0 || W <= 0) return fail(std::string(what) + ": bad B / H / W");
  if (C % cmul || N % cmul || C <= 0 || N <= 0)
    return fail(std::string(what) + ": channels must be positive multiples of " + std::to_string(cmul));
  if ((long long)B * H * W * (C > N ? C : N) >= (1ll << 31)) return fail(std::string(what) + ": tensor too large");
  for (int i = 0; i < np; ++i)
    if (ptrs[i] == nullptr || reinterpret_cast<uintptr_t>(ptrs[i]) % 16)
      return fail(std::string(what) + ": operands must be non-NULL and 16-B aligned");
  return 0;
}

constexpr int CV_STAGES = 2;

template <int KS, int BM, int BN, bool BT, bool PH, int WGM = 2, int WGN = 2, int ST = CV_STAGES, bool AR = false,
          int KT = 64, bool EXT = false>
static void launch_fwd_n(ConvArgs a, hipStream_t stream, ProfScope& prof) {
  constexpr size_t ring = ST * (AR ? BN : BM + BN) * KT * 2;
  // the epilogue's output image (and statistics rows) reuse the ring's LDS
  constexpr size_t lds = ring > (size_t)BM * BN * 2 ? ring : (size_t)BM * BN * 2;
  static_assert(2 * (64 * WGM * WGN / (BN / 8)) * BN * 4 <= lds, "statistics rows exceed the LDS");
  static_assert(lds <= 160 * 1024, "ring exceeds the CU's LDS");
  static_assert(!(BT && BN > 128), "the in-place (MN-contiguous) weight image takes 64 or 128 columns");
  allow_lds_once<conv_fwd_kernel<KS, ST, BM, BN, BT, PH, WGM, WGN, AR, KT, EXT>>(lds);
  a.mt_n = (a.P + BM - 1) / BM;
  const int NT = (a.N + BN - 1) / BN;
  const int grid = ((a.mt_n + 7) / 8) * 8 * NT;
  MOE_LAUNCH(prof, (conv_fwd_kernel<KS, ST, BM, BN, BT, PH, WGM, WGN, AR, KT, EXT>), dim3(grid),
             dim3(64 * WGM * WGN), lds, stream, a);
}

// The 8-wave big tile: 256 x 128, 4 x 2 waves of 64 x 64 (the 128 x 128
// tile's wave tile), one workgroup (two waves per SIMD) per CU with a 96 KiB
// ring.  Per 64-deep K-tile it stages 25 % fewer LDS bytes per flop than the
// 128 x 128 tile (the L2 -> LDS stream bounds the 3x3 layers).  (A 256 x 256
// tile of 2 x 4 waves needs 128 x 64 accumulators per wave: it spills at the
// 256 registers two waves per SIMD leave.)  Returns false when the shape does
// not take it.
template <int KS, bool BT, bool PH>
static bool launch_fwd_big(const ConvArgs& a, hipStream_t stream, ProfScope& prof, int mode) {
  // (a 256 x 256 tile of 2 x 2 waves, 128 x 128 per wave at one workgroup per CU, measured 1.2-4x
  // slower at every C2 shape: profiles/r04/conv/conv_bench_256x256_ab.jsonl)
  if (a.N % 128 != 0) return false;
  switch (mode) {
    case 1: launch_fwd_n<KS, 256, 128, BT, PH, 4, 2>(a, stream, prof); return true;
    // deeper rings (round 5): K-tiles in flight per CU, not the tile shape, bound these layers
    case 2: launch_fwd_n<KS, 256, 128, BT, PH, 4, 2, 3>(a, stream, prof); return true;    // 144 KiB, 1 WG / CU
    case 3: launch_fwd_n<KS, 128, 128, BT, PH, 2, 2, 3>(a, stream, prof); return true;    //  96 KiB, 1 WG / CU
    case 4: launch_fwd_n<KS, 128, 128, BT, PH, 2, 2, 4>(a, stream, prof); return true;    // 128 KiB, 1 WG / CU
    case 5: launch_fwd_n<KS, 128, 128, BT, PH, 4, 2, 4>(a, stream, prof); return true;    // 8 waves of 32 x 64
    default: return false;
  }
}

// The 32-deep K-tile with a 2-deep ring (32 KiB of LDS, 4 workgroups per CU
// against 2) pays where the K loop is short and the grid long: 1x1
// convolutions with at most 512 input channels over >= 16 M outputs, where
// the epilogues of some workgroups overlap the main loops of others
// (tools/conv_bench.py, gpurun_out/r5v: e.g. 128 -> 512 at 92 x 160 43.6 ->
// 35.7 us, the 64 -> 256 stage-1 data gradient 80.8 -> 69.0 us).  The 3x3
// layers (K = 9 C) and 1x1 layers with 1024+ input channels are slower with
// it (the per-barrier work halves): they keep the 64-deep tile.
static int k32_auto(int KS, const ConvArgs& a) {
  return KS == 1 && a.C <= 512 && (long long)a.P * a.N >= 16000000LL ? 1 : 0;
}

// output-channel tiles of 128, or 64 for 64-channel outputs (ResNet stage 1);
// "conv_areg" 1: the 128-row tiles with the A operand in registers (AR)
template <int KS, int BM, bool BT, bool PH>
static void launch_fwd(const ConvArgs& a, hipStream_t stream, ProfScope& prof) {
  if constexpr (BM == 128) {
    if (g_conv_areg == 1 && a.C % 64 == 0 && a.N % 64 == 0) {
      if (a.N % 128 == 0) launch_fwd_n<KS, BM, 128, BT, PH, 2, 2, 2, true>(a, stream, prof);
      else launch_fwd_n<KS, BM, 64, BT, PH, 2, 2, 2, true>(a, stream, prof);
      return;
    }
  }
  if constexpr (BM == 128 || BM == 64) {
    const int k32 = a.C % 64 ? (g_conv_k32 >= 2 ? g_conv_k32 : 1) : (g_conv_k32 >= 0 ? g_conv_k32 : k32_auto(KS, a));
    if (k32 >= 1 && k32 <= 3) {  // 32-deep K-tiles, ring depth 2-4
      const bool w = a.N % 128 == 0;
      switch (k32) {
        case 1: w ? launch_fwd_n<KS, BM, 128, BT, PH, 2, 2, 2, false, 32>(a, stream, prof)
                  : launch_fwd_n<KS, BM, 64, BT, PH, 2, 2, 2, false, 32>(a, stream, prof); break;
        case 2: w ? launch_fwd_n<KS, BM, 128, BT, PH, 2, 2, 3, false, 32>(a, stream, prof)
                  : launch_fwd_n<KS, BM, 64, BT, PH, 2, 2, 3, false, 32>(a, stream, prof); break;
        default: w ? launch_fwd_n<KS, BM, 128, BT, PH, 2, 2, 4, false, 32>(a, stream, prof)
                   : launch_fwd_n<KS, BM, 64, BT, PH, 2, 2, 4, false, 32>(a, stream, prof); break;
      }
      return;
    }
  }
  if (a.N % 128 == 0) launch_fwd_n<KS, BM, 128, BT, PH>(a, stream, prof);
  else launch_fwd_n<KS, BM, 64, BT, PH>(a, stream, prof);
}

// tile rows: 128 (two workgroups per CU); 64 when 128-row tiles would leave
// the chip under-filled (< 1.5 workgroups per CU); 256 rows of 4 waves (one
// workgroup per CU) measured slower at every C2 shape
// rows per partial of rtdetr_conv_fwd_stats (the forward's M-tile height): the
// statistics come as ceil(B Ho Wo / rows) partial rows of [2][N]
static int fwd_bm(long long P, int N) {
  int bm = g_conv_bm;
  if (bm != 64 && bm != 128 && bm != 256) bm = (long long)((P + 127) / 128) * (N / (N % 128 == 0 ? 128 : 64)) < 384 ? 64 : 128;
  return bm;
}

template <int BM, int BN, int WGM, int WGN, int BS>
static void launch_halo(ConvArgs a, hipStream_t stream, ProfScope& prof) {
  constexpr int GI = (BM + 2 + 7) / 8;
  constexpr size_t lds = 3 * GI * 1024 + BS * BN * 128 + 128;
  allow_lds_once<conv3x3_halo_kernel<BM, BN, WGM, WGN, BS>>(lds);
  a.mt_n = (a.P + BM - 1) / BM;
  const int NT = a.N / BN;
  const int grid = ((a.mt_n + 7) / 8) * 8 * NT;
  MOE_LAUNCH(prof, (conv3x3_halo_kernel<BM, BN, WGM, WGN, BS>), dim3(grid), dim3(64 * WGM * WGN), lds, stream, a);
}

static void launch_8ph(ConvArgs a, int KS, hipStream_t stream, ProfScope& prof) {
  constexpr size_t lds = 2 * 2 * 256 * 128;  // 128 KiB (the epilogue's 256 x 256 bf16 image fits)
  a.mt_n = (a.P + 255) / 256;
  const int grid = ((a.mt_n + 7) / 8) * 8 * (a.N / 256);
  if (KS == 3) {
    allow_lds_once<conv_8ph_kernel<3>>(lds);
    MOE_LAUNCH(prof, conv_8ph_kernel<3>, dim3(grid), dim3(512), lds, stream, a);
  } else {
    allow_lds_once<conv_8ph_kernel<1>>(lds);
    MOE_LAUNCH(prof, conv_8ph_kernel<1>, dim3(grid), dim3(512), lds, stream, a);
  }
}

// the 8-phase 256 x 256 kernel's operands: whole 256-column N tiles, 64-channel
// slices, no statistics epilogue; "conv_8ph" 1 forces it where eligible, -1
// (automatic) takes it for grids of at least one wave of the chip
static bool ph8_ok(int C, int N, int KS) { return N % 256 == 0 && C % 64 == 0 && (KS * KS * (C / 64)) % 2 == 0; }
static bool ph8_auto(long long P, int N, int KS) { return KS == 3 && ((P + 255) / 256) * (N / 256) >= 256; }
// whether a forward (not PH / BT) of these operands takes conv_8ph_kernel
static bool ph8_takes(long long P, int C, int N, int KS) {
  return g_conv_8ph != 0 && ph8_ok(C, N, KS) && (g_conv_8ph > 0 || ph8_auto(P, N, KS));
}

// the halo kernel's operands: 3x3, stride 1 (forward, or the stride-1 data
// gradient with the K-contiguous flipped weight), 64-channel multiples, whole
// 128-column N tiles
static bool halo_ok(const ConvArgs& a, int KS) {
  return KS == 3 && a.st == 1 && a.sh == 0 && a.Hs == a.H && a.Ws == a.W && a.C % 64 == 0 && a.N % 128 == 0 &&
         a.stats == nullptr;
}

template <bool BT, bool PH = false>
static void launch_fwd_any(const ConvArgs& a, int KS, hipStream_t stream, ProfScope& prof) {
  if constexpr (!BT && !PH) {
    if (ph8_takes(a.P, a.C, a.N, KS)) {
      launch_8ph(a, KS, stream, prof);
      return;
    }
    if (g_conv_halo > 0 && halo_ok(a, KS)) {
      if (g_conv_halo == 2) launch_halo<128, 128, 2, 2, 2>(a, stream, prof);
      else launch_halo<256, 128, 4, 2, 3>(a, stream, prof);
      return;
    }
  }
  const bool c32 = a.C % 64 != 0 || a.N % 64 != 0;  // 32-channel multiples: the 32-deep, 64-wide tiles only
  if (g_conv_big > 0 && !c32) {  // "conv_big" 1: the 8-wave 256 x 128 tile where N % 128 == 0
    if constexpr (PH) {
      if (launch_fwd_big<3, BT, true>(a, stream, prof, g_conv_big)) return;
    } else {
      if (KS == 3 ? launch_fwd_big<3, BT, false>(a, stream, prof, g_conv_big)
                  : launch_fwd_big<1, BT, false>(a, stream, prof, g_conv_big))
        return;
    }
  }
  int bm = fwd_bm(a.P, a.N);
  if (c32 && bm == 256) bm = 128;
  if constexpr (PH) {  // 3x3 only
    if (bm == 256) launch_fwd<3, 256, BT, true>(a, stream, prof);
    else if (bm == 64) launch_fwd<3, 64, BT, true>(a, stream, prof);
    else launch_fwd<3, 128, BT, true>(a, stream, prof);
  } else if (KS == 3) {
    if (bm == 256) launch_fwd<3, 256, BT, false>(a, stream, prof);
    else if (bm == 64) launch_fwd<3, 64, BT, false>(a, stream, prof);
    else launch_fwd<3, 128, BT, false>(a, stream, prof);
  } else {
    if (bm == 256) launch_fwd<1, 256, BT, false>(a, stream, prof);
    else if (bm == 64) launch_fwd<1, 64, BT, false>(a, stream, prof);
    else launch_fwd<1, 128, BT, false>(a, stream, prof);
  }
}

// The forward with the extended epilogue (rtdetr_conv_fwd_act: the evaluation
// forward's folded layers): the 8-phase kernel where it applies, else the
// default tiles -- 64 / 128 rows (fwd_bm), 32-deep K-tiles where k32_auto takes
// them -- instantiated with EXT; the A/B tuning knobs are not consulted.
template <int KS>
static void launch_fwd_ext(const ConvArgs& a, hipStream_t stream, ProfScope& prof) {
  if (ph8_takes(a.P, a.C, a.N, KS)) {
    launch_8ph(a, KS, stream, prof);
    return;
  }
  const bool w = a.N % 128 == 0;
  const bool k32 = a.C % 64 != 0 || a.N % 64 != 0 || k32_auto(KS, a);
  if (fwd_bm(a.P, a.N) == 64) {
    if (k32) w ? launch_fwd_n<KS, 64, 128, false, false, 2, 2, 2, false, 32, true>(a, stream, prof)
             : launch_fwd_n<KS, 64, 64, false, false, 2, 2, 2, false, 32, true>(a, stream, prof);
    else w ? launch_fwd_n<KS, 64, 128, false, false, 2, 2, CV_STAGES, false, 64, true>(a, stream, prof)
           : launch_fwd_n<KS, 64, 64, false, false, 2, 2, CV_STAGES, false, 64, true>(a, stream, prof);
  } else {
    if (k32) w ? launch_fwd_n<KS, 128, 128, false, false, 2, 2, 2, false, 32, true>(a, stream, prof)
             : launch_fwd_n<KS, 128, 64, false, false, 2, 2, 2, false, 32, true>(a, stream, prof);
    else w ? launch_fwd_n<KS, 128, 128, false, false, 2, 2, CV_STAGES, false, 64, true>(a, stream, prof)
           : launch_fwd_n<KS, 128, 64, false, false, 2, 2, CV_STAGES, false, 64, true>(a, stream, prof);
  }
}

template <int KS, int S, int WBM, int WBN>
static void launch_wgrad_t(const ConvWgArgs& a, hipStream_t stream, ProfScope& prof) {
  constexpr size_t lds = S * (WBM + WBN) * 128;
  allow_lds_once<conv_wgrad_kernel<KS, S, WBM, WBN>>(lds);
  const int tiles = (a.N / WBM) * (KS * KS * a.C / WBN);
  const int grid = (tiles * a.nsplit + 7) / 8 * 8;
  MOE_LAUNCH(prof, (conv_wgrad_kernel<KS, S, WBM, WBN>), dim3(grid), dim3(256), lds, stream, a);
}
template <int KS, int S>
static void launch_wgrad_s(const ConvWgArgs& a, hipStream_t stream, ProfScope& prof) {
  const int bm = wg_bm(a.N), bn = wg_bn(a.C);
  if (bm == 128 && bn == 128) launch_wgrad_t<KS, S, 128, 128>(a, stream, prof);
  else if (bm == 128) launch_wgrad_t<KS, S, 128, 64>(a, stream, prof);
  else if (bn == 128) launch_wgrad_t<KS, S, 64, 128>(a, stream, prof);
  else launch_wgrad_t<KS, S, 64, 64>(a, stream, prof);
}

// 2-deep ring (64 KiB, two workgroups per CU): deeper rings (1 per CU)
// measured no faster where the grid fits one round and up to 2x slower where
// it does not
template <int KS>
static void launch_wgrad(const ConvWgArgs& a, hipStream_t stream, ProfScope& prof) {
  const int s = g_conv_wg_stages >= 2 && g_conv_wg_stages <= 4 ? g_conv_wg_stages : 2;
  if (s == 2) launch_wgrad_s<KS, 2>(a, stream, prof);
  else if (s == 3) launch_wgrad_s<KS, 3>(a, stream, prof);
  else launch_wgrad_s<KS, 4>(a, stream, prof);
}

}  // namespace moe

using namespace moe;

static bool aligned16(const void* p) { return p == nullptr || reinterpret_cast<uintptr_t>(p) % 16 == 0; }

extern "C" int rtdetr_conv_fwd(const void* x, const void* w, void* y, const void* zero, int B, int H, int W, int C,
                               int N, int KS, int stride, const float* bias, const void* resid, int relu,
                               hipStream_t stream) {
  const void* ptrs[4] = {x, w, y, zero};
  // (the forward alone also takes 32-channel multiples: 32-deep K-tiles, a partial N tile)
  if (int rc = conv_check(ptrs, 4, B, H, W, C, N, KS, stride, "rtdetr_conv_fwd", 32)) return rc;
  if (!aligned16(bias) || !aligned16(resid)) return fail("rtdetr_conv_fwd: bias / resid must be 16-B aligned");
  if (B == 0) return 0;
  const int Ho = conv_out(H, KS, stride), Wo = conv_out(W, KS, stride);
  ConvArgs a{static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(w), static_cast<uint16_t*>(y),
             static_cast<const uint16_t*>(zero), B, Ho, Wo, C, N, B * Ho * Wo, 0, H, W, stride, 0,
             bias, static_cast<const uint16_t*>(resid), nullptr, relu ? 1 : 0};
  const double P = a.P;
  ProfScope prof(stream, PROF_CONV, 2.0 * ((double)B * H * W * C + P * (N + (resid ? N : 0))) + 2.0 * N * KS * KS * C,
                 false, 0.0, 2.0 * P * N * KS * KS * C);
  launch_fwd_any<false>(a, KS, stream, prof);
  return check_launch("rtdetr_conv_fwd");
}

extern "C" int rtdetr_conv_fwd_act(const void* x, const void* w, void* y, const void* zero, int B, int H, int W,
                                   int C, int N, int KS, int stride, const float* bias, const void* resid, int act,
                                   int resid_post, long long y_img_rows, long long y_row_off, hipStream_t stream) {
  const void* ptrs[4] = {x, w, y, zero};
  if (int rc = conv_check(ptrs, 4, B, H, W, C, N, KS, stride, "rtdetr_conv_fwd_act", 32)) return rc;
  if (!aligned16(bias) || !aligned16(resid)) return fail("rtdetr_conv_fwd_act: bias / resid must be 16-B aligned");
  if (act < 0 || act > 2) return fail("rtdetr_conv_fwd_act: act must be 0 (none), 1 (ReLU) or 2 (SiLU)");
  if (resid_post && resid == nullptr) return fail("rtdetr_conv_fwd_act: resid_post without resid");
  if (B == 0) return 0;
  const int Ho = conv_out(H, KS, stride), Wo = conv_out(W, KS, stride);
  ConvArgs a{static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(w), static_cast<uint16_t*>(y),
             static_cast<const uint16_t*>(zero), B, Ho, Wo, C, N, B * Ho * Wo, 0, H, W, stride, 0,
             bias, static_cast<const uint16_t*>(resid), nullptr, act};
  a.resid_post = resid_post ? 1 : 0;
  if (y_img_rows != 0 && (y_img_rows < (long long)Ho * Wo || y_row_off < 0 || y_row_off + (long long)Ho * Wo > y_img_rows))
    return fail("rtdetr_conv_fwd_act: the output rows [y_row_off, y_row_off + Ho Wo) must lie within y_img_rows");
  a.yS = y_img_rows;
  a.yoff = y_row_off;
  const double P = a.P;
  ProfScope prof(stream, PROF_CONV, 2.0 * ((double)B * H * W * C + P * (N + (resid ? N : 0))) + 2.0 * N * KS * KS * C,
                 false, 0.0, 2.0 * P * N * KS * KS * C);
  if (KS == 3) launch_fwd_ext<3>(a, stream, prof);
  else launch_fwd_ext<1>(a, stream, prof);
  return check_launch("rtdetr_conv_fwd_act");
}

extern "C" int rtdetr_conv_fwd_stats_rows(int B, int H, int W, int C, int N, int KS, int stride) {
  if (B <= 0 || H <= 0 || W <= 0 || N <= 0 || (KS != 1 && KS != 3) || (stride != 1 && stride != 2)) return 0;
  const long long P = (long long)B * conv_out(H, KS, stride) * conv_out(W, KS, stride);
  if (ph8_takes(P, C, N, KS)) return 256;  // the 8-phase kernel's 256-row M-tiles
  return fwd_bm(P, N);
}

extern "C" int rtdetr_conv_fwd_stats(const void* x, const void* w, void* y, const void* zero, int B, int H, int W,
                                     int C, int N, int KS, int stride, float* part, hipStream_t stream) {
  const void* ptrs[4] = {x, w, y, zero};
  if (int rc = conv_check(ptrs, 4, B, H, W, C, N, KS, stride, "rtdetr_conv_fwd_stats")) return rc;
  if (part == nullptr || !aligned16(part)) return fail("rtdetr_conv_fwd_stats: part must be 16-B aligned");
  if (B == 0) return 0;
  const int Ho = conv_out(H, KS, stride), Wo = conv_out(W, KS, stride);
  ConvArgs a{static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(w), static_cast<uint16_t*>(y),
             static_cast<const uint16_t*>(zero), B, Ho, Wo, C, N, B * Ho * Wo, 0, H, W, stride, 0,
             nullptr, nullptr, nullptr, 0};
  a.stats = part;
  const double P = a.P;
  ProfScope prof(stream, PROF_CONV, 2.0 * ((double)B * H * W * C + P * N) + 2.0 * N * KS * KS * C, false, 0.0,
                 2.0 * P * N * KS * KS * C);
  if (ph8_takes(a.P, C, N, KS)) {  // 256-row partials (rtdetr_conv_fwd_stats_rows says so)
    launch_8ph(a, KS, stream, prof);
    return check_launch("rtdetr_conv_fwd_stats");
  }
  const int bm = fwd_bm(a.P, N);  // (the default tiles: never the A/B "conv_big" shapes)
  if (KS == 3) {
    if (bm == 256) launch_fwd<3, 256, false, false>(a, stream, prof);
    else if (bm == 64) launch_fwd<3, 64, false, false>(a, stream, prof);
    else launch_fwd<3, 128, false, false>(a, stream, prof);
  } else {
    if (bm == 256) launch_fwd<1, 256, false, false>(a, stream, prof);
    else if (bm == 64) launch_fwd<1, 64, false, false>(a, stream, prof);
    else launch_fwd<1, 128, false, false>(a, stream, prof);
  }
  return check_launch("rtdetr_conv_fwd_stats");
}

extern "C" long long rtdetr_conv_dgrad_workspace(int B, int H, int W, int C, int N, int KS) {
  // writing W' costs a launch (~2-3 us in a graph) plus 4 B per weight and
  // buys the K-contiguous operand image, up to ~10 % faster than reading W in
  // place (MN-contiguous): measured to pay from ~64 Ki pixels, or from
  // ~25 GFLOP for 3x3 (tools/conv_bench.py conv_dgrad_flip=0/1)
  const double P = (double)B * H * W;
  bool flip = P >= 65536 || (KS == 3 && 2.0 * P * N * KS * KS * C >= 2.5e10);
  if (g_conv_dgrad_flip == 0 || g_conv_dgrad_flip == 1) flip = g_conv_dgrad_flip == 1;
  return flip ? 2ll * N * KS * KS * C : 0;
}

static int conv_dgrad_impl(const void* dy, const void* w, void* work, bool preflipped, void* dx, const void* zero,
                           int B, int H, int W, int C, int N, int KS, int stride, const void* add,
                           const void* relu_mask, hipStream_t stream) {
  const void* ptrs[4] = {dy, w, dx, zero};
  if (int rc = conv_check(ptrs, 4, B, H, W, C, N, KS, stride, "rtdetr_conv_dgrad")) return rc;
  if (!aligned16(relu_mask) || !aligned16(add)) return fail("rtdetr_conv_dgrad: add / relu_mask must be 16-B aligned");
  const bool flip = rtdetr_conv_dgrad_workspace(B, H, W, C, N, KS) > 0;
  if (preflipped && !flip) return fail("rtdetr_conv_dgrad_preflipped: this shape reads W in place (no flip)");
  if (flip && (work == nullptr || reinterpret_cast<uintptr_t>(work) % 16))
    return fail("rtdetr_conv_dgrad: this shape needs a 16-B aligned workspace of rtdetr_conv_dgrad_workspace() bytes");
  if (B == 0) return 0;
  // the forward GEMM over dY [B Ho Wo][N] with W' (stride 2: dX pixel (y, x) reads dY at ((y + dy) / 2,
  // (x + dx) / 2) when both are even)
  const int Ho = conv_out(H, KS, stride), Wo = conv_out(W, KS, stride);
  ConvArgs a{static_cast<const uint16_t*>(dy), static_cast<const uint16_t*>(w), static_cast<uint16_t*>(dx),
             static_cast<const uint16_t*>(zero), B, H, W, N, C, B * H * W, 0, Ho, Wo, 1, stride == 2 ? 1 : 0,
             nullptr, static_cast<const uint16_t*>(add), static_cast<const uint16_t*>(relu_mask), 0};
  const double P = a.P;
  const double Pdy = (double)B * Ho * Wo;
  if (flip && !preflipped) {
    const long long total = (long long)N * C * KS * KS;
    {
      ProfScope prof(stream, PROF_CONV, 4.0 * total);
      MOE_LAUNCH(prof, conv_weight_flip_kernel, dim3(C / 64, N / 64, KS * KS), dim3(256), 0, stream,
                 static_cast<const uint16_t*>(w), static_cast<uint16_t*>(work), N, C, KS);
      if (int rc = check_launch("rtdetr_conv_dgrad (flip)")) return rc;
    }
  }
  if (flip) a.w = static_cast<const uint16_t*>(work);
  // algorithmic bytes / flops (the stride-2 zero-row taps are not counted)
  const double bytes = 2.0 * (P * (C + (relu_mask ? C : 0) + (add ? C : 0)) + Pdy * N) + 2.0 * N * KS * KS * C;
  const double flops = 2.0 * Pdy * N * KS * KS * C;
  if (stride == 2 && g_conv_dgrad_phase != 0) {
    // one launch per parity class (ry, rx) of the dX pixels, each over its valid taps only
    for (int ry = 0; ry < 2; ++ry)
      for (int rx = 0; rx < 2; ++rx) {
        ConvArgs c = a;
        c.H = (H - ry + 1) / 2;
        c.W = (W - rx + 1) / 2;
        c.P = B * c.H * c.W;
        c.st = 1;
        c.sh = 0;
        c.ry = ry;
        c.rx = rx;
        c.Hd = H;
        c.Wd = W;
        if (c.P == 0) continue;
        ProfScope prof(stream, PROF_CONV, bytes * c.P / P, false, 0.0, flops * (1 + ry) * (1 + rx) * c.P / (9.0 * Pdy));
        if (flip) launch_fwd_any<false, true>(c, KS, stream, prof);
        else launch_fwd_any<true, true>(c, KS, stream, prof);
        if (int rc = check_launch("rtdetr_conv_dgrad (class)")) return rc;
      }
    return 0;
  }
  ProfScope prof(stream, PROF_CONV, bytes, false, 0.0, flops);
  if (flip) launch_fwd_any<false>(a, KS, stream, prof);
  else launch_fwd_any<true>(a, KS, stream, prof);
  return check_launch("rtdetr_conv_dgrad");
}

extern "C" int rtdetr_conv_dgrad(const void* dy, const void* w, void* work, void* dx, const void* zero, int B, int H,
                                 int W, int C, int N, int KS, int stride, const void* add, const void* relu_mask,
                                 hipStream_t stream) {
  return conv_dgrad_impl(dy, w, work, false, dx, zero, B, H, W, C, N, KS, stride, add, relu_mask, stream);
}

extern "C" int rtdetr_conv_dgrad_preflipped(const void* dy, const void* w, const void* wflip, void* dx,
                                            const void* zero, int B, int H, int W, int C, int N, int KS, int stride,
                                            const void* add, const void* relu_mask, hipStream_t stream) {
  if (wflip == nullptr) return fail("rtdetr_conv_dgrad_preflipped: NULL flipped weight");
  return conv_dgrad_impl(dy, w, const_cast<void*>(wflip), true, dx, zero, B, H, W, C, N, KS, stride, add, relu_mask,
                         stream);
}

extern "C" int rtdetr_conv_weight_flip_multi(const void* table, int n, int total_blocks, hipStream_t stream) {
  if (n < 0 || total_blocks < 0) return fail("rtdetr_conv_weight_flip_multi: n, total_blocks must be >= 0");
  if (n == 0 || total_blocks == 0) return 0;
  if (table == nullptr || reinterpret_cast<uintptr_t>(table) % 16)
    return fail("rtdetr_conv_weight_flip_multi: table must be a 16-B aligned device array");
  ProfScope prof(stream, PROF_CONV, 64.0 * 64.0 * 4.0 * total_blocks);
  MOE_LAUNCH(prof, conv_weight_flip_multi_kernel, dim3(total_blocks), dim3(256), 0, stream,
             static_cast<const FlipDesc*>(table), n);
  return check_launch("rtdetr_conv_weight_flip_multi");
}

extern "C" int rtdetr_conv_wgrad_splits(int B, int H, int W, int C, int N, int KS) {
  // as many pixel slices as keep tiles x slices <= 512 (every workgroup
  // resident at once, two per CU: a second round on a few CUs doubles the
  // time), each slice >= 8 pixel K-tiles, <= 256 (each slice costs an fp32
  // partial of the weight; the stage-1 1x1 weights are 1-2 tiles)
  if (N <= 0 || C <= 0 || N % 64 || C % 64) return 1;
  const long long tiles = (long long)(N / wg_bm(N)) * (KS * KS * C / wg_bn(C));
  const long long ktot = ((long long)B * H * W + 63) / 64;
  long long s = 512 / std::max(1ll, tiles);
  s = std::min(s, std::max(1ll, ktot / 8));
  s = std::min(s, 256ll);
  if (g_conv_wg_splits > 0) s = std::min<long long>(g_conv_wg_splits, std::max(1ll, ktot));
  return (int)std::max(1ll, s);
}

extern "C" int rtdetr_conv_wgrad_part(const void* dy, const void* x, float* part, int nsplit, const void* zero,
                                      int B, int H, int W, int C, int N, int KS, int stride, hipStream_t stream) {
  const void* ptrs[4] = {dy, x, part, zero};
  if (int rc = conv_check(ptrs, 4, B, H, W, C, N, KS, stride, "rtdetr_conv_wgrad")) return rc;
  if (nsplit < 1 || nsplit > 256) return fail("rtdetr_conv_wgrad: nsplit must be 1..256");
  const int Ho = conv_out(H, KS, stride), Wo = conv_out(W, KS, stride);
  ConvWgArgs a{static_cast<const uint16_t*>(dy), static_cast<const uint16_t*>(x), part,
               static_cast<const uint16_t*>(zero), B, H, W, C, N, B * Ho * Wo, nsplit, 0, Ho, Wo, stride};
  const int ktot = (a.P + 63) / 64;
  a.kt_per = (ktot + nsplit - 1) / nsplit;
  const long long nw = (long long)N * KS * KS * C;
  const double P = a.P;
  ProfScope prof(stream, PROF_CONV, 2.0 * ((double)B * H * W * C + P * N) + 4.0 * nsplit * nw, false, 0.0,
                 2.0 * P * nw);
  if (KS == 3) launch_wgrad<3>(a, stream, prof);
  else launch_wgrad<1>(a, stream, prof);
  return check_launch("rtdetr_conv_wgrad");
}

extern "C" int rtdetr_conv_wgrad(const void* dy, const void* x, float* part, int nsplit, void* dw, int out_bf16,
                                 const void* zero, int B, int H, int W, int C, int N, int KS, int stride,
                                 hipStream_t stream) {
  if (dw == nullptr || reinterpret_cast<uintptr_t>(dw) % 16) return fail("rtdetr_conv_wgrad: dw NULL or unaligned");
  if (int rc = rtdetr_conv_wgrad_part(dy, x, part, nsplit, zero, B, H, W, C, N, KS, stride, stream)) return rc;
  const long long nw = (long long)N * KS * KS * C;
  ProfScope prof(stream, PROF_CONV, 4.0 * nsplit * nw + (out_bf16 ? 2.0 : 4.0) * nw);
  MOE_LAUNCH(prof, conv_wgrad_reduce_kernel, dim3((unsigned)((nw / 4 + 15) / 16)), dim3(256), 0, stream, part,
             nsplit, nw, dw, out_bf16);
  return check_launch("rtdetr_conv_wgrad (reduce)");
}

extern "C" int rtdetr_conv_wgrad_reduce_batch(int n, const float* const* parts, const int* nsplits,
                                              const long long* nws, void* const* dws, int out_bf16,
                                              hipStream_t stream) {
  if (n < 1 || n > kWgRedBatch || parts == nullptr || nsplits == nullptr || nws == nullptr || dws == nullptr)
    return fail("rtdetr_conv_wgrad_reduce_batch: 1..48 weights, non-NULL arrays");
  WgRedBatch b{};
  b.count = n;
  b.out_bf16 = out_bf16 ? 1 : 0;
  long long blocks = 0;
  double bytes = 0.0;
  for (int q = 0; q < n; ++q) {
    if (parts[q] == nullptr || dws[q] == nullptr || nsplits[q] < 1 || nsplits[q] > 256 || nws[q] < 4 ||
        nws[q] % 4 || (reinterpret_cast<uintptr_t>(parts[q]) | reinterpret_cast<uintptr_t>(dws[q])) % 16)
      return fail("rtdetr_conv_wgrad_reduce_batch: bad descriptor (16-B aligned, nsplit 1..256, n % 4 == 0)");
    b.part[q] = parts[q];
    b.dw[q] = dws[q];
    b.n[q] = nws[q];
    b.nsplit[q] = nsplits[q];
    b.base[q] = (int)blocks;
    blocks += (nws[q] / 4 + 15) / 16;
    bytes += 4.0 * nsplits[q] * nws[q] + (out_bf16 ? 2.0 : 4.0) * nws[q];
  }
  if (blocks > 0x7fffffffLL) return fail("rtdetr_conv_wgrad_reduce_batch: too many blocks");
  b.base[n] = (int)blocks;
  ProfScope prof(stream, PROF_CONV, bytes);
  MOE_LAUNCH(prof, conv_wgrad_reduce_batch_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, b);
  return check_launch("rtdetr_conv_wgrad_reduce_batch");
}

extern "C" int rtdetr_conv3x3_direct_fwd(const void* x, const float* wf, const float* bias, void* y, int B, int H,
                                         int W, int C, int N, int stride, int relu, hipStream_t stream) {
  if (C != 3 || N != 32) return fail("rtdetr_conv3x3_direct_fwd: takes C = 3 -> N = 32 (the ResNet-D stem)");
  if (stride != 1 && stride != 2) return fail("rtdetr_conv3x3_direct_fwd: stride 1 or 2");
  if (B < 0 || H <= 0 || W <= 0) return fail("rtdetr_conv3x3_direct_fwd: bad B / H / W");
  if (B == 0) return 0;
  if (x == nullptr || wf == nullptr || y == nullptr || reinterpret_cast<uintptr_t>(y) % 16)
    return fail("rtdetr_conv3x3_direct_fwd: x, wf non-NULL, y 16-B aligned");
  const int Ho = conv_out(H, 3, stride), Wo = conv_out(W, 3, stride);
  const long long P = (long long)B * Ho * Wo;
  const long long blocks = (P + 255) / 256;
  if (blocks > 0x7fffffffLL) return fail("rtdetr_conv3x3_direct_fwd: too many pixels");
  ProfScope prof(stream, PROF_CONV, 2.0 * ((double)B * H * W * C + P * N), false, 0.0, 2.0 * P * N * 9 * C);
  MOE_LAUNCH(prof, (conv_direct_kernel<32, 3>), dim3((unsigned)blocks), dim3(256), 0, stream,
             static_cast<const uint16_t*>(x), wf, bias, static_cast<uint16_t*>(y), B, H, W, Ho, Wo, stride, relu);
  return check_launch("rtdetr_conv3x3_direct_fwd");
}

extern "C" int rtdetr_conv_set_tuning(const char* key, int value) {
  if (key == nullptr) return fail("rtdetr_conv_set_tuning: key is NULL");
  if (std::string(key) == "conv_bm") {
    g_conv_bm = value;
    return 0;
  }
  if (std::string(key) == "conv_8ph") {
    g_conv_8ph = value;
    return 0;
  }
  if (std::string(key) == "conv_halo") {
    g_conv_halo = value;
    return 0;
  }
  if (std::string(key) == "conv_big") {
    g_conv_big = value;
    return 0;
  }
  if (std::string(key) == "conv_wg_stages") {
    g_conv_wg_stages = value;
    return 0;
  }
  if (std::string(key) == "conv_wg_splits") {
    g_conv_wg_splits = value;
    return 0;
  }
  if (std::string(key) == "conv_dgrad_flip") {
    g_conv_dgrad_flip = value;
    return 0;
  }
  if (std::string(key) == "conv_dgrad_phase") {
    g_conv_dgrad_phase = value;
    return 0;
  }
  if (std::string(key) == "conv_areg") {
    g_conv_areg = value;
    return 0;
  }
  if (std::string(key) == "conv_k32") {
    if (value < -1 || value > 3) return fail("rtdetr_conv_set_tuning: conv_k32 takes -1 (auto) or 0-3");
    g_conv_k32 = value;
    return 0;
  }
  return fail(std::string("rtdetr_conv_set_tuning: unknown key ") + key);
}
