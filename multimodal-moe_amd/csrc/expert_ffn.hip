// Fused expert FFN forward on bf16 MFMA, gfx950:
//   H  = relu(X . W1_g^T + b1_g)   written once to HBM (the backward's mask and
//                                  dW2 operand) and never read back here
//   Yp = H . W2_g^T + b2_g
// for the routed rows of every expert g in ONE launch, where the two-launch
// path (grouped_gemm.hip) writes H and then streams all of it back in.
//
// Work unit: one workgroup (4 waves) per 64 routed rows of one expert.  The
// chunk loop walks F in chunks of 128 columns:
//   H_c[64 x 128] = X[64 x 256] . W1[c]^T     X in registers (MFMA A fragments,
//                                              loaded once), W1 chunk from LDS
//   bias, ReLU, bf16 -> H stored; the bf16 H_c stays in registers as the
//                                              A operand of
//   Y[64 x 256]  += H_c . W2[:, c]^T           W2 chunk from LDS
// Waves: (wm, wf) = (row half, F half of each chunk).  Wave (wm, wf) computes
// H_c for its 32 rows x 64 columns and accumulates a partial Y over those 64
// columns of F (32 x 256 fp32 in accumulators); the two F halves are summed
// once at the end through LDS (p0 + p1: commutative, so deterministic).
// The H accumulators are used as the GEMM2 A fragment without a round trip:
// a lane holds columns {4g..4g+3} of two adjacent 16-column blocks, which is a
// permutation of the MFMA's k slots -- the W2 fragment is read from LDS in the
// same permuted k order (two 8-B reads), and the k-sum is order-free.
//
// Weights stream through a 4-slot LDS ring of 32 KiB granules by LDS-DMA
// (global_load_lds_dwordx4, swizzle on the source address, mfma_lds.h images):
//   slot 0: W1 chunk c, k   0..127   ([128][64] K-tile images x 2)
//   slot 1: W1 chunk c, k 128..255
//   slot 2: W2 rows 0..255, chunk columns  0..63  ([256][64] image)
//   slot 3: W2 rows 0..255, chunk columns 64..127 (first: the gathered X tile)
// with counted `s_waitcnt vmcnt` (loads, stores and LDS-DMA retire in issue
// order on CDNA4, so the H stores issued between granules are counted too:
// every store instruction is issued by every wave -- buffer stores whose
// out-of-range rows the hardware drops, never an exec-skipped branch) and raw
// s_barrier.  Tiles -> XCDs: contiguous runs of row tiles per XCD (tiles are
// expert-major), so each 4 MiB L2 holds the 1 MiB of weights of ~1-2 experts.
#include "mfma_lds.h"
#include "moe_common.h"
#include "prof.h"

namespace moe {

namespace {

constexpr int kFfBM = 64;        // routed rows per workgroup
constexpr int kFfD = 256;        // model width: K of GEMM1, N of GEMM2
constexpr int kFfFC = 128;       // F columns per chunk
constexpr int kFfSlot = 32768;   // ring slot (one granule)
constexpr int kFfG = 8;          // LDS-DMA instructions per wave per granule
constexpr int kFfB1Bytes = 2048 * 4;            // b1 of one expert (F <= 2048, fp32)
constexpr int kFfBiasBytes = kFfB1Bytes + kFfD * 4;

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

struct FfnParams {
  const uint16_t* x;        // [T][256] token rows (gather) or [rows][256] routed rows
  const int32_t* gather;    // routed row r = x[gather[r]], or nullptr
  const uint16_t* w1;       // [G][F][256]
  const void* b1;           // [G][F] fp32 or bf16
  const uint16_t* w2;       // [G][256][F]
  const void* b2;           // [G][256] fp32 or bf16
  const int32_t* offsets;   // [G + 1]
  uint16_t* h;              // [rows][F]
  uint16_t* yp;             // [yp_n][256]
  const int32_t* yp_rows;   // routed row r -> Yp row yp_rows[r] (expert-parallel received layout), or nullptr
  int32_t* prof_rows;
  int G, F, bias_bf16, yp_n;
};

__device__ __forceinline__ void dma16(const void* src, char* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

// s_waitcnt vmcnt(N) (expcnt / lgkmcnt left at their maxima) through the
// builtin, not inline asm: hipcc's waitcnt pass sees it and knows which
// LDS-DMAs it retired, so it adds no `vmcnt(0)` of its own before the reads.
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("" ::: "memory");  // no store / DMA issue crosses the wait (the counts assume program order)
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x70 | 0xF00);
  asm volatile("" ::: "memory");
}

// Workgroup barrier that also retires this wave's LDS reads first (a slot is
// released to the next DMA only after every fragment read from it is back in
// registers) and that the compiler cannot move memory operations across.
__device__ __forceinline__ void barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// W1 granule: rows 128c .. 128c+127 of expert g, k 128h .. 128h+127, as the
// two [128][64] K-tile images (16 KiB each) of the slot.  The LDS offsets are
// kept visibly inside the slot (wave & 3): hipcc's waitcnt pass then proves
// that a DMA into one slot cannot alias fragment reads of another and emits
// no `s_waitcnt vmcnt(0)` before them.
__device__ __forceinline__ void issue_w1(const FfnParams& p, int g, int c, int h, char* slot, int wave, int lane) {
  const uint16_t* base = p.w1 + ((size_t)g * p.F + (size_t)c * kFfFC) * kFfD + h * 128;
#pragma unroll
  for (int j = 0; j < kFfG; ++j) {
    const int ins = (wave & 3) + 4 * j;  // (& 3: bounded LDS offsets, see issue_w1)
    const int m = ins >> 4, ii = ins & 15;
    const int r = ii * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ ((r >> 1) & 7);
    dma16(base + (size_t)r * kFfD + m * 64 + ch * 8, slot + m * 16384 + ii * 1024);
  }
}

// W2 granule: rows 0..255 of expert g, F columns 128c + 64h .. +63, as one
// [256][64] K-tile image.
__device__ __forceinline__ void issue_w2(const FfnParams& p, int g, int c, int h, char* slot, int wave, int lane) {
  const uint16_t* base = p.w2 + (size_t)g * kFfD * p.F + (size_t)c * kFfFC + h * 64;
#pragma unroll
  for (int j = 0; j < kFfG; ++j) {
    const int ins = (wave & 3) + 4 * j;  // (& 3: bounded LDS offsets, see issue_w1)
    const int r = ins * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ ((r >> 1) & 7);
    dma16(base + (size_t)r * p.F + ch * 8, slot + ins * 1024);
  }
}

// H_c partial for one 128-deep K granule: 4 k-steps of 32.
__device__ __forceinline__ void gemm1_half(const char* slot, const bf16x8 (&xf)[2][8], int h, f32x4 (&hacc)[2][4],
                                           int lane, int wf) {
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    const char* img = slot + (kk >> 1) * 16384;
    bf16x8 bf[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = read_frag<128, true>(img, 64 * wf + 16 * j, kk & 1, lane);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        hacc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], xf[i][4 * h + kk], hacc[i][j], 0, 0, 0);
  }
}

// Y partial += H_c (this wave's 64 columns, as permuted-k A fragments) . W2^T.
// The W2 fragments (two 8-B pieces per 16 x 32 block, in the permuted k
// order) are read with inline-asm ds_reads, one group of 4 column blocks
// ahead of the MFMAs that use it, retired by a counted lgkmcnt wait that also
// carries the values (so no MFMA can be scheduled above it): hipcc's own
// waitcnt pass could not tell these reads from the W1 DMA just issued into
// another slot and drained the whole prefetch with a vmcnt(0) every chunk.
// Block jn of the [256][64] image starts at byte 2048 jn, and the chunk
// swizzle of row 16 jn + lr depends on lr only, so every read is one of four
// per-lane base addresses (k half s, piece c1 / c2) plus an immediate offset.
template <int GI>
__device__ __forceinline__ void w2_group(const uint32_t (&ab)[2][2], u32x2 (&v)[8]) {
  constexpr int s = GI >> 2, jn0 = (GI & 3) * 4;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    // (q is unrolled; the offset operand must be a literal, hence the switch)
    switch (q) {
      case 0:
        asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v[0]) : "v"(ab[s][0]), "n"(2048 * (jn0 + 0)) : "memory");
        asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v[1]) : "v"(ab[s][1]), "n"(2048 * (jn0 + 0)) : "memory");
        break;
      case 1:
        asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v[2]) : "v"(ab[s][0]), "n"(2048 * (jn0 + 1)) : "memory");
        asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v[3]) : "v"(ab[s][1]), "n"(2048 * (jn0 + 1)) : "memory");
        break;
      case 2:
        asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v[4]) : "v"(ab[s][0]), "n"(2048 * (jn0 + 2)) : "memory");
        asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v[5]) : "v"(ab[s][1]), "n"(2048 * (jn0 + 2)) : "memory");
        break;
      default:
        asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v[6]) : "v"(ab[s][0]), "n"(2048 * (jn0 + 3)) : "memory");
        asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v[7]) : "v"(ab[s][1]), "n"(2048 * (jn0 + 3)) : "memory");
        break;
    }
  }
}

template <int N>
__device__ __forceinline__ void lgkm_wait_vals(u32x2 (&v)[8]) {
  asm volatile("s_waitcnt lgkmcnt(%8)"
               : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7])
               : "n"(N)
               : "memory");
}

template <int GI>
__device__ __forceinline__ void gemm2_group(const uint32_t (&ab)[2][2], const bf16x8 (&ha)[2][2],
                                            f32x4 (&yacc)[2][16], u32x2 (&cur)[8], u32x2 (&next)[8]) {
  if constexpr (GI + 1 < 8) {
    w2_group<GI + 1>(ab, next);
    lgkm_wait_vals<8>(cur);
  } else {
    lgkm_wait_vals<0>(cur);
  }
  constexpr int s = GI >> 2, jn0 = (GI & 3) * 4;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    bf16x8 b;
    const u32x2 lo = cur[2 * q], hi = cur[2 * q + 1];
    b[0] = (short)(lo.x & 0xffff); b[1] = (short)(lo.x >> 16); b[2] = (short)(lo.y & 0xffff);
    b[3] = (short)(lo.y >> 16);
    b[4] = (short)(hi.x & 0xffff); b[5] = (short)(hi.x >> 16); b[6] = (short)(hi.y & 0xffff);
    b[7] = (short)(hi.y >> 16);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      yacc[i][jn0 + q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, ha[i][s], yacc[i][jn0 + q], 0, 0, 0);
  }
  if constexpr (GI + 1 < 8) gemm2_group<GI + 1>(ab, ha, yacc, next, cur);
}

__device__ __forceinline__ void gemm2_chunk(const char* slot, const bf16x8 (&ha)[2][2], f32x4 (&yacc)[2][16],
                                            int lane) {
  const int lr = lane & 15, lg = lane >> 4;
  const uint32_t base = (uint32_t)reinterpret_cast<uintptr_t>(slot) + lr * 128 + (lg & 1) * 8;
  const int sw = (lr >> 1) & 7;
  uint32_t ab[2][2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int c1 = 4 * s + (lg >> 1);
    ab[s][0] = base + ((c1 ^ sw) << 4);
    ab[s][1] = base + (((c1 + 2) ^ sw) << 4);
  }
  u32x2 b0[8], b1[8];
  w2_group<0>(ab, b0);
  gemm2_group<0>(ab, ha, yacc, b0, b1);
}

// Bias of 4 consecutive columns from the LDS bias array.  Read with inline-asm
// ds_reads: hipcc's waitcnt pass puts an `s_waitcnt vmcnt(0)` before any LDS
// read it cannot separate from an in-flight LDS-DMA (it treated these bias
// reads so, not the ring's fragment reads), which would drain the prefetched
// granules every chunk; the asm read is retired by its own lgkmcnt wait.
__device__ __forceinline__ float4 bias4(const char* lds, int col, int bf) {
  const uint32_t a = (uint32_t)reinterpret_cast<uintptr_t>(lds) + (uint32_t)col * (bf ? 2u : 4u);
  if (bf) {
    u32x2 v;
    asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
    return make_float4(bf2f(v.x & 0xffffu), bf2f(v.x >> 16), bf2f(v.y & 0xffffu), bf2f(v.y >> 16));
  }
  f32x4 v;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
  return make_float4(v[0], v[1], v[2], v[3]);
}

// Final Y of wave (wm, WF): the other F half's partial of this wave's 128
// output columns arrives through LDS (ring memory, free after the loop); the
// columns of the other half leave the same way.  p0 + p1 is commutative, so
// both halves' sums are the same bits whichever wave adds.
template <int WF>
__device__ __forceinline__ void y_out(const f32x4 (&yacc)[2][16], char* smem, const char* lds_b2, int bias_bf16,
                                      __amdgpu_buffer_rsrc_t yres, const int (&orow)[2], int wm, int lane) {
  constexpr int kRow = 128 * 4 + 16;  // padded fp32 row of one half (128 columns)
  const int lr = lane & 15, lg = lane >> 4;
  char* mine = smem + (wm * 2 + WF) * 32 * kRow;        // written by the other F half
  char* other = smem + (wm * 2 + (1 - WF)) * 32 * kRow;  // this wave writes here
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int q = 0; q < 8; ++q)
      *reinterpret_cast<f32x4*>(other + (16 * i + lr) * kRow + (16 * q + 4 * lg) * 4) = yacc[i][8 * (1 - WF) + q];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      constexpr int base = 8 * WF;
      const int col = 16 * (base + q) + 4 * lg;
      const f32x4 o4 = *reinterpret_cast<const f32x4*>(mine + (16 * i + lr) * kRow + (16 * q + 4 * lg) * 4);
      const float4 b = bias4(lds_b2, col, bias_bf16);
      const f32x4 a = yacc[i][base + q];
      u32x2 o;
      o.x = pack2bf((a[0] + o4[0]) + b.x, (a[1] + o4[1]) + b.y);
      o.y = pack2bf((a[2] + o4[2]) + b.z, (a[3] + o4[3]) + b.w);
      // (rows past the tile: an offset beyond the descriptor, dropped by the hardware)
      const uint32_t off = orow[i] >= 0 ? ((uint32_t)orow[i] * kFfD + col) * 2u : 0xfffffff0u;
      __builtin_amdgcn_raw_buffer_store_b64(o, yres, off, 0, 0);
    }
  }
}

}  // namespace

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void expert_ffn_fwd_kernel(FfnParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // biases in their own LDS object: the compiler can tell that no LDS-DMA of
  // the ring aliases them (a ds_read it cannot separate from an in-flight DMA
  // gets an s_waitcnt vmcnt(0) that would drain the prefetch every chunk)
  __shared__ __attribute__((aligned(16))) char s_bias[kFfBiasBytes];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wf = wave & 1;
  const int lr = lane & 15, lg = lane >> 4;
  if (p.prof_rows != nullptr && blockIdx.x == 0 && tid == 0) *p.prof_rows = p.offsets[p.G];

  // ---- tile: contiguous runs of the expert-major row tiles per XCD ----
  int lo = 0, hi = 0;
  if (lane < p.G) {
    lo = p.offsets[lane];
    hi = p.offsets[lane + 1];
  }
  const int tg = (hi - lo + kFfBM - 1) / kFfBM;
  int incl = tg;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  const int total = __shfl(incl, 63, 64);
  const int per_xcd = (total + 7) / 8;
  const int slot_i = blockIdx.x >> 3;
  const int t = (blockIdx.x & 7) * per_xcd + slot_i;
  if (slot_i >= per_xcd || t >= total) return;
  const unsigned long long hit = __ballot(incl > t);
  // (wave-uniform values made scalar: the buffer descriptors below must be SGPRs)
  const int g = __builtin_amdgcn_readfirstlane(__builtin_ctzll(hit));
  const int row0 = __builtin_amdgcn_readfirstlane(__shfl(lo, g, 64) + (t - __shfl(incl - tg, g, 64)) * kFfBM);
  const int nrows = __builtin_amdgcn_readfirstlane(min(kFfBM, __shfl(hi, g, 64) - row0));
  MOE_DASSERT(nrows >= 1 && nrows <= kFfBM && row0 >= 0);

  char* lds_b1 = s_bias;
  char* lds_b2 = s_bias + kFfB1Bytes;
  const int bsz = p.bias_bf16 ? 2 : 4;

  // ---- prologue: X tile (+ biases) -> slot 3, then W1 / W2 granules of chunk 0 ----
  {
    // biases: plain loads and LDS stores (no LDS-DMA targets s_bias, so the
    // compiler's LDS-DMA tracking never makes a bias read wait on the ring)
    const char* b1 = static_cast<const char*>(p.b1) + (size_t)g * p.F * bsz;
    for (int o = tid * 16; o < p.F * bsz; o += 256 * 16)
      *reinterpret_cast<uint4*>(lds_b1 + o) = *reinterpret_cast<const uint4*>(b1 + o);
    const char* b2 = static_cast<const char*>(p.b2) + (size_t)g * kFfD * bsz;
    if (tid * 16 < kFfD * bsz) *reinterpret_cast<uint4*>(lds_b2 + tid * 16) = *reinterpret_cast<const uint4*>(b2 + tid * 16);
    // this lane's two source rows of the X DMA (rows past the tile clamp to its last row)
    int rs[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      int r = (wave + 4 * q) * 8 + (lane >> 3);
      r = min(r, nrows - 1);
      rs[q] = p.gather != nullptr ? p.gather[row0 + r] : row0 + r;
      MOE_DASSERT(rs[q] >= 0);
    }
#pragma unroll
    for (int j = 0; j < kFfG; ++j) {
      const int ins = (wave & 3) + 4 * j;  // (& 3: bounded LDS offsets, see issue_w1)
      const int kt = ins >> 3, ii = ins & 7;
      const int r = ii * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ ((r >> 1) & 7);
      dma16(p.x + (size_t)rs[j & 1] * kFfD + kt * 64 + ch * 8, (smem + 3 * kFfSlot) + kt * 8192 + ii * 1024);
    }
  }
  issue_w1(p, g, 0, 0, (smem + 0 * kFfSlot), wave, lane);
  issue_w1(p, g, 0, 1, (smem + 1 * kFfSlot), wave, lane);
  issue_w2(p, g, 0, 0, (smem + 2 * kFfSlot), wave, lane);
  vm_wait<3 * kFfG>();  // X has landed (the three weight granules may be in flight)
  barrier();
  bf16x8 xf[2][8];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int k8 = 0; k8 < 8; ++k8) xf[i][k8] = read_frag<64, true>((smem + 3 * kFfSlot) + (k8 >> 1) * 8192, 32 * wm + 16 * i, k8 & 1, lane);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  barrier();  // every wave holds its X fragments: slot 3 is free
  issue_w2(p, g, 0, 1, (smem + 3 * kFfSlot), wave, lane);

  const __amdgpu_buffer_rsrc_t hres =
      __builtin_amdgcn_make_buffer_rsrc(p.h + (size_t)row0 * p.F, (short)0, nrows * p.F * 2, 0x00020000);
  f32x4 yacc[2][16];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 16; ++j) yacc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nc = p.F / kFfFC;
  for (int c = 0; c < nc; ++c) {
    const bool more = c + 1 < nc;
    f32x4 hacc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) hacc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // S1: W1 k 0..127 of chunk c (younger: chunk 0 -> B0, C0, D0; later -> H stores of c-1, B_c)
    if (c == 0) vm_wait<3 * kFfG>();
    else vm_wait<2 * kFfG>();
    barrier();
    if (c > 0) {  // slots 2 / 3 were released by the GEMM2 of chunk c-1
      issue_w2(p, g, c, 0, (smem + 2 * kFfSlot), wave, lane);
      issue_w2(p, g, c, 1, (smem + 3 * kFfSlot), wave, lane);
    }
    gemm1_half((smem + 0 * kFfSlot), xf, 0, hacc, lane, wf);
    // S2: W1 k 128..255 (younger: C_c, D_c)
    vm_wait<2 * kFfG>();
    barrier();
    if (more) issue_w1(p, g, c + 1, 0, (smem + 0 * kFfSlot), wave, lane);
    gemm1_half((smem + 1 * kFfSlot), xf, 1, hacc, lane, wf);
    // S3: bias, ReLU, bf16; H stored (8 buffer stores per wave, always issued)
    bf16x8 ha[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rl = 32 * wm + 16 * i + lr;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = c * kFfFC + 64 * wf + 16 * j + 4 * lg;
        const float4 b = bias4(lds_b1, col, p.bias_bf16);
        const float v0 = fmaxf(hacc[i][j][0] + b.x, 0.f), v1 = fmaxf(hacc[i][j][1] + b.y, 0.f);
        const float v2 = fmaxf(hacc[i][j][2] + b.z, 0.f), v3 = fmaxf(hacc[i][j][3] + b.w, 0.f);
        u32x2 o;
        o.x = pack2bf(v0, v1);
        o.y = pack2bf(v2, v3);
        __builtin_amdgcn_raw_buffer_store_b64(o, hres, (rl * p.F + col) * 2, 0, 0);
        bf16x8& a = ha[i][j >> 1];
        const int e = (j & 1) * 4;
        a[e + 0] = (short)(o.x & 0xffff);
        a[e + 1] = (short)(o.x >> 16);
        a[e + 2] = (short)(o.y & 0xffff);
        a[e + 3] = (short)(o.y >> 16);
      }
    }
    // S4: W2 granules of chunk c (younger: A_{c+1} if any, the 8 H stores)
    if (more) vm_wait<2 * kFfG>();
    else vm_wait<kFfG>();
    barrier();
    if (more) issue_w1(p, g, c + 1, 1, (smem + 1 * kFfSlot), wave, lane);
    // (a constant slot base per branch: hipcc then sees that the W1 DMA just
    // issued into slot 1 cannot alias these reads and adds no vmcnt(0))
    if (wf == 0) gemm2_chunk(smem + 2 * kFfSlot, ha, yacc, lane);
    else gemm2_chunk(smem + 3 * kFfSlot, ha, yacc, lane);
  }

  // ---- Y: sum the two F halves through LDS (ring memory), + b2, bf16 ----
  // (wf is wave-uniform but not a compile-time constant: one branch per half
  // keeps every accumulator index static, so yacc stays in registers)
  int orow[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int rl = 32 * wm + 16 * i + lr;
    orow[i] = rl < nrows ? (p.yp_rows != nullptr ? p.yp_rows[row0 + rl] : row0 + rl) : -1;
    MOE_DASSERT(orow[i] < p.yp_n);
  }
  __syncthreads();
  const __amdgpu_buffer_rsrc_t yres =
      __builtin_amdgcn_make_buffer_rsrc(p.yp, (short)0, p.yp_n * kFfD * 2, 0x00020000);
  if (wf == 0) y_out<0>(yacc, smem, lds_b2, p.bias_bf16, yres, orow, wm, lane);
  else y_out<1>(yacc, smem, lds_b2, p.bias_bf16, yres, orow, wm, lane);
}

}  // namespace moe

using namespace moe;

extern "C" int moe_expert_ffn_supported(int G, int F, int d) {
  return (d == kFfD && F >= kFfFC && F % kFfFC == 0 && F <= 2048 && G >= 1 && G <= 64) ? 1 : 0;
}

extern "C" int moe_expert_ffn_fwd(int dtype, const void* x, const int32_t* src_tok, const void* w1, const void* b1,
                                  const void* w2, const void* b2, const int32_t* offsets, int G, int max_rows, int F,
                                  int d, void* h, void* yp, const int32_t* yp_rows, int yp_n, hipStream_t stream) {
  const bool bias16 = (dtype & MOE_BIAS_BF16) != 0;
  if ((dtype & ~MOE_BIAS_BF16) != MOE_BF16) return fail("expert_ffn_fwd: only MOE_BF16 is implemented");
  if (!moe_expert_ffn_supported(G, F, d))
    return fail("expert_ffn_fwd: need d == 256, F % 128 == 0 in [128, 2048], 1 <= G <= 64");
  if (max_rows < 0) return fail("expert_ffn_fwd: max_rows < 0");
  if (yp_rows == nullptr) yp_n = max_rows;
  if (yp_n < 0 || (long long)yp_n * d * 2 > 0x7fffffffLL) return fail("expert_ffn_fwd: bad yp_n");
  if (x == nullptr || w1 == nullptr || b1 == nullptr || w2 == nullptr || b2 == nullptr || offsets == nullptr ||
      (max_rows > 0 && (h == nullptr || yp == nullptr)))
    return fail("expert_ffn_fwd: NULL pointer");
  for (const void* q : {x, w1, b1, w2, b2, (const void*)h, (const void*)yp})
    if (reinterpret_cast<uintptr_t>(q) % 16) return fail("expert_ffn_fwd: operands must be 16-B aligned");
  if (max_rows == 0) return 0;
  FfnParams p{};
  p.x = static_cast<const uint16_t*>(x);
  p.gather = src_tok;
  p.w1 = static_cast<const uint16_t*>(w1);
  p.b1 = b1;
  p.w2 = static_cast<const uint16_t*>(w2);
  p.b2 = b2;
  p.offsets = offsets;
  p.h = static_cast<uint16_t*>(h);
  p.yp = static_cast<uint16_t*>(yp);
  p.yp_rows = yp_rows;
  p.yp_n = yp_n;
  p.G = G;
  p.F = F;
  p.bias_bf16 = bias16 ? 1 : 0;
  const long long tiles = (max_rows + kFfBM - 1) / kFfBM + G;
  const long long grid = (tiles + 7) / 8 * 8;
  const size_t lds = 4 * kFfSlot;  // (+ the static bias array)
  // exactly the dynamic bytes: static (bias) + dynamic must stay within the 160 KB a CU has, or the
  // attribute is refused and the launch fails
  static unsigned long long attr = 0;  // per-device bitmask
  if (int rc = allow_dyn_lds(reinterpret_cast<const void*>(expert_ffn_fwd_kernel), (int)lds, &attr,
                             "expert_ffn_fwd: LDS attribute"))
    return rc;
  // algorithmic bytes: both weights + biases once; per routed row X (d), H (F) and Yp (d)
  const double bb = bias16 ? 2.0 : 4.0;
  ProfScope prof(stream, PROF_GEMM, 4.0 * G * F * d + bb * G * (F + d), true, 2.0 * (2 * d + F), 4.0 * F * d);
  p.prof_rows = prof.rows_slot();
  MOE_LAUNCH(prof, expert_ffn_fwd_kernel, dim3((unsigned)grid), dim3(256), lds, stream, p);
  return check_launch("moe_expert_ffn_fwd");
}
