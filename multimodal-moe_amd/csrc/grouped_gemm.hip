// Grouped expert GEMMs on bf16 MFMA for gfx950.
//
// One kernel template family covers the five expert contractions of the FFN:
//   ROWS mode  (rows of group g = tokens routed to expert g, K/N fixed)
//     fwd   H  = relu(Xp . W1_g^T + b1_g)      A=[rows][K]  B=[N][K]  (trans_b=1)
//     fwd   Yp = H . W2_g^T + b2_g             A=[rows][K]  B=[N][K]  (trans_b=1)
//     dgrad dH = (dYp . W2_g) * (H > 0)        A=[rows][K]  B=[K][N]  (trans_b=0)
//     dgrad dXp = dH . W1_g                    A=[rows][K]  B=[K][N]  (trans_b=0)
//   WGRAD mode (K = rows of group g, M/N fixed)
//     dW2_g = dYp^T . H  (+ db2 = colsum dYp), dW1_g = dH^T . Xp (+ db1)
//
// Tiling: 256 threads = 4 waves in 2x2, block tile BM x 128, K-step 64,
// v_mfma_f32_16x16x32_bf16 with the operands swapped (D = B^T-frag x A-frag) so
// that each lane ends with 4 consecutive output columns of one row.
// Two LDS images per operand tile:
//   K-contiguous  [R][64] bf16, 128-B rows, 16-B chunk c of row r stored at
//                 chunk c ^ ((r>>1)&7): conflict-free ds_read_b128 fragments;
//   MN-contiguous [64][R] bf16 (weights read for dgrad, activations for
//                 wgrad), fragments by ds_read_b64_tr_b16 (hardware transpose),
//                 XOR swizzle so the two 16-lane blocks of each 32-lane half hit
//                 16 distinct 16-B slots.
// Two main loops:
//   v1 (pipe_kernel<...,1>): global -> registers -> LDS, double buffer, one
//      tile of lookahead (handles every shape; kept for A/B);
//   v2 (default): global -> LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB per
//      wave-instruction, swizzle applied to the per-lane SOURCE address), an
//      S-deep ring with S-1 K-tiles in flight, counted `s_waitcnt vmcnt` +
//      raw s_barrier (no vmcnt(0) drain inside the loop).
#include <algorithm>
#include <type_traits>

#include "mfma_lds.h"
#include "moe_common.h"
#include "prof.h"

namespace moe {

enum { MODE_ROWS = 0, MODE_WGRAD = 1 };

// Operand-format flags (template parameter FL of the kernels)
enum {
  FL_MX = 1,    // ROWS: A and B are MXFP8 (e4m3 + E8M0 per 32 along K): v_mfma_scale_f32_16x16x128_f8f6f4
  FL_CQ = 2,    // ROWS: C is written as MXFP8 (e4m3 [rows][N] + exponents [rows][N/32])
  FL_AUX8 = 4,  // ROWS, EPI_RELU_MASK: the mask operand is e4m3 (keep where the byte is > +0)
  FL_Y8 = 8,    // WGRAD: Y is MXFP8, dequantised to bf16 while staging (v1)
  FL_DENSE = 16  // ROWS: a dense (non-expert) layer (MOE_DENSE_LAYER): same code, its own kernel name, so
                 // rocprof summaries keep it apart from the expert GEMMs
};

struct GemmParams {
  const uint16_t* a;
  const uint16_t* b;
  void* c;
  const int32_t* offsets;
  const float* bias;
  const uint16_t* aux;
  float* colsum;
  int32_t* prof_rows;  // profiler slot for offsets[G] (written by block 0), or nullptr
  const uint8_t* as;   // MX: E8M0 block exponents of A [rows][ksb] (ROWS) or of Y [rows][N/32] (WGRAD Y8)
  const uint8_t* bs;   // MX: E8M0 block exponents of B [G][N][ksb]
  uint8_t* cs;         // CQ: E8M0 block exponents of C [rows][N/32]
  int ksb;             // MX: scale bytes per A/B row (= K / 32)
  long long stride_b;  // elements between groups' B (ROWS mode)
  long long stride_c;  // elements between groups' C (WGRAD mode)
  int lda, ldb, ldc;
  int G, M, N, K;
  int dbg;  // measurement only (moe_set_tuning "gemm_debug"): 1 = no C stores, 2 = no main loop
  int xmap; // ROWS tile -> XCD map: 0 = row tiles round-robin over XCDs, 1 = contiguous chunk per XCD
  // split-K (ksplit > 1): the K range of every output tile is cut into ksplit
  // slices run by ksplit workgroups on one XCD; each writes its fp32
  // accumulators to ws, and the last to arrive (per-tile arrival counter in
  // cnt, reset by that block) sums the slices in slice order -- deterministic
  // -- and runs the normal epilogue.
  // WGRAD: groups with fewer than split_min_kt K-tiles (64 rows) are not
  // split -- slice 0 runs the whole group, the other slices exit at once.
  int ksplit;
  int split_min_kt;
  int c_bf16;  // WGRAD: C and colsum written as bf16 (RNE of the fp32 sums) instead of fp32
  float* ws;
  int32_t* cnt;
  // row gathers (no permuted copy of the routed rows in HBM):
  //   ROWS:  routed row r of A is a[a_gather[r]] (GEMM1 reads the token rows x[t]
  //          straight into the LDS ring), variant 2 only;
  //   WGRAD: k-row r of Y is y[b_gather[r]] (dW1 = dH^T Xp from the token rows), variant 1 only.
  const int32_t* a_gather;
  const int32_t* b_gather;
  // gate scaling (the combine transpose folded into the backward GEMMs):
  //   ROWS:  output row r is multiplied by row_scale[r] before the epilogue;
  //   WGRAD: k-row r of X is bf16(x_scale[r] * x[x_gather[r]]) (dYp formed while staging).
  const float* row_scale;
  const int32_t* x_gather;
  const float* x_scale;
  // WGRAD, G = 1 with offsets == nullptr: the group's rows are [0, dense_rows)
  // (a dense linear layer's weight gradient; no device offsets to load)
  int dense_rows;
  int bias_bf16;  // ROWS bias epilogues: bias is bf16 [G][N] (the bf16 parameter itself, no fp32 copy)
  // ROWS: output row r is stored at C row c_rows[r] (the expert-parallel
  // received layout, src/moe/ep.py) instead of row r; nullptr = identity.
  // The epilogue's mask operand (aux) stays indexed by r.
  const int32_t* c_rows;
};

// runtime tuning knobs (moe_set_tuning)
// runtime tuning overrides (moe_set_tuning); 0 = the per-shape choice below
static int g_gemm_variant = 0;
static int g_gemm_stages = 0;
// ring depth of the long-K (>= 1024) row GEMMs whose grid is under one
// workgroup per CU (the decoder's GEMM2: 176 workgroups, 16 K-tiles each)
static int g_deep_stages = 3;
static int g_gemm_debug = 0;
static int g_rows_bm = 0;   // 0 = by tile count, else 64 or 128
static int g_wgrad_bm = 0;  // 0 = by tile count, else 64 or 128
static int g_xcd_map = 0;   // 0 = default (contiguous chunks), 1 = round-robin, 2 = contiguous chunks
static int g_ksplit = 0;    // 0 = per-shape choice, else forced split-K factor (1 = off)
static int g_gemm_pair_off = 0;  // 1: moe_grouped_gemm_bwd_pair issues two launches (A/B)
static int g_wgrad_dma = 0;      // gathered WGRAD: 0 = default (LDS-DMA ring), 1 = register-staged (A/B)
static int g_wgrad_stages = 0;   // gathered WGRAD LDS-DMA ring depth: 0 = default (2), else 2 or 3
// split-K of the HEAVY groups of a weight gradient that is otherwise unsplit
// (the decoder's ~600-row experts): groups of at least this many K-tiles (64
// rows) run as two slices merged in slice order; 0 = off.  In the training
// step the routed counts are skewed (largest expert 2-3x the mean early on):
// the heaviest group's K loop is the launch's tail.
static int g_wgrad_split_hot = 0;
// split-K factor of an under-filled forward GEMM (K-contiguous B, e.g. the
// decoder's GEMM2: 150 tiles of K = 1,024); 0 = off (A/B)
static int g_fwd_ksplit = 0;
// moe_expert_ffn_bwd: the largest mean rows per expert that take the two-launch
// form (dH, then {dXp, dW2, dW1}); above it the two paired launches run (the
// C2 encoder's 1,840 rows per expert: the one-grid form needs two rounds of
// the chip, in-step 110 us vs 98 us paired; the decoder's 600: 49 vs 56 us)
static int g_bwd2_max_rows = 1024;
// split-K of the dXp body inside that grid: 0 = the per-shape choice, 1 = off
static int g_bwd2_dx_split = 0;

// split-K workspace registered per device by the caller (moe_set_splitk_workspace)
struct SplitWs {
  float* ws = nullptr;
  size_t ws_bytes = 0;
  int32_t* cnt = nullptr;
  int n_cnt = 0;
};
static SplitWs g_split_ws[64];

// ---------------------------------------------------------------------------
// tile schedule + operand addressing shared by both main loops
// ---------------------------------------------------------------------------
template <int BM, int BN, bool B_K, int MODE>
struct Tile {
  int g, mt, nt, row0, rows_g, m0, n0, a_row_lim, nk;
  int split, nsplit, tile_id;  // split-K slice of this workgroup, slices of its tile, tile index
  const uint16_t* a_base;  // element (m0 or row0, k=0) of logical A
  const uint16_t* b_base;  // element (k=0, n0) of logical B

  // XCD-aware block -> tile map (speed only; any placement is correct).
  // Workgroups are dealt round-robin over the 8 XCDs, so blocks b and b+8
  // share an XCD (and its 4 MiB L2).  ROWS: the N/BN column tiles of one row
  // tile get consecutive slots on one XCD (they share the 64-128 KiB A panel)
  // and row tiles rotate over the XCDs.  WGRAD (G >= 8): every tile of group g
  // runs on XCD g % 8, so the group's activation rows stream through one L2.
  // The group of a row tile is found wave-parallel: each lane loads one
  // group's offsets (one memory round trip per 64 groups, not one per group),
  // an inclusive lane scan of the tile counts and a ballot pick the group.
  __device__ __forceinline__ bool init(const GemmParams& p, int lane, int bid) {
    // split-K: the ksplit slices of one tile are consecutive slots of one XCD
    // (bid: the workgroup's index within its problem; a multiple-of-8 offset
    // keeps bid & 7 == the XCD when two problems share a launch)
    const int xcd = bid & 7;
    int slot = bid >> 3;
    split = 0;
    nsplit = p.ksplit > 1 ? p.ksplit : 1;
    if (p.ksplit > 1) {
      split = slot % p.ksplit;
      slot /= p.ksplit;
    }
    const int L = (slot << 3) | xcd;
    if constexpr (MODE == MODE_ROWS) {
      const int ntn = p.N / BN;
      nt = slot % ntn;
      int rem = (slot / ntn) * 8 + xcd;  // global row-tile index (round-robin map)
      if (p.G <= 64) {
        // one load of the offsets and one lane scan give both the total (for
        // the contiguous map) and the group: every workgroup's first
        // dependent chain (the generic path below loads and reduces twice)
        int lo = 0, hi = 0;
        if (lane < p.G) {
          lo = p.offsets[lane];
          hi = p.offsets[lane + 1];
        }
        const int tg = (hi - lo + BM - 1) / BM;
        int incl = tg;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int v = __shfl_up(incl, o, 64);
          if (lane >= o) incl += v;
        }
        if (p.xmap == 1) {
          const int C = (__shfl(incl, 63, 64) + 7) / 8;
          const int r = slot / ntn;
          if (r >= C) return false;
          rem = xcd * C + r;
        }
        const unsigned long long hit = __ballot(incl > rem);
        if (!hit) return false;  // beyond the last tile (grid is an upper bound)
        const int src = __builtin_ctzll(hit);
        g = src;
        mt = rem - __shfl(incl - tg, src, 64);
        row0 = __shfl(lo, src, 64) + mt * BM;
        rows_g = __shfl(hi, src, 64) - row0;
        tile_id = rem * ntn + nt;
      } else {
      if (p.xmap == 1) {
        // contiguous map: XCD x owns row tiles [x C, (x+1) C), C = ceil(total / 8), so
        // its L2 sees the weights of ~1-2 experts instead of all of them
        int total = 0;
        for (int c0 = 0; c0 < p.G; c0 += 64) {
          const int gi = c0 + lane;
          int tg = 0;
          if (gi < p.G) tg = (p.offsets[gi + 1] - p.offsets[gi] + BM - 1) / BM;
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) tg += __shfl_xor(tg, o, 64);
          total += tg;
        }
        const int C = (total + 7) / 8;
        const int r = slot / ntn;
        if (r >= C) return false;
        rem = xcd * C + r;
      }
      int before = 0;                          // row tiles of the groups below chunk c0
      g = -1;
      for (int c0 = 0; c0 < p.G; c0 += 64) {
        const int gi = c0 + lane;
        int lo = 0, hi = 0;
        if (gi < p.G) {
          lo = p.offsets[gi];
          hi = p.offsets[gi + 1];
        }
        const int tg = (hi - lo + BM - 1) / BM;
        int incl = tg;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int v = __shfl_up(incl, o, 64);
          if (lane >= o) incl += v;
        }
        const unsigned long long hit = __ballot(before + incl > rem);
        if (hit) {
          const int src = __builtin_ctzll(hit);
          g = c0 + src;
          mt = rem - before - __shfl(incl - tg, src, 64);
          row0 = __shfl(lo, src, 64) + mt * BM;
          rows_g = __shfl(hi, src, 64) - row0;
          break;
        }
        before += __shfl(incl, 63, 64);
      }
      if (g < 0) return false;  // beyond the last tile (grid is an upper bound)
      tile_id = rem * ntn + nt;
      }  // G > 64
    } else {
      const int ntn = p.N / BN;
      const int tpg = (p.M / BM) * ntn;  // tiles per group
      int tile;
      if (p.G >= 8) {
        g = (slot / tpg) * 8 + xcd;
        tile = slot % tpg;
      } else {
        g = L / tpg;
        tile = L % tpg;
      }
      if (g >= p.G) return false;
      mt = tile / ntn;
      nt = tile % ntn;
      if (p.offsets != nullptr) {
        row0 = p.offsets[g];
        rows_g = p.offsets[g + 1] - row0;
      } else {
        row0 = 0;
        rows_g = p.dense_rows;
      }
      tile_id = g * tpg + tile;
      if (nsplit > 1 && (rows_g + 63) / 64 < p.split_min_kt) {  // short group: slice 0 alone
        if (split != 0) return false;
        nsplit = 1;
      }
      if (nsplit > 1) {  // this slice's k-rows (the group's rows) start at row0
        const int nkt = (rows_g + 63) / 64;
        const int chunk = (nkt + p.ksplit - 1) / p.ksplit;
        const int r0 = min(split * chunk, nkt) * 64;
        row0 += r0;
        rows_g = max(0, min(rows_g - r0, chunk * 64));
      }
    }
    m0 = mt * BM;
    n0 = nt * BN;
    MOE_DASSERT(rows_g >= 0 && row0 >= 0);  // expert offsets non-decreasing
    if constexpr (MODE == MODE_ROWS) {
      a_base = p.a + (size_t)row0 * p.lda;
      a_row_lim = rows_g < BM ? rows_g : BM;
      const uint16_t* bg = p.b + (size_t)g * p.stride_b;
      b_base = B_K ? bg + (size_t)n0 * p.ldb : bg + n0;
      nk = p.K / 64;
      if (p.ksplit > 1) {
        const int chunk = (nk + p.ksplit - 1) / p.ksplit;
        const int kt0 = min(split * chunk, nk);
        nk = min(chunk, nk - kt0);
        a_base += kt0 * 64;
        b_base += B_K ? (size_t)kt0 * 64 : (size_t)kt0 * 64 * p.ldb;
      }
    } else {
      a_base = p.a + (size_t)row0 * p.lda + m0;
      b_base = p.b + (size_t)row0 * p.ldb + n0;
      a_row_lim = BM;
      nk = (rows_g + 63) / 64;
    }
    return true;
  }
};

// ---------------------------------------------------------------------------
// epilogue: lane holds C[m = .. + (lane&15)][n = .. + 4*(lane>>4) + r]
// ---------------------------------------------------------------------------
// Bias of this lane's output columns, loaded at kernel start so its latency
// hides behind the main loop (ROWS mode, EPI_BIAS*).
template <int BN, int MODE, int EPI>
__device__ __forceinline__ void prefetch_bias(const GemmParams& p, int g, int n0, int lane, int wn,
                                              float4 (&bpre)[BN / 32]) {
  if constexpr (MODE == MODE_ROWS && (EPI == MOE_EPI_BIAS || EPI == MOE_EPI_BIAS_RELU)) {
    const int ln = 4 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < BN / 32; ++j) {
      const size_t o = (size_t)g * p.N + n0 + wn * (BN / 2) + 16 * j + ln;
      if (p.bias_bf16) {
        const uint2 v = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(p.bias) + o);
        bpre[j] = make_float4(bf2f(v.x & 0xffffu), bf2f(v.x >> 16), bf2f(v.y & 0xffffu), bf2f(v.y >> 16));
      } else {
        bpre[j] = *reinterpret_cast<const float4*>(p.bias + o);
      }
    }
  }
}

template <int BM, int BN, int MODE, int EPI, bool COLSUM>
__device__ __forceinline__ void epilogue(const GemmParams& p, int g, int row0, int a_row_lim, int m0, int n0, int nt,
                                         f32x4 (&acc)[BM / 32][BN / 32], float (&csum)[BM / 32],
                                         const float4 (&bpre)[BN / 32], int lane, int wm, int wn) {
  constexpr int TM = BM / 32, TN = BN / 32;
  const int lm = lane & 15;
  const int ln = 4 * (lane >> 4);
  if constexpr (MODE == MODE_ROWS) {
    uint16_t* C = static_cast<uint16_t*>(p.c);
    // relu-mask operand: every load issued before the first use (rows past the
    // group clamped to a valid one; their results are never stored)
    uint2 hv[EPI == MOE_EPI_RELU_MASK ? TM : 1][EPI == MOE_EPI_RELU_MASK ? TN : 1];
    if constexpr (EPI == MOE_EPI_RELU_MASK) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        int ml = wm * (BM / 2) + 16 * i + lm;
        ml = ml < a_row_lim ? ml : a_row_lim - 1;
#pragma unroll
        for (int j = 0; j < TN; ++j)
          hv[i][j] = *reinterpret_cast<const uint2*>(p.aux + ((size_t)row0 + ml) * p.ldc + n0 + wn * (BN / 2) +
                                                     16 * j + ln);
      }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int ml = wm * (BM / 2) + 16 * i + lm;
      if (ml >= a_row_lim) continue;
      const size_t row = (size_t)row0 + ml;
      const size_t crow = p.c_rows != nullptr ? (size_t)p.c_rows[row] : row;
      const float rs = p.row_scale != nullptr ? p.row_scale[row] : 1.f;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * (BN / 2) + 16 * j + ln;
        float v[4] = {acc[i][j][0] * rs, acc[i][j][1] * rs, acc[i][j][2] * rs, acc[i][j][3] * rs};
        if constexpr (EPI == MOE_EPI_BIAS || EPI == MOE_EPI_BIAS_RELU) {
          v[0] += bpre[j].x; v[1] += bpre[j].y; v[2] += bpre[j].z; v[3] += bpre[j].w;
        }
        if constexpr (EPI == MOE_EPI_BIAS_RELU) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
        }
        if constexpr (EPI == MOE_EPI_RELU_MASK) {
          const uint2 hw = hv[i][j];
          const uint16_t h[4] = {(uint16_t)(hw.x & 0xffff), (uint16_t)(hw.x >> 16),
                                 (uint16_t)(hw.y & 0xffff), (uint16_t)(hw.y >> 16)};
#pragma unroll
          for (int r = 0; r < 4; ++r)  // bf16 > 0: sign clear and not +0
            if ((h[r] & 0x8000u) || h[r] == 0) v[r] = 0.f;
        }
        uint2 o;
        o.x = pack2bf(v[0], v[1]);
        o.y = pack2bf(v[2], v[3]);
        if (!(p.dbg & 1)) *reinterpret_cast<uint2*>(C + crow * p.ldc + n) = o;
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wm * (BM / 2) + 16 * i + lm;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * (BN / 2) + 16 * j + ln;
        const size_t off = (size_t)g * p.stride_c + (size_t)m * p.ldc + n;
        if (p.dbg & 1) continue;
        if (p.c_bf16) {
          uint2 o;
          o.x = pack2bf(acc[i][j][0], acc[i][j][1]);
          o.y = pack2bf(acc[i][j][2], acc[i][j][3]);
          *reinterpret_cast<uint2*>(static_cast<uint16_t*>(p.c) + off) = o;
        } else {
          *reinterpret_cast<float4*>(static_cast<float*>(p.c) + off) =
              make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
        }
      }
    }
    if constexpr (COLSUM) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        float s = csum[i];
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        csum[i] = s;
      }
      if (nt == 0 && wn == 0 && (lane >> 4) == 0) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int m = m0 + wm * (BM / 2) + 16 * i + lm;
          if (p.c_bf16) reinterpret_cast<uint16_t*>(p.colsum)[(size_t)g * p.M + m] = f2bf(csum[i]);
          else p.colsum[(size_t)g * p.M + m] = csum[i];
        }
      }
    }
  }
}

// Epilogue through LDS (v2): each wave writes its accumulators (after bias /
// ReLU) into a row-major [BM][BN] image over the drained stage buffers, then
// the block stores whole rows with 16-B-per-lane global stores (full 128-B
// lines; the register-direct path issues 8-B pieces, which the store path
// handles at half the rate).  The relu-mask operand is read the same way.
// Images: 16-B chunk c of row r at c ^ (r % chunks_per_row).
// Relu-mask operand of the dgrad (EPI_RELU_MASK, bf16): the 16-B chunks this
// thread's epilogue stores cover, loaded before the K loop (its latency -- an
// HBM round trip: the forward wrote H long before -- hides behind the loop
// instead of trailing it) when they fit in 4 registers of 16 B.
template <int BM, int BN, int MODE, int EPI, int FL>
struct MaskPre {
  static constexpr bool ON = MODE == MODE_ROWS && EPI == MOE_EPI_RELU_MASK && !(FL & FL_AUX8) && BM * BN / 2048 <= 4;
  static constexpr int N = ON ? BM * BN / 2048 : 1;
};

template <int BM, int BN, int MODE, int EPI, bool COLSUM, int FL>
__device__ __forceinline__ void epilogue_lds(const GemmParams& p, int g, int row0, int a_row_lim, int m0, int n0,
                                             int nt, f32x4 (&acc)[BM / 32][BN / 32], float (&csum)[BM / 32],
                                             const float4 (&bpre)[BN / 32], char* smem, int tid, int lane, int wm,
                                             int wn, const uint4 (&mpre)[MaskPre<BM, BN, MODE, EPI, FL>::N]) {
  constexpr int TM = BM / 32, TN = BN / 32;
  const int lm = lane & 15;
  const int ln = 4 * (lane >> 4);
  __syncthreads();  // every wave is done with the stage buffers
  if constexpr (MODE == MODE_ROWS) {
    constexpr int CPR = BN / 8;  // 16-B chunks per bf16 row
    float rs[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int ml = wm * (BM / 2) + 16 * i + lm;
      rs[i] = (p.row_scale != nullptr && ml < a_row_lim) ? p.row_scale[(size_t)row0 + ml] : 1.f;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int ml = wm * (BM / 2) + 16 * i + lm;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int nl = wn * (BN / 2) + 16 * j + ln;
        float v[4] = {acc[i][j][0] * rs[i], acc[i][j][1] * rs[i], acc[i][j][2] * rs[i], acc[i][j][3] * rs[i]};
        if constexpr (EPI == MOE_EPI_BIAS || EPI == MOE_EPI_BIAS_RELU) {
          v[0] += bpre[j].x; v[1] += bpre[j].y; v[2] += bpre[j].z; v[3] += bpre[j].w;
        }
        if constexpr (EPI == MOE_EPI_BIAS_RELU) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
        }
        uint2 o;
        o.x = pack2bf(v[0], v[1]);
        o.y = pack2bf(v[2], v[3]);
        const int off = ml * (BN * 2) + (((nl >> 3) ^ (ml & (CPR - 1))) << 4) + (nl & 7) * 2;
        *reinterpret_cast<uint2*>(smem + off) = o;
      }
    }
    __syncthreads();
    uint16_t* C = static_cast<uint16_t*>(p.c);
    constexpr int RPP = 256 / CPR;  // rows per pass
    const int c = tid % CPR;
#pragma unroll
    for (int r0 = 0; r0 < BM; r0 += RPP) {
      const int r = r0 + tid / CPR;
      if (r >= a_row_lim) continue;
      uint4 v = *reinterpret_cast<const uint4*>(smem + r * (BN * 2) + ((c ^ (r & (CPR - 1))) << 4));
      const size_t gofs = ((size_t)row0 + r) * p.ldc + n0 + c * 8;
      const size_t cofs = p.c_rows != nullptr ? (size_t)p.c_rows[row0 + r] * p.ldc + n0 + c * 8 : gofs;
      if constexpr (EPI == MOE_EPI_RELU_MASK && (FL & FL_AUX8)) {  // e4m3 activation: keep where byte > +0
        const uint2 h = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(p.aux) + gofs);
        uint32_t vw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t hw = q < 2 ? h.x : h.y;
          const uint32_t lo = (hw >> (16 * (q & 1))) & 0xffu, hi = (hw >> (16 * (q & 1) + 8)) & 0xffu;
          const uint32_t keep_lo = (lo == 0 || lo >= 0x80u) ? 0u : 0xffffu;
          const uint32_t keep_hi = (hi == 0 || hi >= 0x80u) ? 0u : 0xffff0000u;
          vw[q] &= keep_lo | keep_hi;
        }
        v = make_uint4(vw[0], vw[1], vw[2], vw[3]);
      } else if constexpr (EPI == MOE_EPI_RELU_MASK) {  // keep where the forward activation is > 0
        uint4 h;
        if constexpr (MaskPre<BM, BN, MODE, EPI, FL>::ON) h = mpre[r0 / RPP];
        else h = *reinterpret_cast<const uint4*>(p.aux + gofs);
        uint32_t hw[4] = {h.x, h.y, h.z, h.w};
        uint32_t vw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t lo = hw[q] & 0xffffu, hi = hw[q] >> 16;
          const uint32_t keep_lo = ((lo & 0x8000u) || lo == 0) ? 0u : 0xffffu;
          const uint32_t keep_hi = ((hi & 0x8000u) || hi == 0) ? 0u : 0xffff0000u;
          vw[q] &= keep_lo | keep_hi;
        }
        v = make_uint4(vw[0], vw[1], vw[2], vw[3]);
      }
      if constexpr (FL & FL_CQ) {  // MXFP8 out: 4 consecutive lanes (same row) hold one 32-column block
        int e;
        const uint2 o = mx_quant_chunk(v, e);
        if (!(p.dbg & 1)) {
          *reinterpret_cast<uint2*>(static_cast<uint8_t*>(p.c) + cofs) = o;
          if ((c & 3) == 0) p.cs[cofs / 32] = (uint8_t)(e + 127);
        }
      } else {
        if (!(p.dbg & 1)) *reinterpret_cast<uint4*>(C + cofs) = v;
      }
    }
  } else {
    constexpr int CPR = BN / 4;  // 16-B chunks per fp32 row
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int ml = wm * (BM / 2) + 16 * i + lm;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int nl = wn * (BN / 2) + 16 * j + ln;
        const int off = ml * (BN * 4) + (((nl >> 2) ^ (ml & (CPR - 1))) << 4);
        *reinterpret_cast<float4*>(smem + off) = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      }
    }
    __syncthreads();
    constexpr int RPP = 256 / CPR;
    const int c = tid % CPR;
#pragma unroll 4
    for (int r0 = 0; r0 < BM; r0 += RPP) {
      const int r = r0 + tid / CPR;
      const float4 v = *reinterpret_cast<const float4*>(smem + r * (BN * 4) + ((c ^ (r & (CPR - 1))) << 4));
      const size_t off = (size_t)g * p.stride_c + (size_t)(m0 + r) * p.ldc + n0 + c * 4;
      if (p.dbg & 1) continue;
      if (p.c_bf16) {
        uint2 o;
        o.x = pack2bf(v.x, v.y);
        o.y = pack2bf(v.z, v.w);
        *reinterpret_cast<uint2*>(static_cast<uint16_t*>(p.c) + off) = o;
      } else {
        *reinterpret_cast<float4*>(static_cast<float*>(p.c) + off) = v;
      }
    }
    if constexpr (COLSUM) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        float s = csum[i];
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        csum[i] = s;
      }
      if (nt == 0 && wn == 0 && (lane >> 4) == 0) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int m = m0 + wm * (BM / 2) + 16 * i + lm;
          if (p.c_bf16) reinterpret_cast<uint16_t*>(p.colsum)[(size_t)g * p.M + m] = f2bf(csum[i]);
          else p.colsum[(size_t)g * p.M + m] = csum[i];
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// split-K merge (p.ksplit > 1).  Every slice stores its accumulators (and
// column-sum partials) as fp32 with agent-coherent stores (sc1: written
// through to the coherence point, never parked dirty in one XCD's L2),
// waits for them to complete, and bumps the tile's arrival counter; the last
// slice to arrive resets the counter and replaces its registers by the sum of
// all slices taken in slice order (agent-coherent loads, several slices per
// round trip), so the result does not depend on arrival order.
// Returns true in that block only (it then runs the epilogue).
// No __threadfence: its agent-scope release writes back the whole L2
// (buffer_wbl2), which made every split launch 5-20x slower on MI355X.
// Layout: component c of accumulator q at [(4 q + c) * 256 + tid] -- every
// dword instruction of the block covers 1 KiB contiguous.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void st_agent(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_agent(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int TM, int TN, bool COLSUM, int NB = 1>
__device__ __forceinline__ bool splitk_merge(const GemmParams& p, int tile_id, int split,
                                             f32x4 (&acc)[TM][TN], float (&csum)[TM], int tid) {
  constexpr int NQ = TM * TN;
  constexpr size_t PART = 256 * (NQ * 4 + (COLSUM ? TM : 0));  // floats per slice
  __shared__ int s_arrived;
  float* base = p.ws + (size_t)tile_id * p.ksplit * PART;
  {
    float* mine = base + (size_t)split * PART;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int c = 0; c < 4; ++c) st_agent(mine + ((i * TN + j) * 4 + c) * 256 + tid, acc[i][j][c]);
    if constexpr (COLSUM) {
#pragma unroll
      for (int i = 0; i < TM; ++i) st_agent(mine + (NQ * 4 + i) * 256 + tid, csum[i]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's slice stores have completed
  __syncthreads();
  if (tid == 0) {
    const int old = __hip_atomic_fetch_add(p.cnt + tile_id, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    MOE_DASSERT(old >= 0 && old < p.ksplit);  // split-K arrival counter (reset by the previous launch's last slice)
    if (old == p.ksplit - 1)  // ready for the next launch
      __hip_atomic_store(p.cnt + tile_id, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_arrived = old;
  }
  __syncthreads();
  if (s_arrived != p.ksplit - 1) return false;
  // Sum in slice order from the workspace (this block's own slice included:
  // its stores are this thread's own, already complete), NB slices per memory
  // round trip -- one round trip per slice made the 8-slice merge of the dense
  // weight gradients ~7 us.  NB > 1 costs (NB - 1) x NV registers: only the
  // register-staged WGRAD body (whose staging registers are dead here) has them
  // without dropping below three workgroups per CU.
  constexpr int NV = NQ * 4 + (COLSUM ? TM : 0);  // floats per thread per slice
  f32x4 tot[TM][TN];
  float ctot[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    ctot[i] = 0.f;
#pragma unroll
    for (int j = 0; j < TN; ++j) tot[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  for (int s0 = 0; s0 < p.ksplit; s0 += NB) {
    float v[NB][NV];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      if (s0 + b >= p.ksplit) break;  // (uniform) the last batch may be short
      const float* src = base + (size_t)(s0 + b) * PART;
#pragma unroll
      for (int e = 0; e < NV; ++e) v[b][e] = ld_agent(src + e * 256 + tid);
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      if (s0 + b >= p.ksplit) break;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int c = 0; c < 4; ++c) tot[i][j][c] += v[b][(i * TN + j) * 4 + c];
        if constexpr (COLSUM) ctot[i] += v[b][NQ * 4 + i];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    csum[i] = ctot[i];
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = tot[i][j];
  }
  return true;
}

// MFMA work on one staged MXFP8 K-tile (128 e4m3 per row = one 128-B LDS row,
// the same image as a bf16 K-tile): one v_mfma_scale_f32_16x16x128_f8f6f4 per
// (i, j).  Operand map (measured with tools/mx_probe.hip, exact integer data):
// lane l = 16 q + i supplies row i, k = 16q..16q+15 in its first 16 bytes and
// k = 64+16q..64+16q+15 in its last 16 (16-B chunks q and q + 4), and the E8M0
// exponent of k-block q (k = 32q..32q+31) of row i -- a block's data is spread
// over two lane groups, its scale comes from one lane.  sA / sB hold each tile
// row's exponents for the whole K as dwords (4 k-blocks = one K-tile each).
template <int BM, int BN>
__device__ __forceinline__ void compute_tile_mx(const char* abuf, const char* bbuf, const uint32_t* sA,
                                                const uint32_t* sB, int ksw, int kt,
                                                f32x4 (&acc)[BM / 32][BN / 32], int lane, int wm, int wn) {
  constexpr int TM = BM / 32, TN = BN / 32;
  const int rl = lane & 15, kb = lane >> 4;
  i32x8 af[TM], bfr[TN];
  int sa[TM], sb[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = wm * (BM / 2) + 16 * i + rl;
    const uint4 lo = *reinterpret_cast<const uint4*>(abuf + kimg_off(r, kb));
    const uint4 hi = *reinterpret_cast<const uint4*>(abuf + kimg_off(r, kb + 4));
    af[i] = i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
    sa[i] = (int)(sA[r * ksw + kt] >> (8 * kb));
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int r = wn * (BN / 2) + 16 * j + rl;
    const uint4 lo = *reinterpret_cast<const uint4*>(bbuf + kimg_off(r, kb));
    const uint4 hi = *reinterpret_cast<const uint4*>(bbuf + kimg_off(r, kb + 4));
    bfr[j] = i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
    sb[j] = (int)(sB[r * ksw + kt] >> (8 * kb));
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
      acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bfr[j], af[i], acc[i][j], 0, 0, 0, sb[j], 0, sa[i]);
}

// ---------------------------------------------------------------------------
// v1: register-staged double buffer
// ---------------------------------------------------------------------------
template <int R, bool KCONT>
struct RegStage {
  static constexpr int kPer = R * 64 / 8 / 256;  // 16-B chunks per thread
  uint4 reg[kPer];

  // MN-contiguous tile with gathered k-rows: k-row kk of this thread's chunk i
  // is row gi[i] of gbase (the indices were loaded a tile ahead: load_index).
  __device__ __forceinline__ void load_index(const int32_t* gk, int k_lim, int tid, int (&gi)[kPer]) const {
    static_assert(!KCONT, "gathered k-rows: MN-contiguous tiles");
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int kk = (tid + 256 * i) / (R / 8);
      gi[i] = kk < k_lim ? gk[kk] : -1;
    }
  }
  __device__ __forceinline__ void load_gathered(const uint16_t* gbase, int ld, const int (&gi)[kPer], int tid) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int r = ((tid + 256 * i) % (R / 8)) * 8;
      reg[i] = gi[i] >= 0 ? *reinterpret_cast<const uint4*>(gbase + (size_t)gi[i] * ld + r) : make_uint4(0, 0, 0, 0);
    }
  }
  // scale factors of the k-rows named by load_index (gathered with the same index)
  __device__ __forceinline__ void load_scale(const float* sk, int k_lim, int tid, float (&gs)[kPer]) const {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int kk = (tid + 256 * i) / (R / 8);
      gs[i] = kk < k_lim ? sk[kk] : 0.f;
    }
  }
  // reg[i] = bf16(gs[i] * reg[i]) (RNE, as the combine transpose rounds dYp)
  __device__ __forceinline__ void scale(const float (&gs)[kPer]) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      float f[8];
      unpack8(reg[i], f);
#pragma unroll
      for (int c = 0; c < 8; ++c) f[c] *= gs[i];
      reg[i] = pack8(f);
    }
  }
  __device__ __forceinline__ void load(const uint16_t* base, int ld, int row_lim, int k_lim, int tid,
                                       const int32_t* gk = nullptr, const uint16_t* gbase = nullptr) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int q = tid + 256 * i;
      int r, kk;
      if constexpr (KCONT) {
        r = q >> 3;
        kk = (q & 7) * 8;
      } else {
        constexpr int cpr = R / 8;
        kk = q / cpr;
        r = (q % cpr) * 8;
      }
      const bool ok = r < row_lim && kk < k_lim;
      const uint16_t* p = KCONT ? base + (size_t)r * ld + kk : base + (size_t)kk * ld + r;
      if constexpr (!KCONT) {
        if (gk != nullptr) p = gbase + (size_t)(ok ? gk[kk] : 0) * ld + r;
      }
      reg[i] = ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0, 0, 0, 0);
    }
  }
  __device__ __forceinline__ void store(char* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int q = tid + 256 * i;
      int off;
      if constexpr (KCONT) {
        off = kimg_off(q >> 3, q & 7);
      } else {
        constexpr int cpr = R / 8;
        off = mimg_off<R>(q / cpr, q % cpr);
      }
      *reinterpret_cast<uint4*>(lds + off) = reg[i];
    }
  }
};

// WGRAD Y operand in MXFP8 (FL_Y8): an MN-contiguous [64][128] tile of e4m3
// rows (8 bytes + one exponent per thread-chunk), dequantised to bf16 (exact)
// when stored, so the LDS image and the MFMA loop are the bf16 ones.
struct RegStageY8 {
  static constexpr int kPer = 128 * 64 / 8 / 256;
  uint2 reg[kPer];
  int ex[kPer];

  __device__ __forceinline__ void load(const uint8_t* base, const uint8_t* sbase, int ld, int k_lim, int tid) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int q = tid + 256 * i;
      const int kk = q / 16, r = (q % 16) * 8;
      const bool ok = kk < k_lim;
      reg[i] = ok ? *reinterpret_cast<const uint2*>(base + (size_t)kk * ld + r) : make_uint2(0, 0);
      ex[i] = ok ? (int)sbase[(size_t)kk * (ld / 32) + (r >> 5)] - 127 : 0;
    }
  }
  __device__ __forceinline__ void store(char* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int q = tid + 256 * i;
      *reinterpret_cast<uint4*>(lds + mimg_off<128>(q / 16, q % 16)) = mx_unpack8_bf16(reg[i], ex[i]);
    }
  }
};

template <int BM, int BN, bool A_K, bool B_K, int MODE, int EPI, bool COLSUM, int FL>
__device__ __forceinline__ void gemm_v1_body(const GemmParams& p, int bid, char* smem) {
  constexpr int A_BYTES = BM * 64 * 2;
  constexpr int BUF = (BM + BN) * 64 * 2;
  constexpr int TM = BM / 32, TN = BN / 32;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  if (p.prof_rows != nullptr && bid == 0 && tid == 0)
    *p.prof_rows = p.offsets != nullptr ? p.offsets[p.G] : p.dense_rows;
  Tile<BM, BN, B_K, MODE> t;
  if (!t.init(p, lane, bid)) return;
  float4 bpre[TN];
  prefetch_bias<BN, MODE, EPI>(p, t.g, t.n0, lane, wn, bpre);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float csum[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) csum[i] = 0.f;

  auto k_lim = [&](int kt) -> int { return MODE == MODE_ROWS ? 64 : t.rows_g - kt * 64; };
  auto a_ptr = [&](int kt) { return A_K ? t.a_base + kt * 64 : t.a_base + (size_t)kt * 64 * p.lda; };
  auto b_ptr = [&](int kt) { return B_K ? t.b_base + kt * 64 : t.b_base + (size_t)kt * 64 * p.ldb; };

  constexpr bool Y8 = (FL & FL_Y8) != 0;
  static_assert(!Y8 || (MODE == MODE_WGRAD && BN == 128), "Y8 staging is for WGRAD 128-wide tiles");
  // Y8: byte pointers of Y (e4m3 [rows][N]) and of its exponents ([rows][N/32]) at (row0, n0)
  const uint8_t* yq = Y8 ? reinterpret_cast<const uint8_t*>(p.b) + (size_t)t.row0 * p.N + t.n0 : nullptr;
  const uint8_t* ys = Y8 ? p.as + (size_t)t.row0 * (p.N / 32) + t.n0 / 32 : nullptr;

  RegStage<BM, A_K> la;
  RegStage<BN, B_K> lb;
  RegStageY8 ly;
  // WGRAD with x_gather: k-row r of X is bf16(x_scale[r] * x[x_gather[row0 + r]]); the
  // indices and scales of tile kt+1 are loaded while tile kt computes
  constexpr bool AG = MODE == MODE_WGRAD && !A_K;
  const int32_t* agk = (AG && p.x_gather != nullptr) ? p.x_gather + t.row0 : nullptr;
  const float* ask = (AG && p.x_scale != nullptr) ? p.x_scale + t.row0 : nullptr;
  int ai[AG ? RegStage<BM, A_K>::kPer : 1];
  float as_[AG ? RegStage<BM, A_K>::kPer : 1];
  float dsc[AG ? RegStage<BM, A_K>::kPer : 1];  // scales of the tile in flight (applied at the LDS store)
  auto load_a_index = [&](int kt) {
    if constexpr (AG) {
      if (agk != nullptr && kt < t.nk) {
        la.load_index(agk + kt * 64, k_lim(kt), tid, ai);
        if (ask != nullptr) la.load_scale(ask + kt * 64, k_lim(kt), tid, as_);
      }
    }
  };
  auto load_a = [&](int kt) {
    if constexpr (AG) {
      if (agk != nullptr) {
        la.load_gathered(p.a + t.m0, p.lda, ai, tid);
        // the scale is applied when the tile is written to LDS: multiplying
        // here would wait on these loads before the tile in LDS is computed
        // and before the B loads are issued (two round trips per K-tile)
        if (ask != nullptr) {
#pragma unroll
          for (int i = 0; i < RegStage<BM, A_K>::kPer; ++i) dsc[i] = as_[i];
        }
        load_a_index(kt + 1);
        return;
      }
    }
    la.load(a_ptr(kt), p.lda, t.a_row_lim, k_lim(kt), tid);
  };
  load_a_index(0);
  // WGRAD with b_gather: k-row r of Y is y[b_gather[row0 + r]] (columns from
  // n0); the row indices of tile kt+1 are loaded while tile kt computes, so
  // the data loads of a tile never wait on their index loads
  constexpr bool BG = MODE == MODE_WGRAD && !B_K && !Y8;
  const int32_t* bgk = (BG && p.b_gather != nullptr) ? p.b_gather + t.row0 : nullptr;
  int gi[BG ? RegStage<BN, B_K>::kPer : 1];
  auto load_index = [&](int kt) {
    if constexpr (BG) {
      if (bgk != nullptr && kt < t.nk) lb.load_index(bgk + kt * 64, k_lim(kt), tid, gi);
    }
  };
  auto load_b = [&](int kt) {
    if constexpr (Y8) ly.load(yq + (size_t)kt * 64 * p.N, ys + (size_t)kt * 64 * (p.N / 32), p.N, k_lim(kt), tid);
    else if constexpr (BG) {
      if (bgk != nullptr) {
        lb.load_gathered(p.b + t.n0, p.ldb, gi, tid);
        load_index(kt + 1);
      } else {
        lb.load(b_ptr(kt), p.ldb, BN, k_lim(kt), tid);
      }
    } else lb.load(b_ptr(kt), p.ldb, BN, k_lim(kt), tid);
  };
  load_index(0);
  auto store_b = [&](char* dst) {
    if constexpr (Y8) ly.store(dst, tid);
    else lb.store(dst, tid);
  };
  auto store_a = [&](char* dst) {
    if constexpr (AG) {
      if (ask != nullptr) la.scale(dsc);
    }
    la.store(dst, tid);
  };
  if (t.nk > 0) {
    load_a(0);
    load_b(0);
    store_a(smem);
    store_b(smem + A_BYTES);
  }
  __syncthreads();
  for (int kt = 0; kt < ((p.dbg & 2) ? 0 : t.nk); ++kt) {
    char* cur = smem + (kt & 1) * BUF;
    const bool more = kt + 1 < t.nk;
    if (more) {
      load_a(kt + 1);
      load_b(kt + 1);
    }
    compute_tile<BM, BN, A_K, B_K, COLSUM>(cur, cur + A_BYTES, acc, csum, lane, wm, wn);
    if (more) {
      char* nxt = smem + ((kt + 1) & 1) * BUF;
      store_a(nxt);
      store_b(nxt + A_BYTES);
    }
    __syncthreads();
  }
  constexpr int MERGE_NB = (MODE == MODE_WGRAD && TM * TN <= 8) ? 3 : 1;
  if (t.nsplit > 1 && !splitk_merge<TM, TN, COLSUM, MERGE_NB>(p, t.tile_id, t.split, acc, csum, tid)) return;
  epilogue<BM, BN, MODE, EPI, COLSUM>(p, t.g, t.row0,
                                      t.a_row_lim, t.m0, t.n0, t.nt, acc, csum, bpre, lane, wm, wn);
}

// 64-row tiles fit three workgroups per CU (512 unified VGPRs per lane: <= 168
// arch + acc registers each); pin that so the register allocator never tips a
// variant over the cliff to two.
template <int BM, int BN, bool A_K, bool B_K, int MODE, int EPI, bool COLSUM, int FL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BM <= 64 ? 3 : 1)))
void gemm_v1_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  gemm_v1_body<BM, BN, A_K, B_K, MODE, EPI, COLSUM, FL>(p, blockIdx.x, smem);
}

// A dense linear layer's weight + bias gradients (G = 1, rtdetr_linear_wgrad):
// the same register-staged WGRAD body with colsum, under its own symbol so a
// kernel trace / PMC pass tells it apart from the MoE expert GEMMs.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3)))
void linear_wgrad_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  gemm_v1_body<64, 128, false, false, MODE_WGRAD, MOE_EPI_NONE, true, 0>(p, blockIdx.x, smem);
}

// Several dense weight gradients of different shapes in ONE launch
// (rtdetr_linear_wgrad_batch): problem q owns workgroups [base[q], base[q+1])
// (multiples of 8, so each keeps its XCD-aware slice placement) and its own
// split-K workspace window.  The table travels as the kernel argument.
constexpr int MAX_DENSE_BATCH = 24;
struct DenseProb {
  const uint16_t* gy;
  const uint16_t* x;
  void* dw;
  void* db;
  float* ws;
  int32_t* cnt;
  int K, M, N, ksplit;
};
struct DenseBatch {
  int n, c_bf16, dbg, pad_;
  int base[MAX_DENSE_BATCH + 1];
  DenseProb p[MAX_DENSE_BATCH];
};

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3)))
void linear_wgrad_batch_kernel(DenseBatch b) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int bid = blockIdx.x;
  int q = 0;
  while (q + 1 < b.n && bid >= b.base[q + 1]) ++q;  // uniform: a few scalar compares
  const DenseProb d = b.p[q];
  GemmParams p{};
  p.dbg = b.dbg;
  p.a = d.gy;
  p.b = d.x;
  p.c = d.dw;
  p.colsum = static_cast<float*>(d.db);
  p.c_bf16 = b.c_bf16;
  p.lda = d.M;
  p.ldb = d.N;
  p.ldc = d.N;
  p.stride_c = (long long)d.M * d.N;
  p.G = 1;
  p.M = d.M;
  p.N = d.N;
  p.dense_rows = d.K;
  p.ksplit = d.ksplit;
  p.ws = d.ws;
  p.cnt = d.cnt;
  gemm_v1_body<64, 128, false, false, MODE_WGRAD, MOE_EPI_NONE, true, 0>(p, bid - b.base[q], smem);
}

// ---------------------------------------------------------------------------
// v2: LDS-DMA ring, S stages, S-1 K-tiles in flight
// ---------------------------------------------------------------------------
// Issue the LDS-DMA of one operand tile (R rows x 64 k) into `lds` (a
// wave-uniform base).  1 KiB per wave-instruction, R/32 instructions per wave.
// Rows / k-rows beyond the valid extent are CLAMPED to the last valid one
// (never out of bounds); the caller masks rows (ROWS mode) or zeroes k-rows
// (WGRAD tail) -- a DMA cannot write zeros.
template <int R, bool KCONT>
__device__ __forceinline__ void dma_tile(const uint16_t* base, int ld, int row_lim, int k_lim, char* lds,
                                         int wave, int lane) {
#pragma unroll
  for (int j = 0; j < R / 32; ++j) {
    const int ins = wave + 4 * j;  // wave-instruction index within the tile
    const uint16_t* src;
    if constexpr (KCONT) {  // [R][64]: 8 rows of 128 B per KiB
      int r = ins * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);  // source chunk for LDS slot (r, lane&7)
      r = r < row_lim ? r : row_lim - 1;
      src = base + (size_t)r * ld + c * 8;
    } else {  // [64][R]: 1024 / (2R) k-rows per KiB
      constexpr int cpr = R / 8;            // 16-B chunks per k-row
      constexpr int rows_per = 64 / cpr;    // k-rows per wave-instruction
      int kr = ins * rows_per + lane / cpr;
      const int c = (lane % cpr) ^ mimg_swz<R>(kr);
      kr = kr < k_lim ? kr : k_lim - 1;
      src = base + (size_t)kr * ld + c * 8;
    }
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(lds + ins * 1024), 16, 0, 0);
  }
}

// The same for a K-contiguous A tile whose rows are gathered: rowp[j] is the
// (clamped, gathered) row of wave-instruction j of this lane, sw[j] its chunk
// swizzle; kofs the K-tile's element offset.
template <int R>
__device__ __forceinline__ void dma_tile_rows(const uint16_t* const (&rowp)[R / 32], const int (&sw)[R / 32],
                                              int kofs, char* lds, int wave, int lane) {
#pragma unroll
  for (int j = 0; j < R / 32; ++j) {
    const int ins = wave + 4 * j;
    const uint16_t* src = rowp[j] + kofs + sw[j] * 8;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(lds + ins * 1024), 16, 0, 0);
  }
}

// The same for an MN-contiguous [64][R] tile whose k-rows are gathered: k-row
// kr is row idx[kr] of `base` (the K-tile's 64 row indices, staged in LDS).
template <int R>
__device__ __forceinline__ void dma_tile_krows(const uint16_t* base, int ld, const int32_t* idx, char* lds, int wave,
                                               int lane) {
  constexpr int cpr = R / 8, rows_per = 64 / cpr;
#pragma unroll
  for (int j = 0; j < R / 32; ++j) {
    const int ins = wave + 4 * j;
    const int kr = ins * rows_per + lane / cpr;
    const int c = (lane % cpr) ^ mimg_swz<R>(kr);
    const uint16_t* src = base + (size_t)idx[kr] * ld + c * 8;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(lds + ins * 1024), 16, 0, 0);
  }
}

// 64 dwords of a K-tile's k-row metadata (row indices or scales) by LDS-DMA:
// every wave moves 16 of them (one instruction, lanes 0..15), so the four
// waves' vmcnt counts stay equal.  Rows past `last` read row `last`.
__device__ __forceinline__ void dma_meta64(const void* src, int row, int last, char* lds, int wave, int lane) {
  const int r = min(row + wave * 16 + lane, last);
  if (lane < 16)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(
                                         static_cast<const int32_t*>(src) + r),
                                     (__attribute__((address_space(3))) void*)(lds + wave * 64), 4, 0, 0);
}

// Wait until ring tile kt (and what was issued with it) has landed for this
// wave: at most min(S - 2, newer) younger issues of PER instructions each may
// stay in flight.
template <int S, int PER, int Y = S - 2>
__device__ __forceinline__ void wait_issue(int newer) {
  if constexpr (Y <= 0) {
    wait_vm<0>();
  } else {
    static_assert(Y * PER < 64, "vmcnt");
    if (newer >= Y) wait_vm<Y * PER>();
    else wait_issue<S, PER, Y - 1>(newer);
  }
}

template <int BM, int BN, int S, bool A_K, bool B_K, int MODE, int EPI, bool COLSUM, int FL>
__device__ __forceinline__ void gemm_v2_body(const GemmParams& p, int bid, char* smem) {
  constexpr int A_BYTES = BM * 64 * 2;
  constexpr int BUF = (BM + BN) * 64 * 2;
  constexpr int TM = BM / 32, TN = BN / 32;
  constexpr int GW = BM / 32 + BN / 32;  // LDS-DMA instructions per wave per K-tile
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  if (p.prof_rows != nullptr && bid == 0 && tid == 0)
    *p.prof_rows = p.offsets != nullptr ? p.offsets[p.G] : p.dense_rows;
  Tile<BM, BN, B_K, MODE> t;
  if (!t.init(p, lane, bid)) return;
  float4 bpre[TN];
  prefetch_bias<BN, MODE, EPI>(p, t.g, t.n0, lane, wn, bpre);
  using MP = MaskPre<BM, BN, MODE, EPI, FL>;
  uint4 mpre[MP::N];
  if constexpr (MP::ON) {  // the epilogue's relu-mask chunks (rows as in epilogue_lds' store loop)
    constexpr int CPR = BN / 8, RPP = 256 / CPR;
    const int c = tid % CPR;
#pragma unroll
    for (int k = 0; k < MP::N; ++k) {
      const int r = k * RPP + tid / CPR;
      mpre[k] = r < t.a_row_lim
                    ? *reinterpret_cast<const uint4*>(p.aux + ((size_t)t.row0 + r) * p.ldc + t.n0 + c * 8)
                    : make_uint4(0, 0, 0, 0);
    }
  }

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float csum[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) csum[i] = 0.f;

  // ROWS with a_gather: this lane's source row of every A wave-instruction,
  // found once (the rows are the same for every K-tile)
  constexpr bool GATHER_OK = MODE == MODE_ROWS && A_K && !(FL & FL_MX);
  const bool gather = GATHER_OK && p.a_gather != nullptr;
  const uint16_t* rowp[BM / 32];
  int sw[BM / 32];
  if constexpr (GATHER_OK) {
    if (gather) {
      const int kofs0 = (int)(t.a_base - (p.a + (size_t)t.row0 * p.lda));  // split-K slice offset
#pragma unroll
      for (int j = 0; j < BM / 32; ++j) {
        const int r = (wave + 4 * j) * 8 + (lane >> 3);
        sw[j] = (lane & 7) ^ ((r >> 1) & 7);
        const int rc = r < t.a_row_lim ? r : t.a_row_lim - 1;
        MOE_DASSERT(p.a_gather[t.row0 + rc] >= 0);  // a gather index of a kept row
        rowp[j] = p.a + (size_t)p.a_gather[t.row0 + rc] * p.lda + kofs0;
      }
    }
  }

  // WGRAD with gathered k-rows (one operand): k-row r of X is
  // bf16(x_scale[r] * x[x_gather[r]]) or k-row r of Y is y[b_gather[r]].  The
  // 64 row indices of K-tile j are DMA'd into an index ring (2S slots, behind
  // the stage ring: a wave that runs ahead never overwrites indices another
  // wave is still reading) by issue(j - S + 1), so the K-tile's own DMA reads
  // them from LDS with no dependent global round trip; its scales travel with
  // it (one slot per stage) and are applied to the landed X image in LDS.
  constexpr bool WGG = MODE == MODE_WGRAD && !A_K && !B_K && !(FL & (FL_MX | FL_Y8));
  const int gop = !WGG ? 0 : (p.x_gather != nullptr ? 1 : (p.b_gather != nullptr ? 2 : 0));  // gathered operand
  const bool gscale = gop == 1 && p.x_scale != nullptr;
  char* s_idx = smem + S * BUF;          // [2S][64] int32 row indices
  char* s_scl = s_idx + 2 * S * 256;     // [S][64] fp32 scales (X gather)
  const int32_t* gidx = gop == 1 ? p.x_gather : p.b_gather;
  const int g_last = t.row0 + t.rows_g - 1;
  if (WGG && gop && t.nk > 0) {
    // prologue: indices of K-tiles 0 .. S-2 (plain loads; nothing is in flight yet)
    for (int i = tid; i < (S - 1) * 64; i += 256)
      reinterpret_cast<int32_t*>(s_idx)[i] = gidx[min(t.row0 + i, g_last)];
    __syncthreads();
  }

  const int nk = (p.dbg & 2) ? 0 : t.nk;
  auto issue = [&](int kt) {
    char* buf = smem + (kt % S) * BUF;
    const int klim = MODE == MODE_ROWS ? 64 : t.rows_g - kt * 64;
    const uint16_t* ap = A_K ? t.a_base + kt * 64 : t.a_base + (size_t)kt * 64 * p.lda;
    const uint16_t* bp = B_K ? t.b_base + kt * 64 : t.b_base + (size_t)kt * 64 * p.ldb;
    if constexpr (WGG) {
      if (gop) {
        const int32_t* idx = reinterpret_cast<const int32_t*>(s_idx + (kt % (2 * S)) * 256);
        if (gop == 1) {
          dma_tile_krows<BM>(p.a + t.m0, p.lda, idx, buf, wave, lane);
          dma_tile<BN, false>(bp, p.ldb, BN, klim, buf + A_BYTES, wave, lane);
        } else {
          dma_tile<BM, false>(ap, p.lda, BM, klim, buf, wave, lane);
          dma_tile_krows<BN>(p.b + t.n0, p.ldb, idx, buf + A_BYTES, wave, lane);
        }
        // the indices of K-tile kt + S - 1 (issued even past the last tile:
        // every issue moves the same number of instructions), then the scales
        dma_meta64(gidx, t.row0 + (kt + S - 1) * 64, g_last, s_idx + ((kt + S - 1) % (2 * S)) * 256, wave, lane);
        if (gscale) dma_meta64(p.x_scale, t.row0 + kt * 64, g_last, s_scl + (kt % S) * 256, wave, lane);
        return;
      }
    }
    if constexpr (GATHER_OK) {
      if (gather) dma_tile_rows<BM>(rowp, sw, kt * 64, buf, wave, lane);
      else dma_tile<BM, A_K>(ap, p.lda, t.a_row_lim, klim, buf, wave, lane);
    } else {
      dma_tile<BM, A_K>(ap, p.lda, t.a_row_lim, klim, buf, wave, lane);
    }
    dma_tile<BN, B_K>(bp, p.ldb, BN, klim, buf + A_BYTES, wave, lane);
  };

#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) issue(s);

  // MX: stage the tile rows' E8M0 exponents for the whole K (dwords) behind the
  // ring while the prologue DMA is in flight.
  constexpr bool MX = (FL & FL_MX) != 0;
  static_assert(!MX || (MODE == MODE_ROWS && A_K && B_K), "MX operands: ROWS mode, K-contiguous A and B");
  const int ksw = p.ksb / 4;
  uint32_t* sA = reinterpret_cast<uint32_t*>(smem + S * BUF);
  uint32_t* sB = sA + BM * ksw;
  if constexpr (MX) {
    for (int q = tid; q < (BM + BN) * ksw; q += 256) {
      const int r = q / ksw, w = q - r * ksw;
      uint32_t v;
      if (r < BM) {
        const int rr = r < t.a_row_lim ? r : t.a_row_lim - 1;
        v = reinterpret_cast<const uint32_t*>(p.as + ((size_t)t.row0 + rr) * p.ksb)[w];
      } else {
        v = reinterpret_cast<const uint32_t*>(p.bs + ((size_t)t.g * p.N + t.n0 + (r - BM)) * p.ksb)[w];
      }
      sA[q] = v;
    }
    __syncthreads();
  }

  for (int kt = 0; kt < nk; ++kt) {
    // tile kt has landed for this wave once at most min(S-2, nk-1-kt) newer tiles are pending
    // (a gathered WGRAD issue also moves the next indices and the scales: 1 or 2 more)
    const int newer = nk - 1 - kt;
    if (WGG && gop) {
      if (gscale) wait_issue<S, GW + 2>(newer);
      else wait_issue<S, GW + 1>(newer);
    } else {
      wait_issue<S, GW>(newer);
    }
    __builtin_amdgcn_s_barrier();  // every wave's DMA for tile kt is visible
    char* cur = smem + (kt % S) * BUF;
    if constexpr (WGG) {
      if (gscale) {  // X k-rows *= their gate, bf16 RNE (the rows past the group are zeroed below)
        const int kvalid = min(64, t.rows_g - kt * 64);
        const float* sc = reinterpret_cast<const float*>(s_scl + (kt % S) * 256);
        for (int q = tid; q < 64 * (BM / 8); q += 256) {
          const int kr = q / (BM / 8);
          if (kr >= kvalid) continue;
          uint4* ch = reinterpret_cast<uint4*>(cur + kr * (BM * 2) + (q % (BM / 8)) * 16);
          float f[8];
          unpack8(*ch, f);
          const float sv = sc[kr];
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] *= sv;
          *ch = pack8(f);
        }
        __syncthreads();
      }
    }
    if constexpr (MODE == MODE_WGRAD) {
      const int kvalid = t.rows_g - kt * 64;
      if (kvalid < 64) {  // tail: zero the clamped k-rows of both operands
        for (int q = tid; q < (64 - kvalid) * (BM + BN) / 8; q += 256) {
          const int per = (BM + BN) / 8;  // 16-B chunks per k-row over both images
          const int kr = kvalid + q / per;
          const int c = q % per;
          char* dst = c < BM / 8 ? cur + kr * (BM * 2) + c * 16 : cur + A_BYTES + kr * (BN * 2) + (c - BM / 8) * 16;
          *reinterpret_cast<uint4*>(dst) = make_uint4(0, 0, 0, 0);
        }
        __syncthreads();
      }
    }
    if (kt + S - 1 < nk) issue(kt + S - 1);  // refills the slot read in iteration kt-1
    if constexpr (MX) compute_tile_mx<BM, BN>(cur, cur + A_BYTES, sA, sB, ksw, kt, acc, lane, wm, wn);
    else compute_tile<BM, BN, A_K, B_K, COLSUM>(cur, cur + A_BYTES, acc, csum, lane, wm, wn);
  }
  static_assert(S * (BM + BN) * 64 * 2 >= BM * BN * (MODE == MODE_ROWS ? 2 : 4), "epilogue image exceeds LDS");
  (void)gidx;
  (void)g_last;
  if (t.nsplit > 1 && !splitk_merge<TM, TN, COLSUM>(p, t.tile_id, t.split, acc, csum, tid)) return;
  epilogue_lds<BM, BN, MODE, EPI, COLSUM, FL>(p, t.g, t.row0, t.a_row_lim, t.m0, t.n0, t.nt, acc, csum, bpre, smem,
                                              tid, lane, wm, wn, mpre);
}

template <int BM, int BN, int S, bool A_K, bool B_K, int MODE, int EPI, bool COLSUM, int FL>
__global__ __launch_bounds__(256) void gemm_v2_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  gemm_v2_body<BM, BN, S, A_K, B_K, MODE, EPI, COLSUM, FL>(p, blockIdx.x, smem);
}

// Two independent grouped GEMMs in ONE launch (the backward's dgrad and wgrad
// of the same weight: their grids fill the chip together and one kernel
// boundary disappears): workgroups [0, n1) run problem 1, the rest problem 2.
// n1 is a multiple of 8, so each problem keeps its XCD-aware tile map.
// Both bodies are 64-row tiles: three workgroups per CU (see gemm_v1_kernel).
template <class P1, class P2>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3)))
void gemm_pair_kernel(GemmParams p1, GemmParams p2, int n1) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if ((int)blockIdx.x < n1) P1::run(p1, blockIdx.x, smem);
  else P2::run(p2, (int)blockIdx.x - n1, smem);
}
// Three independent grouped GEMMs in ONE launch (the expert FFN backward's
// second half, moe_expert_ffn_bwd): workgroups [0, n1) problem 1, [n1, n12)
// problem 2, the rest problem 3; n1 and n12 are multiples of 8 (XCD maps).
template <class P1, class P2, class P3>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3)))
void gemm_triple_kernel(GemmParams p1, GemmParams p2, GemmParams p3, int n1, int n12) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x;
  if (b < n1) P1::run(p1, b, smem);
  else if (b < n12) P2::run(p2, b - n1, smem);
  else P3::run(p3, b - n12, smem);
}
template <int BM, int BN, int S, bool A_K, bool B_K, int MODE, int EPI, bool COLSUM, int FL>
struct BodyV2 {
  static __device__ __forceinline__ void run(const GemmParams& p, int bid, char* smem) {
    gemm_v2_body<BM, BN, S, A_K, B_K, MODE, EPI, COLSUM, FL>(p, bid, smem);
  }
};
template <int BM, int BN, bool A_K, bool B_K, int MODE, int EPI, bool COLSUM, int FL>
struct BodyV1 {
  static __device__ __forceinline__ void run(const GemmParams& p, int bid, char* smem) {
    gemm_v1_body<BM, BN, A_K, B_K, MODE, EPI, COLSUM, FL>(p, bid, smem);
  }
};

// ---------------------------------------------------------------------------
// host launch helpers
// ---------------------------------------------------------------------------
// Raise a kernel's dynamic-LDS cap once (first launch), so that later launches
// -- including ones captured into a hipGraph -- make no attribute call.
template <auto FN>
static void allow_lds(size_t bytes) {
  // (raised to 159 KiB at once -- the MX exponent stage makes the size depend
  // on K; 1 KiB is left for the kernels' static LDS, e.g. the split-K flag)
  // (per device; a failure is reported through moe_last_error and the launch
  // that follows fails its check_launch)
  static unsigned long long done = 0;
  if (bytes > 65536) (void)allow_dyn_lds(reinterpret_cast<const void*>(FN), 159 * 1024, &done, "grouped_gemm: dynamic LDS");
}

// the 6-deep ring is instantiated for the 64-row bf16 row GEMMs only
template <int BM, int MODE, int FL>
constexpr bool deep_ring_ok() {
  return MODE == MODE_ROWS && BM == 64 && !(FL & (FL_MX | FL_CQ | FL_AUX8));
}

template <int BM, int BN, bool A_K, bool B_K, int MODE, int EPI, bool COLSUM, int FL = 0>
static void launch(const GemmParams& p, dim3 grid, hipStream_t s, const ProfScope& prof, int variant, int stages) {
  // MX: the exponent stage behind the ring ((BM + BN) rows x K/32 bytes)
  const size_t xs = (FL & FL_MX) ? (size_t)(BM + BN) * p.ksb : 0;
  // (the index / scale rings of a gathered v2 WGRAD: 768 B per stage, added per branch below)
  const size_t gx = (MODE == MODE_WGRAD && (p.x_gather != nullptr || p.b_gather != nullptr)) ? 768 : 0;
  if (variant == 1 && !(FL & (FL_MX | FL_CQ | FL_AUX8))) {
    constexpr size_t lds = 2 * (BM + BN) * 64 * 2;
    constexpr auto fn = gemm_v1_kernel<BM, BN, A_K, B_K, MODE, EPI, COLSUM, FL & (FL_Y8 | FL_DENSE)>;
    allow_lds<fn>(lds);
    MOE_LAUNCH(prof, fn, grid, dim3(256), lds, s, p);
  } else if (stages == 2) {
    const size_t lds = 2 * (BM + BN) * 64 * 2 + xs + 2 * gx;
    constexpr auto fn = gemm_v2_kernel<BM, BN, 2, A_K, B_K, MODE, EPI, COLSUM, FL & ~FL_Y8>;
    allow_lds<fn>(lds);
    MOE_LAUNCH(prof, fn, grid, dim3(256), lds, s, p);
  } else if (stages >= 6 && deep_ring_ok<BM, MODE, FL>()) {
    // (one workgroup per CU: the deep ring of the long-K, sub-chip grids)
    if constexpr (deep_ring_ok<BM, MODE, FL>()) {
      const size_t lds = 6 * (BM + BN) * 64 * 2 + 6 * gx;
      constexpr auto fn = gemm_v2_kernel<BM, BN, 6, A_K, B_K, MODE, EPI, COLSUM, FL & ~FL_Y8>;
      allow_lds<fn>(lds);
      MOE_LAUNCH(prof, fn, grid, dim3(256), lds, s, p);
    }
  } else if (stages >= 4) {
    const size_t lds = 4 * (BM + BN) * 64 * 2 + xs + 4 * gx;
    constexpr auto fn = gemm_v2_kernel<BM, BN, 4, A_K, B_K, MODE, EPI, COLSUM, FL & ~FL_Y8>;
    allow_lds<fn>(lds);
    MOE_LAUNCH(prof, fn, grid, dim3(256), lds, s, p);
  } else {
    const size_t lds = 3 * (BM + BN) * 64 * 2 + xs + 3 * gx;
    constexpr auto fn = gemm_v2_kernel<BM, BN, 3, A_K, B_K, MODE, EPI, COLSUM, FL & ~FL_Y8>;
    allow_lds<fn>(lds);
    MOE_LAUNCH(prof, fn, grid, dim3(256), lds, s, p);
  }
}

// Split-K workspace window: the device's registered workspace, or what a
// first problem of a paired launch left of it.
struct WsWin {
  float* ws = nullptr;
  size_t bytes = 0;
  int32_t* cnt = nullptr;
  int n_cnt = 0;
};
static WsWin device_ws() {
  WsWin w;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return w;
  w.ws = g_split_ws[dev].ws;
  w.bytes = g_split_ws[dev].ws_bytes;
  w.cnt = g_split_ws[dev].cnt;
  w.n_cnt = g_split_ws[dev].n_cnt;
  return w;
}

// Split-K factor for a launch of `tiles` output tiles (grid before splitting,
// a multiple of 8) when the window holds `part_floats` per slice; 1 = no split.
static int pick_split(int want, long long tiles, long long part_floats, const WsWin& w) {
  if (want <= 1) return 1;
  if (w.ws == nullptr || w.cnt == nullptr || tiles > w.n_cnt) return 1;
  while (want > 1 && (size_t)tiles * want * part_floats * 4 > w.bytes) --want;
  return want;
}

// Bind the chosen split to p; returns the window left after this problem.
static WsWin bind_split(GemmParams& p, int S, long long tiles, long long part_floats, const WsWin& w) {
  p.ksplit = S;
  if (S <= 1) return w;
  p.ws = w.ws;
  p.cnt = w.cnt;
  WsWin rest = w;
  const size_t used = (size_t)tiles * S * part_floats;
  rest.ws = w.ws + used;
  rest.bytes = w.bytes - used * 4;
  rest.cnt = w.cnt + tiles;
  rest.n_cnt = w.n_cnt - (int)tiles;
  return rest;
}

// ---------------------------------------------------------------------------
// launch plans: the per-shape choices of one grouped GEMM (kbench.py sweeps at
// the C2 shapes, MI355X; profiles/r01/kbench_*.jsonl)
// ---------------------------------------------------------------------------
struct RowsPlan {
  GemmParams p{};
  long long grid = 0;  // workgroups (tiles x split)
  int bm = 64, variant = 2, stages = 2, epi = 0;
  bool trans_b = true, dense = false;
  double bytes_fixed = 0, bytes_row = 0, flops_row = 0;
};
struct WgradPlan {
  GemmParams p{};
  long long grid = 0;
  int bm = 64, variant = 1, stages = 2;
  bool colsum = false;
  double bytes_fixed = 0, bytes_row = 0, flops_row = 0;
};

static int plan_rows(RowsPlan& pl, const void* a, const void* b, void* c, const int32_t* offsets, int G, int max_rows,
                     int N, int K, int trans_b, int epilogue, const float* bias, const void* aux,
                     const int32_t* a_gather, WsWin& win, const float* row_scale = nullptr) {
  if (G < 1 || G > 1024) return fail("grouped_gemm: G out of range");
  if (N <= 0 || K <= 0 || N % 128 != 0 || K % 64 != 0) return fail("grouped_gemm: need N % 128 == 0 and K % 64 == 0");
  if (max_rows < 0) return fail("grouped_gemm: max_rows < 0");
  if ((epilogue == MOE_EPI_BIAS || epilogue == MOE_EPI_BIAS_RELU) && bias == nullptr)
    return fail("grouped_gemm: bias epilogue without bias");
  if ((epilogue == MOE_EPI_RELU_MASK || epilogue == MOE_EPI_RELU_MASK_MX) && aux == nullptr)
    return fail("grouped_gemm: relu-mask epilogue without aux");
  if (epilogue < 0 || epilogue > 4) return fail("grouped_gemm: bad epilogue");
  GemmParams& p = pl.p;
  p = GemmParams{};
  p.dbg = g_gemm_debug;
  p.a = static_cast<const uint16_t*>(a);
  p.b = static_cast<const uint16_t*>(b);
  p.c = c;
  p.offsets = offsets;
  p.bias = bias;
  p.aux = static_cast<const uint16_t*>(aux);
  p.a_gather = a_gather;
  p.row_scale = row_scale;
  p.stride_b = (long long)N * K;
  p.lda = K;
  p.ldb = trans_b ? K : N;
  p.ldc = N;
  p.G = G;
  p.N = N;
  p.K = K;
  pl.trans_b = trans_b != 0;
  pl.epi = epilogue;
  // 64-row tiles (two 48-64 KiB workgroups per CU, one's epilogue overlapping
  // the other's main loop); LDS-DMA ring of 2 stages, 3 for K >= 1024 on grids
  // under one tile per CU (the deeper ring covers the longer K loop)
  const int nt = N / 128;
  pl.bm = g_rows_bm ? g_rows_bm : 64;
  const int mtiles = ((max_rows + pl.bm - 1) / pl.bm + G + 7) / 8 * 8;  // padded to the XCD count
  const long long tiles = (long long)mtiles * nt;
  // tile -> XCD map: contiguous row-tile chunks per XCD, so each L2 holds the
  // weights of ~1-2 experts instead of all of them (kbench: decoder dH 11.3 ->
  // 9.1 us, dX 15.0 -> 12.0, the rest unchanged; C2 step PMC: 52.9 -> 41.1 MB
  // of HBM traffic per grouped-GEMM launch at the same speed,
  // profiles/r02/xcd_map_ab.json).  xcd_map 1 forces round-robin (A/B).
  p.xmap = g_xcd_map == 1 ? 0 : 1;
  // split-K when the grid leaves CUs idle and K is long, for the dgrads
  // (MN-contiguous B; kbench: decoder dX 15.0 -> 11.5 us with the map above;
  // the K-contiguous forward GEMM2 only loses to the merge latency)
  int want = g_ksplit ? g_ksplit : ((!trans_b && tiles < 256 && K / 64 >= 16) ? 2 : 1);
  if (!g_ksplit && trans_b && g_fwd_ksplit > 1 && tiles < 256 && K / 64 >= 16) want = g_fwd_ksplit;
  if (want > K / 64) want = K / 64;
  const long long part = 256LL * (pl.bm / 32) * (128 / 32) * 4;
  const int S = pick_split(want, tiles, part, win);
  win = bind_split(p, S, tiles, part, win);
  pl.grid = tiles * S;
  pl.variant = (g_gemm_variant && !a_gather) ? g_gemm_variant : 2;  // the row gather needs the LDS-DMA ring
  pl.stages = g_gemm_stages ? g_gemm_stages : ((K >= 1024 && pl.grid < 256) ? g_deep_stages : 2);
  // algorithmic bytes: weights + bias once; per routed row A (K), C (N) and the relu-mask operand (N)
  const bool has_bias = epilogue == MOE_EPI_BIAS || epilogue == MOE_EPI_BIAS_RELU;
  const double mask_bytes = epilogue == MOE_EPI_RELU_MASK ? 2.0 * N : (epilogue == MOE_EPI_RELU_MASK_MX ? 1.0 * N : 0.0);
  pl.bytes_fixed = 2.0 * G * N * K + (has_bias ? 4.0 * G * N : 0.0);
  pl.bytes_row = 2.0 * K + 2.0 * N + mask_bytes;
  pl.flops_row = 2.0 * N * K;
  return 0;
}

static int plan_wgrad(WgradPlan& pl, const void* x, const void* y, void* c, void* colsum, const int32_t* offsets,
                      int G, int M, int N, int rows_hint, int out_bf16, const int32_t* b_gather, WsWin& win,
                      const int32_t* x_gather = nullptr, const float* x_scale = nullptr) {
  if (G < 1 || G > 1024) return fail("grouped_gemm_wgrad: G out of range");
  if (M <= 0 || N <= 0 || M % 64 != 0 || N % 128 != 0)
    return fail("grouped_gemm_wgrad: need M % 64 == 0 and N % 128 == 0");
  GemmParams& p = pl.p;
  p = GemmParams{};
  p.dbg = g_gemm_debug;
  p.a = static_cast<const uint16_t*>(x);
  p.b = static_cast<const uint16_t*>(y);
  p.c = c;
  p.offsets = offsets;
  p.colsum = static_cast<float*>(colsum);
  p.c_bf16 = out_bf16 ? 1 : 0;
  p.b_gather = b_gather;
  p.x_gather = x_gather;
  p.x_scale = x_gather != nullptr ? x_scale : nullptr;
  p.stride_c = (long long)M * N;
  p.lda = M;
  p.ldb = N;
  p.ldc = N;
  p.G = G;
  p.M = M;
  p.N = N;
  p.K = 0;
  pl.colsum = colsum != nullptr;
  const int ntn = N / 128;
  // 64-row tiles.  Gathered k-rows (one operand): the LDS-DMA ring with the
  // row indices staged in LDS ahead of the tiles (gemm_v2_body); both
  // operands gathered, or wgrad_dma = 1: the register-staged double buffer
  const bool gath = b_gather != nullptr || x_gather != nullptr;
  const bool both = b_gather != nullptr && x_gather != nullptr;
  const bool big = M % 128 == 0 && g_wgrad_bm == 128 && !gath;
  pl.bm = big ? 128 : 64;
  if (gath) pl.variant = (!both && g_wgrad_dma != 1) ? 2 : 1;
  else pl.variant = g_gemm_variant ? g_gemm_variant : 1;
  pl.stages = gath ? (g_wgrad_stages ? g_wgrad_stages : 2) : (g_gemm_stages ? g_gemm_stages : 2);
  int gpad = G >= 8 ? (G + 7) / 8 * 8 : G;
  // split-K over each group's rows: the output (G M N) is too small a grid to
  // fill the chip with K = the whole group; only for long groups: rows_hint / G
  // >= 1024 (kbench: encoder dW, 1,840 rows per expert, 30.0 -> 26.6 us;
  // decoder groups of ~600 rows lose to the merge latency, 11.5 -> 15.5 us)
  const long long tpg = (long long)(M / pl.bm) * ntn;
  long long tiles = tpg * gpad;
  // G = 1 (a dense linear layer's weight gradient, rtdetr TokenLinear): a
  // 256 x 256 output is only 8 tiles, so cut the rows over up to 8 slices
  // (>= 4 K-tiles each); tools/mm_probe_small.py, 2,400 rows: 21.9 -> 14.0 us,
  // against 21.1 us for hipBLASLt's dY^T X without the bias column sum
  const long long nkt = (rows_hint + 63) / 64;
  const int dense_want = (int)std::max(1LL, std::min({8LL, 256 / std::max(1LL, tiles), nkt / 4}));
  int want = g_ksplit ? g_ksplit
                      : (G == 1 ? dense_want : ((tiles <= 512 && rows_hint >= 1024LL * G) ? 2 : 1));
  p.split_min_kt = 0;
  if (want == 1 && g_wgrad_split_hot > 0 && G > 1 && !g_ksplit) {
    want = 2;
    p.split_min_kt = g_wgrad_split_hot;
  }
  if (want > 1 && tiles % 8 != 0) {  // split grids map 8-slot XCD rows: pad the group count
    gpad = (G + 7) / 8 * 8;
    tiles = tpg * gpad;
  }
  const long long part = 256LL * (pl.bm / 32) * 4 * 4 + 256LL * (pl.bm / 32);
  const int S = pick_split(want, tiles, part, win);
  if (S == 1) {
    gpad = G >= 8 ? (G + 7) / 8 * 8 : G;
    tiles = tpg * gpad;
  }
  win = bind_split(p, S, tiles, part, win);
  pl.grid = tiles * S;
  // algorithmic bytes: C (+ colsum) once; per routed row one row of X (M) and of Y (N)
  const double osz = out_bf16 ? 2.0 : 4.0;
  pl.bytes_fixed = osz * G * M * N + (colsum ? osz * G * M : 0.0);
  pl.bytes_row = 2.0 * (M + N);
  pl.flops_row = 2.0 * M * N;
  return 0;
}

// kernel instantiation of a rows plan (callers check the plan's fields)
template <int BM, int EPI, bool BK, int FL>
static void launch_rows_bm(const RowsPlan& pl, hipStream_t s, const ProfScope& prof) {
  launch<BM, 128, true, BK, MODE_ROWS, EPI, false, FL>(pl.p, dim3(pl.grid), s, prof, pl.variant, pl.stages);
}
template <int BM, bool BK>
static void launch_rows_epi(const RowsPlan& pl, hipStream_t s, const ProfScope& prof) {
  switch (pl.epi) {
    case MOE_EPI_NONE: launch_rows_bm<BM, MOE_EPI_NONE, BK, 0>(pl, s, prof); break;
    case MOE_EPI_BIAS: launch_rows_bm<BM, MOE_EPI_BIAS, BK, 0>(pl, s, prof); break;
    case MOE_EPI_BIAS_RELU: launch_rows_bm<BM, MOE_EPI_BIAS_RELU, BK, 0>(pl, s, prof); break;
    case MOE_EPI_RELU_MASK: launch_rows_bm<BM, MOE_EPI_RELU_MASK, BK, 0>(pl, s, prof); break;
    default: launch_rows_bm<BM, MOE_EPI_RELU_MASK, BK, FL_AUX8>(pl, s, prof); break;
  }
}
template <bool BK>
static void launch_rows_dense(const RowsPlan& pl, hipStream_t s, const ProfScope& prof) {
  switch (pl.epi) {
    case MOE_EPI_BIAS: launch_rows_bm<64, MOE_EPI_BIAS, BK, FL_DENSE>(pl, s, prof); break;
    case MOE_EPI_BIAS_RELU: launch_rows_bm<64, MOE_EPI_BIAS_RELU, BK, FL_DENSE>(pl, s, prof); break;
    case MOE_EPI_RELU_MASK: launch_rows_bm<64, MOE_EPI_RELU_MASK, BK, FL_DENSE>(pl, s, prof); break;
    default: launch_rows_bm<64, MOE_EPI_NONE, BK, FL_DENSE>(pl, s, prof); break;
  }
}
static void launch_rows(const RowsPlan& pl, hipStream_t s, const ProfScope& prof) {
  if (pl.dense && pl.bm == 64 && pl.epi <= MOE_EPI_RELU_MASK) {
    if (pl.trans_b) launch_rows_dense<true>(pl, s, prof);
    else launch_rows_dense<false>(pl, s, prof);
    return;
  }
  if (pl.bm == 128) {
    if (pl.trans_b) launch_rows_epi<128, true>(pl, s, prof);
    else launch_rows_epi<128, false>(pl, s, prof);
  } else {
    if (pl.trans_b) launch_rows_epi<64, true>(pl, s, prof);
    else launch_rows_epi<64, false>(pl, s, prof);
  }
}
template <int FL>
static void launch_wgrad(const WgradPlan& pl, hipStream_t s, const ProfScope& prof) {
  if (pl.bm == 128) {
    if (pl.colsum) launch<128, 128, false, false, MODE_WGRAD, MOE_EPI_NONE, true, FL>(pl.p, dim3(pl.grid), s, prof, pl.variant, pl.stages);
    else launch<128, 128, false, false, MODE_WGRAD, MOE_EPI_NONE, false, FL>(pl.p, dim3(pl.grid), s, prof, pl.variant, pl.stages);
  } else {
    if (pl.colsum) launch<64, 128, false, false, MODE_WGRAD, MOE_EPI_NONE, true, FL>(pl.p, dim3(pl.grid), s, prof, pl.variant, pl.stages);
    else launch<64, 128, false, false, MODE_WGRAD, MOE_EPI_NONE, false, FL>(pl.p, dim3(pl.grid), s, prof, pl.variant, pl.stages);
  }
}

// Paired launch: a dgrad (ROWS, trans_b = 0, BM 64, ring of 2 or 3 stages)
// and a weight gradient (WGRAD, BM 64, register-staged, colsum) of the same
// expert weight.  Other plans fall back to two launches.
// The weight gradient's workgroups come FIRST: they are few (one per output
// tile) and each runs the group's whole K loop; dispatched ahead of the
// dgrad's many short workgroups they overlap them instead of trailing them
// (kbench: the reverse order ran the two back to back inside the launch).
// SW: the weight gradient's body -- 0 = register-staged (v1), 2 / 3 = the
// LDS-DMA ring of that depth (gathered k-rows, gemm_v2_body).
template <int S, int SW, int EPI, int FLR, int FLW>
static void launch_pair_k(const RowsPlan& r, const WgradPlan& w, hipStream_t s, const ProfScope& prof) {
  using R = BodyV2<64, 128, S, true, false, MODE_ROWS, EPI, false, FLR>;
  using W = std::conditional_t<SW == 0, BodyV1<64, 128, false, false, MODE_WGRAD, MOE_EPI_NONE, true, FLW>,
                               BodyV2<64, 128, (SW ? SW : 2), false, false, MODE_WGRAD, MOE_EPI_NONE, true, FLW>>;
  constexpr auto fn = gemm_pair_kernel<W, R>;
  const size_t lds_r = (size_t)S * (64 + 128) * 64 * 2;
  const size_t lds_w = SW == 0 ? 2 * (64 + 128) * 64 * 2 : (size_t)SW * ((64 + 128) * 64 * 2 + 768);
  const size_t lds = lds_r > lds_w ? lds_r : lds_w;
  allow_lds<fn>(lds);
  MOE_LAUNCH(prof, fn, dim3(r.grid + w.grid), dim3(256), lds, s, w.p, r.p, (int)w.grid);
}
static bool pair_ok(const RowsPlan& r, const WgradPlan& w) {
  return r.bm == 64 && !r.trans_b && r.variant == 2 && (r.stages == 2 || r.stages == 3) && w.grid % 8 == 0 &&
         w.bm == 64 && (w.variant == 1 || (w.variant == 2 && (w.stages == 2 || w.stages == 3))) && w.colsum &&
         (r.epi == MOE_EPI_NONE || r.epi == MOE_EPI_RELU_MASK || r.epi == MOE_EPI_RELU_MASK_MX);
}
template <int S, int FLW>
static void launch_pair_s(const RowsPlan& r, const WgradPlan& w, hipStream_t s, const ProfScope& prof) {
#define GG_PAIR(SW_)                                                                          \
  switch (r.epi) {                                                                             \
    case MOE_EPI_NONE: launch_pair_k<S, SW_, MOE_EPI_NONE, 0, FLW>(r, w, s, prof); break;       \
    case MOE_EPI_RELU_MASK: launch_pair_k<S, SW_, MOE_EPI_RELU_MASK, 0, FLW>(r, w, s, prof); break; \
    default: launch_pair_k<S, SW_, MOE_EPI_RELU_MASK, FL_AUX8, FLW>(r, w, s, prof); break;      \
  }
  if (w.variant == 1) {
    GG_PAIR(0)
  } else if (w.stages == 3) {
    GG_PAIR(3)
  } else {
    GG_PAIR(2)
  }
#undef GG_PAIR
}
template <int FLW>
static void launch_pair(const RowsPlan& r, const WgradPlan& w, hipStream_t s, const ProfScope& prof) {
  if (r.stages == 3) launch_pair_s<3, FLW>(r, w, s, prof);
  else launch_pair_s<2, FLW>(r, w, s, prof);
}

// The expert FFN backward's second launch: dW2 (+ db2) and dW1 (+ db1) as
// gathered-k-row LDS-DMA weight gradients and dXp as the dgrad, all three in
// one grid.  The caller checks triple_ok.
static bool triple_ok(const RowsPlan& r, const WgradPlan& w2, const WgradPlan& w1) {
  auto wok = [](const WgradPlan& w) {
    return w.bm == 64 && w.variant == 2 && (w.stages == 2 || w.stages == 3) && w.colsum && w.grid % 8 == 0;
  };
  return r.bm == 64 && !r.trans_b && r.variant == 2 && (r.stages == 2 || r.stages == 3) && r.epi == MOE_EPI_NONE &&
         r.grid % 8 == 0 && wok(w2) && wok(w1) && w2.stages == w1.stages;
}
template <int S, int SW>
static void launch_triple_k(const RowsPlan& r, const WgradPlan& w2, const WgradPlan& w1, hipStream_t s,
                            const ProfScope& prof) {
  using R = BodyV2<64, 128, S, true, false, MODE_ROWS, MOE_EPI_NONE, false, 0>;
  using W = BodyV2<64, 128, SW, false, false, MODE_WGRAD, MOE_EPI_NONE, true, 0>;
  constexpr auto fn = gemm_triple_kernel<W, W, R>;
  const size_t lds_r = (size_t)S * (64 + 128) * 64 * 2;
  const size_t lds_w = (size_t)SW * ((64 + 128) * 64 * 2 + 768);
  const size_t lds = lds_r > lds_w ? lds_r : lds_w;
  allow_lds<fn>(lds);
  const int n1 = (int)w2.grid, n12 = (int)(w2.grid + w1.grid);
  MOE_LAUNCH(prof, fn, dim3(r.grid + w2.grid + w1.grid), dim3(256), lds, s, w2.p, w1.p, r.p, n1, n12);
}
static void launch_triple(const RowsPlan& r, const WgradPlan& w2, const WgradPlan& w1, hipStream_t s,
                          const ProfScope& prof) {
  if (r.stages == 3) {
    if (w2.stages == 3) launch_triple_k<3, 3>(r, w2, w1, s, prof);
    else launch_triple_k<3, 2>(r, w2, w1, s, prof);
  } else {
    if (w2.stages == 3) launch_triple_k<2, 3>(r, w2, w1, s, prof);
    else launch_triple_k<2, 2>(r, w2, w1, s, prof);
  }
}

}  // namespace moe

using namespace moe;

extern "C" int moe_set_splitk_workspace(void* ws, size_t ws_bytes, int32_t* counters, int n_counters) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return fail("set_splitk_workspace: no device");
  if ((ws == nullptr) != (counters == nullptr) || n_counters < 0)
    return fail("set_splitk_workspace: ws and counters must both be set or both NULL");
  if (ws != nullptr && (reinterpret_cast<uintptr_t>(ws) & 15) != 0)
    return fail("set_splitk_workspace: ws must be 16-B aligned");
  g_split_ws[dev].ws = static_cast<float*>(ws);
  g_split_ws[dev].ws_bytes = ws ? ws_bytes : 0;
  g_split_ws[dev].cnt = counters;
  g_split_ws[dev].n_cnt = counters ? n_counters : 0;
  return 0;
}

extern "C" int moe_set_tuning(const char* key, int value) {
  const std::string k = key ? key : "";
  if (k == "gemm_variant" && value >= 0 && value <= 2) { g_gemm_variant = value; return 0; }
  if (k == "gemm_stages" && (value == 0 || (value >= 2 && value <= 4))) { g_gemm_stages = value; return 0; }
  if (k == "deep_stages" && (value == 0 || value == 2 || value == 3 || value == 4 || value == 6)) {
    g_deep_stages = value ? value : 3;  // (0: the default)
    return 0;
  }
  if (k == "gemm_debug" && value >= 0 && value <= 3) { g_gemm_debug = value; return 0; }
  if (k == "rows_bm" && (value == 0 || value == 64 || value == 128)) { g_rows_bm = value; return 0; }
  if (k == "wgrad_bm" && (value == 0 || value == 64 || value == 128)) { g_wgrad_bm = value; return 0; }
  if (k == "xcd_map" && value >= 0 && value <= 2) { g_xcd_map = value; return 0; }
  if (k == "ksplit" && value >= 0 && value <= 8) { g_ksplit = value; return 0; }
  if (k == "gemm_pair" && value >= 0 && value <= 1) { g_gemm_pair_off = value ? 0 : 1; return 0; }
  if (k == "wgrad_dma" && value >= 0 && value <= 1) { g_wgrad_dma = value; return 0; }
  if (k == "wgrad_stages" && (value == 0 || value == 2 || value == 3)) { g_wgrad_stages = value; return 0; }
  if (k == "wgrad_split_hot" && value >= 0 && value <= 1024) { g_wgrad_split_hot = value; return 0; }
  if (k == "fwd_ksplit" && value >= 0 && value <= 8) { g_fwd_ksplit = value; return 0; }
  if (k == "bwd2_max_rows" && value >= 0) { g_bwd2_max_rows = value; return 0; }
  if (k == "bwd2_dx_split" && value >= 0 && value <= 1) { g_bwd2_dx_split = value; return 0; }
  if (k == "msda_generic" && value >= 0 && value <= 3) { g_msda_generic = value; return 0; }
  return fail("moe_set_tuning: unknown key or value");
}

extern "C" int moe_grouped_gemm_gather(int dtype, const void* a, const int32_t* a_gather, const void* b, void* c,
                                       const int32_t* offsets, int G, int max_rows, int N, int K, int trans_b,
                                       int epilogue, const float* bias, const void* aux, hipStream_t stream) {
  const bool bias16 = (dtype & MOE_BIAS_BF16) != 0;
  const bool dense = (dtype & MOE_DENSE_LAYER) != 0;  // a dense layer on this kernel: profiled apart from the experts
  if ((dtype & ~(MOE_BIAS_BF16 | MOE_DENSE_LAYER)) != MOE_BF16) return fail("grouped_gemm: only MOE_BF16 is implemented");
  RowsPlan pl;
  WsWin win = device_ws();
  if (plan_rows(pl, a, b, c, offsets, G, max_rows, N, K, trans_b, epilogue, bias, aux, a_gather, win)) return -1;
  pl.p.bias_bf16 = bias16 ? 1 : 0;
  pl.dense = dense;
  if (bias16) pl.bytes_fixed -= 2.0 * G * N;  // bias bytes: 2 per element, not 4
  if (max_rows == 0) return 0;
  ProfScope prof(stream, dense ? PROF_LINEAR : PROF_GEMM, pl.bytes_fixed, true, pl.bytes_row, pl.flops_row);
  pl.p.prof_rows = prof.rows_slot();
  launch_rows(pl, stream, prof);
  return check_launch("moe_grouped_gemm");
}

extern "C" int moe_grouped_gemm_scatter(int dtype, const void* a, const int32_t* a_gather, const void* b, void* c,
                                        const int32_t* c_rows, const int32_t* offsets, int G, int max_rows, int N,
                                        int K, int trans_b, int epilogue, const float* bias, const void* aux,
                                        hipStream_t stream) {
  if ((dtype & ~MOE_BIAS_BF16) != MOE_BF16) return fail("grouped_gemm_scatter: only MOE_BF16 is implemented");
  if (c_rows == nullptr) return fail("grouped_gemm_scatter: c_rows is NULL");
  RowsPlan pl;
  WsWin win = device_ws();
  if (plan_rows(pl, a, b, c, offsets, G, max_rows, N, K, trans_b, epilogue, bias, aux, a_gather, win)) return -1;
  pl.p.bias_bf16 = (dtype & MOE_BIAS_BF16) ? 1 : 0;
  pl.p.c_rows = c_rows;
  if (pl.p.bias_bf16) pl.bytes_fixed -= 2.0 * G * N;
  if (max_rows == 0) return 0;
  ProfScope prof(stream, PROF_GEMM, pl.bytes_fixed, true, pl.bytes_row, pl.flops_row);
  pl.p.prof_rows = prof.rows_slot();
  launch_rows(pl, stream, prof);
  return check_launch("moe_grouped_gemm_scatter");
}

extern "C" int moe_grouped_gemm(int dtype, const void* a, const void* b, void* c,
                                const int32_t* offsets, int G, int max_rows, int N, int K,
                                int trans_b, int epilogue, const float* bias, const void* aux,
                                const float* scales, hipStream_t stream) {
  (void)scales;
  return moe_grouped_gemm_gather(dtype, a, nullptr, b, c, offsets, G, max_rows, N, K, trans_b, epilogue, bias, aux,
                                 stream);
}

extern "C" int moe_grouped_gemm_wgrad_rows(int dtype, const void* x, const void* y, void* c,
                                           void* colsum, const int32_t* offsets, int G, int M,
                                           int N, int rows_hint, int out_bf16, hipStream_t stream);

extern "C" int moe_grouped_gemm_wgrad(int dtype, const void* x, const void* y, float* c,
                                      float* colsum, const int32_t* offsets, int G, int M,
                                      int N, hipStream_t stream) {
  return moe_grouped_gemm_wgrad_rows(dtype, x, y, c, colsum, offsets, G, M, N, 0, 0, stream);
}

extern "C" int moe_grouped_gemm_wgrad_gather(int dtype, const void* x, const void* y, const int32_t* y_gather,
                                             void* c, void* colsum, const int32_t* offsets, int G, int M, int N,
                                             int rows_hint, int out_bf16, hipStream_t stream) {
  if (dtype != MOE_BF16) return fail("grouped_gemm_wgrad: only MOE_BF16 is implemented");
  WgradPlan pl;
  WsWin win = device_ws();
  if (plan_wgrad(pl, x, y, c, colsum, offsets, G, M, N, rows_hint, out_bf16, y_gather, win)) return -1;
  ProfScope prof(stream, PROF_GEMM, pl.bytes_fixed, true, pl.bytes_row, pl.flops_row);
  pl.p.prof_rows = prof.rows_slot();
  launch_wgrad<0>(pl, stream, prof);
  return check_launch("moe_grouped_gemm_wgrad");
}

extern "C" int moe_grouped_gemm_wgrad_rows(int dtype, const void* x, const void* y, void* c,
                                           void* colsum, const int32_t* offsets, int G, int M,
                                           int N, int rows_hint, int out_bf16, hipStream_t stream) {
  return moe_grouped_gemm_wgrad_gather(dtype, x, y, nullptr, c, colsum, offsets, G, M, N, rows_hint, out_bf16,
                                       stream);
}

extern "C" int rtdetr_linear_wgrad(const void* gy, const void* x, void* dw, void* db, const int32_t* offsets,
                                   int K, int M, int N, int out_bf16, hipStream_t stream) {
  (void)offsets;  // rows are [0, K): the kernel takes them from its parameters
  WgradPlan pl;
  WsWin win = device_ws();
  if (db == nullptr) return fail("rtdetr_linear_wgrad: db (the bias gradient) is required");
  if (K <= 0) return fail("rtdetr_linear_wgrad: K must be positive");
  if (plan_wgrad(pl, gy, x, dw, db, nullptr, 1, M, N, K, out_bf16, nullptr, win)) return -1;
  pl.p.dense_rows = K;
  ProfScope prof(stream, PROF_LINEAR, pl.bytes_fixed + pl.bytes_row * K, false, 0.0, pl.flops_row * K);
  if (pl.bm == 64 && pl.variant == 1) {
    constexpr size_t lds = 2 * (64 + 128) * 64 * 2;
    MOE_LAUNCH(prof, linear_wgrad_kernel, dim3(pl.grid), dim3(256), lds, stream, pl.p);
  } else {  // a tuning knob (bm 128 / the DMA ring) asked for another body
    launch_wgrad<0>(pl, stream, prof);
  }
  return check_launch("rtdetr_linear_wgrad");
}

extern "C" int rtdetr_linear_wgrad_batch(int n, const void* const* gy, const void* const* x, void* const* dw,
                                         void* const* db, const int* K, const int* M, const int* N, int out_bf16,
                                         hipStream_t stream) {
  if (n <= 0) return 0;
  if (n > MAX_DENSE_BATCH) return fail("rtdetr_linear_wgrad_batch: at most 24 problems per launch");
  WsWin win = device_ws();
  DenseBatch b{};
  b.n = n;
  b.c_bf16 = out_bf16 ? 1 : 0;
  b.dbg = g_gemm_debug;
  constexpr long long part = 256LL * 2 * 4 * 4 + 256LL * 2;  // fp32 floats per slice of a 64 x 128 tile
  // Split each problem's rows so that the whole batch is ~3 workgroups per CU
  // of about equal K-loop length: slices of >= 4 K-tiles, at most 8 per tile.
  long long iters = 0;
  for (int q = 0; q < n; ++q) {
    if (gy[q] == nullptr || x[q] == nullptr || dw[q] == nullptr || db[q] == nullptr)
      return fail("rtdetr_linear_wgrad_batch: null operand");
    if (K[q] <= 0 || M[q] <= 0 || N[q] <= 0 || M[q] % 64 != 0 || N[q] % 128 != 0)
      return fail("rtdetr_linear_wgrad_batch: need K > 0, M % 64 == 0 and N % 128 == 0");
    iters += (long long)(M[q] / 64) * (N[q] / 128) * ((K[q] + 63) / 64);
  }
  const long long per_wg = std::max(4LL, (iters + 767) / 768);  // K-tiles per workgroup
  double bytes = 0.0, flops = 0.0;
  long long grid = 0;
  for (int q = 0; q < n; ++q) {
    DenseProb& d = b.p[q];
    d.gy = static_cast<const uint16_t*>(gy[q]);
    d.x = static_cast<const uint16_t*>(x[q]);
    d.dw = dw[q];
    d.db = db[q];
    d.K = K[q];
    d.M = M[q];
    d.N = N[q];
    const long long tiles = ((long long)(M[q] / 64) * (N[q] / 128) + 7) / 8 * 8;
    const long long nkt = (K[q] + 63) / 64;
    int want = (int)std::min(8LL, std::max(1LL, (nkt + per_wg - 1) / per_wg));
    want = pick_split(want, tiles, part, win);
    GemmParams tmp{};
    win = bind_split(tmp, want, tiles, part, win);
    d.ksplit = tmp.ksplit;
    d.ws = tmp.ws;
    d.cnt = tmp.cnt;
    b.base[q] = (int)grid;
    grid += tiles * d.ksplit;
    const double osz = out_bf16 ? 2.0 : 4.0;
    bytes += osz * ((double)M[q] * N[q] + M[q]) + 2.0 * K[q] * (M[q] + N[q]);
    flops += 2.0 * M[q] * N[q] * K[q];
  }
  b.base[n] = (int)grid;
  ProfScope prof(stream, PROF_LINEAR, bytes, false, 0.0, flops);
  constexpr size_t lds = 2 * (64 + 128) * 64 * 2;
  MOE_LAUNCH(prof, linear_wgrad_batch_kernel, dim3((unsigned)grid), dim3(256), lds, stream, b);
  return check_launch("rtdetr_linear_wgrad_batch");
}

extern "C" int moe_grouped_gemm_bwd_pair_scatter(const void* a, const int32_t* a_gather, const float* row_scale,
                                                 const void* b, void* c, const int32_t* c_rows,
                                                 const int32_t* offsets, int G, int max_rows, int N, int K,
                                                 int epilogue, const void* aux, const void* wx,
                                                 const int32_t* wx_gather, const float* wx_scale, const void* wy,
                                                 const int32_t* wy_gather, void* wc, void* wcolsum, int M2, int N2,
                                                 int out_bf16, hipStream_t stream) {
  RowsPlan r;
  WgradPlan w;
  WsWin win = device_ws();
  if (plan_rows(r, a, b, c, offsets, G, max_rows, N, K, 0, epilogue, nullptr, aux, a_gather, win, row_scale))
    return -1;
  r.p.c_rows = c_rows;
  if (wc == nullptr) {  // dgrad only (the caller computes the weight gradient elsewhere)
    if (wcolsum != nullptr) return fail("grouped_gemm_bwd_pair: wcolsum without wc");
    if (max_rows == 0) return 0;
    ProfScope prof(stream, PROF_GEMM, r.bytes_fixed, true, r.bytes_row, r.flops_row);
    r.p.prof_rows = prof.rows_slot();
    launch_rows(r, stream, prof);
    return check_launch("moe_grouped_gemm_bwd_pair (dgrad)");
  }
  if (plan_wgrad(w, wx, wy, wc, wcolsum, offsets, G, M2, N2, max_rows, out_bf16, wy_gather, win, wx_gather,
                 wx_scale))
    return -1;
  if (max_rows == 0) {  // no routed rows: the weight gradient is zero
    ProfScope prof(stream, PROF_GEMM, w.bytes_fixed, true, w.bytes_row, w.flops_row);
    w.p.prof_rows = prof.rows_slot();
    launch_wgrad<0>(w, stream, prof);
    return check_launch("moe_grouped_gemm_bwd_pair (wgrad)");
  }
  if (g_gemm_pair_off || !pair_ok(r, w)) {  // two launches
    {
      ProfScope prof(stream, PROF_GEMM, r.bytes_fixed, true, r.bytes_row, r.flops_row);
      r.p.prof_rows = prof.rows_slot();
      launch_rows(r, stream, prof);
    }
    if (check_launch("moe_grouped_gemm_bwd_pair (dgrad)")) return -1;
    ProfScope prof(stream, PROF_GEMM, w.bytes_fixed, true, w.bytes_row, w.flops_row);
    w.p.prof_rows = prof.rows_slot();
    launch_wgrad<0>(w, stream, prof);
    return check_launch("moe_grouped_gemm_bwd_pair (wgrad)");
  }
  ProfScope prof(stream, PROF_GEMM, r.bytes_fixed + w.bytes_fixed, true, r.bytes_row + w.bytes_row,
                 r.flops_row + w.flops_row);
  r.p.prof_rows = prof.rows_slot();
  launch_pair<0>(r, w, stream, prof);
  return check_launch("moe_grouped_gemm_bwd_pair");
}

// The routed expert FFN backward in TWO launches (single-GPU bf16 layer):
//   1. dH = relu'(H) * (gate[r] dy[tok[r]] . W2_g)                     (dgrad)
//   2. dXp = dH . W1_g,  dW2 = dYp^T H (+ db2),  dW1 = dH^T x[tok] (+ db1) (one grid)
// where dYp = bf16(gate * dy[tok]) is formed while staging.  The paired form
// ({dH, dW2} then {dXp, dW1}) runs the two weight gradients -- the long K
// loops, skewed by the routed counts -- one after the other; here they run
// beside each other and beside dXp, after the short dH launch.
extern "C" int moe_expert_ffn_bwd(const void* dy, const int32_t* tok, const float* gate, const void* x, const void* h,
                                  const void* w1, const void* w2, const int32_t* offsets, int G, int max_rows, int F,
                                  int d, void* dh, void* dxp, void* dw1, void* db1, void* dw2, void* db2, int out_bf16,
                                  hipStream_t stream) {
  if (dy == nullptr || tok == nullptr || gate == nullptr || x == nullptr || h == nullptr || w1 == nullptr ||
      w2 == nullptr || dh == nullptr || dxp == nullptr || dw1 == nullptr || db1 == nullptr || dw2 == nullptr ||
      db2 == nullptr || offsets == nullptr)
    return fail("expert_ffn_bwd: NULL pointer");
  if (max_rows <= 0 || g_gemm_pair_off || (long long)max_rows > (long long)g_bwd2_max_rows * G) {
    // paired launches: no rows (they write the zero weight gradients), the A/B
    // switch, or experts long enough that the one-grid form needs two rounds
    if (moe_grouped_gemm_bwd_pair_scatter(dy, tok, gate, w2, dh, nullptr, offsets, G, max_rows, F, d,
                                          MOE_EPI_RELU_MASK, h, dy, tok, gate, h, nullptr, dw2, db2, d, F, out_bf16,
                                          stream))
      return -1;
    return moe_grouped_gemm_bwd_pair_scatter(dh, nullptr, nullptr, w1, dxp, nullptr, offsets, G, max_rows, d, F,
                                             MOE_EPI_NONE, nullptr, dh, nullptr, nullptr, x, tok, dw1, db1, F, d,
                                             out_bf16, stream);
  }
  WsWin win = device_ws();
  RowsPlan r2, r1;
  WgradPlan wg2, wg1;
  if (plan_rows(r2, dy, w2, dh, offsets, G, max_rows, F, d, 0, MOE_EPI_RELU_MASK, nullptr, h, tok, win, gate))
    return -1;
  {  // launch 1: dH (its split-K window, if any, is free again after this launch)
    ProfScope prof(stream, PROF_GEMM, r2.bytes_fixed, true, r2.bytes_row, r2.flops_row);
    r2.p.prof_rows = prof.rows_slot();
    launch_rows(r2, stream, prof);
    if (check_launch("moe_expert_ffn_bwd (dH)")) return -1;
  }
  win = device_ws();
  if (plan_wgrad(wg2, dy, h, dw2, db2, offsets, G, d, F, max_rows, out_bf16, nullptr, win, tok, gate)) return -1;
  if (plan_wgrad(wg1, dh, x, dw1, db1, offsets, G, F, d, max_rows, out_bf16, tok, win)) return -1;
  {
    const int ks_saved = g_ksplit;
    if (g_bwd2_dx_split == 1) g_ksplit = 1;  // (plan-time override: the dXp body unsplit)
    const int rc = plan_rows(r1, dh, w1, dxp, offsets, G, max_rows, d, F, 0, MOE_EPI_NONE, nullptr, nullptr, nullptr,
                             win);
    g_ksplit = ks_saved;
    if (rc) return -1;
  }
  if (!triple_ok(r1, wg2, wg1)) {  // separate launches (shapes the one-grid form does not take)
    {
      ProfScope prof(stream, PROF_GEMM, r1.bytes_fixed, true, r1.bytes_row, r1.flops_row);
      r1.p.prof_rows = prof.rows_slot();
      launch_rows(r1, stream, prof);
    }
    if (check_launch("moe_expert_ffn_bwd (dXp)")) return -1;
    ProfScope p2(stream, PROF_GEMM, wg2.bytes_fixed, true, wg2.bytes_row, wg2.flops_row);
    wg2.p.prof_rows = p2.rows_slot();
    launch_wgrad<0>(wg2, stream, p2);
    if (check_launch("moe_expert_ffn_bwd (dW2)")) return -1;
    ProfScope p1(stream, PROF_GEMM, wg1.bytes_fixed, true, wg1.bytes_row, wg1.flops_row);
    wg1.p.prof_rows = p1.rows_slot();
    launch_wgrad<0>(wg1, stream, p1);
    return check_launch("moe_expert_ffn_bwd (dW1)");
  }
  ProfScope prof(stream, PROF_GEMM, r1.bytes_fixed + wg2.bytes_fixed + wg1.bytes_fixed, true,
                 r1.bytes_row + wg2.bytes_row + wg1.bytes_row, r1.flops_row + wg2.flops_row + wg1.flops_row);
  r1.p.prof_rows = prof.rows_slot();
  launch_triple(r1, wg2, wg1, stream, prof);
  return check_launch("moe_expert_ffn_bwd");
}

extern "C" int moe_grouped_gemm_bwd_pair(const void* a, const int32_t* a_gather, const float* row_scale,
                                         const void* b, void* c, const int32_t* offsets, int G, int max_rows, int N,
                                         int K, int epilogue, const void* aux, const void* wx,
                                         const int32_t* wx_gather, const float* wx_scale, const void* wy,
                                         const int32_t* wy_gather, void* wc, void* wcolsum, int M2, int N2,
                                         int out_bf16, hipStream_t stream) {
  return moe_grouped_gemm_bwd_pair_scatter(a, a_gather, row_scale, b, c, nullptr, offsets, G, max_rows, N, K,
                                           epilogue, aux, wx, wx_gather, wx_scale, wy, wy_gather, wc, wcolsum, M2,
                                           N2, out_bf16, stream);
}

// ---------------------------------------------------------------------------
// MXFP8 expert GEMMs (config C5; SURVEY 8a rows a5/a7 with the fp8 expert path)
// ---------------------------------------------------------------------------
extern "C" int moe_grouped_gemm_mx(const void* a, const void* a_scales, const void* b, const void* b_scales,
                                   void* c, void* c_scales, const int32_t* offsets, int G, int max_rows, int N,
                                   int K, int epilogue, const float* bias, hipStream_t stream) {
  if (G < 1 || G > 1024) return fail("grouped_gemm_mx: G out of range");
  if (N <= 0 || K <= 0 || N % 128 != 0 || K % 128 != 0 || K > 8192)
    return fail("grouped_gemm_mx: need N % 128 == 0 and K % 128 == 0 (K <= 8192)");
  if (max_rows < 0) return fail("grouped_gemm_mx: max_rows < 0");
  if (epilogue < 0 || epilogue > 2) return fail("grouped_gemm_mx: epilogue must be NONE, BIAS or BIAS_RELU");
  if (epilogue != MOE_EPI_NONE && bias == nullptr) return fail("grouped_gemm_mx: bias epilogue without bias");
  if (a_scales == nullptr || b_scales == nullptr) return fail("grouped_gemm_mx: missing operand scales");
  if (max_rows == 0) return 0;
  GemmParams p{};
  p.dbg = g_gemm_debug;
  p.xmap = g_xcd_map == 1 ? 0 : 1;  // contiguous row-tile chunks per XCD (see plan_rows)
  // e4m3 rows addressed as 16-bit pairs: the bf16 tile machinery moves [R][128 B] K-tiles
  p.a = static_cast<const uint16_t*>(a);
  p.b = static_cast<const uint16_t*>(b);
  p.c = c;
  p.cs = static_cast<uint8_t*>(c_scales);
  p.as = static_cast<const uint8_t*>(a_scales);
  p.bs = static_cast<const uint8_t*>(b_scales);
  p.ksb = K / 32;
  p.offsets = offsets;
  p.bias = bias;
  p.stride_b = (long long)N * K / 2;
  p.lda = K / 2;
  p.ldb = K / 2;
  p.ldc = N;
  p.G = G;
  p.N = N;
  p.K = K / 2;
  const int nt = N / 128;
  const int BMsel = g_rows_bm ? g_rows_bm : 64;
  const int mtiles = ((max_rows + BMsel - 1) / BMsel + G + 7) / 8 * 8;
  dim3 grid(mtiles * nt);
  const int stages = g_gemm_stages ? g_gemm_stages : ((K >= 2048 && (long long)mtiles * nt < 256) ? 3 : 2);
  const bool cq = c_scales != nullptr;
  const bool has_bias = epilogue != MOE_EPI_NONE;
  // algorithmic bytes: e4m3 weights + exponents (+ bias) once; per routed row A (K + K/32), C (2N or N + N/32)
  ProfScope prof(stream, PROF_GEMM_FP8, G * N * (K + K / 32.0) + (has_bias ? 4.0 * G * N : 0.0), true,
                 K + K / 32.0 + (cq ? N + N / 32.0 : 2.0 * N), 2.0 * N * K);
  p.prof_rows = prof.rows_slot();
#define GM_ROWS(BM, EPI)                                                                                     \
  do {                                                                                                       \
    if (cq) launch<BM, 128, true, true, MODE_ROWS, EPI, false, FL_MX | FL_CQ>(p, grid, stream, prof, 2, stages); \
    else launch<BM, 128, true, true, MODE_ROWS, EPI, false, FL_MX>(p, grid, stream, prof, 2, stages);       \
  } while (0)
#define GM_EPI(BM)                                                \
  switch (epilogue) {                                            \
    case MOE_EPI_NONE: GM_ROWS(BM, MOE_EPI_NONE); break;          \
    case MOE_EPI_BIAS: GM_ROWS(BM, MOE_EPI_BIAS); break;          \
    default: GM_ROWS(BM, MOE_EPI_BIAS_RELU); break;               \
  }
  if (BMsel == 128) {
    GM_EPI(128)
  } else {
    GM_EPI(64)
  }
#undef GM_EPI
#undef GM_ROWS
  return check_launch("moe_grouped_gemm_mx");
}

extern "C" int moe_grouped_gemm_wgrad_mx(const void* x, const void* y, const void* y_scales, float* c,
                                         float* colsum, const int32_t* offsets, int G, int M, int N,
                                         hipStream_t stream) {
  if (G < 1 || G > 1024) return fail("grouped_gemm_wgrad_mx: G out of range");
  if (M <= 0 || N <= 0 || M % 64 != 0 || N % 128 != 0)
    return fail("grouped_gemm_wgrad_mx: need M % 64 == 0 and N % 128 == 0");
  if (y_scales == nullptr) return fail("grouped_gemm_wgrad_mx: missing Y scales");
  GemmParams p{};
  p.dbg = g_gemm_debug;
  p.a = static_cast<const uint16_t*>(x);
  p.b = static_cast<const uint16_t*>(y);
  p.as = static_cast<const uint8_t*>(y_scales);
  p.c = c;
  p.offsets = offsets;
  p.colsum = colsum;
  p.stride_c = (long long)M * N;
  p.lda = M;
  p.ldb = N;
  p.ldc = N;
  p.G = G;
  p.M = M;
  p.N = N;
  p.K = 0;
  const int ntn = N / 128;
  const int gpad = G >= 8 ? (G + 7) / 8 * 8 : G;
  // algorithmic bytes: fp32 C (+ colsum) once; per routed row one bf16 row of X (M) and one MXFP8 row of Y
  ProfScope prof(stream, PROF_GEMM, 4.0 * G * M * N + (colsum ? 4.0 * G * M : 0.0), true,
                 2.0 * M + N + N / 32.0, 2.0 * M * N);
  p.prof_rows = prof.rows_slot();
  dim3 grid((M / 64) * ntn * gpad);
  if (colsum) launch<64, 128, false, false, MODE_WGRAD, MOE_EPI_NONE, true, FL_Y8>(p, grid, stream, prof, 1, 2);
  else launch<64, 128, false, false, MODE_WGRAD, MOE_EPI_NONE, false, FL_Y8>(p, grid, stream, prof, 1, 2);
  return check_launch("moe_grouped_gemm_wgrad_mx");
}
