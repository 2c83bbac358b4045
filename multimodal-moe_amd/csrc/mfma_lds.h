// bf16 MFMA tile helpers shared by the grouped expert GEMMs (grouped_gemm.hip)
// and the implicit-GEMM convolutions (conv.hip), gfx950.
//
// Two LDS images of a 64-deep K-tile of an operand with R rows:
//   K-contiguous  [R][64] bf16, 128-B rows, 16-B chunk c of row r stored at
//                 chunk c ^ ((r>>1)&7): conflict-free ds_read_b128 fragments;
//   MN-contiguous [64][R] bf16 (k-rows of R contiguous elements), fragments by
//                 ds_read_b64_tr_b16 (hardware transpose), XOR swizzle so the two
//                 16-lane blocks of each 32-lane half hit 16 distinct 16-B slots.
// Fragments feed v_mfma_f32_16x16x32_bf16 with the operands swapped
// (D = B^T-frag x A-frag) so that each lane ends with 4 consecutive output
// columns of one row.
#pragma once

#include "moe_common.h"

namespace moe {

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

// byte offset of 16-B chunk c of row r in a K-contiguous [R][64] image
__device__ __forceinline__ int kimg_off(int r, int c) {
  return r * 128 + ((c ^ ((r >> 1) & 7)) << 4);
}
// chunk swizzle of an MN-contiguous [64][R] image (R = 128 or 64 bf16 per k-row)
template <int R>
__device__ __forceinline__ int mimg_swz(int r) {
  if constexpr (R == 128) return ((r & 3) << 1) | (((r >> 3) & 1) << 3);
  else return (((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2);
}
template <int R>
__device__ __forceinline__ int mimg_off(int r, int c) {
  return r * (R * 2) + ((c ^ mimg_swz<R>(r)) << 4);
}

// Fragment (8 bf16 along k) for operand row block `row_base` (16 rows) at k-step ks.
template <int R, bool KCONT>
__device__ __forceinline__ bf16x8 read_frag(const char* lds, int row_base, int ks, int lane) {
  if constexpr (KCONT) {
    const int r = row_base + (lane & 15);
    const int c = ks * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(lds + kimg_off(r, c));
  } else {
    const int i = lane & 15;
    const int q = i >> 2, p = i & 3;
    const int kr = ks * 32 + 8 * (lane >> 4) + q;
    const int col = row_base + 4 * p;
    const int c = col >> 3;
    const int half = (col & 7) * 2;  // 0 or 8 bytes
    char* base = const_cast<char*>(lds);
    lds_bf16x4* p0 = (lds_bf16x4*)(base + mimg_off<R>(kr, c) + half);
    lds_bf16x4* p1 = (lds_bf16x4*)(base + mimg_off<R>(kr + 4, c) + half);
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(p0);
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(p1);
    bf16x8 v;
    v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
    v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
    return v;
  }
}

__device__ __forceinline__ float sum8(bf16x8 v) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += bf2f((uint16_t)v[i]);
  return s;
}

// MFMA work on one staged K-tile (2 k-steps of 32).
template <int BM, int BN, bool A_K, bool B_K, bool COLSUM>
__device__ __forceinline__ void compute_tile(const char* abuf, const char* bbuf,
                                             f32x4 (&acc)[BM / 32][BN / 32], float (&csum)[BM / 32],
                                             int lane, int wm, int wn) {
  constexpr int TM = BM / 32, TN = BN / 32;
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    bf16x8 af[TM], bfr[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = read_frag<BM, A_K>(abuf, wm * (BM / 2) + 16 * i, ks, lane);
#pragma unroll
    for (int j = 0; j < TN; ++j) bfr[j] = read_frag<BN, B_K>(bbuf, wn * (BN / 2) + 16 * j, ks, lane);
    if constexpr (COLSUM) {
#pragma unroll
      for (int i = 0; i < TM; ++i) csum[i] += sum8(af[i]);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
  }
}

// The same for WGM x WGN waves: wave (wm, wn) owns rows wm BM/WGM + 16 i and
// columns wn BN/WGN + 16 j of the tile (compute_tile is the 2 x 2 case).
template <int BM, int BN, int WGM, int WGN, bool A_K, bool B_K>
__device__ __forceinline__ void compute_tile_w(const char* abuf, const char* bbuf,
                                               f32x4 (&acc)[BM / (16 * WGM)][BN / (16 * WGN)], int lane, int wm,
                                               int wn) {
  constexpr int TM = BM / (16 * WGM), TN = BN / (16 * WGN);
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    bf16x8 af[TM], bfr[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = read_frag<BM, A_K>(abuf, wm * (BM / WGM) + 16 * i, ks, lane);
#pragma unroll
    for (int j = 0; j < TN; ++j) bfr[j] = read_frag<BN, B_K>(bbuf, wn * (BN / WGN) + 16 * j, ks, lane);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
  }
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}


}  // namespace moe
