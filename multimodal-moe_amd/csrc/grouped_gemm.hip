// Grouped expert GEMMs on bf16 MFMA for gfx950.
//
// One kernel template covers the five expert contractions of the MoE FFN:
//   ROWS mode  (rows of group g = tokens routed to expert g, K/N fixed)
//     fwd   H  = relu(Xp . W1_g^T + b1_g)      A=[rows][K]  B=[N][K]  (trans_b=1)
//     fwd   Yp = H . W2_g^T + b2_g             A=[rows][K]  B=[N][K]  (trans_b=1)
//     dgrad dH = (dYp . W2_g) * (H > 0)        A=[rows][K]  B=[K][N]  (trans_b=0)
//     dgrad dXp = dH . W1_g                    A=[rows][K]  B=[K][N]  (trans_b=0)
//   WGRAD mode (K = rows of group g, M/N fixed)
//     dW2_g = dYp^T . H  (+ db2 = colsum dYp), dW1_g = dH^T . Xp (+ db1)
//
// Tiling: 256 threads = 4 waves in 2x2, block tile BM x BN (BM in {64,128},
// BN = 128), K-step 64, v_mfma_f32_16x16x32_bf16 with the operands swapped
// (D = B^T-frag x A-frag) so that each lane ends with 4 consecutive output
// columns of one row (8-B bf16 / 16-B fp32 stores).  Operands are staged
// global -> registers -> LDS (double-buffered, one barrier per K-step, next
// tile's global loads in flight under the current tile's MFMAs).
// Two LDS images:
//   K-contiguous  [R][64] bf16, 128-B rows, 16-B chunk c of row r stored at
//                 chunk c ^ ((r>>1)&7): conflict-free ds_read_b128 fragments;
//   MN-contiguous [64][R] bf16 (weights read for dgrad, activations for
//                 wgrad), fragments by ds_read_b64_tr_b16 (hardware
//                 transpose), chunk XOR swizzle chosen so that the two 16-lane
//                 blocks of each 32-lane half hit 16 distinct 16-B slots.
#include "moe_common.h"

namespace moe {

enum { MODE_ROWS = 0, MODE_WGRAD = 1 };

struct GemmParams {
  const uint16_t* a;
  const uint16_t* b;
  void* c;
  const int32_t* offsets;
  const float* bias;
  const uint16_t* aux;
  float* colsum;
  long long stride_b;  // elements between groups' B (ROWS mode)
  long long stride_c;  // elements between groups' C (WGRAD mode)
  int lda, ldb, ldc;
  int G, M, N, K;
};

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

// byte offset of 16-B chunk c of row r in a K-contiguous [R][64] image
__device__ __forceinline__ int kimg_off(int r, int c) {
  return r * 128 + ((c ^ ((r >> 1) & 7)) << 4);
}
// byte offset of 16-B chunk c of k-row r in an MN-contiguous [64][R] image
template <int R>
__device__ __forceinline__ int mimg_off(int r, int c) {
  if constexpr (R == 128) {
    const int f = ((r & 3) << 1) | (((r >> 3) & 1) << 3);
    return r * 256 + ((c ^ f) << 4);
  } else {
    const int f = (((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2);
    return r * 128 + ((c ^ f) << 4);
  }
}

// Operand loader for one K-step tile: R rows of the operand (m or n) x 64 k.
// KCONT: storage is [row][k] (row stride ld); else [k][row] (k stride ld).
template <int R, bool KCONT>
struct TileLoader {
  static constexpr int kChunks = R * 64 / 8;  // 16-B chunks per tile
  static constexpr int kPer = kChunks / 256;  // per thread
  uint4 reg[kPer];

  // base: pointer to element (row0, k0) of the operand (already group-offset);
  // row_lim / k_lim: valid extents (rows beyond -> zeros).
  __device__ __forceinline__ void load(const uint16_t* base, int ld, int row_lim, int k_lim,
                                       int tid) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int q = tid + 256 * i;
      int r, kk;
      if constexpr (KCONT) {
        r = q >> 3;
        kk = (q & 7) * 8;
      } else {
        constexpr int cpr = R / 8;  // chunks per k-row
        kk = q / cpr;
        r = (q % cpr) * 8;
      }
      const bool ok = KCONT ? (r < row_lim && kk < k_lim) : (kk < k_lim && r < row_lim);
      const uint16_t* p = KCONT ? base + (size_t)r * ld + kk : base + (size_t)kk * ld + r;
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

// Fragment (8 bf16 along k) for operand row `row` (0..R-1) at k-step ks.
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

template <int BM, int BN, bool A_K, bool B_K, int MODE, int EPI, bool COLSUM>
__global__ __launch_bounds__(256) void grouped_gemm_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int A_BYTES = BM * 64 * 2;
  constexpr int B_BYTES = BN * 64 * 2;
  constexpr int BUF = A_BYTES + B_BYTES;
  constexpr int TM = BM / 32;  // 16-row sub-tiles per wave
  constexpr int TN = BN / 32;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // ---- tile -> (group, m-tile, n-tile) ----
  int g, mt, nt, row0, rows_g;
  if constexpr (MODE == MODE_ROWS) {
    int rem = blockIdx.x;
    g = 0;
    for (; g < p.G; ++g) {
      const int n_g = p.offsets[g + 1] - p.offsets[g];
      const int t_g = (n_g + BM - 1) / BM;
      if (rem < t_g) break;
      rem -= t_g;
    }
    if (g >= p.G) return;  // beyond the last tile (grid is an upper bound)
    mt = rem;
    nt = blockIdx.y;
    row0 = p.offsets[g] + mt * BM;
    rows_g = p.offsets[g + 1] - row0;  // valid rows from row0
  } else {
    g = blockIdx.y;
    const int ntn = p.N / BN;
    mt = blockIdx.x / ntn;
    nt = blockIdx.x % ntn;
    row0 = p.offsets[g];
    rows_g = p.offsets[g + 1] - row0;  // K extent of this group
  }
  const int m0 = mt * BM, n0 = nt * BN;

  // ---- operand base pointers and limits ----
  // A logical [m][k]; B logical [k][n].
  const uint16_t* a_base;
  const uint16_t* b_base;
  int a_row_lim, nk;
  if constexpr (MODE == MODE_ROWS) {
    a_base = p.a + (size_t)row0 * p.lda;           // [rows][K]
    a_row_lim = rows_g < BM ? rows_g : BM;
    const uint16_t* bg = p.b + (size_t)g * p.stride_b;
    b_base = B_K ? bg + (size_t)n0 * p.ldb : bg + n0;  // [N][K] or [K][N]
    nk = p.K / 64;
  } else {
    a_base = p.a + (size_t)row0 * p.lda + m0;      // X [rows][M], k = row
    b_base = p.b + (size_t)row0 * p.ldb + n0;      // Y [rows][N]
    a_row_lim = BM;
    nk = (rows_g + 63) / 64;
  }

  TileLoader<BM, A_K> la;
  TileLoader<BN, B_K> lb;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float csum[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) csum[i] = 0.f;

  auto k_lim_of = [&](int kt) -> int {
    if constexpr (MODE == MODE_ROWS) return 64;
    else return rows_g - kt * 64;
  };
  auto a_ptr = [&](int kt) -> const uint16_t* {
    return A_K ? a_base + kt * 64 : a_base + (size_t)kt * 64 * p.lda;
  };
  auto b_ptr = [&](int kt) -> const uint16_t* {
    return B_K ? b_base + kt * 64 : b_base + (size_t)kt * 64 * p.ldb;
  };

  if (nk > 0) {
    la.load(a_ptr(0), p.lda, a_row_lim, k_lim_of(0), tid);
    lb.load(b_ptr(0), p.ldb, BN, k_lim_of(0), tid);
    la.store(smem, tid);
    lb.store(smem + A_BYTES, tid);
  }
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * BUF;
    const bool more = kt + 1 < nk;
    if (more) {
      la.load(a_ptr(kt + 1), p.lda, a_row_lim, k_lim_of(kt + 1), tid);
      lb.load(b_ptr(kt + 1), p.ldb, BN, k_lim_of(kt + 1), tid);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = read_frag<BM, A_K>(cur, wm * (BM / 2) + 16 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[j] = read_frag<BN, B_K>(cur + A_BYTES, wn * (BN / 2) + 16 * j, ks, lane);
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
    if (more) {
      char* nxt = smem + ((kt + 1) & 1) * BUF;
      la.store(nxt, tid);
      lb.store(nxt + A_BYTES, tid);
    }
    __syncthreads();
  }

  // ---- epilogue: lane holds C[m = .. + (lane&15)][n = .. + 4*(lane>>4) + r] ----
  const int lm = lane & 15;
  const int ln = 4 * (lane >> 4);
  if constexpr (MODE == MODE_ROWS) {
    uint16_t* C = static_cast<uint16_t*>(p.c);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int ml = wm * (BM / 2) + 16 * i + lm;
      if (ml >= a_row_lim) continue;
      const size_t row = (size_t)row0 + ml;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * (BN / 2) + 16 * j + ln;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if constexpr (EPI == MOE_EPI_BIAS || EPI == MOE_EPI_BIAS_RELU) {
          const float4 bv = *reinterpret_cast<const float4*>(p.bias + (size_t)g * p.N + n);
          v[0] += bv.x; v[1] += bv.y; v[2] += bv.z; v[3] += bv.w;
        }
        if constexpr (EPI == MOE_EPI_BIAS_RELU) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
        }
        if constexpr (EPI == MOE_EPI_RELU_MASK) {
          const uint2 hv = *reinterpret_cast<const uint2*>(p.aux + row * p.ldc + n);
          const uint16_t h[4] = {(uint16_t)(hv.x & 0xffff), (uint16_t)(hv.x >> 16),
                                 (uint16_t)(hv.y & 0xffff), (uint16_t)(hv.y >> 16)};
#pragma unroll
          for (int r = 0; r < 4; ++r)  // bf16 > 0: sign clear and not +0
            if ((h[r] & 0x8000u) || h[r] == 0) v[r] = 0.f;
        }
        uint2 o;
        o.x = pack2bf(v[0], v[1]);
        o.y = pack2bf(v[2], v[3]);
        *reinterpret_cast<uint2*>(C + row * p.ldc + n) = o;
      }
    }
  } else {
    float* C = static_cast<float*>(p.c) + (size_t)g * p.stride_c;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wm * (BM / 2) + 16 * i + lm;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * (BN / 2) + 16 * j + ln;
        *reinterpret_cast<float4*>(C + (size_t)m * p.ldc + n) =
            make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
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
          p.colsum[(size_t)g * p.M + m] = csum[i];
        }
      }
    }
  }
}

template <int BM, int BN, bool A_K, bool B_K, int MODE, int EPI, bool COLSUM>
static void launch(const GemmParams& p, dim3 grid, hipStream_t s) {
  constexpr int BUF = (BM + BN) * 64 * 2;
  hipLaunchKernelGGL((grouped_gemm_kernel<BM, BN, A_K, B_K, MODE, EPI, COLSUM>), grid,
                     dim3(256), 2 * BUF, s, p);
}

}  // namespace moe

using namespace moe;

extern "C" int moe_grouped_gemm(int dtype, const void* a, const void* b, void* c,
                                const int32_t* offsets, int G, int max_rows, int N, int K,
                                int trans_b, int epilogue, const float* bias, const void* aux,
                                const float* scales, hipStream_t stream) {
  (void)scales;
  if (dtype != MOE_BF16) return fail("grouped_gemm: only MOE_BF16 is implemented");
  if (G < 1 || G > 1024) return fail("grouped_gemm: G out of range");
  if (N <= 0 || K <= 0 || N % 128 != 0 || K % 64 != 0)
    return fail("grouped_gemm: need N % 128 == 0 and K % 64 == 0");
  if (max_rows < 0) return fail("grouped_gemm: max_rows < 0");
  if ((epilogue == MOE_EPI_BIAS || epilogue == MOE_EPI_BIAS_RELU) && bias == nullptr)
    return fail("grouped_gemm: bias epilogue without bias");
  if (epilogue == MOE_EPI_RELU_MASK && aux == nullptr)
    return fail("grouped_gemm: relu-mask epilogue without aux");
  if (epilogue < 0 || epilogue > 3) return fail("grouped_gemm: bad epilogue");
  if (max_rows == 0) return 0;

  GemmParams p{};
  p.a = static_cast<const uint16_t*>(a);
  p.b = static_cast<const uint16_t*>(b);
  p.c = c;
  p.offsets = offsets;
  p.bias = bias;
  p.aux = static_cast<const uint16_t*>(aux);
  p.colsum = nullptr;
  p.stride_b = (long long)N * K;
  p.stride_c = 0;
  p.lda = K;
  p.ldb = trans_b ? K : N;
  p.ldc = N;
  p.G = G;
  p.M = 0;
  p.N = N;
  p.K = K;

  // Pick the row tile so the launch has >= ~2 waves of workgroups per chip.
  const int nt = N / 128;
  const int tiles128 = (max_rows + 127) / 128 + G;
  const bool big = (long long)tiles128 * nt >= 512;
  const int BMsel = big ? 128 : 64;
  const int mtiles = (max_rows + BMsel - 1) / BMsel + G;
  dim3 grid(mtiles, nt);

#define GG_ROWS(BM, BK_, EPI) launch<BM, 128, true, BK_, MODE_ROWS, EPI, false>(p, grid, stream)
#define GG_EPI(BM, BK_)                                             \
  switch (epilogue) {                                              \
    case MOE_EPI_NONE: GG_ROWS(BM, BK_, MOE_EPI_NONE); break;       \
    case MOE_EPI_BIAS: GG_ROWS(BM, BK_, MOE_EPI_BIAS); break;       \
    case MOE_EPI_BIAS_RELU: GG_ROWS(BM, BK_, MOE_EPI_BIAS_RELU); break; \
    default: GG_ROWS(BM, BK_, MOE_EPI_RELU_MASK); break;            \
  }
  if (BMsel == 128) {
    if (trans_b) { GG_EPI(128, true) } else { GG_EPI(128, false) }
  } else {
    if (trans_b) { GG_EPI(64, true) } else { GG_EPI(64, false) }
  }
#undef GG_EPI
#undef GG_ROWS
  return check_launch("moe_grouped_gemm");
}

extern "C" int moe_grouped_gemm_wgrad(int dtype, const void* x, const void* y, float* c,
                                      float* colsum, const int32_t* offsets, int G, int M,
                                      int N, hipStream_t stream) {
  if (dtype != MOE_BF16) return fail("grouped_gemm_wgrad: only MOE_BF16 is implemented");
  if (G < 1 || G > 1024) return fail("grouped_gemm_wgrad: G out of range");
  if (M <= 0 || N <= 0 || M % 64 != 0 || N % 128 != 0)
    return fail("grouped_gemm_wgrad: need M % 64 == 0 and N % 128 == 0");
  GemmParams p{};
  p.a = static_cast<const uint16_t*>(x);
  p.b = static_cast<const uint16_t*>(y);
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
  const bool big = M % 128 == 0 && (long long)(M / 128) * ntn * G >= 512;
  if (big) {
    dim3 grid((M / 128) * ntn, G);
    if (colsum) launch<128, 128, false, false, MODE_WGRAD, MOE_EPI_NONE, true>(p, grid, stream);
    else launch<128, 128, false, false, MODE_WGRAD, MOE_EPI_NONE, false>(p, grid, stream);
  } else {
    dim3 grid((M / 64) * ntn, G);
    if (colsum) launch<64, 128, false, false, MODE_WGRAD, MOE_EPI_NONE, true>(p, grid, stream);
    else launch<64, 128, false, false, MODE_WGRAD, MOE_EPI_NONE, false>(p, grid, stream);
  }
  return check_launch("moe_grouped_gemm_wgrad");
}
