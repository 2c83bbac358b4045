// Narrow dense linears of the RT-DETR heads (the dense body
// around the MoE path): the score heads (256 -> 1 over the 2,400 queries, and
// over all 154,560 memory tokens for the query ranking), the box heads' last
// layers (256 -> 4) and the query-position head's first layer (4 -> 512,
// ReLU).  hipBLASLt runs these as 1-8-column GEMMs on a few workgroups
// (5-8 us each in the graphed C2 step, 31 us for the ranking head) plus a
// separate ReLU / ReLU-backward launch; here each is one HBM-streaming pass:
//   narrow_out  : y[m, :N] = act(x[m, :] W^T + b), N <= 8 -- a row's K/8
//                 16-B chunks over LPR lanes, an xor butterfly per output
//   smallk      : y[m, n] = act(sum_{k < K} x[m, k] W[n, k] + b[n]), K <= 8
//                 -- 8 consecutive outputs per thread
//   narrow_dgrad: gx[m, k] = (sum_{n < N} g[m, n] W[n, k]) * [mask[m, k] > 0],
//                 N <= 8 -- the data gradient through a narrow layer with the
//                 previous layer's ReLU mask applied in the same pass
// fp32 accumulation, the bias added in fp32, one rounding to bf16 (as the
// library GEMM's bias epilogue); the sum order is fixed (deterministic).
#include <algorithm>

#include "moe_common.h"
#include "prof.h"

namespace moe {

__device__ __forceinline__ float bias_at(const void* b, int b_bf16, int n) {
  if (b == nullptr) return 0.f;
  return b_bf16 ? bf2f(static_cast<const uint16_t*>(b)[n]) : static_cast<const float*>(b)[n];
}

template <int NO>
__global__ __launch_bounds__(256) void linear_narrow_out_kernel(const uint16_t* __restrict__ x,
                                                                const uint16_t* __restrict__ w, const void* b,
                                                                int b_bf16, uint16_t* __restrict__ y, long long M,
                                                                int K, int N, int lpr_log2, int relu) {
  const int lpr = 1 << lpr_log2;
  const int tid = threadIdx.x, sub = tid & (lpr - 1);
  const long long r = (long long)blockIdx.x * (256 >> lpr_log2) + (tid >> lpr_log2);
  const int nch = K >> 3;
  float acc[NO];
#pragma unroll
  for (int n = 0; n < NO; ++n) acc[n] = 0.f;
  if (r < M) {
    const uint4* xr = reinterpret_cast<const uint4*>(x + r * K);
    for (int c = sub; c < nch; c += lpr) {
      float xv[8];
      unpack8(xr[c], xv);
#pragma unroll
      for (int n = 0; n < NO; ++n) {
        if (n < N) {
          float wv[8];
          unpack8(reinterpret_cast<const uint4*>(w + (size_t)n * K)[c], wv);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[n] = fmaf(xv[j], wv[j], acc[n]);
        }
      }
    }
  }
  // lanes of one row are an aligned power-of-two group of one wave
  for (int off = lpr >> 1; off > 0; off >>= 1)
#pragma unroll
    for (int n = 0; n < NO; ++n) acc[n] += __shfl_xor(acc[n], off);
  // after the butterfly every lane of the group holds all N sums: lane sub
  // writes the columns n with n % lpr == sub (all of them when lpr < N)
  if (r < M) {
#pragma unroll
    for (int n = 0; n < NO; ++n) {
      if (n < N && (n & (lpr - 1)) == sub) {
        float v = acc[n] + bias_at(b, b_bf16, n);
        if (relu) v = fmaxf(v, 0.f);
        y[r * N + n] = f2bf(v);
      }
    }
  }
}

// A thread keeps one 8-output chunk (its 8 K weights and biases in registers,
// loaded once) and walks the rows with a stride of the rows in flight: the
// per-row work is one x row load and one 16-B store (loading the weights per
// output per row made this 15 us for the 2,400 x 4 -> 512 layer).
__global__ __launch_bounds__(256) void linear_smallk_kernel(const uint16_t* __restrict__ x,
                                                            const uint16_t* __restrict__ w, const void* b, int b_bf16,
                                                            uint16_t* __restrict__ y, long long M, int K, int N,
                                                            int relu) {
  const int nc = N >> 3;
  const long long lanes = (long long)gridDim.x * 256;
  const long long rows_in_flight = lanes / nc;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows_in_flight * nc) return;
  const int n0 = (int)(i % nc) * 8;
  float wr[8][8], bs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    bs[j] = bias_at(b, b_bf16, n0 + j);
#pragma unroll
    for (int k = 0; k < 8; ++k) wr[j][k] = k < K ? bf2f(w[(size_t)(n0 + j) * K + k]) : 0.f;
  }
  for (long long r = i / nc; r < M; r += rows_in_flight) {
    float xv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) xv[k] = k < K ? bf2f(x[r * K + k]) : 0.f;
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (k < K) s = fmaf(xv[k], wr[j][k], s);
      s += bs[j];
      o[j] = relu ? fmaxf(s, 0.f) : s;
    }
    reinterpret_cast<uint4*>(y + r * N)[n0 >> 3] = pack8(o);
  }
}

template <int NO>
__global__ __launch_bounds__(256) void linear_narrow_dgrad_kernel(const uint16_t* __restrict__ g,
                                                                  const uint16_t* __restrict__ w,
                                                                  const uint16_t* __restrict__ mask,
                                                                  uint16_t* __restrict__ gx, long long M, int K,
                                                                  int N) {
  const int kc = K >> 3;
  const long long total = M * kc;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const long long r = i / kc;
    const int c = (int)(i - r * kc);
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = 0.f;
#pragma unroll
    for (int n = 0; n < NO; ++n) {
      if (n < N) {
        const float gv = bf2f(g[r * N + n]);
        float wv[8];
        unpack8(reinterpret_cast<const uint4*>(w + (size_t)n * K)[c], wv);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = fmaf(gv, wv[j], o[j]);
      }
    }
    uint4 v = pack8(o);
    if (mask != nullptr) {  // keep where the mask element is > 0 (bf16: sign clear, not zero)
      const uint4 em = reinterpret_cast<const uint4*>(mask + r * K)[c];
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
    reinterpret_cast<uint4*>(gx + r * K)[c] = v;
  }
}

static int ew_grid(long long items) {
  const long long g = (items + 255) / 256;
  return (int)(g > 16384 ? 16384 : (g < 1 ? 1 : g));
}

static bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace moe

using namespace moe;

extern "C" int rtdetr_linear_narrow_supported(int K, int N) {
  return ((N >= 1 && N <= 8 && K >= 8 && K % 8 == 0) || (K >= 1 && K <= 8 && N >= 8 && N % 8 == 0)) ? 1 : 0;
}

extern "C" int rtdetr_linear_narrow_fwd(const void* x, const void* w, const void* b, int b_bf16, void* y, long long M,
                                        int K, int N, int relu, hipStream_t stream) {
  if (M < 0) return fail("rtdetr_linear_narrow_fwd: M < 0");
  if (!rtdetr_linear_narrow_supported(K, N))
    return fail("rtdetr_linear_narrow_fwd: needs N <= 8 with K % 8 == 0, or K <= 8 with N % 8 == 0");
  if (M == 0) return 0;  // (empty tensors may carry NULL pointers)
  if (x == nullptr || w == nullptr || y == nullptr) return fail("rtdetr_linear_narrow_fwd: null pointer");
  const uint16_t* x16 = static_cast<const uint16_t*>(x);
  const uint16_t* w16 = static_cast<const uint16_t*>(w);
  uint16_t* y16 = static_cast<uint16_t*>(y);
  ProfScope prof(stream, PROF_LINEAR, 2.0 * M * (K + N) + 2.0 * K * N, false, 0.0, 2.0 * M * K * N);
  if (N <= 8 && K % 8 == 0) {
    if (!al16(x) || !al16(w)) return fail("rtdetr_linear_narrow_fwd: x and w must be 16-B aligned");
    int lg = 0;
    while ((1 << (lg + 1)) <= K / 8 && lg < 6) ++lg;  // lanes per row: largest power of two <= K / 8, <= 64
    const long long rows_per_block = 256 >> lg;
    const int grid = (int)((M + rows_per_block - 1) / rows_per_block);
    if (N == 1)
      MOE_LAUNCH(prof, linear_narrow_out_kernel<1>, dim3(grid), dim3(256), 0, stream, x16, w16, b, b_bf16, y16, M, K,
                 N, lg, relu);
    else if (N <= 4)
      MOE_LAUNCH(prof, linear_narrow_out_kernel<4>, dim3(grid), dim3(256), 0, stream, x16, w16, b, b_bf16, y16, M, K,
                 N, lg, relu);
    else
      MOE_LAUNCH(prof, linear_narrow_out_kernel<8>, dim3(grid), dim3(256), 0, stream, x16, w16, b, b_bf16, y16, M, K,
                 N, lg, relu);
  } else {
    if (!al16(y)) return fail("rtdetr_linear_narrow_fwd: y must be 16-B aligned");
    // ~8 rows per thread (at least one chunk of rows per 256 threads), <= 2,048 workgroups
    const long long want = (M * (N / 8) + 8 * 256 - 1) / (8 * 256);
    const int grid = (int)std::max(1LL, std::min(2048LL, std::max(want, (long long)(N / 8 + 255) / 256)));
    MOE_LAUNCH(prof, linear_smallk_kernel, dim3(grid), dim3(256), 0, stream, x16, w16, b, b_bf16, y16, M, K, N, relu);
  }
  return check_launch("rtdetr_linear_narrow_fwd");
}

extern "C" int rtdetr_linear_narrow_dgrad(const void* g, const void* w, const void* mask, void* gx, long long M, int K,
                                          int N, hipStream_t stream) {
  if (M < 0 || N < 1 || N > 8 || K < 8 || K % 8 != 0)
    return fail("rtdetr_linear_narrow_dgrad: needs M >= 0, 1 <= N <= 8 and K % 8 == 0");
  if (M == 0) return 0;
  if (g == nullptr || w == nullptr || gx == nullptr) return fail("rtdetr_linear_narrow_dgrad: null pointer");
  if (!al16(w) || !al16(gx) || (mask != nullptr && !al16(mask)))
    return fail("rtdetr_linear_narrow_dgrad: w, gx and mask must be 16-B aligned");
  ProfScope prof(stream, PROF_LINEAR, 2.0 * M * (N + K * (mask ? 2 : 1)) + 2.0 * K * N, false, 0.0, 2.0 * M * K * N);
  const uint16_t* g16 = static_cast<const uint16_t*>(g);
  const uint16_t* w16 = static_cast<const uint16_t*>(w);
  const uint16_t* m16 = static_cast<const uint16_t*>(mask);
  uint16_t* o16 = static_cast<uint16_t*>(gx);
  const int grid = ew_grid(M * (K / 8));
  if (N == 1)
    MOE_LAUNCH(prof, linear_narrow_dgrad_kernel<1>, dim3(grid), dim3(256), 0, stream, g16, w16, m16, o16, M, K, N);
  else if (N <= 4)
    MOE_LAUNCH(prof, linear_narrow_dgrad_kernel<4>, dim3(grid), dim3(256), 0, stream, g16, w16, m16, o16, M, K, N);
  else
    MOE_LAUNCH(prof, linear_narrow_dgrad_kernel<8>, dim3(grid), dim3(256), 0, stream, g16, w16, m16, o16, M, K, N);
  return check_launch("rtdetr_linear_narrow_dgrad");
}
