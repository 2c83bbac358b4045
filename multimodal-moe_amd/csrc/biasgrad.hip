// Bias gradient of the RT-DETR body's linear layers:
//   db[n] = sum_m dy[m, n]      dy bf16 [M, N] row-major, fp32 accumulation
// Deterministic two-launch reduction, no atomics:
//   bias_grad_part : block p sums rows [p*rpb, (p+1)*rpb) -> partials[p][N]
//                    (16-B row vectors when N % 8 == 0, one column per lane
//                    otherwise; RL row lanes per block, reduced in LDS in a
//                    fixed order)
//   bias_grad_final: 8 partial lanes x 32 columns per block, fixed order,
//                    written as fp32 or bf16 (the bias dtype)
// Replaces torch's column sum (a 64-block reduce_kernel per layer, 61 per
// training step at C2, and ~45 us for the 154,560-row value projection).
#include "moe_common.h"
#include "prof.h"

namespace moe {

template <int VEC>
__global__ __launch_bounds__(256) void bias_grad_part_kernel(const uint16_t* __restrict__ dy, long long M, int N,
                                                             long long rpb, float* __restrict__ partials) {
  __shared__ float s_acc[256 * VEC];
  const int tid = threadIdx.x;
  const int NV = N / VEC;        // vectors per row
  const int RL = 256 / NV;       // row lanes
  const int rl = tid / NV;
  const int cv = tid - rl * NV;
  const long long r0 = (long long)blockIdx.x * rpb;
  const long long r1 = min(M, r0 + rpb);
  float acc[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) acc[i] = 0.f;
  if (rl < RL) {
    constexpr int U = 4;  // loads in flight per thread
    for (long long r = r0 + rl; r < r1; r += (long long)U * RL) {
      if constexpr (VEC == 8) {
        uint4 raw[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long long rr = r + (long long)u * RL;
          raw[u] = rr < r1 ? reinterpret_cast<const uint4*>(dy + rr * N)[cv] : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          float v[8];
          unpack8(raw[u], v);
#pragma unroll
          for (int i = 0; i < 8; ++i) acc[i] += v[i];
        }
      } else {
        uint16_t raw[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long long rr = r + (long long)u * RL;
          raw[u] = rr < r1 ? dy[rr * N + cv] : (uint16_t)0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc[0] += bf2f(raw[u]);
      }
    }
#pragma unroll
    for (int i = 0; i < VEC; ++i) s_acc[rl * N + cv * VEC + i] = acc[i];
  }
  __syncthreads();
  for (int c = tid; c < N; c += 256) {
    float s = 0.f;
    for (int l = 0; l < RL; ++l) s += s_acc[l * N + c];
    partials[(size_t)blockIdx.x * N + c] = s;
  }
}

__global__ __launch_bounds__(256) void bias_grad_final_kernel(const float* __restrict__ partials, int P, int N,
                                                              void* __restrict__ out, int out_bf16) {
  __shared__ float s_acc[8][32];
  const int cl = threadIdx.x & 31;
  const int pl = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  float s = 0.f;
  if (c < N) {
    constexpr int U = 8;
    for (int p = pl; p < P; p += 8 * U) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = (p + 8 * u < P) ? partials[(size_t)(p + 8 * u) * N + c] : 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u) s += v[u];
    }
  }
  s_acc[pl][cl] = s;
  __syncthreads();
  if (pl == 0 && c < N) {
    float t = 0.f;
#pragma unroll
    for (int l = 0; l < 8; ++l) t += s_acc[l][cl];
    if (out_bf16) static_cast<uint16_t*>(out)[c] = f2bf(t);
    else static_cast<float*>(out)[c] = t;
  }
}

}  // namespace moe

using namespace moe;

extern "C" int rtdetr_bias_grad_parts(long long M, int N) {
  if (M <= 0 || N <= 0) return 1;
  // ~128 rows per block at small M, at most 256 blocks (one per CU) at large M
  long long p = (M + 127) / 128;
  return (int)(p > 256 ? 256 : p);
}

extern "C" int rtdetr_bias_grad(const void* dy, long long M, int N, float* partials, int P, void* out, int out_bf16,
                                hipStream_t stream) {
  if (M < 0 || N <= 0 || P < 1 || dy == nullptr || partials == nullptr || out == nullptr)
    return fail("bias_grad: bad arguments");
  const bool vec = (N % 8 == 0) && N / 8 <= 256 && (reinterpret_cast<uintptr_t>(dy) & 15) == 0;
  if (!vec && N > 256) return fail("bias_grad: N must be a multiple of 8 (<= 2048) or <= 256");
  const long long rpb = M > 0 ? (M + P - 1) / P : 1;
  ProfScope prof(stream, PROF_CONV_EPI, 2.0 * M * N + 8.0 * P * N + (out_bf16 ? 2.0 : 4.0) * N);
  if (vec)
    MOE_LAUNCH(prof, bias_grad_part_kernel<8>, dim3(P), dim3(256), 0, stream, static_cast<const uint16_t*>(dy), M, N,
               rpb, partials);
  else
    MOE_LAUNCH(prof, bias_grad_part_kernel<1>, dim3(P), dim3(256), 0, stream, static_cast<const uint16_t*>(dy), M, N,
               rpb, partials);
  int rc = check_launch("rtdetr_bias_grad(part)");
  if (rc != 0) return rc;
  hipLaunchKernelGGL(bias_grad_final_kernel, dim3((N + 31) / 32), dim3(256), 0, stream, partials, P, N, out, out_bf16);
  return check_launch("rtdetr_bias_grad(final)");
}
