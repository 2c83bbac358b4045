// Residual add + LayerNorm of the RT-DETR body's post-norm sites (SURVEY.md
// 8(a) row a8: every AIFI / decoder layer computes norm(x + sublayer(x)),
// including norm(x + MoEFFN(x)); 8(f).1 body):
//   out[t] = (s[t] - mean_t) * rstd_t * gamma + beta,   s = a + b (b optional)
// bf16 rows of d = 128 / 256 / 512 columns, fp32 statistics (biased variance,
// two-pass in registers), one bf16 rounding of the output.
//   add_ln_fwd   : 16 lanes per row (16-B chunks), 16 rows per 256-thread
//                  pass, grid-stride; gamma / beta of the lane's columns held
//                  in registers; mean / rstd saved (fp32 [T]) for the backward
//   add_ln_bwd   : per row: xh = (s - mean) rstd, g = dout gamma,
//                  ds = rstd (g - mean(g) - xh mean(g xh)) -> bf16 (the
//                  gradient of a and of b); per block fixed-order partials of
//                  dgamma = sum dout xh and dbeta = sum dout
//   add_ln_final : fixed-order sum of the block partials -> [dgamma; dbeta]
//                  in the parameter dtype
// Deterministic (no atomics).  Replaces the residual add + torch's
// native_layer_norm (fwd) and native_layer_norm_backward (two kernels) at
// every post-norm site: ~14 us + ~21 us per site and step at C2.
#include "moe_common.h"
#include "prof.h"

namespace moe {

template <bool WBF16>
__device__ __forceinline__ void load_w8(const void* w, int col, float* f) {
  if constexpr (WBF16) {
    unpack8(*reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(w) + col), f);
  } else {
    const float4* p = reinterpret_cast<const float4*>(static_cast<const float*>(w) + col);
    const float4 u = p[0], v = p[1];
    f[0] = u.x; f[1] = u.y; f[2] = u.z; f[3] = u.w;
    f[4] = v.x; f[5] = v.y; f[6] = v.z; f[7] = v.w;
  }
}

// s = a (+ b) of this lane's NC chunks of row t (fp32)
template <int NC>
__device__ __forceinline__ void load_sum(const uint16_t* __restrict__ a, const uint16_t* __restrict__ b, int t,
                                         int d, int sub, float (&v)[NC][8]) {
  uint4 ra[NC], rb[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) ra[c] = reinterpret_cast<const uint4*>(a + (size_t)t * d)[sub + 16 * c];
  if (b != nullptr) {
#pragma unroll
    for (int c = 0; c < NC; ++c) rb[c] = reinterpret_cast<const uint4*>(b + (size_t)t * d)[sub + 16 * c];
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    unpack8(ra[c], v[c]);
    if (b != nullptr) {
      float w[8];
      unpack8(rb[c], w);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[c][i] += w[i];
    }
  }
}

template <int NC, bool WBF16>
__global__ __launch_bounds__(256) void add_ln_fwd_kernel(const uint16_t* __restrict__ a,
                                                         const uint16_t* __restrict__ b, const void* gamma,
                                                         const void* beta, int T, float eps,
                                                         uint16_t* __restrict__ out, float* __restrict__ mean_out,
                                                         float* __restrict__ rstd_out,
                                                         const uint16_t* __restrict__ pos = nullptr,
                                                         uint16_t* __restrict__ out2 = nullptr) {
  constexpr int d = NC * 128;
  const int tid = threadIdx.x, sub = tid & 15;
  float gm[NC][8], bt[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    load_w8<WBF16>(gamma, (sub + 16 * c) * 8, gm[c]);
    load_w8<WBF16>(beta, (sub + 16 * c) * 8, bt[c]);
  }
  for (int t = blockIdx.x * 16 + (tid >> 4); t < T; t += gridDim.x * 16) {
    float v[NC][8];
    load_sum<NC>(a, b, t, d, sub, v);
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[c][i];
    const float mean = row16_sum(s) * (1.0f / d);
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float e = v[c][i] - mean;
        q += e * e;
      }
    const float rstd = rsqrtf(row16_sum(q) * (1.0f / d) + eps);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (v[c][i] - mean) * rstd * gm[c][i] + bt[c][i];
      const uint4 ob = pack8(o);
      reinterpret_cast<uint4*>(out + (size_t)t * d)[sub + 16 * c] = ob;
      if (out2 != nullptr) {  // out2 = out + pos, the bf16 add of the rounded output (torch's `out + pos`)
        float f[8], q2[8];
        unpack8(ob, f);
        unpack8(reinterpret_cast<const uint4*>(pos + (size_t)t * d)[sub + 16 * c], q2);
#pragma unroll
        for (int i = 0; i < 8; ++i) f[i] += q2[i];
        reinterpret_cast<uint4*>(out2 + (size_t)t * d)[sub + 16 * c] = pack8(f);
      }
    }
    if (sub == 0) {
      mean_out[t] = mean;
      rstd_out[t] = rstd;
    }
  }
}

template <int NC, bool WBF16>
__global__ __launch_bounds__(256) void add_ln_bwd_kernel(const uint16_t* __restrict__ dout,
                                                         const uint16_t* __restrict__ a,
                                                         const uint16_t* __restrict__ b, const void* gamma,
                                                         const float* __restrict__ mean_in,
                                                         const float* __restrict__ rstd_in, int T,
                                                         uint16_t* __restrict__ ds, float* __restrict__ partials,
                                                         const uint16_t* __restrict__ dout2 = nullptr) {
  constexpr int d = NC * 128;
  __shared__ float s_red[16][2 * d];
  const int tid = threadIdx.x, sub = tid & 15, rg = tid >> 4;
  float gm[NC][8], adg[NC][8], adb[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    load_w8<WBF16>(gamma, (sub + 16 * c) * 8, gm[c]);
#pragma unroll
    for (int i = 0; i < 8; ++i) adg[c][i] = adb[c][i] = 0.f;
  }
  for (int t = blockIdx.x * 16 + rg; t < T; t += gridDim.x * 16) {
    float v[NC][8], go[NC][8];
    uint4 rd[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) rd[c] = reinterpret_cast<const uint4*>(dout + (size_t)t * d)[sub + 16 * c];
    if (dout2 != nullptr) {  // the output's second consumer (out + pos): its gradient summed in bf16 as autograd would
      uint4 r2[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) r2[c] = reinterpret_cast<const uint4*>(dout2 + (size_t)t * d)[sub + 16 * c];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        float f[8], g2[8];
        unpack8(rd[c], f);
        unpack8(r2[c], g2);
#pragma unroll
        for (int i = 0; i < 8; ++i) f[i] += g2[i];
        rd[c] = pack8(f);
      }
    }
    load_sum<NC>(a, b, t, d, sub, v);
    const float mean = mean_in[t], rstd = rstd_in[t];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      unpack8(rd[c], go[c]);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float xh = (v[c][i] - mean) * rstd;
        v[c][i] = xh;
        const float g = go[c][i] * gm[c][i];
        s1 += g;
        s2 += g * xh;
        adg[c][i] += go[c][i] * xh;
        adb[c][i] += go[c][i];
      }
    }
    const float m1 = row16_sum(s1) * (1.0f / d), m2 = row16_sum(s2) * (1.0f / d);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = rstd * (go[c][i] * gm[c][i] - m1 - v[c][i] * m2);
      reinterpret_cast<uint4*>(ds + (size_t)t * d)[sub + 16 * c] = pack8(o);
    }
  }
  // block partials of dgamma / dbeta: the 16 row groups summed in a fixed order
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int col = (sub + 16 * c) * 8 + i;
      s_red[rg][col] = adg[c][i];
      s_red[rg][d + col] = adb[c][i];
    }
  __syncthreads();
  for (int col = tid; col < 2 * d; col += 256) {
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) s += s_red[r][col];
    partials[(size_t)blockIdx.x * 2 * d + col] = s;
  }
}

// out[n] = sum_p partials[p][n] (fixed order), n < N; fp32 or bf16 out.
// 16 columns x 16 partial lanes per block; each lane issues all its loads
// (P <= 256: at most 16) before summing -- one memory round trip, not P / 8
__global__ __launch_bounds__(256) void add_ln_final_kernel(const float* __restrict__ partials, int P, int N,
                                                           void* __restrict__ out, int out_bf16) {
  __shared__ float s_acc[16][17];
  const int cl = threadIdx.x & 15, pl = threadIdx.x >> 4;
  const int n = blockIdx.x * 16 + cl;
  float v[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int p = pl + 16 * u;
    v[u] = (n < N && p < P) ? partials[(size_t)p * N + n] : 0.f;
  }
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < 16; ++u) s += v[u];
  s_acc[pl][cl] = s;
  __syncthreads();
  if (pl == 0 && n < N) {
    float t = 0.f;
#pragma unroll
    for (int l = 0; l < 16; ++l) t += s_acc[l][cl];
    if (out_bf16) static_cast<uint16_t*>(out)[n] = f2bf(t);
    else static_cast<float*>(out)[n] = t;
  }
}

// Batched finals (linear.DeferredWgrad after the backward): problem q sums its
// P[q] partial rows of N[q] columns into out[q]; blocks [base[q], base[q+1]).
constexpr int kLnFinMax = 48;
struct LnFinalBatch {
  const float* part[kLnFinMax];
  void* out[kLnFinMax];
  int P[kLnFinMax], N[kLnFinMax], bf16[kLnFinMax], base[kLnFinMax + 1];
  int n;
};

__global__ __launch_bounds__(256) void add_ln_final_batch_kernel(LnFinalBatch b) {
  __shared__ float s_acc[16][17];
  int q = 0;
  while (q + 1 < b.n && (int)blockIdx.x >= b.base[q + 1]) ++q;
  const int cl = threadIdx.x & 15, pl = threadIdx.x >> 4;
  const int n = (blockIdx.x - b.base[q]) * 16 + cl;
  const int P = b.P[q], N = b.N[q];
  const float* partials = b.part[q];
  float v[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int p = pl + 16 * u;
    v[u] = (n < N && p < P) ? partials[(size_t)p * N + n] : 0.f;
  }
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < 16; ++u) s += v[u];
  s_acc[pl][cl] = s;
  __syncthreads();
  if (pl == 0 && n < N) {
    float t = 0.f;
#pragma unroll
    for (int l = 0; l < 16; ++l) t += s_acc[l][cl];
    if (b.bf16[q]) static_cast<uint16_t*>(b.out[q])[n] = f2bf(t);
    else static_cast<float*>(b.out[q])[n] = t;
  }
}

}  // namespace moe

using namespace moe;

// every operand read or written with 16-B vector accesses (row loads, pack8
// stores, float4 weight loads, partial / dgamma_dbeta vectors) must be 16-B
// aligned; NULL optional operands pass (0 has no low bits)
static int add_ln_check(const void* a, const void* b, const void* gamma, long long T, int d, const char* what,
                        const void* const* more = nullptr, int n_more = 0) {
  if (T < 0 || T > (1LL << 30)) return fail(std::string(what) + ": T out of range");
  if (d != 128 && d != 256 && d != 512) return fail(std::string(what) + ": d must be 128, 256 or 512");
  if (a == nullptr || gamma == nullptr) return fail(std::string(what) + ": a and gamma are required");
  uintptr_t bits = reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) | reinterpret_cast<uintptr_t>(gamma);
  for (int i = 0; i < n_more; ++i) bits |= reinterpret_cast<uintptr_t>(more[i]);
  if (bits & 15) return fail(std::string(what) + ": rows, weights and outputs must be 16-B aligned");
  return 0;
}

extern "C" int rtdetr_add_layer_norm_parts(long long T) {
  const long long p = (T + 15) / 16;
  return (int)(p < 1 ? 1 : p > 256 ? 256 : p);
}

extern "C" int rtdetr_add_layer_norm_pos_fwd(const void* a, const void* b, const void* gamma, const void* beta,
                                             int w_bf16, long long T, int d, float eps, const void* pos, void* out,
                                             void* out2, float* mean, float* rstd, hipStream_t stream) {
  const void* fwd_ops[4] = {beta, out, pos, out2};
  if (add_ln_check(a, b, gamma, T, d, "add_layer_norm_fwd", fwd_ops, 4)) return -1;
  if ((pos == nullptr) != (out2 == nullptr)) return fail("add_layer_norm_pos_fwd: pos and out2 go together");
  if (beta == nullptr || out == nullptr || mean == nullptr || rstd == nullptr)
    return fail("add_layer_norm_fwd: beta, out, mean and rstd are required");
  if (T == 0) return 0;
  long long grid = (T + 15) / 16;
  if (grid > 2048) grid = 2048;
  // bytes: a (+ b) read, out written, mean / rstd written, weights once (+ pos read, out2 written)
  ProfScope prof(stream, PROF_CONV_EPI,
                 2.0 * T * d * ((b != nullptr ? 3.0 : 2.0) + (pos != nullptr ? 2.0 : 0.0)) + 8.0 * T +
                     (w_bf16 ? 4.0 : 8.0) * d);
  const auto* pb = static_cast<const uint16_t*>(pos);
  auto* o2 = static_cast<uint16_t*>(out2);
  const auto* ab = static_cast<const uint16_t*>(a);
  const auto* bb = static_cast<const uint16_t*>(b);
  auto* ob = static_cast<uint16_t*>(out);
#define LNF(NC, WB) \
  MOE_LAUNCH(prof, (add_ln_fwd_kernel<NC, WB>), dim3((unsigned)grid), dim3(256), 0, stream, ab, bb, gamma, beta, \
             (int)T, eps, ob, mean, rstd, pb, o2)
  if (w_bf16) {
    if (d == 128) { LNF(1, true); } else if (d == 256) { LNF(2, true); } else { LNF(4, true); }
  } else {
    if (d == 128) { LNF(1, false); } else if (d == 256) { LNF(2, false); } else { LNF(4, false); }
  }
#undef LNF
  return check_launch("rtdetr_add_layer_norm_fwd");
}

extern "C" int rtdetr_add_layer_norm_fwd(const void* a, const void* b, const void* gamma, const void* beta,
                                         int w_bf16, long long T, int d, float eps, void* out, float* mean,
                                         float* rstd, hipStream_t stream) {
  return rtdetr_add_layer_norm_pos_fwd(a, b, gamma, beta, w_bf16, T, d, eps, nullptr, out, nullptr, mean, rstd,
                                       stream);
}

extern "C" int rtdetr_add_layer_norm_bwd2(const void* dout, const void* dout2, const void* a, const void* b,
                                          const void* gamma, int w_bf16, const float* mean, const float* rstd,
                                          long long T, int d, void* ds, float* partials, int P, void* dgamma_dbeta,
                                          hipStream_t stream) {
  const void* bwd_ops[5] = {dout, ds, partials, dgamma_dbeta, dout2};
  if (add_ln_check(a, b, gamma, T, d, "add_layer_norm_bwd", bwd_ops, 5)) return -1;
  if (dout == nullptr || mean == nullptr || rstd == nullptr || ds == nullptr || partials == nullptr)
    return fail("add_layer_norm_bwd: dout, mean, rstd, ds and partials are required");
  if (P != rtdetr_add_layer_norm_parts(T)) return fail("add_layer_norm_bwd: P must be rtdetr_add_layer_norm_parts(T)");
  // bytes: dout, a (+ b) read, ds written, per-row statistics, partials out and back, [dgamma; dbeta]
  ProfScope prof(stream, PROF_CONV_EPI,
                 2.0 * T * d * ((b != nullptr ? 4.0 : 3.0) + (dout2 != nullptr ? 1.0 : 0.0)) + 8.0 * T + 16.0 * P * d +
                     (w_bf16 ? 6.0 : 12.0) * d);
  const auto* d2 = static_cast<const uint16_t*>(dout2);
  const auto* db = static_cast<const uint16_t*>(dout);
  const auto* ab = static_cast<const uint16_t*>(a);
  const auto* bb = static_cast<const uint16_t*>(b);
  auto* sb = static_cast<uint16_t*>(ds);
#define LNB(NC, WB) \
  MOE_LAUNCH(prof, (add_ln_bwd_kernel<NC, WB>), dim3(P), dim3(256), 0, stream, db, ab, bb, gamma, mean, rstd, \
             (int)T, sb, partials, d2)
  if (w_bf16) {
    if (d == 128) { LNB(1, true); } else if (d == 256) { LNB(2, true); } else { LNB(4, true); }
  } else {
    if (d == 128) { LNB(1, false); } else if (d == 256) { LNB(2, false); } else { LNB(4, false); }
  }
#undef LNB
  int rc = check_launch("rtdetr_add_layer_norm_bwd");
  if (rc != 0 || dgamma_dbeta == nullptr) return rc;  // (NULL: the partials stay for a batched final)
  hipLaunchKernelGGL(add_ln_final_kernel, dim3((2 * d + 15) / 16), dim3(256), 0, stream, partials, P, 2 * d,
                     dgamma_dbeta, w_bf16);
  return check_launch("rtdetr_add_layer_norm_bwd(final)");
}

extern "C" int rtdetr_add_layer_norm_final_batch(int n, const float* const* partials, const int* P, const int* N,
                                                 void* const* out, const int* out_bf16, hipStream_t stream) {
  if (n < 1 || n > kLnFinMax || partials == nullptr || P == nullptr || N == nullptr || out == nullptr ||
      out_bf16 == nullptr)
    return fail("rtdetr_add_layer_norm_final_batch: 1..48 problems, non-NULL arrays");
  LnFinalBatch b{};
  b.n = n;
  int blocks = 0;
  for (int q = 0; q < n; ++q) {
    if (partials[q] == nullptr || out[q] == nullptr || P[q] < 1 || P[q] > 256 || N[q] < 1)
      return fail("rtdetr_add_layer_norm_final_batch: bad problem");
    b.part[q] = partials[q];
    b.out[q] = out[q];
    b.P[q] = P[q];
    b.N[q] = N[q];
    b.bf16[q] = out_bf16[q];
    b.base[q] = blocks;
    blocks += (N[q] + 15) / 16;
  }
  b.base[n] = blocks;
  hipLaunchKernelGGL(add_ln_final_batch_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, b);
  return check_launch("rtdetr_add_layer_norm_final_batch");
}

extern "C" int rtdetr_add_layer_norm_bwd(const void* dout, const void* a, const void* b, const void* gamma,
                                         int w_bf16, const float* mean, const float* rstd, long long T, int d,
                                         void* ds, float* partials, int P, void* dgamma_dbeta,
                                         hipStream_t stream) {
  return rtdetr_add_layer_norm_bwd2(dout, nullptr, a, b, gamma, w_bf16, mean, rstd, T, d, ds, partials, P,
                                    dgamma_dbeta, stream);
}
