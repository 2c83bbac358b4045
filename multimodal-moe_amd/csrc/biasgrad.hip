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
    // loads in flight per thread: with 16-B row vectors a wide gradient has few
    // row lanes per block (N = 1,536: one, 192 threads), so 8 rows per thread
    // keep ~50 KB per CU in flight (4: the value projection's 475 MB column sum
    // ran at 3.7 TB/s)
    constexpr int U = VEC == 8 ? 8 : 4;
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

// Narrow dense linear (out_features M not a multiple of 64: the decoder's
// class heads M = 1, box-head last layers M = 4, attention weights M = 96):
//   dW[m, n] = sum_k gy[k, m] x[k, n]     db[m] = sum_k gy[k, m]
// hipBLASLt ran these few-tile, long-K products on 1-8 workgroups (25-34 us
// each at K = 2,400 rows).  Here one wave owns 128 columns x 16 outputs x a
// slice of rows (4 outputs when M <= 4; gy staged in LDS as fp32 and read as broadcasts, x streamed
// as bf16 pairs, 16 rows in flight; ~1,024 waves), writing fp32 partials [S][M*N + M (+1: even)]; the
// final kernel sums the S slices in a fixed order (deterministic).
constexpr int kNwCB = 128;  // columns (n) per wave
constexpr int kNwU = 16;    // x rows in flight

// TR: the narrow side is the layer's input (N_in <= 128, e.g. the query
// position head's 4 -> 512 layer): the kernel runs on (gy, x) = (x, dY),
// stores its [m, n] sums transposed and takes the bias partial from the
// streamed operand's column sums.
template <int kNwMT, bool TR>  // outputs (m) per wave: 4 (M <= 4) or 16
__device__ __forceinline__ void narrow_wgrad_part_body(const uint16_t* __restrict__ gy,
                                                       const uint16_t* __restrict__ x, int K, int M, int N, int R,
                                                       float* __restrict__ part, int bx, int by, int bz) {
  __shared__ float s_g[64][kNwMT];
  __shared__ float s_db[64];
  const int lane = threadIdx.x;
  const int n = bx * kNwCB + 2 * lane;
  const int m0 = by * kNwMT;
  const int s = bz;
  const int k0 = s * R;
  const int k1 = min(K, k0 + R);
  const bool ncol = n < N;
  const size_t Q = ((size_t)M * N + (TR ? N : M) + 1) & ~(size_t)1;  // slice stride (even)
  float acc[kNwMT][2];
  float xs0 = 0.f, xs1 = 0.f;  // TR: column sums of the streamed operand
#pragma unroll
  for (int m = 0; m < kNwMT; ++m) acc[m][0] = acc[m][1] = 0.f;
  float dbs = 0.f;  // this lane's column of gy is m0 + lane % kNwMT (kNwMT divides 64)
  for (int kc = k0; kc < k1; kc += 64) {
    const int rows = min(64, k1 - kc);
#pragma unroll
    for (int j = 0; j < kNwMT; ++j) {
      const int i = lane + 64 * j;
      const int r = i / kNwMT, m = i % kNwMT;
      const float v = (r < rows && m0 + m < M) ? bf2f(gy[(size_t)(kc + r) * M + m0 + m]) : 0.f;
      s_g[r][m] = v;
      dbs += v;
    }
    __syncthreads();
    for (int r = 0; r < rows; r += kNwU) {
      uint32_t xv[kNwU];
#pragma unroll
      for (int u = 0; u < kNwU; ++u)
        xv[u] = (ncol && r + u < rows) ? *reinterpret_cast<const uint32_t*>(x + (size_t)(kc + r + u) * N + n) : 0u;
#pragma unroll
      for (int u = 0; u < kNwU; ++u) {
        const float x0 = bf2f((uint16_t)(xv[u] & 0xffffu)), x1 = bf2f((uint16_t)(xv[u] >> 16));
        if constexpr (TR) { xs0 += x0; xs1 += x1; }
        const float4* g4 = reinterpret_cast<const float4*>(s_g[(r + u) & 63]);
#pragma unroll
        for (int q = 0; q < kNwMT / 4; ++q) {
          const float4 g = g4[q];
          acc[4 * q + 0][0] += g.x * x0; acc[4 * q + 0][1] += g.x * x1;
          acc[4 * q + 1][0] += g.y * x0; acc[4 * q + 1][1] += g.y * x1;
          acc[4 * q + 2][0] += g.z * x0; acc[4 * q + 2][1] += g.z * x1;
          acc[4 * q + 3][0] += g.w * x0; acc[4 * q + 3][1] += g.w * x1;
        }
      }
    }
    __syncthreads();
  }
  float* ps = part + (size_t)s * Q;
  if (ncol) {
#pragma unroll
    for (int m = 0; m < kNwMT; ++m)
      if (m0 + m < M) {
        if constexpr (TR) {
          ps[(size_t)n * M + m0 + m] = acc[m][0];
          ps[(size_t)(n + 1) * M + m0 + m] = acc[m][1];
        } else {
          *reinterpret_cast<float2*>(ps + (size_t)(m0 + m) * N + n) = make_float2(acc[m][0], acc[m][1]);
        }
      }
    if (TR && by == 0) *reinterpret_cast<float2*>(ps + (size_t)M * N + n) = make_float2(xs0, xs1);
  }
  if (!TR && bx == 0) {  // bias partial: the 64 / kNwMT lanes of each column, fixed order
    s_db[lane] = dbs;
    __syncthreads();
    if (lane < kNwMT && m0 + lane < M) {
      float t = 0.f;
      for (int j = lane; j < 64; j += kNwMT) t += s_db[j];
      ps[(size_t)M * N + m0 + lane] = t;
    }
  }
}

template <int kNwMT, bool TR>
__global__ __launch_bounds__(64) void narrow_wgrad_part_kernel(const uint16_t* __restrict__ gy,
                                                               const uint16_t* __restrict__ x, int K, int M, int N,
                                                               int R, float* __restrict__ part) {
  narrow_wgrad_part_body<kNwMT, TR>(gy, x, K, M, N, R, part, blockIdx.x, blockIdx.y, blockIdx.z);
}

// Batched narrow weight gradients (the decoder's score / box / query-position
// heads after the backward, linear.DeferredWgrad): problem q (the kernel's
// orientation: narrow side Mk, streamed side Nk) owns blocks [base[q],
// base[q+1]) of one launch; groups g sum the partial slices of their member
// problems (a weight applied several times -- the shared query-position head
// -- gets one gradient, fixed problem then slice order: deterministic).
constexpr int kNbMax = 32;
struct NarrowBatch {
  const uint16_t* g[kNbMax];  // the kernel's narrow operand (gy, or x when transposed)
  const uint16_t* x[kNbMax];  // the streamed operand
  long long poff[kNbMax];     // float offset of the problem's slices in part
  int K[kNbMax], Mk[kNbMax], Nk[kNbMax], R[kNbMax], S[kNbMax], base[kNbMax + 1];
  unsigned char mt4[kNbMax], tr[kNbMax];
  int n;
};
struct NarrowGroups {
  void* dw[kNbMax];
  void* db[kNbMax];
  int M[kNbMax], N[kNbMax];  // the layer's outputs / inputs (dW [M][N], db [M])
  int first[kNbMax], count[kNbMax], base[kNbMax + 1];
  int n, out_bf16;
};

__global__ __launch_bounds__(64) void narrow_wgrad_part_batch_kernel(NarrowBatch b, float* __restrict__ part) {
  int q = 0;
  while (q + 1 < b.n && (int)blockIdx.x >= b.base[q + 1]) ++q;
  const int local = blockIdx.x - b.base[q];
  const int gx = (b.Nk[q] + kNwCB - 1) / kNwCB, gy = b.mt4[q] ? 1 : (b.Mk[q] + 15) / 16;
  const int bx = local % gx, by = (local / gx) % gy, bz = local / (gx * gy);
  float* pp = part + b.poff[q];
  if (b.mt4[q]) {
    if (b.tr[q]) narrow_wgrad_part_body<4, true>(b.g[q], b.x[q], b.K[q], b.Mk[q], b.Nk[q], b.R[q], pp, bx, by, bz);
    else narrow_wgrad_part_body<4, false>(b.g[q], b.x[q], b.K[q], b.Mk[q], b.Nk[q], b.R[q], pp, bx, by, bz);
  } else {
    if (b.tr[q]) narrow_wgrad_part_body<16, true>(b.g[q], b.x[q], b.K[q], b.Mk[q], b.Nk[q], b.R[q], pp, bx, by, bz);
    else narrow_wgrad_part_body<16, false>(b.g[q], b.x[q], b.K[q], b.Mk[q], b.Nk[q], b.R[q], pp, bx, by, bz);
  }
}

// one block per 32 outputs of a group: 8 slice lanes, the group's problems in
// order, each problem's slices in order, then a fixed 8-lane sum
__global__ __launch_bounds__(256) void narrow_wgrad_final_batch_kernel(NarrowBatch b, NarrowGroups gr,
                                                                       const float* __restrict__ part) {
  __shared__ float s_acc[8][32];
  int g = 0;
  while (g + 1 < gr.n && (int)blockIdx.x >= gr.base[g + 1]) ++g;
  const size_t MN = (size_t)gr.M[g] * gr.N[g], NB = gr.M[g];
  const size_t Q = (MN + NB + 1) & ~(size_t)1;
  const int cl = threadIdx.x & 31, pl = threadIdx.x >> 5;
  const size_t c = (size_t)(blockIdx.x - gr.base[g]) * 32 + cl;
  float t = 0.f;
  if (c < MN + NB) {
    for (int j = 0; j < gr.count[g]; ++j) {
      const int q = gr.first[g] + j;
      const float* pp = part + b.poff[q];
      for (int p = pl; p < b.S[q]; p += 8) t += pp[(size_t)p * Q + c];
    }
  }
  s_acc[pl][cl] = t;
  __syncthreads();
  if (pl == 0 && c < MN + NB) {
    float r = 0.f;
#pragma unroll
    for (int l = 0; l < 8; ++l) r += s_acc[l][cl];
    void* out = c < MN ? gr.dw[g] : gr.db[g];
    const size_t i = c < MN ? c : c - MN;
    if (gr.out_bf16) static_cast<uint16_t*>(out)[i] = f2bf(r);
    else static_cast<float*>(out)[i] = r;
  }
}

// 8 slice lanes x 32 outputs per block (fixed-order sums, as bias_grad_final)
// (MN dW sums followed by NB bias sums per slice)
__global__ __launch_bounds__(256) void narrow_wgrad_final_kernel(const float* __restrict__ part, int S, size_t MN,
                                                                 int NB, void* __restrict__ dw, void* __restrict__ db,
                                                                 int out_bf16) {
  __shared__ float s_acc[8][32];
  const size_t M = NB;  // bias entries
  const size_t Q = (MN + NB + 1) & ~(size_t)1;
  const int cl = threadIdx.x & 31;
  const int pl = threadIdx.x >> 5;
  const size_t c = (size_t)blockIdx.x * 32 + cl;
  float t = 0.f;
  if (c < MN + M) {
    constexpr int U = 8;
    for (int p = pl; p < S; p += 8 * U) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = p + 8 * u < S ? part[(size_t)(p + 8 * u) * Q + c] : 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u) t += v[u];
    }
  }
  s_acc[pl][cl] = t;
  __syncthreads();
  if (pl == 0 && c < MN + M) {
    float r = 0.f;
#pragma unroll
    for (int l = 0; l < 8; ++l) r += s_acc[l][cl];
    void* out = c < MN ? dw : db;
    const size_t i = c < MN ? c : c - MN;
    if (out_bf16) static_cast<uint16_t*>(out)[i] = f2bf(r);
    else static_cast<float*>(out)[i] = r;
  }
}

}  // namespace moe

using namespace moe;

// Row slices: about 1,024 waves over the grid, at most 256 slices, >= 8 rows each.
static int narrow_rows(int K, int M, int N) {
  const int wps = ((N + kNwCB - 1) / kNwCB) * (M <= 4 ? 1 : (M + 15) / 16);
  int s = 1024 / wps;
  s = s < 1 ? 1 : (s > 256 ? 256 : s);
  int r = (K + s - 1) / s;
  return r < 8 ? 8 : r;
}

static int narrow_slices(int K, int M, int N) {
  const int r = narrow_rows(K, M, N);
  return (K + r - 1) / r;
}

// Kernel orientation of a layer with M outputs and N inputs: direct when M <=
// 128 and N is even (the kernel's narrow side is M), otherwise transposed (TR).
static bool narrow_tr(int M, int N) { return !(M <= 128 && N % 2 == 0); }

extern "C" int rtdetr_linear_wgrad_narrow_parts(int K, int M, int N) {
  if (K <= 0 || M <= 0 || N <= 0) return 0;
  const bool tr = narrow_tr(M, N);
  return narrow_slices(K, tr ? N : M, tr ? M : N) * ((M * N + M + 1) & ~1);
}

extern "C" int rtdetr_linear_wgrad_narrow(const void* gy, const void* x, void* dw, void* db, float* part, int K, int M,
                                          int N, int out_bf16, hipStream_t stream) {
  if (gy == nullptr || x == nullptr || dw == nullptr || db == nullptr || part == nullptr)
    return fail("rtdetr_linear_wgrad_narrow: null pointer");
  const bool tr = narrow_tr(M, N);
  const int Mk = tr ? N : M, Nk = tr ? M : N;  // the kernel's narrow and streamed sides
  const void* gk = tr ? x : gy;
  const void* xk = tr ? gy : x;
  if (K <= 0 || Mk <= 0 || Nk <= 0 || Mk > 128 || Nk % 2 != 0 || Nk > 4096)
    return fail("rtdetr_linear_wgrad_narrow: needs K > 0 and M <= 128 with N even (or N <= 128 with M even), "
                "the other side <= 4096");
  if ((reinterpret_cast<uintptr_t>(xk) & 3) != 0 || (reinterpret_cast<uintptr_t>(part) & 7) != 0)
    return fail("rtdetr_linear_wgrad_narrow: the wide operand must be 4-byte and part 8-byte aligned");
  const int R = narrow_rows(K, Mk, Nk);
  const int S = (K + R - 1) / R;
  const double Q = (double)M * N + M;
  ProfScope prof(stream, PROF_LINEAR, 2.0 * K * (M + N) + 8.0 * S * Q + (out_bf16 ? 2.0 : 4.0) * Q, false, 0.0,
                 2.0 * K * M * N);
  const dim3 grid((Nk + kNwCB - 1) / kNwCB, Mk <= 4 ? 1 : (Mk + 15) / 16, S);
  const uint16_t* g16 = static_cast<const uint16_t*>(gk);
  const uint16_t* x16 = static_cast<const uint16_t*>(xk);
  if (Mk <= 4 && tr)
    MOE_LAUNCH(prof, (narrow_wgrad_part_kernel<4, true>), grid, dim3(64), 0, stream, g16, x16, K, Mk, Nk, R, part);
  else if (Mk <= 4)
    MOE_LAUNCH(prof, (narrow_wgrad_part_kernel<4, false>), grid, dim3(64), 0, stream, g16, x16, K, Mk, Nk, R, part);
  else if (tr)
    MOE_LAUNCH(prof, (narrow_wgrad_part_kernel<16, true>), grid, dim3(64), 0, stream, g16, x16, K, Mk, Nk, R, part);
  else
    MOE_LAUNCH(prof, (narrow_wgrad_part_kernel<16, false>), grid, dim3(64), 0, stream, g16, x16, K, Mk, Nk, R, part);
  int rc = check_launch("rtdetr_linear_wgrad_narrow(part)");
  if (rc != 0) return rc;
  const size_t MN = (size_t)M * N;
  hipLaunchKernelGGL(narrow_wgrad_final_kernel, dim3((unsigned)((MN + M + 31) / 32)), dim3(256), 0, stream, part, S,
                     MN, M, dw, db, out_bf16);
  return check_launch("rtdetr_linear_wgrad_narrow(final)");
}

// Batched: problems q = (gy [K][M], x [K][N]) in groups (consecutive problems
// of one group share M, N and the outputs dw [M][N], db [M]).  part: at least
// rtdetr_linear_wgrad_narrow_batch_parts floats.  Two launches for all.
static int narrow_batch_setup(int n, const int* K, const int* M, const int* N, const void* const* gy,
                              const void* const* x, NarrowBatch& b, long long& floats) {
  if (n < 1 || n > kNbMax) return fail("rtdetr_linear_wgrad_narrow_batch: 1..32 problems");
  b = NarrowBatch{};
  b.n = n;
  floats = 0;
  int blocks = 0;
  for (int q = 0; q < n; ++q) {
    const bool tr = narrow_tr(M[q], N[q]);
    const int Mk = tr ? N[q] : M[q], Nk = tr ? M[q] : N[q];
    if (K[q] <= 0 || Mk <= 0 || Nk <= 0 || Mk > 128 || Nk % 2 != 0 || Nk > 4096)
      return fail("rtdetr_linear_wgrad_narrow_batch: a problem outside the narrow shapes");
    b.tr[q] = tr;
    b.mt4[q] = Mk <= 4;
    b.Mk[q] = Mk;
    b.Nk[q] = Nk;
    b.K[q] = K[q];
    b.R[q] = narrow_rows(K[q], Mk, Nk);
    b.S[q] = (K[q] + b.R[q] - 1) / b.R[q];
    if (gy != nullptr) {
      b.g[q] = static_cast<const uint16_t*>(tr ? x[q] : gy[q]);
      b.x[q] = static_cast<const uint16_t*>(tr ? gy[q] : x[q]);
      if (b.g[q] == nullptr || b.x[q] == nullptr || (reinterpret_cast<uintptr_t>(b.x[q]) & 3))
        return fail("rtdetr_linear_wgrad_narrow_batch: null or misaligned operand");
    }
    b.poff[q] = floats;
    floats += (long long)b.S[q] * (((long long)M[q] * N[q] + M[q] + 1) & ~1LL);
    floats = (floats + 1) & ~1LL;
    b.base[q] = blocks;
    blocks += ((Nk + kNwCB - 1) / kNwCB) * (Mk <= 4 ? 1 : (Mk + 15) / 16) * b.S[q];
  }
  b.base[n] = blocks;
  return 0;
}

extern "C" long long rtdetr_linear_wgrad_narrow_batch_parts(int n, const int* K, const int* M, const int* N) {
  NarrowBatch b;
  long long floats = 0;
  if (narrow_batch_setup(n, K, M, N, nullptr, nullptr, b, floats)) return -1;
  return floats;
}

extern "C" int rtdetr_linear_wgrad_narrow_batch(int n, const void* const* gy, const void* const* x, const int* K,
                                                const int* M, const int* N, int n_groups, const int* group_count,
                                                void* const* dw, void* const* db, float* part, long long part_floats,
                                                int out_bf16, hipStream_t stream) {
  if (gy == nullptr || x == nullptr || K == nullptr || M == nullptr || N == nullptr || group_count == nullptr ||
      dw == nullptr || db == nullptr || part == nullptr || (reinterpret_cast<uintptr_t>(part) & 7))
    return fail("rtdetr_linear_wgrad_narrow_batch: null pointer or misaligned part");
  NarrowBatch b;
  long long floats = 0;
  if (int rc = narrow_batch_setup(n, K, M, N, gy, x, b, floats)) return rc;
  if (floats > part_floats) return fail("rtdetr_linear_wgrad_narrow_batch: part too small");
  if (n_groups < 1 || n_groups > n) return fail("rtdetr_linear_wgrad_narrow_batch: bad group count");
  NarrowGroups gr{};
  gr.n = n_groups;
  gr.out_bf16 = out_bf16;
  int q = 0, blocks = 0;
  double bytes = 0.0, flops = 0.0;
  for (int g = 0; g < n_groups; ++g) {
    if (group_count[g] < 1 || q + group_count[g] > n) return fail("rtdetr_linear_wgrad_narrow_batch: bad groups");
    for (int j = 1; j < group_count[g]; ++j)
      if (M[q + j] != M[q] || N[q + j] != N[q]) return fail("rtdetr_linear_wgrad_narrow_batch: group shapes differ");
    if (dw[g] == nullptr || db[g] == nullptr) return fail("rtdetr_linear_wgrad_narrow_batch: null output");
    gr.dw[g] = dw[g];
    gr.db[g] = db[g];
    gr.M[g] = M[q];
    gr.N[g] = N[q];
    gr.first[g] = q;
    gr.count[g] = group_count[g];
    gr.base[g] = blocks;
    blocks += (int)(((size_t)M[q] * N[q] + M[q] + 31) / 32);
    for (int j = 0; j < group_count[g]; ++j) {
      bytes += 2.0 * K[q + j] * (M[q + j] + N[q + j]);
      flops += 2.0 * K[q + j] * M[q + j] * N[q + j];
    }
    q += group_count[g];
  }
  if (q != n) return fail("rtdetr_linear_wgrad_narrow_batch: groups do not cover the problems");
  gr.base[n_groups] = blocks;
  ProfScope prof(stream, PROF_LINEAR, bytes + 8.0 * floats, false, 0.0, flops);
  MOE_LAUNCH(prof, narrow_wgrad_part_batch_kernel, dim3((unsigned)b.base[n]), dim3(64), 0, stream, b, part);
  if (int rc = check_launch("rtdetr_linear_wgrad_narrow_batch(part)")) return rc;
  hipLaunchKernelGGL(narrow_wgrad_final_batch_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, b, gr,
                     static_cast<const float*>(part));
  return check_launch("rtdetr_linear_wgrad_narrow_batch(final)");
}

extern "C" int rtdetr_bias_grad_parts(long long M, int N) {
  if (M <= 0 || N <= 0) return 1;
  // ~128 rows per block at small M, at most 512 blocks (two per CU) at large M
  long long p = (M + 127) / 128;
  return (int)(p > 512 ? 512 : p);
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
