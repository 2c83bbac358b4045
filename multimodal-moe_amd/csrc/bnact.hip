// Training-mode BatchNorm (batch statistics) fused with what follows it in the
// RT-DETR HybridEncoder (the dense body around the MoE path):
//   ConvNormLayer(act="silu"):  y = silu(BN(x))
//   RepVggBlock:                y = silu(BN1(x1) + BN2(x2))
// over NHWC (channels_last) bf16 activations x_i [M = N*H*W, C], fp32 affine /
// statistics.  torch runs each BN as three MIOpen kernels forward and three
// backward plus separate add / silu / silu_backward passes; here:
//   forward:  bn_stats (per-block partial sums of x and x^2, both branches in
//             one launch) -> bn_finalize (mean, invstd, scale/shift, running
//             stats) -> bn_apply (normalise, sum branches, activate; one pass)
//   backward: bn_bwd_reduce (g = dy * act'(z) recomputed from x, partial sums
//             of g and g * xhat_i) -> bn_bwd_finalize (dgamma, dbeta and the
//             per-channel coefficients of dx) -> bn_bwd_dx (every branch's dx
//             in one pass).
// Deterministic: fixed partition of rows into blocks, fixed reduction trees,
// no atomics.  Rows per block are fixed by M alone, so eager and graph runs
// agree bit for bit.  Each thread moves 16-B chunks (8 channels); C is a power
// of two in [8, 2048] so a block's 256 threads tile whole rows.
#include "moe_common.h"
#include "prof.h"

namespace moe {

struct BnArgs {
  const uint4* x[2];
  const float* gamma[2];
  const float* beta[2];
  float* run_mean[2];
  float* run_var[2];
  int nb;  // branches: 1 or 2
  // row map of y (forward) / dy (backward): row r of the [M, C] layout lives
  // at row (r / rhw) * rbs + r % rhw -- a batch-strided slice of a wider
  // tensor (the decoder's memory [B, S, C], one level's rows per image);
  // rhw == 0: contiguous (row r at row r)
  long long rhw, rbs;
  // forward: y = act(z) + resid (resid bf16 [M, C] in x's layout, or NULL);
  // act(z) is rounded to bf16 first, then the fp32 sum rounded once -- the
  // same bits as a bf16 activation followed by torch's bf16 add
  const uint4* resid;
};

__device__ __forceinline__ long long map_row(const BnArgs& a, long long r) {
  return a.rhw ? (r / a.rhw) * a.rbs + r % a.rhw : r;
}

constexpr int BN_MAX_BLOCKS = 2048;  // partial rows a finalize reduces (the convolution-epilogue statistics: one per M tile)
constexpr int BN_BLOCKS = 1024;      // partial-sum blocks of bn_stats / bn_bwd_reduce (4 per CU)
constexpr int BN_FIN_T = 1024;        // finalize threads: 8 channels x 128 block lanes

__device__ __forceinline__ void load8f(const float* p, float* v) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

__device__ __forceinline__ float sigmoidf_(float z) { return 1.f / (1.f + __expf(-z)); }

// partial sums of x and x^2: part[br][blk][2][C]
__global__ __launch_bounds__(256) void bn_stats_kernel(BnArgs a, long long M, int C, int rpb,
                                                       float* __restrict__ part) {
  extern __shared__ float sm[];  // [2][groups][C] = 2 * 256 * 8 floats
  const int br = blockIdx.y, cch = C >> 3, groups = 256 / cch;
  const int t = threadIdx.x, cc = t % cch, g = t / cch;
  const long long r0 = (long long)blockIdx.x * rpb;
  const long long r1 = r0 + rpb < M ? r0 + rpb : M;
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
  const uint4* x = a.x[br];
  long long r = r0 + g;
  for (; r + 3 * groups < r1; r += 4 * groups) {  // 4 rows in flight per thread
    uint4 u[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) u[k] = x[(r + (long long)k * groups) * cch + cc];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float v[8];
      unpack8(u[k], v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[j] += v[j];
        q[j] = fmaf(v[j], v[j], q[j]);
      }
    }
  }
  for (; r < r1; r += groups) {
    float v[8];
    unpack8(x[r * cch + cc], v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s[j] += v[j];
      q[j] = fmaf(v[j], v[j], q[j]);
    }
  }
  float* ss = sm;
  float* sq = sm + groups * C;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ss[g * C + cc * 8 + j] = s[j];
    sq[g * C + cc * 8 + j] = q[j];
  }
  __syncthreads();
  float* p = part + ((size_t)br * gridDim.x + blockIdx.x) * 2 * C;
  for (int c = t; c < C; c += 256) {
    float a1 = 0.f, a2 = 0.f;
    for (int k = 0; k < groups; ++k) {
      a1 += ss[k * C + c];
      a2 += sq[k * C + c];
    }
    p[c] = a1;
    p[C + c] = a2;
  }
}

// Sum of nblk (<= BN_MAX_BLOCKS) partial rows of `width` floats for 8
// channels per block: thread (k, c) adds blocks k, k+128, ... (all loads issued
// before the adds), then a fixed tree over k in LDS.  Result for channel
// c0 + c, slot w, in red[w][0][c].
template <int WIDTH>
__device__ __forceinline__ void reduce_partials(const float* __restrict__ part, int nblk, int C, int c0,
                                                double* red /*[WIDTH][128][8]*/) {
  constexpr int KL = BN_FIN_T / 8, PER = BN_MAX_BLOCKS / KL;
  const int t = threadIdx.x, c = t & 7, k = t >> 3;
  float v[WIDTH][PER];
#pragma unroll
  for (int w = 0; w < WIDTH; ++w)
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int b = k + u * KL;
      v[w][u] = b < nblk ? part[((size_t)b * WIDTH + w) * C + c0 + c] : 0.f;
    }
#pragma unroll
  for (int w = 0; w < WIDTH; ++w) {
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < PER; ++u) acc += (double)v[w][u];
    red[(w * KL + k) * 8 + c] = acc;
  }
  __syncthreads();
  for (int h = KL / 2; h > 0; h >>= 1) {
    if (k < h)
#pragma unroll
      for (int w = 0; w < WIDTH; ++w) red[(w * KL + k) * 8 + c] += red[(w * KL + k + h) * 8 + c];
    __syncthreads();
  }
}

// saved[br][4][C] = mean, invstd, scale = gamma * invstd, shift = beta - mean * scale;
// running stats: (1 - m) r + m stat, unbiased variance (torch.nn.BatchNorm2d)
__global__ __launch_bounds__(BN_FIN_T) void bn_finalize_kernel(BnArgs a, const float* __restrict__ part, int nblk,
                                                               long long M, int C, float eps, float momentum,
                                                               float* __restrict__ saved) {
  __shared__ double red[2 * (BN_FIN_T / 8) * 8];
  const int br = blockIdx.y, c0 = blockIdx.x * 8;
  reduce_partials<2>(part + (size_t)br * nblk * 2 * C, nblk, C, c0, red);
  const int t = threadIdx.x;
  if (t < 8) {
    const int c = c0 + t;
    const double mean = red[t] / (double)M;
    const double var = fmax(red[(BN_FIN_T / 8) * 8 + t] / (double)M - mean * mean, 0.0);
    const float invstd = (float)(1.0 / sqrt(var + (double)eps));
    const float sc = a.gamma[br][c] * invstd;
    float* sv = saved + (size_t)br * 4 * C;
    sv[c] = (float)mean;
    sv[C + c] = invstd;
    sv[2 * C + c] = sc;
    sv[3 * C + c] = a.beta[br][c] - (float)mean * sc;
    if (a.run_mean[br] != nullptr) {
      a.run_mean[br][c] = (1.f - momentum) * a.run_mean[br][c] + momentum * (float)mean;
      a.run_var[br][c] = (1.f - momentum) * a.run_var[br][c] + momentum * (float)(var * (double)M / (double)(M - 1));
    }
  }
}

// z = sum_i x_i * scale_i + shift_i for one 8-channel chunk (NB branches,
// compile-time so that xs stays in registers)
template <int NB>
__device__ __forceinline__ void bn_z(const BnArgs& a, const float* __restrict__ saved, int C, long long i, int c0,
                                     float* z, float (*xs)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = 0.f;
#pragma unroll
  for (int br = 0; br < NB; ++br) {
    float sc[8], sh[8];
    unpack8(a.x[br][i], xs[br]);
    load8f(saved + (size_t)br * 4 * C + 2 * C + c0, sc);
    load8f(saved + (size_t)br * 4 * C + 3 * C + c0, sh);
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] += fmaf(xs[br][j], sc[j], sh[j]);
  }
}

template <int ACT, int NB>
__global__ __launch_bounds__(256) void bn_apply_kernel(BnArgs a, const float* __restrict__ saved, long long nchunk,
                                                       int C, uint4* __restrict__ y) {
  const int cch = C >> 3;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nchunk; i += (long long)gridDim.x * 256) {
    const int cc = (int)(i % cch), c0 = cc * 8;
    float z[8], xs[NB][8];
    bn_z<NB>(a, saved, C, i, c0, z, xs);
    if constexpr (ACT == 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) z[j] = z[j] * sigmoidf_(z[j]);
    }
    uint4 o = pack8(z);
    if (a.resid != nullptr) {
      float r[8];
      unpack8(o, z);
      unpack8(a.resid[i], r);
#pragma unroll
      for (int j = 0; j < 8; ++j) z[j] += r[j];
      o = pack8(z);
    }
    y[a.rhw ? map_row(a, i / cch) * cch + cc : i] = o;
  }
}

// Inference-mode BatchNorm (running statistics) + branch sum + act (+ resid):
// scale = gamma * rsqrt(running_var + eps), shift = beta - running_mean *
// scale per channel, computed by every workgroup into LDS, then the apply
// pass -- one launch per BatchNorm (torch: a batch_norm kernel, then SiLU and
// the branch add as separate passes).
template <int ACT, int NB>
__global__ __launch_bounds__(256) void bn_eval_kernel(BnArgs a, float eps, long long nchunk, int C,
                                                      uint4* __restrict__ y) {
  extern __shared__ float ss[];  // [NB][2][C]
  for (int i = threadIdx.x; i < NB * C; i += 256) {
    const int br = i / C, c = i - br * C;
    const float sc = a.gamma[br][c] * rsqrtf(a.run_var[br][c] + eps);
    ss[(br * 2) * C + c] = sc;
    ss[(br * 2 + 1) * C + c] = a.beta[br][c] - a.run_mean[br][c] * sc;
  }
  __syncthreads();
  const int cch = C >> 3;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nchunk; i += (long long)gridDim.x * 256) {
    const int c0 = (int)(i % cch) * 8;
    float z[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = 0.f;
#pragma unroll
    for (int br = 0; br < NB; ++br) {
      float xs[8];
      unpack8(a.x[br][i], xs);
#pragma unroll
      for (int j = 0; j < 8; ++j) z[j] += fmaf(xs[j], ss[(br * 2) * C + c0 + j], ss[(br * 2 + 1) * C + c0 + j]);
    }
    if constexpr (ACT == 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) z[j] = z[j] * sigmoidf_(z[j]);
    }
    uint4 o = pack8(z);
    if (a.resid != nullptr) {  // act rounded to bf16 first, then the fp32 sum rounded once (as bn_apply)
      float r[8];
      unpack8(o, z);
      unpack8(a.resid[i], r);
#pragma unroll
      for (int j = 0; j < 8; ++j) z[j] += r[j];
      o = pack8(z);
    }
    y[i] = o;
  }
}

// g = dy * act'(z)
template <int ACT>
__device__ __forceinline__ void bn_grad_in(const uint4* __restrict__ dy, long long i, const float* z, float* g) {
  unpack8(dy[i], g);
  if constexpr (ACT == 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float s = sigmoidf_(z[j]);
      g[j] *= s * (1.f + z[j] * (1.f - s));
    }
  }
}

// partials part[blk][1 + nb][C]: sum g, sum g * x_i (xhat applied in the
// finalize: sum g xhat = invstd (sum g x - mean sum g))
template <int ACT, int NB>
__device__ __forceinline__ void bn_bwd_row(const BnArgs& a, const uint4* __restrict__ dy,
                                           const float* __restrict__ saved, int C, long long i, long long idy, int c0,
                                           float* sg, float (*sgx)[8]) {
  float z[8], xs[NB][8], gv[8];
  bn_z<NB>(a, saved, C, i, c0, z, xs);
  bn_grad_in<ACT>(dy, idy, z, gv);
#pragma unroll
  for (int j = 0; j < 8; ++j) sg[j] += gv[j];
#pragma unroll
  for (int br = 0; br < NB; ++br)
#pragma unroll
    for (int j = 0; j < 8; ++j) sgx[br][j] = fmaf(gv[j], xs[br][j], sgx[br][j]);
}

template <int ACT, int NB>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(BnArgs a, const uint4* __restrict__ dy,
                                                            const float* __restrict__ saved, long long M, int C,
                                                            int rpb, float* __restrict__ part) {
  extern __shared__ float sm[];  // [3][groups][C]
  const int cch = C >> 3, groups = 256 / cch, width = 1 + NB;
  const int t = threadIdx.x, cc = t % cch, g = t / cch, c0 = cc * 8;
  const long long r0 = (long long)blockIdx.x * rpb;
  const long long r1 = r0 + rpb < M ? r0 + rpb : M;
  float sg[8], sgx[NB][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sg[j] = 0.f;
#pragma unroll
    for (int br = 0; br < NB; ++br) sgx[br][j] = 0.f;
  }
  long long r = r0 + g;
  for (; r + groups < r1; r += 2 * groups) {
    bn_bwd_row<ACT, NB>(a, dy, saved, C, r * cch + cc, map_row(a, r) * cch + cc, c0, sg, sgx);
    bn_bwd_row<ACT, NB>(a, dy, saved, C, (r + groups) * cch + cc, map_row(a, r + groups) * cch + cc, c0, sg, sgx);
  }
  if (r < r1) bn_bwd_row<ACT, NB>(a, dy, saved, C, r * cch + cc, map_row(a, r) * cch + cc, c0, sg, sgx);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sm[g * C + c0 + j] = sg[j];
#pragma unroll
    for (int br = 0; br < NB; ++br) sm[((1 + br) * groups + g) * C + c0 + j] = sgx[br][j];
  }
  __syncthreads();
  float* p = part + (size_t)blockIdx.x * width * C;
  for (int c = t; c < C; c += 256) {
    for (int w = 0; w < width; ++w) {
      float acc = 0.f;
      for (int k = 0; k < groups; ++k) acc += sm[(w * groups + k) * C + c];
      p[w * C + c] = acc;
    }
  }
}

// dgb[br][2][C] = dgamma, dbeta; coef[br][3][C] = (A, B, D) with
// dx_i = A g + B x_i + D:  A = scale, B = -scale * invstd * Sgx / M,
// D = -scale * Sg / M - B * mean
template <int NB>
__global__ __launch_bounds__(BN_FIN_T) void bn_bwd_finalize_kernel(const float* __restrict__ part, int nblk,
                                                                   long long M, int C,
                                                                   const float* __restrict__ saved,
                                                                   float* __restrict__ coef, float* __restrict__ dgb) {
  constexpr int KL = BN_FIN_T / 8;
  __shared__ double red[(1 + NB) * KL * 8];
  const int c0 = blockIdx.x * 8;
  reduce_partials<1 + NB>(part, nblk, C, c0, red);
  const int t = threadIdx.x;
  if (t < 8 * NB) {
    const int br = t >> 3, c = c0 + (t & 7);
    const float* sv = saved + (size_t)br * 4 * C;
    const double mean = sv[c], inv = sv[C + c], sc = sv[2 * C + c];
    const double sg = red[t & 7];
    const double sgx = inv * (red[((1 + br) * KL) * 8 + (t & 7)] - mean * sg);  // sum g * xhat
    const double B = -sc * inv * sgx / (double)M;
    float* cf = coef + (size_t)br * 3 * C;
    cf[c] = (float)sc;
    cf[C + c] = (float)B;
    cf[2 * C + c] = (float)(-sc * sg / (double)M - B * mean);
    dgb[(size_t)br * 2 * C + c] = (float)sgx;
    dgb[(size_t)br * 2 * C + C + c] = (float)sg;
  }
}

template <int ACT, int NB>
__global__ __launch_bounds__(256) void bn_bwd_dx_kernel(BnArgs a, const uint4* __restrict__ dy,
                                                        const float* __restrict__ saved,
                                                        const float* __restrict__ coef, long long nchunk, int C,
                                                        uint4* __restrict__ dx0, uint4* __restrict__ dx1) {
  const int cch = C >> 3;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nchunk; i += (long long)gridDim.x * 256) {
    const int cc = (int)(i % cch), c0 = cc * 8;
    float z[8], xs[NB][8], gv[8];
    bn_z<NB>(a, saved, C, i, c0, z, xs);
    bn_grad_in<ACT>(dy, a.rhw ? map_row(a, i / cch) * cch + cc : i, z, gv);
#pragma unroll
    for (int br = 0; br < NB; ++br) {
      float A[8], B[8], D[8], o[8];
      const float* cf = coef + (size_t)br * 3 * C;
      load8f(cf + c0, A);
      load8f(cf + C + c0, B);
      load8f(cf + 2 * C + c0, D);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = fmaf(A[j], gv[j], fmaf(B[j], xs[br][j], D[j]));
      (br == 0 ? dx0 : dx1)[i] = pack8(o);
    }
  }
}

static int bn_grid(long long nchunk) {
  long long g = (nchunk + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

// rows per block and block count of the reductions: a function of M only
static void bn_blocks(long long M, int* nblk, int* rpb) {
  long long n = (M + 63) / 64;
  if (n > BN_BLOCKS) n = BN_BLOCKS;
  if (n < 1) n = 1;
  *rpb = (int)((M + n - 1) / n);
  *nblk = (int)((M + *rpb - 1) / *rpb);
}

static int bn_check(int nb, long long M, int C, int act) {
  if (nb < 1 || nb > 2) return fail("bn_act: 1 or 2 branches");
  if (C < 8 || C > 2048 || (C & (C - 1))) return fail("bn_act: C must be a power of two in [8, 2048]");
  if (M < 2) return fail("bn_act: need at least 2 rows (unbiased running variance)");
  if (act < 0 || act > 1) return fail("bn_act: act must be 0 (none) or 1 (silu)");
  return 0;
}

}  // namespace moe

using namespace moe;

extern "C" size_t rtdetr_bn_act_workspace(long long M, int C, int nb) {
  (void)M;
  return (size_t)BN_BLOCKS * 3 * C * (nb > 1 ? 2 : 1) * sizeof(float);
}

static int bn_rows_check(long long M, long long hw, long long bs) {
  if (hw == 0) return 0;
  if (hw < 0 || bs < hw || M % hw) return fail("bn_act rows: need 0 < hw <= bstride and M a multiple of hw");
  return 0;
}

static int bn_act_fwd_impl(const void* const* x, const float* const* gamma, const float* const* beta,
                           float* const* run_mean, float* const* run_var, int nb, long long M, int C, int act,
                           float eps, float momentum, float* saved, float* ws, const float* part, int part_blocks,
                           const void* resid, void* y, long long y_hw, long long y_bstride, hipStream_t stream) {
  if (int rc = bn_check(nb, M, C, act)) return rc;
  if (int rc = bn_rows_check(M, y_hw, y_bstride)) return rc;
  if (!x || !gamma || !beta || !saved || !y || (!ws && !part)) return fail("bn_act_fwd: NULL argument");
  if (part != nullptr && (part_blocks < 1 || part_blocks > BN_MAX_BLOCKS))
    return fail("bn_act_fwd_part: need 1 <= part_blocks <= 2048");
  BnArgs a{};
  a.nb = nb;
  a.rhw = y_hw;
  a.rbs = y_bstride;
  a.resid = static_cast<const uint4*>(resid);
  if (reinterpret_cast<uintptr_t>(resid) % 16) return fail("bn_act_fwd: resid must be 16-B aligned");
  for (int i = 0; i < nb; ++i) {
    if (!x[i] || !gamma[i] || !beta[i]) return fail("bn_act_fwd: NULL branch pointer");
    a.x[i] = static_cast<const uint4*>(x[i]);
    a.gamma[i] = gamma[i];
    a.beta[i] = beta[i];
    a.run_mean[i] = run_mean ? run_mean[i] : nullptr;
    a.run_var[i] = run_var ? run_var[i] : nullptr;
    if ((a.run_mean[i] == nullptr) != (a.run_var[i] == nullptr)) return fail("bn_act_fwd: running mean without var");
  }
  int nblk, rpb;
  bn_blocks(M, &nblk, &rpb);
  const long long nchunk = M * (C / 8);
  if (part == nullptr) {
    ProfScope prof(stream, PROF_CONV_EPI, 2.0 * nb * M * C);
    MOE_LAUNCH(prof, bn_stats_kernel, dim3(nblk, nb), dim3(256), 2 * 2048 * sizeof(float), stream, a, M, C, rpb, ws);
  } else {
    nblk = part_blocks;  // the producing convolution's epilogue wrote them (rtdetr_conv_fwd_stats)
  }
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(C / 8, nb), dim3(BN_FIN_T), 0, stream, a, part ? part : ws, nblk, M, C,
                     eps, momentum, saved);
  {
    ProfScope prof(stream, PROF_CONV_EPI, 2.0 * (nb + 1) * M * C);
#define BN_APPLY(A, N)                                                                                  \
  MOE_LAUNCH(prof, (bn_apply_kernel<A, N>), dim3(bn_grid(nchunk)), dim3(256), 0, stream, a, saved, nchunk, C, \
             static_cast<uint4*>(y))
    if (act == 1) {
      if (nb == 2) BN_APPLY(1, 2); else BN_APPLY(1, 1);
    } else {
      if (nb == 2) BN_APPLY(0, 2); else BN_APPLY(0, 1);
    }
#undef BN_APPLY
  }
  return check_launch("rtdetr_bn_act_fwd");
}

extern "C" int rtdetr_bn_act_fwd(const void* const* x, const float* const* gamma, const float* const* beta,
                                 float* const* run_mean, float* const* run_var, int nb, long long M, int C, int act,
                                 float eps, float momentum, float* saved, float* ws, void* y, hipStream_t stream) {
  return bn_act_fwd_impl(x, gamma, beta, run_mean, run_var, nb, M, C, act, eps, momentum, saved, ws, nullptr, 0,
                         nullptr, y, 0, 0, stream);
}

extern "C" int rtdetr_bn_act_fwd_part(const void* const* x, const float* const* gamma, const float* const* beta,
                                      float* const* run_mean, float* const* run_var, int nb, long long M, int C,
                                      int act, float eps, float momentum, const float* part, int part_blocks,
                                      float* saved, void* y, hipStream_t stream) {
  if (part == nullptr) return fail("bn_act_fwd_part: part is NULL");
  return bn_act_fwd_impl(x, gamma, beta, run_mean, run_var, nb, M, C, act, eps, momentum, saved, nullptr, part,
                         part_blocks, nullptr, y, 0, 0, stream);
}

extern "C" int rtdetr_bn_act_fwd_rows(const void* const* x, const float* const* gamma, const float* const* beta,
                                      float* const* run_mean, float* const* run_var, int nb, long long M, int C,
                                      int act, float eps, float momentum, const float* part, int part_blocks,
                                      float* ws, float* saved, const void* resid, void* y, long long y_hw,
                                      long long y_bstride, hipStream_t stream) {
  return bn_act_fwd_impl(x, gamma, beta, run_mean, run_var, nb, M, C, act, eps, momentum, saved,
                         part ? nullptr : ws, part, part_blocks, resid, y, y_hw, y_bstride, stream);
}

extern "C" int rtdetr_bn_act_bwd_rows(const void* dy, long long dy_hw, long long dy_bstride, const void* const* x,
                                      const float* const* gamma, int nb, long long M, int C, int act,
                                      const float* saved, float* ws, float* coef, void* const* dx, float* dgb,
                                      hipStream_t stream) {
  if (int rc = bn_check(nb, M, C, act)) return rc;
  if (int rc = bn_rows_check(M, dy_hw, dy_bstride)) return rc;
  if (!dy || !x || !gamma || !saved || !ws || !coef || !dx || !dgb) return fail("bn_act_bwd: NULL argument");
  BnArgs a{};
  a.nb = nb;
  a.rhw = dy_hw;
  a.rbs = dy_bstride;
  for (int i = 0; i < nb; ++i) {
    if (!x[i] || !dx[i]) return fail("bn_act_bwd: NULL branch pointer");
    a.x[i] = static_cast<const uint4*>(x[i]);
    a.gamma[i] = gamma[i];
  }
  int nblk, rpb;
  bn_blocks(M, &nblk, &rpb);
  const long long nchunk = M * (C / 8);
  const size_t shm = 3 * 2048 * sizeof(float);
  {
    ProfScope prof(stream, PROF_CONV_EPI, 2.0 * (nb + 1) * M * C);
#define BN_RED(A, N)                                                                                 \
  MOE_LAUNCH(prof, (bn_bwd_reduce_kernel<A, N>), dim3(nblk), dim3(256), shm, stream, a,              \
             static_cast<const uint4*>(dy), saved, M, C, rpb, ws)
    if (act == 1) {
      if (nb == 2) BN_RED(1, 2); else BN_RED(1, 1);
    } else {
      if (nb == 2) BN_RED(0, 2); else BN_RED(0, 1);
    }
#undef BN_RED
  }
  if (nb == 2)
    hipLaunchKernelGGL(bn_bwd_finalize_kernel<2>, dim3(C / 8), dim3(BN_FIN_T), 0, stream, ws, nblk, M, C, saved, coef,
                       dgb);
  else
    hipLaunchKernelGGL(bn_bwd_finalize_kernel<1>, dim3(C / 8), dim3(BN_FIN_T), 0, stream, ws, nblk, M, C, saved, coef,
                       dgb);
  {
    ProfScope prof(stream, PROF_CONV_EPI, 2.0 * (2 * nb + 1) * M * C);
    uint4* d0 = static_cast<uint4*>(dx[0]);
    uint4* d1 = nb > 1 ? static_cast<uint4*>(dx[1]) : nullptr;
#define BN_DX(A, N)                                                                                   \
  MOE_LAUNCH(prof, (bn_bwd_dx_kernel<A, N>), dim3(bn_grid(nchunk)), dim3(256), 0, stream, a,           \
             static_cast<const uint4*>(dy), saved, coef, nchunk, C, d0, d1)
    if (act == 1) {
      if (nb == 2) BN_DX(1, 2); else BN_DX(1, 1);
    } else {
      if (nb == 2) BN_DX(0, 2); else BN_DX(0, 1);
    }
#undef BN_DX
  }
  return check_launch("rtdetr_bn_act_bwd");
}

extern "C" int rtdetr_bn_act_eval(const void* const* x, const float* const* gamma, const float* const* beta,
                                  const float* const* run_mean, const float* const* run_var, int nb, long long M,
                                  int C, int act, float eps, const void* resid, void* y, hipStream_t stream) {
  if (int rc = bn_check(nb, M, C, act)) return rc;
  if (!x || !gamma || !beta || !run_mean || !run_var || !y) return fail("bn_act_eval: NULL argument");
  if (reinterpret_cast<uintptr_t>(resid) % 16 || reinterpret_cast<uintptr_t>(y) % 16)
    return fail("bn_act_eval: y / resid must be 16-B aligned");
  BnArgs a{};
  a.nb = nb;
  a.resid = static_cast<const uint4*>(resid);
  for (int i = 0; i < nb; ++i) {
    if (!x[i] || !gamma[i] || !beta[i] || !run_mean[i] || !run_var[i]) return fail("bn_act_eval: NULL branch pointer");
    if (reinterpret_cast<uintptr_t>(x[i]) % 16) return fail("bn_act_eval: x must be 16-B aligned");
    a.x[i] = static_cast<const uint4*>(x[i]);
    a.gamma[i] = gamma[i];
    a.beta[i] = beta[i];
    a.run_mean[i] = const_cast<float*>(run_mean[i]);  // (read only here)
    a.run_var[i] = const_cast<float*>(run_var[i]);
  }
  const long long nchunk = M * (C / 8);
  const size_t shm = (size_t)nb * 2 * C * sizeof(float);
  ProfScope prof(stream, PROF_CONV_EPI, 2.0 * (nb + 1 + (resid ? 1 : 0)) * M * C);
#define BN_EVAL(A, N)                                                                                  \
  MOE_LAUNCH(prof, (bn_eval_kernel<A, N>), dim3(bn_grid(nchunk)), dim3(256), shm, stream, a, eps, nchunk, C, \
             static_cast<uint4*>(y))
  if (act == 1) {
    if (nb == 2) BN_EVAL(1, 2); else BN_EVAL(1, 1);
  } else {
    if (nb == 2) BN_EVAL(0, 2); else BN_EVAL(0, 1);
  }
#undef BN_EVAL
  return check_launch("rtdetr_bn_act_eval");
}

extern "C" int rtdetr_bn_act_bwd(const void* dy, const void* const* x, const float* const* gamma, int nb,
                                 long long M, int C, int act, const float* saved, float* ws, float* coef,
                                 void* const* dx, float* dgb, hipStream_t stream) {
  return rtdetr_bn_act_bwd_rows(dy, 0, 0, x, gamma, nb, M, C, act, saved, ws, coef, dx, dgb, stream);
}
