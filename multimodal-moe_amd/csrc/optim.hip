// Flat mixed-precision AdamW for the training step (bench/TrainStep; the
// reference's optimizer is Ultralytics' AdamW inside RTDETR.train,
// SURVEY.md 3.1 -- same update rule, torch.optim.AdamW semantics).
//
// One pass over every trainable parameter, read where autograd left the
// gradients (a device table of {grad pointer, dtype, numel, flat offset,
// bf16 weight pointer, lr group}), three launches per step in place of
// ~400 (per-tensor bf16->fp32 grad casts, foreach norm + scale for the
// gradient clip, the fused AdamW, fp32->bf16 weight casts):
//   train_grad_sqnorm       per-chunk sum of squares of the gradients
//   train_grad_norm_finalize one block: total norm (fixed order), clip scale
//   train_adamw_step        g *= scale; decoupled weight decay; moments;
//                           fp32 master update; bf16 weight written back
// Masters, exp_avg and exp_avg_sq are flat fp32 buffers (each tensor's
// segment starts at a multiple of 8 elements, so chunk interiors are
// 16-B/32-B vector accesses).  HBM-bound: ~28 B per parameter per step.
#include "moe_common.h"
#include "prof.h"

namespace moe {

struct OptTensor {        // 48 B, mirrored by src/rtdetr_moe/optim.py
  const void* grad;       // bf16 or fp32 [numel]
  uint16_t* lowp;         // bf16 weight to refresh, or nullptr (fp32 weight = the master itself)
  long long numel;
  long long moff;         // offset of the tensor in the flat master / moment buffers (multiple of 8)
  int gdtype;             // 0 bf16, 1 fp32, 2 no gradient this step (tensor skipped, as torch.optim does)
  int group;              // lr group
  float* hi_out;          // fp32 weight to write (a sharded master's parameter), or nullptr
};
static_assert(sizeof(OptTensor) == 48, "OptTensor layout");

constexpr int OPT_CHUNK = 2048;  // elements per workgroup (256 threads x 8)
constexpr int OPT_MAX_GROUPS = 4;

struct AdamArgs {
  float lr[OPT_MAX_GROUPS];
  float wd, beta1, beta2, eps;
};

__device__ __forceinline__ void load_grad8(const OptTensor& t, long long e, bool full, float (&g)[8]) {
  if (t.gdtype == 0) {
    const uint16_t* gp = static_cast<const uint16_t*>(t.grad) + e;
    if (full) {
      unpack8(*reinterpret_cast<const uint4*>(gp), g);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) g[i] = (e + i < t.numel) ? bf2f(gp[i]) : 0.f;
    }
  } else {
    const float* gp = static_cast<const float*>(t.grad) + e;
    if (full) {
      const float4 a = *reinterpret_cast<const float4*>(gp), b = *reinterpret_cast<const float4*>(gp + 4);
      g[0] = a.x; g[1] = a.y; g[2] = a.z; g[3] = a.w; g[4] = b.x; g[5] = b.y; g[6] = b.z; g[7] = b.w;
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) g[i] = (e + i < t.numel) ? gp[i] : 0.f;
    }
  }
}

// Data-parallel gradient staging: every tensor's gradient (bf16 or fp32; a
// tensor without one contributes zeros) widened to fp32 into one flat buffer
// at the record's offset, so the ranks' sum is ONE fp32 all-reduce (no bf16
// rounding per ring hop) and the optimizer reads the reduced sums in place.
__global__ __launch_bounds__(256) void grad_pack_kernel(const OptTensor* __restrict__ tens,
                                                        const int2* __restrict__ chunks, float* __restrict__ flat) {
  const int2 ch = chunks[blockIdx.x];
  const OptTensor t = tens[ch.x];
  const long long e = (long long)ch.y * OPT_CHUNK + threadIdx.x * 8;
  if (e >= t.numel) return;
  const bool full = e + 8 <= t.numel;
  float g[8];
  if (t.gdtype == 2) {
#pragma unroll
    for (int i = 0; i < 8; ++i) g[i] = 0.f;
  } else {
    load_grad8(t, e, full, g);
  }
  float* dst = flat + t.moff + e;
  if (full) {
    reinterpret_cast<float4*>(dst)[0] = make_float4(g[0], g[1], g[2], g[3]);
    reinterpret_cast<float4*>(dst)[1] = make_float4(g[4], g[5], g[6], g[7]);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (e + i < t.numel) dst[i] = g[i];
  }
}

__global__ __launch_bounds__(256) void grad_sqnorm_kernel(const OptTensor* __restrict__ tens,
                                                          const int2* __restrict__ chunks,
                                                          float* __restrict__ partials) {
  __shared__ float red[4];
  const int2 ch = chunks[blockIdx.x];
  const OptTensor t = tens[ch.x];
  const long long e = (long long)ch.y * OPT_CHUNK + threadIdx.x * 8;
  float s = 0.f;
  if (e < t.numel && t.gdtype != 2) {
    float g[8];
    // a vector load needs the 8 elements inside the tensor and a 16-B/32-B
    // aligned address (grad allocations are 256-B aligned; e is a multiple of 8)
    load_grad8(t, e, e + 8 <= t.numel, g);
#pragma unroll
    for (int i = 0; i < 8; ++i) s += g[i] * g[i];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partials[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// coef[0] = total gradient norm (of the rank-mean gradient), coef[1] = the
// scale applied to the stored gradient: inv_world * min(1, max_norm / (norm + 1e-6))
// (torch.nn.utils.clip_grad_norm_); max_norm <= 0: no clipping.  Also counts
// the step of every tensor that has a gradient (torch.optim keeps one step
// count per parameter; a skipped tensor's bias corrections do not advance).
__global__ __launch_bounds__(1024) void grad_norm_finalize_kernel(const float* __restrict__ partials, int n,
                                                                  float max_norm, float inv_world,
                                                                  float* __restrict__ coef,
                                                                  const OptTensor* __restrict__ tens, int n_tensors,
                                                                  int32_t* __restrict__ tsteps) {
  __shared__ float red[16];
  for (int i = threadIdx.x; i < n_tensors; i += 1024)
    if (tens[i].gdtype != 2) tsteps[i] += 1;
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 1024) s += partials[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float tot = 0.f;
    for (int w = 0; w < 16; ++w) tot += red[w];
    const float norm = sqrtf(tot) * inv_world;
    float clip = 1.f;
    if (max_norm > 0.f) clip = fminf(1.f, max_norm / (norm + 1e-6f));
    coef[0] = norm;
    coef[1] = clip * inv_world;
  }
}

__global__ __launch_bounds__(256) void adamw_step_kernel(const OptTensor* __restrict__ tens,
                                                         const int2* __restrict__ chunks,
                                                         const float* __restrict__ coef,
                                                         float* __restrict__ master, float* __restrict__ exp_avg,
                                                         float* __restrict__ exp_avg_sq,
                                                         const int32_t* __restrict__ tsteps, AdamArgs a) {
  const int2 ch = chunks[blockIdx.x];
  const OptTensor t = tens[ch.x];
  const long long e = (long long)ch.y * OPT_CHUNK + threadIdx.x * 8;
  if (e >= t.numel || t.gdtype == 2) return;
  const bool full = e + 8 <= t.numel;
  const float scale = coef[1];
  const float lr = a.lr[t.group];
  const float decay = 1.f - lr * a.wd;
  // bias corrections of this tensor's step count, in double like torch's host math
  const int ts = tsteps[ch.x];
  const float bc1 = (float)(1.0 - pow((double)a.beta1, ts));
  const float bc2_sqrt = (float)sqrt(1.0 - pow((double)a.beta2, ts));
  const float step = lr / bc1;
  float g[8];
  load_grad8(t, e, full, g);
  float* mp = master + t.moff + e;
  float* m1 = exp_avg + t.moff + e;
  float* m2 = exp_avg_sq + t.moff + e;
  float p[8], v1[8], v2[8];
  if (full) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float4 x = reinterpret_cast<const float4*>(mp)[h];
      const float4 y = reinterpret_cast<const float4*>(m1)[h];
      const float4 z = reinterpret_cast<const float4*>(m2)[h];
      p[4 * h] = x.x; p[4 * h + 1] = x.y; p[4 * h + 2] = x.z; p[4 * h + 3] = x.w;
      v1[4 * h] = y.x; v1[4 * h + 1] = y.y; v1[4 * h + 2] = y.z; v1[4 * h + 3] = y.w;
      v2[4 * h] = z.x; v2[4 * h + 1] = z.y; v2[4 * h + 2] = z.z; v2[4 * h + 3] = z.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const bool ok = e + i < t.numel;
      p[i] = ok ? mp[i] : 0.f;
      v1[i] = ok ? m1[i] : 0.f;
      v2[i] = ok ? m2[i] : 0.f;
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float gi = g[i] * scale;
    p[i] *= decay;
    v1[i] = a.beta1 * v1[i] + (1.f - a.beta1) * gi;
    v2[i] = a.beta2 * v2[i] + (1.f - a.beta2) * gi * gi;
    const float denom = sqrtf(v2[i]) / bc2_sqrt + a.eps;
    p[i] -= step * v1[i] / denom;
  }
  if (full) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      reinterpret_cast<float4*>(mp)[h] = make_float4(p[4 * h], p[4 * h + 1], p[4 * h + 2], p[4 * h + 3]);
      reinterpret_cast<float4*>(m1)[h] = make_float4(v1[4 * h], v1[4 * h + 1], v1[4 * h + 2], v1[4 * h + 3]);
      reinterpret_cast<float4*>(m2)[h] = make_float4(v2[4 * h], v2[4 * h + 1], v2[4 * h + 2], v2[4 * h + 3]);
    }
    if (t.lowp != nullptr) {
      uint4 o;
      o.x = pack2bf(p[0], p[1]);
      o.y = pack2bf(p[2], p[3]);
      o.z = pack2bf(p[4], p[5]);
      o.w = pack2bf(p[6], p[7]);
      *reinterpret_cast<uint4*>(t.lowp + e) = o;
    }
    if (t.hi_out != nullptr) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
        reinterpret_cast<float4*>(t.hi_out + e)[h] = make_float4(p[4 * h], p[4 * h + 1], p[4 * h + 2], p[4 * h + 3]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (e + i < t.numel) {
        mp[i] = p[i];
        m1[i] = v1[i];
        m2[i] = v2[i];
        if (t.lowp != nullptr) t.lowp[e + i] = f2bf(p[i]);
        if (t.hi_out != nullptr) t.hi_out[e + i] = p[i];
      }
    }
  }
}

}  // namespace moe

using namespace moe;

extern "C" int train_grad_sqnorm(const void* tensors, const int32_t* chunks, int n_chunks, float* partials,
                                 hipStream_t stream) {
  if (n_chunks < 0 || (n_chunks > 0 && (tensors == nullptr || chunks == nullptr || partials == nullptr)))
    return fail("train_grad_sqnorm: bad arguments");
  if (n_chunks == 0) return 0;
  ProfScope prof(stream, PROF_OPTIM, 4.0 * n_chunks);
  MOE_LAUNCH(prof, grad_sqnorm_kernel, dim3(n_chunks), dim3(256), 0, stream,
             static_cast<const OptTensor*>(tensors), reinterpret_cast<const int2*>(chunks), partials);
  return check_launch("train_grad_sqnorm");
}

extern "C" int train_grad_pack(const void* tensors, const int32_t* chunks, int n_chunks, float* flat,
                               hipStream_t stream) {
  if (n_chunks < 0 || (n_chunks > 0 && (tensors == nullptr || chunks == nullptr || flat == nullptr)))
    return fail("train_grad_pack: bad arguments");
  if (reinterpret_cast<uintptr_t>(flat) % 16) return fail("train_grad_pack: flat buffer must be 16-B aligned");
  if (n_chunks == 0) return 0;
  // bytes: <= 4 read + 4 written per element
  ProfScope prof(stream, PROF_OPTIM, 8.0 * OPT_CHUNK * n_chunks);
  MOE_LAUNCH(prof, grad_pack_kernel, dim3(n_chunks), dim3(256), 0, stream, static_cast<const OptTensor*>(tensors),
             reinterpret_cast<const int2*>(chunks), flat);
  return check_launch("train_grad_pack");
}

extern "C" int train_grad_norm_finalize(const float* partials, int n, float max_norm, float inv_world, float* coef,
                                        const void* tensors, int n_tensors, int32_t* tensor_steps,
                                        hipStream_t stream) {
  if (n < 0 || coef == nullptr || (n > 0 && partials == nullptr)) return fail("train_grad_norm_finalize: bad arguments");
  if (n_tensors < 0 || (n_tensors > 0 && (tensors == nullptr || tensor_steps == nullptr)))
    return fail("train_grad_norm_finalize: bad tensor table");
  ProfScope prof(stream, PROF_OPTIM, 4.0 * n + 8.0 + 56.0 * n_tensors);
  MOE_LAUNCH(prof, grad_norm_finalize_kernel, dim3(1), dim3(1024), 0, stream, partials, n, max_norm, inv_world, coef,
             static_cast<const OptTensor*>(tensors), n_tensors, tensor_steps);
  return check_launch("train_grad_norm_finalize");
}

extern "C" int train_adamw_step(const void* tensors, const int32_t* chunks, int n_chunks, const float* coef,
                                float* master, float* exp_avg, float* exp_avg_sq, const int32_t* tensor_steps,
                                const float* lrs, int n_groups, float weight_decay, float beta1, float beta2,
                                float eps, hipStream_t stream) {
  if (n_groups < 1 || n_groups > OPT_MAX_GROUPS || lrs == nullptr) return fail("train_adamw_step: 1..4 lr groups");
  if (n_chunks < 0 || coef == nullptr || master == nullptr || exp_avg == nullptr || exp_avg_sq == nullptr)
    return fail("train_adamw_step: bad arguments");
  if (tensor_steps == nullptr) return fail("train_adamw_step: tensor_steps is NULL");
  if (n_chunks == 0) return 0;
  AdamArgs a{};
  for (int i = 0; i < n_groups; ++i) a.lr[i] = lrs[i];
  a.wd = weight_decay;
  a.beta1 = beta1;
  a.beta2 = beta2;
  a.eps = eps;
  // bytes: per element grad (<= 4) + master/m/v read and written (24) + bf16 weight (<= 2)
  ProfScope prof(stream, PROF_OPTIM, 30.0 * OPT_CHUNK * n_chunks);
  MOE_LAUNCH(prof, adamw_step_kernel, dim3(n_chunks), dim3(256), 0, stream, static_cast<const OptTensor*>(tensors),
             reinterpret_cast<const int2*>(chunks), coef, master, exp_avg, exp_avg_sq, tensor_steps, a);
  return check_launch("train_adamw_step");
}
