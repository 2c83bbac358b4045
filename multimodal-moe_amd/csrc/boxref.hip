// Decoder box refinement of RT-DETR, one launch each way:
//   y = sigmoid(delta + inverse_sigmoid(ref)),
//   inverse_sigmoid(x) = log(max(x', eps) / max(1 - x', eps)), x' = clamp(x, 0, 1)
// forward over [B, Q, 4] per decoder layer; backward returns
//   d delta = (g_boxes + g_inter) y (1 - y)
//   d ref   = g_boxes y (1 - y) d inverse_sigmoid / d ref     (torch's clamp masks)
// -- the refined boxes feed the loss (g_boxes, with a gradient to the incoming
// reference) and the next layer's reference (g_inter, detached from it), as in
// the upstream decoder.  Replaces ~17 element-wise launches forward and ~16
// backward per decoder layer.
#include "moe_common.h"
#include "prof.h"

namespace moe {

__device__ __forceinline__ float box_in(const void* d, int bf16, long long i) {
  return bf16 ? bf2f(static_cast<const uint16_t*>(d)[i]) : static_cast<const float*>(d)[i];
}

__device__ __forceinline__ float inv_sigmoid(float x, float eps) {
  const float xc = fminf(fmaxf(x, 0.f), 1.f);
  return logf(fmaxf(xc, eps) / fmaxf(1.f - xc, eps));
}

__global__ __launch_bounds__(256) void box_refine_fwd_kernel(const void* __restrict__ delta, int delta_bf16,
                                                             const float* __restrict__ ref, long long n, float eps,
                                                             float* __restrict__ y) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float z = box_in(delta, delta_bf16, i) + inv_sigmoid(ref[i], eps);
  y[i] = 1.f / (1.f + expf(-z));
}

__global__ __launch_bounds__(256) void box_refine_bwd_kernel(const float* __restrict__ g_boxes,
                                                             const float* __restrict__ g_inter,
                                                             const float* __restrict__ y,
                                                             const float* __restrict__ ref, long long n, float eps,
                                                             void* __restrict__ g_delta, int delta_bf16,
                                                             float* __restrict__ g_ref) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float yi = y[i];
  const float s = yi * (1.f - yi);
  const float gb = g_boxes ? g_boxes[i] : 0.f;
  const float gi = g_inter ? g_inter[i] : 0.f;
  const float gd = (gb + gi) * s;
  if (delta_bf16) static_cast<uint16_t*>(g_delta)[i] = f2bf(gd);
  else static_cast<float*>(g_delta)[i] = gd;
  if (g_ref != nullptr) {
    const float x = ref[i];
    float d = 0.f;
    if (x >= 0.f && x <= 1.f) {
      const float a = fmaxf(x, eps), b = fmaxf(1.f - x, eps);
      d = (x >= eps ? 1.f / a : 0.f) + ((1.f - x) >= eps ? 1.f / b : 0.f);
    }
    g_ref[i] = gb * s * d;
  }
}

}  // namespace moe

using namespace moe;

extern "C" int rtdetr_box_refine_fwd(const void* delta, int delta_bf16, const float* ref, long long n, float eps,
                                     float* y, hipStream_t stream) {
  if (n < 0 || (n > 0 && (delta == nullptr || ref == nullptr || y == nullptr)))
    return fail("box_refine_fwd: bad arguments");
  if (n == 0) return 0;
  ProfScope prof(stream, PROF_CONV_EPI, (delta_bf16 ? 2.0 : 4.0) * n + 8.0 * n);
  MOE_LAUNCH(prof, box_refine_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, delta, delta_bf16,
             ref, n, eps, y);
  return check_launch("rtdetr_box_refine_fwd");
}

extern "C" int rtdetr_box_refine_bwd(const float* g_boxes, const float* g_inter, const float* y, const float* ref,
                                     long long n, float eps, void* g_delta, int delta_bf16, float* g_ref,
                                     hipStream_t stream) {
  if (n < 0 || (n > 0 && (y == nullptr || ref == nullptr || g_delta == nullptr)))
    return fail("box_refine_bwd: bad arguments");
  if (n == 0) return 0;
  ProfScope prof(stream, PROF_CONV_EPI, 20.0 * n);
  MOE_LAUNCH(prof, box_refine_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, g_boxes, g_inter,
             y, ref, n, eps, g_delta, delta_bf16, g_ref);
  return check_launch("rtdetr_box_refine_bwd");
}
