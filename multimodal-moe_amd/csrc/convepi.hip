// Fused epilogues of the frozen-BatchNorm convolutions of the RT-DETR backbone
// (the dense body around the MoE path).  With the BatchNorm
// statistics frozen (rtdetrv2_r50vd `freeze_norm`), conv + BN is a convolution
// with per-output-channel scaled weights plus a channel bias; these kernels
// apply that bias together with what follows it in one pass over the NHWC
// (channels_last) activation:
//   bias_act:      y = act(x + bias[c])                  (branch2a / 2b: ReLU)
//   add_bias_relu: y = relu(a + b + bias[c])             (block output: branch2c + shortcut)
// bf16 storage, fp32 arithmetic, one rounding.  Each thread moves 16-B chunks
// (8 channels); C is a multiple of 8, so a chunk never straddles a pixel.
#include "moe_common.h"
#include "prof.h"

namespace moe {

template <int ACT>
__global__ __launch_bounds__(256) void bias_act_kernel(const uint4* __restrict__ x, const float* __restrict__ bias,
                                                       long long nchunk, int cchunks, uint4* __restrict__ y) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nchunk; i += (long long)gridDim.x * 256) {
    const int c0 = (int)(i % cchunks) * 8;
    float v[8];
    unpack8(x[i], v);
    const float4 b0 = *reinterpret_cast<const float4*>(bias + c0);
    const float4 b1 = *reinterpret_cast<const float4*>(bias + c0 + 4);
    v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
    v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
    if constexpr (ACT == 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
    }
    y[i] = pack8(v);
  }
}

__global__ __launch_bounds__(256) void add_bias_relu_kernel(const uint4* __restrict__ a, const uint4* __restrict__ b,
                                                            const float* __restrict__ bias, long long nchunk,
                                                            int cchunks, uint4* __restrict__ y) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nchunk; i += (long long)gridDim.x * 256) {
    const int c0 = (int)(i % cchunks) * 8;
    float va[8], vb[8];
    unpack8(a[i], va);
    unpack8(b[i], vb);
    float bb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (bias != nullptr) {
      const float4 b0 = *reinterpret_cast<const float4*>(bias + c0);
      const float4 b1 = *reinterpret_cast<const float4*>(bias + c0 + 4);
      bb[0] = b0.x; bb[1] = b0.y; bb[2] = b0.z; bb[3] = b0.w;
      bb[4] = b1.x; bb[5] = b1.y; bb[6] = b1.z; bb[7] = b1.w;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) va[j] = fmaxf(va[j] + vb[j] + bb[j], 0.f);
    y[i] = pack8(va);
  }
}

// Backward of a block output y = relu(...) whose activation feeds two
// consumers (the next block's branch2a and its shortcut): the two incoming
// gradients are summed and masked in one pass -- what autograd would do as an
// accumulate (add_) plus a ReLU backward (threshold_backward), two passes
// more over the largest activations of the network.  g2 may be null.
__global__ __launch_bounds__(256) void relu_grad2_kernel(const uint4* __restrict__ g1, const uint4* __restrict__ g2,
                                                         const uint4* __restrict__ y, long long nchunk,
                                                         uint4* __restrict__ out) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nchunk; i += (long long)gridDim.x * 256) {
    float v1[8], v2[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    unpack8(g1[i], v1);
    if (g2 != nullptr) unpack8(g2[i], v2);
    const uint4 yv = y[i];
    const uint32_t yw[4] = {yv.x, yv.y, yv.z, yv.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t h = (yw[j >> 1] >> (16 * (j & 1))) & 0xffffu;
      const bool pos = !(h & 0x8000u) && h != 0;  // bf16 y > 0
      v1[j] = pos ? v1[j] + v2[j] : 0.f;
    }
    out[i] = pack8(v1);
  }
}

// Frozen-BN weight fold for many convolutions in one launch:
//   out_t[r][i] = bf16(float(w_t[r][i]) * scale_t[r])   (r = output channel)
// over a table of tensors (forward: W' = W * s; backward: dW = dW' * s).
struct FoldRec {      // 32 B, mirrored by src/rtdetr_moe/backbone.py
  const uint16_t* w;  // bf16 [rows][inner] (any dense layout with the output channel outermost)
  const float* scale; // fp32 [rows]
  uint16_t* out;      // bf16, same layout as w
  int rows, inner;    // inner = elements per output channel (multiple of 8)
};
static_assert(sizeof(FoldRec) == 32, "FoldRec layout");

__global__ __launch_bounds__(256) void fold_scale_multi_kernel(const FoldRec* __restrict__ recs,
                                                               const int2* __restrict__ chunks) {
  const int2 ch = chunks[blockIdx.x];  // (tensor, chunk of 2048 elements)
  const FoldRec r = recs[ch.x];
  const long long e = (long long)ch.y * 2048 + threadIdx.x * 8;
  const long long n = (long long)r.rows * r.inner;
  if (e >= n) return;
  const float s = r.scale[e / r.inner];  // 8 consecutive elements share a row (inner % 8 == 0)
  float v[8];
  unpack8(*reinterpret_cast<const uint4*>(r.w + e), v);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] *= s;
  *reinterpret_cast<uint4*>(r.out + e) = pack8(v);
}

// The same product for up to 64 tensors whose addresses are only known at
// launch time (the folds' backward, dW_l = dW'_l * scale_l, on gradients
// autograd allocates): the table travels as the kernel argument; tensor q
// owns blocks [base[q], base[q+1]) of 2048 elements each.
constexpr int kFoldBatch = 64;
struct FoldBatch {
  const uint16_t* in[kFoldBatch];
  const float* scale[kFoldBatch];
  uint16_t* out[kFoldBatch];
  int rows[kFoldBatch], inner[kFoldBatch], base[kFoldBatch + 1];
  int n;
};

__global__ __launch_bounds__(256) void fold_scale_batch_kernel(FoldBatch b) {
  int q = 0;
  while (q + 1 < b.n && (int)blockIdx.x >= b.base[q + 1]) ++q;
  const long long e = (long long)(blockIdx.x - b.base[q]) * 2048 + threadIdx.x * 8;
  const long long n = (long long)b.rows[q] * b.inner[q];
  if (e >= n) return;
  const float s = b.scale[q][e / b.inner[q]];
  float v[8];
  unpack8(*reinterpret_cast<const uint4*>(b.in[q] + e), v);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] *= s;
  *reinterpret_cast<uint4*>(b.out[q] + e) = pack8(v);
}

}  // namespace moe

using namespace moe;

static int epi_grid(long long nchunk) {
  // enough waves to fill 256 CUs several times over; grid-stride beyond that
  long long g = (nchunk + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

extern "C" int rtdetr_bias_act_nhwc(const void* x, const float* bias, long long M, int C, int act, void* y,
                                    hipStream_t stream) {
  if (C <= 0 || C % 8 != 0) return fail("bias_act: C must be a positive multiple of 8");
  if (act < 0 || act > 1) return fail("bias_act: act must be 0 (none) or 1 (relu)");
  if (bias == nullptr) return fail("bias_act: bias is required");
  if (M <= 0) return 0;
  const long long nchunk = M * (C / 8);
  ProfScope prof(stream, PROF_CONV_EPI, 4.0 * M * C);
  if (act == 1)
    MOE_LAUNCH(prof, bias_act_kernel<1>, dim3(epi_grid(nchunk)), dim3(256), 0, stream,
               static_cast<const uint4*>(x), bias, nchunk, C / 8, static_cast<uint4*>(y));
  else
    MOE_LAUNCH(prof, bias_act_kernel<0>, dim3(epi_grid(nchunk)), dim3(256), 0, stream,
               static_cast<const uint4*>(x), bias, nchunk, C / 8, static_cast<uint4*>(y));
  return check_launch("rtdetr_bias_act_nhwc");
}

extern "C" int rtdetr_add_bias_relu_nhwc(const void* a, const void* b, const float* bias, long long M, int C,
                                         void* y, hipStream_t stream) {
  if (C <= 0 || C % 8 != 0) return fail("add_bias_relu: C must be a positive multiple of 8");
  if (M <= 0) return 0;
  const long long nchunk = M * (C / 8);
  ProfScope prof(stream, PROF_CONV_EPI, 6.0 * M * C);
  MOE_LAUNCH(prof, add_bias_relu_kernel, dim3(epi_grid(nchunk)), dim3(256), 0, stream,
             static_cast<const uint4*>(a), static_cast<const uint4*>(b), bias, nchunk, C / 8,
             static_cast<uint4*>(y));
  return check_launch("rtdetr_add_bias_relu_nhwc");
}

extern "C" int rtdetr_relu_grad2_nhwc(const void* g1, const void* g2, const void* y, long long M, int C, void* out,
                                      hipStream_t stream) {
  if (C <= 0 || C % 8 != 0) return fail("relu_grad2: C must be a positive multiple of 8");
  if (g1 == nullptr || y == nullptr || out == nullptr) return fail("relu_grad2: g1, y and out are required");
  if (M <= 0) return 0;
  const long long nchunk = M * (C / 8);
  ProfScope prof(stream, PROF_CONV_EPI, (g2 ? 8.0 : 6.0) * M * C);
  MOE_LAUNCH(prof, relu_grad2_kernel, dim3(epi_grid(nchunk)), dim3(256), 0, stream, static_cast<const uint4*>(g1),
             static_cast<const uint4*>(g2), static_cast<const uint4*>(y), nchunk, static_cast<uint4*>(out));
  return check_launch("rtdetr_relu_grad2_nhwc");
}

extern "C" int rtdetr_fold_scale_multi(const void* records, const int32_t* chunks, int n_chunks, hipStream_t stream) {
  if (n_chunks < 0 || (n_chunks > 0 && (records == nullptr || chunks == nullptr)))
    return fail("fold_scale_multi: bad arguments");
  if (n_chunks == 0) return 0;
  ProfScope prof(stream, PROF_CONV_EPI, 4.0 * 2048 * n_chunks);
  MOE_LAUNCH(prof, fold_scale_multi_kernel, dim3(n_chunks), dim3(256), 0, stream,
             static_cast<const FoldRec*>(records), reinterpret_cast<const int2*>(chunks));
  return check_launch("rtdetr_fold_scale_multi");
}

extern "C" int rtdetr_fold_scale_batch(int n, const void* const* in, const float* const* scale, void* const* out,
                                       const int* rows, const int* inner, hipStream_t stream) {
  if (n < 1 || n > kFoldBatch || in == nullptr || scale == nullptr || out == nullptr || rows == nullptr ||
      inner == nullptr)
    return fail("fold_scale_batch: 1..64 tensors, non-NULL arrays");
  FoldBatch b{};
  b.n = n;
  int blocks = 0;
  double bytes = 0.0;
  for (int q = 0; q < n; ++q) {
    if (in[q] == nullptr || scale[q] == nullptr || out[q] == nullptr || rows[q] < 1 || inner[q] < 8 ||
        inner[q] % 8 || (reinterpret_cast<uintptr_t>(in[q]) | reinterpret_cast<uintptr_t>(out[q])) % 16)
      return fail("fold_scale_batch: bad tensor (inner a multiple of 8, 16-B aligned bf16)");
    b.in[q] = static_cast<const uint16_t*>(in[q]);
    b.scale[q] = scale[q];
    b.out[q] = static_cast<uint16_t*>(out[q]);
    b.rows[q] = rows[q];
    b.inner[q] = inner[q];
    b.base[q] = blocks;
    const long long numel = (long long)rows[q] * inner[q];
    blocks += (int)((numel + 2047) / 2048);
    bytes += 4.0 * numel + 4.0 * rows[q];
  }
  b.base[n] = blocks;
  ProfScope prof(stream, PROF_CONV_EPI, bytes);
  MOE_LAUNCH(prof, fold_scale_batch_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, b);
  return check_launch("rtdetr_fold_scale_batch");
}
