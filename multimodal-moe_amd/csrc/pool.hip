// ResNet-D shortcut downsampling of the RT-DETR backbone:
// AvgPool2d(2, 2) over channels_last (NHWC) bf16 activations with even H, W.
//   forward : y[b, i, j, c] = RNE(0.25 * sum of the 2x2 window, fp32)
//   backward: gx[b, 2i+di, 2j+dj, c] = RNE(0.25 * gy[b, i, j, c])
// One thread per 8-channel (16-B) vector of an output pixel.  Replaces the
// reshape-mean forward (torch reduce kernel) and its broadcast-multiply
// backward (~1.8 TB/s on the stage-2 shortcut, 120 M elements).
#include "moe_common.h"
#include "prof.h"

namespace moe {

__global__ __launch_bounds__(256) void avgpool2x2_fwd_kernel(const uint16_t* __restrict__ x, int H, int W, int C8,
                                                             long long n, uint16_t* __restrict__ y) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int W2 = W >> 1, H2 = H >> 1;
  const int cv = (int)(i % C8);
  long long p = i / C8;
  const int ow = (int)(p % W2);
  p /= W2;
  const int oh = (int)(p % H2);
  const long long b = p / H2;
  const uint4* xr = reinterpret_cast<const uint4*>(x);
  const long long row0 = ((b * H + 2 * oh) * W + 2 * ow) * C8 + cv;
  const long long row1 = row0 + (long long)W * C8;
  const uint4 a = xr[row0], bq = xr[row0 + C8], c = xr[row1], d = xr[row1 + C8];
  float va[8], vb[8], vc[8], vd[8], o[8];
  unpack8(a, va);
  unpack8(bq, vb);
  unpack8(c, vc);
  unpack8(d, vd);
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] = (((va[k] + vb[k]) + vc[k]) + vd[k]) * 0.25f;
  reinterpret_cast<uint4*>(y)[i] = pack8(o);
}

__global__ __launch_bounds__(256) void avgpool2x2_bwd_kernel(const uint16_t* __restrict__ gy,
                                                             const uint16_t* __restrict__ add, int H, int W, int C8,
                                                             long long n, uint16_t* __restrict__ gx) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int W2 = W >> 1, H2 = H >> 1;
  const int cv = (int)(i % C8);
  long long p = i / C8;
  const int ow = (int)(p % W2);
  p /= W2;
  const int oh = (int)(p % H2);
  const long long b = p / H2;
  float v[8];
  unpack8(reinterpret_cast<const uint4*>(gy)[i], v);
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] *= 0.25f;
  uint4* xr = reinterpret_cast<uint4*>(gx);
  const long long row0 = ((b * H + 2 * oh) * W + 2 * ow) * C8 + cv;
  const long long row1 = row0 + (long long)W * C8;
  if (add == nullptr) {
    const uint4 q = pack8(v);
    xr[row0] = q;
    xr[row0 + C8] = q;
    xr[row1] = q;
    xr[row1 + C8] = q;
    return;
  }
  // gx = (gy / 4 upsampled) + add: the quarter rounded to bf16 first, as the
  // separate pool backward + add would, then the fp32 sum rounded once
  const uint4 q = pack8(v);
  float qv[8];
  unpack8(q, qv);
  const uint4* ar = reinterpret_cast<const uint4*>(add);
  const long long rows[4] = {row0, row0 + C8, row1, row1 + C8};
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float a[8];
    unpack8(ar[rows[r]], a);
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] += qv[k];
    xr[rows[r]] = pack8(a);
  }
}

// Stem max pool (MaxPool2d(3, 2, 1), forward only: the stem is frozen, so
// nothing upstream takes a gradient):  y[b, i, j, c] = max over the in-bounds
// taps x[b, 2i-1+dy, 2j-1+dx, c], dy, dx in 0..2 (padding never wins; NaN
// propagates).  One thread per 8-channel vector of an output pixel; the three
// input rows a thread reads are shared with its neighbours through L2.
// Replaces torch's max_pool_forward_nhwc (157 us at 8 x 64 x 368 x 640).
__device__ __forceinline__ float max_nan(float m, float v) { return (v > m || v != v) ? v : m; }

__global__ __launch_bounds__(256) void maxpool3x3s2_fwd_kernel(const uint16_t* __restrict__ x, int H, int W, int Ho,
                                                               int Wo, int C8, long long n,
                                                               uint16_t* __restrict__ y) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int cv = (int)(i % C8);
  long long p = i / C8;
  const int ow = (int)(p % Wo);
  p /= Wo;
  const int oh = (int)(p % Ho);
  const long long b = p / Ho;
  const uint4* xr = reinterpret_cast<const uint4*>(x);
  float m[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) m[c] = -INFINITY;
#pragma unroll
  for (int dy = 0; dy < 3; ++dy) {
    const int ih = 2 * oh - 1 + dy;
    if (ih < 0 || ih >= H) continue;
    uint4 v[3];
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const int iw = 2 * ow - 1 + dx;
      v[dx] = (iw >= 0 && iw < W) ? xr[((b * H + ih) * W + iw) * C8 + cv] : make_uint4(0xff80ff80u, 0xff80ff80u,
                                                                                         0xff80ff80u, 0xff80ff80u);
    }
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      float f[8];
      unpack8(v[dx], f);
#pragma unroll
      for (int c = 0; c < 8; ++c) m[c] = max_nan(m[c], f[c]);
    }
  }
  uint32_t o[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) o[c] = (uint32_t)f2bf(m[2 * c]) | ((uint32_t)f2bf(m[2 * c + 1]) << 16);
  reinterpret_cast<uint4*>(y)[i] = make_uint4(o[0], o[1], o[2], o[3]);
}

// Encoder FPN top-down step: cat([nearest-upsample x2 of
// high, low], channels) over channels_last bf16 in one pass, and its
// transpose.  out [B, H, W, Ch + Cl]:  out[.., :Ch] = high[b, y/2, x/2, :]
// (2 Hh >= H, 2 Wh >= W: the crop of an odd-sized level), out[.., Ch:] = low.
// Backward: dhigh[b, i, j] = sum of g over the in-range 2x2 block (fp32, one
// rounding), dlow = g[.., Ch:] as a dense tensor -- one launch, i < n1 the
// high role, else the low role.  Replaces F.interpolate + torch.cat and their
// backward (upsample_nearest2d_backward + the slice copies).
__global__ __launch_bounds__(256) void upcat_fwd_kernel(const uint4* __restrict__ high, const uint4* __restrict__ low,
                                                        int H, int W, int Hh, int Wh, int Ch8, int Cl8, long long n,
                                                        uint4* __restrict__ out) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int C8 = Ch8 + Cl8;
  const int cv = (int)(i % C8);
  const long long p = i / C8;  // b * H * W + y * W + x
  if (cv < Ch8) {
    const int x = (int)(p % W);
    const long long q = p / W;
    const int y = (int)(q % H);
    const long long b = q / H;
    out[i] = high[((b * Hh + (y >> 1)) * Wh + (x >> 1)) * Ch8 + cv];
  } else {
    out[i] = low[p * Cl8 + (cv - Ch8)];
  }
}

__global__ __launch_bounds__(256) void upcat_bwd_kernel(const uint4* __restrict__ g, int H, int W, int Hh, int Wh,
                                                        int Ch8, int Cl8, long long n1, long long n,
                                                        uint4* __restrict__ dhigh, uint4* __restrict__ dlow) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int C8 = Ch8 + Cl8;
  if (i < n1) {
    const int cv = (int)(i % Ch8);
    long long p = i / Ch8;
    const int j = (int)(p % Wh);
    p /= Wh;
    const int r = (int)(p % Hh);
    const long long b = p / Hh;
    float acc[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] = 0.f;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const int y = 2 * r + dy, x = 2 * j + dx;
        if (y < H && x < W) {
          float f[8];
          unpack8(g[((b * H + y) * W + x) * C8 + cv], f);
#pragma unroll
          for (int c = 0; c < 8; ++c) acc[c] += f[c];
        }
      }
    dhigh[i] = pack8(acc);
  } else {
    const long long k = i - n1;
    const int cv = (int)(k % Cl8);
    const long long p = k / Cl8;
    dlow[k] = g[p * C8 + Ch8 + cv];
  }
}

}  // namespace moe

using namespace moe;

static int upcat_args_ok(const void* a, const void* b, const void* c, int B, int H, int W, int Hh, int Wh, int Ch,
                         int Cl) {
  if (a == nullptr || b == nullptr || c == nullptr || B < 0 || H <= 0 || W <= 0 || Hh <= 0 || Wh <= 0) return 0;
  if ((Ch & 7) || (Cl & 7) || Ch <= 0 || Cl <= 0) return 0;
  if (2 * Hh < H || 2 * Wh < W || Hh > H || Wh > W) return 0;
  for (const void* q : {a, b, c})
    if (reinterpret_cast<uintptr_t>(q) & 15) return 0;
  return 1;
}

extern "C" int rtdetr_upcat_nhwc_fwd(const void* high, const void* low, int B, int H, int W, int Hh, int Wh, int Ch,
                                     int Cl, void* out, hipStream_t stream) {
  if (!upcat_args_ok(high, low, out, B, H, W, Hh, Wh, Ch, Cl))
    return fail("upcat_fwd: need Ch, Cl % 8 == 0, H/2 <= Hh <= H (same for W), 16-B aligned pointers");
  const long long n = (long long)B * H * W * ((Ch + Cl) / 8);
  if (n == 0) return 0;
  ProfScope prof(stream, PROF_CONV_EPI, 2.0 * B * ((double)Hh * Wh * Ch + 2.0 * H * W * Cl + (double)H * W * Ch));
  MOE_LAUNCH(prof, upcat_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
             static_cast<const uint4*>(high), static_cast<const uint4*>(low), H, W, Hh, Wh, Ch / 8, Cl / 8, n,
             static_cast<uint4*>(out));
  return check_launch("rtdetr_upcat_nhwc_fwd");
}

extern "C" int rtdetr_upcat_nhwc_bwd(const void* g, int B, int H, int W, int Hh, int Wh, int Ch, int Cl, void* dhigh,
                                     void* dlow, hipStream_t stream) {
  if (!upcat_args_ok(g, dhigh, dlow, B, H, W, Hh, Wh, Ch, Cl))
    return fail("upcat_bwd: need Ch, Cl % 8 == 0, H/2 <= Hh <= H (same for W), 16-B aligned pointers");
  const long long n1 = (long long)B * Hh * Wh * (Ch / 8);
  const long long n = n1 + (long long)B * H * W * (Cl / 8);
  if (n == 0) return 0;
  ProfScope prof(stream, PROF_CONV_EPI, 2.0 * B * ((double)H * W * (Ch + 2.0 * Cl) + (double)Hh * Wh * Ch));
  MOE_LAUNCH(prof, upcat_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
             static_cast<const uint4*>(g), H, W, Hh, Wh, Ch / 8, Cl / 8, n1, n, static_cast<uint4*>(dhigh),
             static_cast<uint4*>(dlow));
  return check_launch("rtdetr_upcat_nhwc_bwd");
}

extern "C" int rtdetr_maxpool3x3s2_nhwc_fwd(const void* x, int B, int H, int W, int C, void* y, hipStream_t stream) {
  if (x == nullptr || y == nullptr || B < 0 || H <= 0 || W <= 0 || (C & 7) || C <= 0 ||
      (reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(y) & 15))
    return fail("maxpool3x3s2_fwd: need C % 8 == 0 and 16-B aligned x, y");
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const long long n = (long long)B * Ho * Wo * (C / 8);
  if (n == 0) return 0;
  ProfScope prof(stream, PROF_CONV_EPI, 2.0 * B * C * ((double)H * W + (double)Ho * Wo));
  MOE_LAUNCH(prof, maxpool3x3s2_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
             static_cast<const uint16_t*>(x), H, W, Ho, Wo, C / 8, n, static_cast<uint16_t*>(y));
  return check_launch("rtdetr_maxpool3x3s2_nhwc_fwd");
}

static int pool_args_ok(const void* a, const void* b, int B, int H, int W, int C) {
  if (a == nullptr || b == nullptr || B < 0 || H <= 0 || W <= 0 || C <= 0) return 0;
  if ((H & 1) || (W & 1) || (C & 7)) return 0;
  if ((reinterpret_cast<uintptr_t>(a) & 15) || (reinterpret_cast<uintptr_t>(b) & 15)) return 0;
  return 1;
}

extern "C" int rtdetr_avgpool2x2_nhwc_fwd(const void* x, int B, int H, int W, int C, void* y, hipStream_t stream) {
  if (!pool_args_ok(x, y, B, H, W, C)) return fail("avgpool2x2_fwd: need even H, W, C % 8 == 0, 16-B aligned");
  const long long n = (long long)B * (H / 2) * (W / 2) * (C / 8);
  if (n == 0) return 0;
  ProfScope prof(stream, PROF_CONV_EPI, 2.0 * B * H * W * C * 1.25);
  MOE_LAUNCH(prof, avgpool2x2_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
             static_cast<const uint16_t*>(x), H, W, C / 8, n, static_cast<uint16_t*>(y));
  return check_launch("rtdetr_avgpool2x2_nhwc_fwd");
}

extern "C" int rtdetr_avgpool2x2_nhwc_bwd_add(const void* gy, const void* add, int B, int H, int W, int C, void* gx,
                                              hipStream_t stream) {
  if (!pool_args_ok(gy, gx, B, H, W, C) || reinterpret_cast<uintptr_t>(add) % 16)
    return fail("avgpool2x2_bwd: need even H, W, C % 8 == 0, 16-B aligned");
  const long long n = (long long)B * (H / 2) * (W / 2) * (C / 8);
  if (n == 0) return 0;
  ProfScope prof(stream, PROF_CONV_EPI, 2.0 * B * H * W * C * (add ? 2.25 : 1.25));
  MOE_LAUNCH(prof, avgpool2x2_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
             static_cast<const uint16_t*>(gy), static_cast<const uint16_t*>(add), H, W, C / 8, n,
             static_cast<uint16_t*>(gx));
  return check_launch("rtdetr_avgpool2x2_nhwc_bwd");
}

extern "C" int rtdetr_avgpool2x2_nhwc_bwd(const void* gy, int B, int H, int W, int C, void* gx, hipStream_t stream) {
  return rtdetr_avgpool2x2_nhwc_bwd_add(gy, nullptr, B, H, W, C, gx, stream);
}
