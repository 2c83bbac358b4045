// MXFP8 producers for the fp8 expert path (SURVEY 8a rows a4/a5 at config C5):
// row quantizer (expert weights, tests) and the fp8 variant of the token
// permute, which quantizes each token row once and writes it to each of its
// expert destinations (256-B rows + 8 scale bytes at d = 256, half the bf16
// dispatch bytes).
//
// Format: OCP e4m3 elements, one E8M0 exponent byte per 32 consecutive
// elements of a row (block exponent rule in moe_common.h: mx_exponent).
// Geometry as the bf16 row movers (dispatch.hip): 16 lanes per row, lane owns
// 16-B chunks (8 bf16) `sub + 16 c`, so 4 consecutive lanes hold one 32-element
// block and its amax is a 4-lane butterfly.
#include "moe_common.h"
#include "prof.h"

namespace moe {

__global__ __launch_bounds__(256) void quantize_mx_kernel(const uint16_t* __restrict__ x, long long R, int K,
                                                          uint8_t* __restrict__ q, uint8_t* __restrict__ s) {
  const int tid = threadIdx.x;
  const int sub = tid & 15;
  const int nchunk = K >> 7;  // 16-lane passes over a row
  for (long long rb = (long long)blockIdx.x * 16; rb < R; rb += (long long)gridDim.x * 16) {
    const long long r = rb + (tid >> 4);
    if (r >= R) continue;  // whole 16-lane group leaves together
    const uint4* src = reinterpret_cast<const uint4*>(x + r * K);
    for (int c = 0; c < nchunk; ++c) {
      const int ch = sub + 16 * c;
      int e;
      const uint2 o = mx_quant_chunk(src[ch], e);
      reinterpret_cast<uint2*>(q + r * K)[ch] = o;
      if ((ch & 3) == 0) s[r * (K / 32) + (ch >> 2)] = (uint8_t)(e + 127);
    }
  }
}

__global__ __launch_bounds__(256) void permute_fwd_mx_kernel(
    const uint16_t* __restrict__ x, const int32_t* __restrict__ topk_idx,
    const int32_t* __restrict__ local_rank, const int32_t* __restrict__ rank_base,
    const int32_t* __restrict__ offsets, int T, int d, int E, int k, int cap,
    uint8_t* __restrict__ xq, uint8_t* __restrict__ xs, int32_t* __restrict__ pos,
    int32_t* __restrict__ prof_rows) {
  const int tid = threadIdx.x;
  if (prof_rows != nullptr && blockIdx.x == 0 && tid == 0) *prof_rows = offsets[E];
  const int sub = tid & 15;
  const int nchunk = d >> 7;
  const int sb = d / 32;
  for (int tb = blockIdx.x * 16; tb < T; tb += gridDim.x * 16) {
    const int t = tb + (tid >> 4);
    if (t >= T) continue;
    int pj[8];
    _Pragma("unroll") for (int j = 0; j < 8; ++j) if (j < k) {
      const int e = topk_idx[(size_t)t * k + j];
      const int blk = t / kRouterBlockTokens;
      const int r = rank_base[((size_t)blk * k + j) * E + e] + local_rank[(size_t)t * k + j];
      pj[j] = (cap <= 0 || r < cap) ? offsets[e] + r : -1;
      if (sub == j) pos[(size_t)t * k + j] = pj[j];
    }
    const uint4* src = reinterpret_cast<const uint4*>(x + (size_t)t * d);
    for (int c = 0; c < nchunk; ++c) {
      const int ch = sub + 16 * c;
      int e;
      const uint2 o = mx_quant_chunk(src[ch], e);
      _Pragma("unroll") for (int j = 0; j < 8; ++j) if (j < k) {
        if (pj[j] < 0) continue;
        reinterpret_cast<uint2*>(xq + (size_t)pj[j] * d)[ch] = o;
        if ((ch & 3) == 0) xs[(size_t)pj[j] * sb + (ch >> 2)] = (uint8_t)(e + 127);
      }
    }
  }
}

}  // namespace moe

using namespace moe;

static int mx_grid(long long R) {
  long long g = (R + 15) / 16;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

extern "C" int moe_quantize_mx(const void* x, long long R, int K, void* q, void* scales, hipStream_t stream) {
  if (K <= 0 || K % 128 != 0 || K > 8192) return fail("quantize_mx: K must be a multiple of 128 in [128, 8192]");
  if (R < 0) return fail("quantize_mx: R < 0");
  if (R == 0) return 0;
  // bytes: bf16 read, e4m3 + one scale byte per 32 written
  ProfScope prof(stream, PROF_QUANT, (double)R * K * (2.0 + 1.0 + 1.0 / 32.0));
  MOE_LAUNCH(prof, quantize_mx_kernel, dim3(mx_grid(R)), dim3(256), 0, stream, static_cast<const uint16_t*>(x), R,
             K, static_cast<uint8_t*>(q), static_cast<uint8_t*>(scales));
  return check_launch("moe_quantize_mx");
}

extern "C" int moe_permute_fwd_mx(const void* x, const int32_t* topk_idx, const int32_t* local_rank,
                                  const int32_t* rank_base, const int32_t* offsets, int T, int d, int E, int k,
                                  int cap, void* xq, void* xs, int32_t* pos, hipStream_t stream) {
  if (d <= 0 || d % 128 != 0 || d > 4096) return fail("permute_mx: d must be a multiple of 128 in [128,4096]");
  if (E < 1 || E > 64 || k < 1 || k > 8) return fail("permute_mx: need 1<=E<=64, 1<=k<=8");
  if (T <= 0) return 0;
  // bytes: x read once, idx/local_rank read, pos written; per kept row d e4m3 + d/32 scales
  ProfScope prof(stream, PROF_ROWMOVE, 2.0 * T * d + 12.0 * T * k, true, d + d / 32.0);
  MOE_LAUNCH(prof, permute_fwd_mx_kernel, dim3(mx_grid(T)), dim3(256), 0, stream, static_cast<const uint16_t*>(x),
             topk_idx, local_rank, rank_base, offsets, T, d, E, k, cap, static_cast<uint8_t*>(xq),
             static_cast<uint8_t*>(xs), pos, prof.rows_slot());
  return check_launch("moe_permute_fwd_mx");
}
