// Shared device helpers for the gfx950 MoE kernels (wave64, bf16 storage).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/moe_hip.h"

// Device-side asserts of the debug build (build_ext.py --debug: -DMOE_DEBUG);
// compiled out otherwise.  A failing assert traps the wave.
#ifdef MOE_DEBUG
#include <cassert>
#define MOE_DASSERT(c) assert(c)
#else
#define MOE_DASSERT(c) ((void)0)
#endif

namespace moe {

extern int g_msda_generic;  // msda.hip: 1 = generic fused MSDA kernels (moe_set_tuning "msda_generic")

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;
// Router block: the tokens of one router workgroup, whose within-block ranks
// come from one wave's ballots (<= 64).  16 tokens: 4x as many workgroups as
// 64-token blocks (the decoder's 2,400 tokens were 38 workgroups, a latency
// chain per workgroup on a mostly idle chip).
constexpr int kRouterBlockTokens = 16;

// ---- bf16 <-> f32 (round-to-nearest-even; NaN kept NaN via the hw cvt) ----
__device__ __forceinline__ float bf2f(uint16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
__device__ __forceinline__ uint16_t f2bf(float f) {
  // v_cvt_pk_bf16_f32 is emitted for the plain cast at -O3 (RNE, NaN-safe).
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

// Unpack 8 bf16 held in a uint4 (16 B) into floats.
__device__ __forceinline__ void unpack8(const uint4 v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack2bf(f[0], f[1]);
  v.y = pack2bf(f[2], f[3]);
  v.z = pack2bf(f[4], f[5]);
  v.w = pack2bf(f[6], f[7]);
  return v;
}

// ---- MXFP8 (OCP e4m3 elements, one E8M0 scale per 32 consecutive elements) ----
// Block scale: the smallest power of two 2^e with amax <= 448 * 2^e (no element
// saturates), found from amax's exponent and mantissa bits (1.75 = 448 / 2^8),
// clamped to the E8M0 range; the stored byte is e + 127.  The oracle
// (oracle/moe_oracle.py: mx_exponent) restates the same integer rule.
typedef int i32x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int mx_exponent(float amax) {
  const uint32_t u = __float_as_uint(amax);
  if (amax == 0.f) return -127;
  int e = (int)((u >> 23) & 0xff) - 127 - 8 + ((u & 0x7fffffu) > 0x600000u ? 1 : 0);
  return e < -127 ? -127 : (e > 127 ? 127 : e);
}
// Four floats already scaled into [-448, 448] -> four e4m3 bytes (RNE, v_cvt_pk_fp8_f32).
__device__ __forceinline__ uint32_t pack4fp8(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (uint32_t)w;
}
// Quantize 8 floats of one 32-element block whose exponent is e: two dwords of e4m3.
__device__ __forceinline__ uint2 mx_pack8(const float* f, int e) {
  uint2 o;
  o.x = pack4fp8(ldexpf(f[0], -e), ldexpf(f[1], -e), ldexpf(f[2], -e), ldexpf(f[3], -e));
  o.y = pack4fp8(ldexpf(f[4], -e), ldexpf(f[5], -e), ldexpf(f[6], -e), ldexpf(f[7], -e));
  return o;
}
// e4m3 byte i (0..3) of w, times 2^e, as a float (exact).
__device__ __forceinline__ float fp8_at(uint32_t w, int i, int e) {
  float v;
  switch (i) {
    case 0: v = __builtin_amdgcn_cvt_f32_fp8((int)w, 0); break;
    case 1: v = __builtin_amdgcn_cvt_f32_fp8((int)w, 1); break;
    case 2: v = __builtin_amdgcn_cvt_f32_fp8((int)w, 2); break;
    default: v = __builtin_amdgcn_cvt_f32_fp8((int)w, 3); break;
  }
  return ldexpf(v, e);
}
// 8 e4m3 bytes of one block with exponent e -> 8 bf16 (exact: 4-bit significands).
__device__ __forceinline__ uint4 mx_unpack8_bf16(uint2 q, int e) {
  uint4 o;
  o.x = (__float_as_uint(fp8_at(q.x, 0, e)) >> 16) | (__float_as_uint(fp8_at(q.x, 1, e)) & 0xffff0000u);
  o.y = (__float_as_uint(fp8_at(q.x, 2, e)) >> 16) | (__float_as_uint(fp8_at(q.x, 3, e)) & 0xffff0000u);
  o.z = (__float_as_uint(fp8_at(q.y, 0, e)) >> 16) | (__float_as_uint(fp8_at(q.y, 1, e)) & 0xffff0000u);
  o.w = (__float_as_uint(fp8_at(q.y, 2, e)) >> 16) | (__float_as_uint(fp8_at(q.y, 3, e)) & 0xffff0000u);
  return o;
}

// Number of set bits of `mask` at lanes below this lane (v_mbcnt).
__device__ __forceinline__ int mbcnt(unsigned long long mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
}

// Butterfly sum over aligned groups of `W` lanes (W power of two <= 64).
template <int W>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <int W>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Cross-lane moves inside a 16-lane DPP row (no LDS round trip, unlike
// __shfl_xor's ds_bpermute).  row_xor<H> reads the lane whose index differs in
// bit H and in every lower bit (xor 2H-1: quad_perm for H <= 2, row_half_mirror
// for H = 4, row_mirror for H = 8).  The four masks 15, 7, 3, 1 are a basis of
// the row's lane-index space, so a butterfly over H = 8, 4, 2, 1 all-reduces
// the row, and stage H pairs every lane with one of the opposite bit H.
template <int H>
__device__ __forceinline__ int row_xor_i(int v) {
  constexpr int ctrl = H == 1 ? 0xB1 : H == 2 ? 0x1B : H == 4 ? 0x141 : 0x140;
  static_assert(H == 1 || H == 2 || H == 4 || H == 8, "row_xor: H in {1,2,4,8}");
  return __builtin_amdgcn_update_dpp(0, v, ctrl, 0xF, 0xF, false);
}
template <int H>
__device__ __forceinline__ float row_xor(float v) {
  return __int_as_float(row_xor_i<H>(__float_as_int(v)));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += row_xor<8>(v);
  v += row_xor<4>(v);
  v += row_xor<2>(v);
  v += row_xor<1>(v);
  return v;
}
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, row_xor<8>(v));
  v = fmaxf(v, row_xor<4>(v));
  v = fmaxf(v, row_xor<2>(v));
  v = fmaxf(v, row_xor<1>(v));
  return v;
}

// MX-quantize one 16-B chunk (8 bf16) held by each lane, where 4 consecutive
// lanes hold one 32-element block: the block amax by a 4-lane butterfly, then
// e4m3 bytes and the block exponent.
__device__ __forceinline__ uint2 mx_quant_chunk(const uint4 v, int& e) {
  float f[8];
  unpack8(v, f);
  float m = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) m = fmaxf(m, fabsf(f[i]));
  m = group_max<4>(m);
  e = mx_exponent(m);
  return mx_pack8(f, e);
}

}  // namespace moe

// ---- error reporting (thread-local, see moe_last_error) ----
namespace moe {
void set_error(const std::string& msg);
int fail(const std::string& msg);          // returns -1
int check_launch(const char* what);        // returns 0 or -(1000 + err)

// Raise a kernel's dynamic-LDS limit once per device (the attribute is
// per-device state in HIP).  Returns 0, or fail() with the HIP error when the
// attribute cannot be set.  `done` is the kernel's own per-device bitmask.
inline int allow_dyn_lds(const void* fn, int bytes, unsigned long long* done, const char* what) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return fail(std::string(what) + ": no device");
  const unsigned long long bit = 1ull << dev;
  if (__atomic_load_n(done, __ATOMIC_ACQUIRE) & bit) return 0;
  const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e != hipSuccess) return fail(std::string(what) + ": hipFuncSetAttribute failed: " + hipGetErrorString(e));
  __atomic_fetch_or(done, bit, __ATOMIC_RELEASE);
  return 0;
}
}  // namespace moe
