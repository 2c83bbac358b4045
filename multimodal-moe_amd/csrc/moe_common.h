// Shared device helpers for the gfx950 MoE kernels (wave64, bf16 storage).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/moe_hip.h"

namespace moe {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;
constexpr int kRouterBlockTokens = 64;  // one wave's ballot covers one block

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

}  // namespace moe

// ---- error reporting (thread-local, see moe_last_error) ----
namespace moe {
void set_error(const std::string& msg);
int fail(const std::string& msg);          // returns -1
int check_launch(const char* what);        // returns 0 or -(1000 + err)
}  // namespace moe
