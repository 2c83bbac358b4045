// Multi-head self-attention of the RT-DETR encoder (AIFI, 920 tokens per
// image at 1280x736) and decoder (300 queries) layers, head dim 32, on the
// bf16 MFMA -- replaces torch's scaled_dot_product_attention (which on ROCm
// dispatches Triton-generated AOTriton kernels).  Called by
// src/rtdetr_moe/linear.py::TokenSelfAttention (the reference's engine runs
// nn.MultiheadAttention inside RTDETR.train, src/models/vision/rtdetr.py:82-94).
//
// Operands are read in place from the projection outputs: q, k, v rows of
// token t of image b and head h start at ptr + (b L + t) ld + 32 h (so the
// fused [q | k] projection and the v projection need no head transposes), and
// o / dq / dk / dv are written the same way.  Softmax in base 2: scores are
// scaled by scale*log2(e); lse holds m + log2(l) of each query row.
//
// All three kernels use v_mfma_f32_16x16x32_bf16 with K = 32 = the head dim
// (one instruction per 16x16 score block) and keep every per-row softmax
// quantity on ONE lane: the score block is computed transposed (A = the
// 16-row key/value tile, B = the 16 query rows), so lane l owns query l & 15
// and keys 4 (l >> 4) + i of each 16-key block; the next product takes those
// scores as its B operand with a lane-local key permutation (chunk c of 32
// keys: fragment element j <-> key 32c + 16 (j >> 2) + 4 (l >> 4) + (j & 3)),
// matched by the transposed LDS image of the other operand.
//   attn_fwd_kernel      workgroup = 64 queries of one (b, h), 4 waves x 16;
//                        K / V^T tiles of 64 keys double-buffered in LDS
//                        (register prefetch, one barrier per tile); online
//                        softmax; O^T accumulated per lane.
//   attn_bwd_dq_kernel   same shape: recomputes P, dP = dO V^T and
//                        dS = P (dP - delta), dQ = scale dS K; writes
//                        delta = rowsum(dO * O) for the next kernel.
//   attn_bwd_dkdv_kernel workgroup = 64 keys, 4 waves x 16, key on the lane:
//                        S, dP over query tiles of 64, dV = P^T dO,
//                        dK = scale dS^T Q.
// No atomics: dQ and dK/dV are each summed inside one workgroup in a fixed
// order, so the backward is bitwise repeatable (the split costs recomputing S
// and dP once more than an atomic dQ would).
#include "moe_common.h"
#include "prof.h"

namespace moe {

constexpr int AT_D = 32;           // head dim
constexpr int AT_T = 64;           // tile rows (queries or keys)
constexpr int AT_RP = 40;          // row-major tile pitch in bf16 (80 B: conflict-free 16-B fragment reads)
constexpr int AT_TP = 72;          // transposed tile pitch in bf16 (144 B)

struct AttnPtrs {
  const uint16_t* q;
  const uint16_t* k;
  const uint16_t* v;
  long long ldq, ldk, ldv;
};

__device__ __forceinline__ uint4 ld16(const uint16_t* base, long long row, long long ld, int col, bool ok) {
  if (!ok) return make_uint4(0, 0, 0, 0);
  return *reinterpret_cast<const uint4*>(base + row * ld + col);
}

// row-major tile [64][AT_RP]: thread (r = tid >> 2, c = tid & 3) stores its 16-B chunk
__device__ __forceinline__ void st_rows(uint16_t* t, int tid, uint4 v) {
  *reinterpret_cast<uint4*>(t + (tid >> 2) * AT_RP + (tid & 3) * 8) = v;
}
// transposed tile [32][AT_TP]: element (row r, col 8c + e) -> t[(8c + e) * AT_TP + r]
__device__ __forceinline__ void st_trans(uint16_t* t, int tid, uint4 v) {
  const int r = tid >> 2, c = tid & 3;
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    t[(8 * c + 2 * e) * AT_TP + r] = (uint16_t)(w[e] & 0xffffu);
    t[(8 * c + 2 * e + 1) * AT_TP + r] = (uint16_t)(w[e] >> 16);
  }
}
// A/B fragment of 16 rows x 32 (K): lane l reads row r0 + (l & 15), elements 8 (l >> 4) ... + 7
__device__ __forceinline__ bf16x8 frag_rows(const uint16_t* t, int r0, int lane) {
  return *reinterpret_cast<const bf16x8*>(t + (r0 + (lane & 15)) * AT_RP + 8 * (lane >> 4));
}
// permuted-K fragment from a transposed tile: lane l, row d = d0 + (l & 15), chunk c of
// 32 columns: columns 32c + 4g + 0..3 then 32c + 16 + 4g + 0..3 (g = l >> 4)
__device__ __forceinline__ bf16x8 frag_trans(const uint16_t* t, int d0, int c, int lane) {
  const uint16_t* p = t + (d0 + (lane & 15)) * AT_TP + 32 * c + 4 * (lane >> 4);
  const bf16x4 a = *reinterpret_cast<const bf16x4*>(p);
  const bf16x4 b = *reinterpret_cast<const bf16x4*>(p + 16);
  bf16x8 r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}
// the lane-local B operand of chunk c from two 16-key score blocks
__device__ __forceinline__ bf16x8 pack_pair(const f32x4& a, const f32x4& b) {
  bf16x8 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    r[i] = (short)f2bf(a[i]);
    r[4 + i] = (short)f2bf(b[i]);
  }
  return r;
}
__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float xor_max16_32(float v) {
  v = fmaxf(v, __shfl_xor(v, 16, 64));
  return fmaxf(v, __shfl_xor(v, 32, 64));
}
__device__ __forceinline__ float xor_sum16_32(float v) {
  v += __shfl_xor(v, 16, 64);
  return v + __shfl_xor(v, 32, 64);
}
// store 4 consecutive fp32 of one row as bf16 (8 B)
__device__ __forceinline__ void st4(uint16_t* p, const f32x4& v, float s) {
  uint2 w;
  w.x = pack2bf(v[0] * s, v[1] * s);
  w.y = pack2bf(v[2] * s, v[3] * s);
  *reinterpret_cast<uint2*>(p) = w;
}

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnPtrs a, uint16_t* __restrict__ o, long long ldo,
                                                       float* __restrict__ lse, int H, int L, float sl2) {
  __shared__ __attribute__((aligned(16))) uint16_t ks[2][AT_T * AT_RP];
  __shared__ __attribute__((aligned(16))) uint16_t vt[2][AT_D * AT_TP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const long long base = (long long)b * L;
  const int q = blockIdx.x * AT_T + wave * 16 + (lane & 15);
  const bf16x8 qf = __builtin_bit_cast(bf16x8, ld16(a.q + h * AT_D, base + q, a.ldq, 8 * g, q < L));
  const int lr = tid >> 2, lc = (tid & 3) * 8;  // this thread's row / column of a tile load
  const int nt = (L + AT_T - 1) / AT_T;
  uint4 kreg = ld16(a.k + h * AT_D, base + lr, a.ldk, lc, lr < L);
  uint4 vreg = ld16(a.v + h * AT_D, base + lr, a.ldv, lc, lr < L);
  st_rows(ks[0], tid, kreg);
  st_trans(vt[0], tid, vreg);
  __syncthreads();
  f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  float m_run = -INFINITY, l_run = 0.f;
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    const int k0 = t * AT_T;
    if (t + 1 < nt) {  // next tile in flight during this tile's math
      const int r = k0 + AT_T + lr;
      kreg = ld16(a.k + h * AT_D, base + r, a.ldk, lc, r < L);
      vreg = ld16(a.v + h * AT_D, base + r, a.ldv, lc, r < L);
    }
    f32x4 s[4];
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int m = 0; m < 4; ++m) s[m] = mfma(frag_rows(ks[cur], 16 * m, lane), qf, z);
    float mx = -INFINITY;
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = k0 + 16 * m + 4 * g + i;
        s[m][i] = key < L ? s[m][i] * sl2 : -INFINITY;
        mx = fmaxf(mx, s[m][i]);
      }
    mx = xor_max16_32(mx);
    const float m_new = fmaxf(m_run, mx);
    const float alpha = exp2f(m_run - m_new);
    float ps = 0.f;
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s[m][i] = exp2f(s[m][i] - m_new);
        ps += s[m][i];
      }
    l_run = l_run * alpha + ps;
    m_run = m_new;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) acc[hf] *= alpha;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const bf16x8 pf = pack_pair(s[2 * c], s[2 * c + 1]);
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) acc[hf] = mfma(frag_trans(vt[cur], 16 * hf, c, lane), pf, acc[hf]);
    }
    if (t + 1 < nt) {
      st_rows(ks[cur ^ 1], tid, kreg);
      st_trans(vt[cur ^ 1], tid, vreg);
    }
    __syncthreads();
  }
  const float l_tot = xor_sum16_32(l_run);
  if (q < L) {
    const float inv = 1.f / l_tot;
    uint16_t* op = o + (base + q) * ldo + h * AT_D + 4 * g;
    st4(op, acc[0], inv);
    st4(op + 16, acc[1], inv);
    if (g == 0) lse[(long long)bh * L + q] = m_run + log2f(l_tot);
  }
}

// ---------------------------------------------------------------------------
// backward: dQ (and delta)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(AttnPtrs a, const uint16_t* __restrict__ o, long long ldo,
                                                          const uint16_t* __restrict__ dout, long long lddo,
                                                          const float* __restrict__ lse, float* __restrict__ delta,
                                                          uint16_t* __restrict__ dq, long long lddq, int H, int L,
                                                          float sl2, float scale) {
  __shared__ __attribute__((aligned(16))) uint16_t ks[2][AT_T * AT_RP];
  __shared__ __attribute__((aligned(16))) uint16_t vs[2][AT_T * AT_RP];
  __shared__ __attribute__((aligned(16))) uint16_t kt[2][AT_D * AT_TP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const long long base = (long long)b * L;
  const int q = blockIdx.x * AT_T + wave * 16 + (lane & 15);
  const bool qok = q < L;
  const bf16x8 qf = __builtin_bit_cast(bf16x8, ld16(a.q + h * AT_D, base + q, a.ldq, 8 * g, qok));
  const uint4 dor = ld16(dout + h * AT_D, base + q, lddo, 8 * g, qok);
  const uint4 orr = ld16(o + h * AT_D, base + q, ldo, 8 * g, qok);
  const bf16x8 dof = __builtin_bit_cast(bf16x8, dor);
  float dl = 0.f;
  {
    float x[8], y[8];
    unpack8(dor, x);
    unpack8(orr, y);
#pragma unroll
    for (int i = 0; i < 8; ++i) dl += x[i] * y[i];
  }
  dl = xor_sum16_32(dl);
  const float lq = qok ? lse[(long long)bh * L + q] : INFINITY;
  if (qok && g == 0) delta[(long long)bh * L + q] = dl;
  const int lr = tid >> 2, lc = (tid & 3) * 8;
  const int nt = (L + AT_T - 1) / AT_T;
  uint4 kreg = ld16(a.k + h * AT_D, base + lr, a.ldk, lc, lr < L);
  uint4 vreg = ld16(a.v + h * AT_D, base + lr, a.ldv, lc, lr < L);
  st_rows(ks[0], tid, kreg);
  st_trans(kt[0], tid, kreg);
  st_rows(vs[0], tid, vreg);
  __syncthreads();
  f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    const int k0 = t * AT_T;
    if (t + 1 < nt) {
      const int r = k0 + AT_T + lr;
      kreg = ld16(a.k + h * AT_D, base + r, a.ldk, lc, r < L);
      vreg = ld16(a.v + h * AT_D, base + r, a.ldv, lc, r < L);
    }
    f32x4 s[4], dp[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      s[m] = mfma(frag_rows(ks[cur], 16 * m, lane), qf, z);
      dp[m] = mfma(frag_rows(vs[cur], 16 * m, lane), dof, z);
    }
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = k0 + 16 * m + 4 * g + i;
        const float p = key < L ? exp2f(s[m][i] * sl2 - lq) : 0.f;
        s[m][i] = p * (dp[m][i] - dl);  // dS
      }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const bf16x8 df = pack_pair(s[2 * c], s[2 * c + 1]);
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) acc[hf] = mfma(frag_trans(kt[cur], 16 * hf, c, lane), df, acc[hf]);
    }
    if (t + 1 < nt) {
      st_rows(ks[cur ^ 1], tid, kreg);
      st_trans(kt[cur ^ 1], tid, kreg);
      st_rows(vs[cur ^ 1], tid, vreg);
    }
    __syncthreads();
  }
  if (qok) {
    uint16_t* p = dq + (base + q) * lddq + h * AT_D + 4 * g;
    st4(p, acc[0], scale);
    st4(p + 16, acc[1], scale);
  }
}

// ---------------------------------------------------------------------------
// backward: dK, dV (key on the lane)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void attn_bwd_dkdv_kernel(AttnPtrs a, const uint16_t* __restrict__ dout,
                                                            long long lddo, const float* __restrict__ lse,
                                                            const float* __restrict__ delta,
                                                            uint16_t* __restrict__ dk, long long lddk,
                                                            uint16_t* __restrict__ dv, long long lddv, int H, int L,
                                                            float sl2, float scale) {
  __shared__ __attribute__((aligned(16))) uint16_t qs[2][AT_T * AT_RP];
  __shared__ __attribute__((aligned(16))) uint16_t dos[2][AT_T * AT_RP];
  __shared__ __attribute__((aligned(16))) uint16_t qt[2][AT_D * AT_TP];
  __shared__ __attribute__((aligned(16))) uint16_t dot_[2][AT_D * AT_TP];
  __shared__ float lses[2][AT_T], dels[2][AT_T];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const long long base = (long long)b * L;
  const int key = blockIdx.x * AT_T + wave * 16 + (lane & 15);
  const bool kok = key < L;
  const bf16x8 kf = __builtin_bit_cast(bf16x8, ld16(a.k + h * AT_D, base + key, a.ldk, 8 * g, kok));
  const bf16x8 vf = __builtin_bit_cast(bf16x8, ld16(a.v + h * AT_D, base + key, a.ldv, 8 * g, kok));
  const int lr = tid >> 2, lc = (tid & 3) * 8;
  const int nt = (L + AT_T - 1) / AT_T;
  const float* lse_bh = lse + (long long)bh * L;
  const float* del_bh = delta + (long long)bh * L;
  uint4 qreg = ld16(a.q + h * AT_D, base + lr, a.ldq, lc, lr < L);
  uint4 dreg = ld16(dout + h * AT_D, base + lr, lddo, lc, lr < L);
  float lreg = 0.f, ereg = 0.f;
  if (tid < AT_T) {
    lreg = tid < L ? lse_bh[tid] : INFINITY;
    ereg = tid < L ? del_bh[tid] : 0.f;
  }
  st_rows(qs[0], tid, qreg);
  st_trans(qt[0], tid, qreg);
  st_rows(dos[0], tid, dreg);
  st_trans(dot_[0], tid, dreg);
  if (tid < AT_T) {
    lses[0][tid] = lreg;
    dels[0][tid] = ereg;
  }
  __syncthreads();
  f32x4 adk[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  f32x4 adv[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    const int q0 = t * AT_T;
    if (t + 1 < nt) {
      const int r = q0 + AT_T + lr;
      qreg = ld16(a.q + h * AT_D, base + r, a.ldq, lc, r < L);
      dreg = ld16(dout + h * AT_D, base + r, lddo, lc, r < L);
      if (tid < AT_T) {
        const int qq = q0 + AT_T + tid;
        lreg = qq < L ? lse_bh[qq] : INFINITY;
        ereg = qq < L ? del_bh[qq] : 0.f;
      }
    }
    f32x4 s[4], dp[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      s[n] = mfma(frag_rows(qs[cur], 16 * n, lane), kf, z);    // S[q = 16n + 4g + i][key]
      dp[n] = mfma(frag_rows(dos[cur], 16 * n, lane), vf, z);  // dP[q][key]
    }
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 16 * n + 4 * g + i;
        const float p = exp2f(s[n][i] * sl2 - lses[cur][r]);  // 0 for padding queries (lse = +inf)
        s[n][i] = p;
        dp[n][i] = p * (dp[n][i] - dels[cur][r]);             // dS
      }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const bf16x8 pf = pack_pair(s[2 * c], s[2 * c + 1]);
      const bf16x8 df = pack_pair(dp[2 * c], dp[2 * c + 1]);
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        adv[hf] = mfma(frag_trans(dot_[cur], 16 * hf, c, lane), pf, adv[hf]);
        adk[hf] = mfma(frag_trans(qt[cur], 16 * hf, c, lane), df, adk[hf]);
      }
    }
    if (t + 1 < nt) {
      st_rows(qs[cur ^ 1], tid, qreg);
      st_trans(qt[cur ^ 1], tid, qreg);
      st_rows(dos[cur ^ 1], tid, dreg);
      st_trans(dot_[cur ^ 1], tid, dreg);
      if (tid < AT_T) {
        lses[cur ^ 1][tid] = lreg;
        dels[cur ^ 1][tid] = ereg;
      }
    }
    __syncthreads();
  }
  if (kok) {
    uint16_t* pk = dk + (base + key) * lddk + h * AT_D + 4 * g;
    uint16_t* pv = dv + (base + key) * lddv + h * AT_D + 4 * g;
    st4(pk, adk[0], scale);
    st4(pk + 16, adk[1], scale);
    st4(pv, adv[0], 1.f);
    st4(pv + 16, adv[1], 1.f);
  }
}

static int attn_check(const void* const* ptrs, int np, const long long* lds, int nl, int B, int H, int L,
                      int head_dim, const char* what) {
  if (head_dim != AT_D) return fail(std::string(what) + ": head_dim must be 32");
  if (B < 0 || H <= 0 || L < 0) return fail(std::string(what) + ": bad B / H / L");
  for (int i = 0; i < np; ++i)
    if (ptrs[i] == nullptr || reinterpret_cast<uintptr_t>(ptrs[i]) % 16)
      return fail(std::string(what) + ": operands must be non-NULL and 16-B aligned");
  for (int i = 0; i < nl; ++i)
    if (lds[i] < (long long)H * AT_D || lds[i] % 8)
      return fail(std::string(what) + ": row strides must be multiples of 8 elements and >= H * 32");
  if ((long long)L * H > (1ll << 30)) return fail(std::string(what) + ": too many rows");
  return 0;
}

}  // namespace moe

using namespace moe;

extern "C" int rtdetr_attn_fwd(const void* q, long long ldq, const void* k, long long ldk, const void* v,
                               long long ldv, void* o, long long ldo, float* lse, int B, int H, int L, int head_dim,
                               float scale, hipStream_t stream) {
  const void* ptrs[5] = {q, k, v, o, lse};
  const long long lds[4] = {ldq, ldk, ldv, ldo};
  if (int rc = attn_check(ptrs, 5, lds, 4, B, H, L, head_dim, "rtdetr_attn_fwd")) return rc;
  if (B == 0 || L == 0) return 0;
  const double n = (double)B * H * L;
  ProfScope prof(stream, PROF_ATTN, n * AT_D * 2 * 4 + 4 * n, false, 0.0, 4.0 * n * L * AT_D);
  AttnPtrs a{static_cast<const uint16_t*>(q), static_cast<const uint16_t*>(k), static_cast<const uint16_t*>(v),
             ldq, ldk, ldv};
  const float sl2 = scale * 1.4426950408889634f;
  MOE_LAUNCH(prof, attn_fwd_kernel, dim3((L + AT_T - 1) / AT_T, B * H), dim3(256), 0, stream, a,
             static_cast<uint16_t*>(o), ldo, lse, H, L, sl2);
  return check_launch("rtdetr_attn_fwd");
}

extern "C" int rtdetr_attn_bwd(const void* q, long long ldq, const void* k, long long ldk, const void* v,
                               long long ldv, const void* o, long long ldo, const void* dout, long long lddo,
                               const float* lse, float* delta, void* dq, long long lddq, void* dk, long long lddk,
                               void* dv, long long lddv, int B, int H, int L, int head_dim, float scale,
                               hipStream_t stream) {
  const void* ptrs[11] = {q, k, v, o, dout, lse, delta, dq, dk, dv, q};
  const long long lds[8] = {ldq, ldk, ldv, ldo, lddo, lddq, lddk, lddv};
  if (int rc = attn_check(ptrs, 10, lds, 8, B, H, L, head_dim, "rtdetr_attn_bwd")) return rc;
  if (B == 0 || L == 0) return 0;
  AttnPtrs a{static_cast<const uint16_t*>(q), static_cast<const uint16_t*>(k), static_cast<const uint16_t*>(v),
             ldq, ldk, ldv};
  const float sl2 = scale * 1.4426950408889634f;
  const double n = (double)B * H * L;
  const dim3 grid((L + AT_T - 1) / AT_T, B * H);
  {
    // reads q, k, v, o, dO, lse; writes dq, delta; S, dP, dQ: 3 products
    ProfScope prof(stream, PROF_ATTN, n * AT_D * 2 * 6 + 8 * n, false, 0.0, 6.0 * n * L * AT_D);
    MOE_LAUNCH(prof, attn_bwd_dq_kernel, grid, dim3(256), 0, stream, a, static_cast<const uint16_t*>(o), ldo,
               static_cast<const uint16_t*>(dout), lddo, lse, delta, static_cast<uint16_t*>(dq), lddq, H, L, sl2,
               scale);
    if (int rc = check_launch("rtdetr_attn_bwd (dq)")) return rc;
  }
  // reads q, k, v, dO, lse, delta; writes dk, dv; S, dP, dV, dK: 4 products
  ProfScope prof(stream, PROF_ATTN, n * AT_D * 2 * 6 + 8 * n, false, 0.0, 8.0 * n * L * AT_D);
  MOE_LAUNCH(prof, attn_bwd_dkdv_kernel, grid, dim3(256), 0, stream, a, static_cast<const uint16_t*>(dout), lddo,
             lse, delta, static_cast<uint16_t*>(dk), lddk, static_cast<uint16_t*>(dv), lddv, H, L, sl2, scale);
  return check_launch("rtdetr_attn_bwd (dk, dv)");
}
