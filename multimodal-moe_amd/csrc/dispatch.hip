// Token dispatch / combine kernels for gfx950.
//
// Geometry shared by all three: 16 lanes own one token; a lane moves the
// token row in 16-B chunks (chunk = lane + 16 i), so one wave-instruction
// touches four contiguous 256-B row segments; 256-thread blocks, 16 tokens
// per block-iteration, grid-stride over tokens.  All three are HBM-bound
// row movers: permute reads T rows and writes A rows; combine reads A rows
// and writes T rows; combine_bwd reads T + A rows and writes A rows.
#include "moe_common.h"
#include "prof.h"

namespace moe {

__device__ __forceinline__ int assignment_pos(const int32_t* __restrict__ topk_idx,
                                              const int32_t* __restrict__ local_rank,
                                              const int32_t* __restrict__ rank_base,
                                              const int32_t* __restrict__ offsets, int t,
                                              int j, int E, int k, int cap) {
  const int e = topk_idx[(size_t)t * k + j];
  const int blk = t / kRouterBlockTokens;
  const int r = rank_base[((size_t)blk * k + j) * E + e] + local_rank[(size_t)t * k + j];
  return (cap <= 0 || r < cap) ? offsets[e] + r : -1;
}

__global__ __launch_bounds__(256) void permute_fwd_kernel(
    const uint16_t* __restrict__ x, const int32_t* __restrict__ topk_idx,
    const int32_t* __restrict__ local_rank, const int32_t* __restrict__ rank_base,
    const int32_t* __restrict__ offsets, int T, int d, int E, int k, int cap,
    uint16_t* __restrict__ xp, int32_t* __restrict__ pos, int32_t* __restrict__ prof_rows) {
  const int tid = threadIdx.x;
  if (prof_rows != nullptr && blockIdx.x == 0 && tid == 0) *prof_rows = offsets[E];
  const int sub = tid & 15;
  const int nchunk = d >> 7;
  for (int tb = blockIdx.x * 16; tb < T; tb += gridDim.x * 16) {
    const int t = tb + (tid >> 4);
    if (t >= T) continue;
    int pj[8];
    _Pragma("unroll") for (int j = 0; j < 8; ++j) if (j < k) {
      pj[j] = assignment_pos(topk_idx, local_rank, rank_base, offsets, t, j, E, k, cap);
      if (sub == j) pos[(size_t)t * k + j] = pj[j];
    }
    const uint4* src = reinterpret_cast<const uint4*>(x + (size_t)t * d);
    for (int c = 0; c < nchunk; ++c) {
      const int ch = sub + 16 * c;
      const uint4 v = src[ch];
      _Pragma("unroll") for (int j = 0; j < 8; ++j) if (j < k)
        if (pj[j] >= 0) reinterpret_cast<uint4*>(xp + (size_t)pj[j] * d)[ch] = v;
    }
  }
}

// Index half of the dispatch without moving rows: pos[t,j] and the inverse
// map src_tok[pos] = t, which the grouped GEMMs use to gather the token rows
// straight into their LDS tiles (no permuted copy in HBM).  One thread per
// assignment (t, j).
__global__ __launch_bounds__(256) void route_index_kernel(
    const int32_t* __restrict__ topk_idx, const int32_t* __restrict__ local_rank,
    const int32_t* __restrict__ rank_base, const int32_t* __restrict__ offsets, int T, int E, int k, int cap,
    int32_t* __restrict__ pos, int32_t* __restrict__ src_tok, int32_t* __restrict__ prof_rows) {
  const int a = blockIdx.x * 256 + threadIdx.x;
  if (prof_rows != nullptr && a == 0) *prof_rows = offsets[E];
  if (a >= T * k) return;
  const int t = a / k, j = a - t * k;
  const int pj = assignment_pos(topk_idx, local_rank, rank_base, offsets, t, j, E, k, cap);
  pos[a] = pj;
  if (pj >= 0) src_tok[pj] = t;
}

__global__ __launch_bounds__(256) void combine_fwd_kernel(
    const uint16_t* __restrict__ yp, const int32_t* __restrict__ pos,
    const float* __restrict__ topk_w, int T, int d, int k, uint16_t* __restrict__ y,
    const uint16_t* __restrict__ resid) {
  const int tid = threadIdx.x;
  const int sub = tid & 15;
  const int nchunk = d >> 7;
  for (int tb = blockIdx.x * 16; tb < T; tb += gridDim.x * 16) {
    const int t = tb + (tid >> 4);
    if (t >= T) continue;
    int pj[8];
    float wj[8];
    _Pragma("unroll") for (int j = 0; j < 8; ++j) if (j < k) {
      pj[j] = pos[(size_t)t * k + j];
      wj[j] = topk_w[(size_t)t * k + j];
    }
    for (int c = 0; c < nchunk; ++c) {
      const int ch = sub + 16 * c;
      float acc[8];
      if (resid != nullptr) {  // the layer's residual: y = x + sum (one bf16 rounding)
        unpack8(reinterpret_cast<const uint4*>(resid + (size_t)t * d)[ch], acc);
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = 0.f;
      }
      _Pragma("unroll") for (int j = 0; j < 8; ++j) if (j < k) {
        if (pj[j] < 0) continue;
        float v[8];
        unpack8(reinterpret_cast<const uint4*>(yp + (size_t)pj[j] * d)[ch], v);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] += wj[j] * v[i];
      }
      reinterpret_cast<uint4*>(y + (size_t)t * d)[ch] = pack8(acc);
    }
  }
}

__global__ __launch_bounds__(256) void combine_bwd_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ yp,
    const int32_t* __restrict__ pos, const float* __restrict__ topk_w, int T, int d, int k,
    uint16_t* __restrict__ dyp, float* __restrict__ dw) {
  const int tid = threadIdx.x;
  const int sub = tid & 15;
  const int nchunk = d >> 7;
  for (int tb = blockIdx.x * 16; tb < T; tb += gridDim.x * 16) {
    const int t = tb + (tid >> 4);
    const bool valid = t < T;  // keep all 16 lanes of a group in the shuffles
    int pj[8];
    float wj[8], dot[8];
    _Pragma("unroll") for (int j = 0; j < 8; ++j) if (j < k) {
      pj[j] = valid ? pos[(size_t)t * k + j] : -1;
      wj[j] = valid ? topk_w[(size_t)t * k + j] : 0.f;
      dot[j] = 0.f;
    }
    for (int c = 0; c < nchunk; ++c) {
      const int ch = sub + 16 * c;
      float g[8];
      if (valid) {
        unpack8(reinterpret_cast<const uint4*>(dy + (size_t)t * d)[ch], g);
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) g[i] = 0.f;
      }
      _Pragma("unroll") for (int j = 0; j < 8; ++j) if (j < k) {
        if (pj[j] < 0) continue;
        float v[8], o[8];
        unpack8(reinterpret_cast<const uint4*>(yp + (size_t)pj[j] * d)[ch], v);
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          s += g[i] * v[i];
          o[i] = wj[j] * g[i];
        }
        dot[j] += s;
        reinterpret_cast<uint4*>(dyp + (size_t)pj[j] * d)[ch] = pack8(o);
      }
    }
    _Pragma("unroll") for (int j = 0; j < 8; ++j) if (j < k) {
      const float s = group_sum<16>(dot[j]);
      if (valid && sub == 0) dw[(size_t)t * k + j] = s;
    }
  }
}

}  // namespace moe

using namespace moe;

static int rows_grid(int T) {
  int g = (T + 15) / 16;
  return g > 4096 ? 4096 : (g < 1 ? 1 : g);
}

static int check_row_width(int d, const char* who) {
  if (d <= 0 || d % 128 != 0 || d > 4096)
    return fail(std::string(who) + ": d must be a multiple of 128 in [128,4096]");
  return 0;
}

extern "C" int moe_permute_fwd(const void* x, const int32_t* topk_idx,
                               const int32_t* local_rank, const int32_t* rank_base,
                               const int32_t* offsets, int T, int d, int E, int k, int cap,
                               void* xp, int32_t* pos, hipStream_t stream) {
  if (check_row_width(d, "permute")) return -1;
  if (E < 1 || E > 64 || k < 1 || k > 8) return fail("permute: need 1<=E<=64, 1<=k<=8");
  if (T <= 0) return 0;
  // bytes: x read once, idx/local_rank read, pos written, kept rows written
  ProfScope prof(stream, PROF_ROWMOVE, 2.0 * T * d + 12.0 * T * k, true, 2.0 * d);
  MOE_LAUNCH(prof, permute_fwd_kernel, dim3(rows_grid(T)), dim3(256), 0, stream,
                     static_cast<const uint16_t*>(x), topk_idx, local_rank, rank_base,
                     offsets, T, d, E, k, cap, static_cast<uint16_t*>(xp), pos, prof.rows_slot());
  return check_launch("moe_permute_fwd");
}

extern "C" int moe_route_index(const int32_t* topk_idx, const int32_t* local_rank, const int32_t* rank_base,
                               const int32_t* offsets, int T, int E, int k, int cap, int32_t* pos,
                               int32_t* src_tok, hipStream_t stream) {
  if (E < 1 || E > 64 || k < 1 || k > 8) return fail("route_index: need 1<=E<=64, 1<=k<=8");
  if (T <= 0) return 0;
  // bytes: idx / local_rank / rank_base reads and pos writes per assignment, src_tok per kept row
  ProfScope prof(stream, PROF_ROWMOVE, 16.0 * T * k, true, 4.0);
  const long long A = (long long)T * k;
  MOE_LAUNCH(prof, route_index_kernel, dim3((unsigned)((A + 255) / 256)), dim3(256), 0, stream, topk_idx,
             local_rank, rank_base, offsets, T, E, k, cap, pos, src_tok, prof.rows_slot());
  return check_launch("moe_route_index");
}

extern "C" int moe_combine_res_fwd(const void* yp, const int32_t* pos, const float* topk_w, const void* resid,
                                   int T, int d, int k, void* y, hipStream_t stream) {
  if (check_row_width(d, "combine")) return -1;
  if (k < 1 || k > 8) return fail("combine: need 1<=k<=8");
  if (T <= 0) return 0;
  // bytes: T*k expert rows + pos/w (+ the residual rows) read, y written
  ProfScope prof(stream, PROF_ROWMOVE,
                 2.0 * T * d + 2.0 * T * k * d + 8.0 * T * k + (resid != nullptr ? 2.0 * T * d : 0.0));
  MOE_LAUNCH(prof, combine_fwd_kernel, dim3(rows_grid(T)), dim3(256), 0, stream,
                     static_cast<const uint16_t*>(yp), pos, topk_w, T, d, k,
                     static_cast<uint16_t*>(y), static_cast<const uint16_t*>(resid));
  return check_launch("moe_combine_fwd");
}

extern "C" int moe_combine_fwd(const void* yp, const int32_t* pos, const float* topk_w,
                               int T, int d, int k, void* y, hipStream_t stream) {
  return moe_combine_res_fwd(yp, pos, topk_w, nullptr, T, d, k, y, stream);
}

extern "C" int moe_combine_bwd(const void* dy, const void* yp, const int32_t* pos,
                               const float* topk_w, int T, int d, int k, void* dyp, float* dw,
                               hipStream_t stream) {
  if (check_row_width(d, "combine_bwd")) return -1;
  if (k < 1 || k > 8) return fail("combine_bwd: need 1<=k<=8");
  if (T <= 0) return 0;
  // bytes: dy + T*k expert rows + pos/w read, dyp rows + dw written
  ProfScope prof(stream, PROF_ROWMOVE, 2.0 * T * d + 4.0 * T * k * d + 12.0 * T * k);
  MOE_LAUNCH(prof, combine_bwd_kernel, dim3(rows_grid(T)), dim3(256), 0, stream,
                     static_cast<const uint16_t*>(dy), static_cast<const uint16_t*>(yp), pos,
                     topk_w, T, d, k, static_cast<uint16_t*>(dyp), dw);
  return check_launch("moe_combine_bwd");
}

namespace moe {

// ---------------------------------------------------------------------------
// Expert-parallel receive map: rank r received, from source
// w, cnt[w][e] rows for each of its El local experts, held at received row
// (w El + e) S + j, j < cnt[w][e] (the fixed-capacity layout of src/moe/ep.py).
// The local experts' GEMMs read them in compact expert-major order (expert e's
// rows from source 0, then source 1, ...):
//   offsets[e] = sum_{e' < e} sum_w cnt[w][e'],  offsets[El] = the total
//   gather[offsets[e] + sum_{w' < w} cnt[w'][e] + j] = (w El + e) S + j
//   gather[offsets[El] ...] = 0 (every one of the W El S entries is written)
// One workgroup per (w, e) pair (its prefix recomputed from the <= 1024
// counts), so the map is one launch with no host sync; workgroup 0 also
// writes offsets and the overflow of this rank's send histogram,
// sum_e max(hist[e] - S, 0) (assignments the exchange dropped).
__global__ __launch_bounds__(256) void ep_compaction_kernel(const int32_t* __restrict__ cnt,
                                                            const int32_t* __restrict__ hist, int W, int El, int E,
                                                            int S, int32_t* __restrict__ gather,
                                                            int32_t* __restrict__ offsets,
                                                            int32_t* __restrict__ overflow) {
  __shared__ int s_start, s_pad;
  const int b = blockIdx.x, w = b / El, e = b % El;
  if (threadIdx.x == 0) {
    int st = 0, tot = 0;
    for (int ww = 0; ww < W; ++ww)
      for (int ee = 0; ee < El; ++ee) {
        const int c = min(cnt[ww * El + ee], S);
        tot += c;
        if (ee < e || (ee == e && ww < w)) st += c;
      }
    s_start = st;
    // this pair's S - n padding entries of the tail [tot, W El S), in compact
    // pair order: (pairs before it) S - st entries precede them
    s_pad = tot + (e * W + w) * S - st;
  }
  if (b == 0) {
    for (int ee = threadIdx.x; ee <= El; ee += blockDim.x) {
      int o = 0;
      for (int e2 = 0; e2 < ee; ++e2)
        for (int ww = 0; ww < W; ++ww) o += min(cnt[ww * El + e2], S);
      offsets[ee] = o;
    }
    if (overflow != nullptr && threadIdx.x == 0) {
      int ov = 0;
      for (int ee = 0; ee < E; ++ee) ov += max(hist[ee] - S, 0);
      *overflow = ov;
    }
  }
  __syncthreads();
  const int n = min(cnt[b], S), st = s_start;
  const int src0 = b * S;
  for (int j = threadIdx.x; j < n; j += blockDim.x) gather[st + j] = src0 + j;
  // the tail past the received rows points at received row 0 (a valid row for
  // any reader that loads a whole tile's indices): no memset of the map
  for (int j = n + threadIdx.x; j < S; j += blockDim.x) gather[s_pad + (j - n)] = 0;
}

}  // namespace moe

extern "C" int moe_ep_compaction(const int32_t* recv_cnt, const int32_t* hist, int W, int El, int E, int S,
                                 int32_t* gather, int32_t* offsets, int32_t* overflow, hipStream_t stream) {
  if (W < 1 || El < 1 || W * El > 1024 || S < 1 || E < 0) return fail("ep_compaction: need 1 <= W El <= 1024, S >= 1");
  if (recv_cnt == nullptr || gather == nullptr || offsets == nullptr || (overflow != nullptr && hist == nullptr))
    return fail("ep_compaction: NULL pointer");
  ProfScope prof(stream, PROF_SCAN, 4.0 * W * El + 4.0 * (El + 1) + 4.0 * E);
  MOE_LAUNCH(prof, ep_compaction_kernel, dim3(W * El), dim3(256), 0, stream, recv_cnt, hist, W, El, E, S, gather,
             offsets, overflow);
  return check_launch("moe_ep_compaction");
}
