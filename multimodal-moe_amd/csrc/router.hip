// Router kernels for gfx950.
//
//  router_topk_fwd : logits = x.Wg^T + ctx_bias[ctx(t)], fp32 softmax, top-k
//                    (ties -> lower expert id), gates, per-block routing
//                    counts + within-block ranks (wave ballot), aux partials.
//                    One block = kRouterBlockTokens (16) tokens, 4 waves (1
//                    for E > 32);
//                    16 lanes per token, each lane owning d/16 channels read as
//                    16-B chunks (a token row is read by 16 lanes, 4 tokens per
//                    wave-instruction).
//  route_scan      : one workgroup; each (slot, expert) column split into
//                    1024/(k*E) block segments (coalesced row reads), segment
//                    sums -> exclusive prefixes, then hist / kept offsets
//                    (capacity) / slot-major rank bases.
//  token_bwd       : per token: gather-sum of dXp rows (dispatch transpose,
//                    no atomics), gate + softmax + z-loss backward, and the
//                    router's dx term dlogits.Wg, fused.
#include <algorithm>
#include <cmath>

#include "moe_common.h"
#include "prof.h"

namespace moe {

// ---------------------------------------------------------------------------
// router forward
// ---------------------------------------------------------------------------
// Reduce-scatter stage H of the router's 16-lane expert ownership: position
// e0 (bit H and all higher in-row bits clear) ends holding the pair sum for
// expert e0 | (sub & H).
template <int H, int EP>
__device__ __forceinline__ void rs_stage(float (&v)[EP], int sub) {
  const bool hi = (sub & H) != 0;
#pragma unroll
  for (int e0 = 0; e0 < EP; ++e0) {
    if ((e0 & (16 - 2 * H)) != 0 || (e0 & H) != 0) continue;
    const float keep = hi ? v[e0 | H] : v[e0];
    const float send = hi ? v[e0] : v[e0 | H];
    v[e0] = keep + row_xor<H>(send);
  }
}
// Arg-max stage H: larger logit wins, ties -> lower expert id.
template <int H>
__device__ __forceinline__ void argmax_stage(float& bv, int& best) {
  const float ov = row_xor<H>(bv);
  const int oi = row_xor_i<H>(best);
  if (ov > bv || (ov == bv && oi < best)) { bv = ov; best = oi; }
}

template <int EMAX, int NW, int TPB>
__global__ __launch_bounds__(NW * 64) void router_topk_fwd_kernel(
    const uint16_t* __restrict__ x, const float* __restrict__ wg,
    const float* __restrict__ ctx_bias, const int32_t* __restrict__ ctx_img, int n_ctx,
    int tpi, int T, int d, int E, int k, int normalize,
    int32_t* __restrict__ topk_idx, float* __restrict__ topk_w,
    float* __restrict__ probs_out, float* __restrict__ lse_out,
    int32_t* __restrict__ local_rank, int32_t* __restrict__ block_counts,
    float* __restrict__ aux_partials) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_wg = reinterpret_cast<float*>(smem);               // [E][d]
  int32_t* s_idx = reinterpret_cast<int32_t*>(s_wg + E * d);  // [TPB][8]
  float* s_aux = reinterpret_cast<float*>(s_idx + TPB * 8);   // [NW][EMAX+1]
  float* s_cb = s_aux + NW * (EMAX + 1);                       // [n_ctx][E] the context-bias table

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int sub = lane & 15;   // lane within the token group
  const int grp = lane >> 4;   // token group within the wave (0..3)
  const int blk = blockIdx.x;

  // One token per 16-lane group, 4 per wave per iteration; NW waves cover the
  // block's TPB tokens in TPB/(4 NW) iterations.  Every global load of the
  // workgroup -- the token rows (up to PF 16-B chunks per lane; d=256 is fully
  // covered), Wg, the whole [n_ctx][E] context-bias table and each token's
  // context id -- is independent of the others and issued up front: one
  // memory round trip before the token loop (the per-token bias row is then
  // an LDS lookup, and the loop issues no global loads: on gfx9 vmcnt also
  // counts the loop's stores).
  constexpr int NT = NW * 64;
  constexpr int ITERS = TPB / (4 * NW);
  static_assert(ITERS >= 1 && ITERS * 4 * NW == TPB, "TPB must be a multiple of 4 NW");
  constexpr int PF = 2;
  const int nchunk = d >> 7;  // 16-B chunks per lane (d / 8 / 16)
  const bool has_ctx = ctx_bias != nullptr && ctx_img != nullptr;
  uint4 xpre[ITERS][PF];
  int cid[ITERS];
#pragma unroll
  for (int it = 0; it < ITERS; ++it) {
    const int t = blk * TPB + it * NW * 4 + wave * 4 + grp;
    const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)t * d);
#pragma unroll
    for (int c = 0; c < PF; ++c)
      xpre[it][c] = (t < T && c < nchunk) ? xr[sub + 16 * c] : make_uint4(0u, 0u, 0u, 0u);
    cid[it] = (has_ctx && t < T) ? ctx_img[t / tpi] : 0;
  }
  // Wg (fp32 [E][d]) and the context-bias table into LDS, 16 B / 4 B per thread-iteration
  {
    const int n4 = (E * d) >> 2;
    const float4* src = reinterpret_cast<const float4*>(wg);
    float4* dst = reinterpret_cast<float4*>(s_wg);
    for (int i = tid; i < n4; i += NT) dst[i] = src[i];
  }
  if (has_ctx)
    for (int i = tid; i < n_ctx * E; i += NT) s_cb[i] = ctx_bias[i];
  for (int i = tid; i < TPB * 8; i += NT) s_idx[i] = -1;
  __syncthreads();

  // Expert ownership inside a 16-lane token group: lane `sub` owns experts
  // e = 16 q + sub (q < Q).  The partial dot products are reduce-scattered to
  // their owners (15/16 EP DPP row moves instead of 4 EMAX), and softmax /
  // top-k run on Q values per lane with DPP row butterflies for the max, the
  // sum and the arg-max of each top-k round.
  constexpr int EP = EMAX < 16 ? 16 : EMAX;
  constexpr int Q = EP / 16;
  float psum[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) psum[q] = 0.f;
  float pz = 0.f;

#pragma unroll
  for (int it = 0; it < ITERS; ++it) {
    const int tl = it * NW * 4 + wave * 4 + grp;  // token within block
    const int t = blk * TPB + tl;
    const bool valid = t < T;
    float v[EP];
#pragma unroll
    for (int e = 0; e < EP; ++e) v[e] = 0.f;
    if (valid) {
      const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)t * d);
      for (int c = 0; c < nchunk; ++c) {
        const int ch = sub + 16 * c;  // chunk index within the row
        float xv[8];
        uint4 raw;
        if (c == 0) raw = xpre[it][0];
        else if (c == 1) raw = xpre[it][1];
        else raw = xr[ch];
        unpack8(raw, xv);
#pragma unroll
        for (int e = 0; e < EMAX; ++e) {
          if (e < E) {
            const float4* w4 = reinterpret_cast<const float4*>(s_wg + e * d + ch * 8);
            const float4 w0 = w4[0], w1 = w4[1];
            v[e] += xv[0] * w0.x + xv[1] * w0.y + xv[2] * w0.z + xv[3] * w0.w +
                    xv[4] * w1.x + xv[5] * w1.y + xv[6] * w1.z + xv[7] * w1.w;
          }
        }
      }
    }
    // reduce-scatter: after the stage with mask m, position e0 (bit m clear)
    // holds the pair sum for expert e0 | (sub & m)
    rs_stage<8>(v, sub);
    rs_stage<4>(v, sub);
    rs_stage<2>(v, sub);
    rs_stage<1>(v, sub);
    if (!valid) continue;  // uniform per 16-lane group; group shuffles only below

    float logit[Q];
    bool own[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int e = 16 * q + sub;
      own[q] = e < E;
      logit[q] = v[16 * q] + ((own[q] && has_ctx) ? s_cb[cid[it] * E + e] : 0.f);
    }
    float m = -INFINITY;
#pragma unroll
    for (int q = 0; q < Q; ++q)
      if (own[q]) m = fmaxf(m, logit[q]);
    m = row16_max(m);
    float p[Q];
    float sl = 0.f;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      p[q] = own[q] ? expf(logit[q] - m) : 0.f;
      sl += p[q];
    }
    const float ssm = row16_sum(sl);
    const float inv = 1.f / ssm;
#pragma unroll
    for (int q = 0; q < Q; ++q) p[q] *= inv;
    const float lse = m + logf(ssm);

    // top-k on logits (monotone in probs); ties -> lower expert id
    uint32_t taken = 0;  // bit q: owned expert 16q+sub already selected
    int sel[8];
    float selp[8];
    float ssum = 0.f;
    _Pragma("unroll") for (int j = 0; j < 8; ++j) if (j < k) {
      int best = 0x7fffffff;
      float bv = -INFINITY;
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (own[q] && !((taken >> q) & 1u) && (best == 0x7fffffff || logit[q] > bv)) {
          bv = logit[q];
          best = 16 * q + sub;
        }
      argmax_stage<8>(bv, best);
      argmax_stage<4>(bv, best);
      argmax_stage<2>(bv, best);
      argmax_stage<1>(bv, best);
      if ((best & 15) == sub) taken |= 1u << (best >> 4);
      sel[j] = best;
      selp[j] = expf(bv - m) * inv;  // bit-identical to the owner's p
      ssum += selp[j];
    }
    const bool renorm = normalize && k > 1;
    if (sub < k) {
      int si = 0;
      float sp = 0.f;
      _Pragma("unroll") for (int j = 0; j < 8; ++j) if (j < k)
        if (j == sub) { si = sel[j]; sp = selp[j]; }
      topk_idx[(size_t)t * k + sub] = si;
      topk_w[(size_t)t * k + sub] = renorm ? sp / ssum : sp;
      s_idx[tl * 8 + sub] = si;
    }
#pragma unroll
    for (int q = 0; q < Q; ++q)
      if (own[q]) probs_out[(size_t)t * E + 16 * q + sub] = p[q];
    if (sub == 0) lse_out[t] = lse;
#pragma unroll
    for (int q = 0; q < Q; ++q) psum[q] += p[q];
    pz += lse * lse;
  }

  // Aux partials: lane sub of each group holds its owned experts' sums;
  // combine the four groups of the wave, then the NW waves, in a fixed order.
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    float u = psum[q];
    u += __shfl_xor(u, 16, 64);
    u += __shfl_xor(u, 32, 64);
    psum[q] = u;
  }
  pz += __shfl_xor(pz, 16, 64);
  pz += __shfl_xor(pz, 32, 64);
  if (lane < 16) {
#pragma unroll
    for (int q = 0; q < Q; ++q)
      if (16 * q + lane < E) s_aux[wave * (EMAX + 1) + 16 * q + lane] = psum[q];
    if (lane == 0) s_aux[wave * (EMAX + 1) + EMAX] = pz;
  }
  __syncthreads();
  for (int i = tid; i <= E; i += NT) {  // E + 1 columns (more than one wave's lanes when NW = 1, E = 64)
    const int src = (i == E) ? EMAX : i;
    float u = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) u += s_aux[w * (EMAX + 1) + src];
    aux_partials[(size_t)blk * (E + 1) + i] = u;
  }

  // Within-block stable ranks: wave 0, lane l = token l of the block.
  if (wave == 0) {
    const int t = blk * TPB + lane;
    _Pragma("unroll") for (int j = 0; j < 8; ++j) if (j < k) {
      const int e_l = lane < TPB ? s_idx[lane * 8 + j] : -1;
      int rank = 0;
      for (int e = 0; e < E; ++e) {
        const unsigned long long mask = __ballot(e_l == e);
        if (e_l == e) rank = mbcnt(mask);
        if (lane == 0) block_counts[((size_t)blk * k + j) * E + e] = __popcll(mask);
      }
      if (lane < TPB && t < T) local_rank[(size_t)t * k + j] = rank;
    }
  }
}

// ---------------------------------------------------------------------------
// route scan (single workgroup)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void route_scan_kernel(
    const int32_t* __restrict__ counts, int nblk, int k, int E, int cap,
    int32_t* __restrict__ rank_base, int32_t* __restrict__ hist,
    int32_t* __restrict__ offsets) {
  // Thread = (segment, column): consecutive threads read consecutive columns
  // of a counts row (coalesced), and the router blocks are split into nseg
  // contiguous segments so every column is scanned by 1024/ncol threads.
  __shared__ int32_t s_seg[1024];  // per (segment, column) sums -> exclusive prefixes
  __shared__ int32_t s_tot[8 * 64];
  __shared__ int32_t s_slot[8 * 64];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int ncol = k * E;
  const int nseg = 1024 / ncol;  // ncol <= 512 -> nseg >= 2
  const int bs = (nblk + nseg - 1) / nseg;
  const int col = tid % ncol;
  const int seg = tid / ncol;
  const bool active = seg < nseg;
  const int b_lo = active ? min(seg * bs, nblk) : nblk;
  const int b_hi = active ? min(b_lo + bs, nblk) : nblk;
  constexpr int CH = 8;  // loads issued together before their use

  // Phase 0: per-segment column sums.
  int s = 0;
  for (int b0 = b_lo; b0 < b_hi; b0 += CH) {
    int v[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) v[i] = (b0 + i < b_hi) ? counts[(size_t)(b0 + i) * ncol + col] : 0;
#pragma unroll
    for (int i = 0; i < CH; ++i) s += v[i];
  }
  if (active) s_seg[seg * ncol + col] = s;
  __syncthreads();
  // Column totals and per-segment exclusive prefixes (fixed order).
  if (tid < ncol) {
    int acc = 0;
    for (int g = 0; g < nseg; ++g) {
      const int t = s_seg[g * ncol + tid];
      s_seg[g * ncol + tid] = acc;
      acc += t;
    }
    s_tot[tid] = acc;
  }
  __syncthreads();
  // hist / kept offsets / slot bases (one wave, E <= 64 lanes).
  if (wave == 0) {
    int h = 0;
    if (lane < E)
      _Pragma("unroll") for (int j = 0; j < 8; ++j) if (j < k) {
        if (lane < E) s_slot[j * E + lane] = h;
        h += s_tot[j * E + lane];
      }
    const int kept = (lane < E) ? ((cap > 0 && h > cap) ? cap : h) : 0;
    // inclusive wave scan of kept
    int inc = kept;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(inc, o, 64);
      if (lane >= o) inc += v;
    }
    if (lane < E) {
      hist[lane] = h;
      offsets[lane] = inc - kept;
    }
    if (lane == E - 1) offsets[E] = inc;
  }
  __syncthreads();
  // Phase 1: running exclusive sum over the segment's blocks, plus the slot base.
  if (!active) return;
  int carry = s_slot[col] + s_seg[seg * ncol + col];
  for (int b0 = b_lo; b0 < b_hi; b0 += CH) {
    int v[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) v[i] = (b0 + i < b_hi) ? counts[(size_t)(b0 + i) * ncol + col] : 0;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      if (b0 + i < b_hi) rank_base[(size_t)(b0 + i) * ncol + col] = carry;
      carry += v[i];
    }
  }
}

// Column sums of the router's aux partials [nblk, E+1] by one 256-thread
// workgroup: 256 / (E+1) strided block segments (coalesced rows), combined in
// segment order -- a fixed summation order shared by route_dispatch and
// aux_loss_fwd, so both give bit-identical losses.  Valid for tid <= E.
__device__ __forceinline__ float aux_colsum(const float* __restrict__ partials, int nblk, int E, float* s_aux,
                                            int tid) {
  const int nc = E + 1, nseg = 256 / nc;
  const int c = tid % nc, seg = tid / nc;
  if (seg < nseg) {
    float acc = 0.f;
    for (int bb = seg; bb < nblk; bb += nseg) acc += partials[(size_t)bb * nc + c];
    s_aux[tid] = acc;
  }
  __syncthreads();
  float colsum = 0.f;
  if (tid <= E)
    for (int sg = 0; sg < nseg; ++sg) colsum += s_aux[sg * nc + tid];
  return colsum;
}

// ---------------------------------------------------------------------------
// route dispatch: scan + index + aux loss in one launch (replaces route_scan,
// route_index and aux_loss_fwd).  Workgroup b owns
// router block b (kRouterBlockTokens tokens): it sums the counts of every router block into
// column totals and its own exclusive prefix (coalesced rows, a few KiB read
// per workgroup from L2: no second launch, no inter-workgroup hand-off),
// forms the slot bases / hist / kept offsets (one wave), and writes pos,
// the row -> token map and the row gates of its tokens.  Workgroup 0 also
// writes hist / offsets and the layer's aux losses.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void route_dispatch_kernel(
    const int32_t* __restrict__ counts, int nblk, int T, int k, int E, int cap,
    const int32_t* __restrict__ topk_idx, const int32_t* __restrict__ local_rank, const float* __restrict__ topk_w,
    const float* __restrict__ aux_partials, float lb_coef, float z_coef,
    int32_t* __restrict__ hist, int32_t* __restrict__ offsets, int32_t* __restrict__ pos,
    int32_t* __restrict__ src_tok, float* __restrict__ row_gate, float* __restrict__ aux_out,
    float* __restrict__ wcoef, int32_t* __restrict__ prof_rows) {
  __shared__ int32_t s_pre[256];      // per (segment, column): prefix sums
  __shared__ int32_t s_tot[256];      // ... and totals
  __shared__ int32_t s_col_pre[512];  // column prefix over blocks < b
  __shared__ int32_t s_base[512];     // slot base + prefix per column
  __shared__ int32_t s_off[65];
  __shared__ float s_term[65];
  __shared__ float s_aux[256];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int b = blockIdx.x;
  const int ncol = k * E;  // <= 512
  // Phase A: column totals and this block's prefix over all router blocks.
  // ncol <= 256: 256 / ncol block segments per column, every thread busy, one
  // or two 8-deep load batches each (the workgroup's latency is a couple of L2
  // round trips, not nblk of them); combined in LDS in segment order.
  // ncol > 256: one segment, columns tid and tid + 256.
  constexpr int CH = 8;
  if (ncol <= 256) {
    const int nseg = 256 / ncol;
    const int col = tid % ncol, seg = tid / ncol;
    int pre = 0, tot = 0;
    if (seg < nseg) {
      const int bs = (nblk + nseg - 1) / nseg;
      const int lo = seg * bs, hi = min(lo + bs, nblk);
      for (int b0 = lo; b0 < hi; b0 += CH) {
        int v[CH];
#pragma unroll
        for (int i = 0; i < CH; ++i) v[i] = (b0 + i < hi) ? counts[(size_t)(b0 + i) * ncol + col] : 0;
#pragma unroll
        for (int i = 0; i < CH; ++i) {
          tot += v[i];
          pre += (b0 + i < b) ? v[i] : 0;
        }
      }
      s_pre[tid] = pre;
      s_tot[tid] = tot;
    }
    __syncthreads();
    if (tid < ncol) {
      int p = 0, t = 0;
      for (int sg = 0; sg < nseg; ++sg) {
        p += s_pre[sg * ncol + tid];
        t += s_tot[sg * ncol + tid];
      }
      s_col_pre[tid] = p;
      s_base[tid] = t;  // column total, for now
    }
  } else {
    for (int pass = 0; pass < 2; ++pass) {
      const int col = tid + 256 * pass;
      if (col < ncol) {
        int pre = 0, tot = 0;
        for (int b0 = 0; b0 < nblk; b0 += CH) {
          int v[CH];
#pragma unroll
          for (int i = 0; i < CH; ++i) v[i] = (b0 + i < nblk) ? counts[(size_t)(b0 + i) * ncol + col] : 0;
#pragma unroll
          for (int i = 0; i < CH; ++i) {
            tot += v[i];
            pre += (b0 + i < b) ? v[i] : 0;
          }
        }
        s_col_pre[col] = pre;
        s_base[col] = tot;
      }
    }
  }
  __syncthreads();
  // Phase B (wave 0, lane e): hist, kept offsets, slot bases (slot-major priority)
  if (wave == 0) {
    int h = 0;
    int sb[8];
    _Pragma("unroll") for (int j = 0; j < 8; ++j) if (j < k) {
      sb[j] = h;
      if (lane < E) h += s_base[j * E + lane];
    }
    const int kept = (lane < E) ? ((cap > 0 && h > cap) ? cap : h) : 0;
    int inc = kept;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(inc, o, 64);
      if (lane >= o) inc += v;
    }
    if (lane < E) {
      s_off[lane] = inc - kept;
      _Pragma("unroll") for (int j = 0; j < 8; ++j) if (j < k)
        s_base[j * E + lane] = sb[j] + s_col_pre[j * E + lane];
      if (b == 0) {
        hist[lane] = h;
        offsets[lane] = inc - kept;
      }
    }
    if (lane == E - 1) {
      s_off[E] = inc;
      if (b == 0) offsets[E] = inc;
      if (b == 0 && prof_rows != nullptr) *prof_rows = inc;
    }
    if (b == 0 && aux_out != nullptr && lane < E) s_term[lane] = (float)h;  // hist, for the aux loss
  }
  __syncthreads();
  // aux losses (workgroup 0): lb = E sum_e f_e P_e, z = mean lse^2 (aux_colsum order)
  if (b == 0 && aux_out != nullptr) {
    const float invT = 1.f / (float)(T > 0 ? T : 1);
    const float invA = 1.f / (float)(T * k > 0 ? T * k : 1);
    const float colsum = aux_colsum(aux_partials, nblk, E, s_aux, tid);
    float term = 0.f;
    if (tid <= E) {
      if (tid < E) {
        const float f = s_term[tid] * invA;
        term = f * (colsum * invT);
        wcoef[tid] = lb_coef * (float)E * f * invT;
      } else {
        term = colsum * invT;
        wcoef[E] = z_coef * invT;
      }
    }
    __syncthreads();
    if (tid <= E) s_term[tid] = term;
    __syncthreads();
    if (tid == 0) {
      float acc = 0.f;
      for (int i = 0; i < E; ++i) acc += s_term[i];
      const float lb = (float)E * acc, z = s_term[E];
      aux_out[0] = lb;
      aux_out[1] = z;
      aux_out[2] = lb_coef * lb + z_coef * z;
    }
  }
  // Phase C: this block's assignments
  for (int a = tid; a < kRouterBlockTokens * k; a += 256) {
    const int t = b * kRouterBlockTokens + a / k;
    if (t >= T) break;
    const int j = a - (a / k) * k;
    const size_t ai = (size_t)t * k + j;
    const int e = topk_idx[ai];
    const int r = s_base[j * E + e] + local_rank[ai];
    const int p = (cap <= 0 || r < cap) ? s_off[e] + r : -1;
    pos[ai] = p;
    if (p >= 0) {
      src_tok[p] = t;
      if (row_gate != nullptr) row_gate[p] = topk_w[ai];
    }
  }
}

// ---------------------------------------------------------------------------
// aux losses from the router's per-block partials, one block:
//   P_e = sum_b partials[b][e] / T, f_e = hist[e] / (T k), lb = E sum_e f_e P_e,
//   z = sum_b partials[b][E] / T;  out = {lb, z, lb_coef lb + z_coef z}
//   wcoef = d out[2] / d partials[b][.] (the same for every b):
//           lb_coef E f_e / T (e < E), z_coef / T (e = E)
// Replaces ~12 tiny torch launches forward and ~8 backward per MoE layer.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void aux_loss_fwd_kernel(const float* __restrict__ partials, int nblk, int E,
                                                           const int32_t* __restrict__ hist, int T, int k,
                                                           float lb_coef, float z_coef, float* __restrict__ out,
                                                           float* __restrict__ wcoef) {
  __shared__ float s_term[65];
  __shared__ float s_aux[256];
  const int e = threadIdx.x;
  const float invT = 1.f / (float)(T > 0 ? T : 1);
  const float invA = 1.f / (float)(T * k > 0 ? T * k : 1);
  const float colsum = aux_colsum(partials, nblk, E, s_aux, e);
  if (e <= E) {
    if (e < E) {
      const float f = (float)hist[e] * invA;
      s_term[e] = f * (colsum * invT);
      wcoef[e] = lb_coef * (float)E * f * invT;
    } else {
      s_term[E] = colsum * invT;
      wcoef[E] = z_coef * invT;
    }
  }
  __syncthreads();
  if (e == 0) {
    float acc = 0.f;
    for (int i = 0; i < E; ++i) acc += s_term[i];
    const float lb = (float)E * acc, z = s_term[E];
    out[0] = lb;
    out[1] = z;
    out[2] = lb_coef * lb + z_coef * z;
  }
}

// ---------------------------------------------------------------------------
// token backward: dispatch transpose + router backward
// ---------------------------------------------------------------------------
// dl[e] = the value lane (e mod 16) of this 16-lane row holds in dlq[e / 16]
// (DPP row_newbcast, no LDS round trip).
template <int EP, int E0, int Q>
__device__ __forceinline__ void row_bcast_all(const float (&dlq)[Q], float (&dl)[EP]) {
  if constexpr (E0 < EP) {
    dl[E0] = __int_as_float(
        __builtin_amdgcn_update_dpp(0, __float_as_int(dlq[E0 >> 4]), 0x150 + (E0 & 15), 0xF, 0xF, false));
    row_bcast_all<EP, E0 + 1, Q>(dlq, dl);
  }
}

template <int EMAX>
__global__ __launch_bounds__(256) void token_bwd_kernel(
    const uint16_t* __restrict__ dxp, const int32_t* __restrict__ pos,
    const float* __restrict__ probs, const int32_t* __restrict__ topk_idx,
    const float* __restrict__ topk_w, const float* __restrict__ dw,
    const float* __restrict__ lse, const float* __restrict__ dprob_bias,
    const float* __restrict__ zc_ptr,
    const float* __restrict__ wg, int T, int d, int E, int k, int normalize,
    uint16_t* __restrict__ dx, float* __restrict__ dlogits,
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ yp, float* __restrict__ dw_out,
    const uint16_t* __restrict__ dres) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_wg = reinterpret_cast<float*>(smem);  // [E][d]
  const int tid = threadIdx.x;
  {
    const int n4 = (E * d) >> 2;
    const float4* src = reinterpret_cast<const float4*>(wg);
    float4* dst = reinterpret_cast<float4*>(s_wg);
    for (int i = tid; i < n4; i += 256) dst[i] = src[i];
  }
  __syncthreads();

  const int lane = tid & 63;
  const int sub = lane & 15;
  const int grp = lane >> 4;
  const int nchunk = d >> 7;
  const float zc = zc_ptr != nullptr ? *zc_ptr : 0.f;
  // 16 tokens per block-iteration (4 waves x 4 groups); grid-stride.
  for (int tb = blockIdx.x * 16; tb < T; tb += gridDim.x * 16) {
    const int t = tb + (tid >> 6) * 4 + grp;
    if (t >= T) continue;
    // ---- router backward: lane sub owns experts 16 q + sub (as in the forward) ----
    constexpr int EP = EMAX < 16 ? 16 : EMAX;
    constexpr int Q = EP / 16;
    float p[Q], dp[Q];
    bool own[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int e = 16 * q + sub;
      own[q] = e < E;
      p[q] = own[q] ? probs[(size_t)t * E + e] : 0.f;
      dp[q] = (own[q] && dprob_bias != nullptr) ? dprob_bias[e] : 0.f;
    }
    int pj[8];
    _Pragma("unroll") for (int j = 0; j < 8; ++j) if (j < k) pj[j] = pos[(size_t)t * k + j];
    int sel[8];
    float selw[8], seldw[8];
    if (dw == nullptr) {
      // the combine transpose's gate gradient, here: dw[t,j] = <dy[t], Yp[pos[t,j]]>
      // (16 lanes per token, 16-B chunks, fixed-order row sum)
      float part[8];
      _Pragma("unroll") for (int j = 0; j < 8; ++j) part[j] = 0.f;
      for (int c = 0; c < nchunk; ++c) {
        const int ch = sub + 16 * c;
        float g[8];
        unpack8(reinterpret_cast<const uint4*>(dy + (size_t)t * d)[ch], g);
        _Pragma("unroll") for (int j = 0; j < 8; ++j) if (j < k) {
          if (pj[j] < 0) continue;
          float v[8];
          unpack8(reinterpret_cast<const uint4*>(yp + (size_t)pj[j] * d)[ch], v);
#pragma unroll
          for (int i = 0; i < 8; ++i) part[j] += g[i] * v[i];
        }
      }
      _Pragma("unroll") for (int j = 0; j < 8; ++j) if (j < k) {
        seldw[j] = row16_sum(part[j]);
        if (dw_out != nullptr && sub == j) dw_out[(size_t)t * k + j] = seldw[j];
      }
    }
    float Sl = 0.f, wdw = 0.f;
    _Pragma("unroll") for (int j = 0; j < 8; ++j) if (j < k) {
      sel[j] = topk_idx[(size_t)t * k + j];
      selw[j] = topk_w[(size_t)t * k + j];
      if (dw != nullptr) seldw[j] = dw[(size_t)t * k + j];
      wdw += selw[j] * seldw[j];
      if ((sel[j] & 15) == sub) {
#pragma unroll
        for (int q = 0; q < Q; ++q)
          if (q == (sel[j] >> 4)) Sl += p[q];
      }
    }
    const float S = row16_sum(Sl);  // sum of the selected probabilities
    const bool renorm = normalize && k > 1;
    _Pragma("unroll") for (int j = 0; j < 8; ++j) if (j < k) {
      const float g = renorm ? (seldw[j] - wdw) / S : seldw[j];
      if ((sel[j] & 15) == sub) {
#pragma unroll
        for (int q = 0; q < Q; ++q)
          if (q == (sel[j] >> 4)) dp[q] += g;
      }
    }
    float dotl = 0.f;
#pragma unroll
    for (int q = 0; q < Q; ++q) dotl += p[q] * dp[q];
    const float dot = row16_sum(dotl);
    const float zt = zc * lse[t];
    float dlq[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) dlq[q] = own[q] ? p[q] * (dp[q] - dot) + zt * p[q] : 0.f;
    float dl[EP];  // every expert's dlogit, broadcast from its owner (DPP row_newbcast)
    row_bcast_all<EP, 0, Q>(dlq, dl);
    // ---- dx = sum_j dXp[pos] + dlogits . Wg ----
    // (dlogits is stored after dx: on gfx9 vmcnt also counts stores, so a
    // store issued before the dXp gathers would delay their wait)
    for (int c = 0; c < nchunk; ++c) {
      const int ch = sub + 16 * c;
      float acc[8];
      if (dres != nullptr) {  // the residual branch's gradient (combine with resid: dres = dy)
        unpack8(reinterpret_cast<const uint4*>(dres + (size_t)t * d)[ch], acc);
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = 0.f;
      }
      _Pragma("unroll") for (int j = 0; j < 8; ++j) if (j < k) {
        if (pj[j] < 0) continue;
        float v[8];
        unpack8(reinterpret_cast<const uint4*>(dxp + (size_t)pj[j] * d)[ch], v);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] += v[i];
      }
#pragma unroll
      for (int e = 0; e < EMAX; ++e) {
        if (e < E) {
          const float4* w4 = reinterpret_cast<const float4*>(s_wg + e * d + ch * 8);
          const float4 w0 = w4[0], w1 = w4[1];
          acc[0] += dl[e] * w0.x; acc[1] += dl[e] * w0.y;
          acc[2] += dl[e] * w0.z; acc[3] += dl[e] * w0.w;
          acc[4] += dl[e] * w1.x; acc[5] += dl[e] * w1.y;
          acc[6] += dl[e] * w1.z; acc[7] += dl[e] * w1.w;
        }
        // keep the compiler from hoisting every expert's Wg reads at once
        // (E x 8 registers: occupancy 1 wave/SIMD at E = 32)
        if ((e & 7) == 7) asm volatile("" ::: "memory");
      }
      reinterpret_cast<uint4*>(dx + (size_t)t * d)[ch] = pack8(acc);
    }
#pragma unroll
    for (int q = 0; q < Q; ++q)
      if (own[q]) dlogits[(size_t)t * E + 16 * q + sub] = dlq[q];
  }
}


// ---------------------------------------------------------------------------
// Router weight gradients (the router's backward after
// token_bwd): dWg[e][c] = sum_t dlogits[t][e] x[t][c] and the context-bias
// gradient dcb[ctx][e] = sum of dlogits[t][e] over the tokens t of the images
// with ctx_img[t / tpi] == ctx.  Replaces torch's fp32 copy of x, the fp32
// GEMM dlogits^T x and the atomic index_add_ (whose arrival order made dcb
// non-repeatable).
//
// One launch, no workspace: workgroup j owns the CW columns [j CW, j CW + CW)
// of dWg for every expert (CW = 32 / EM, EM the expert count rounded up) and
// context j of dcb.  Its NT threads (1,024 for E <= 16, else 256) stride over
// ALL T tokens (thread i: tokens i, i + NT, ...), U tokens' loads in flight
// per round (dlogits row, CW x columns, the token's context), keeping
// E x CW + E fp32 sums; the per-thread sums are then added in LDS in a fixed
// order.  Every sum has a fixed association: bitwise repeatable, and dWg does
// not depend on whether dcb is formed.  dlogits (T E 4 B) is re-read by every
// workgroup from L2; x is read once in total (each workgroup its own columns).
// ---------------------------------------------------------------------------
template <int EM>
struct RwCfg {
  static constexpr int CW = EM >= 32 ? 1 : 32 / EM;          // dWg columns per workgroup
  static constexpr int NT = EM <= 16 ? 1024 : 256;            // threads (16 waves: 4 per SIMD at <= 128 VGPRs)
  static constexpr int U = EM == 8 ? 4 : (EM == 16 ? 2 : (EM == 32 ? 4 : 2));  // tokens per round in flight
  static constexpr int NV = EM * CW + EM;                    // per-thread sums: dWg block + dcb row
  static constexpr int NVP = NV <= 64 ? 64 : 128;            // outputs rounded to a power of two
  static constexpr int TPO = 256 / NVP;                      // threads per output in the final sum
  static constexpr int RS = 260;                             // LDS row stride (floats): conflict-free reads
  static constexpr size_t lds() { return (size_t)NV * RS * 4 + (size_t)NVP * TPO * 4; }
};

template <int EM, bool VEC>
__global__ __launch_bounds__(RwCfg<EM>::NT) void router_wgrad_kernel(const float* __restrict__ dlogits,
                                                                     const uint16_t* __restrict__ x,
                                                                     const int32_t* __restrict__ ctx_img, int T,
                                                                     int tpi, int E, int d, int C,
                                                                     float* __restrict__ dwg,
                                                                     float* __restrict__ dcb) {
  using K = RwCfg<EM>;
  constexpr int CW = K::CW, NT = K::NT, U = K::U, NV = K::NV, TPO = K::TPO, RS = K::RS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red = reinterpret_cast<float*>(smem);  // [NV][RS]: slot i holds the sum of threads i, i + 256, ...
  float* red2 = red + NV * RS;                   // [NVP][TPO]
  const int tid = threadIdx.x, j = blockIdx.x;
  const bool has_w = j * CW < d;
  const bool has_c = dcb != nullptr && j < C;
  const int c0 = has_w ? j * CW : 0;  // (a context-only workgroup reads column 0, unused)
  float acc[EM * CW], accb[EM];
#pragma unroll
  for (int i = 0; i < EM * CW; ++i) acc[i] = 0.f;
#pragma unroll
  for (int e = 0; e < EM; ++e) accb[e] = 0.f;
  for (int t0 = tid; t0 < T; t0 += NT * U) {
    float dl[U][EM];
    float xv[U][CW];
    int ci[U];
    // every load of the round first, from clamped (always valid) addresses, with
    // no use in between -- one memory round trip per U tokens (a use of any one
    // load waits for all loads issued before it)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int tc = min(t0 + NT * u, T - 1);
      const float* row = dlogits + (size_t)tc * E;
      if constexpr (VEC) {  // E % 4 == 0: 16-B loads (a runtime branch here was merged into dword loads)
#pragma unroll
        for (int q = 0; q < EM / 4; ++q) {
          const float4 v = reinterpret_cast<const float4*>(row)[min(q, (E >> 2) - 1)];
          dl[u][4 * q] = v.x; dl[u][4 * q + 1] = v.y; dl[u][4 * q + 2] = v.z; dl[u][4 * q + 3] = v.w;
        }
      } else {
#pragma unroll
        for (int e = 0; e < EM; ++e) dl[u][e] = row[min(e, E - 1)];
      }
      const uint16_t* xr = x + (size_t)tc * d + c0;
      if constexpr (CW == 4) {
        const uint2 v = *reinterpret_cast<const uint2*>(xr);
        xv[u][0] = __uint_as_float(v.x << 16); xv[u][1] = __uint_as_float(v.x & 0xffff0000u);
        xv[u][2] = __uint_as_float(v.y << 16); xv[u][3] = __uint_as_float(v.y & 0xffff0000u);
      } else if constexpr (CW == 2) {
        const uint32_t v = *reinterpret_cast<const uint32_t*>(xr);
        xv[u][0] = __uint_as_float(v << 16); xv[u][1] = __uint_as_float(v & 0xffff0000u);
      } else {
        xv[u][0] = bf2f(*xr);
      }
      ci[u] = has_c ? ctx_img[tc / tpi] : -1;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool ok = t0 + NT * u < T;
      const bool in_c = ok && ci[u] == j;
#pragma unroll
      for (int e = 0; e < EM; ++e) {
        const float g = (ok && e < E) ? dl[u][e] : 0.f;
#pragma unroll
        for (int w = 0; w < CW; ++w) acc[e * CW + w] += g * xv[u][w];
        accb[e] += in_c ? g : 0.f;
      }
    }
  }
  // fixed-order sum over the NT threads: the groups of 256 threads add their
  // sums into the 256 slots one group after another (slot i = thread i +
  // thread i + 256 + ...); output o is then split over TPO threads (thread p
  // takes slots p, p + TPO, ... in order) and the TPO partials added in order
#pragma unroll
  for (int q = 0; q < NT / 256; ++q) {
    if (tid / 256 == q) {
      const int sl = tid & 255;
#pragma unroll
      for (int i = 0; i < EM * CW; ++i) red[i * RS + sl] = q == 0 ? acc[i] : red[i * RS + sl] + acc[i];
#pragma unroll
      for (int e = 0; e < EM; ++e)
        red[(EM * CW + e) * RS + sl] = q == 0 ? accb[e] : red[(EM * CW + e) * RS + sl] + accb[e];
    }
    __syncthreads();
  }
  const int o = tid / TPO, part = tid - o * TPO;  // (threads 256 .. NT - 1 only pass the barrier)
  if (tid < 256 && o < NV) {
    float v[256 / TPO];  // all reads first, then the fixed-order sum
#pragma unroll
    for (int i = 0; i < 256 / TPO; ++i) v[i] = red[o * RS + part + TPO * i];
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < 256 / TPO; ++i) sum += v[i];
    red2[o * TPO + part] = sum;
  }
  __syncthreads();
  if (tid >= 256 || part != 0 || o >= NV) return;
  float sum = red2[o * TPO];
#pragma unroll
  for (int q = 1; q < TPO; ++q) sum += red2[o * TPO + q];
  if (o < EM * CW) {
    const int e = o / CW, w = o - e * CW;
    if (has_w && e < E) dwg[(size_t)e * d + c0 + w] = sum;
  } else {
    const int e = o - EM * CW;
    if (has_c && e < E) dcb[(size_t)j * E + e] = sum;
  }
}

}  // namespace moe

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------
using namespace moe;

extern "C" int moe_router_num_blocks(int T) { return (T + kRouterBlockTokens - 1) / kRouterBlockTokens; }

// Raise the dynamic-LDS cap of a kernel (once, on its first launch) so a
// launch needing more than 64 KiB succeeds; later launches make no call.
template <auto FN>
static void allow_lds(size_t bytes) {
  // (per device; a failure is reported through moe_last_error and the launch
  // that follows fails its check_launch)
  static unsigned long long done = 0;
  (void)allow_dyn_lds(reinterpret_cast<const void*>(FN), 96 * 1024, &done, "router: dynamic LDS");
  (void)bytes;
}

static int emax_for(int E) { return E <= 8 ? 8 : E <= 16 ? 16 : E <= 32 ? 32 : 64; }

extern "C" int moe_router_topk_fwd(const void* x, const float* wg, const float* ctx_bias,
                                   const int32_t* ctx_img, int n_ctx, int tokens_per_image, int T,
                                   int d, int E, int k, int normalize, int32_t* topk_idx,
                                   float* topk_w, float* probs, float* lse,
                                   int32_t* local_rank, int32_t* block_counts,
                                   float* aux_partials, hipStream_t stream) {
  if (T < 0 || d <= 0 || d % 128 != 0 || d > 1024) return fail("router: d must be a multiple of 128 in [128,1024]");
  if (E < 1 || E > 64 || k < 1 || k > 8 || k > E) return fail("router: need 1<=E<=64, 1<=k<=min(8,E)");
  if ((size_t)E * d * 4 > 64 * 1024) return fail("router: E*d*4 must fit 64 KiB of LDS");
  if (ctx_img != nullptr && tokens_per_image <= 0) return fail("router: tokens_per_image must be > 0");
  if ((ctx_bias != nullptr) != (ctx_img != nullptr)) return fail("router: ctx_bias and ctx_img go together");
  if (ctx_bias != nullptr && (n_ctx < 1 || (size_t)n_ctx * E > 4096))
    return fail("router: need 1 <= n_ctx and n_ctx * E <= 4096 (the context-bias table is staged in LDS)");
  if (T == 0) return 0;
  const int nblk = moe_router_num_blocks(T);
  const int em = emax_for(E);
  constexpr int TPB = kRouterBlockTokens;
  const int nw = em <= 32 ? TPB / 4 : 4;
  const size_t shmem = (size_t)E * d * 4 + TPB * 8 * 4 + nw * (em + 1) * 4 +
                       (ctx_bias != nullptr ? (size_t)n_ctx * E * 4 : 0);
  const uint16_t* xb = static_cast<const uint16_t*>(x);
  // bytes: x, Wg once, per-token outputs (idx, w, probs, lse, local rank), per-block partials
  ProfScope prof(stream, PROF_ROUTER,
                 2.0 * T * d + 4.0 * E * d + 12.0 * T * k + 4.0 * T * (E + 1) + 4.0 * nblk * (k * E + E + 1));
#define LAUNCH_R(EM, NW)                                                                                    \
  allow_lds<router_topk_fwd_kernel<EM, NW, TPB>>(shmem);                                                     \
  MOE_LAUNCH(prof, (router_topk_fwd_kernel<EM, NW, TPB>), dim3(nblk), dim3(NW * 64), shmem, stream, xb, wg,  \
             ctx_bias, ctx_img, n_ctx, tokens_per_image, T, d, E, k, normalize, topk_idx, topk_w, probs, lse, \
             local_rank, block_counts, aux_partials)
  switch (em) {
    case 8: LAUNCH_R(8, TPB / 4); break;
    case 16: LAUNCH_R(16, TPB / 4); break;
    case 32: LAUNCH_R(32, TPB / 4); break;
    default: LAUNCH_R(64, TPB / 16); break;
  }
#undef LAUNCH_R
  return check_launch("moe_router_topk_fwd");
}

extern "C" int moe_route_scan(const int32_t* block_counts, int nblk, int k, int E, int cap,
                              int32_t* rank_base, int32_t* hist, int32_t* offsets,
                              hipStream_t stream) {
  if (E < 1 || E > 64 || k < 1 || k > 8) return fail("route_scan: need 1<=E<=64, 1<=k<=8");
  if (nblk < 0) return fail("route_scan: nblk < 0");
  ProfScope prof(stream, PROF_SCAN, 8.0 * nblk * k * E + 12.0 * E);
  MOE_LAUNCH(prof, route_scan_kernel, dim3(1), dim3(1024), 0, stream, block_counts, nblk, k,
                     E, cap, rank_base, hist, offsets);
  return check_launch("moe_route_scan");
}

extern "C" int moe_route_dispatch(const int32_t* block_counts, int nblk, int T, int k, int E, int cap,
                                  const int32_t* topk_idx, const int32_t* local_rank, const float* topk_w,
                                  const float* aux_partials, float lb_coef, float z_coef, int32_t* hist,
                                  int32_t* offsets, int32_t* pos, int32_t* src_tok, float* row_gate,
                                  float* aux_out3, float* wcoef, hipStream_t stream) {
  if (E < 1 || E > 64 || k < 1 || k > 8 || k > E) return fail("route_dispatch: need 1<=E<=64, 1<=k<=min(8,E)");
  if (nblk != moe_router_num_blocks(T)) return fail("route_dispatch: nblk must be moe_router_num_blocks(T)");
  if ((aux_out3 == nullptr) != (wcoef == nullptr) || (aux_out3 != nullptr && aux_partials == nullptr))
    return fail("route_dispatch: aux_out3, wcoef and aux_partials go together");
  if (row_gate != nullptr && topk_w == nullptr) return fail("route_dispatch: row_gate needs topk_w");
  if (T <= 0) return 0;
  // bytes: every workgroup reads the block counts (L2), per assignment idx/rank/gate read and pos written,
  // per kept row src_tok (+ gate) written
  ProfScope prof(stream, PROF_SCAN, 4.0 * nblk * k * E + 16.0 * T * k + 4.0 * nblk * (E + 1), true,
                 row_gate ? 8.0 : 4.0);
  MOE_LAUNCH(prof, route_dispatch_kernel, dim3(nblk), dim3(256), 0, stream, block_counts, nblk, T, k, E, cap,
             topk_idx, local_rank, topk_w, aux_partials, lb_coef, z_coef, hist, offsets, pos, src_tok, row_gate,
             aux_out3, wcoef, prof.rows_slot());
  return check_launch("moe_route_dispatch");
}

extern "C" int moe_token_bwd_res(const void* dxp, const int32_t* pos, const float* probs,
                                 const int32_t* topk_idx, const float* topk_w, const float* dw,
                                 const void* dy, const void* yp, float* dw_out, const void* dres,
                                 const float* lse, const float* dprob_bias, const float* zc,
                                 const float* wg, int T, int d, int E, int k, int normalize,
                                 void* dx, float* dlogits, hipStream_t stream);

extern "C" int moe_token_bwd_dw(const void* dxp, const int32_t* pos, const float* probs,
                                const int32_t* topk_idx, const float* topk_w, const float* dw,
                                const void* dy, const void* yp, float* dw_out,
                                const float* lse, const float* dprob_bias, const float* zc,
                                const float* wg, int T, int d, int E, int k, int normalize,
                                void* dx, float* dlogits, hipStream_t stream) {
  return moe_token_bwd_res(dxp, pos, probs, topk_idx, topk_w, dw, dy, yp, dw_out, nullptr, lse, dprob_bias, zc,
                           wg, T, d, E, k, normalize, dx, dlogits, stream);
}

extern "C" int moe_token_bwd(const void* dxp, const int32_t* pos, const float* probs,
                             const int32_t* topk_idx, const float* topk_w, const float* dw,
                             const float* lse, const float* dprob_bias, const float* zc,
                             const float* wg, int T, int d, int E, int k, int normalize,
                             void* dx, float* dlogits, hipStream_t stream) {
  if (dw == nullptr) return fail("token_bwd: dw is NULL (moe_token_bwd_dw computes it from dy and yp)");
  return moe_token_bwd_dw(dxp, pos, probs, topk_idx, topk_w, dw, nullptr, nullptr, nullptr, lse, dprob_bias, zc,
                          wg, T, d, E, k, normalize, dx, dlogits, stream);
}

extern "C" int moe_token_bwd_res(const void* dxp, const int32_t* pos, const float* probs,
                                 const int32_t* topk_idx, const float* topk_w, const float* dw,
                                 const void* dy, const void* yp, float* dw_out, const void* dres,
                                 const float* lse, const float* dprob_bias, const float* zc,
                                 const float* wg, int T, int d, int E, int k, int normalize,
                                 void* dx, float* dlogits, hipStream_t stream) {
  if (dw == nullptr && (dy == nullptr || yp == nullptr)) return fail("token_bwd: need dw, or dy and yp");
  if (d <= 0 || d % 128 != 0 || d > 1024) return fail("token_bwd: d must be a multiple of 128 in [128,1024]");
  if (E < 1 || E > 64 || k < 1 || k > 8 || k > E) return fail("token_bwd: need 1<=E<=64, 1<=k<=min(8,E)");
  if ((size_t)E * d * 4 > 64 * 1024) return fail("token_bwd: E*d*4 must fit 64 KiB of LDS");
  if (T <= 0) return 0;
  const int em = emax_for(E);
  int grid = (T + 15) / 16;
  if (grid > 2048) grid = 2048;
  const size_t shmem = (size_t)E * d * 4;
  const uint16_t* dxpb = static_cast<const uint16_t*>(dxp);
  uint16_t* dxb = static_cast<uint16_t*>(dx);
  // bytes: T*k rows of dXp, per-token routing state, Wg; dx and dlogits written
  // (+ dy and the T*k rows of Yp when dw is formed here)
  ProfScope prof(stream, PROF_TOKEN_BWD,
                 2.0 * T * k * d + 2.0 * T * d + 8.0 * T * E + 20.0 * T * k + 4.0 * T + 4.0 * E * d +
                     (dw == nullptr ? 2.0 * T * d + 2.0 * T * k * d : 0.0) +
                     (dres != nullptr && dres != dy ? 2.0 * T * d : 0.0));
  const uint16_t* dyb = static_cast<const uint16_t*>(dy);
  const uint16_t* ypb = static_cast<const uint16_t*>(yp);
#define LAUNCH_B(EM)                                                                          \
  allow_lds<token_bwd_kernel<EM>>(shmem);                                                   \
  MOE_LAUNCH(prof, token_bwd_kernel<EM>, dim3(grid), dim3(256), shmem, stream, dxpb, pos, \
                     probs, topk_idx, topk_w, dw, lse, dprob_bias, zc, wg, T, d, E, k,      \
                     normalize, dxb, dlogits, dyb, ypb, dw_out, static_cast<const uint16_t*>(dres))
  switch (em) {
    case 8: LAUNCH_B(8); break;
    case 16: LAUNCH_B(16); break;
    case 32: LAUNCH_B(32); break;
    default: LAUNCH_B(64); break;
  }
#undef LAUNCH_B
  return check_launch("moe_token_bwd");
}

extern "C" int moe_aux_loss_fwd(const float* aux_partials, int nblk, int E, const int32_t* hist, int T, int k,
                                float lb_coef, float z_coef, float* out3, float* wcoef, hipStream_t stream) {
  if (E < 1 || E > 64 || nblk < 0 || k < 1) return fail("aux_loss_fwd: need 1 <= E <= 64, nblk >= 0, k >= 1");
  if (aux_partials == nullptr || hist == nullptr || out3 == nullptr || wcoef == nullptr)
    return fail("aux_loss_fwd: NULL pointer");
  ProfScope prof(stream, PROF_ROUTER, 4.0 * nblk * (E + 1) + 4.0 * E + 12.0 + 4.0 * (E + 1));
  MOE_LAUNCH(prof, aux_loss_fwd_kernel, dim3(1), dim3(256), 0, stream, aux_partials, nblk, E, hist, T, k, lb_coef,
             z_coef, out3, wcoef);
  return check_launch("moe_aux_loss_fwd");
}

// Reserved workspace query (the chunked variant that used it was measured no
// faster and removed in round 5): always 0, so callers pass part = NULL.
extern "C" long long moe_router_wgrad_workspace(int B, int tpi, int E, int d) {
  (void)B, (void)tpi, (void)E, (void)d;
  return 0;
}

extern "C" int moe_router_wgrad(const float* dlogits, const void* x, const int32_t* ctx_img, int B, int tpi, int E,
                                int d, int C, float* part, float* dwg, float* dcb, hipStream_t stream) {
  if (B < 0 || tpi < 1 || E < 1 || E > 64 || d < 8 || d > 1024 || d % 8 || C < 0)
    return fail("router_wgrad: need B >= 0, tpi >= 1, 1 <= E <= 64, d % 8 == 0 in [8, 1024], C >= 0");
  if (reinterpret_cast<uintptr_t>(x) % 16 || reinterpret_cast<uintptr_t>(dlogits) % 16)
    return fail("router_wgrad: x and dlogits must be 16-B aligned");
  if (dlogits == nullptr || x == nullptr || dwg == nullptr) return fail("router_wgrad: NULL pointer");
  if (dcb != nullptr && (ctx_img == nullptr || C < 1)) return fail("router_wgrad: dcb needs ctx_img and C >= 1");
  if ((long long)B * tpi > 0x7fffffffLL / 1024) return fail("router_wgrad: too many tokens");
  const int T = B * tpi;
  if (T == 0) {  // no tokens: zero gradients
    if (hipMemsetAsync(dwg, 0, sizeof(float) * E * d, stream) != hipSuccess) return fail("router_wgrad: memset");
    if (dcb != nullptr && hipMemsetAsync(dcb, 0, sizeof(float) * C * E, stream) != hipSuccess)
      return fail("router_wgrad: memset");
    return 0;
  }
  // bytes: dlogits and x once, dWg and dcb written (+ one context id per token)
  ProfScope prof(stream, PROF_ROUTER_WGRAD,
                 4.0 * T * E + 2.0 * T * d + 4.0 * E * d + (dcb != nullptr ? 4.0 * C * E + 4.0 * B : 0.0));
  (void)part;  // reserved (moe_router_wgrad_workspace is 0)
#define LAUNCH_RW(EM_)                                                                                        \
  do {                                                                                                        \
    using K = RwCfg<EM_>;                                                                                     \
    const int ncb = d / K::CW;                                                                                \
    const int grid = dcb != nullptr && C > ncb ? C : ncb;                                                     \
    static unsigned long long lds_v = 0, lds_s = 0; /* per device; > 64 KiB of dynamic LDS at E > 32 */      \
    if (int rc = allow_dyn_lds(reinterpret_cast<const void*>(router_wgrad_kernel<EM_, true>), (int)K::lds(),  \
                               &lds_v, "router_wgrad"))                                                       \
      return rc;                                                                                              \
    if (int rc = allow_dyn_lds(reinterpret_cast<const void*>(router_wgrad_kernel<EM_, false>), (int)K::lds(), \
                               &lds_s, "router_wgrad"))                                                       \
      return rc;                                                                                              \
    if (E % 4 == 0)                                                                                           \
      MOE_LAUNCH(prof, (router_wgrad_kernel<EM_, true>), dim3(grid), dim3(K::NT), K::lds(), stream, dlogits,    \
                 static_cast<const uint16_t*>(x), ctx_img, T, tpi, E, d, C, dwg, dcb);                        \
    else                                                                                                      \
      MOE_LAUNCH(prof, (router_wgrad_kernel<EM_, false>), dim3(grid), dim3(K::NT), K::lds(), stream, dlogits,   \
                 static_cast<const uint16_t*>(x), ctx_img, T, tpi, E, d, C, dwg, dcb);                        \
  } while (0)
  switch (emax_for(E)) {
    case 8: LAUNCH_RW(8); break;
    case 16: LAUNCH_RW(16); break;
    case 32: LAUNCH_RW(32); break;
    default: LAUNCH_RW(64); break;
  }
#undef LAUNCH_RW
  return check_launch("moe_router_wgrad");
}
