// Hungarian matching on the GPU (RT-DETR set criterion; SURVEY.md 8(f).1 --
// the reference's training path matches predictions to ground truth inside
// Ultralytics' RTDETR loss with scipy.optimize.linear_sum_assignment).
//
// One 64-lane workgroup per problem (prediction set s, image b): cost
// C[s][b][q][m] for Q queries x M padded targets, the first n_valid[b]
// targets real.  The algorithm is scipy 1.15's rectangular LSAP (Crouse's
// shortest augmenting path, the form linear_sum_assignment runs on the
// transposed [n, Q] problem), restated step for step so that the matching --
// ties included -- is the one scipy returns: the same double arithmetic in the
// same order, the same "remaining" column list with swap removal, and the same
// tie rule for the next column (the lowest reduced cost; among equal ones the
// LAST unassigned in list order, else the first).  The wave parallelises the
// column scan of every Dijkstra step and the dual updates; bookkeeping is done
// by lane 0.  Output: assign[s][b][m] = matched query of target m, -1 for
// padding.  No host round trip: the criterion that follows can be captured in
// the training step's hipGraph.
#include "moe_common.h"
#include "prof.h"

namespace moe {

__device__ __forceinline__ double wave_min_d(double x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = fmin(x, __shfl_xor(x, o, 64));
  return x;
}
__device__ __forceinline__ int wave_max_i(int x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = max(x, __shfl_xor(x, o, 64));
  return x;
}
__device__ __forceinline__ int wave_min_i(int x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = min(x, __shfl_xor(x, o, 64));
  return x;
}

// cost(q, m) of one problem: an explicit [Q][M] matrix
struct MatrixCost {
  const float* C;
  int M;
  __device__ __forceinline__ float operator()(int q, int m) const { return C[(size_t)q * M + m]; }
};

template <class CostFn>
__device__ void lsap_solve(const CostFn& cost_qm, int n, int Q, int M, int32_t* __restrict__ out,
                           int32_t* __restrict__ status, char* smem);

__global__ __launch_bounds__(64) void lsap_kernel(const float* __restrict__ cost, const int32_t* __restrict__ n_valid,
                                                  int B, int Q, int M, int32_t* __restrict__ assign,
                                                  int32_t* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int p = blockIdx.x;
  lsap_solve(MatrixCost{cost + (size_t)p * Q * M, M}, n_valid[p % B], Q, M, assign + (size_t)p * M, status, smem);
}

template <class CostFn>
__device__ void lsap_solve(const CostFn& cost_qm, int n, int Q, int M, int32_t* __restrict__ out,
                           int32_t* __restrict__ status, char* smem) {
  double* u = reinterpret_cast<double*>(smem);  // [M]
  double* v = u + M;                            // [Q]
  double* spc = v + Q;                          // [Q] shortest path costs
  int* path = reinterpret_cast<int*>(spc + Q);  // [Q]
  int* row4col = path + Q;                      // [Q]
  int* remaining = row4col + Q;                 // [Q]
  int* col4row = remaining + Q;                 // [M]
  uint8_t* SR = reinterpret_cast<uint8_t*>(col4row + M);  // [M]
  uint8_t* SC = SR + M;                                   // [Q]
  __shared__ int s_i, s_sink, s_index;
  __shared__ double s_minval;

  const int lane = threadIdx.x;
  for (int m = lane; m < M; m += 64) out[m] = -1;
  if (n <= 0) return;
  if (n > Q || n > M) {
    if (lane == 0) atomicExch(status, 1);
    return;
  }
  // scipy transposes when rows > cols: rows = targets, cols = queries (Q > n);
  // a square problem (n == Q) keeps rows = queries, cols = targets
  const bool tr = Q > n;
  const int nr = n, nc = tr ? Q : n;
  for (int m = lane; m < nr; m += 64) {
    u[m] = 0.0;
    col4row[m] = -1;
  }
  for (int j = lane; j < nc; j += 64) {
    v[j] = 0.0;
    row4col[j] = -1;
    path[j] = -1;
  }
  __syncthreads();

  for (int cur = 0; cur < nr; ++cur) {
    for (int it = lane; it < nc; it += 64) {
      remaining[it] = nc - it - 1;
      spc[it] = INFINITY;
      SC[it] = 0;
    }
    for (int m = lane; m < nr; m += 64) SR[m] = 0;
    if (lane == 0) {
      s_i = cur;
      s_sink = -1;
      s_minval = 0.0;
    }
    int nrem = nc;
    __syncthreads();
    while (true) {
      const int i = s_i;
      const double minval = s_minval;
      if (lane == 0) SR[i] = 1;
      const double ui = u[i];
      // relax every remaining column, then the lowest reduced cost with scipy's tie rule
      double lo = INFINITY;
      for (int it = lane; it < nrem; it += 64) {
        const int j = remaining[it];
        const double r = minval + (double)(tr ? cost_qm(j, i) : cost_qm(i, j)) - ui - v[j];
        if (r < spc[j]) {
          path[j] = i;
          spc[j] = r;
        }
        lo = fmin(lo, spc[j]);
      }
      const double L = wave_min_d(lo);
      int last_un = -1, first_eq = 0x7fffffff;
      for (int it = lane; it < nrem; it += 64) {
        const int j = remaining[it];
        if (spc[j] == L) {
          first_eq = min(first_eq, it);
          if (row4col[j] == -1) last_un = max(last_un, it);
        }
      }
      last_un = wave_max_i(last_un);
      first_eq = wave_min_i(first_eq);
      __syncthreads();  // every lane has read remaining / spc before lane 0 edits them
      if (lane == 0) {
        const int index = last_un >= 0 ? last_un : first_eq;
        const int j = remaining[index];
        s_minval = L;
        if (row4col[j] == -1) s_sink = j;
        else s_i = row4col[j];
        SC[j] = 1;
        remaining[index] = remaining[nrem - 1];
        s_index = index;
      }
      --nrem;
      __syncthreads();
      if (s_sink != -1 || L == INFINITY || nrem == 0) break;  // nrem == 0 only if infeasible
    }
    const double minval = s_minval;
    if (s_sink == -1) {  // infeasible (non-finite costs)
      if (lane == 0) atomicExch(status, 2);
      return;
    }
    // dual updates (u of the visited rows other than cur use spc before any v change)
    for (int m = lane; m < nr; m += 64)
      if (SR[m] && m != cur) u[m] += minval - spc[col4row[m]];
    if (lane == 0) u[cur] += minval;
    for (int j = lane; j < nc; j += 64)
      if (SC[j]) v[j] -= minval - spc[j];
    __syncthreads();
    if (lane == 0) {  // augment along the path back to cur (at most cur + 1 hops)
      int j = s_sink;
      for (int hop = 0; hop <= cur; ++hop) {
        const int i = path[j];
        row4col[j] = i;
        const int t = col4row[i];
        col4row[i] = j;
        j = t;
        if (i == cur) break;
      }
    }
    __syncthreads();
  }
  for (int r = lane; r < nr; r += 64) {
    if (tr) out[r] = col4row[r];  // row = target
    else out[col4row[r]] = r;     // row = query
  }
}

// ---------------------------------------------------------------------------
// RT-DETR set criterion on the device (the HungarianMatcher cost and the
// VFL + L1 + GIoU losses of SetCriterion.forward_padded), fused:
//   * lsap_rtdetr_kernel: the matching cost is evaluated inside the solver
//     (focal class cost, L1 and GIoU of cxcywh boxes, weights 2 / 5 / 2) --
//     no [S,B,Q,M] cost tensor and none of its ~25 element-wise launches;
//   * set_loss_kernel: per prediction set, the three losses AND their
//     gradients w.r.t. logits and boxes in one pass (the loss is a leaf of
//     the graph; the backward only scales the stored gradients).
// ---------------------------------------------------------------------------
struct CritArgs {
  const float* logits;  // [S][B][Q][C]
  const float* boxes;   // [S][B][Q][4] cxcywh
  const float* tgt;     // [B][M][4] cxcywh
  const int32_t* labels;  // [B][M]
  int S, B, Q, C, M;
};

__device__ __forceinline__ float4 cxcywh_xyxy(float4 b) {
  return make_float4(b.x - 0.5f * b.z, b.y - 0.5f * b.w, b.x + 0.5f * b.z, b.y + 0.5f * b.w);
}

// GIoU of xyxy boxes with the criterion's clamps (criterion.py _pairwise_giou)
__device__ __forceinline__ float giou_xyxy(float4 a, float4 b, float* iou_out = nullptr) {
  const float area_a = fmaxf(a.z - a.x, 0.f) * fmaxf(a.w - a.y, 0.f);
  const float area_b = fmaxf(b.z - b.x, 0.f) * fmaxf(b.w - b.y, 0.f);
  const float iw = fmaxf(fminf(a.z, b.z) - fmaxf(a.x, b.x), 0.f);
  const float ih = fmaxf(fminf(a.w, b.w) - fmaxf(a.y, b.y), 0.f);
  const float inter = iw * ih;
  const float uni = area_a + area_b - inter;
  const float iou = inter / fmaxf(uni, 1e-9f);
  const float ew = fmaxf(fmaxf(a.z, b.z) - fminf(a.x, b.x), 0.f);
  const float eh = fmaxf(fmaxf(a.w, b.w) - fminf(a.y, b.y), 0.f);
  const float area = ew * eh;
  if (iou_out) *iou_out = iou;
  return iou - (area - uni) / fmaxf(area, 1e-9f);
}

struct RtdetrCost {
  const float* logits;  // this (s, b): [Q][C]
  const float* boxes;   // [Q][4]
  const float* tgt;     // this b: [M][4]
  const int32_t* labels;
  int C;
  __device__ __forceinline__ float operator()(int q, int m) const {
    const int c = min(max(labels[m], 0), C - 1);  // clamp(0, C - 1) as forward_padded
    const float p = 1.f / (1.f + expf(-logits[(size_t)q * C + c]));
    const float neg = (1.f - 0.25f) * (p * p) * (-logf(1.f - p + 1e-8f));
    const float pos = 0.25f * ((1.f - p) * (1.f - p)) * (-logf(p + 1e-8f));
    const float4 bq = *reinterpret_cast<const float4*>(boxes + (size_t)q * 4);
    const float4 tm = *reinterpret_cast<const float4*>(tgt + (size_t)m * 4);
    const float l1 = ((fabsf(bq.x - tm.x) + fabsf(bq.y - tm.y)) + fabsf(bq.z - tm.z)) + fabsf(bq.w - tm.w);
    const float cg = -giou_xyxy(cxcywh_xyxy(bq), cxcywh_xyxy(tm));
    return (5.f * l1 + 2.f * (pos - neg)) + 2.f * cg;
  }
};

__global__ __launch_bounds__(64) void lsap_rtdetr_kernel(CritArgs a, const int32_t* __restrict__ n_valid,
                                                         int32_t* __restrict__ assign, int32_t* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int p = blockIdx.x;  // s * B + b
  const int b = p % a.B;
  const RtdetrCost fn{a.logits + (size_t)p * a.Q * a.C, a.boxes + (size_t)p * a.Q * 4, a.tgt + (size_t)b * a.M * 4,
                      a.labels + (size_t)b * a.M, a.C};
  lsap_solve(fn, n_valid[b], a.Q, a.M, assign + (size_t)p * a.M, status, smem);
}

// torch.maximum / minimum backward: the gradient goes to the larger (smaller)
// input, half to each on a tie
__device__ __forceinline__ float max_share(float a, float b) { return a > b ? 1.f : (a == b ? 0.5f : 0.f); }
__device__ __forceinline__ float min_share(float a, float b) { return a < b ? 1.f : (a == b ? 0.5f : 0.f); }

// d giou / d (cx, cy, w, h) of the source box (target constant), reverse mode
// through the forward of giou_xyxy; clamp(min) passes where input >= min
__device__ __forceinline__ float4 giou_grad_cxcywh(float4 sb, float4 tb) {
  const float4 a = cxcywh_xyxy(sb), b = cxcywh_xyxy(tb);
  const float aw = a.z - a.x, ah = a.w - a.y, awc = fmaxf(aw, 0.f), ahc = fmaxf(ah, 0.f);
  const float area_b = fmaxf(b.z - b.x, 0.f) * fmaxf(b.w - b.y, 0.f);
  const float ltx = fmaxf(a.x, b.x), lty = fmaxf(a.y, b.y), rbx = fminf(a.z, b.z), rby = fminf(a.w, b.w);
  const float iw = rbx - ltx, ih = rby - lty, iwc = fmaxf(iw, 0.f), ihc = fmaxf(ih, 0.f);
  const float inter = iwc * ihc;
  const float uni = awc * ahc + area_b - inter, uc = fmaxf(uni, 1e-9f);
  const float ex1 = fminf(a.x, b.x), ey1 = fminf(a.y, b.y), ex2 = fmaxf(a.z, b.z), ey2 = fmaxf(a.w, b.w);
  const float ew = ex2 - ex1, eh = ey2 - ey1, ewc = fmaxf(ew, 0.f), ehc = fmaxf(eh, 0.f);
  const float area = ewc * ehc, ac = fmaxf(area, 1e-9f);
  // giou = inter / uc - (area - uni) / ac
  const float g_q = -1.f;
  float g_area = g_q / ac + g_q * (-(area - uni) / (ac * ac)) * (area >= 1e-9f ? 1.f : 0.f);
  float g_uni = g_q * (-1.f / ac);
  float g_inter = 1.f / uc;
  g_uni += -inter / (uc * uc) * (uni >= 1e-9f ? 1.f : 0.f);
  const float g_area_a = g_uni;
  g_inter += -g_uni;
  const float g_iw = g_inter * ihc * (iw >= 0.f ? 1.f : 0.f);
  const float g_ih = g_inter * iwc * (ih >= 0.f ? 1.f : 0.f);
  float gx1 = 0.f, gy1 = 0.f, gx2 = 0.f, gy2 = 0.f;
  gx2 += g_iw * min_share(a.z, b.z);  // rbx = min(a2, b2)
  gx1 += -g_iw * max_share(a.x, b.x); // ltx = max(a0, b0)
  gy2 += g_ih * min_share(a.w, b.w);
  gy1 += -g_ih * max_share(a.y, b.y);
  const float g_aw = g_area_a * ahc * (aw >= 0.f ? 1.f : 0.f);
  const float g_ah = g_area_a * awc * (ah >= 0.f ? 1.f : 0.f);
  gx2 += g_aw; gx1 -= g_aw; gy2 += g_ah; gy1 -= g_ah;
  const float g_ew = g_area * ehc * (ew >= 0.f ? 1.f : 0.f);
  const float g_eh = g_area * ewc * (eh >= 0.f ? 1.f : 0.f);
  gx2 += g_ew * max_share(a.z, b.z);  // ex2 = max(a2, b2)
  gx1 += -g_ew * min_share(a.x, b.x); // ex1 = min(a0, b0)
  gy2 += g_eh * max_share(a.w, b.w);
  gy1 += -g_eh * min_share(a.y, b.y);
  return make_float4(gx1 + gx2, gy1 + gy2, 0.5f * (gx2 - gx1), 0.5f * (gy2 - gy1));
}

__device__ __forceinline__ float block_sum256(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// One block per prediction set.  comps[s] = {VFL, L1, GIoU} / num_boxes;
// d_logits[s] = d VFL / d logits; d_boxes_l1[s], d_boxes_giou[s] = d L1, d GIoU / d boxes.
__global__ __launch_bounds__(256) void set_loss_kernel(CritArgs a, const int32_t* __restrict__ n_valid,
                                                       const int32_t* __restrict__ assign,
                                                       const float* __restrict__ num_boxes, float vfl_alpha,
                                                       float* __restrict__ comps, float* __restrict__ d_logits,
                                                       float* __restrict__ d_l1, float* __restrict__ d_giou) {
  extern __shared__ float s_score[];  // [B][Q][C] VFL target score (IoU at the matched (q, label)), -1 = unmatched
  __shared__ float red[4];
  const int s = blockIdx.x, tid = threadIdx.x;
  const int BQC = a.B * a.Q * a.C, BQ = a.B * a.Q;
  const float inv_nb = 1.f / *num_boxes;
  for (int i = tid; i < BQC; i += 256) s_score[i] = -1.f;
  float* dl1 = d_l1 + (size_t)s * BQ * 4;
  float* dgi = d_giou + (size_t)s * BQ * 4;
  for (int i = tid; i < BQ * 4; i += 256) {
    dl1[i] = 0.f;
    dgi[i] = 0.f;
  }
  __syncthreads();
  // matched pairs: L1 + GIoU (+ gradients), VFL target scores
  float l1_acc = 0.f, gi_acc = 0.f;
  for (int i = tid; i < a.B * a.M; i += 256) {
    const int b = i / a.M, m = i % a.M;
    if (m >= n_valid[b]) continue;
    const int q = assign[((size_t)s * a.B + b) * a.M + m];
    if (q < 0) continue;
    const size_t bq = ((size_t)s * a.B + b) * a.Q + q;
    const float4 sb = *reinterpret_cast<const float4*>(a.boxes + bq * 4);
    const float4 tb = *reinterpret_cast<const float4*>(a.tgt + ((size_t)b * a.M + m) * 4);
    const float dx = sb.x - tb.x, dy = sb.y - tb.y, dw = sb.z - tb.z, dh = sb.w - tb.w;
    l1_acc += ((fabsf(dx) + fabsf(dy)) + fabsf(dw)) + fabsf(dh);
    float iou;
    const float giou = giou_xyxy(cxcywh_xyxy(sb), cxcywh_xyxy(tb), &iou);
    gi_acc += 1.f - giou;
    const size_t lq = (size_t)(b * a.Q + q) * 4;
    dl1[lq + 0] = (dx > 0.f ? 1.f : (dx < 0.f ? -1.f : 0.f)) * inv_nb;
    dl1[lq + 1] = (dy > 0.f ? 1.f : (dy < 0.f ? -1.f : 0.f)) * inv_nb;
    dl1[lq + 2] = (dw > 0.f ? 1.f : (dw < 0.f ? -1.f : 0.f)) * inv_nb;
    dl1[lq + 3] = (dh > 0.f ? 1.f : (dh < 0.f ? -1.f : 0.f)) * inv_nb;
    const float4 gg = giou_grad_cxcywh(sb, tb);  // d giou; the loss is 1 - giou
    dgi[lq + 0] = -gg.x * inv_nb;
    dgi[lq + 1] = -gg.y * inv_nb;
    dgi[lq + 2] = -gg.z * inv_nb;
    dgi[lq + 3] = -gg.w * inv_nb;
    s_score[(size_t)(b * a.Q + q) * a.C + min(max(a.labels[(size_t)b * a.M + m], 0), a.C - 1)] = iou;
  }
  __syncthreads();
  // varifocal loss over every (b, q, c): w * BCE(x, t), w = alpha p^2 (1 - onehot) + t (detached)
  float vfl_acc = 0.f;
  const float* lg = a.logits + (size_t)s * BQC;
  float* dlg = d_logits + (size_t)s * BQC;
  for (int i = tid; i < BQC; i += 256) {
    const float x = lg[i];
    const float sc = s_score[i];
    const float t = sc >= 0.f ? sc : 0.f, onehot = sc >= 0.f ? 1.f : 0.f;
    const float p = 1.f / (1.f + expf(-x));
    const float w = vfl_alpha * (p * p) * (1.f - onehot) + t;
    const float mx = fmaxf(-x, 0.f);
    const float bce = (1.f - t) * x + mx + logf(expf(-mx) + expf(-x - mx));
    vfl_acc += w * bce;
    dlg[i] = w * (p - t) * inv_nb;
  }
  const float vfl = block_sum256(vfl_acc, red);
  const float l1 = block_sum256(l1_acc, red);
  const float gl = block_sum256(gi_acc, red);
  if (tid == 0) {
    comps[s * 3 + 0] = vfl * inv_nb;
    comps[s * 3 + 1] = l1 * inv_nb;
    comps[s * 3 + 2] = gl * inv_nb;
  }
}

// backward: d logits = g[s,0] d_logits; d boxes = g[s,1] d_l1 + g[s,2] d_giou
__global__ __launch_bounds__(256) void set_loss_bwd_kernel(const float* __restrict__ g, int S, long long per_set_l,
                                                           long long per_set_b, const float* __restrict__ d_logits,
                                                           const float* __restrict__ d_l1,
                                                           const float* __restrict__ d_giou,
                                                           float* __restrict__ g_logits, float* __restrict__ g_boxes) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long nl = S * per_set_l, nb = S * per_set_b;
  if (i < nl) g_logits[i] = g[(i / per_set_l) * 3 + 0] * d_logits[i];
  if (i < nb) {
    const long long s = i / per_set_b;
    g_boxes[i] = g[s * 3 + 1] * d_l1[i] + g[s * 3 + 2] * d_giou[i];
  }
}

}  // namespace moe

using namespace moe;

extern "C" int rtdetr_hungarian_match(const float* cost, const int32_t* n_valid, int S, int B, int Q, int M,
                                      int32_t* assign, int32_t* status, hipStream_t stream) {
  if (S < 1 || B < 1 || Q < 1 || M < 1 || Q > 4096 || M > 1024)
    return fail("rtdetr_hungarian_match: need S, B >= 1, 1 <= Q <= 4096, 1 <= M <= 1024");
  if (cost == nullptr || n_valid == nullptr || assign == nullptr || status == nullptr)
    return fail("rtdetr_hungarian_match: NULL pointer");
  const size_t shmem = (size_t)M * 8 + 2 * (size_t)Q * 8 + 3 * (size_t)Q * 4 + (size_t)M * 4 + (size_t)M + Q + 16;
  if (shmem > 64 * 1024) return fail("rtdetr_hungarian_match: Q/M too large for LDS");
  ProfScope prof(stream, PROF_MATCH, 4.0 * S * B * Q * M + 4.0 * S * B * M);
  MOE_LAUNCH(prof, lsap_kernel, dim3(S * B), dim3(64), shmem, stream, cost, n_valid, B, Q, M, assign, status);
  return check_launch("rtdetr_hungarian_match");
}

static size_t lsap_smem(int Q, int M) {
  return (size_t)M * 8 + 2 * (size_t)Q * 8 + 3 * (size_t)Q * 4 + (size_t)M * 4 + (size_t)M + Q + 16;
}

extern "C" int rtdetr_set_criterion_match(const float* logits, const float* boxes, const float* tgt_boxes,
                                          const int32_t* tgt_labels, const int32_t* n_valid, int S, int B, int Q,
                                          int C, int M, int32_t* assign, int32_t* status, hipStream_t stream) {
  if (S < 1 || B < 1 || Q < 1 || C < 1 || M < 1 || Q > 4096 || M > 1024)
    return fail("rtdetr_set_criterion_match: bad shape");
  if (!logits || !boxes || !tgt_boxes || !tgt_labels || !n_valid || !assign || !status)
    return fail("rtdetr_set_criterion_match: NULL pointer");
  const size_t shmem = lsap_smem(Q, M);
  if (shmem > 64 * 1024) return fail("rtdetr_set_criterion_match: Q/M too large for LDS");
  CritArgs a{logits, boxes, tgt_boxes, tgt_labels, S, B, Q, C, M};
  ProfScope prof(stream, PROF_MATCH, 4.0 * S * B * Q * (C + 4) + 20.0 * B * M);
  MOE_LAUNCH(prof, lsap_rtdetr_kernel, dim3(S * B), dim3(64), shmem, stream, a, n_valid, assign, status);
  return check_launch("rtdetr_set_criterion_match");
}

extern "C" int rtdetr_set_criterion_loss(const float* logits, const float* boxes, const float* tgt_boxes,
                                         const int32_t* tgt_labels, const int32_t* n_valid, const int32_t* assign,
                                         const float* num_boxes, float vfl_alpha, int S, int B, int Q, int C, int M,
                                         float* comps, float* d_logits, float* d_l1, float* d_giou,
                                         hipStream_t stream) {
  if (S < 1 || B < 1 || Q < 1 || C < 1 || M < 1) return fail("rtdetr_set_criterion_loss: bad shape");
  if ((size_t)B * Q * C * 4 > 64 * 1024) return fail("rtdetr_set_criterion_loss: B*Q*C must fit 64 KiB of LDS");
  CritArgs a{logits, boxes, tgt_boxes, tgt_labels, S, B, Q, C, M};
  ProfScope prof(stream, PROF_MATCH, 8.0 * S * B * Q * (C + 8) + 40.0 * S * B * M);
  MOE_LAUNCH(prof, set_loss_kernel, dim3(S), dim3(256), (size_t)B * Q * C * 4, stream, a, n_valid, assign,
             num_boxes, vfl_alpha, comps, d_logits, d_l1, d_giou);
  return check_launch("rtdetr_set_criterion_loss");
}

extern "C" int rtdetr_set_criterion_loss_bwd(const float* g_comps, int S, int B, int Q, int C, const float* d_logits,
                                             const float* d_l1, const float* d_giou, float* g_logits,
                                             float* g_boxes, hipStream_t stream) {
  if (S < 1 || B < 1 || Q < 1 || C < 1) return fail("rtdetr_set_criterion_loss_bwd: bad shape");
  const long long pl = (long long)B * Q * C, pb = (long long)B * Q * 4;
  const long long n = S * (pl > pb ? pl : pb);
  ProfScope prof(stream, PROF_MATCH, 8.0 * S * (pl + 3 * pb));
  MOE_LAUNCH(prof, set_loss_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, g_comps, S, pl, pb,
             d_logits, d_l1, d_giou, g_logits, g_boxes);
  return check_launch("rtdetr_set_criterion_loss_bwd");
}
