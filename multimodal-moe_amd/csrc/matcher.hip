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

__global__ __launch_bounds__(64) void lsap_kernel(const float* __restrict__ cost, const int32_t* __restrict__ n_valid,
                                                  int B, int Q, int M, int32_t* __restrict__ assign,
                                                  int32_t* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
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
  const int p = blockIdx.x;
  const int n = n_valid[p % B];
  const float* C = cost + (size_t)p * Q * M;  // cost(row m, col q) = C[q * M + m]
  int32_t* out = assign + (size_t)p * M;
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
        const double r = minval + (double)(tr ? C[(size_t)j * M + i] : C[(size_t)i * M + j]) - ui - v[j];
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
