// Row-wise top-k of fp32 scores for RT-DETR's query selection (SURVEY.md
// 8(f).1: the decoder keeps the k = 300 best-scoring of S = 19,320 memory
// tokens per image -- torch.topk ran it as one single-workgroup sort per row,
// 128 us for 8 rows).  One workgroup of 1,024 threads per row, the row staged
// in LDS as order-preserving uint32 keys:
//   1. radix select, 4 passes of 8 bits (MSB first): a 256-bin LDS histogram
//      of the keys matching the prefix found so far, then the digit at which
//      the count from the top reaches k -> T, the k-th largest key, and r, the
//      number of keys equal to T that belong to the top k;
//   2. ordered compaction in index order (wave ballots + a scan over the 16
//      waves): every key > T and the first r keys == T;
//   3. bitonic sort of the k candidates in LDS, key descending, index
//      ascending (ties: the lower index first).
// Deterministic (no atomics decide the output), sorted like torch.topk(...,
// sorted=True); which of several equal scores is kept is defined here (lower
// index), where torch leaves it unspecified.
#include "moe_common.h"
#include "prof.h"

namespace moe {

constexpr int kTopkThreads = 1024;
constexpr int kTopkMaxN = 32768;  // keys staged in LDS (128 KiB)
constexpr int kTopkMaxK = 1024;

__device__ __forceinline__ uint32_t order_key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // ascending uint order = ascending float order
}

__global__ __launch_bounds__(kTopkThreads) void topk_rows_kernel(const float* __restrict__ x, int n, int k,
                                                                long long* __restrict__ idx_out,
                                                                float* __restrict__ val_out) {
  extern __shared__ uint32_t keys[];  // [n]
  __shared__ int hist[256];
  __shared__ int s_digit, s_above;
  __shared__ int wave_cnt[2][kTopkThreads / 64];
  __shared__ uint32_t ck[kTopkMaxK];
  __shared__ int ci[kTopkMaxK];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* row = x + (size_t)blockIdx.x * n;
  for (int i = tid; i < n; i += kTopkThreads) keys[i] = order_key(row[i]);
  uint32_t prefix = 0, pmask = 0;
  int krem = k;  // how many of the keys matching the prefix still belong to the top k
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int b = tid; b < 256; b += kTopkThreads) hist[b] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += kTopkThreads) {
      const uint32_t u = keys[i];
      if ((u & pmask) == prefix) atomicAdd(&hist[(u >> shift) & 255], 1);
    }
    __syncthreads();
    if (tid == 0) {  // from the top digit down: the digit where the running count reaches krem
      int above = 0, d = 255;
      for (; d > 0; --d) {
        if (above + hist[d] >= krem) break;
        above += hist[d];
      }
      s_digit = d;
      s_above = above;
    }
    __syncthreads();
    prefix |= (uint32_t)s_digit << shift;
    pmask |= 255u << shift;
    krem -= s_above;
    __syncthreads();
  }
  const uint32_t T = prefix;  // the k-th largest key; krem keys equal to T are taken (lowest indices)
  // compaction (the sort below orders the candidates): every key > T into
  // slots [0, k - krem) in any order, then the krem keys == T with the lowest
  // indices into [k - krem, k) -- their rank in index order from wave ballots
  // and a scan over the 16 waves of each 1,024-index chunk
  const int ngt = k - krem;
  int gt_seen = 0, eq_seen = 0;
  const unsigned long long below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  for (int base = 0; base < n; base += kTopkThreads) {
    const int i = base + tid;
    const uint32_t u = i < n ? keys[i] : 0u;
    const bool gt = i < n && u > T, eq = i < n && u == T;
    const unsigned long long bg = __ballot(gt), be = __ballot(eq);
    if (lane == 0) {
      wave_cnt[0][wave] = __popcll(bg);
      wave_cnt[1][wave] = __popcll(be);
    }
    __syncthreads();
    int gbase = 0, ebase = 0, gtot = 0, etot = 0;
    for (int w = 0; w < kTopkThreads / 64; ++w) {
      if (w < wave) {
        gbase += wave_cnt[0][w];
        ebase += wave_cnt[1][w];
      }
      gtot += wave_cnt[0][w];
      etot += wave_cnt[1][w];
    }
    if (gt) {
      const int slot = gt_seen + gbase + __popcll(bg & below);
      ck[slot] = u;
      ci[slot] = i;
    } else if (eq) {
      const int r = eq_seen + ebase + __popcll(be & below);
      if (r < krem) {
        ck[ngt + r] = u;
        ci[ngt + r] = i;
      }
    }
    gt_seen += gtot;
    eq_seen += etot;
    __syncthreads();  // wave_cnt is rewritten by the next chunk
  }
  // bitonic sort of the k candidates (padded to a power of two): key descending, index ascending
  int P = 1;
  while (P < k) P <<= 1;
  for (int s = k + tid; s < P; s += kTopkThreads) {
    ck[s] = 0u;
    ci[s] = 0x7fffffff;
  }
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < P / 2; t += kTopkThreads) {
        const int a = 2 * t - (t & (stride - 1)), b = a + stride;
        const bool desc = (a & size) == 0;  // first half of each block sorts "before" order
        const uint32_t ka = ck[a], kb = ck[b];
        const int ia = ci[a], ib = ci[b];
        const bool a_first = ka > kb || (ka == kb && ia < ib);  // a precedes b in the output order
        if (a_first != desc) {
          ck[a] = kb;
          ck[b] = ka;
          ci[a] = ib;
          ci[b] = ia;
        }
      }
      __syncthreads();
    }
  }
  for (int s = tid; s < k; s += kTopkThreads) {
    idx_out[(size_t)blockIdx.x * k + s] = ci[s];
    if (val_out != nullptr) val_out[(size_t)blockIdx.x * k + s] = row[ci[s]];
  }
}

}  // namespace moe

using namespace moe;

extern "C" int rtdetr_topk_rows(const float* x, int rows, int n, int k, long long* idx, float* val, hipStream_t stream) {
  if (rows < 0 || n <= 0 || k <= 0 || k > n || k > kTopkMaxK || n > kTopkMaxN)
    return fail("rtdetr_topk_rows: needs 0 < k <= min(n, 1024) and n <= 32768");
  if (rows == 0) return 0;
  if (x == nullptr || idx == nullptr) return fail("rtdetr_topk_rows: null pointer");
  static unsigned long long attr_done = 0;  // per-device bitmask
  const size_t lds = (size_t)n * sizeof(uint32_t);
  if (int rc = allow_dyn_lds(reinterpret_cast<const void*>(topk_rows_kernel), (int)(kTopkMaxN * sizeof(uint32_t)),
                             &attr_done, "rtdetr_topk_rows"))
    return rc;
  ProfScope prof(stream, PROF_ROUTER, 4.0 * rows * n + 8.0 * rows * k);
  MOE_LAUNCH(prof, topk_rows_kernel, dim3(rows), dim3(kTopkThreads), lds, stream, x, n, k, idx, val);
  return check_launch("rtdetr_topk_rows");
}
