/*
 * moe_hip.h -- C-ABI of libmoe_hip.so, the MI355X (gfx950) kernels of the
 * context-aware MoE FFN that sits inside the RT-DETR encoder (AIFI) and
 * decoder layers.
 *
 * Boundary.  The reference (scaleoutsystems/multimodal-MoE @2026-02-20) has no
 * native code and no FFI: its operator API is the Python module
 * src/models/vision/rtdetr.py (RtdetrTrainConfig :36-48, train_rtdetr_detector
 * :77-95, eval_rtdetr_detector :98-128), whose engine (Ultralytics RTDETR,
 * :58-64, :82-94, :112-127) owns the transformer FFN that this library
 * replaces.  The MoE itself is planned but unwritten in the reference
 * (notes/MoE_in_ZOD_Thesis_Proposal_revisedTimeline.txt:214-220: "expert
 * modules, gating module, routing utilities (e.g., Top-k routing), and
 * load-balancing terms"), with context as an additive router bias
 * (notes/related_work.md:64-68) and the context id from
 * scripts/add_solar_context_bins.py:87-107.  Each entry point below names the
 * row of SURVEY.md section 8(a) it implements; INTEGRATION.md shows the ctypes
 * binding the Python side uses.
 *
 * Conventions (all entry points):
 *   - every pointer is a DEVICE pointer owned by the caller (torch allocator);
 *     nothing is allocated, freed or synchronised inside; work is ordered on
 *     `stream` only, so every call is hipGraph-capturable;
 *   - bf16 tensors are passed as `const void*` (raw 16-bit storage);
 *   - return 0 on success, a negative code on failure: -1 bad shape/argument,
 *     -(1000 + hipError_t) for a HIP launch error; moe_last_error() returns a
 *     thread-local message for the last failure;
 *   - no host<->device copies: hist/offsets stay on the device.
 *
 * Shapes: T tokens, d model width (multiple of 128, <= 1024), E experts
 * (1..64), k slots (1..8, k <= E), F expert hidden width (multiple of 128).
 */
#ifndef MOE_HIP_H_
#define MOE_HIP_H_

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Number of router blocks (16 tokens each) for T tokens (size of the
 * per-block workspaces below). */
int moe_router_num_blocks(int T);

/* a2+a3: router logits, fp32 softmax, top-k, gates, per-block
 * routing counts and aux-loss partials, fused.
 *   logits[t,e] = sum_c x[t,c] * wg[e,c] + ctx_bias[ctx_img[t / tokens_per_image], e]
 *   probs = softmax(logits) (fp32), lse[t] = logsumexp(logits[t])
 *   topk_idx[t,j], j=0..k-1: experts by descending prob, ties -> lower index
 *   topk_w[t,j] = probs[t, idx] (normalize==0 or k==1) or renormalised to sum 1
 *   local_rank[t,j] = #{t' < t in the same router block : idx[t',j] == idx[t,j]}
 *   block_counts[b, j, e] = #{t in block b : idx[t,j] == e}
 *   aux_partials[b, e] = sum_{t in b} probs[t,e]; aux_partials[b, E] = sum lse^2
 * x: bf16 [T,d]; wg: fp32 [E,d]; ctx_bias: fp32 [n_ctx,E] (n_ctx E <= 4096) or
 * NULL; ctx_img: int32 [T/tokens_per_image] or NULL. Workspaces sized by
 * moe_router_num_blocks(T). */
int moe_router_topk_fwd(const void* x, const float* wg, const float* ctx_bias,
                        const int32_t* ctx_img, int n_ctx, int tokens_per_image,
                        int T, int d, int E, int k, int normalize,
                        int32_t* topk_idx, float* topk_w, float* probs, float* lse,
                        int32_t* local_rank, int32_t* block_counts,
                        float* aux_partials, hipStream_t stream);

/* a4, index half: exclusive scans of the block counts.
 * Assignment (t,j) to expert e has rank r = slot_base[j,e] + sum_{b'<b}
 * block_counts[b',j,e] + local_rank[t,j] (slot-major, then token order; this
 * is the capacity priority).  kept_e = min(hist_e, cap) (cap <= 0: no limit).
 * Outputs: rank_base[b,j,e] (int32 [nblk,k,E]), hist[e] (unclipped counts),
 * offsets[0..E] = exclusive scan of kept counts (offsets[E] = rows in Xp). */
int moe_route_scan(const int32_t* block_counts, int nblk, int k, int E, int cap,
                   int32_t* rank_base, int32_t* hist, int32_t* offsets,
                   hipStream_t stream);

/* a4, data half: scatter token rows into the expert-contiguous
 * buffer.  pos[t,j] = offsets[e] + r if r < cap else -1;  xp[pos[t,j]] = x[t].
 * x: bf16 [T,d]; xp: bf16 [>= offsets[E], d]; pos: int32 [T,k]. */
int moe_permute_fwd(const void* x, const int32_t* topk_idx, const int32_t* local_rank,
                    const int32_t* rank_base, const int32_t* offsets,
                    int T, int d, int E, int k, int cap,
                    void* xp, int32_t* pos, hipStream_t stream);

/* a4, index half without the row copy: pos[t,j] as
 * moe_permute_fwd, and src_tok[pos[t,j]] = t for every kept assignment
 * (int32 [>= offsets[E]]).  The bf16 expert GEMMs read routed row r as token
 * row src_tok[r] (moe_grouped_gemm_gather / _wgrad_gather): the permuted copy
 * of x never exists in HBM. */
int moe_route_index(const int32_t* topk_idx, const int32_t* local_rank, const int32_t* rank_base,
                    const int32_t* offsets, int T, int E, int k, int cap, int32_t* pos, int32_t* src_tok,
                    hipStream_t stream);

/* a3 + a4 in ONE launch, from the router's outputs: the
 * moe_route_scan totals and prefixes (recomputed per 16-token router block
 * from block_counts, so no second pass), hist / offsets, pos and src_tok as
 * moe_route_index, optionally row_gate[pos[t,j]] = topk_w[t,j] (fp32 [>=
 * offsets[E]]) and the aux losses of moe_aux_loss_fwd (aux_out3 / wcoef /
 * aux_partials non-NULL together).  nblk = moe_router_num_blocks(T). */
int moe_route_dispatch(const int32_t* block_counts, int nblk, int T, int k, int E, int cap,
                       const int32_t* topk_idx, const int32_t* local_rank, const float* topk_w,
                       const float* aux_partials, float lb_coef, float z_coef, int32_t* hist, int32_t* offsets,
                       int32_t* pos, int32_t* src_tok, float* row_gate, float* aux_out3, float* wcoef,
                       hipStream_t stream);

/* a6: y[t] = sum_j topk_w[t,j] * yp[pos[t,j]] (pos<0 skipped),
 * fp32 accumulation, bf16 out. */
int moe_combine_fwd(const void* yp, const int32_t* pos, const float* topk_w,
                    int T, int d, int k, void* y, hipStream_t stream);

/* a6 + the caller's residual branch (the AIFI and
 * decoder layers compute norm(x + FFN(x))): y[t] = resid[t] + sum_j ...,
 * summed in fp32 and rounded to bf16 once; resid bf16 [T,d] or NULL (then
 * moe_combine_fwd).  Removes the separate residual add of every MoE layer. */
int moe_combine_res_fwd(const void* yp, const int32_t* pos, const float* topk_w, const void* resid,
                        int T, int d, int k, void* y, hipStream_t stream);

/* a7, combine transpose: dyp[pos[t,j]] = topk_w[t,j] * dy[t] (bf16)
 * and dw[t,j] = <dy[t], yp[pos[t,j]]> (fp32; 0 when dropped). */
int moe_combine_bwd(const void* dy, const void* yp, const int32_t* pos,
                    const float* topk_w, int T, int d, int k,
                    void* dyp, float* dw, hipStream_t stream);

/* a7, dispatch transpose + router backward, fused per token:
 *   dprobs[t,e]  = d(topk gates)/d(probs) applied to dw, plus dprob_bias[e]
 *   dlogits[t,e] = softmax_bwd(probs[t], dprobs[t]) + zc * lse[t] * probs[t,e]
 *   dx[t,c]      = sum_j dxp[pos[t,j], c] + sum_e dlogits[t,e] * wg[e,c]
 * dprob_bias: fp32 [E] or NULL (load-balance grad); zc: one fp32 on the
 * device (z-loss grad scale, 2 * dL/dz / T) or NULL for 0 -- a device scalar so
 * that the backward never synchronises with the host.
 * dx: bf16 [T,d]; dlogits: fp32 [T,E]. */
int moe_token_bwd(const void* dxp, const int32_t* pos, const float* probs,
                  const int32_t* topk_idx, const float* topk_w, const float* dw,
                  const float* lse, const float* dprob_bias, const float* zc,
                  const float* wg, int T, int d, int E, int k, int normalize,
                  void* dx, float* dlogits, hipStream_t stream);
/* Same, with the combine transpose's gate gradient formed here when dw is
 * NULL: dw[t,j] = <dy[t], yp[pos[t,j]]> (dy bf16 [T,d], yp bf16 [rows,d]),
 * optionally stored to dw_out fp32 [T,k] -- the single-GPU backward then has
 * no combine_bwd launch (dYp is formed inside moe_grouped_gemm_bwd_pair). */
int moe_token_bwd_dw(const void* dxp, const int32_t* pos, const float* probs,
                     const int32_t* topk_idx, const float* topk_w, const float* dw,
                     const void* dy, const void* yp, float* dw_out,
                     const float* lse, const float* dprob_bias, const float* zc,
                     const float* wg, int T, int d, int E, int k, int normalize,
                     void* dx, float* dlogits, hipStream_t stream);

/* moe_token_bwd_dw plus a residual gradient: dx[t] += dres[t] (bf16 [T,d]
 * or NULL), inside the same fp32 sum -- with moe_combine_res_fwd the layer's
 * dx = dy + dispatch transpose + router term, so autograd never accumulates
 * the residual branch's gradient with a separate add. */
int moe_token_bwd_res(const void* dxp, const int32_t* pos, const float* probs,
                      const int32_t* topk_idx, const float* topk_w, const float* dw,
                      const void* dy, const void* yp, float* dw_out, const void* dres,
                      const float* lse, const float* dprob_bias, const float* zc,
                      const float* wg, int T, int d, int E, int k, int normalize,
                      void* dx, float* dlogits, hipStream_t stream);

/* Router weight gradients after moe_token_bwd_*: dwg fp32 [E,d] = dlogits^T x
 * (dlogits fp32 [T,E] from token_bwd, x bf16 [T,d] the router input, T = B
 * tpi image-major, d % 8 == 0, x and dlogits 16-B aligned) and, when dcb is
 * not NULL, the context-bias gradient dcb fp32 [C,E]: row c = the sum of
 * dlogits over the tokens of the images with ctx_img[b] == c.  One launch,
 * fixed-order sums (bitwise repeatable; replaces a torch fp32 GEMM and an
 * atomic index_add).  part: reserved, pass NULL (moe_router_wgrad_workspace
 * returns 0; a chunked variant that used it was measured no faster at C2 and
 * removed in round 5).
 * Reference: the router backward of SURVEY 8(a) row a7. */
long long moe_router_wgrad_workspace(int B, int tpi, int E, int d);
int moe_router_wgrad(const float* dlogits, const void* x, const int32_t* ctx_img, int B, int tpi, int E, int d,
                     int C, float* part, float* dwg, float* dcb, hipStream_t stream);

/* Grouped GEMM data types / epilogues.  MOE_BIAS_BF16 OR'd into the dtype of
 * moe_grouped_gemm / moe_grouped_gemm_gather: the bias epilogues read a bf16
 * bias [G][N] (the bf16 parameter itself; no fp32 copy per call). */
enum moe_dtype { MOE_BF16 = 0, MOE_FP8_E4M3 = 1, MOE_BIAS_BF16 = 0x100, MOE_DENSE_LAYER = 0x200 };
/* MOE_DENSE_LAYER OR'd into moe_grouped_gemm / _gather's dtype: the call is a
 * dense (non-expert) layer run on the grouped GEMM with G = 1 (the detector's
 * MLP heads); same arithmetic, counted by the library profiler with the dense
 * linears (kind 11) instead of the expert GEMMs. */
enum moe_epilogue {
  MOE_EPI_NONE = 0,      /* C = A.B                                   */
  MOE_EPI_BIAS = 1,      /* C = A.B + bias[g, n]                      */
  MOE_EPI_BIAS_RELU = 2, /* C = relu(A.B + bias[g, n])                */
  MOE_EPI_RELU_MASK = 3, /* C = (A.B) * (aux[row, n] > 0)   (dgrad)   */
  MOE_EPI_RELU_MASK_MX = 4 /* same, aux is e4m3 [rows, N] (byte > +0)  */
};

/* a5/a7, rows-grouped GEMM (expert FFN forward and dgrad):
 * for every group g with rows [offsets[g], offsets[g+1]):
 *   C[r, n] = epi( sum_k A[r, k] * B_g(k, n) ),   r in group g
 * A: bf16 [rows, K] row-major.  B_g = b + g * K * N:
 *   trans_b = 1: stored [N][K] (nn.Linear weight; forward),
 *   trans_b = 0: stored [K][N] (dgrad through the same weight).
 * bias: fp32 [G, N] (EPI_BIAS*); aux: bf16 [rows, N] (EPI_RELU_MASK) or e4m3
 * [rows, N] (EPI_RELU_MASK_MX; sign/zero only, no exponents needed).
 * C: bf16 [rows, N].  K, N multiples of 64; offsets int32 [G+1] on device;
 * max_rows is a host upper bound of offsets[G] (grid sizing, no sync). */
int moe_grouped_gemm(int dtype /* MOE_BF16; fp8: moe_grouped_gemm_mx */, const void* a, const void* b, void* c,
                     const int32_t* offsets, int G, int max_rows, int N, int K,
                     int trans_b, int epilogue, const float* bias, const void* aux,
                     const float* scales, hipStream_t stream);

/* a7, expert weight gradient (K = the group's rows):
 *   C_g[m, n] = sum_{r in group g} X[r, m] * Y[r, n]     (fp32 [G, M, N])
 *   colsum_g[m] = sum_{r in group g} X[r, m]             (fp32 [G, M], optional)
 * X: bf16 [rows, M]; Y: bf16 [rows, N]; M, N multiples of 64.
 * (dW2 = dYp^T H with colsum = db2; dW1 = dH^T Xp with colsum = db1.) */
int moe_grouped_gemm_wgrad(int dtype, const void* x, const void* y, float* c,
                           float* colsum, const int32_t* offsets, int G,
                           int M, int N, hipStream_t stream);
/* Same, with rows_hint = a host upper bound of offsets[G] (0: unknown) and
 * out_bf16 = 1 to write C and colsum as bf16 (RNE of the fp32 sums; the
 * gradients of bf16 expert weights, no separate cast pass).  The launch splits
 * each group's K range over 2 workgroups (split-K, see
 * moe_set_splitk_workspace) when the groups average >= 1024 rows. */
int moe_grouped_gemm_wgrad_rows(int dtype, const void* x, const void* y, void* c,
                                void* colsum, const int32_t* offsets, int G, int M,
                                int N, int rows_hint, int out_bf16, hipStream_t stream);

/* moe_grouped_gemm with routed row r of A read as a[a_gather[r]] (a: bf16
 * [T, K] token rows; a_gather: int32 [>= offsets[G]], moe_route_index's
 * src_tok); a_gather == NULL is moe_grouped_gemm. */
int moe_grouped_gemm_gather(int dtype, const void* a, const int32_t* a_gather, const void* b, void* c,
                            const int32_t* offsets, int G, int max_rows, int N, int K, int trans_b,
                            int epilogue, const float* bias, const void* aux, hipStream_t stream);
/* moe_grouped_gemm_gather whose output row r is stored at row c_rows[r] of c
 * (the expert-parallel received layout, like moe_expert_ffn_fwd's yp_rows):
 * the second expert GEMM of the two-launch EP forward for layers with few rows
 * per expert (src/moe/ep.py).  Rows of c no r maps to are left untouched. */
int moe_grouped_gemm_scatter(int dtype, const void* a, const int32_t* a_gather, const void* b, void* c,
                             const int32_t* c_rows, const int32_t* offsets, int G, int max_rows, int N, int K,
                             int trans_b, int epilogue, const float* bias, const void* aux, hipStream_t stream);
/* a5: the expert FFN forward in ONE launch,
 *   h  = relu(x[src_tok[r]] . W1_g^T + b1_g)   bf16 [>= offsets[G], F]
 *   yp = h . W2_g^T + b2_g                      bf16 [>= offsets[G], d]
 * for the routed rows r of every expert g (src_tok == NULL: x holds the
 * routed rows themselves).  Same contract as moe_grouped_gemm_gather(EPI_BIAS_RELU)
 * followed by moe_grouped_gemm(EPI_BIAS) on h, without h's second pass:
 * h is written once (the backward's mask / dW2 operand) and never read here.
 * w1 bf16 [G, F, d], w2 bf16 [G, d, F]; b1 [G, F], b2 [G, d] fp32, or bf16
 * with MOE_BIAS_BF16 in dtype.  Needs moe_expert_ffn_supported(G, F, d)
 * (d == 256, F % 128 == 0 and F <= 2048, G <= 64) and 16-B aligned operands.
 * The reference has no MoE: the expert is "a standard MLP block"
 * (notes/related_work.md:23). */
int moe_expert_ffn_supported(int G, int F, int d);
int moe_expert_ffn_fwd(int dtype, const void* x, const int32_t* src_tok, const void* w1, const void* b1,
                       const void* w2, const void* b2, const int32_t* offsets, int G, int max_rows, int F, int d,
                       void* h, void* yp, const int32_t* yp_rows, int yp_n, hipStream_t stream);
/* (yp_rows, yp_n): NULL, ignored -> yp row r is routed row r; else routed row
 * r is stored at yp row yp_rows[r] of the yp_n-row buffer (the expert-parallel
 * received layout: moe_ep_compaction's gather map), rows of yp that no routed
 * row maps to are left untouched. */

/* Expert-parallel receive map (src/moe/ep.py): rank r
 * received, from source w, recv_cnt[w El + e] rows for local expert e (capped
 * at S), held at received row (w El + e) S + j.  Writes offsets int32 [El + 1]
 * (expert-major compact order, sources in rank order inside an expert) and
 * gather int32 [>= W El S]: compact row -> received row (the expert GEMMs read
 * the received rows through it and write back through it), and, when
 * overflow != NULL, *overflow = sum_e max(hist[e] - S, 0) of this rank's send
 * histogram hist int32 [E] (assignments the fixed-capacity exchange dropped).
 * One launch, no host sync.  Replaces a chain of torch index ops. */
int moe_ep_compaction(const int32_t* recv_cnt, const int32_t* hist, int W, int El, int E, int S, int32_t* gather,
                      int32_t* offsets, int32_t* overflow, hipStream_t stream);
/* moe_grouped_gemm_wgrad_rows with k-row r of Y read as y[y_gather[r]]
 * (dW1 = dH^T Xp from the token rows); y_gather == NULL: contiguous. */
int moe_grouped_gemm_wgrad_gather(int dtype, const void* x, const void* y, const int32_t* y_gather, void* c,
                                  void* colsum, const int32_t* offsets, int G, int M, int N, int rows_hint,
                                  int out_bf16, hipStream_t stream);
/* A dense linear layer's weight and bias gradients in one launch (the
 * decoder/encoder TokenLinear backward; replaces the two torch ops
 * dW = dy^T x, db = dy.sum(0) of nn.Linear's autograd):
 *   dw[m, n] = sum_r gy[r, m] x[r, n],  db[m] = sum_r gy[r, m],  r < K.
 * gy bf16 [K, M], x bf16 [K, N] row-major; dw [M, N], db [M] fp32 or bf16
 * (out_bf16); offsets: unused (may be NULL; kept for the ABI: the kernel takes
 * the rows [0, K) from its parameters).  M % 64 == 0, N % 128 == 0.
 * K is split over up to 8 workgroup slices (split-K workspace). */
int rtdetr_linear_wgrad(const void* gy, const void* x, void* dw, void* db, const int32_t* offsets,
                        int K, int M, int N, int out_bf16, hipStream_t stream);
/* n <= 24 such gradients of mixed shapes in ONE launch (the dense layers'
 * weight gradients deferred to the end of the backward): problem q is
 * (gy[q] [K[q], M[q]], x[q] [K[q], N[q]]) -> dw[q] [M[q], N[q]], db[q] [M[q]];
 * outputs may be row slices of larger buffers (contiguous).  Each problem's
 * rows are split so the whole batch is ~3 workgroups per CU.  The problem
 * table travels as the kernel argument (host arrays, read at the call). */
int rtdetr_linear_wgrad_batch(int n, const void* const* gy, const void* const* x, void* const* dw,
                              void* const* db, const int* K, const int* M, const int* N, int out_bf16,
                              hipStream_t stream);
/* Narrow dense linear gradients (out_features M <= 128 with N even: the
 * decoder's class heads M = 1, box-head last layers M = 4, attention weights
 * M = 96; or in_features N <= 128 with M even: the query position head's
 * 4 -> 512 layer): dw [M, N] = gy^T x and db [M] = colsum(gy) in out_bf16 ?
 * bf16 : fp32, from bf16 gy [K, M] and x [K, N] (the wide one 4-byte
 * aligned; the other side <= 4096), deterministic
 * (fixed-order sum of row-slice partials).  part: fp32 workspace of
 * rtdetr_linear_wgrad_narrow_parts(K, M, N) floats, 8-byte aligned.  Replaces
 * torch's gy.t().mm(x) + column sum (linear.py _TokenLinear.backward; the
 * reference's nn.Linear heads, src/models/vision/rtdetr.py). */
int rtdetr_linear_wgrad_narrow_parts(int K, int M, int N);
int rtdetr_linear_wgrad_narrow(const void* gy, const void* x, void* dw, void* db, float* part, int K, int M, int N,
                               int out_bf16, hipStream_t stream);
/* Batched (linear.DeferredWgrad, after the backward): n <= 32 narrow problems
 * q = (gy[q] [K[q], M[q]], x[q] [K[q], N[q]]) in n_groups consecutive groups
 * (group g = the next group_count[g] problems, one shape), each group's dW /
 * db the fixed-order sum over its problems (a head applied several times, the
 * query position head once per decoder layer, gets its single gradient) into
 * dw[g] / db[g].  Two launches for all (26 per C2 step before, two per head).
 * part: rtdetr_linear_wgrad_narrow_batch_parts(n, K, M, N) floats (-1: a
 * problem outside the narrow shapes), 8-byte aligned. */
long long rtdetr_linear_wgrad_narrow_batch_parts(int n, const int* K, const int* M, const int* N);
int rtdetr_linear_wgrad_narrow_batch(int n, const void* const* gy, const void* const* x, const int* K, const int* M,
                                     const int* N, int n_groups, const int* group_count, void* const* dw,
                                     void* const* db, float* part, long long part_floats, int out_bf16,
                                     hipStream_t stream);
/* Row-wise top-k of fp32 scores (RT-DETR query selection: k = 300 of the S
 * memory tokens per image): x fp32 [rows][n], n <= 32768, 0 < k <= min(n,
 * 1024); idx int64 [rows][k] sorted by value descending (equal values: the
 * lower index first; at the cut the lowest indices among equal values are
 * kept); val fp32 [rows][k] or NULL.  One 1,024-thread workgroup per row:
 * radix select over LDS-staged keys, ordered compaction, bitonic sort.
 * Replaces torch.topk (decoder.RTDETRDecoder.forward; the reference's
 * RT-DETR query selection). */
int rtdetr_topk_rows(const float* x, int rows, int n, int k, long long* idx, float* val, hipStream_t stream);
/* The ResNet-D stem's first convolution, relu?(conv3x3(x, w, pad 1, stride) +
 * bias) for C = 3 -> N = 32 (the frozen BatchNorm folded into w / bias): x
 * bf16 NHWC [B, H, W, 3]; wf fp32 [9 C][N] (row (ky 3 + kx) C + c holds
 * w[:, c, ky, kx]); bias fp32 [N] or NULL; y bf16 NHWC [B, Ho, Wo, N], 16-B
 * aligned.  One thread per output pixel on the vector ALU (3 input channels
 * are too shallow for the implicit GEMM's K-tiles), the weights through
 * scalar loads; fp32 sums, one rounding.  Replaces MIOpen's convolution + a
 * bias/ReLU pass (backbone.PResNet's stem; the reference's RT-DETR backbone). */
int rtdetr_conv3x3_direct_fwd(const void* x, const float* wf, const float* bias, void* y, int B, int H, int W, int C,
                              int N, int stride, int relu, hipStream_t stream);
/* Narrow dense linears (csrc/narrow.hip), bf16 rows, fp32 accumulation, the
 * bias (bf16 when b_bf16, else fp32; NULL = none) added in fp32, one rounding:
 *   fwd:   y [M, N] = act(x [M, K] w[N, K]^T + b), act = ReLU when relu; for
 *          N <= 8 with K % 8 == 0 (the score heads, the box heads' 256 -> 4
 *          layers, the query ranking's head over all memory tokens) or K <= 8
 *          with N % 8 == 0 (the query position head's 4 -> 512 layer);
 *   dgrad: gx [M, K] = g [M, N] w [N, K], N <= 8, K % 8 == 0, then zeroed
 *          where mask [M, K] (bf16, e.g. the layer's input: the previous
 *          layer's ReLU) is <= 0 (mask NULL: no mask) -- threshold_backward
 *          fused.
 * Replace hipBLASLt's 1-8 column GEMMs (+ a ReLU / ReLU-backward launch) in
 * linear.py's _TokenLinear / _MLPHip (the reference's nn.Linear heads,
 * src/models/vision/rtdetr.py).  rtdetr_linear_narrow_supported(K, N): 1
 * when fwd takes the shape. */
int rtdetr_linear_narrow_supported(int K, int N);
int rtdetr_linear_narrow_fwd(const void* x, const void* w, const void* b, int b_bf16, void* y, long long M, int K,
                             int N, int relu, hipStream_t stream);
int rtdetr_linear_narrow_dgrad(const void* g, const void* w, const void* mask, void* gx, long long M, int K, int N,
                               hipStream_t stream);
/* a7: one backward step of an expert weight in ONE launch --
 *   dgrad: C[r, n] = epi( s_r sum_k A(r, k) B_g[k][n] )   (trans_b = 0; epilogue
 *          NONE / RELU_MASK / RELU_MASK_MX with aux); A(r, .) = a[a_gather[r]]
 *          (or a[r] when a_gather is NULL); s_r = row_scale[r] (or 1);
 *   wgrad: WC_g[m, n] = sum_r WX(r, m) WY(r, n), wcolsum_g[m] = sum_r WX(r, m),
 *          WX(r, .) = bf16(wx_scale[r] * wx[wx_gather[r]]) (or wx[r]),
 *          WY(r, .) = wy[wy_gather[r]] (or wy[r]).
 * With a = wx = dy, the gathers = src_tok and the scales = the row gates,
 * this is the combine transpose (dYp = gate * dy[token]) fused into the
 * dH / dW2 step.  The two halves are independent (same offsets, M2 x N2 the
 * weight's shape); sharing the launch fills the chip with both grids and
 * removes a kernel boundary.  bf16 operands; C bf16 [rows, N]; WC/wcolsum bf16
 * (out_bf16) or fp32. */
int moe_grouped_gemm_bwd_pair(const void* a, const int32_t* a_gather, const float* row_scale, const void* b,
                              void* c, const int32_t* offsets, int G, int max_rows, int N, int K, int epilogue,
                              const void* aux, const void* wx, const int32_t* wx_gather, const float* wx_scale,
                              const void* wy, const int32_t* wy_gather, void* wc, void* wcolsum, int M2, int N2,
                              int out_bf16, hipStream_t stream);
/* (wc = wcolsum = NULL: the dgrad alone.) */
/* The same, with dgrad row r stored at C row c_rows[r] (c_rows int32 [>=
 * offsets[G]], e.g. moe_ep_compaction's gather: dXp lands in the expert-
 * parallel received layout with no separate row-gather pass); the relu-mask
 * operand aux stays indexed by r.  c_rows == NULL is moe_grouped_gemm_bwd_pair. */
int moe_grouped_gemm_bwd_pair_scatter(const void* a, const int32_t* a_gather, const float* row_scale, const void* b,
                                      void* c, const int32_t* c_rows, const int32_t* offsets, int G, int max_rows,
                                      int N, int K, int epilogue, const void* aux, const void* wx,
                                      const int32_t* wx_gather, const float* wx_scale, const void* wy,
                                      const int32_t* wy_gather, void* wc, void* wcolsum, int M2, int N2,
                                      int out_bf16, hipStream_t stream);

/* The routed expert FFN backward of the single-GPU bf16 layer in TWO launches
 * (replaces the two moe_grouped_gemm_bwd_pair calls): launch 1 the dgrad
 * dH = relu'(H) * (gate[r] dy[tok[r]] . W2_g) into dh bf16 [max_rows, F];
 * launch 2 ONE grid of dXp = dH . W1_g (dxp bf16 [max_rows, d]), dW2_g =
 * dYp^T H + db2 (dYp = bf16(gate * dy[tok]) formed while staging) and dW1_g =
 * dH^T x[tok] + db1 -- the two weight gradients' K loops (the routed counts)
 * run beside each other instead of in two launches.  dy, x bf16 [T, d]; h bf16
 * [max_rows, F] (the forward's H); w1 bf16 [G, F, d], w2 bf16 [G, d, F]; tok,
 * gate [max_rows] (row -> token, gate); dw1/db1/dw2/db2 bf16 (out_bf16 = 1) or
 * fp32 [G, F, d] / [G, F] / [G, d, F] / [G, d].  Same sums, in the same order,
 * as the paired calls (bitwise equal).  Reference: SURVEY 8(a) row a7. */
int moe_expert_ffn_bwd(const void* dy, const int32_t* tok, const float* gate, const void* x, const void* h,
                       const void* w1, const void* w2, const int32_t* offsets, int G, int max_rows, int F, int d,
                       void* dh, void* dxp, void* dw1, void* db1, void* dw2, void* db2, int out_bf16,
                       hipStream_t stream);

/* ---- MXFP8 expert path (config C5: 32-expert top-4 fp8 expert GEMMs) ----
 * Format: OCP e4m3 elements with one E8M0 exponent byte per 32 consecutive
 * elements of a row ("MXFP8"); the block exponent e is the smallest with
 * amax <= 448 * 2^e (nothing saturates), stored as e + 127.  Forward GEMMs
 * run on v_mfma_scale_f32_16x16x128_f8f6f4 (hardware-applied block scales);
 * the backward keeps the e4m3 activations (ReLU mask from the e4m3 H, wgrad
 * operands dequantised exactly to bf16) and the bf16 weights for dgrad. */

/* Row quantizer: x bf16 [R, K] -> q e4m3 [R, K], scales uint8 [R, K/32].
 * K multiple of 128 (<= 8192).  Used for the expert weights (R = G*N). */
int moe_quantize_mx(const void* x, long long R, int K, void* q, void* scales, hipStream_t stream);

/* a4 in MXFP8: as moe_permute_fwd, but each token row is quantized
 * once and written to its kept destinations as e4m3 xq [rows, d] with
 * exponents xs [rows, d/32]. */
int moe_permute_fwd_mx(const void* x, const int32_t* topk_idx, const int32_t* local_rank,
                       const int32_t* rank_base, const int32_t* offsets, int T, int d, int E, int k,
                       int cap, void* xq, void* xs, int32_t* pos, hipStream_t stream);

/* a5 in MXFP8, rows-grouped, B stored [N][K] per group (nn.Linear):
 *   C[r, n] = epi( sum_k deq(A)[r, k] * deq(B_g)[n, k] )
 * a e4m3 [rows, K] + a_scales [rows, K/32]; b e4m3 [G, N, K] + b_scales
 * [G, N, K/32]; epilogue NONE / BIAS / BIAS_RELU (bias fp32 [G, N]).
 * c_scales == NULL: C is bf16 [rows, N]; else C is e4m3 [rows, N] with
 * exponents c_scales [rows, N/32] (quantized from the bf16-rounded result).
 * N % 128 == 0, K % 128 == 0. */
int moe_grouped_gemm_mx(const void* a, const void* a_scales, const void* b, const void* b_scales,
                        void* c, void* c_scales, const int32_t* offsets, int G, int max_rows, int N,
                        int K, int epilogue, const float* bias, hipStream_t stream);

/* a7: moe_grouped_gemm_wgrad with Y in MXFP8 (e4m3 [rows, N] +
 * y_scales [rows, N/32]); X stays bf16 (colsum over X as before). */
int moe_grouped_gemm_wgrad_mx(const void* x, const void* y, const void* y_scales, float* c,
                              float* colsum, const int32_t* offsets, int G, int M, int N,
                              hipStream_t stream);

/* ---- SURVEY 8(f).1 (next row): RT-DETR multi-scale deformable attention ----
 * Sampling core of the decoder's cross-attention (replaces the per-level
 * grid_sample chain of the reference engine's MSDeformableAttention):
 *   out[b,q,h,:] = sum_{l,p} attn[b,q,h,l,p] * bilinear(value_l[b,:,:,h,:], loc[b,q,h,l,p,:])
 * grid_sample conventions: align_corners = 0, zero padding, pixel = loc*size - 0.5.
 * value: bf16 [B, S, H, D] (levels flattened; level l = rows starts[l] ..
 * starts[l] + h_l*w_l); shapes: int32 [L, 2] (h, w); starts: int32 [L];
 * loc: fp32 [B, Q, H, L, P, 2]; attn: fp32 [B, Q, H, L, P]; out: bf16 [B, Q, H*D].
 * D in {32, 64}; L <= 4; P <= 16. */
int rtdetr_msda_fwd(const void* value, const int32_t* shapes, const int32_t* starts,
                    const float* loc, const float* attn, int B, int S, int Q, int H, int D,
                    int L, int P, void* out, hipStream_t stream);

/* Backward: grad_value fp32 [B, S, H, D] (zeroed here, then accumulated with
 * fp32 atomics), grad_loc fp32 [B, Q, H, L, P, 2], grad_attn fp32 [B, Q, H, L, P]. */
int rtdetr_msda_bwd(const void* value, const int32_t* shapes, const int32_t* starts,
                    const float* loc, const float* attn, const void* grad_out, int B, int S,
                    int Q, int H, int D, int L, int P, float* grad_value, float* grad_loc,
                    float* grad_attn, hipStream_t stream);
/* Same with grad_value bf16 [B,S,H,D], accumulated by packed bf16 atomics
 * (global_atomic_pk_add_bf16) -- the training step's variant. */
int rtdetr_msda_bwd_bf16(const void* value, const int32_t* shapes, const int32_t* starts,
                         const float* loc, const float* attn, const void* grad_out, int B, int S, int Q,
                         int H, int D, int L, int P, void* grad_value, float* grad_loc, float* grad_attn,
                         hipStream_t stream);

/* Fused decoder cross-attention core: the sampling locations and attention
 * weights are formed in the kernel from the raw linear outputs
 *   loc[.., l, p, :] = ref[b, q, :2] + bf16(off[.., l, p, :] / P) * ref[b, q, 2:] * offset_scale
 *   attn[b, q, h, :] = softmax(logits[b, q, h, :])   (over the L*P samples, fp32)
 * off bf16 [B,Q,H,L,P,2], ref fp32 [B,Q,4] (cx, cy, w, h; no gradient),
 * logits bf16 [B,Q,H,L*P], L*P <= 16.  Backward: grad_value bf16 (packed bf16
 * atomics), grad_off bf16 (same shape as off), grad_logits bf16 (softmax
 * backward fused). */
int rtdetr_msda_fused_fwd(const void* value, const int32_t* shapes, const int32_t* starts, const void* off,
                          const float* ref, const void* logits, float offset_scale, int B, int S, int Q,
                          int H, int D, int L, int P, void* out, hipStream_t stream);
int rtdetr_msda_fused_bwd(const void* value, const int32_t* shapes, const int32_t* starts, const void* off,
                          const float* ref, const void* logits, float offset_scale, const void* grad_out,
                          int B, int S, int Q, int H, int D, int L, int P, void* grad_value,
                          void* grad_off, void* grad_logits, hipStream_t stream);
/* The same with a strided value: token (b, s) starts ldv elements after token
 * (b, s-1) (ldv >= H*D) -- one [B*S, 6*H*D] value projection shared by the six
 * decoder layers, each reading its column slice; grad_value has the same
 * stride and is accumulated into (zeroed first only when zero_grad_value and
 * ldv == H*D). */
int rtdetr_msda_fused_fwd_ld(const void* value, long long ldv, const int32_t* shapes, const int32_t* starts,
                             const void* off, const float* ref, const void* logits, float offset_scale, int B, int S,
                             int Q, int H, int D, int L, int P, void* out, hipStream_t stream);
int rtdetr_msda_fused_bwd_ld(const void* value, long long ldv, const int32_t* shapes, const int32_t* starts,
                             const void* off, const float* ref, const void* logits, float offset_scale,
                             const void* grad_out, int B, int S, int Q, int H, int D, int L, int P, void* grad_value,
                             int zero_grad_value, void* grad_off, void* grad_logits, hipStream_t stream);
/* Deterministic variant of rtdetr_msda_fused_bwd_ld for the decoder's L = 3,
 * P = 4 (D = 32 or 64): the value gradient of the column slice is WRITTEN,
 * every element (rows no sample touches get zeros), as fp32 sums in a fixed
 * order rounded once to bf16 -- the corner contributions are recorded by the
 * per-sample kernel, bucketed by tile of value rows (stable counting sort) and
 * summed per tile -- instead of packed bf16 atomics in arrival order.
 * grad_off / grad_logits as rtdetr_msda_fused_bwd_ld.  hw_host: the L level
 * sizes h_l w_l in HOST memory (they size the tile grid); work: a device
 * workspace of rtdetr_msda_vgrad_workspace(B, Q, H, L, P) bytes, 16-B aligned.
 * Three launches, no host sync. */
long long rtdetr_msda_vgrad_workspace(int B, int Q, int H, int L, int P);
int rtdetr_msda_fused_bwd_det(const void* value, long long ldv, const int32_t* shapes, const int32_t* starts,
                              const int32_t* hw_host, const void* off, const float* ref, const void* logits,
                              float offset_scale, const void* grad_out, int B, int S, int Q, int H, int D, int L,
                              int P, void* grad_value, void* grad_off, void* grad_logits, void* work,
                              long long work_bytes, hipStream_t stream);

/* ---- frozen-BatchNorm convolution epilogues of the backbone ----
 * With frozen BN statistics, conv + BN = conv with per-channel scaled weights
 * + a channel bias; these apply the bias with what follows it, in one pass
 * over bf16 NHWC (channels_last) activations viewed as [M = B*H*W, C]:
 *   rtdetr_bias_act_nhwc:      y = act(x + bias[c]), act 0 none / 1 ReLU (x == y allowed)
 *   rtdetr_add_bias_relu_nhwc: y = relu(a + b + bias[c]) (bias may be NULL)
 * bias fp32 [C]; C % 8 == 0. */
int rtdetr_bias_act_nhwc(const void* x, const float* bias, long long M, int C, int act, void* y,
                         hipStream_t stream);
int rtdetr_add_bias_relu_nhwc(const void* a, const void* b, const float* bias, long long M, int C,
                              void* y, hipStream_t stream);
/* Frozen-BN weight fold of many convolutions in one launch (forward
 * W' = W * scale[c_out], backward dW = dW' * scale[c_out]): `records` is a
 * device array of 32-B {const bf16* w; const float* scale; bf16* out;
 * int32 rows; int32 inner} (rows = output channels, inner = elements per
 * output channel, a multiple of 8; 16-B aligned tensors); `chunks` device
 * int32 pairs {record, chunk of 2048 elements}.  out = RNE(float(w) * scale). */
int rtdetr_fold_scale_multi(const void* records, const int32_t* chunks, int n_chunks, hipStream_t stream);
/* The same product for n <= 64 tensors given as host pointer arrays (the
 * table goes in the kernel argument: the folds' backward dW_l = dW'_l *
 * scale_l on gradients allocated during the backward, graph-capture safe):
 * out_q[r, :] = bf16(in_q[r, :] * scale_q[r]), bf16 [rows_q, inner_q], inner a
 * multiple of 8.  One launch for every backbone convolution (52 at C2). */
int rtdetr_fold_scale_batch(int n, const void* const* in, const float* const* scale, void* const* out,
                            const int* rows, const int* inner, hipStream_t stream);

/* ResNet-D shortcut AvgPool2d(2, 2) over channels_last bf16 [B, H, W, C]
 * (even H, W; C % 8 == 0; 16-B aligned): y = RNE(0.25 * window sum, fp32);
 * backward gx = RNE(0.25 * gy) broadcast to the 2x2 window (H, W = input
 * dims in both calls).  Reference engine: Ultralytics/RT-DETR PResNet
 * (rtdetr.py:82-94, upstream resnet-d variant). */
int rtdetr_avgpool2x2_nhwc_fwd(const void* x, int B, int H, int W, int C, void* y, hipStream_t stream);
int rtdetr_avgpool2x2_nhwc_bwd(const void* gy, int B, int H, int W, int C, void* gx, hipStream_t stream);
/* the same, plus an addend of gx's shape: gx = (pool backward) + add (add may
 * be NULL).  The backbone's stage outputs: the encoder's gradient of a stage
 * output joins the ResNet-D shortcut's gradient here, before branch2a's dgrad
 * epilogue adds both and applies the ReLU mask (GradLink, backbone.stage_taps). */
int rtdetr_avgpool2x2_nhwc_bwd_add(const void* gy, const void* add, int B, int H, int W, int C, void* gx,
                                   hipStream_t stream);
/* The stem's MaxPool2d(3, 2, 1) forward over channels_last bf16 (the stem is
 * frozen: no backward): y [B, (H-1)/2+1, (W-1)/2+1, C], C % 8 == 0, x and y
 * 16-B aligned; padding never wins, NaN propagates.  Replaces nn.MaxPool2d in
 * the reference's ResNet stem (Ultralytics RT-DETR backbone). */
int rtdetr_maxpool3x3s2_nhwc_fwd(const void* x, int B, int H, int W, int C, void* y, hipStream_t stream);
/* The encoder's FPN top-down concat (HybridEncoder CCFM): out [B, H, W, Ch +
 * Cl] = cat([nearest x2 upsample of high [B, Hh, Wh, Ch] cropped to H x W,
 * low [B, H, W, Cl]], channels), channels_last bf16; Ch, Cl % 8 == 0, H/2 <=
 * Hh <= H and W/2 <= Wh <= W, 16-B aligned.  Backward: dhigh = the 2x2 block
 * sums of g[.., :Ch] (fp32, one rounding), dlow = g[.., Ch:] dense, one launch.
 * Replaces F.interpolate(scale 2, nearest) + torch.cat of the reference's
 * RT-DETR encoder (Ultralytics RTDETRDecoder's HybridEncoder neck). */
int rtdetr_upcat_nhwc_fwd(const void* high, const void* low, int B, int H, int W, int Hh, int Wh, int Ch, int Cl,
                          void* out, hipStream_t stream);
int rtdetr_upcat_nhwc_bwd(const void* g, int B, int H, int W, int Hh, int Wh, int Ch, int Cl, void* dhigh, void* dlow,
                          hipStream_t stream);

/* Bias gradient of a linear layer: out[n] = sum_m dy[m, n] over bf16 dy [M, N]
 * (row-major), fp32 accumulation in a fixed order (deterministic, no atomics),
 * out fp32 (out_bf16 = 0) or bf16.  Two launches: P row-block partials into
 * `partials` (fp32 [P, N], caller-owned), then the column totals.
 * rtdetr_bias_grad_parts(M, N) returns the P the caller should allocate for.
 * N a multiple of 8 (<= 2048, 16-B aligned dy) or N <= 256.
 * Replaces AddmmBackward's torch column sum (reference engine: Ultralytics
 * RT-DETR linear layers, rtdetr.py:82-94). */
int rtdetr_bias_grad_parts(long long M, int N);
int rtdetr_bias_grad(const void* dy, long long M, int N, float* partials, int P, void* out, int out_bf16,
                     hipStream_t stream);

/* Residual add + LayerNorm over the last dim of bf16 rows (the post-norm
 * sites of the AIFI / decoder layers, norm(x + sublayer(x)), incl. the MoE
 * layers' norm(x + MoEFFN(x)); reference engine: Ultralytics RT-DETR
 * transformer layers, rtdetr.py:82-94):
 *   out = (s - mean) * rstd * gamma + beta,  s = a + b (b may be NULL),
 * fp32 statistics (biased variance), bf16 out, mean / rstd fp32 [T] saved for
 * the backward.  d = 128, 256 or 512; gamma / beta bf16 (w_bf16 = 1) or fp32.
 * Backward: ds = d out / d s (bf16 [T, d]; the gradient of a and of b) and
 * [dgamma; dbeta] (2 x d, the parameter dtype) from P block partials
 * (fp32 [P, 2d], caller-owned, P = rtdetr_add_layer_norm_parts(T)), summed
 * in a fixed order (deterministic, no atomics).  Replaces the residual add
 * and torch's native_layer_norm / native_layer_norm_backward. */
int rtdetr_add_layer_norm_parts(long long T);
int rtdetr_add_layer_norm_fwd(const void* a, const void* b, const void* gamma, const void* beta, int w_bf16,
                              long long T, int d, float eps, void* out, float* mean, float* rstd,
                              hipStream_t stream);
int rtdetr_add_layer_norm_bwd(const void* dout, const void* a, const void* b, const void* gamma, int w_bf16,
                              const float* mean, const float* rstd, long long T, int d, void* ds, float* partials,
                              int P, void* dgamma_dbeta, hipStream_t stream);
/* The decoder's `t = LN(a + b); q = t + pos` in one pass: out2 = bf16(out +
 * pos) (pos, out2 bf16 [T, d], both or neither).  bwd2: the gradient of out
 * is dout + dout2 (summed in bf16 per element, as autograd's accumulation of
 * the two consumers'; dout2 may be NULL); pos's gradient is dout2 itself. */
int rtdetr_add_layer_norm_pos_fwd(const void* a, const void* b, const void* gamma, const void* beta, int w_bf16,
                                  long long T, int d, float eps, const void* pos, void* out, void* out2, float* mean,
                                  float* rstd, hipStream_t stream);
int rtdetr_add_layer_norm_bwd2(const void* dout, const void* dout2, const void* a, const void* b, const void* gamma,
                               int w_bf16, const float* mean, const float* rstd, long long T, int d, void* ds,
                               float* partials, int P, void* dgamma_dbeta, hipStream_t stream);
/* bwd / bwd2 with dgamma_dbeta NULL stop after the row pass (partials
 * written, no final); the finals of many LayerNorms then run as ONE launch
 * after the backward (linear.DeferredWgrad): problem q sums its P[q] <= 256
 * partial rows of N[q] = 2d columns into out[q] ([dgamma; dbeta], bf16 when
 * out_bf16[q]), the same fixed order as the single final.  n <= 48. */
int rtdetr_add_layer_norm_final_batch(int n, const float* const* partials, const int* P, const int* N,
                                      void* const* out, const int* out_bf16, hipStream_t stream);

/* Decoder box refinement (one launch each way), over n = B*Q*4 elements:
 *   y = sigmoid(delta + log(max(x', eps) / max(1 - x', eps))), x' = clamp(ref, 0, 1)
 * delta bf16 (delta_bf16 = 1) or fp32; ref, y fp32.  Backward:
 *   g_delta = (g_boxes + g_inter) y (1 - y)          (either gradient may be NULL)
 *   g_ref   = g_boxes y (1 - y) d inverse_sigmoid / d ref   (g_ref NULL: not needed) */
int rtdetr_box_refine_fwd(const void* delta, int delta_bf16, const float* ref, long long n, float eps, float* y,
                          hipStream_t stream);
int rtdetr_box_refine_bwd(const float* g_boxes, const float* g_inter, const float* y, const float* ref,
                          long long n, float eps, void* g_delta, int delta_bf16, float* g_ref,
                          hipStream_t stream);

/* Backward of a block output feeding two consumers:
 *   out = (g1 + g2) * (y > 0)   (bf16 NHWC [M, C]; g2 may be NULL)
 * the gradient accumulation and the ReLU mask in one pass. */
int rtdetr_relu_grad2_nhwc(const void* g1, const void* g2, const void* y, long long M, int C, void* out,
                           hipStream_t stream);

/* Training-mode BatchNorm (batch statistics) of nb = 1 or 2 NHWC bf16 branches
 * x[i] [M, C] (C a power of two in [8, 2048], M >= 2), summed and activated
 * (encoder ConvNormLayer act="silu" / RepVggBlock; torch.nn.BatchNorm2d
 * semantics, reference engine: RT-DETR HybridEncoder):
 *   y = act(sum_i (x_i - mean_i) invstd_i gamma_i + beta_i), act 0 none / 1 silu.
 * Host arrays of nb pointers; gamma/beta/running stats fp32 [C] (running
 * arrays may be NULL: no update; else momentum update, unbiased variance).
 * saved fp32 [nb][4][C] = mean, invstd, scale, shift (kept for backward);
 * ws: rtdetr_bn_act_workspace(M, C, nb) bytes of device scratch.
 * Backward: dx[i] bf16 [M, C]; coef fp32 [nb][3][C] scratch; dgb fp32
 * [nb][2][C] = dgamma, dbeta.  Deterministic (no atomics). */
size_t rtdetr_bn_act_workspace(long long M, int C, int nb);
int rtdetr_bn_act_fwd(const void* const* x, const float* const* gamma, const float* const* beta,
                      float* const* run_mean, float* const* run_var, int nb, long long M, int C, int act, float eps,
                      float momentum, float* saved, float* ws, void* y, hipStream_t stream);
int rtdetr_bn_act_bwd(const void* dy, const void* const* x, const float* const* gamma, int nb, long long M, int C,
                      int act, const float* saved, float* ws, float* coef, void* const* dx, float* dgb,
                      hipStream_t stream);
/* Inference-mode (running statistics) BatchNorm of nb = 1 or 2 branches +
 * their sum + act (0 none, 1 SiLU) [+ resid, added after the activation] in
 * ONE pass: y = act(sum_i x_i scale_i + shift_i), scale = gamma *
 * rsqrt(running_var + eps), shift = beta - running_mean * scale (fp32 affine
 * and statistics [C]; x_i / y / resid NHWC bf16 [M, C], 16-B aligned; C a
 * power of two in [8, 2048]).  The HybridEncoder's / decoder input
 * projections' BatchNorms in the evaluation forward (torch: batch_norm, then
 * SiLU and the branch add as separate passes). */
int rtdetr_bn_act_eval(const void* const* x, const float* const* gamma, const float* const* beta,
                       const float* const* run_mean, const float* const* run_var, int nb, long long M, int C, int act,
                       float eps, const void* resid, void* y, hipStream_t stream);
/* rtdetr_bn_act_fwd with the batch statistics already summed per row block
 * by the producing convolution (rtdetr_conv_fwd_stats): part fp32
 * [nb][part_blocks][2][C] (sum, sum of squares of the bf16 x_i),
 * 1 <= part_blocks <= 2048; no statistics pass, no workspace. */
int rtdetr_bn_act_fwd_part(const void* const* x, const float* const* gamma, const float* const* beta,
                           float* const* run_mean, float* const* run_var, int nb, long long M, int C, int act,
                           float eps, float momentum, const float* part, int part_blocks, float* saved, void* y,
                           hipStream_t stream);
/* The same with y (forward) / dy (backward) a batch-strided slice of a wider
 * row-major tensor: row r of the [M, C] layout is row (r / hw) * bstride +
 * r % hw of y / dy (hw = 0: contiguous).  The decoder's memory [B, S, C]:
 * level l's BatchNorm output written straight into its rows (y = memory +
 * start_l C, hw = h_l w_l, bstride = S) and its gradient read from d memory
 * in place -- no concatenation forward, no strided copy backward.  fwd_rows:
 * part (conv-epilogue statistics, ws unused) or ws (a statistics pass);
 * resid (bf16 [M, C] in x's layout, or NULL): y = act(z) + resid, act(z)
 * rounded to bf16 before the add (the bits of a bf16 activation then a bf16
 * add) -- the CSPRep layer's bottleneck output + shortcut branch, whose
 * gradient is dy for both (no separate add either way). */
int rtdetr_bn_act_fwd_rows(const void* const* x, const float* const* gamma, const float* const* beta,
                           float* const* run_mean, float* const* run_var, int nb, long long M, int C, int act,
                           float eps, float momentum, const float* part, int part_blocks, float* ws, float* saved,
                           const void* resid, void* y, long long y_hw, long long y_bstride, hipStream_t stream);
int rtdetr_bn_act_bwd_rows(const void* dy, long long dy_hw, long long dy_bstride, const void* const* x,
                           const float* const* gamma, int nb, long long M, int C, int act, const float* saved,
                           float* ws, float* coef, void* const* dx, float* dgb, hipStream_t stream);

/* Process-wide tuning overrides (not thread-safe; set before launching).  By
 * default (0) every launch picks its own kernel variant, ring depth and tile
 * height from its shape; these force one (kernel benchmarks and tests):
 *   "gemm_variant" 0 auto, 1 register-staged double buffer, 2 LDS-DMA ring
 *   "gemm_stages"  0 auto, 2..4 ring slots for variant 2
 *   "rows_bm", "wgrad_bm"  0 auto, 64 or 128 row-tile height
 *   "gemm_debug"   0; 1 = skip C stores, 2 = skip the main loop (time attribution only)
 *   "xcd_map"      0 auto, 1 row tiles round-robin over XCDs, 2 contiguous chunk per XCD
 *   "ksplit"       0 auto, 1 no split-K, 2..8 forced split-K factor (needs the workspace below)
 *   "gemm_pair"    1 (default) one launch per moe_grouped_gemm_bwd_pair, 0 two launches (A/B)
 * Returns 0, or -1 for an unknown key/value. */
int moe_set_tuning(const char* key, int value);

/* Split-K workspace of the grouped GEMMs for the CURRENT device (caller-owned,
 * kept alive while any launch or captured graph may use it).  When a launch's
 * grid would leave CUs idle (ROWS: < 256 tiles with K >= 512; WGRAD: <= 512
 * tiles), its K range is cut into slices run by separate workgroups of one
 * XCD; each writes fp32 partials to `ws` and the last to arrive per tile
 * (arrival counter in `counters`, which must be zero on registration and are
 * left zero after every launch) sums them in slice order (deterministic) and
 * applies the epilogue.  A launch whose slices do not fit `ws_bytes` or whose
 * tile count exceeds n_counters runs unsplit; NULL/NULL unregisters.  Launches
 * sharing one workspace must be stream-ordered.  "ksplit" in moe_set_tuning
 * forces the factor (1 = off). */
int moe_set_splitk_workspace(void* ws, size_t ws_bytes, int32_t* counters, int n_counters);

/* a3: the layer's aux losses from the router's partials, one block:
 *   P_e = sum_b aux_partials[b][e] / T, f_e = hist[e] / (T k),
 *   out3 = {lb = E sum_e f_e P_e, z = sum_b aux_partials[b][E] / T,
 *           lb_coef lb + z_coef z}
 *   wcoef[E+1] = d out3[2] / d aux_partials[b][.] (same for every b):
 *           lb_coef E f_e / T (e < E), z_coef / T (e = E)
 * (the backward is g * wcoef broadcast over the blocks). */
int moe_aux_loss_fwd(const float* aux_partials, int nblk, int E, const int32_t* hist, int T, int k,
                     float lb_coef, float z_coef, float* out3, float* wcoef, hipStream_t stream);

/* Hungarian matching of the set criterion on the device (the reference's
 * RT-DETR loss matches with scipy.optimize.linear_sum_assignment on the host).
 * cost fp32 [S][B][Q][M]: S prediction sets, B images, Q queries, M padded
 * targets of which the first n_valid[b] are real (n_valid int32 [B], <= Q).
 * assign int32 [S][B][M] <- query matched to each real target, -1 for the
 * padding: the assignment scipy 1.15's linear_sum_assignment returns for
 * cost[s][b][:, :n] (same algorithm, arithmetic and tie rule).  *status is
 * set to 1 (n_valid > Q or > M) or 2 (non-finite costs) on failure, else left
 * untouched (zero it before the first launch).  One 64-lane workgroup per
 * (s, b); Q <= 4096, M <= 1024 within 64 KiB of LDS. */
int rtdetr_hungarian_match(const float* cost, const int32_t* n_valid, int S, int B, int Q, int M,
                           int32_t* assign, int32_t* status, hipStream_t stream);

/* RT-DETR set criterion fused (SetCriterion.loss_padded): S prediction sets,
 * B images, Q queries, C classes, M padded targets (first n_valid[b] real);
 * logits fp32 [S,B,Q,C], boxes fp32 [S,B,Q,4] cxcywh, tgt_boxes fp32 [B,M,4],
 * tgt_labels int32 [B,M].
 *   _match: Hungarian matching with the matching cost (2 focal class + 5 L1 +
 *           2 GIoU) evaluated inside the solver; assign int32 [S,B,M] as
 *           rtdetr_hungarian_match.
 *   _loss:  one workgroup per set: comps[S][3] = {VFL, L1, GIoU} / num_boxes
 *           (num_boxes: device scalar; VFL weight alpha p^2 (1 - onehot) + IoU),
 *           and their gradients d_logits [S,B,Q,C], d_l1 / d_giou [S,B,Q,4].
 *           B*Q*C*4 bytes must fit 64 KiB (LDS score map).
 *   _loss_bwd: g_logits = g[s,0] d_logits, g_boxes = g[s,1] d_l1 + g[s,2] d_giou. */
int rtdetr_set_criterion_match(const float* logits, const float* boxes, const float* tgt_boxes,
                               const int32_t* tgt_labels, const int32_t* n_valid, int S, int B, int Q,
                               int C, int M, int32_t* assign, int32_t* status, hipStream_t stream);
int rtdetr_set_criterion_loss(const float* logits, const float* boxes, const float* tgt_boxes,
                              const int32_t* tgt_labels, const int32_t* n_valid, const int32_t* assign,
                              const float* num_boxes, float vfl_alpha, int S, int B, int Q, int C, int M,
                              float* comps, float* d_logits, float* d_l1, float* d_giou, hipStream_t stream);
int rtdetr_set_criterion_loss_bwd(const float* g_comps, int S, int B, int Q, int C, const float* d_logits,
                                  const float* d_l1, const float* d_giou, float* g_logits, float* g_boxes,
                                  hipStream_t stream);

/* Multi-head self-attention of the encoder (AIFI) and decoder layers on the
 * bf16 MFMA, head_dim 32 (replaces torch's scaled_dot_product_attention, i.e.
 * AOTriton kernels, inside nn.MultiheadAttention; the reference's engine runs
 * it inside RTDETR.train, src/models/vision/rtdetr.py:82-94).  bf16 operands
 * addressed in place: row of (image b, token t, head h) at ptr + (b L + t) ld
 * + 32 h, ld in elements (multiple of 8, >= 32 H), pointers 16-B aligned.
 * Scores are scaled by `scale`; softmax over all L keys (no mask).
 *   rtdetr_attn_fwd: o = softmax(scale q k^T) v; lse [B, H, L] fp32 =
 *     per-row max + log2(sum) of the base-2 softmax (for the backward).
 *   rtdetr_attn_bwd: dq, dk, dv from dout, the forward's o and lse; delta
 *     [B, H, L] fp32 scratch (rowsum(dout * o)).  Two launches (dQ, then dK and
 *     dV), no atomics: bitwise repeatable. */
int rtdetr_attn_fwd(const void* q, long long ldq, const void* k, long long ldk, const void* v, long long ldv,
                    void* o, long long ldo, float* lse, int B, int H, int L, int head_dim, float scale,
                    hipStream_t stream);
int rtdetr_attn_bwd(const void* q, long long ldq, const void* k, long long ldk, const void* v, long long ldv,
                    const void* o, long long ldo, const void* dout, long long lddo, const float* lse, float* delta,
                    void* dq, long long lddq, void* dk, long long lddk, void* dv, long long lddv, int B, int H,
                    int L, int head_dim, float scale, hipStream_t stream);

/* Implicit-GEMM convolutions of the RT-DETR body (the
 * backbone and the HybridEncoder's RepVGG / CSP convolutions, which the
 * reference's engine trains inside RTDETR.train, src/models/vision/rtdetr.py:
 * 82-94), bf16 MFMA, padding (KS - 1) / 2, KS in {1, 3}, stride 1 (or 2 with
 * KS = 3: the ResNet-D stage-entry and HybridEncoder downsampling 3x3
 * convolutions), no bias.  B, H, W are the INPUT x / dx dims; the output y / dy
 * is [B, Ho, Wo] with Ho = (H - 1) / stride + 1 (W likewise).
 * x / dy / y: NHWC bf16 [B, H, W, channels]; w: [N][KS][KS][C] bf16 (a
 * channels_last [N, C, KS, KS] weight); C and N multiples of 64 (the forward
 * also takes multiples of 32: 32-deep K-tiles, a partial last output-channel
 * tile -- the stem's 32 -> 32 / 32 -> 64 layers); zero: >= 256
 * zero bytes on the device (read for padding neighbours); pointers 16-B aligned.
 *   rtdetr_conv_fwd         y[B,Ho,Wo,N] = conv(x[B,H,W,C], w)   (no im2col buffer),
 *                           with an optional fused epilogue (NULL / 0 = off):
 *                           y = relu?((y + resid[B,H,W,N]) + bias[N]) (fp32 on
 *                           the bf16 result: rtdetr_add_bias_relu_nhwc's
 *                           arithmetic; bias fp32, resid bf16 NHWC)
 *   rtdetr_conv_dgrad       dx[B,H,W,C] = conv^T(dy[B,Ho,Wo,N], w): the forward
 *                           GEMM over dy with the flipped, transposed weight
 *                           (stride 2: dx(y, x) reads dy((y+dy)/2, (x+dx)/2)
 *                           for the taps with both even, a zero row otherwise),
 *                           written to work first when
 *                           rtdetr_conv_dgrad_workspace() > 0 (bytes; large
 *                           problems), else read in place from w (work may be
 *                           NULL); add (bf16 [B,H,W,C] or NULL): dx += add
 *                           (fp32 sum of the two bf16 values); relu_mask (bf16
 *                           [B,H,W,C] or NULL): then dx = 0 where relu_mask <= 0
 *                           (the ReLU backward of the activation that fed the
 *                           convolution, with its other consumer's gradient
 *                           'add' -- rtdetr_relu_grad2_nhwc's arithmetic, fused)
 *   rtdetr_conv_wgrad       dw[N][KS][KS][C] = sum over pixels dy (x) x[neighbour]:
 *                           nsplit pixel slices write fp32 partials to part
 *                           [nsplit][N KS KS C], summed in slice order
 *                           (deterministic) into dw (bf16 if out_bf16 else fp32);
 *                           nsplit from rtdetr_conv_wgrad_splits (called
 *                           with the OUTPUT dims Ho, Wo: its pixel count is the
 *                           GEMM's K).
 * MIOpen, which these replace, zero-fills its atomic split-K weight-gradient
 * outputs outside a captured hipGraph for some solvers: replays then add onto
 * the previous step's sums (tools/miopen_graph_probe.py). */
int rtdetr_conv_fwd(const void* x, const void* w, void* y, const void* zero, int B, int H, int W, int C, int N,
                    int KS, int stride, const float* bias, const void* resid, int relu, hipStream_t stream);
/* rtdetr_conv_fwd with the activation named (act 0 none, 1 ReLU, 2 SiLU) and,
 * with resid_post, the residual added AFTER the activation in bf16:
 * y = bf16(bf16(act(conv + bias)) + resid) (round 6: the evaluation forward's
 * re-parameterised RepVgg blocks -- 3x3 + 1x1 + both running-statistics
 * BatchNorms folded into one 3x3 weight and bias -- and the folded
 * ConvNormLayers of the HybridEncoder; torch's SiLU-then-add order).
 * y_img_rows > 0: image b's output rows (and resid rows) are written at rows
 * b y_img_rows + y_row_off + pixel of y (the decoder's input projections
 * writing their level of the memory [B, S, N] in place); 0 = dense. */
int rtdetr_conv_fwd_act(const void* x, const void* w, void* y, const void* zero, int B, int H, int W, int C, int N,
                        int KS, int stride, const float* bias, const void* resid, int act, int resid_post,
                        long long y_img_rows, long long y_row_off, hipStream_t stream);
/* rtdetr_conv_fwd (no epilogue) that also writes the BatchNorm statistics of
 * its bf16 output: part fp32 [ceil(B Ho Wo / rows)][2][N], row block r = the
 * column sums and sums of squares over output pixels [r rows, (r + 1) rows),
 * rows = rtdetr_conv_fwd_stats_rows(...) (the forward's M-tile height).  For
 * rtdetr_bn_act_fwd_part (the encoder's ConvNormLayer / RepVgg BatchNorms). */
int rtdetr_conv_fwd_stats_rows(int B, int H, int W, int C, int N, int KS, int stride);
int rtdetr_conv_fwd_stats(const void* x, const void* w, void* y, const void* zero, int B, int H, int W, int C,
                          int N, int KS, int stride, float* part, hipStream_t stream);
long long rtdetr_conv_dgrad_workspace(int B, int H, int W, int C, int N, int KS);
int rtdetr_conv_dgrad(const void* dy, const void* w, void* work, void* dx, const void* zero, int B, int H, int W,
                      int C, int N, int KS, int stride, const void* add, const void* relu_mask, hipStream_t stream);
/* Batched weight flip (round 4): rtdetr_conv_weight_flip_multi writes W' for
 * every weight of a device table of n descriptors {const bf16* w; bf16* wt;
 * int N, C, KS, block0} (32 B each, block0 = the prefix sum of (C/64)(N/64)KS^2
 * blocks; total_blocks their sum) in ONE launch; rtdetr_conv_dgrad_preflipped
 * is rtdetr_conv_dgrad for a shape that flips (workspace > 0) reading W' from
 * wflip instead of writing it (w is still checked, not read). */
int rtdetr_conv_weight_flip_multi(const void* table, int n, int total_blocks, hipStream_t stream);
int rtdetr_conv_dgrad_preflipped(const void* dy, const void* w, const void* wflip, void* dx, const void* zero, int B,
                                 int H, int W, int C, int N, int KS, int stride, const void* add, const void* relu_mask,
                                 hipStream_t stream);
int rtdetr_conv_wgrad_splits(int B, int H, int W, int C, int N, int KS);
int rtdetr_conv_wgrad(const void* dy, const void* x, float* part, int nsplit, void* dw, int out_bf16,
                      const void* zero, int B, int H, int W, int C, int N, int KS, int stride, hipStream_t stream);
/* rtdetr_conv_wgrad in two halves (round 6): rtdetr_conv_wgrad_part writes
 * only the nsplit fp32 slices to part; rtdetr_conv_wgrad_reduce_batch sums
 * the slices of n <= 48 weights (parts[q] [nsplits[q]][nws[q]] -> dws[q],
 * bf16 if out_bf16 else fp32) in ONE launch, each exactly as
 * rtdetr_conv_wgrad's own reduction (bitwise).  The training step defers the
 * reductions of a whole backward to one or two such launches instead of one
 * launch per convolution. */
int rtdetr_conv_wgrad_part(const void* dy, const void* x, float* part, int nsplit, const void* zero, int B, int H,
                           int W, int C, int N, int KS, int stride, hipStream_t stream);
int rtdetr_conv_wgrad_reduce_batch(int n, const float* const* parts, const int* nsplits, const long long* nws,
                                   void* const* dws, int out_bf16, hipStream_t stream);
/* Measurement / A-B knobs (0, or -1 for conv_dgrad_flip, = automatic):
 * "conv_bm" forward pixel-tile rows 64 / 128 / 256; "conv_wg_stages"
 * weight-gradient LDS ring depth 2..4; "conv_wg_splits" weight-gradient pixel
 * slices returned by rtdetr_conv_wgrad_splits; "conv_dgrad_flip" 1 = always
 * write the flipped weight, 0 = always read it in place. */
int rtdetr_conv_set_tuning(const char* key, int value);

/* Training-step optimizer (the bench step's AdamW; reference: Ultralytics'
 * AdamW inside RTDETR.train, src/models/vision/rtdetr.py:82-94, with
 * torch.optim.AdamW + torch.nn.utils.clip_grad_norm_ semantics) over flat
 * fp32 master / exp_avg / exp_avg_sq buffers, reading each gradient where
 * autograd left it.  `tensors`: device array of 48-B records
 *   { const void* grad; uint16_t* bf16_weight_or_NULL; int64 numel;
 *     int64 flat_offset (multiple of 8); int32 grad_dtype (0 bf16, 1 fp32,
 *     2 no gradient: tensor skipped as torch.optim does);
 *     int32 lr_group; int32 pad[2]; }
 * `chunks`: device int32 pairs {tensor, chunk} covering every tensor in
 * 2048-element chunks; `tensor_steps`: device int32 per tensor, the AdamW
 * step count (zero-initialised; counted per tensor like torch.optim, so a
 * tensor without a gradient neither moves nor advances).  Per step:
 *   train_grad_sqnorm        partials[c] = sum of squares of chunk c
 *   train_grad_norm_finalize coef[0] = ||g|| * inv_world,
 *                            coef[1] = inv_world * min(1, max_norm / (coef[0] + 1e-6))
 *                            (max_norm <= 0: no clip); fixed summation order;
 *                            tensor_steps[i] += 1 for tensors with a gradient
 *   train_adamw_step         g *= coef[1]; w *= 1 - lr wd; m = b1 m + (1-b1) g;
 *                            v = b2 v + (1-b2) g^2; with t = tensor_steps[i]:
 *                            w -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps);
 *                            bf16 weight (if any) = RNE(w)
 * lrs: HOST array of n_groups (1..4) learning rates.
 *   train_grad_pack          data-parallel staging: every
 *                            record's gradient widened to fp32 at
 *                            flat[flat_offset ...] (zeros for grad_dtype 2),
 *                            so the ranks' gradient sum is one fp32
 *                            all-reduce; flat must be 16-B aligned. */
int train_grad_pack(const void* tensors, const int32_t* chunks, int n_chunks, float* flat, hipStream_t stream);
int train_grad_sqnorm(const void* tensors, const int32_t* chunks, int n_chunks, float* partials,
                      hipStream_t stream);
int train_grad_norm_finalize(const float* partials, int n, float max_norm, float inv_world, float* coef,
                             const void* tensors, int n_tensors, int32_t* tensor_steps, hipStream_t stream);
int train_adamw_step(const void* tensors, const int32_t* chunks, int n_chunks, const float* coef,
                     float* master, float* exp_avg, float* exp_avg_sq, const int32_t* tensor_steps,
                     const float* lrs, int n_groups, float weight_decay, float beta1, float beta2, float eps,
                     hipStream_t stream);

/* Launch profiler (measurement only; no reference counterpart).
 * While enabled, every kernel launch of the library carries a hipEvent pair
 * stamped by its own dispatch packet (hipExtLaunchKernel: kernel execution
 * start/end, host gaps excluded) plus its algorithmic work: HBM bytes (every
 * operand read once, every output written once) and flops (grouped GEMM:
 * 2 N K per routed row; 0 for the other kinds), with the routed row count read
 * back from the device offsets.  Kinds: 0 grouped GEMM, 1 permute/combine row
 * moves, 2 router, 3 route scan, 4 token backward, 5 deformable attention,
 * 6 MXFP8 weight quantizer, 7 backbone convolution epilogues, 8 optimizer,
 * 9 Hungarian matching, 10 fp8 grouped GEMM, 11 dense linear weight gradients,
 * 12 self-attention, 13 implicit-GEMM convolutions, 14 router weight /
 * context-bias gradients.
 * Not thread-safe, not for graph capture.  enable(0|1) also clears; get()
 * waits for the record. */
enum moe_prof_kind {
  MOE_PROF_GEMM = 0,
  MOE_PROF_ROWMOVE = 1,
  MOE_PROF_ROUTER = 2,
  MOE_PROF_SCAN = 3,
  MOE_PROF_TOKEN_BWD = 4,
  MOE_PROF_MSDA = 5,
  MOE_PROF_QUANT = 6,
  MOE_PROF_CONV_EPI = 7,
  MOE_PROF_OPTIM = 8,
  MOE_PROF_MATCH = 9,
  MOE_PROF_GEMM_FP8 = 10, /* grouped GEMM on the fp8 (MXFP8) MFMA: priced at the fp8 peak */
  MOE_PROF_LINEAR = 11,   /* dense linear weight + bias gradients (rtdetr_linear_wgrad) */
  MOE_PROF_ATTN = 12,     /* multi-head self-attention (rtdetr_attn_fwd / rtdetr_attn_bwd) */
  MOE_PROF_CONV = 13,     /* implicit-GEMM convolutions (rtdetr_conv_*) */
  MOE_PROF_ROUTER_WGRAD = 14 /* router weight / context-bias gradients (moe_router_wgrad) */
};
int moe_profile_enable(int on);
int moe_profile_count(void);
int moe_profile_get(int i, int* kind, float* ms, double* flops, double* bytes);
int moe_profile_clear(void);

/* Host-side launch counts per moe_prof_kind (MOE_PROF_*): every kernel launch
 * the library issues increments its kind's count, profiling on or off and
 * inside hipGraph capture (a captured launch counts once, when captured).
 * out[i] = count of kind i for i < n (0 past the last kind).  How a caller
 * proves the HIP path ran (tests/test_gpu_dropin.py).  reset() zeroes them.
 * Not thread-safe. */
int moe_launch_counts(long long* out, int n);
int moe_launch_counts_reset(void);

/* Thread-local message for the last non-zero return code. */
const char* moe_last_error(void);

/* Library build identification ("moe_hip <version> gfx950"). */
const char* moe_version(void);

#ifdef __cplusplus
}
#endif

#endif /* MOE_HIP_H_ */
