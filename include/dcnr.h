/*
 * dcnr.h -- C ABI of libdcnr.so, the MI355X (gfx950) DCN-R ranking hot path.
 *
 * Drop-in boundary for the reference's DCN-R path.  The reference
 * (Krist-Marrakesh/Hybrid-Hotel-Recommendation-System-Based-on-Friends-
 * Recommendations) has no FFI of its own: its boundary is the PyTorch module
 * DCN_RecSys and its callers.  Each entry point below replaces one reference
 * interface (file:line in the reference repository):
 *
 *   dcnr_forward          DCN_RecSys.forward            train.py:155-170 (dup main.py:114-127)
 *                         incl. ResBlock.forward          train.py:112-122
 *                         and CrossLayer.forward          train.py:96-99
 *   dcnr_gather_cross     the front of DCN_RecSys.forward: embedding gathers,
 *                         x0 concat and the cross network   train.py:156-159,166-168
 *                         (BASELINE configs[1])
 *   dcnr_backward         loss.backward() through the model   train.py:225
 *   dcnr_bce_with_logits  nn.BCEWithLogitsLoss()(preds, y)    train.py:206,224,233,376
 *   dcnr_adam_step        torch.optim.AdamW/Adam(...).step()  train.py:201-204,226
 *   dcnr_cosine_topk      NearestNeighbors(metric='cosine', algorithm='brute')
 *                         .kneighbors(vec, n_neighbors=k)      main.py:196-203,268-270,300
 *   dcnr_row_inv_norms    the row normalisation inside sklearn's cosine metric
 *   dcnr_gather_rows      the batch assembly of TensorDataset + DataLoader
 *                         (train.py:195-196) on a device-resident dataset
 *   dcnr_candidate_union  _generate_candidates' union of positives and their
 *                         neighbours[1:]                      main.py:196-203
 *   dcnr_ranking_batch    preprocess_for_ranking              main.py:215-230
 *   dcnr_rank_by_score    sorted(zip(scores, ids), reverse=True) main.py:325
 *   dcnr_mmr_rerank       rerank_with_mmr                     main.py:133-169
 *
 * Conventions
 *  - All tensor pointers are DEVICE pointers owned by the caller; the
 *    library allocates nothing on the hot path (workspace is caller-owned,
 *    size from dcnr_workspace_size / dcnr_cosine_topk_workspace_size).
 *    dcnr_forward (train mode: the embedding backward's id sort) and
 *    dcnr_backward (the cross backward) fork part of their work onto one
 *    library-owned stream per device (created on first use) and join it back
 *    into `stream` before they return their last kernels; callers see
 *    ordinary stream semantics.
 *  - Parameter tables are HOST arrays of device pointers:
 *      params: in the reference's state_dict() order (train.py:136-153):
 *        user_embedding.weight, item_embedding.weight,
 *        cat_embeddings.{k}.weight (k < n_cat),
 *        initial_deep_layer.weight [H,D], initial_deep_layer.bias [H],
 *        for j < n_res: res_blocks.{j}.{layer1.weight, layer1.bias,
 *            bn1.weight, bn1.bias, bn1.running_mean, bn1.running_var,
 *            bn1.num_batches_tracked (int64 scalar), layer2.weight,
 *            layer2.bias, bn2.weight, bn2.bias, bn2.running_mean,
 *            bn2.running_var, bn2.num_batches_tracked},
 *        for l < n_cross: cross_network.{l}.b [D], cross_network.{l}.w.weight [1,D],
 *        final_linear.weight [1,H+D], final_linear.bias [1]
 *      grads: in named_parameters() order (the same list without the BN
 *        running_mean / running_var / num_batches_tracked buffers).
 *    Every floating tensor is fp32, contiguous, row-major.
 *  - Index tensors are int64 (torch.long) like the reference; indices are
 *    clamped in-kernel (never an out-of-bounds access) and, with
 *    DCNR_FLAG_CHECK_INDICES, an out-of-range index is reported as
 *    DCNR_INDEX_OOB by dcnr_check_errors (torch raises IndexError there).
 *  - Everything is stream-ordered and asynchronous on `stream` (a
 *    hipStream_t); functions return after enqueueing.  No entry point
 *    synchronises except dcnr_check_errors.
 *  - Status codes are returned, never thrown or aborted across the ABI;
 *    dcnr_last_error() gives a thread-local message for the last failure.
 *  - Eval-mode forward is re-entrant (no shared scratch); train-mode forward
 *    mutates BN running statistics and must be serialised by the caller.
 */
#ifndef DCNR_H
#define DCNR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DCNR_ABI_VERSION 4

typedef void* dcnr_stream_t; /* hipStream_t */

typedef enum {
  DCNR_OK = 0,
  DCNR_BAD_ARG = 1,
  DCNR_INDEX_OOB = 2,
  DCNR_HIP_ERROR = 3,
  DCNR_UNSUPPORTED_SHAPE = 4,
  DCNR_WORKSPACE_TOO_SMALL = 5
} dcnr_status;

typedef enum { DCNR_PREC_FP32 = 0, DCNR_PREC_BF16 = 1 } dcnr_precision;
typedef enum { DCNR_EVAL = 0, DCNR_TRAIN = 1 } dcnr_mode;

#define DCNR_FLAG_CHECK_INDICES 1u
/* Train workspace keeps every residual block's backward intermediates (du,
 * dt2, da, dt1) in buffers of their own instead of reusing one set: the
 * stage-by-stage parity tests read them (dcnr_workspace_offset).  Same
 * kernels, same results; more workspace.  In eval mode it keeps the
 * unfused tail (BN affine finalize launch, the last block's output h_R in
 * the workspace, separate head dot); without it the bf16 eval forward ends
 * in the last GEMM's head epilogue and never stores h_R; likewise the bf16
 * train forward does not store h_R (the backward rebuilds it from t2 and
 * h_{R-1}), so DCNR_WS_H at index R is only meaningful with this flag. */
#define DCNR_FLAG_KEEP_INTERMEDIATES 2u
/* bf16 eval forward: take the fused deep tower (one persistent launch, the
 * activations on chip) at any batch size it supports.  Without the flag it
 * is taken from 16384 samples on, where it overtakes the layer-by-layer path;
 * below that the layer path is faster (the tower walks a tile's layers in
 * sequence on one CU).  Same results either way up to bf16 rounding order. */
#define DCNR_FLAG_FUSED_TOWER 4u
/* Train mode (ABI 4): the backward leaves the embedding tables' gradient rows
 * that the batch did not reference as they were (no 142 MB zero fill at the
 * bench shape) and instead marks, in a byte map at the end of the workspace
 * (DCNR_WS_ROW_MAP: one byte per table row, the tables in order, 1 = this
 * call wrote the row), every row it wrote.  dcnr_adam_step_rows reads the map
 * and treats unmarked rows' gradients as exactly 0, which is bit-identical to
 * the dense-gradient step.  Only with accumulate = 0 (the flag and accumulate
 * together are DCNR_BAD_ARG).  Same workspace offsets for every other tensor. */
#define DCNR_FLAG_ROW_MAP 8u

/* Optional collective hook for SyncBN across data-parallel ranks: called
 * (stream-ordered, from the calling thread) with a device buffer of `count`
 * fp64 values that must be summed over all ranks in place before the call
 * returns or is stream-ordered before later work on `stream`.  NULL = local
 * BN (each rank normalises with its own batch statistics). */
typedef int (*dcnr_allreduce_fn)(void* ctx, double* device_buf, int64_t count, dcnr_stream_t stream);

/* Optional data-parallel hook of dcnr_backward: called (from the calling
 * thread, while the call enqueues its work) as soon as every kernel that
 * writes a group of gradients has been enqueued on `stream`:
 *   DCNR_GRADS_DENSE      initial_deep_layer .. final_linear (every
 *                         parameter after the embedding tables)
 *   DCNR_GRADS_EMBEDDING  user, item and categorical tables (last)
 * A caller starts that group's exchange from here (ordered after the
 * stream's work so far), so the dense group's exchange runs under the
 * embedding backward.  Nonzero return = failure (dcnr_backward fails). */
#define DCNR_GRADS_DENSE 0
#define DCNR_GRADS_EMBEDDING 1
typedef int (*dcnr_grad_ready_fn)(void* ctx, int32_t group, dcnr_stream_t stream);

typedef struct {
  int64_t n_users;          /* user_embedding rows      (train.py:136) */
  int64_t n_items;          /* item_embedding rows      (train.py:137) */
  int32_t n_cat;            /* number of categorical tables (len(cat_dims)) */
  const int64_t* cat_rows;  /* HOST array [n_cat]: cat_dims.values() (train.py:138-139) */
  int32_t emb_dim;          /* params['emb_dim'] */
  int32_t n_num;            /* n_num_features */
  int32_t hidden;           /* params['hidden_dim'] */
  int32_t n_cross;          /* params['n_cross_layers'] */
  int32_t n_res;            /* params.get('n_res_blocks', 2) */
  float dropout;            /* params['dropout'] (applied in train mode only) */
  int32_t precision;        /* dcnr_precision of the deep-tower GEMMs/activations */
  uint32_t flags;           /* DCNR_FLAG_* */
  dcnr_allreduce_fn bn_allreduce; /* SyncBN hook or NULL */
  void* bn_allreduce_ctx;
  dcnr_grad_ready_fn grad_ready;  /* gradient-group hook or NULL (ABI 2) */
  void* grad_ready_ctx;
  /* ABI 3.  With DCNR_FLAG_CHECK_INDICES: where dcnr_forward's last kernel
   * stores the call's index-error word (0 = every id in range), e.g. a slot
   * of pinned host memory the caller polls once an event recorded after the
   * call has completed -- no copy of its own on the stream.  NULL: the word
   * stays in the workspace (dcnr_check_errors / a caller's copy). */
  int32_t* error_mirror;
} dcnr_model_desc;

int dcnr_abi_version(void);
const char* dcnr_last_error(void);

/* Input dim D = 2*emb_dim + sum(int(sqrt(n_cat_k))+1) + n_num (train.py:139-141). */
int64_t dcnr_input_dim(const dcnr_model_desc* desc);

/* Workspace bytes for a batch of B in `mode`.  A train-mode workspace holds
 * the saved activations that dcnr_backward consumes. */
dcnr_status dcnr_workspace_size(const dcnr_model_desc* desc, int64_t B, int mode, size_t* bytes);

/* Where a stored tensor lives in the workspace of (desc, B, mode), for tests
 * that check each stage against a recomputation from the kernels' own stored
 * inputs.  Row-major with leading dimension Hp = hidden rounded up to 8
 * (Dp for x0, Dq = Dp rounded up to 32 for dx0); element type bf16 in bf16
 * mode, else fp32 (masks: 1 bit per element, Hp/8 bytes per row; BN vectors,
 * zc, dx0, xcoef, sc: fp32).  dx0 is the deep tower's part of d loss/d x0;
 * the cross network's part is sum_k xcoef[b][k] V_k with V = (w_0 .. w_{L-1},
 * w_f[H:]), xcoef [B][L+1]; sc [B][2L+1] holds the forward's per-sample cross
 * scalars (x_l . w_l for l < L, x_0 . w_m for m < L, x_0 . w_f[H:]).  `index` is
 * the block j (h: 0..n_res; bn_*: 2j for bn1, 2j+1 for bn2).  *offset = -1
 * when that tensor is not materialised in this configuration. */
typedef enum {
  DCNR_WS_X0 = 0, DCNR_WS_H = 1, DCNR_WS_T1 = 2, DCNR_WS_T2 = 3, DCNR_WS_A1 = 4,
  DCNR_WS_MASK_A1 = 5, DCNR_WS_MASK_H = 6, DCNR_WS_BN_MEAN = 7, DCNR_WS_BN_INVSTD = 8,
  DCNR_WS_BN_SCALE = 9, DCNR_WS_BN_SHIFT = 10, DCNR_WS_DU = 11, DCNR_WS_DT2 = 12,
  DCNR_WS_DA = 13, DCNR_WS_DT1 = 14, DCNR_WS_G = 15, DCNR_WS_DX0 = 16, DCNR_WS_ZC = 17,
  DCNR_WS_XCOEF = 18, DCNR_WS_SC = 19, DCNR_WS_ROW_MAP = 20, DCNR_WS_KINDS = 21
} dcnr_ws_tensor;
dcnr_status dcnr_workspace_offset(const dcnr_model_desc* desc, int64_t B, int mode, int kind,
                                  int index, int64_t* offset);

/* DCN_RecSys.forward: logits[B] (fp32, device).  mode = DCNR_TRAIN uses
 * batch statistics (B >= 2), updates BN running stats and
 * num_batches_tracked in `params`, applies dropout with `dropout_seed`, and
 * keeps the activations backward needs in `ws`. */
dcnr_status dcnr_forward(const dcnr_model_desc* desc, void* const* params,
                         const int64_t* user_ids, const int64_t* item_ids,
                         const int64_t* cat_features /* [B,n_cat] */,
                         const float* num_features /* [B,n_num] */, int64_t B, int mode,
                         uint64_t dropout_seed, float* logits, void* ws, size_t ws_bytes,
                         dcnr_stream_t stream);

/* The embedding gathers, x0 concat and cross network of DCN_RecSys.forward
 * on their own (train.py:156-159 and 166-168), fp32:
 *   x0[b]        = [U[u_b] | I[i_b] | C_0[c_b0] .. C_{K-1}[c_b,K-1] | num_b]   (bit-exact copy)
 *   cross_out[b] = x_L,  x_{l+1} = x_l + x_l * (x_l . w_l) + b_l     (CrossLayer, train.py:96-99)
 * x0 [B][ld_x0] and cross_out [B][ld_cross] are fp32 device buffers (either
 * may be NULL; ld >= D).  params as for dcnr_forward (only the embedding
 * tables and cross_network.* are read).  oob_flag: optional device int32 that
 * is set nonzero when an id is out of range (ids are clamped in-kernel).
 * Stateless and re-entrant. */
dcnr_status dcnr_gather_cross(const dcnr_model_desc* desc, void* const* params,
                              const int64_t* user_ids, const int64_t* item_ids,
                              const int64_t* cat_features, const float* num_features, int64_t B,
                              float* x0, int64_t ld_x0, float* cross_out, int64_t ld_cross,
                              int32_t* oob_flag, dcnr_stream_t stream);

/* Backward of the last train-mode dcnr_forward on `ws`: given dL/dlogits
 * [B], writes dL/dparam for every parameter into `grads`.  accumulate = 0
 * overwrites (embedding grads are zeroed, then every referenced row gets the
 * sum of its samples' dx0 rows, i.e. embedding_dense_backward semantics);
 * accumulate = 1 adds into grads.  Deterministic: the embedding sums run in
 * a fixed order after a stable sort of the ids, and every other reduction is
 * fixed-order too, so two calls on the same inputs give bit-identical
 * gradients. */
dcnr_status dcnr_backward(const dcnr_model_desc* desc, void* const* params, void* const* grads,
                          const int64_t* user_ids, const int64_t* item_ids,
                          const int64_t* cat_features, const float* num_features, int64_t B,
                          const float* dlogits, uint64_t dropout_seed, int accumulate, void* ws, size_t ws_bytes,
                          dcnr_stream_t stream);

/* The embedding rows the batch of the last train-mode dcnr_forward on `ws`
 * touched, read from that forward's stable id sort (the sorted (id, sample)
 * pairs the backward's fixed-order sums walk; still in `ws` after
 * dcnr_backward): the data-parallel sparse gradient exchange
 * (SURVEY.md 8(e) option B; the gradient rows come from train.py:156-158
 * under train.py:225) buckets them by owner without a torch.unique.
 * For each of n_tables tables (indices into the model's tables: 0 = user,
 * 1 = item, 2.. = categorical) writes the flat element offsets
 * elem_off[i] + row * width of its distinct rows, ascending, to
 * out_offsets[i*B ..] and their number to table_counts[i]; owner_counts[r]
 * (r < world <= DCNR_TOUCHED_MAX_WORLD) counts the offsets in
 * [r*shard_elems, (r+1)*shard_elems).
 * Stream-ordered; outputs are device memory. */
#define DCNR_TOUCHED_MAX_WORLD 64

/* The sparse exchange's send buffers, built on the device from
 * dcnr_emb_touched_rows' output (SURVEY.md 8(e) option B; the rows of the
 * dense gradient of train.py:156-158 under train.py:225): for each of
 * n_tables tables, the table_counts[t] (device) offsets offsets[t*ld ..] and
 * the `width`-float gradient rows of `grad` they address are appended, tables
 * in order, to out_offsets / out_rows [sum(table_counts)][width].  Offsets
 * ascend within a table and the tables are in flat order, so the list is
 * grouped by shard owner.  Stream-ordered; no host synchronisation. */
dcnr_status dcnr_sparse_pack(const float* grad, const int64_t* offsets, int64_t ld,
                             const int64_t* table_counts, int32_t n_tables, int32_t width,
                             int64_t* out_offsets, float* out_rows, dcnr_stream_t stream);

/* The owner's half of the sparse exchange: zeroes shard [shard_elems] (flat
 * elements [shard_lo, shard_lo + shard_elems) of the gradient) and adds the
 * rows the n_sources ranks sent, back to back in `offsets` / `rows`
 * (source_counts[r] rows from rank r: a HOST array), sources in rank order --
 * every shard row is summed 0 + g_0 + g_1 + ..., the same bits run to run.
 * Within one source the offsets are distinct.  Offsets outside the shard are
 * skipped. */
dcnr_status dcnr_sparse_accumulate(float* shard, int64_t shard_lo, int64_t shard_elems, int32_t width,
                                   const int64_t* offsets, const float* rows,
                                   const int64_t* source_counts, int32_t n_sources,
                                   dcnr_stream_t stream);
dcnr_status dcnr_emb_touched_rows(const dcnr_model_desc* desc, const void* ws, size_t ws_bytes,
                                  int64_t B, int32_t n_tables, const int32_t* tables,
                                  const int64_t* elem_off, int64_t shard_elems, int32_t world,
                                  int64_t* out_offsets, int64_t* table_counts,
                                  int64_t* owner_counts, dcnr_stream_t stream);

size_t dcnr_bce_workspace_size(void);

/* BCEWithLogitsLoss (mean): loss[0] = mean(max(z,0) - z*y + log1p(exp(-|z|)));
 * if dlogits != NULL also writes dlogits = grad_scale * (sigmoid(z) - y) / B.
 * Deterministic (fixed-order fp64 reduction through `ws`). */
dcnr_status dcnr_bce_with_logits(const float* logits, const float* labels, int64_t B,
                                 float* loss, float* dlogits, float grad_scale, void* ws,
                                 size_t ws_bytes, dcnr_stream_t stream);

/* One torch.optim.AdamW (decoupled = 1) or Adam (decoupled = 0) step over
 * n_tensors tensors (host arrays of device pointers + element counts).
 * `step` is the 1-based step number after increment (torch's state['step']). */
dcnr_status dcnr_adam_step(int32_t n_tensors, float* const* params, const float* const* grads,
                           float* const* exp_avg, float* const* exp_avg_sq, const int64_t* numel,
                           float lr, float beta1, float beta2, float eps, float weight_decay,
                           int64_t step, int decoupled, dcnr_stream_t stream);

/* dcnr_adam_step over gradients some of whose rows are not stored (ABI 4,
 * the same step, train.py:201-204, 226): tensor i with row_map[i] != NULL is
 * [numel[i] / row_width[i]][row_width[i]] and element e's gradient is
 * grads[i][e] where row_map[i][e / row_width[i]] != 0, else exactly 0 (the
 * row is not read) -- bit-identical to dcnr_adam_step on the dense gradient
 * with those rows zeroed.  row_map[i] == NULL: dense.  row_map / row_width are
 * HOST arrays (row_map entries device pointers, e.g. into the DCNR_WS_ROW_MAP
 * of the train workspace, offset to the table's first row). */
dcnr_status dcnr_adam_step_rows(int32_t n_tensors, float* const* params, const float* const* grads,
                                float* const* exp_avg, float* const* exp_avg_sq, const int64_t* numel,
                                const uint8_t* const* row_map, const int32_t* row_width,
                                float lr, float beta1, float beta2, float eps, float weight_decay,
                                int64_t step, int decoupled, dcnr_stream_t stream);

/* 1/||row|| for each row of table [N,d] (0-norm rows -> 1, as sklearn's normalize). */
dcnr_status dcnr_row_inv_norms(const float* table, int64_t N, int32_t d, float* inv_norms,
                               dcnr_stream_t stream);

size_t dcnr_cosine_topk_workspace_size(int64_t N, int64_t Q, int32_t k);

/* k nearest rows of `table` [N,d] to each query [Q,d] by cosine distance
 * dist = clip(1 - <q/|q|, x/|x|>, 0, 2) (fp32), ascending; ties by lower
 * row index.  idx int64 [Q,k], dist fp32 [Q,k].  1 <= k <= min(64, N).
 * Q = 0 returns DCNR_OK without touching the query / output / workspace
 * pointers (which may then be NULL). */
dcnr_status dcnr_cosine_topk(const float* table, const float* inv_norms, int64_t N, int32_t d,
                             const float* queries, int64_t Q, int32_t k, int64_t* idx,
                             float* dist, void* ws, size_t ws_bytes, dcnr_stream_t stream);

/* Fit-time bf16 copy of the normalised table for the batched scan:
 * packed[r][c] = bf16(table[r][c] * inv_norms[r]) (fp32 product, round to
 * nearest even), uint16 [N,d], d % 8 == 0.  Optional: 2 bytes per element
 * resident beside the fp32 table halve the batched (Q >= 16, d = 32 or 64)
 * scan's HBM stream; results are identical with or without it.  Part of
 * NearestNeighbors.fit (main.py:268-270) -- sklearn keeps its own copy of
 * the fitted data there too. */
dcnr_status dcnr_cosine_pack_rows(const float* table, const float* inv_norms, int64_t N, int32_t d,
                                  uint16_t* packed, dcnr_stream_t stream);

/* dcnr_cosine_topk reading `packed` (from dcnr_cosine_pack_rows over the same
 * table, or NULL) for its coarse bf16 scan; same results, same workspace. */
dcnr_status dcnr_cosine_topk_packed(const float* table, const float* inv_norms, const uint16_t* packed,
                                    int64_t N, int32_t d, const float* queries, int64_t Q, int32_t k,
                                    int64_t* idx, float* dist, void* ws, size_t ws_bytes,
                                    dcnr_stream_t stream);

/* Merge of row-sharded top-k lists (the cfg5 index split over ranks, SURVEY
 * 8(e)): dist fp32 / idx int64 [lists][Q][k] (global rows; padding entries
 * (FLT_MAX, -1) sort last) -> the k best per query, ascending by (dist, row),
 * the order dcnr_cosine_topk gives over the whole table.  lists * k <= 2048.
 * Replaces nothing in the reference (one sklearn index per process,
 * main.py:268-270); the single-index result is reproduced exactly. */
dcnr_status dcnr_topk_merge(const float* dist, const int64_t* idx, int32_t lists, int64_t Q,
                            int32_t k, int64_t* out_idx, float* out_dist, dcnr_stream_t stream);

/* Batch assembly of a device-resident dataset (TensorDataset + DataLoader,
 * train.py:195-196): for each of n_arrays (<= 8) arrays of n_src rows of
 * row_bytes[a] bytes (a multiple of 4), dst[a] row i = src[a] row idx[i]
 * (idx clamped to [0, n_src)).  Host arrays of device pointers. */
dcnr_status dcnr_gather_rows(const int64_t* idx, int64_t n, int64_t n_src, int32_t n_arrays,
                             const void* const* src, void* const* dst, const int64_t* row_bytes,
                             dcnr_stream_t stream);

/* ---- serving: the steps either side of scoring in /recommendations ----
 * All operate on at most 4096 items per call (DCNR_UNSUPPORTED_SHAPE above). */

/* Candidate set of _generate_candidates (main.py:196-203): the union of
 * positives[Q] (embedding rows of the positive hotels) and, for each, the
 * neighbour rows knn_idx[q][1..k-1] (the dcnr_cosine_topk output for
 * n_neighbors = k, position 0 dropped as main.py:201 does); negative rows are
 * skipped.  out_rows: the distinct rows ascending; out_count[0] (device
 * int32) = their number.  Q*k <= 4096. */
dcnr_status dcnr_candidate_union(const int64_t* positives, int64_t Q, const int64_t* knn_idx,
                                 int32_t k, int64_t* out_rows, int32_t* out_count,
                                 dcnr_stream_t stream);

/* Ranking batch of preprocess_for_ranking (main.py:215-230) for one user:
 * user_ids[i] = user_row, item_ids[i] = item_rows[i], and the item's
 * categorical codes / scaled numeric features gathered from per-item tables
 * item_cat [n_items][n_cat] (int64) and item_num [n_items][n_num] (fp32). */
dcnr_status dcnr_ranking_batch(const int64_t* item_rows, int64_t n, int64_t user_row,
                               const int64_t* item_cat, int32_t n_cat, const float* item_num,
                               int32_t n_num, int64_t n_items, int64_t* user_ids,
                               int64_t* item_ids, int64_t* cat_features, float* num_features,
                               dcnr_stream_t stream);

/* order[i] = index of the i-th highest score; equal scores keep input order
 * (Python's stable sorted(..., reverse=True), main.py:325).  n <= 4096. */
dcnr_status dcnr_rank_by_score(const float* scores, int64_t n, int64_t* order,
                               dcnr_stream_t stream);

/* rerank_with_mmr (main.py:133-169) over n candidates given in ranked order:
 * rows[i] = embedding row of candidate i in `table` [., d] (-1: no embedding),
 * scores[i] its score.  Writes out_pos[0 .. top_k) = positions (into the ranked
 * list) of the re-ranked items, -1 padded; out_count[0] (device int32) = their
 * number.  Cosine similarity via inv_norms (dcnr_row_inv_norms). */
dcnr_status dcnr_mmr_rerank(const float* table, const float* inv_norms, int32_t d,
                            const int64_t* rows, const float* scores, int64_t n,
                            float lambda_param, int32_t top_k, int64_t* out_pos,
                            int32_t* out_count, dcnr_stream_t stream);

/* The deep tower's Linear layer as a standalone bf16 call (nn.Linear forward,
 * train.py:143,105,109): C[M,N] = X[M,K] . W[N,K]^T + bias, X/W bf16
 * row-major (K, ldx, ldw multiples of 8), C bf16 (out_f32 = 0) or fp32.
 * Used by the deep tower internally; exported for unit tests and kernel
 * benchmarks. */
dcnr_status dcnr_linear_bf16(const void* X, int64_t ldx, int64_t M, int32_t K, const void* W,
                             int64_t ldw, int32_t N, const float* bias, void* C, int64_t ldc,
                             int out_f32, dcnr_stream_t stream);

/* The deep tower's weight gradient as a standalone bf16 call (backward of
 * nn.Linear, train.py:225): dW[N][K] (fp32) (+)= sum_b dY[b][n] * X[b][k],
 * dY [B][ldy] and X [B][ldx] bf16 row-major (N, K, ldy, ldx multiples of 8).
 * Workspace: dcnr_linear_wgrad_workspace_size bytes.  Used by the deep tower
 * internally; exported for unit tests and kernel benchmarks. */
size_t dcnr_linear_wgrad_workspace_size(int32_t N, int32_t K, int64_t B);
dcnr_status dcnr_linear_wgrad_bf16(const void* dY, int64_t ldy, const void* X, int64_t ldx,
                                   int64_t B, int32_t N, int32_t K, float* dW, int accumulate,
                                   void* ws, size_t ws_bytes, dcnr_stream_t stream);

/* Kernel-timing instrumentation (measurement only, off by default): when
 * enabled, every launch the library makes is bracketed by HIP events on its
 * stream and attributed to one of these classes. */
typedef enum {
  DCNR_K_GATHER_CROSS = 0, /* gather + x0 + cross forward                 */
  DCNR_K_GEMM_FWD = 1,     /* deep-tower Linear forward (MFMA)             */
  DCNR_K_GEMM_DX = 2,      /* deep-tower dX GEMMs (MFMA)                   */
  DCNR_K_GEMM_DW = 3,      /* deep-tower dW split-K GEMMs (MFMA)           */
  DCNR_K_ROWWISE = 4,      /* BN stats/apply, ReLU, dropout, residual      */
  DCNR_K_REDUCE = 5,       /* partial-sum / split-K reductions, BN finalize */
  DCNR_K_CROSS_BWD = 6,    /* cross backward + embedding-grad scatter      */
  DCNR_K_HEAD = 7,         /* head dot, logits, BCE                         */
  DCNR_K_ADAM = 8,         /* fused Adam/AdamW                              */
  DCNR_K_KNN = 9,          /* cosine top-k                                  */
  DCNR_K_PACK = 10,        /* weight packing / zero fills                  */
  DCNR_K_SERVE = 11,       /* candidate union, ranking batch, sort, MMR     */
  DCNR_K_EMB_SORT = 12,    /* embedding-backward stable id sort             */
  DCNR_K_EMB_SUM = 13,     /* embedding-backward per-row segmented sums     */
  DCNR_K_TOWER = 14,       /* fused eval deep tower (one persistent launch) */
  DCNR_K_COUNT = 15
} dcnr_kernel_class;

/* on = 0: off; 1: every launch timed per class with HIP events on its
 * stream (the backward's weight-gradient GEMMs then run on the caller's
 * stream, each launch priced alone); 2: only DCNR_K_GEMM_DW timed, on the
 * side stream where it overlaps the dX chain (its concurrent wall time). */
void dcnr_profile_enable(int on);
/* Synchronises the recorded events and returns, per class, the summed kernel
 * milliseconds and launch counts since the last collect (arrays of n). */
dcnr_status dcnr_profile_collect(double* ms, int64_t* launches, int32_t n);
/* ... plus, per class, the summed ALGORITHMIC bytes of those launches (the
 * operands each function must move: inputs read once, outputs written once;
 * split-K slabs count only in their reduction) -- the numerator of each
 * class's HBM roofline fraction. */
dcnr_status dcnr_profile_collect_bytes(double* ms, int64_t* launches, double* bytes, int32_t n);

/* Synchronises `stream` and reports kernel-side errors recorded in ws
 * (DCNR_INDEX_OOB when DCNR_FLAG_CHECK_INDICES saw an out-of-range id). */
dcnr_status dcnr_check_errors(void* ws, size_t ws_bytes, dcnr_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* DCNR_H */
