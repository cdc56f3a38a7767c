/*
 * grk.h -- C ABI of libgrk.so, the MI355X (gfx950) hot path of the TencentGR
 * sequence-recommender training step.
 *
 * The reference (Puiching-Memory/Tencent_Recommendation_2025) has no native
 * code and no FFI: its hot path is PyTorch ops called from Python
 * (SURVEY.md §8(b)).  Each entry point below replaces the device work of one
 * reference call site, cited per function; the Python host layer
 * (tencent_recommendation_2025_amd/kernels.py) binds them with ctypes and
 * exposes them as torch.library ops under the reference's nn.Module surface.
 *
 * Conventions
 *  - All pointers are DEVICE pointers unless noted; the caller (the torch
 *    caching allocator) owns every buffer, including workspace.  The library
 *    never allocates, frees or synchronises, so every call can be captured
 *    into a hipGraph -- with one exception: grk_gemm, on the FIRST call for a
 *    new shape, times its hipBLASLt candidates (a scratch buffer is allocated,
 *    the device synchronised, the buffer freed) and allocates one hipBLASLt
 *    workspace per stream the first time it sees the stream.  Calls for
 *    known shapes on known streams allocate nothing (the trainer warms every
 *    shape up on the capture stream before capturing).
 *  - Work is enqueued on `stream` (a hipStream_t passed as void*).
 *  - Return 0 on success, else a GRK_E* code; grk_last_error() returns the
 *    thread-local message.  Shape/argument errors are detected on the host
 *    before any launch.  Out-of-range indices are detected on the device: the
 *    offending lookup reads/writes nothing and, if `err_flag` is non-NULL,
 *    *err_flag is set to 1 (the torch layer checks it lazily).
 *  - Matrices are row-major with an explicit leading dimension in elements.
 */
#ifndef GRK_H_
#define GRK_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { GRK_OK = 0, GRK_EINVAL = 1, GRK_EHIP = 2, GRK_EUNSUPPORTED = 3 };
enum { GRK_F32 = 0, GRK_BF16 = 1, GRK_F16 = 2 };    /* floating dtypes */
enum { GRK_F32_BF16 = 3 };  /* pair logits: fp32 h, bf16 e_pos / e_neg (and their gradients) */
enum { GRK_FP8_E4M3 = 4 };  /* attention q/k/v: OCP fp8 e4m3 (gfx950's fp8 format) */
enum { GRK_I32 = 0, GRK_I64 = 1 };                  /* index dtypes */

/* How a lookup derives its row id from the index tensor value v at token
 * (n = b*T + t):  model/BaseLine/model.py:240-247 and :326-328. */
enum {
  GRK_IDX_PLAIN = 0,      /* row = v                                   */
  GRK_IDX_ITEM_MASK = 1,  /* row = v * (token_type[n] == 1)            */
  GRK_IDX_USER_MASK = 2,  /* row = v * (token_type[n] == 2)            */
  GRK_IDX_POSITION = 3    /* row = (t + 1) * (v != 0)                  */
};

#define GRK_MAX_FEATURES 48

/* Returns the last error message of the calling thread ("" if none). */
const char* grk_last_error(void);
/* Library version string. */
const char* grk_version(void);

/* A non-blocking HIP stream of the caller's own on the current device, outside
 * any framework's stream pool (torch hands out pooled streams round-robin, so
 * a "new" torch stream can be the very stream a process group's collectives
 * record their events on; capturing a HIP graph on that stream makes the
 * process group's watchdog query of those events fail).  Trainer captures its
 * step on one of these. */
int grk_stream_create(void** stream);
/* The same with a HIP stream priority (lower = more urgent; clamped into the device's
 * range): the deferred tables' flush slice runs on a low-priority stream beside the step. */
int grk_stream_create_priority(void** stream, int priority);
int grk_stream_destroy(void* stream);

/* ------------------------------------------------------------------------
 * Embedding tables
 * ------------------------------------------------------------------------ */

/* One feature of a fused multi-table lookup.  Replaces one
 * `nn.Embedding.__call__` (model/BaseLine/model.py:242,243,247,275,328) or one
 * `sparse_emb[k](t).sum(2)` bag-sum (model/BaseLine/model.py:277). */
typedef struct grk_feature {
  const void* table;     /* [num_rows, dim], call dtype                     */
  const void* idx;       /* [num_tokens, idx_ld] index tensor, call itype   */
  int64_t num_rows;
  int64_t idx_ld;        /* elements between consecutive tokens            */
  int32_t bag;           /* index columns per token: 1 = gather, >1 = sum  */
  int32_t out_col;       /* first output column (elements)                 */
  int32_t idx_mode;      /* GRK_IDX_*                                       */
  int32_t flags;         /* GRK_FEAT_* (0: none)                            */
} grk_feature;

/* grk_feature.flags: row 0 of the table is a zero padding row, so bag slots
 * that resolve to it add nothing and are not read (round 4: the projected
 * feature tables, whose user-feature slots are padding on every item token). */
#define GRK_FEAT_SKIP_ROW0 1

/* out[n, f.out_col : f.out_col+dim] = sum_a table_f[row(n, a)] for every
 * feature f and token n < num_tokens.  Bag sums accumulate in fp32 from slot
 * 0 upward and round once.  Bit-exact with the reference lookups.
 * token_type: int32 [num_tokens] (needed by *_MASK modes), seq_len = T
 * (needed by GRK_IDX_POSITION). */
int grk_embedding_gather(const grk_feature* features, int num_features, int dim, int dtype, int itype,
                         int64_t num_tokens, const int32_t* token_type, int32_t seq_len, void* out,
                         int64_t out_ld, int32_t* err_flag, void* stream);

/* One lookup that received a gradient (source of gradient rows).  The item
 * table has three (seq, pos, neg: model/BaseLine/model.py:243,376-377).
 * Several tables stored in one flat buffer (a "table group") are reduced in
 * one call: lookup rows are shifted by row_offset into the group's rows. */
typedef struct grk_lookup {
  const void* idx;       /* index tensor as in grk_feature                 */
  const void* grad;      /* [num_tokens, grad_ld] upstream grad, grad dtype */
  int64_t num_tokens;
  int64_t idx_ld;
  int64_t grad_ld;
  int64_t row_offset;    /* group row of this lookup's table row 0         */
  int64_t table_rows;    /* rows of this lookup's table (range check)      */
  int32_t bag;
  int32_t grad_col;      /* first column of this lookup's grad rows        */
  int32_t idx_mode;
  int32_t pad_;
} grk_lookup;

/* Workspace bytes for grk_embedding_backward with `num_occurrences` =
 * sum over lookups of num_tokens * bag (0 = query failed). */
size_t grk_embedding_backward_workspace(int64_t num_occurrences, int64_t num_rows, int dim);

/* Stable LSD radix sort of (uint32 key, uint64 value) pairs by the low
 * end_bit bits of the keys (digits of up to 11 bits, three launches per digit) -- the
 * occurrence grouping inside grk_embedding_backward, exposed for tests and
 * reuse.  keys_in / vals_in are not modified; keys_tmp / vals_tmp are n-element
 * scratch; workspace: grk_sort_pairs_workspace(n) bytes. */
size_t grk_sort_pairs_workspace(int64_t n);
int grk_sort_pairs(const uint32_t* keys_in, const uint64_t* vals_in, uint32_t* keys_out, uint64_t* vals_out,
                   uint32_t* keys_tmp, uint64_t* vals_tmp, int64_t n, int end_bit, void* workspace,
                   size_t workspace_bytes, void* stream);

/* Deterministic scatter-add gradient of one table, replacing autograd's
 * embedding_dense_backward.  Occurrences (lookup order,
 * then token, then bag slot) are stably sorted by row id and reduced in fp32
 * by a load-balanced segmented reduction: every row with <= 512 occurrences
 * is summed sequentially in occurrence order (bit-identical to the reference
 * CPU backward for a single lookup); hotter rows use a fixed blocked order
 * (deterministic).  Rows == padding_idx are skipped (padding_idx < 0: none).
 *
 * Outputs (any may be NULL):
 *   dense_out  [num_rows, dim] fp32 (bf16 with GRK_BWD_DENSE_BF16): zero-filled then written
 *   uniq_ids   int64 [num_occurrences]: sorted unique row ids
 *   uniq_rows  fp32  [num_occurrences, dim]: their gradient rows
 *   uniq_count int32 [1]: number of unique rows
 * num_rows = rows of the group; padding_idx is a table-local row (each
 * lookup's row padding_idx is skipped).  Any number of lookups.
 *   row_slot   int32 [num_rows]: row_slot[id] = position in uniq_*;
 *              entries of untouched rows are left as they were (-1 by
 *              contract; grk_table_adamw restores them).
 * flags: GRK_BWD_ORDERED (every row in occurrence order, as above) or
 *   GRK_BWD_CHUNKED: a row spanning several chunks of the sorted list
 *   (grk_embedding_chunked_size() occurrences each: 256 unless the library
 *   was built with -DGRK_CHUNKED_CH=64 / 128) is summed per chunk (occurrence
 *   order) and the chunk sums are added in chunk order -- deterministic, not
 *   the sequential order.  For tables that are intermediates with no
 *   reference counterpart (the fused trainer's projected feature rows);
 *   honoured when dim is 64 x (8 bf16 / 4 or 8 fp32 elements), otherwise the
 *   call runs ordered. */
/* | GRK_BWD_DENSE_BF16 (with GRK_BWD_CHUNKED, bf16 gradients of 512 columns):
 *   dense_out is bf16 [num_rows, dim], each row rounded once from its fp32 sum
 *   (the intermediate tables are bf16: no fp32 buffer, no cast afterwards). */
enum { GRK_BWD_ORDERED = 0, GRK_BWD_CHUNKED = 1, GRK_BWD_DENSE_BF16 = 2 };
int grk_embedding_chunked_size(void);
int grk_embedding_backward(const grk_lookup* lookups, int num_lookups, int dim, int grad_dtype, int itype,
                           const int32_t* token_type, int32_t seq_len, int64_t num_rows, int64_t padding_idx,
                           void* dense_out, int64_t* uniq_ids, float* uniq_rows, int32_t* uniq_count,
                           int32_t* row_slot, int flags, void* workspace, size_t workspace_bytes,
                           int32_t* err_flag, void* stream);

/* ------------------------------------------------------------------------
 * Table optimizer: AdamW (model/BaseLine/main.py:131,189;
 * model/BaseLineO1/main.py:174,249), torch single-tensor update order.
 * ------------------------------------------------------------------------ */
enum { GRK_ADAM_DENSE = 0, GRK_ADAM_LAZY = 1 };

typedef struct grk_adamw_hparams {
  float lr, beta1, beta2, eps, weight_decay;
  float step_size;        /* lr / (1 - beta1^t)                             */
  float bias_corr2_sqrt;  /* sqrt(1 - beta2^t)                              */
  float pad_;
} grk_adamw_hparams;

/* mode GRK_ADAM_DENSE: every row of the table moves (reference semantics:
 * rows without gradient see g = 0), gradient rows found via row_slot.
 * mode GRK_ADAM_LAZY: only the uniq_count rows are updated (documented
 * deviation).  Both restore row_slot[uniq_ids[*]] = -1 when
 * uniq_ids is given; with uniq_ids NULL, row_slot is a caller-owned fixed map
 * (an identity map + a dense gradient in uniq_rows = plain dense AdamW). */
int grk_table_adamw(void* param, int param_dtype, float* exp_avg, float* exp_avg_sq, int64_t num_rows, int dim,
                    const int64_t* uniq_ids, const float* uniq_rows, const int32_t* uniq_count, int64_t max_uniq,
                    int32_t* row_slot, grk_adamw_hparams hp, int mode, void* stream);


/* Dense AdamW of num_rows rows from a dense gradient [num_rows, grad_ld]
 * (grad_dtype GRK_F32 / GRK_BF16): the update of tables whose gradient comes
 * out of a dense op (the dnn-projected feature tables, model.py).  Same update
 * order as grk_table_adamw; param / moments may point inside a larger table. */
int grk_table_adamw_dense(void* param, int param_dtype, float* exp_avg, float* exp_avg_sq, int64_t num_rows,
                          int dim, const void* grad, int grad_dtype, int64_t grad_ld, grk_adamw_hparams hp,
                          void* stream);

/* Deferred dense-parity updates.  A table whose rows carry last[row] (int32:
 * the step the row was last updated at) may skip the g = 0 updates of rows
 * outside a step's batch; before a row is read it is brought to step t by
 * replaying the skipped steps (last[row], t] in registers with those steps'
 * hyper-parameters hp_ring[s % ring_len] (the caller keeps them there), with
 * the same per-element arithmetic as grk_table_adamw -- bit-identical to
 * updating every row every step.  ids != NULL: rows ids[0 .. num_ids)
 * (duplicates allowed, each replayed once); ids == NULL: every row (flush).
 * Sets last[row] = t. */
int grk_table_adamw_catchup(void* param, int param_dtype, float* exp_avg, float* exp_avg_sq, int64_t num_rows,
                            int dim, int32_t* last, const int64_t* ids, int64_t num_ids,
                            const grk_adamw_hparams* hp_ring, int32_t ring_len, int32_t t, void* stream);

/* last[uniq_ids[0 .. *uniq_count)] = t: the rows a GRK_ADAM_LAZY update of step t moved. */
int grk_stamp_rows(int32_t* last, const int64_t* uniq_ids, const int32_t* uniq_count, int64_t max_uniq, int32_t t,
                   void* stream);

/* Device-clock forms of the four calls above, for a training step captured
 * once in a HIP graph and replayed (train.Trainer graph mode): the step t is
 * read at kernel time from *t_dev (int32 in device memory, advanced inside
 * the graph) and the hyper-parameters from hp_ring[t % ring_len] (filled by
 * the caller ahead of the steps that use them).  Same arithmetic, same
 * semantics as the by-value forms with t = *t_dev and hp = hp_ring[t % ring_len]. */
int grk_table_adamw_dev(void* param, int param_dtype, float* exp_avg, float* exp_avg_sq, int64_t num_rows, int dim,
                        const int64_t* uniq_ids, const float* uniq_rows, const int32_t* uniq_count, int64_t max_uniq,
                        int32_t* row_slot, const grk_adamw_hparams* hp_ring, int32_t ring_len, const int32_t* t_dev,
                        int mode, void* stream);
int grk_table_adamw_dense_dev(void* param, int param_dtype, float* exp_avg, float* exp_avg_sq, int64_t num_rows,
                              int dim, const void* grad, int grad_dtype, int64_t grad_ld,
                              const grk_adamw_hparams* hp_ring, int32_t ring_len, const int32_t* t_dev, void* stream);
int grk_table_adamw_catchup_dev(void* param, int param_dtype, float* exp_avg, float* exp_avg_sq, int64_t num_rows,
                                int dim, int32_t* last, const int64_t* ids, int64_t num_ids,
                                const grk_adamw_hparams* hp_ring, int32_t ring_len, const int32_t* t_dev,
                                void* stream);
int grk_stamp_rows_dev(int32_t* last, const int64_t* uniq_ids, const int32_t* uniq_count, int64_t max_uniq,
                       const int32_t* t_dev, void* stream);

/* Rolling flush of a deferred table (replaces the every-num_slices-steps full
 * flush; same reference call site as grk_table_adamw_catchup,
 * model/BaseLine/main.py:189 optimizer.step() over every table row): brings
 * slice s = (*t_dev mod num_slices) of the rows, [s * per, min((s + 1) * per,
 * num_rows)) with per = ceil(num_rows / num_slices), to step *t_dev.  Called
 * once per step, every row is replayed at least every num_slices steps, so the
 * ring must hold the hyper-parameters of steps (t - num_slices, t]. */
int grk_table_adamw_catchup_slice_dev(void* param, int param_dtype, float* exp_avg, float* exp_avg_sq,
                                      int64_t num_rows, int dim, int32_t* last, const grk_adamw_hparams* hp_ring,
                                      int32_t ring_len, const int32_t* t_dev, int32_t num_slices, void* stream);

/* l2_emb term of the BaseLine training script (model/BaseLine/main.py:184-185:
 * loss += l2_emb * torch.norm(item_emb.weight)) for the fused optimizer.
 * grk_table_l2_norm: *norm = ||param||_F (fp64 partial sums over a fixed grid,
 * deterministic), *l2_coef = l2 / ||param|| (0 for a zero table) -- the scale of
 * the term's gradient l2 * W / ||W||.  param 16-byte aligned; workspace of
 * grk_table_l2_norm_workspace() bytes.
 * grk_table_adamw_l2_dev: grk_table_adamw_dev in dense mode with every row's
 * gradient g + (*l2_coef) * p (p = the parameters before this step's update). */
/* grk_table_adamw_dev over a whole table whose gradient comes as dense blocks:
 * ranges (sorted by row_start, disjoint, at most 64) give rows [row_start,
 * row_end) the gradient rows grad + (row - row_start) * grad_ld (bf16 or
 * fp32); every other row takes g = 0 (dense parity).  One launch.
 * shadow (may be NULL; fp32 params only, 16-byte aligned): the updated
 * parameters rounded to bf16, same [num_rows, dim] layout -- the bf16 GEMM
 * operands of the dense layers (optim.DenseFlat), kept in step by the update. */
typedef struct grk_grad_range {
  int64_t row_start, row_end;
  const void* grad;
  int64_t grad_ld;
  int32_t grad_dtype;
  int32_t pad_;
} grk_grad_range;
int grk_table_adamw_ranges_dev(void* param, int param_dtype, float* exp_avg, float* exp_avg_sq, int64_t num_rows,
                               int dim, const grk_grad_range* ranges, int num_ranges,
                               const grk_adamw_hparams* hp_ring, int32_t ring_len, const int32_t* t_dev,
                               void* shadow, void* stream);

size_t grk_table_l2_norm_workspace(void);
int grk_table_l2_norm(const void* param, int param_dtype, int64_t num_rows, int dim, float l2, float* norm,
                      float* l2_coef, void* workspace, size_t workspace_bytes, void* stream);
int grk_table_adamw_l2_dev(void* param, int param_dtype, float* exp_avg, float* exp_avg_sq, int64_t num_rows, int dim,
                           const int64_t* uniq_ids, const float* uniq_rows, const int32_t* uniq_count,
                           int64_t max_uniq, int32_t* row_slot, const grk_adamw_hparams* hp_ring, int32_t ring_len,
                           const int32_t* t_dev, const float* l2_coef, void* stream);

/* ------------------------------------------------------------------------
 * Causal attention (MFMA 32x32x16 bf16)
 *   GRK_ATTN_SOFTMAX: softmax(scale * QK^T + mask) V with dropout -- the
 *     reference's F.scaled_dot_product_attention with log2feats' mask
 *     (model/BaseLine/model.py:39-43,331-335); fully-masked rows give 0.
 *   GRK_ATTN_HSTU: SiLU(scale * QK^T + rab[h, min(i-j, nb-1)]) * inv_n * mask,
 *     times V (north star; no reference -- oracle/hstu.py).
 * mask[b,i,j] = (j <= i) && key_valid[b,j]  (key_valid NULL = all valid).
 * Q/K/V are bf16 [B*T, ld] with head h at columns [h*hd, (h+1)*hd).
 * ------------------------------------------------------------------------ */
enum { GRK_ATTN_SOFTMAX = 0, GRK_ATTN_HSTU = 1 };
/* GRK_ACT_SILU: q/k/v point at PRE-activations (the uvqk projection output);
 * the kernels apply SiLU on load (rounded to bf16, as F.silu on bf16) and
 * the backward writes dq/dk/dv w.r.t. the pre-activations (x dSiLU), i.e.
 * the HSTU `u, v, q, k = split(SiLU(uvqk(x)))` is fused away. */
enum { GRK_ACT_NONE = 0, GRK_ACT_SILU = 1 };

typedef struct grk_attn_args {
  int32_t kind;                    /* GRK_ATTN_*                                  */
  int32_t batch, heads, seq_len, head_dim;   /* head_dim in {16, 32, 64, 128, 256, 512} */
  int32_t num_buckets;             /* hstu: rab columns                           */
  const void* q; const void* k; const void* v;   /* bf16                        */
  int64_t ldq, ldk, ldv;           /* row strides (elements), multiples of 8      */
  const uint8_t* key_valid;        /* [batch, seq_len] or NULL                    */
  const float* rab;                /* hstu: [heads, num_buckets] fp32             */
  float scale;                     /* softmax: 1/sqrt(hd); hstu: alpha            */
  float inv_n;                     /* hstu: 1/n                                   */
  float dropout_p;                 /* softmax training dropout                    */
  int32_t precise;                 /* 1: P / dS fed to MFMA as bf16 hi+lo pairs;
                                      2 (fp32 fidelity): Q/K/V and dO as well, each
                                      product as hi*hi + hi*lo + lo*hi; q/k/v then
                                      have dtype qkv_dtype (whole-sequence kernels,
                                      and head_dim 256 / 512 in the wide-head
                                      kernels; GRK_EUNSUPPORTED elsewhere)       */
  uint64_t seed;                   /* dropout stream                              */
  int32_t out_dtype;               /* GRK_F32 / GRK_BF16 for out, dq, dk, dv      */
  int32_t act;                     /* GRK_ACT_*: activation applied to q/k/v      */
  const int32_t* seq_range;        /* optional [B, 3] from grk_seq_ranges (first
                                      valid key, contiguous flag, order); NULL =
                                      derived from key_valid inside every launch
                                      (workgroups then in batch order)          */
  const uint64_t* seed_dev;        /* optional: the dropout seed in device memory,
                                      read by the kernels when they run (replaces
                                      `seed`): a step replayed from a HIP graph
                                      draws a fresh mask every replay           */
  int32_t qkv_dtype;               /* precise == 2: GRK_F32 / GRK_F16 / GRK_BF16
                                      q/k/v (read exactly, split into bf16 hi+lo).
                                      precise 0 / 1: GRK_BF16, or GRK_FP8_E4M3 --
                                      q/k/v are fp8 ACTIVATIONS (act NONE; long-
                                      sequence config C5): QK^T on the fp8 MFMA
                                      (forward, dK/dV), every other product on
                                      bf16 MFMA over the exactly widened values;
                                      head_dim 64 / 128, no time bias; 8-byte
                                      aligned, ld in elements (= bytes)         */
  /* HSTU time bias (SURVEY §8 a9 rab_time; whole-sequence, chunked and
   * wide-head kernels; not with fp8 q/k/v):
   * S[i,j] += rab_t[h, tb(ts[i] - ts[j])] with
   * tb(d) = min(2 l + h1, num_time_buckets - 1), l = floor(log2(|d| + 1)),
   * h1 = the bit below the leading one of |d| + 1 (0 when l = 0): half-octave
   * buckets of the time gap, integer-exact.  Gaps are taken of the times
   * relative to the sequence's first valid event, clamped to +-(2^30 - 1). */
  const int64_t* timestamps;       /* [batch, seq_len] event times or NULL        */
  const float* rab_t;              /* [heads, num_time_buckets] fp32              */
  int32_t num_time_buckets;        /* 0 = no time bias; <= 64                     */
  float* drab_t;                   /* backward: [heads, num_time_buckets] fp32,
                                      the time-bias gradient is ADDED into it    */
  int64_t* drab_t_ws;              /* backward: int64 [heads, num_time_buckets]
                                      scratch (fixed-point accumulator)          */
  /* Jagged (valid-token) layout, optional: the rows of q/k/v, out, dout, dq,
   * dk, dv hold only each sequence's span [start_b, seq_len) (start_b =
   * seq_range[3 b], REQUIRED with it), packed back to back: token (b, t) is row
   * row_base[b] + t (int64 [batch]; grk_jagged_layout builds both).  Padding
   * rows before start_b are neither read nor written.  NULL = the padded
   * [batch * seq_len] layout.  Whole-sequence kernels (T * head_dim within
   * their LDS budget) only: other shapes return GRK_EUNSUPPORTED.  The rows
   * [*num_rows, capacity) past the spans (dead capacity rows of the step) of
   * every output written (out; dq / dk / dv) are set to zero, so no stale
   * value reaches the row-wise ops and weight gradients around. */
  const int64_t* row_base;
  const int64_t* num_rows;         /* jagged: span rows (device), with row_base */
  int64_t capacity;                /* jagged: rows of the q/k/v / output buffers */
} grk_attn_args;

/* 1 when grk_attention_* with precise == 2 (fp32 fidelity) runs for this
 * sequence length and head_dim (the whole-sequence kernels' LDS; head_dim 256
 * and 512 at any length), else 0. */
int grk_attention_fidelity_supported(int seq_len, int head_dim);

/* ranges int32 [batch, 3]: ranges[b][0] = first j with key_valid[b, j] (T for
 * an all-padding row), ranges[b][1] = 1 if the valid keys are exactly
 * [first, T) else 0, ranges[i][2] = the sequence with the i-th largest
 * T - first (ties by index): the whole-sequence attention kernels take their
 * workgroups in that order (longest first; results do not depend on it).  One
 * call per step serves every attention launch of that step (all layers, fwd
 * and bwd). */
int grk_seq_ranges(const uint8_t* key_valid, int batch, int seq_len, int32_t* ranges, void* stream);

/* Jagged (valid-token) layout of a left-padded batch (the reference runs every
 * token-wise op over all B*T rows, model/BaseLine/model.py:331-350, 379-384;
 * the rows before a sequence's first valid key are dead).  Writes
 * ranges [batch, 3] (= grk_seq_ranges), row_base int64 [batch] (token (b, t) of
 * the span [start_b, seq_len) is row row_base[b] + t), row_map int32 [capacity]
 * (row r <- token index b * seq_len + t; -1 for the dead rows r >= n) and
 * *num_rows = n (int64, device).  next_token_type (optional, int32 [batch,
 * seq_len]): err_flag bit 1 if a token before its span has next_token_type == 1;
 * bit 2 if the spans hold more than capacity rows: then the trailing spans that
 * do not fit are dropped (ranges start = seq_len: an empty sequence to every
 * kernel, row_base -seq_len, *num_rows = the kept rows <= capacity), so no
 * kernel of the step addresses a row past capacity.  err_flag is OR-ed into,
 * never cleared. */
int grk_jagged_layout(const uint8_t* key_valid, int batch, int seq_len, int64_t capacity,
                      const int32_t* next_token_type, int32_t* ranges, int64_t* row_base, int32_t* row_map,
                      int64_t* num_rows, int32_t* err_flag, void* stream);

/* Projected-table index of the fused model (model._projection; the reference's
 * per-feature lookups model/BaseLine/model.py:254-277 restated over the stacked
 * projected tables P): out[r, out_col_k + j] = src_k[r, j] > 0 ? src_k[r, j] +
 * offset_k : 0 for every block k (its feature's index columns; offset_k = its
 * table's first P row), int64 out [rows, >= sum of widths]; the blocks tile the
 * columns in order (out_col_0 = 0).  src int32 or int64 (itype), at most 64
 * blocks.  One launch. */
typedef struct grk_index_block {
  const void* src;       /* [rows, src_ld] index values, itype              */
  int64_t src_ld;        /* elements between consecutive rows              */
  int64_t width;         /* index columns of this block                    */
  int64_t out_col;       /* first output column                            */
  int64_t offset;        /* added to every non-zero value                  */
} grk_index_block;
int grk_proj_index(const grk_index_block* blocks, int num_blocks, int itype, int64_t rows, int64_t* out,
                   int64_t out_ld, void* stream);

/* Dense column blocks written into a row-major [rows, out_ld] buffer (bf16 or
 * fp32) in ONE launch -- the gather buffer's mm-embedding columns (fp32
 * [rows, 32] -> the dnn operand, model/BaseLine/model.py:290-299) and its
 * constant [1, 0, ...] bias / padding columns (one source row broadcast:
 * src_ld = 0).  Blocks in column order, disjoint; fp32 -> bf16 rounds to
 * nearest even. */
typedef struct grk_column_block {
  const void* src;       /* [rows, src_ld] or one row (src_ld = 0)           */
  int64_t src_ld;        /* elements; 0 = broadcast row 0                    */
  int32_t width;         /* columns                                          */
  int32_t out_col;       /* first output column                              */
  int32_t src_dtype;     /* GRK_F32 / GRK_BF16                               */
  int32_t pad_;
} grk_column_block;
int grk_write_columns(const grk_column_block* blocks, int num_blocks, int64_t rows, void* out, int64_t out_ld,
                      int out_dtype, void* stream);

/* Rows of the item / user tables a training batch reads (model/BaseLine/
 * model.py:331-350, 376-377), -1 for padding: item_ids [3n] = (item ids of item
 * tokens | pos | neg), user_ids [n] = user ids of user tokens (NULL: skipped).
 * seq / pos / neg / token_type: n elements each of itype.  The ids the deferred
 * dense-parity table AdamW catches up before the forward. */
int grk_batch_row_ids(const void* seq, const void* pos, const void* neg, const void* token_type, int itype,
                      int64_t n, int64_t* item_ids, int64_t* user_ids, void* stream);

/* Multi-tensor row gather for the jagged layout: for each copy,
 * dst + r * dst_ld <- src + row_map[r] * src_ld (row_bytes bytes; zeros where
 * row_map[r] < 0), r in [0, rows), all copies in one launch.  row_bytes,
 * strides and pointers multiples of 4; at most 64 copies. */
typedef struct grk_row_copy {
  const void* src;
  void* dst;
  int64_t row_bytes, src_ld, dst_ld;
} grk_row_copy;
int grk_gather_rows(const grk_row_copy* copies, int num_copies, const int32_t* row_map, int64_t rows, void* stream);

/* Row-sharded tables (sharding.ShardExchange.route; replaces the sort-based torch
 * route): the distinct ids of ids[n] grouped by owner (id % world) and ascending
 * inside an owner -> send_ids[0, n_uniq); send_counts[world] = distinct ids per
 * owner (the all-to-all split sizes); inverse[i] = slot of ids[i] in send_ids (-1
 * for ids outside [0, global_rows)); bad[0] = how many such ids; n_uniq (may be
 * NULL).  rows_per_owner * world >= global_rows (local row = id / world).  ws:
 * grk_route_workspace(world, rows_per_owner) bytes.  Deterministic, graph-safe. */
size_t grk_route_workspace(int world, int64_t rows_per_owner);
int grk_route(const int64_t* ids, int64_t n, int world, int64_t rows_per_owner, int64_t global_rows,
              int64_t* send_ids, int64_t* inverse, int64_t* send_counts, int64_t* n_uniq, int64_t* bad, void* ws,
              size_t ws_bytes, void* stream);

/* The dense gradients of one all-reduce bucket into its fp32 flat buffer
 * (sharding.GradBuckets): dst[dst_offset + e] = src[e] for e < count (bf16 / fp32
 * -> fp32), zeros where src is NULL; at most 64 ranges per launch. */
typedef struct grk_pack_range {
  const void* src;
  int64_t count;
  int64_t dst_offset;
  int32_t src_dtype;
  int32_t pad_;
} grk_pack_range;
int grk_flat_pack(const grk_pack_range* ranges, int num_ranges, float* dst, void* stream);

/* Row-sharded tables + jagged rows (train.jagged_remaps): for every role (at most 8)
 * out[r] = inv[row_map[r]] for r < rows; a dead row (row_map[r] < 0) reads
 * inv[first padding position of the role] -- the role's id at position i is ids[i],
 * or 0 where tt is given and tt[i] != tt_want; position 0 when no id is 0.  One launch. */
typedef struct grk_remap_role {
  const int64_t* inv;   /* [n] fetched-row slot of every [B, T] position */
  int64_t* out;         /* [rows] */
  const int64_t* ids;   /* [n] the role's ids */
  const int64_t* tt;    /* [n] token types or NULL */
  int64_t tt_want;
  int64_t n;
} grk_remap_role;
int grk_jagged_remap(const grk_remap_role* roles, int num_roles, const int32_t* row_map, int64_t rows, void* stream);

/* out [B*T, ldo] (out_dtype); lse fp32 [B, H, T] (softmax: natural-log
 * logsumexp of the masked scaled scores, -inf for fully-masked rows). */
int grk_attention_fwd(const grk_attn_args* a, void* out, int64_t ldo, float* lse, void* stream);

/* Gradients of grk_attention_fwd for upstream dout (dout_dtype).  Softmax
 * needs the forward out/lse and a delta workspace fp32 [B, H, T]; hstu
 * accumulates drab fp32 [H, nb] (NULL = rab is frozen, its gradient is not
 * computed) through drab_ws, an int64 [H, nb] scratch: the partial sums are
 * 64-bit fixed point (value * 2^32), so drab is deterministic.  dq/dk/dv are written
 * (not accumulated) in out_dtype; deterministic. */
int grk_attention_bwd(const grk_attn_args* a, const void* out, int64_t ldo, const void* dout, int64_t lddo,
                      int dout_dtype, const float* lse, float* delta_ws, void* dq, int64_t lddq, void* dk,
                      int64_t lddk, void* dv, int64_t lddv, float* drab, int64_t* drab_ws, void* stream);

/* grk_attention_bwd in two independent halves, for callers that schedule
 * them separately (two streams, or timing one kernel):
 *   GRK_ATTN_BWD_DQ   -- softmax delta, dq, and drab (with its scratch reset
 *                        and fixed-point finalize);
 *   GRK_ATTN_BWD_DKDV -- dk and dv (softmax: reads the delta the DQ half wrote).
 * parts = GRK_ATTN_BWD_DQ | GRK_ATTN_BWD_DKDV is grk_attention_bwd.  Arguments
 * a half does not use may be NULL (DQ: dk/dv; DKDV: dq, drab). */
#define GRK_ATTN_BWD_DQ 1
#define GRK_ATTN_BWD_DKDV 2
/* Flags for the DQ half (hstu with drab):
 *   GRK_ATTN_BWD_WS_CLEAN -- drab_ws (int64 [H, nb] + ONE extra slot, a counter)
 *                        and drab_t_ws are zero on entry and are left zero on
 *                        return: no reset launch, and the whole-sequence dq
 *                        kernel's last workgroup finalizes drab (no finalize
 *                        launch).  A caller keeps one such scratch per stream;
 *   GRK_ATTN_BWD_DRAB_SET -- drab / drab_t are written, not accumulated (the
 *                        caller's buffers need no zero fill). */
#define GRK_ATTN_BWD_WS_CLEAN 4
#define GRK_ATTN_BWD_DRAB_SET 8
int grk_attention_bwd_parts(const grk_attn_args* a, const void* out, int64_t ldo, const void* dout, int64_t lddo,
                            int dout_dtype, const float* lse, float* delta_ws, void* dq, int64_t lddq, void* dk,
                            int64_t lddk, void* dv, int64_t lddv, float* drab, int64_t* drab_ws, int parts,
                            void* stream);

/* ------------------------------------------------------------------------
 * HSTU output gate (north star; no reference -- oracle/hstu.py)
 *   y = dropout(LayerNorm(o; gamma, beta, eps) * SiLU(u))
 * the tail of the HSTU layer before out_linear, with u the first D columns of
 * the uvqk pre-activation.  o, u, y, gy, dout, du: bf16 rows (16-byte
 * aligned, strides multiples of 8); gamma/beta/dgamma/dbeta fp32 [dim];
 * dim multiple of 8, <= 2048.  stats fp32 [rows, 2] = (mean, rstd) saved by
 * the forward for the backward.  Dropout: counter hash of (seed, row, col),
 * identical in both directions; seed_dev (optional, device memory) replaces
 * seed with the value it holds when the kernel runs (HIP-graph replay).
 * ------------------------------------------------------------------------ */
/* fp8 HSTU layer (config C5): out[n, c] = e4m3(SiLU(pre[n, c])) for the
 * layer's v|q|k pre-activation columns (bf16 in, OCP e4m3 out: fp32 SiLU,
 * round to nearest even, clamped to +-448); and the straight-through backward
 * g[n, c] *= dSiLU(pre[n, c]) in place (bf16).  cols multiple of 8; pre / g
 * rows 16-byte aligned, out rows 8-byte aligned. */
int grk_silu_fp8(const void* pre, int64_t ldpre, int64_t rows, int cols, void* out, int64_t ldout, void* stream);
int grk_dsilu_mul(void* g, int64_t ldg, const void* pre, int64_t ldpre, int64_t rows, int cols, void* stream);

/* Embedding combine (round 4), the first block's input in log2feats
 * (replaces model/BaseLine/model.py:313-321, the seqs = item + user features,
 * *= sqrt(d), += pos_emb, emb_dropout chain; the ReLUs of itemdnn / userdnn,
 * model.py:302-309, folded in with relu != 0):
 *   y = dropout((act(a) + act(b)) * scale + pos),  act = ReLU if relu else identity
 * bf16 rows (strides multiples of 8, 16-byte aligned); b and pos optional.
 * Backward: g = gy * keep / (1 - p); gpos = g; ga = g * scale * [a > 0 if relu],
 * gb likewise (each output optional).  The dropout decisions are the
 * norm-gate's counter hash of (seed, row, col); seed_dev as there. */
int grk_emb_combine_fwd(const void* a, int64_t lda, const void* b, int64_t ldb, const void* pos, int64_t ldp,
                        float scale, int relu, int64_t rows, int dim, float dropout_p, uint64_t seed,
                        const uint64_t* seed_dev, void* y, int64_t ldy, void* stream);
int grk_emb_combine_bwd(const void* gy, int64_t ldgy, const void* a, int64_t lda, const void* b, int64_t ldb,
                        float scale, int relu, int64_t rows, int dim, float dropout_p, uint64_t seed,
                        const uint64_t* seed_dev, void* ga, int64_t ldga, void* gb, int64_t ldgb, void* gpos,
                        int64_t ldgp, void* stream);

int grk_norm_gate_fwd(const void* o, int64_t ldo, const void* u, int64_t ldu, const float* gamma,
                      const float* beta, float eps, int64_t rows, int dim, float dropout_p, uint64_t seed,
                      const uint64_t* seed_dev, void* y, int64_t ldy, float* stats, void* stream);

size_t grk_norm_gate_bwd_workspace(int64_t rows, int dim);

/* dout = dL/do, du = dL/du (w.r.t. the pre-activation u), dgamma/dbeta
 * written (not accumulated); fixed-order, deterministic reductions. */
int grk_norm_gate_bwd(const void* gy, int64_t ldgy, const void* o, int64_t ldo, const void* u, int64_t ldu,
                      const float* gamma, const float* beta, const float* stats, int64_t rows, int dim,
                      float dropout_p, uint64_t seed, const uint64_t* seed_dev, void* dout, int64_t lddo, void* du,
                      int64_t lddu,
                      float* dgamma, float* dbeta, void* ws, size_t ws_bytes, void* stream);

/* Residual add + LayerNorm of the HSTU block's residual stream (replaces the
 * `seqs = seqs + mha_outputs` / `attention_layernorms[i](seqs)` /
 * `last_layernorm(log_feats)` pair of model/BaseLine/model.py:330-345 under
 * bf16 autocast).  s, y, s_out bf16 [rows, dim]: s_out = bf16(s + y); with y
 * NULL the LayerNorm reads s and s_out is not written.  x = LN(s_out) * gamma
 * + beta (fp32 math) stored as x_dtype (bf16: the next GEMM's operand; fp32:
 * the last norm); stats [rows, 2] = (mean, rstd). */
int grk_add_norm_fwd(const void* s, int64_t lds, const void* y, int64_t ldy, const float* gamma, const float* beta,
                     float eps, int64_t rows, int dim, void* s_out, int64_t ldso, void* x, int64_t ldx, int x_dtype,
                     float* stats, void* stream);
size_t grk_add_norm_bwd_workspace(int64_t rows, int dim);
/* ds = gs + dL/ds_out through the LayerNorm for upstream gx (x_dtype) and the
 * residual stream's own gradient gs (bf16, NULL = 0), rounded once to bf16
 * (ds is the gradient of both s and y); dgamma/dbeta written, fixed-order. */
int grk_add_norm_bwd(const void* gx, int64_t ldgx, int gx_dtype, const void* gs, int64_t ldgs, const void* s_new,
                     int64_t lds, const float* gamma, const float* stats, int64_t rows, int dim, void* ds,
                     int64_t ldds, float* dgamma, float* dbeta, void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Pair logits + BCE (model/BaseLine/model.py:379-382; main.py:177-182)
 * ------------------------------------------------------------------------ */
/* Floats of `partials` workspace needed for num_rows rows. */
size_t grk_pair_logits_partials(int64_t num_rows);

/* pos/neg_logits[n] = <h_n, e_pos_n> / <h_n, e_neg_n>, zeroed where
 * next_token_type[n] != 1 (NULL: every row valid).  If `loss` is non-NULL it
 * also writes the reference BCE loss (mean over valid rows of
 * softplus(-pos) plus mean of softplus(neg)) and the valid-row count, reduced
 * in a fixed order.  Inputs share `dtype`, or GRK_F32_BF16: h fp32, e_pos /
 * e_neg bf16 (the same logits as promoting e to fp32, bitwise). */
int grk_pair_logits_fwd(const void* h, int64_t ldh, const void* e_pos, int64_t ldp, const void* e_neg, int64_t ldn,
                        const int32_t* next_token_type, int64_t num_rows, int dim, int dtype, float* pos_logits,
                        float* neg_logits, float* partials, float* loss, int32_t* count, void* stream);

/* dh = gp*e_pos + gn*e_neg, de_pos = gp*h, de_neg = gn*h per row.
 * Either gpos/gneg (fp32 per-row upstream grads of the logits; rows with
 * next_token_type != 1 get 0, as the forward masked them) are given, or -- when
 * pos_logits/neg_logits are non-NULL -- the BCE coefficients
 * gp = g*(sigmoid(pos)-1)/count, gn = g*sigmoid(neg)/count on valid rows,
 * with g = *grad_loss (device scalar; NULL = 1).  Outputs may be NULL; with
 * GRK_F32_BF16, dh is fp32 and de_pos / de_neg bf16. */
int grk_pair_logits_bwd(const void* h, int64_t ldh, const void* e_pos, int64_t ldp, const void* e_neg, int64_t ldn,
                        int64_t num_rows, int dim, int dtype, const float* gpos, const float* gneg,
                        const float* pos_logits, const float* neg_logits, const int32_t* next_token_type,
                        const int32_t* count, const float* grad_loss, void* dh, int64_t lddh, void* de_pos,
                        int64_t lddp, void* de_neg, int64_t lddn, void* stream);

/* ------------------------------------------------------------------------
 * In-batch sampled softmax (north star; no reference -- oracle/loss.py)
 *   z_ij = <h_i, e_j> / tau - log_q[j] over valid columns j; j != i masked when
 *   item_ids[j] == item_ids[i]; loss = mean_valid_i (logsumexp_j z_ij - z_ii)
 * log_q (optional fp32 [num_rows], natural log, NULL = 0): the logQ correction
 * -- log of the sampling probability of position j's item, subtracted from
 * every logit of column j (Yi et al., RecSys 2019).
 * h, e: bf16 [num_rows, ld] (dim in {32, 64, 128, 256, 512}); valid uint8.
 * Only valid positions take part: the kernels list them on the device
 * (compact index = rank among the valid positions) and size their grids for
 * num_rows, so nothing waits on the host.  Workspace: one buffer of
 * grk_sampled_softmax_workspace(num_rows, dim) bytes, reusable between calls.
 * ------------------------------------------------------------------------ */
size_t grk_sampled_softmax_workspace(int64_t num_rows, int dim);

/* Writes lse2 fp32 [num_rows] (log2-domain logsumexp of the c-th valid row at
 * index c, c < count), the loss and the valid-row count (fixed-order
 * reduction). */
int grk_sampled_softmax_fwd(const void* h, int64_t ldh, const void* e, int64_t lde, const int64_t* item_ids,
                            const uint8_t* valid, int64_t num_rows, int dim, float tau, const float* log_q,
                            float* lse2, float* loss, int32_t* count, void* workspace, size_t workspace_bytes,
                            void* stream);

/* Fused backward (no nv x nv matrix): with G = (softmax - I) * grad_loss /
 * (count * tau) on valid (row, column) pairs, dh = G e and de = G^T h, fp32
 * [num_rows, ld] (16-byte aligned rows, ld >= dim, ld % 4 == 0); rows of
 * positions that are not valid are zero.  G enters the MFMA as bf16 hi + lo:
 * fp32-level error.  grad_loss: device scalar (NULL = 1). */
int grk_sampled_softmax_bwd(const void* h, int64_t ldh, const void* e, int64_t lde, const int64_t* item_ids,
                            const uint8_t* valid, int64_t num_rows, int dim, float tau, const float* log_q,
                            const float* lse2, const float* grad_loss, float* dh, int64_t lddh, float* de, int64_t ldde,
                            void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Plain GEMM for the dense layers around the hot path (HSTU uvqk /
 * out_linear, itemdnn / userdnn: forward, dX and the weight gradients), on
 * hipBLASLt with a workspace so its stream-K kernels are eligible
 * (replaces the torch.nn.Linear / torch.addmm calls of
 * model/BaseLine/model.py:86-92,129-139 for the fused path).
 * Row-major, as torch tensors: C[m, n] = alpha * op(A) @ op(B) + beta * C_in
 * (+ bias[n] broadcast over rows); C_in = c_in, or C itself when c_in is NULL
 * (c_in has C's dtype and ldc).  op(A) is [m, k]: A stored [m, k] (lda >= k)
 * or, trans_a, [k, m] (lda >= m); op(B) is [k, n]: B stored [k, n] (ldb >= n)
 * or, trans_b, [n, k] (ldb >= k).  A, B bf16; C bf16 or fp32 (fp32 C with
 * beta = 1 accumulates a weight gradient in place); bias bf16 or fp32 or
 * NULL.  fp32 accumulation.  One plan per shape: the fastest of hipBLASLt's
 * heuristic candidates, timed on the shape's first call (see
 * grk_gemm_tuning), then fixed for the process. */
int grk_gemm(int trans_a, int trans_b, int64_t m, int64_t n, int64_t k, const void* a, int64_t lda, const void* b,
             int64_t ldb, int ab_dtype, void* c, int64_t ldc, int c_dtype, const void* c_in, float alpha, float beta,
             const void* bias, int bias_dtype, void* stream);

/* grk_gemm with an epilogue: GRK_GEMM_EP_RELU stores max(alpha op(A) op(B) + beta C
 * (+ bias), 0) -- the itemdnn / userdnn ReLU (model/BaseLine/model.py:302-309) in the
 * GEMM's store instead of a separate pass. */
#define GRK_GEMM_EP_NONE 0
#define GRK_GEMM_EP_RELU 1
int grk_gemm_ex(int trans_a, int trans_b, int64_t m, int64_t n, int64_t k, const void* a, int64_t lda, const void* b,
                int64_t ldb, int ab_dtype, void* c, int64_t ldc, int c_dtype, const void* c_in, float alpha,
                float beta, const void* bias, int bias_dtype, int epilogue, void* stream);

/* grk's own MFMA GEMM (csrc/grk_mgemm.hip), which grk_gemm / grk_gemm_ex run for
 * every shape grk_gemm_mfma_supported accepts (hipBLASLt for the rest; env
 * GRK_GEMM_BACKEND=hipblaslt forces hipBLASLt).  Replaces the bf16-autocast
 * forward and input-gradient products of the dense layers
 * (model/BaseLine/model.py:129-139,302-309 and the HSTU uvqk / out_linear):
 *   C[m, n] = act(A . op(B) + bias[n] + C_in[m, n]),  A [m, k] (lda) bf16,
 *   b_layout 0: B [n, k] (ldb) -> op(B) = B^T;  1: B [k, n] (ldb) -> op(B) = B;
 *   C bf16 or fp32 (ldc); C_in NULL or a C-shaped matrix of C's dtype and ldc
 *   (may be C itself: accumulate); bias NULL or [n] fp32 / bf16; act by
 *   GRK_GEMM_EP_*.  n, k, lda, ldb, ldc multiples of 8, pointers 16-byte aligned;
 *   fp32 accumulation, one rounding at the store, deterministic.
 * grk_gemm_mfma_supported: 1 when a grk_gemm_ex call with these arguments runs
 * here (trans_a 0, alpha 1, beta 0 or 1). */
int grk_gemm_mfma_supported(int trans_a, int b_layout, int64_t m, int64_t n, int64_t k, int64_t lda, int64_t ldb,
                            int64_t ldc, int c_dtype, float alpha, float beta);
int grk_gemm_mfma(int b_layout, int64_t m, int64_t n, int64_t k, const void* a, int64_t lda, const void* b,
                  int64_t ldb, void* c, int64_t ldc, int c_dtype, const void* c_in, const void* bias, int bias_dtype,
                  int epilogue, void* stream);

/* Number of hipBLASLt candidates grk_gemm times for each NEW shape (1..256,
 * default 256; env GRK_GEMM_TUNE at load).  1 = the heuristic's first pick,
 * with no timing: the same kernel in every process. */
int grk_gemm_tuning(int candidates);

/* Weight gradient of a dense layer (the dW / db half of autograd for
 * nn.Linear / Conv1d(k=1), model/BaseLine/model.py:65-78,129-139,302-309 and
 * the HSTU projections, under bf16 autocast):
 *   dw[m][n] = sum_k dy[k][m] * x[k][n]      (fp32 accumulation; dw fp32 or bf16)
 *   db[m]    = sum_k dy[k][m]                (fp32; NULL = not wanted)
 * dy [k, m] and x [k, n] bf16 row-major (row strides ld_dy, ld_x, multiples of
 * 8; 16-byte aligned), m and n multiples of 8.  Split-K MFMA kernel + an
 * in-order slice reduction: deterministic.  workspace: caller-owned device
 * memory of grk_wgrad_workspace(k, m, n) bytes. */
size_t grk_wgrad_workspace(int64_t k, int64_t m, int64_t n);
int grk_wgrad(const void* dy, int64_t ld_dy, const void* x, int64_t ld_x, int64_t k, int64_t m, int64_t n, void* dw,
              int64_t ld_dw, int dw_dtype, float* db, void* workspace, size_t workspace_bytes, void* stream);

/* Grouped GEMMs of the projected feature tables (model._projection; replaces the
 * torch.bmm stacks over the per-feature tables of model/BaseLine/model.py:254-310
 * as restated by the projection P_f = E_f W_f^T).  One group per table, at most
 * 32 per launch; operands bf16, fp32 accumulation, every pointer 16-byte aligned
 * and every row stride of a / b a multiple of 8 elements.
 *
 * grk_grouped_gemm: C_g [rows_g, n] = A_g [rows_g, k] . op(B_g), A K-contiguous
 * (row stride lda); b_layout 0: B_g [n, k] (C = A B^T), 1: B_g [k, n] (C = A B);
 * C fp32 or bf16 (c_dtype), row stride ldc; k a multiple of 32.  (b_rows unused.)
 *
 * grk_grouped_wgrad: C_g [m, n] fp32 (row stride ldc, a multiple of 4) =
 * A_g^T B_g with A_g [rows_g, m], B_g [rows_g, n] row-major, rows_g a multiple
 * of 32; B's rows past b_rows are read as its row b_rows - 1 (A's rows there
 * must be zero: they then add exact zeros).  Split-K slices summed in slice
 * order (deterministic); workspace of grk_grouped_wgrad_workspace() bytes. */
typedef struct grk_gemm_group {
  const void* a;
  int64_t lda;
  const void* b;
  int64_t ldb;
  void* c;
  int64_t ldc;
  int64_t rows;
  int64_t b_rows;
} grk_gemm_group;
int grk_grouped_gemm(const grk_gemm_group* groups, int num_groups, int b_layout, int64_t n, int64_t k, int c_dtype,
                     void* stream);
size_t grk_grouped_wgrad_workspace(const grk_gemm_group* groups, int num_groups, int64_t m, int64_t n);
int grk_grouped_wgrad(const grk_gemm_group* groups, int num_groups, int64_t m, int64_t n, void* workspace,
                      size_t workspace_bytes, void* stream);

/* Exact maximum-inner-product top-k retrieval: the ANN step of inference
 * (model/BaseLine/infer.py:213-225 runs an external faiss HNSW binary with
 * --faiss_metric_type=0 (inner product) --query_ann_top_k=10 over the
 * embedding.fbin / id.u64bin written by save_item_emb, model/BaseLine/
 * model.py:402-433, and query.fbin; results read back by read_result_ids,
 * infer.py:51-65).  Brute force on the GPU instead of a graph index:
 *   for each query q: the k items i maximising dot(queries[q], items[i]),
 *   ordered by score descending, ties by item index ascending.
 * queries [num_queries, dim] and items [num_items, dim] row-major, both of
 * `dtype` (GRK_F32 / GRK_BF16), row strides ld_q / ld_i (elements), 16-byte
 * aligned rows; dim a multiple of 8 and <= 512; 1 <= k <= 16.
 * Pass 1 scores every (query, item) pair with bf16 MFMA and keeps 16
 * candidates per query per item slice; pass 2 re-scores the candidates in
 * fp32 (fixed summation order) and selects the k best, so scores and order
 * are those of fp32 arithmetic.  out_scores [num_queries, k] fp32, out_ids
 * [num_queries, k] int64 = item_ids[i] (uint64 retrieval ids; NULL = the
 * item index i); slots past num_items get id -1 and score -inf (as faiss).
 * workspace: grk_mips_topk_workspace(num_queries, num_items) bytes. */
size_t grk_mips_topk_workspace(int64_t num_queries, int64_t num_items);
int grk_mips_topk(const void* queries, int64_t ld_q, const void* items, int64_t ld_i, int dtype,
                  int64_t num_queries, int64_t num_items, int dim, int k, const uint64_t* item_ids,
                  float* out_scores, int64_t* out_ids, void* workspace, size_t workspace_bytes, void* stream);

/* Negative sampling on the device: the per-position random negative of
 * MyDataset.__getitem__ (model/BaseLine/dataset.py:136-162; _random_neq,
 * :79-95) for a whole tensorised batch.  For every sequence b and position t
 * with next_token_type == 1 and pos != 0: neg[b,t] = a uniform id in
 * [1, num_items] not in excl[b, 0:excl_len] (0 entries ignored), redrawn up to
 * max_tries (<= 65535) times (the reference redraws without bound; if every try is
 * excluded the last draw is kept and bit 2 of *err_flag is set); other
 * positions 0.  Draws are splitmix64(seed, b, t, attempt): deterministic, so
 * oracle/sampler.py restates them bit-exactly (the reference's np.random
 * stream is not reproducible on a GPU).  pos / next_token_type / neg int32
 * [batch, seq_len], seq_len <= 65535; excl int32 [batch, excl_len], any length, any order,
 * duplicates allowed (set semantics; lists of <= 8192 entries are sorted in LDS and
 * binary-searched, longer ones scanned in global memory).
 * item_feat (optional, int32 [num_items + 1, num_feat], row 0 = the default
 * feature values): neg_feat[b,t,:] = item_feat[neg[b,t],:] -- the
 * fill_missing_feat(item_feat_dict[neg]) rows of dataset.py:161-162,
 * tensorised.  item_ok (optional, uint8 [num_items + 1]): a draw v with
 * item_ok[v] == 0 is redrawn like an excluded one -- the reference's
 * `str(t) not in self.item_feat_dict` test (dataset.py:92); NULL = every id
 * has a feature row. */
int grk_sample_negatives(const int32_t* pos, const int32_t* next_token_type, int64_t batch, int32_t seq_len,
                         const int32_t* excl, int32_t excl_len, int64_t num_items, uint64_t seed,
                         int32_t max_tries, const int32_t* item_feat, int32_t num_feat, const uint8_t* item_ok,
                         int32_t* neg, int32_t* neg_feat, int32_t* err_flag, void* stream);

/* Residual quantisation -- the code search of config 4's RQ-VAE semantic-ID
 * tokenizer (BASELINE.json configs[3]; the reference has no tokenizer: the
 * semantic ids it produces enter the O1 model as item_sparse features,
 * model/BaseLineO1/model.py:271-280, 355).  z [n, dim] fp32 row-major (row
 * stride ld_z, 16-byte aligned), codebooks [levels, codes, dim] fp32
 * contiguous; dim in {16, 32, 64, 128}, 1 <= levels <= 8.  Per row:
 * r_0 = z; code_l = argmin_k sum_j (r_l[j] - C_l[k][j])^2 in fp32 (difference,
 * square and running sum each rounded, j ascending; lowest k on ties);
 * r_{l+1} = r_l - C_l[code_l].  out_codes int32 [n, levels]; optional (NULL =
 * skipped): out_quant [n, dim] = C_0[code_0] + C_1[code_1] + ... (level
 * order), out_dist [n, levels] = the minimum distances, out_resid [n, dim] =
 * r_levels.  Bit-exact vs oracle/rqvae.py. */
int grk_rq_assign(const float* z, int64_t ld_z, const float* codebooks, int64_t n, int dim, int codes, int levels,
                  int32_t* out_codes, float* out_quant, float* out_dist, float* out_resid, void* stream);

/* Host-side batch assembly of the columnar token store (seqstore.SeqStore,
 * SURVEY.md §8(f) #1).  Replaces the per-token feature dicts of
 * MyDataset.__getitem__ + fill_missing_feat (model/BaseLine/dataset.py:
 * 136-169, 254-262) and feat2tensor (model/BaseLine/model.py:186-224) for a
 * whole batch: no GPU, no allocation, plain loads and stores on host memory
 * (DataLoader workers call it).
 *
 * The store holds, per token t: sparse[t, f_sparse] int32 feature ids,
 * arr[t, f_array, a_cap] int32 array values (zero past each length) with
 * arr_len[t, f_array], mm[t, f_mm] int32 rows of the multimodal tables. */
typedef struct grk_store_view {
  const int32_t* sparse; /* [tokens, f_sparse] */
  const int32_t* arr;    /* [tokens, f_array, a_cap] */
  const int32_t* arr_len;/* [tokens, f_array] */
  const int32_t* mm;     /* [tokens, f_mm] */
  int64_t tokens;
  int32_t f_sparse, f_array, a_cap, f_mm;
} grk_store_view;

enum { GRK_STORE_SPARSE = 0, GRK_STORE_ARRAY = 1, GRK_STORE_MM = 2 };

/* One output column: kind, its column in the store block, width (ARRAY: the
 * output row width A, 1 <= A <= a_cap; MM: the table's row length; SPARSE: 1),
 * mm_table (MM only: fp32 [mm_rows, width], row 0 = the zero row, mm_rows
 * bounds the stored row ids), out (SPARSE: int64 [n]; ARRAY: int64 [n, A];
 * MM: fp32 [n, width]). */
typedef struct grk_store_col {
  int32_t kind, src_col, width, pad_;
  int64_t mm_rows;
  const float* mm_table;
  void* out;
} grk_store_col;

/* Output position i (0 <= i < n) is token tok[i] where sel[i] != 0 and the
 * default (feature id 0 / array [0] padded with 0 / mm table row 0) where
 * sel[i] == 0: out SPARSE[i] = sparse[tok, c]; ARRAY[i, j] = arr[tok, c, j]
 * for j < arr_len[tok, c], else 0; MM[i, :] = mm_table[mm[tok, c], :].
 * Fails (GRK_EINVAL, nothing written) when a selected tok[i] or a stored mm row
 * is out of range. */
int grk_store_features(const grk_store_view* store, const int64_t* tok, const uint8_t* sel, int64_t n,
                       const grk_store_col* cols, int num_cols);

/* widths[c] = max(1, max over selected i of arr_len[tok[i], c]) for c < f_array:
 * the batch's longest array per array feature (feat2tensor pads to it). */
int grk_store_array_widths(const grk_store_view* store, const int64_t* tok, const uint8_t* sel, int64_t n,
                           int32_t* widths);

#ifdef __cplusplus
}
#endif
#endif /* GRK_H_ */
