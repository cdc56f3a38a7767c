// Index arithmetic of the fused training step, one launch each instead of a
// chain of torch elementwise kernels (round 4: ~5 launches per call for the
// projected lookups' index, ~10 per step for the deferred tables' catch-up ids).
//
//  * grk_proj_index: the projected feature tables P = E_f W_f^T of the fused
//    model (model._projection) are looked up as ONE bag over the stacked P: a
//    token's bag is the concatenation of its features' index columns, each
//    shifted to its table's first P row, padding (0) kept at 0 -- the
//    reference's per-feature nn.Embedding(padding_idx=0) lookups
//    (model/BaseLine/model.py:254-277) restated over P.
//  * grk_write_columns: the dense column blocks of the gather buffer (mm
//    embeddings, the dnn operands' constant bias / padding columns) in one
//    launch (were one copy kernel per block).
//  * grk_batch_row_ids: the rows of the item / user tables a training batch
//    reads (model/BaseLine/model.py:331-350, 376-377: item ids of item tokens,
//    pos, neg; user ids of user tokens), -1 for padding -- the ids the deferred
//    dense-parity AdamW brings up to date before the forward
//    (optim.FusedAdamW.begin_step).
// Integer work of a few hundred KB: launch-bound; grid-stride, 256 threads.
#include <string.h>

#include "grk_common.h"

namespace grk {
namespace {

constexpr int kMaxIndexBlocks = 64;
struct IndexBlocks {
  grk_index_block b[kMaxIndexBlocks];
};

template <typename I>
__global__ void __launch_bounds__(256) k_proj_index(IndexBlocks ib, int nb, int64_t rows, int64_t width,
                                                    int64_t* __restrict__ out, int64_t out_ld) {
  const int64_t total = rows * width;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / width;
    const int c = (int)(i - r * width);
    int k = 0;
    while (k + 1 < nb && c >= ib.b[k + 1].out_col) ++k;
    const grk_index_block& b = ib.b[k];
    const int64_t v = (int64_t)reinterpret_cast<const I*>(b.src)[r * b.src_ld + (c - b.out_col)];
    out[r * out_ld + c] = v > 0 ? v + b.offset : 0;
  }
}

template <typename I>
__global__ void __launch_bounds__(256) k_batch_row_ids(const I* __restrict__ seq, const I* __restrict__ pos,
                                                       const I* __restrict__ neg, const I* __restrict__ tt, int64_t n,
                                                       int64_t* __restrict__ item, int64_t* __restrict__ user) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = (int64_t)seq[i], t = (int64_t)tt[i];
    const int64_t p = (int64_t)pos[i], q = (int64_t)neg[i];
    item[i] = (t == 1 && s > 0) ? s : -1;
    item[n + i] = p > 0 ? p : -1;
    item[2 * n + i] = q > 0 ? q : -1;
    if (user) user[i] = (t == 2 && s > 0) ? s : -1;
  }
}

// Dense column blocks into a row-major buffer (the gather buffer's mm-embedding
// columns and its constant [1, 0, ...] bias / padding columns): one thread per
// output element, blocks found by their column range, dtype converted on the
// way (fp32 -> bf16 rounds to nearest even, as torch's copy_).
constexpr int kMaxColumnBlocks = 16;
struct ColumnBlocks {
  grk_column_block b[kMaxColumnBlocks];
};

template <typename OT>
__global__ void __launch_bounds__(256) k_write_columns(ColumnBlocks cb, int nb, int64_t rows, int width,
                                                       OT* __restrict__ out, int64_t out_ld) {
  const int64_t total = rows * width;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / width;
    int c = (int)(i - r * width);
    int k = 0;
    while (k + 1 < nb && c >= cb.b[k].width) {
      c -= cb.b[k].width;
      ++k;
    }
    const grk_column_block& b = cb.b[k];
    const int64_t si = (b.src_ld ? r * b.src_ld : 0) + c;
    const float v = b.src_dtype == GRK_F32 ? reinterpret_cast<const float*>(b.src)[si]
                                           : bf16_to_f32(reinterpret_cast<const bf16_t*>(b.src)[si]);
    OT* dst = out + r * out_ld + b.out_col + c;
    if constexpr (sizeof(OT) == 4) *dst = v;
    else *dst = f32_to_bf16(v);
  }
}

}  // namespace
}  // namespace grk

using namespace grk;

extern "C" int grk_write_columns(const grk_column_block* blocks, int num_blocks, int64_t rows, void* out,
                                 int64_t out_ld, int out_dtype, void* stream) {
  clear_error();
  GRK_CHECK_ARG(num_blocks >= 1 && num_blocks <= kMaxColumnBlocks, "num_blocks must be in [1, %d]", kMaxColumnBlocks);
  GRK_CHECK_ARG(out_dtype == GRK_F32 || out_dtype == GRK_BF16, "out_dtype must be GRK_F32 or GRK_BF16");
  GRK_CHECK_ARG(rows >= 0 && blocks && (out || rows == 0), "bad rows / blocks / out");
  ColumnBlocks cb;
  memset(&cb, 0, sizeof(cb));
  int width = 0;
  for (int k = 0; k < num_blocks; ++k) {
    const grk_column_block& b = blocks[k];
    GRK_CHECK_ARG(b.src && b.width >= 1 && (b.src_ld == 0 || b.src_ld >= b.width), "block %d: src / width / src_ld", k);
    GRK_CHECK_ARG(b.src_dtype == GRK_F32 || b.src_dtype == GRK_BF16, "block %d: src_dtype", k);
    GRK_CHECK_ARG(b.out_col >= 0 && b.out_col + b.width <= out_ld, "block %d: columns past out_ld", k);
    GRK_CHECK_ARG(k == 0 || b.out_col >= blocks[k - 1].out_col + blocks[k - 1].width,
                  "block %d: blocks must be in column order and disjoint", k);
    cb.b[k] = b;
    width += b.width;
  }
  if (rows == 0) return GRK_OK;
  const int g = grid_for(rows * width, 256);
  if (out_dtype == GRK_F32)
    k_write_columns<float><<<g, 256, 0, (hipStream_t)stream>>>(cb, num_blocks, rows, width, (float*)out, out_ld);
  else
    k_write_columns<bf16_t><<<g, 256, 0, (hipStream_t)stream>>>(cb, num_blocks, rows, width, (bf16_t*)out, out_ld);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

extern "C" int grk_proj_index(const grk_index_block* blocks, int num_blocks, int itype, int64_t rows, int64_t* out,
                              int64_t out_ld, void* stream) {
  clear_error();
  GRK_CHECK_ARG(num_blocks >= 1 && num_blocks <= kMaxIndexBlocks, "num_blocks must be in [1, %d]", kMaxIndexBlocks);
  GRK_CHECK_ARG(itype == GRK_I32 || itype == GRK_I64, "itype must be GRK_I32 or GRK_I64");
  GRK_CHECK_ARG(rows >= 0 && blocks && (out || rows == 0), "bad rows / blocks / out");
  IndexBlocks ib;
  memset(&ib, 0, sizeof(ib));
  int64_t col = 0;
  for (int k = 0; k < num_blocks; ++k) {
    const grk_index_block& b = blocks[k];
    GRK_CHECK_ARG(b.src && b.width >= 1 && b.src_ld >= b.width && b.offset >= 0,
                  "block %d: src / width / src_ld / offset", k);
    GRK_CHECK_ARG(b.out_col == col, "block %d: out_col %lld (the blocks tile the columns in order: expected %lld)", k,
                  (long long)b.out_col, (long long)col);
    ib.b[k] = b;
    col += b.width;
  }
  GRK_CHECK_ARG(out_ld >= col, "out_ld %lld < %lld columns", (long long)out_ld, (long long)col);
  if (rows == 0) return GRK_OK;
  const int g = grid_for(rows * col, 256);
  if (itype == GRK_I64)
    k_proj_index<int64_t><<<g, 256, 0, (hipStream_t)stream>>>(ib, num_blocks, rows, col, out, out_ld);
  else
    k_proj_index<int32_t><<<g, 256, 0, (hipStream_t)stream>>>(ib, num_blocks, rows, col, out, out_ld);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

extern "C" int grk_batch_row_ids(const void* seq, const void* pos, const void* neg, const void* token_type, int itype,
                                 int64_t n, int64_t* item_ids, int64_t* user_ids, void* stream) {
  clear_error();
  GRK_CHECK_ARG(itype == GRK_I32 || itype == GRK_I64, "itype must be GRK_I32 or GRK_I64");
  GRK_CHECK_ARG(n >= 0 && (n == 0 || (seq && pos && neg && token_type && item_ids)), "bad inputs");
  if (n == 0) return GRK_OK;
  const int g = grid_for(n, 256);
  hipStream_t s = (hipStream_t)stream;
  if (itype == GRK_I64)
    k_batch_row_ids<int64_t><<<g, 256, 0, s>>>((const int64_t*)seq, (const int64_t*)pos, (const int64_t*)neg,
                                              (const int64_t*)token_type, n, item_ids, user_ids);
  else
    k_batch_row_ids<int32_t><<<g, 256, 0, s>>>((const int32_t*)seq, (const int32_t*)pos, (const int32_t*)neg,
                                              (const int32_t*)token_type, n, item_ids, user_ids);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}
