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
//  * grk_batch_row_ids: the rows of the item / user tables a training batch
//    reads (model/BaseLine/model.py:331-350, 376-377: item ids of item tokens,
//    pos, neg; user ids of user tokens), -1 for padding -- the ids the deferred
//    dense-parity AdamW brings up to date before the forward
//    (optim.FusedAdamW.begin_step).
// Integer work of a few hundred KB: launch-bound; grid-stride, 256 threads.
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

}  // namespace
}  // namespace grk

using namespace grk;

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
