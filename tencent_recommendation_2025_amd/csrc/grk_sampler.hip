// GPU negative sampler: the per-position random negative of MyDataset.__getitem__
// (model/BaseLine/dataset.py:136-162, _random_neq at :79-95), drawn on the device
// for a whole tensorised batch instead of per sample in DataLoader workers.
//
// Reference semantics, per sequence b:
//   ts   = the item ids of the user's sequence (dataset.py:136-139);
//   for every position t whose next token is an item (next_token_type == 1)
//   with a non-zero positive: neg[t] = uniform draw from [1, item_num] not in ts
//   and with a feature row (redrawn until both hold: `t in s or str(t) not in
//   self.item_feat_dict`, dataset.py:92), other positions 0 (dataset.py:156-161).
// Here ts is the caller's exclusion list excl[b, 0:excl_len] (0 entries are
// ignored); the torch side passes the batch window's item tokens and positives.
// "Has a feature row" is the optional byte mask item_ok[id] (NULL: every id has one).
// The draws come from a counter-based generator (splitmix64 of seed, b, t and the
// attempt number), so the result is a pure function of (inputs, seed): the oracle
// (oracle/sampler.py) restates it bit-exactly.  The reference's np.random stream
// cannot be reproduced on a GPU; the distribution is the same (uniform over the
// allowed ids).
//
// One workgroup per sequence, one lane per position.  Exclusion lists of up to
// kLdsExcl entries are staged once in LDS and bitonic-sorted there (padding
// 0x7FFFFFFF: never drawn), so every membership test is a 13-step binary search
// over LDS; longer lists (users with very long histories) are scanned in global
// memory (L2-served: one workgroup rereads its own row).  The list's order and
// duplicates do not matter (set semantics, as the reference's `ts`), so no
// length cap and no truncation.  Integer work on a few KB per sequence:
// launch-bound, never HBM- or MFMA-bound.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "grk.h"
#include "grk_common.h"

namespace grk {
namespace {

constexpr int kSampBlock = 256;
constexpr int kLdsExcl = 8192;  // LDS: 32 KiB of int32
constexpr int32_t kPadId = 0x7FFFFFFF;

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// draw a (0-based) of position (b, t): an id in [1, num_items], by the high word of
// a 64x64-bit product (no modulo bias beyond 2^-32 relative)
__device__ __forceinline__ int32_t draw(uint64_t seed, int64_t b, int32_t t, int32_t a, int64_t num_items) {
  uint64_t x = splitmix64(seed ^ splitmix64(((uint64_t)b << 32) ^ ((uint64_t)(uint32_t)t << 16) ^ (uint64_t)a));
  return (int32_t)(__umul64hi(x, (uint64_t)num_items) + 1);
}

__global__ void __launch_bounds__(kSampBlock)
    k_sample_negatives(const int32_t* __restrict__ pos, const int32_t* __restrict__ ntt, int32_t T,
                       const int32_t* __restrict__ excl, int32_t excl_len, int64_t num_items, uint64_t seed,
                       int32_t max_tries, const int32_t* __restrict__ item_feat, int32_t num_feat,
                       const uint8_t* __restrict__ item_ok, int32_t* __restrict__ neg, int32_t* __restrict__ neg_feat, int32_t* err_flag) {
  __shared__ int32_t ex[kLdsExcl];
  const int64_t b = blockIdx.x;
  const int32_t* e = excl + b * (int64_t)excl_len;
  const bool in_lds = excl_len <= kLdsExcl;
  int n2 = 1;  // sorted image size: a power of two >= excl_len
  if (in_lds) {
    while (n2 < excl_len) n2 <<= 1;
    for (int i = threadIdx.x; i < n2; i += kSampBlock) ex[i] = i < excl_len ? e[i] : kPadId;
    __syncthreads();
    for (int k = 2; k <= n2; k <<= 1)          // bitonic sort, ascending
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = threadIdx.x; i < n2; i += kSampBlock) {
          const int l = i ^ j;
          if (l > i) {
            const int32_t x = ex[i], y = ex[l];
            if (((i & k) == 0) ? (x > y) : (x < y)) { ex[i] = y; ex[l] = x; }
          }
        }
        __syncthreads();
      }
  }
  for (int32_t t = threadIdx.x; t < T; t += kSampBlock) {
    const int64_t o = b * (int64_t)T + t;
    int32_t v = 0;
    if (ntt[o] == 1 && pos[o] != 0) {
      bool hit = true;
      for (int32_t a = 0; a < max_tries && hit; ++a) {
        v = draw(seed, b, t, a, num_items);
        hit = item_ok != nullptr && item_ok[v] == 0;
        if (in_lds) {
          int base = 0;  // number of entries < v (binary search over the sorted image)
          for (int half = n2 >> 1; half >= 1; half >>= 1)
            if (ex[base + half - 1] < v) base += half;
          hit |= ex[base] == v;
        } else {
          for (int i = 0; i < excl_len && !hit; ++i) hit = e[i] == v;
        }
      }
      if (hit && err_flag) atomicOr(err_flag, 2);  // every try was excluded: the last draw is kept
    }
    neg[o] = v;
    if (item_feat)
      for (int f = 0; f < num_feat; ++f) neg_feat[o * num_feat + f] = item_feat[(int64_t)v * num_feat + f];
  }
}

}  // namespace
}  // namespace grk

using namespace grk;

extern "C" int grk_sample_negatives(const int32_t* pos, const int32_t* next_token_type, int64_t batch,
                                    int32_t seq_len, const int32_t* excl, int32_t excl_len, int64_t num_items,
                                    uint64_t seed, int32_t max_tries, const int32_t* item_feat, int32_t num_feat,
                                    const uint8_t* item_ok, int32_t* neg, int32_t* neg_feat, int32_t* err_flag, void* stream) {
  clear_error();
  GRK_CHECK_ARG(batch >= 0 && seq_len > 0, "bad batch (%lld) / seq_len (%d)", (long long)batch, seq_len);
  GRK_CHECK_ARG(num_items >= 1 && num_items < 0x7FFFFFFFLL, "num_items must be in [1, 2^31 - 1)");
  GRK_CHECK_ARG(excl_len >= 0, "excl_len (%d) must be >= 0", excl_len);
  GRK_CHECK_ARG(excl_len == 0 || excl, "excl is NULL");
  GRK_CHECK_ARG(max_tries >= 1 && max_tries <= 65535, "max_tries must be in [1, 65535]");
  GRK_CHECK_ARG(seq_len <= 65535, "seq_len must be <= 65535");
  GRK_CHECK_ARG(!item_feat || (num_feat > 0 && neg_feat), "item_feat needs num_feat > 0 and neg_feat");
  if (batch == 0) return GRK_OK;
  GRK_CHECK_ARG(pos && next_token_type && neg, "NULL pos / next_token_type / neg");
  hipStream_t s = (hipStream_t)stream;
  k_sample_negatives<<<dim3((unsigned)batch), kSampBlock, 0, s>>>(pos, next_token_type, seq_len, excl, excl_len,
                                                                   num_items, seed, max_tries, item_feat,
                                                                   num_feat, item_ok, neg, neg_feat, err_flag);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}
