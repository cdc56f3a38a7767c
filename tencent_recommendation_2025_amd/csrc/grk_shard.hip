// Row-sharded table exchange on the device (sharding.ShardExchange.route,
// sharding.GradBuckets): SURVEY.md §8(e), the multi-GPU scale-out of the north star.
//
//  * grk_route: the routing plan of one table's ids for a step -- the distinct ids
//    grouped by owner rank (owner = id % world, local row = id / world) and ascending
//    inside an owner, the per-owner counts (the all-to-all split sizes), each id's
//    slot in that order (the inverse map the model's lookups read the fetched rows
//    through), and the count of ids outside [0, global_rows).  A presence bitmap over
//    the composite key owner * rows_per_owner + local orders the distinct ids without
//    a sort: mark (atomicOr), per-word popcount prefix, emit, rank lookup -- five
//    launches over a bitmap of world * rows_per_owner bits (1M rows: 128 KB), against
//    the ~20 torch launches per table of the sort-based route it replaces
//    (ShardExchange._route_torch, kept for gloo / CPU).  Deterministic: the bitmap and
//    every rank are functions of the id set.
//  * grk_flat_pack: the dense gradients of one all-reduce bucket copied (bf16 / fp32 ->
//    fp32) into the bucket's flat buffer in one launch (was one torch cast / cat
//    kernel per parameter); a range with a null source is zero-filled (a parameter
//    without a gradient this step).
#include <string.h>

#include <algorithm>

#include "grk_common.h"

namespace grk {
namespace {

constexpr int kRouteThreads = 256;
constexpr int kRouteWordsPerBlock = 1024;  // bitmap words per workgroup in the count / emit passes

__global__ void __launch_bounds__(kRouteThreads) k_route_mark(const int64_t* __restrict__ ids, int64_t n, int world,
                                                              int64_t rows_per_owner, int64_t global_rows,
                                                              unsigned* __restrict__ bitmap,
                                                              unsigned long long* __restrict__ bad) {
  __shared__ unsigned wbad[kRouteThreads / 64];
  unsigned nbad = 0;
  // A batch repeats ids in runs (the padding row of every non-item token, hot items):
  // atomics on one word serialise (one table's 41k ids took 0.4 ms), so a lane whose
  // id equals its left neighbour's, or whose bit is already visible, adds nothing.
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t span = (n + stride - 1) / stride * stride;  // every lane runs every round (the shuffle)
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < span; i += stride) {
    const int64_t id = i < n ? ids[i] : -1;
    const int64_t left = __shfl_up(id, 1);
    if (i >= n) continue;
    if (id < 0 || id >= global_rows) {
      ++nbad;
      continue;
    }
    if ((threadIdx.x & 63) != 0 && left == id) continue;
    const uint64_t key = (uint64_t)(id % world) * (uint64_t)rows_per_owner + (uint64_t)(id / world);
    const unsigned bit = 1u << (key & 31);
    if (__builtin_nontemporal_load(&bitmap[key >> 5]) & bit) continue;
    atomicOr(&bitmap[key >> 5], bit);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) nbad += __shfl_xor(nbad, off);
  if ((threadIdx.x & 63) == 0) wbad[threadIdx.x >> 6] = nbad;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned t = 0;
#pragma unroll
    for (int w = 0; w < kRouteThreads / 64; ++w) t += wbad[w];
    if (t) atomicAdd(bad, (unsigned long long)t);
  }
}

// Set bits per block of kRouteWordsPerBlock words.
__global__ void __launch_bounds__(kRouteThreads) k_route_count(const unsigned* __restrict__ bitmap, int64_t nwords,
                                                               unsigned* __restrict__ bcount) {
  __shared__ unsigned red[kRouteThreads / 64];
  const int64_t w0 = (int64_t)blockIdx.x * kRouteWordsPerBlock;
  unsigned c = 0;
  for (int k = threadIdx.x; k < kRouteWordsPerBlock; k += blockDim.x)
    if (w0 + k < nwords) c += __popc(bitmap[w0 + k]);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned t = 0;
#pragma unroll
    for (int w = 0; w < kRouteThreads / 64; ++w) t += red[w];
    bcount[blockIdx.x] = t;
  }
}

// Exclusive scan of the block counts in place (one workgroup), total at bcount[nb].
__global__ void __launch_bounds__(1024) k_route_scan(unsigned* __restrict__ bcount, int nb) {
  __shared__ unsigned part[1024];
  __shared__ unsigned carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int base = 0; base < nb; base += 1024) {
    const int i = base + threadIdx.x;
    const unsigned v = i < nb ? bcount[i] : 0u;
    part[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
      const unsigned u = threadIdx.x >= o ? part[threadIdx.x - o] : 0u;
      __syncthreads();
      part[threadIdx.x] += u;
      __syncthreads();
    }
    if (i < nb) bcount[i] = carry + part[threadIdx.x] - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry += part[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) bcount[nb] = carry;
}

// Per word: the rank of its first set bit (word_prefix), and every set bit's id
// written at its rank (send_ids: owner-major, ascending local row).
__global__ void __launch_bounds__(kRouteThreads) k_route_emit(const unsigned* __restrict__ bitmap, int64_t nwords,
                                                              const unsigned* __restrict__ boff, int world,
                                                              int64_t rows_per_owner,
                                                              unsigned* __restrict__ word_prefix,
                                                              int64_t* __restrict__ send_ids) {
  constexpr int PER = kRouteWordsPerBlock / kRouteThreads;  // consecutive words per thread
  __shared__ unsigned part[kRouteThreads];
  const int64_t w0 = (int64_t)blockIdx.x * kRouteWordsPerBlock + (int64_t)threadIdx.x * PER;
  unsigned bits[PER], c = 0;
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    bits[e] = w0 + e < nwords ? bitmap[w0 + e] : 0u;
    c += __popc(bits[e]);
  }
  part[threadIdx.x] = c;
  __syncthreads();
  for (int o = 1; o < kRouteThreads; o <<= 1) {
    const unsigned u = threadIdx.x >= o ? part[threadIdx.x - o] : 0u;
    __syncthreads();
    part[threadIdx.x] += u;
    __syncthreads();
  }
  unsigned run = boff[blockIdx.x] + part[threadIdx.x] - c;
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    if (w0 + e >= nwords) break;
    word_prefix[w0 + e] = run;
    unsigned b = bits[e];
    while (b) {
      const int k = __ffs(b) - 1;
      b &= b - 1;
      const uint64_t key = (uint64_t)(w0 + e) * 32 + k;
      const int64_t owner = (int64_t)(key / (uint64_t)rows_per_owner);
      const int64_t local = (int64_t)(key % (uint64_t)rows_per_owner);
      send_ids[run++] = local * world + owner;
    }
  }
}

__device__ __forceinline__ int64_t route_rank(const unsigned* __restrict__ bitmap,
                                              const unsigned* __restrict__ word_prefix, uint64_t key) {
  const unsigned w = bitmap[key >> 5];
  return (int64_t)word_prefix[key >> 5] + __popc(w & ((1u << (key & 31)) - 1u));
}

// Every id's slot (-1 for ids outside the table); workgroup 0 also writes the
// per-owner counts and the distinct-id total.
__global__ void __launch_bounds__(kRouteThreads) k_route_inverse(const int64_t* __restrict__ ids, int64_t n,
                                                                 int world, int64_t rows_per_owner,
                                                                 int64_t global_rows, int64_t nbits,
                                                                 const unsigned* __restrict__ bitmap,
                                                                 const unsigned* __restrict__ word_prefix,
                                                                 const unsigned* __restrict__ total,
                                                                 int64_t* __restrict__ inverse,
                                                                 int64_t* __restrict__ send_counts,
                                                                 int64_t* __restrict__ n_uniq,
                                                                 const unsigned long long* __restrict__ nbad,
                                                                 int64_t* __restrict__ bad) {
  if (blockIdx.x == 0 && (int)threadIdx.x <= world) {
    // rank of the first key of owner w (w = world: the total)
    auto first = [&](int w) -> int64_t {
      const uint64_t k = (uint64_t)w * (uint64_t)rows_per_owner;
      return k >= (uint64_t)nbits ? (int64_t)*total : route_rank(bitmap, word_prefix, k);
    };
    const int w = threadIdx.x;
    if (w < world) send_counts[w] = first(w + 1) - first(w);
    else {
      if (n_uniq) *n_uniq = first(world);
      *bad = (int64_t)*nbad;
    }
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t id = ids[i];
    if (id < 0 || id >= global_rows) {
      inverse[i] = -1;
      continue;
    }
    const uint64_t key = (uint64_t)(id % world) * (uint64_t)rows_per_owner + (uint64_t)(id / world);
    inverse[i] = route_rank(bitmap, word_prefix, key);
  }
}

constexpr int kPackMax = 64;
constexpr int kPackPiece = 2048;  // elements per workgroup
struct PackRanges {
  grk_pack_range r[kPackMax];
  int64_t piece0[kPackMax + 1];   // first piece of each range (prefix of ceil(count / kPackPiece))
  int n;
};

__global__ void __launch_bounds__(256) k_flat_pack(PackRanges pr, float* __restrict__ dst) {
  const int64_t piece = blockIdx.x;
  int k = 0;
  while (k + 1 < pr.n && piece >= pr.piece0[k + 1]) ++k;
  const grk_pack_range& r = pr.r[k];
  const int64_t e0 = (piece - pr.piece0[k]) * kPackPiece;
  float* out = dst + r.dst_offset;
#pragma unroll
  for (int j = 0; j < kPackPiece / 256; ++j) {
    const int64_t e = e0 + j * 256 + threadIdx.x;
    if (e >= r.count) break;
    float v = 0.f;
    if (r.src) v = r.src_dtype == GRK_F32 ? reinterpret_cast<const float*>(r.src)[e]
                                          : bf16_to_f32(reinterpret_cast<const bf16_t*>(r.src)[e]);
    out[e] = v;
  }
}

// Jagged rows under the row-sharded tables (train.jagged_remaps): each role's
// fetched-row index carried into the jagged row order, out[r] = inv[row_map[r]]; a
// dead row (row_map -1) reads the slot of the role's first padding id (position 0
// when the role has none), found by the wave that needs it, 64 ids per ballot.
constexpr int kRemapMax = 8;
struct RemapRoles {
  grk_remap_role r[kRemapMax];
};

__global__ void __launch_bounds__(256) k_jagged_remap(RemapRoles rr, const int32_t* __restrict__ row_map,
                                                      int64_t rows) {
  const grk_remap_role& R = rr.r[blockIdx.y];
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int m = r < rows ? row_map[r] : 0;
  const bool dead = r < rows && m < 0;
  int64_t pad = 0;
  if (__ballot(dead)) {  // wave-uniform: the first position whose id is the padding id 0
    const int lane = threadIdx.x & 63;
    pad = -1;
    for (int64_t b = 0; b < R.n && pad < 0; b += 64) {
      const int64_t i = b + lane;
      bool z = false;
      if (i < R.n) {
        const int64_t id = R.ids[i];
        z = R.tt ? (R.tt[i] != R.tt_want || id == 0) : id == 0;
      }
      const unsigned long long mask = __ballot(z);
      if (mask) pad = b + __ffsll((long long)mask) - 1;
    }
    if (pad < 0) pad = 0;
  }
  if (r < rows) R.out[r] = dead ? R.inv[pad] : R.inv[m];
}

}  // namespace
}  // namespace grk

using namespace grk;

static int64_t route_nwords(int world, int64_t rows_per_owner) {
  const int64_t nbits = (int64_t)world * rows_per_owner;
  return (nbits + 31) / 32;
}

extern "C" size_t grk_route_workspace(int world, int64_t rows_per_owner) {
  if (world < 1 || rows_per_owner < 1) return 0;
  const int64_t nwords = route_nwords(world, rows_per_owner);
  const int64_t nb = (nwords + kRouteWordsPerBlock - 1) / kRouteWordsPerBlock;
  // bitmap, word prefix, block offsets (+ total), the bad-id counter
  return sizeof(unsigned long long) + (size_t)(2 * nwords + nb + 1) * sizeof(unsigned);
}

extern "C" int grk_route(const int64_t* ids, int64_t n, int world, int64_t rows_per_owner, int64_t global_rows,
                         int64_t* send_ids, int64_t* inverse, int64_t* send_counts, int64_t* n_uniq,
                         int64_t* bad, void* ws, size_t ws_bytes, void* stream) {
  clear_error();
  GRK_CHECK_ARG(world >= 1 && world <= 64, "world must be in [1, 64]");
  GRK_CHECK_ARG(rows_per_owner >= 1 && global_rows >= 0 && global_rows <= (int64_t)world * rows_per_owner,
                "rows_per_owner * world must cover global_rows");
  GRK_CHECK_ARG((int64_t)world * rows_per_owner < ((int64_t)1 << 37), "bitmap too large");
  GRK_CHECK_ARG(n >= 0 && (n == 0 || (ids && send_ids && inverse)), "bad ids / outputs");
  GRK_CHECK_ARG(send_counts && bad && ws, "send_counts, bad and ws are required");
  GRK_CHECK_ARG(ws_bytes >= grk_route_workspace(world, rows_per_owner), "workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int64_t nbits = (int64_t)world * rows_per_owner;
  const int64_t nwords = route_nwords(world, rows_per_owner);
  const int64_t nb = (nwords + kRouteWordsPerBlock - 1) / kRouteWordsPerBlock;
  GRK_CHECK_ARG(nb < (1 << 30), "bitmap too large");
  unsigned long long* nbad = (unsigned long long*)ws;  // [bad-id counter | bitmap | word prefix | block offsets]
  unsigned* bitmap = (unsigned*)(nbad + 1);
  unsigned* word_prefix = bitmap + nwords;
  unsigned* boff = word_prefix + nwords;
  // the counter and the bitmap start at zero (a kernel, not hipMemsetAsync: graph-safe)
  GRK_CHECK_HIP(zero_async(ws, sizeof(unsigned long long) + (size_t)nwords * sizeof(unsigned), s));
  const int gmark = (int)std::min<int64_t>(std::max<int64_t>((n + kRouteThreads - 1) / kRouteThreads, 1), 2048);
  k_route_mark<<<gmark, kRouteThreads, 0, s>>>(ids, n, world, rows_per_owner, global_rows, bitmap, nbad);
  GRK_LAUNCH_CHECK();
  k_route_count<<<(unsigned)nb, kRouteThreads, 0, s>>>(bitmap, nwords, boff);
  GRK_LAUNCH_CHECK();
  k_route_scan<<<1, 1024, 0, s>>>(boff, (int)nb);
  GRK_LAUNCH_CHECK();
  k_route_emit<<<(unsigned)nb, kRouteThreads, 0, s>>>(bitmap, nwords, boff, world, rows_per_owner, word_prefix,
                                                      send_ids);
  GRK_LAUNCH_CHECK();
  k_route_inverse<<<gmark, kRouteThreads, 0, s>>>(ids, n, world, rows_per_owner, global_rows, nbits, bitmap,
                                                  word_prefix, boff + nb, inverse, send_counts, n_uniq, nbad, bad);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

extern "C" int grk_flat_pack(const grk_pack_range* ranges, int num_ranges, float* dst, void* stream) {
  clear_error();
  GRK_CHECK_ARG(num_ranges >= 0 && num_ranges <= kPackMax, "num_ranges must be in [0, %d]", kPackMax);
  GRK_CHECK_ARG(num_ranges == 0 || (ranges && dst), "bad ranges / dst");
  if (num_ranges == 0) return GRK_OK;
  PackRanges pr;
  memset(&pr, 0, sizeof(pr));
  pr.n = num_ranges;
  int64_t pieces = 0;
  for (int k = 0; k < num_ranges; ++k) {
    const grk_pack_range& r = ranges[k];
    GRK_CHECK_ARG(r.count >= 0 && r.dst_offset >= 0, "range %d: count / dst_offset", k);
    GRK_CHECK_ARG(!r.src || r.src_dtype == GRK_F32 || r.src_dtype == GRK_BF16, "range %d: src_dtype", k);
    pr.r[k] = r;
    pr.piece0[k] = pieces;
    pieces += (r.count + kPackPiece - 1) / kPackPiece;
  }
  pr.piece0[num_ranges] = pieces;
  if (pieces == 0) return GRK_OK;
  GRK_CHECK_ARG(pieces < ((int64_t)1 << 31), "too many elements");
  k_flat_pack<<<(unsigned)pieces, 256, 0, (hipStream_t)stream>>>(pr, dst);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

extern "C" int grk_jagged_remap(const grk_remap_role* roles, int num_roles, const int32_t* row_map, int64_t rows,
                                void* stream) {
  clear_error();
  GRK_CHECK_ARG(num_roles >= 0 && num_roles <= kRemapMax, "num_roles must be in [0, %d]", kRemapMax);
  GRK_CHECK_ARG(rows >= 0 && (rows == 0 || num_roles == 0 || (roles && row_map)), "bad roles / row_map");
  if (rows == 0 || num_roles == 0) return GRK_OK;
  RemapRoles rr;
  memset(&rr, 0, sizeof(rr));
  for (int k = 0; k < num_roles; ++k) {
    GRK_CHECK_ARG(roles[k].inv && roles[k].out && roles[k].ids && roles[k].n >= 1, "role %d: inv / out / ids / n", k);
    rr.r[k] = roles[k];
  }
  const dim3 grid((unsigned)((rows + 255) / 256), (unsigned)num_roles);
  k_jagged_remap<<<grid, 256, 0, (hipStream_t)stream>>>(rr, row_map, rows);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}
