// Embedding-table hot path for gfx950: fused multi-table gather / bag-sum and
// the deterministic scatter-add gradient.
//
// Reference call sites replaced:
//   forward : nn.Embedding lookups in feat2emb / log2feats
//             (model/BaseLine/model.py:242-247,275,277,328;
//              model/BaseLineO1/model.py:345-350,380,383,439)
//   backward: autograd embedding_dense_backward of those lookups.
//
// Both directions are HBM-bound byte movers: one 16-byte vector per lane,
// consecutive lanes on consecutive bytes of one row, no LDS, no MFMA.
#include <string.h>

#include <stdlib.h>

#include <algorithm>
#include <utility>

#include "grk_common.h"

namespace grk {

struct FeatArgs {
  grk_feature f[GRK_MAX_FEATURES];
};

constexpr int kLookupsPerLaunch = 16;

struct LookupArgs {
  grk_lookup l[kLookupsPerLaunch];
  int64_t occ_off[kLookupsPerLaunch + 1];  // occurrence offsets, absolute
  int num;
};

template <typename I>
__device__ __forceinline__ int64_t resolve_row(const I* idx, int64_t n, int32_t a, int64_t ld, int mode,
                                               const int32_t* token_type, int32_t T) {
  int64_t v = (int64_t)idx[n * ld + a];
  switch (mode) {
    case GRK_IDX_ITEM_MASK: return token_type[n] == 1 ? v : 0;
    case GRK_IDX_USER_MASK: return token_type[n] == 2 ? v : 0;
    case GRK_IDX_POSITION: return v != 0 ? (int64_t)(n % T) + 1 : 0;
    default: return v;
  }
}

// ---------------------------------------------------------------- gather ----
// grid.y = feature; grid.x strides over (token, 16-byte chunk) units of that
// feature.  Each lane moves one 16-byte vector per unit; UNROLL units are in
// flight per lane (the launcher uses 1, see grk_embedding_gather).
template <typename T, typename I, int UNROLL>
__global__ void __launch_bounds__(256) k_gather(FeatArgs args, int dim, int64_t num_tokens,
                                                const int32_t* __restrict__ token_type, int32_t T_len,
                                                T* __restrict__ out, int64_t out_ld, int32_t* err_flag) {
  constexpr int VEC = Vec16<T>::N;
  const grk_feature& f = args.f[blockIdx.y];
  const int chunks = dim / VEC;
  const int64_t units = num_tokens * chunks;
  const T* table = reinterpret_cast<const T*>(f.table);
  const I* idx = reinterpret_cast<const I*>(f.idx);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; base < units; base += stride * UNROLL) {
    Vec16<T> acc[UNROLL];
    int64_t nn[UNROLL];
    int cc[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      int64_t unit = base + u * stride;
      nn[u] = unit / chunks;
      cc[u] = (int)(unit - nn[u] * chunks);
      if (unit >= units) continue;
      if (f.bag == 1) {
        int64_t row = resolve_row(idx, nn[u], 0, f.idx_ld, f.idx_mode, token_type, T_len);
        if (row < 0 || row >= f.num_rows) {
          if (err_flag) *err_flag = 1;
          acc[u].v = {};
        } else {
          acc[u].load(table + row * dim + cc[u] * VEC);
        }
      } else {
        float s[VEC];
#pragma unroll
        for (int e = 0; e < VEC; ++e) s[e] = 0.f;
        for (int a = 0; a < f.bag; ++a) {
          int64_t row = resolve_row(idx, nn[u], a, f.idx_ld, f.idx_mode, token_type, T_len);
          if (row < 0 || row >= f.num_rows) {
            if (err_flag) *err_flag = 1;
            continue;
          }
          if (row == 0 && (f.flags & GRK_FEAT_SKIP_ROW0)) continue;  // a zero padding row adds nothing
          Vec16<T> r;
          r.load(table + row * dim + cc[u] * VEC);
          if (a == 0) {
#pragma unroll
            for (int e = 0; e < VEC; ++e) s[e] = r.get(e);
          } else {
#pragma unroll
            for (int e = 0; e < VEC; ++e) s[e] = s[e] + r.get(e);
          }
        }
#pragma unroll
        for (int e = 0; e < VEC; ++e) acc[u].set(e, s[e]);
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      int64_t unit = base + u * stride;
      if (unit >= units) continue;
      acc[u].store(out + nn[u] * out_ld + f.out_col + cc[u] * VEC);
    }
  }
}

// One wave per (token, feature) row when a row is 64 x 16 bytes (bf16 d=512,
// fp32 d=256): lane = 16-byte column chunk, so a unit needs no index
// arithmetic; the token's index (and bag) words are wave-uniform scalar loads,
// and kGatherRows tokens per wave keep that many rows in flight.  Same values
// as k_gather (bag sums in fp32 from slot 0, one rounding; with
// GRK_FEAT_SKIP_ROW0 the zero padding row's slots are not read -- adding +0
// changes no sum, up to the sign of an all-zero result).
constexpr int kGatherRows = 1;

template <typename T, typename I>
__global__ void __launch_bounds__(256) k_gather_wave(FeatArgs args, int64_t num_tokens,
                                                     const int32_t* __restrict__ token_type, int32_t T_len,
                                                     T* __restrict__ out, int64_t out_ld, int32_t* err_flag) {
  constexpr int VEC = Vec16<T>::N;
  constexpr int dim = 64 * VEC;
  const grk_feature& f = args.f[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t n0 = ((int64_t)blockIdx.x * 4 + wave) * kGatherRows;
  const T* table = reinterpret_cast<const T*>(f.table);
  const I* idx = reinterpret_cast<const I*>(f.idx);
  if (f.bag == 1) {
    int64_t row[kGatherRows];
#pragma unroll
    for (int r = 0; r < kGatherRows; ++r) {
      const int64_t n = n0 + r;
      row[r] = n < num_tokens ? resolve_row(idx, n, 0, f.idx_ld, f.idx_mode, token_type, T_len) : 0;
    }
    Vec16<T> v[kGatherRows];
#pragma unroll
    for (int r = 0; r < kGatherRows; ++r) {
      if (row[r] < 0 || row[r] >= f.num_rows) {
        if (n0 + r < num_tokens && err_flag) *err_flag = 1;
        v[r].v = {};
      } else {
        v[r].load(table + row[r] * dim + lane * VEC);
      }
    }
#pragma unroll
    for (int r = 0; r < kGatherRows; ++r)
      if (n0 + r < num_tokens) v[r].store(out + (n0 + r) * out_ld + f.out_col + lane * VEC);
    return;
  }
  for (int r = 0; r < kGatherRows; ++r) {
    const int64_t n = n0 + r;
    if (n >= num_tokens) return;
    float s[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) s[e] = 0.f;
    for (int a = 0; a < f.bag; ++a) {
      const int64_t row = resolve_row(idx, n, a, f.idx_ld, f.idx_mode, token_type, T_len);
      if (row < 0 || row >= f.num_rows) {
        if (err_flag) *err_flag = 1;
        continue;
      }
      if (row == 0 && (f.flags & GRK_FEAT_SKIP_ROW0)) continue;  // wave-uniform: a zero padding row
      Vec16<T> x;
      x.load(table + row * dim + lane * VEC);
      if (a == 0) {
#pragma unroll
        for (int e = 0; e < VEC; ++e) s[e] = x.get(e);
      } else {
#pragma unroll
        for (int e = 0; e < VEC; ++e) s[e] = s[e] + x.get(e);
      }
    }
    Vec16<T> acc;
#pragma unroll
    for (int e = 0; e < VEC; ++e) acc.set(e, s[e]);
    acc.store(out + n * out_ld + f.out_col + lane * VEC);
  }
}

// -------------------------------------------------------------- backward ----
// Occurrences [occ_off[0], occ_off[num]) of one launch batch: sort key =
// group row (sentinel for padding / out-of-range), payload = address of the
// occurrence's gradient row.  The radix sort is stable, so after sorting the
// payloads of one key are in occurrence order.
// Keys are built in tiles of kKeyTile occurrences per 256-thread block (4 per
// thread), the radix sort's tile: with hist0 the block also counts the first
// digit (the low bits0 bits) of its keys into hist0[digit][tile], the sort's first
// histogram (grk_sort.hip), so that pass needs no launch of its own.
// Blocks past key_blocks (first launch of a call only) instead zero the dense
// output (16-byte words, grid-stride) and the unique-row count: the fill then
// overlaps the key build instead of taking a launch of its own.
constexpr int kKeyTile = 1024;
struct KeyFill {
  uint4* zero_dst;
  int64_t zero_vecs;
  int32_t* zero_count;
};
template <typename I>
__global__ void __launch_bounds__(256) k_build_keys(LookupArgs la, int esize, const int32_t* __restrict__ token_type,
                                                    int32_t T_len, int64_t num_rows, int64_t padding_idx,
                                                    unsigned* __restrict__ keys, unsigned long long* __restrict__ gptr,
                                                    int32_t* err_flag, unsigned key_blocks,
                                                    unsigned* __restrict__ hist0, int ntiles, int bits0,
                                                    KeyFill fill) {
  if (blockIdx.x >= key_blocks) {
    const int64_t nb = gridDim.x - key_blocks, t = (int64_t)(blockIdx.x - key_blocks) * blockDim.x + threadIdx.x;
    const int64_t stride = nb * blockDim.x;
    for (int64_t v = t; v < fill.zero_vecs; v += stride) fill.zero_dst[v] = make_uint4(0, 0, 0, 0);
    if (fill.zero_count && t == 0) *fill.zero_count = 0;
    return;
  }
  __shared__ unsigned cnt[2048];
  const int nb0 = 1 << bits0;
  if (hist0) {
    for (int d = threadIdx.x; d < nb0; d += blockDim.x) cnt[d] = 0;
    __syncthreads();
  }
  const int64_t end = la.occ_off[la.num];
#pragma unroll
  for (int rd = 0; rd < kKeyTile / 256; ++rd) {
    const int64_t o = la.occ_off[0] + (int64_t)blockIdx.x * kKeyTile + rd * 256 + threadIdx.x;
    if (o >= end) break;
    int l = 0;
    while (l + 1 < la.num && o >= la.occ_off[l + 1]) ++l;
    const grk_lookup& L = la.l[l];
    const int64_t rel = o - la.occ_off[l];
    const int64_t n = rel / L.bag;
    const int a = (int)(rel - n * L.bag);
    const int64_t row = resolve_row(reinterpret_cast<const I*>(L.idx), n, a, L.idx_ld, L.idx_mode, token_type, T_len);
    unsigned key = (unsigned)num_rows;  // sentinel: sorts after every real row
    if (row < 0 || row >= L.table_rows || L.row_offset + row >= num_rows) {
      if (err_flag) *err_flag = 1;
    } else if (row != padding_idx) {
      key = (unsigned)(L.row_offset + row);
    }
    keys[o] = key;
    gptr[o] = (unsigned long long)((const char*)L.grad + (n * L.grad_ld + L.grad_col) * esize);
    if (hist0) atomicAdd(&cnt[key & (unsigned)(nb0 - 1)], 1u);
  }
  if (hist0) {
    __syncthreads();
    for (int d = threadIdx.x; d < nb0; d += blockDim.x) hist0[(int64_t)d * ntiles + blockIdx.x] = cnt[d];
  }
}

__global__ void k_segments(const unsigned* __restrict__ keys, const int* __restrict__ pos, int64_t n,
                           unsigned sentinel, int* __restrict__ seg_start, int* __restrict__ seg_end,
                           unsigned* __restrict__ seg_key, int64_t* __restrict__ uniq_ids,
                           int32_t* __restrict__ count) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned k = keys[i];
  if (k == sentinel) return;
  int u = pos[i] - 1;
  if (i == 0 || keys[i - 1] != k) {
    seg_start[u] = (int)i;
    seg_key[u] = k;
    if (uniq_ids) uniq_ids[u] = (int64_t)k;
  }
  bool last_of_seg = (i == n - 1) || keys[i + 1] != k;
  if (last_of_seg) {
    seg_end[u] = (int)(i + 1);
    if (i == n - 1 || keys[i + 1] == sentinel) *count = u + 1;
  }
}

// Chunked dense mode with num_rows <= n: segment bounds indexed by the ROW
// (seg_start[key], seg_end[key]) -- no segment numbering (head positions: three
// launches) is needed when nothing is written per unique row.  The distinct-row
// count is added once per wave (one add per head contended on a single word:
// 29 us per call on MI355X, round 4).
// Grid-stride (kSegKeyBlocks workgroups at most): the distinct-row count is summed
// per workgroup and added once per workgroup -- one atomic per wave on the single
// counter serialised (~14k waves at C2: 29-46 us per call).
constexpr int kSegKeyBlocks = 512;
__global__ void __launch_bounds__(256) k_segments_key(const unsigned* __restrict__ keys, int64_t n, unsigned sentinel,
                                                      int* __restrict__ seg_start, int* __restrict__ seg_end,
                                                      int32_t* __restrict__ count) {
  __shared__ int wsum[4];
  int heads = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const unsigned k = keys[i];
    if (k == sentinel) continue;
    const bool head = i == 0 || keys[i - 1] != k;
    if (head) {
      seg_start[k] = (int)i;
      ++heads;
    }
    if (i == n - 1 || keys[i + 1] != k) seg_end[k] = (int)(i + 1);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) heads += __shfl_xor(heads, off);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = heads;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    if (t) atomicAdd(count, t);
  }
}

// ------------------------------------------------- segmented reduction ----
// The sorted occurrence list is cut into fixed chunks of kRedChunk entries,
// one row group (dim/VEC lanes, VEC = one 16-byte vector of grads) per chunk,
// so the work per row group is bounded whatever the row lengths.  Every row is
// summed strictly in occurrence order (bit-exact with the reference's CPU
// embedding_dense_backward):
//   * a row whose occurrences all fall in one chunk is summed by that chunk
//     and written directly;
//   * a row crossing a chunk edge with <= 2*kRedChunk occurrences is re-summed
//     sequentially by k_seg_combine / k_seg_combine_edges;
//   * a longer ("hot") row is summed by k_seg_hot, one wave per 64 columns.
constexpr int kRedChunk = 256;
constexpr int kRedPipe = 8;  // occurrence rows loaded ahead of the in-order adds

template <typename G>
struct RowVec {
  static constexpr int VEC = 16 / sizeof(G);
  float v[VEC];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int e = 0; e < VEC; ++e) v[e] = 0.f;
  }
};

template <typename G>
__device__ __forceinline__ void load_row(Vec16<G>& r, unsigned long long ptr, int c) {
  r.load(reinterpret_cast<const G*>(ptr) + c);
}

template <typename A>
__device__ __forceinline__ void store_final(const A& acc, unsigned key, int64_t u, int dim, int c,
                                            float* dense_out, float* uniq_rows, int32_t* row_slot) {
  constexpr int VEC = A::VEC;
#pragma unroll
  for (int e = 0; e < VEC; e += 4) {
    float4 r = make_float4(acc.v[e], acc.v[e + 1], acc.v[e + 2], acc.v[e + 3]);
    if (dense_out) *reinterpret_cast<float4*>(dense_out + (int64_t)key * dim + c + e) = r;
    if (uniq_rows) *reinterpret_cast<float4*>(uniq_rows + u * dim + c + e) = r;
  }
  if (row_slot && c == 0) row_slot[key] = (int32_t)u;
}

// GRK_BWD_DENSE_BF16: the dense row rounded to bf16 once (the intermediate
// tables' own dtype: no fp32 buffer and no cast kernel after the call).
template <typename A>
__device__ __forceinline__ void store_final(const A& acc, unsigned key, int64_t u, int dim, int c,
                                            bf16_t* dense_out, float* uniq_rows, int32_t* row_slot) {
  constexpr int VEC = A::VEC;
#pragma unroll
  for (int e = 0; e < VEC; e += 4) {
    if (dense_out) {
      uint2 t;
      t.x = (unsigned)f32_to_bf16(acc.v[e]) | ((unsigned)f32_to_bf16(acc.v[e + 1]) << 16);
      t.y = (unsigned)f32_to_bf16(acc.v[e + 2]) | ((unsigned)f32_to_bf16(acc.v[e + 3]) << 16);
      *reinterpret_cast<uint2*>(dense_out + (int64_t)key * dim + c + e) = t;
    }
    if (uniq_rows)
      *reinterpret_cast<float4*>(uniq_rows + u * dim + c + e) =
          make_float4(acc.v[e], acc.v[e + 1], acc.v[e + 2], acc.v[e + 3]);
  }
  if (row_slot && c == 0) row_slot[key] = (int32_t)u;
}

// Sequential in-order sum of the sorted occurrences [s, e) with kRedPipe rows in flight.
template <typename G>
__device__ __forceinline__ void seq_sum(RowVec<G>& acc, const unsigned long long* __restrict__ gptr, int s, int e,
                                        int c) {
  constexpr int VEC = RowVec<G>::VEC;
  for (int p = s; p < e; p += kRedPipe) {
    Vec16<G> r[kRedPipe];
#pragma unroll
    for (int j = 0; j < kRedPipe; ++j)
      if (p + j < e) load_row<G>(r[j], gptr[p + j], c);
#pragma unroll
    for (int j = 0; j < kRedPipe; ++j)
      if (p + j < e)
#pragma unroll
        for (int x = 0; x < VEC; ++x) acc.v[x] += r[j].get(x);
  }
}

template <typename G>
__global__ void __launch_bounds__(256) k_seg_chunks(const unsigned* __restrict__ keys,
                                                    const unsigned long long* __restrict__ gptr,
                                                    const int* __restrict__ pos, const int* __restrict__ seg_start,
                                                    const int* __restrict__ seg_end, int64_t n, unsigned sentinel,
                                                    int dim, float* __restrict__ dense_out,
                                                    float* __restrict__ uniq_rows, int32_t* __restrict__ row_slot) {
  constexpr int VEC = RowVec<G>::VEC;
  const int tpr = dim / VEC;
  const int groups = blockDim.x / tpr;
  const int64_t chunk = (int64_t)blockIdx.x * groups + threadIdx.x / tpr;
  const int c = (threadIdx.x % tpr) * VEC;
  const int64_t p0 = chunk * kRedChunk;
  if ((int)(threadIdx.x / tpr) >= groups || p0 >= n) return;
  const int64_t p1 = min(n, p0 + kRedChunk);
  RowVec<G> acc;
  acc.zero();
  int64_t ps = p0;                 // start of the current piece
  unsigned cur = keys[p0];
  if (cur == sentinel) return;
  auto flush = [&](int64_t pe) {   // piece [ps, pe) of key cur
    const int u = pos[ps] - 1;
    const int su = seg_start[u], eu = seg_end[u];
    if (su >= p0 && eu <= p1) store_final(acc, cur, u, dim, c, dense_out, uniq_rows, row_slot);
    // else: a row crossing an edge -- k_seg_combine (<= 2*kRedChunk) or k_seg_hot sums it
  };
  for (int64_t p = p0; p < p1; p += kRedPipe) {
    Vec16<G> r[kRedPipe];
    unsigned k[kRedPipe];
#pragma unroll
    for (int j = 0; j < kRedPipe; ++j) {
      k[j] = p + j < p1 ? keys[p + j] : sentinel;
      if (k[j] != sentinel) load_row<G>(r[j], gptr[p + j], c);
    }
#pragma unroll
    for (int j = 0; j < kRedPipe; ++j) {
      if (k[j] == sentinel) continue;
      if (k[j] != cur) {
        flush(p + j);
        acc.zero();
        cur = k[j];
        ps = p + j;
      }
#pragma unroll
      for (int x = 0; x < VEC; ++x) acc.v[x] += r[j].get(x);
    }
    if (k[kRedPipe - 1] == sentinel && p + kRedPipe <= p1) {  // reached the padding tail
      flush(p + kRedPipe);
      return;
    }
  }
  flush(p1);
}

template <typename G>
__global__ void __launch_bounds__(256) k_seg_combine(const unsigned long long* __restrict__ gptr,
                                                     const int* __restrict__ seg_start,
                                                     const int* __restrict__ seg_end,
                                                     const unsigned* __restrict__ seg_key,
                                                     const int32_t* __restrict__ count, int64_t max_rows, int dim,
                                                     float* __restrict__ dense_out, float* __restrict__ uniq_rows,
                                                     int32_t* __restrict__ row_slot) {
  constexpr int VEC = RowVec<G>::VEC;
  const int tpr = dim / VEC;
  const int groups = blockDim.x / tpr;
  const int64_t u = (int64_t)blockIdx.x * groups + threadIdx.x / tpr;
  const int c = (threadIdx.x % tpr) * VEC;
  if ((int)(threadIdx.x / tpr) >= groups || u >= max_rows || u >= *count) return;
  const int su = seg_start[u], eu = seg_end[u];
  if (su / kRedChunk == (eu - 1) / kRedChunk) return;  // written by k_seg_chunks
  if (eu - su > 2 * kRedChunk) return;                  // hot row: k_seg_hot
  RowVec<G> acc;
  acc.zero();
  seq_sum<G>(acc, gptr, su, eu, c);
  store_final(acc, seg_key[u], u, dim, c, dense_out, uniq_rows, row_slot);
}

// ------------------------------------ segmented reduction, one wave per row ----
// dim == 64 * VEC (bf16 d=512, fp32 d=256: one 16-byte vector per lane covers
// a row).  Same chunking and summation order as k_seg_chunks /
// k_seg_combine, restructured for memory-level parallelism: the chunk's keys,
// scan positions and gradient-row addresses are loaded into lanes up front and
// broadcast with readlane, so row loads take scalar base addresses with
// kWavePipe rows in flight instead of a key -> address -> row chain per
// step; whether a piece is a whole segment follows from the neighbouring keys
// (keys[p0-1], keys[p1]), so seg_start / seg_end are read only for the (at
// most two) pieces that cross the chunk's edges.
// (GRK_WAVE_PIPE: a build constant for A/B builds, scripts/build_variant.sh)
#ifndef GRK_WAVE_PIPE
#define GRK_WAVE_PIPE 16
#endif
constexpr int kWavePipe = GRK_WAVE_PIPE;
static_assert(kWavePipe == 8 || kWavePipe == 16 || kWavePipe == 32, "GRK_WAVE_PIPE: 8, 16 or 32");

// (readlane returns int: both halves go through unsigned, or the low word
// would sign-extend into the high one)
__device__ __forceinline__ unsigned long long readlane64(unsigned lo, unsigned hi, int l) {
  return ((unsigned long long)(unsigned)__builtin_amdgcn_readlane(hi, l) << 32) |
         (unsigned long long)(unsigned)__builtin_amdgcn_readlane(lo, l);
}

// 16-byte row-vector load through a global-address-space pointer (a flat
// load would also count against lgkmcnt and serialise with scalar loads).
template <typename G>
__device__ __forceinline__ void load_row_global(Vec16<G>& r, unsigned long long ptr, int c) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(1))) const u32x4 gu32x4;
  const u32x4 t = *reinterpret_cast<gu32x4*>(ptr + (unsigned long long)c * sizeof(G));
  if constexpr (sizeof(G) == 2) r.v = make_uint4(t.x, t.y, t.z, t.w);
  else r.v = make_float4(__uint_as_float(t.x), __uint_as_float(t.y), __uint_as_float(t.z), __uint_as_float(t.w));
}

// One lane's LW consecutive gradient elements of a row in the one-wave-per-row
// kernels (64 * LW = dim): one 16-byte vector (bf16 x 8, fp32 x 4) or two (fp32 x 8).
template <typename G, int LW>
struct WaveVec {
  static constexpr int PER = 16 / sizeof(G);
  static constexpr int NV = LW / PER;
  Vec16<G> r[NV];
  __device__ __forceinline__ void load(unsigned long long ptr, int c) {
#pragma unroll
    for (int i = 0; i < NV; ++i) load_row_global<G>(r[i], ptr, c + i * PER);
  }
  __device__ __forceinline__ float get(int x) const { return r[x / PER].get(x % PER); }
};
template <int LW>
struct WaveAcc {
  static constexpr int VEC = LW;
  float v[LW];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int e = 0; e < LW; ++e) v[e] = 0.f;
  }
};

template <typename G, int LW, int CH = kRedChunk, typename OT = float>
__device__ __forceinline__ void seg_chunks_wave_body(int64_t chunk, int lane, const unsigned* __restrict__ keys,
                                                     const unsigned long long* __restrict__ gptr,
                                                     const int* __restrict__ pos, const int* __restrict__ seg_start,
                                                     const int* __restrict__ seg_end, int64_t n, unsigned sentinel,
                                                     int dim, OT* __restrict__ dense_out,
                                                     float* __restrict__ uniq_rows, int32_t* __restrict__ row_slot,
                                                     float* __restrict__ partials = nullptr) {
  constexpr int VEC = LW;
  constexpr int KP = CH / 64;  // chunk entries per lane
  const int64_t p0 = chunk * CH;
  if (p0 >= n) return;
  const int64_t p1 = min(n, p0 + CH);
  const int c = lane * VEC;
  unsigned kr[KP], glo[KP], ghi[KP];
  int pr[KP];
  const unsigned long long g0 = gptr[p0];  // stands in past p1: every row load stays valid and unconditional
#pragma unroll
  for (int k = 0; k < KP; ++k) {
    const int64_t i = p0 + k * 64 + lane;
    kr[k] = i < p1 ? keys[i] : sentinel;
    pr[k] = i < p1 && pos ? pos[i] : 0;   // null pos: key-indexed segments, nothing stored per unique row
    const unsigned long long g = i < p1 ? gptr[i] : g0;
    glo[k] = (unsigned)g;
    ghi[k] = (unsigned)(g >> 32);
  }
  unsigned cur = __builtin_amdgcn_readfirstlane(kr[0]);
  if (cur == sentinel) return;
  const unsigned kprev = p0 > 0 ? keys[p0 - 1] : sentinel;
  const unsigned knext = p1 < n ? keys[p1] : sentinel;
  WaveAcc<LW> acc;
  acc.zero();
  int64_t ps = p0, pe = p0;          // current piece [ps, pe) of key cur
  int u = __builtin_amdgcn_readfirstlane(pr[0]) - 1;
  auto flush = [&]() {
    const bool whole = (ps > p0 || kprev != cur) && (pe < p1 || knext != cur);
    if (whole) {
      store_final(acc, cur, u, dim, c, dense_out, uniq_rows, row_slot);
    } else if (partials) {  // chunked mode: the piece's sum goes to the chunk's head (0) or tail (1) slot
      const int slot = (ps == p0 && kprev == cur) ? 0 : 1;
      float* dst = partials + (chunk * 2 + slot) * dim + c;
#pragma unroll
      for (int e = 0; e < LW; e += 4)
        *reinterpret_cast<float4*>(dst + e) = make_float4(acc.v[e], acc.v[e + 1], acc.v[e + 2], acc.v[e + 3]);
    }
    // else: a row crossing an edge -- k_seg_combine_edges (<= 2*CH) or k_seg_hot sums it
  };
  bool done = false;
#pragma unroll
  for (int k = 0; k < KP; ++k) {
    for (int s0 = 0; s0 < 64 && !done; s0 += kWavePipe) {
      WaveVec<G, LW> r[kWavePipe];
      unsigned kk[kWavePipe];
#pragma unroll
      for (int j = 0; j < kWavePipe; ++j) {
        kk[j] = (unsigned)__builtin_amdgcn_readlane(kr[k], s0 + j);
        r[j].load(readlane64(glo[k], ghi[k], s0 + j), c);
      }
#pragma unroll
      for (int j = 0; j < kWavePipe; ++j) {
        if (done) break;
        if (kk[j] == sentinel) {  // sorted: the rest of the chunk is padding / past the end
          done = true;
          break;
        }
        if (kk[j] != cur) {
          flush();
          acc.zero();
          cur = kk[j];
          ps = p0 + k * 64 + s0 + j;
          u = __builtin_amdgcn_readlane(pr[k], s0 + j) - 1;  // int: scan positions fit
        }
#pragma unroll
        for (int x = 0; x < VEC; ++x) acc.v[x] += r[j].get(x);
        pe = p0 + k * 64 + s0 + j + 1;
      }
    }
  }
  flush();
}

// seq_sum for one wave: the row addresses of 64 occurrences at a time are
// loaded into lanes and broadcast, kWavePipe rows in flight, in-order adds.
template <typename G, int LW>
__device__ __forceinline__ void seq_sum_wave(WaveAcc<LW>& acc, const unsigned long long* __restrict__ gptr, int s,
                                             int e, int lane, int c) {
  constexpr int VEC = LW;
  for (int b = s; b < e; b += 64) {
    const unsigned long long g = gptr[b + lane < e ? b + lane : s];
    const unsigned lo = (unsigned)g, hi = (unsigned)(g >> 32);
    const int m = min(64, e - b);
    for (int s0 = 0; s0 < m; s0 += kWavePipe) {
      WaveVec<G, LW> r[kWavePipe];
#pragma unroll
      for (int j = 0; j < kWavePipe; ++j) r[j].load(readlane64(lo, hi, s0 + j), c);
#pragma unroll
      for (int j = 0; j < kWavePipe; ++j)
        if (s0 + j < m)
#pragma unroll
          for (int x = 0; x < VEC; ++x) acc.v[x] += r[j].get(x);
    }
  }
}

template <typename G, int LW, int CH>
__global__ void __launch_bounds__(256) k_seg_chunks_wave(const unsigned* __restrict__ keys,
                                                         const unsigned long long* __restrict__ gptr,
                                                         const int* __restrict__ pos, const int* __restrict__ seg_start,
                                                         const int* __restrict__ seg_end, int64_t n, unsigned sentinel,
                                                         int dim, float* __restrict__ dense_out,
                                                         float* __restrict__ uniq_rows,
                                                         int32_t* __restrict__ row_slot) {
  seg_chunks_wave_body<G, LW, CH>((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), threadIdx.x & 63, keys, gptr, pos,
                              seg_start, seg_end, n, sentinel, dim, dense_out, uniq_rows, row_slot);
}

// One wave per chunk edge b (occurrence b * kRedChunk): finishes the row that
// first crosses a chunk edge at b, i.e. crosses b and starts in chunk b - 1,
// when it has at most 2 * kRedChunk occurrences (longer rows: k_seg_hot).
template <typename G, int LW, int CH = kRedChunk>
__device__ __forceinline__ void seg_edge_body(int64_t edge, int lane, const unsigned* __restrict__ keys,
                                              const unsigned long long* __restrict__ gptr,
                                              const int* __restrict__ pos, const int* __restrict__ seg_start,
                                              const int* __restrict__ seg_end, int64_t n, unsigned sentinel, int dim,
                                              float* __restrict__ dense_out, float* __restrict__ uniq_rows,
                                              int32_t* __restrict__ row_slot) {
  const int64_t b = edge + 1;
  const int64_t pb = b * CH;
  if (pb >= n) return;
  const unsigned key = keys[pb];
  if (key == sentinel || keys[pb - 1] != key) return;
  const int u = pos[pb] - 1;
  const int su = seg_start[u], eu = seg_end[u];
  if (su / CH != b - 1) return;  // also crosses an earlier edge: finished there
  if (eu - su > 2 * CH) return;  // hot row: k_seg_hot
  const int c = lane * LW;
  WaveAcc<LW> acc;
  acc.zero();
  seq_sum_wave<G, LW>(acc, gptr, su, eu, lane, c);
  store_final(acc, key, u, dim, c, dense_out, uniq_rows, row_slot);
}

template <typename G, int LW, int CH>
__global__ void __launch_bounds__(256) k_seg_combine_edges(const unsigned* __restrict__ keys,
                                                           const unsigned long long* __restrict__ gptr,
                                                           const int* __restrict__ pos,
                                                           const int* __restrict__ seg_start,
                                                           const int* __restrict__ seg_end, int64_t n,
                                                           unsigned sentinel, int dim, float* __restrict__ dense_out,
                                                           float* __restrict__ uniq_rows,
                                                           int32_t* __restrict__ row_slot) {
  seg_edge_body<G, LW, CH>((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), threadIdx.x & 63, keys, gptr, pos, seg_start,
                       seg_end, n, sentinel, dim, dense_out, uniq_rows, row_slot);
}

// ------------------------------------------- chunked (fixed-order) mode ----
// GRK_BWD_CHUNKED: for tables whose rows are an intermediate with no reference
// counterpart (the projected feature rows P = E W of the fused trainer: the
// reference's gradient is dE = sum dY W, accumulated in a different order
// anyway), rows crossing chunk edges are not re-summed in occurrence order:
// every chunk stores the sums of its edge-crossing pieces (head piece: the
// row continuing from the previous chunk -> slot 0, tail piece: the row
// continuing into the next -> slot 1), and one wave per such row adds its
// pieces in chunk order.  Deterministic (fixed order), and a hot row of k
// occurrences costs k / kRedChunk dependent adds instead of k.
//
// The chunk length is a build constant (GRK_CHUNKED_CH, 256 by default; 64 /
// 128 for A/B builds: more waves in flight on a call of ~0.5M occurrences, more
// pieces per hot row); grk_embedding_chunked_size() reports it, so callers
// that restate the order (oracle/embedding.chunked_backward) take it from there.
#ifndef GRK_CHUNKED_CH
#define GRK_CHUNKED_CH 256
#endif
constexpr int kPartialChunk = GRK_CHUNKED_CH;
static_assert(kPartialChunk == 64 || kPartialChunk == 128 || kPartialChunk == 256, "GRK_CHUNKED_CH: 64, 128 or 256");

template <typename G, int LW, int CH, typename OT = float>
__global__ void __launch_bounds__(256) k_seg_chunks_partial(const unsigned* __restrict__ keys,
                                                            const unsigned long long* __restrict__ gptr,
                                                            const int* __restrict__ pos,
                                                            const int* __restrict__ seg_start,
                                                            const int* __restrict__ seg_end, int64_t n,
                                                            unsigned sentinel, int dim, OT* __restrict__ dense_out,
                                                            float* __restrict__ uniq_rows,
                                                            int32_t* __restrict__ row_slot,
                                                            float* __restrict__ partials) {
  seg_chunks_wave_body<G, LW, CH, OT>((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), threadIdx.x & 63, keys, gptr,
                                      pos, seg_start, seg_end, n, sentinel, dim, dense_out, uniq_rows, row_slot,
                                      partials);
}

// One wave per chunk edge b: the row first crossing b (it starts in chunk
// b - 1, whose tail slot holds its first piece) = tail(b - 1) + head(b) + ...
// + head(last chunk of the row), added in that order.
template <int LW, int CH, typename OT = float>
__global__ void __launch_bounds__(256) k_seg_partials_combine(const unsigned* __restrict__ keys,
                                                              const int* __restrict__ pos,
                                                              const int* __restrict__ seg_start,
                                                              const int* __restrict__ seg_end, int64_t n,
                                                              unsigned sentinel, int dim,
                                                              const float* __restrict__ partials,
                                                              OT* __restrict__ dense_out,
                                                              float* __restrict__ uniq_rows,
                                                              int32_t* __restrict__ row_slot) {
  constexpr int PIPE = 8;
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6) + 1;
  const int64_t pb = b * CH;
  if (pb >= n) return;
  const unsigned key = keys[pb];
  if (key == sentinel || keys[pb - 1] != key) return;
  const int u = pos ? pos[pb] - 1 : 0;
  const int seg = pos ? u : (int)key;   // null pos: segment bounds indexed by row
  const int su = seg_start[seg], eu = seg_end[seg];
  if (su / CH != b - 1) return;  // crosses an earlier edge: combined there
  const int64_t last = (eu - 1) / CH;
  const int c = lane * LW;
  WaveAcc<LW> acc;
  const float* t = partials + ((b - 1) * 2 + 1) * dim + c;
#pragma unroll
  for (int e = 0; e < LW; ++e) acc.v[e] = t[e];
  for (int64_t k0 = b; k0 <= last; k0 += PIPE) {
    float4 r[PIPE][LW / 4];
#pragma unroll
    for (int j = 0; j < PIPE; ++j)
      if (k0 + j <= last)
#pragma unroll
        for (int e = 0; e < LW / 4; ++e)
          r[j][e] = *reinterpret_cast<const float4*>(partials + (k0 + j) * 2 * dim + c + 4 * e);
#pragma unroll
    for (int j = 0; j < PIPE; ++j)
      if (k0 + j <= last)
#pragma unroll
        for (int e = 0; e < LW / 4; ++e) {
          acc.v[4 * e] += r[j][e].x;
          acc.v[4 * e + 1] += r[j][e].y;
          acc.v[4 * e + 2] += r[j][e].z;
          acc.v[4 * e + 3] += r[j][e].w;
        }
  }
  store_final(acc, key, u, dim, c, dense_out, uniq_rows, row_slot);
}

// ------------------------------------ chunked mode, column-sliced by XCD ----
// The projected feature rows' backward (dim 512, bf16 gradient rows, dense
// output only: ~860k occurrences over ~41k distinct gradient rows per call at
// C2).  k_seg_chunks_partial reads each occurrence's whole 1 KiB row: every XCD
// sees random rows of the whole ~41 MB gradient, its 4 MiB L2 misses nearly all
// of them, and PMC counted ~8x the algorithmic bytes.  Here workgroup w runs on
// XCD w % 8 and handles only column slice x = w % 8 (64 columns = one 128-byte
// line per row), so an XCD's working set is 1/8 of the gradient (~5 MB).  A wave
// takes 8 consecutive chunks, one per 8-lane group (8 bf16 columns per lane);
// each group walks its chunk exactly as k_seg_chunks_partial's wave does (same
// pieces, same head / tail partial slots, same in-order fp32 adds per column),
// so the output is bitwise the same.  A batch of 64 occurrences' keys and row
// addresses per group goes through LDS (a wave's own region: no barrier).
#ifndef GRK_COLS_PIPE
#define GRK_COLS_PIPE 16   // rows in flight per lane (A/B builds: 8)
#endif
template <int CH, typename OT>
__global__ void __launch_bounds__(256) k_seg_chunks_cols(const unsigned* __restrict__ keys,
                                                         const unsigned long long* __restrict__ gptr, int64_t n,
                                                         unsigned sentinel, OT* __restrict__ dense_out,
                                                         float* __restrict__ partials) {
  constexpr int dim = 512, PIPE = GRK_COLS_PIPE;
  __shared__ unsigned skey[4][8][64];              // [wave][group][batch entry]
  __shared__ unsigned long long sptr[4][8][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, gi = lane >> 3, sub = lane & 7;
  const int x = blockIdx.x & 7;
  const int64_t chunk = ((int64_t)(blockIdx.x >> 3) * 4 + wave) * 8 + gi;
  const int c = x * 64 + sub * 8;
  const int64_t p0 = chunk * CH;
  const bool live = p0 < n;
  const int64_t p1 = live ? min(n, p0 + CH) : p0;
  unsigned cur = live ? keys[p0] : sentinel;
  bool done = cur == sentinel;
  if (__ballot(!done) == 0) return;
  const unsigned kprev = live && p0 > 0 ? keys[p0 - 1] : sentinel;
  const unsigned knext = live && p1 < n ? keys[p1] : sentinel;
  const unsigned long long g0 = live ? gptr[p0] : gptr[0];   // stands in past p1
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  int ps = 0, pe = 0;   // the current piece [p0 + ps, p0 + pe)
  const int len = (int)(p1 - p0);
  auto flush = [&]() {
    const bool whole = (ps > 0 || kprev != cur) && (pe < len || knext != cur);
    if (whole) {
      OT* d = dense_out + (int64_t)cur * dim + c;
      if constexpr (sizeof(OT) == 2) {
        uint4 t;
        t.x = (unsigned)f32_to_bf16(acc[0]) | ((unsigned)f32_to_bf16(acc[1]) << 16);
        t.y = (unsigned)f32_to_bf16(acc[2]) | ((unsigned)f32_to_bf16(acc[3]) << 16);
        t.z = (unsigned)f32_to_bf16(acc[4]) | ((unsigned)f32_to_bf16(acc[5]) << 16);
        t.w = (unsigned)f32_to_bf16(acc[6]) | ((unsigned)f32_to_bf16(acc[7]) << 16);
        *reinterpret_cast<uint4*>(d) = t;
      } else {
        *reinterpret_cast<float4*>(d) = make_float4(acc[0], acc[1], acc[2], acc[3]);
        *reinterpret_cast<float4*>(d + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
      }
    } else {   // the piece's sum goes to the chunk's head (0) or tail (1) slot
      const int slot = (ps == 0 && kprev == cur) ? 0 : 1;
      float* dst = partials + (chunk * 2 + slot) * dim + c;
      *reinterpret_cast<float4*>(dst) = make_float4(acc[0], acc[1], acc[2], acc[3]);
      *reinterpret_cast<float4*>(dst + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
    }
  };
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(1))) const u32x4 gu32x4;
  unsigned* mk = skey[wave][gi];
  unsigned long long* mp = sptr[wave][gi];
#pragma unroll 1
  for (int b = 0; b < CH; b += 64) {
    // the group's batch: entries b .. b + 63 of its chunk, 8 per lane
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int64_t i = p0 + b + 8 * k + sub;
      mk[8 * k + sub] = i < p1 ? keys[i] : sentinel;
      mp[8 * k + sub] = i < p1 ? gptr[i] : g0;
    }
    __builtin_amdgcn_wave_barrier();   // LDS accesses of one wave run in order: no barrier beyond this fence
#pragma unroll 1
    for (int j0 = 0; j0 < 64; j0 += PIPE) {
      u32x4 r[PIPE];
      unsigned kk[PIPE];
#pragma unroll
      for (int j = 0; j < PIPE; ++j) {
        kk[j] = mk[j0 + j];
        r[j] = *reinterpret_cast<gu32x4*>(mp[j0 + j] + (unsigned long long)c * 2);
      }
#pragma unroll
      for (int j = 0; j < PIPE; ++j) {
        const unsigned kj = kk[j];
        done = done || kj == sentinel;   // sorted: the rest of the chunk is padding / past the end
        if (!done) {
          const int at = b + j0 + j;
          if (kj != cur) {
            flush();
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[e] = 0.f;
            cur = kj;
            ps = at;
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            acc[2 * e] += __uint_as_float(r[j][e] << 16);
            acc[2 * e + 1] += __uint_as_float(r[j][e] & 0xFFFF0000u);
          }
          pe = at + 1;
        }
      }
      if (__ballot(!done) == 0) break;
    }
    if (__ballot(!done) == 0) break;
    __builtin_amdgcn_wave_barrier();
  }
  if (live && pe > ps) flush();
}

// ------------------------------------------------------------- hot rows ----
// Rows with more than 2 * kRedChunk occurrences (the rows of cardinality-10
// feature tables take thousands per call), summed bit-exactly in occurrence
// order like every other row: the reference's CPU embedding_dense_backward is
// a sequential fp32 add per row in occurrence order, so the
// only parallelism inside one row is across its columns.  One wave per
// (row, column slice: 32 bf16 / 64 fp32 columns); each lane owns one column and
// keeps its running sum in a register.  A wave is latency-bound (its adds are
// one dependent chain), so narrow slices put more waves and more loads in
// flight on each hot row.
//   * loads: 16-byte vectors, 16 (bf16) / 4 (fp32) occurrences per wave
//     instruction, 4 / 8 instructions per tile of 64 / 32 occurrences, 32
//     load instructions (8 / 4 tiles) in flight.  A tile's row addresses are
//     loaded right after the data loads of the tile that many tiles earlier,
//     in the same order in the prologue as in the loop, so every wait on them
//     is a partial vmcnt;
//   * bf16: the tile is written to LDS as loaded ([occurrence][32 columns],
//     64-B rows, 16-byte writes) and read back with the gfx950 transposing
//     read ds_read_b64_tr_b16, which hands each lane its column for 4
//     consecutive occurrences (the four 64-B rows a 16-lane group reads fall on
//     disjoint banks; lanes 32-63 repeat lanes 0-31's reads);
//     fp32: written transposed ([column][occurrence], rows padded to 136 B)
//     and read 8 bytes at a time.
template <typename G>
__host__ __device__ constexpr int kHotSlice() { return sizeof(G) == 2 ? 32 : 64; }

template <typename G>
__host__ __device__ constexpr int kHotImgBytes() {
  return sizeof(G) == 2 ? 64 * (kHotSlice<G>() * 2) : kHotSlice<G>() * (32 * 4 + 8);
}

// bx = chunk edge - 1 (the wave's former blockIdx.x), by = column slice
template <typename G, int CH = kRedChunk>
__device__ __forceinline__ void seg_hot_body(int64_t bx, int by, int lane, unsigned char* __restrict__ img,
                                             const unsigned* __restrict__ keys,
                                             const unsigned long long* __restrict__ gptr,
                                             const int* __restrict__ pos, const int* __restrict__ seg_start,
                                             const int* __restrict__ seg_end, int64_t n, unsigned sentinel, int dim,
                                             float* __restrict__ dense_out, float* __restrict__ uniq_rows,
                                             int32_t* __restrict__ row_slot) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(1))) const u32x4 gu32x4;
  constexpr int ES = sizeof(G);
  constexpr int SLICE = kHotSlice<G>();
  constexpr int EPV = 16 / ES;       // elements per 16-byte vector
  constexpr int LPO = SLICE / EPV;   // lanes per occurrence slice (4 bf16, 16 fp32)
  constexpr int OPI = 64 / LPO;      // occurrences per load instruction (16, 4)
  constexpr int TILE = ES == 2 ? 64 : 32;  // occurrences per tile: 128 B of one column
  constexpr int IPT = TILE / OPI;    // load instructions per tile (4, 8)
  constexpr int ROWB = ES == 2 ? SLICE * 2 : TILE * ES + 8;  // bf16: [occ][cols] rows; fp32: [col][occs] rows
  constexpr int IMG_ROWS = ES == 2 ? TILE : SLICE;
  constexpr int EPR = 8 / ES;        // elements per 8-byte LDS read
  constexpr int S = 32 / IPT;        // tiles in flight
  static_assert(IMG_ROWS * ROWB == kHotImgBytes<G>(), "hot-row image size");
  const int64_t b = bx + 1;  // chunk edge: the row that first crosses it
  const int64_t pb = b * CH;
  if (pb >= n) return;
  const unsigned key = keys[pb];
  if (key == sentinel || keys[pb - 1] != key) return;
  const int u = pos[pb] - 1;
  const int su = seg_start[u], eu = seg_end[u];
  if (su / CH != b - 1 || eu - su <= 2 * CH) return;
  const int c0 = by * SLICE;
  const int cols = min(SLICE, dim - c0);
  const int wv = (lane % LPO) * EPV;                     // this lane's columns [wv, wv + EPV) of the slice
  const int vcol = c0 + wv < dim ? c0 + wv : c0;         // clamped into the row past dim
  const int wocc = lane / LPO;
  const int ntiles = (eu - su + TILE - 1) / TILE;
  auto addr = [&](int t) -> unsigned long long {  // lane j < TILE: address of occurrence j of tile t
    const int i = su + t * TILE + (lane < TILE ? lane : 0);
    return gptr[i < eu ? i : eu - 1];
  };
  auto issue = [&](u32x4 (&d)[IPT], unsigned long long a) {
    // all of the tile's address shuffles first (one LDS round trip), then its loads
    const unsigned lo = (unsigned)a, hi = (unsigned)(a >> 32);
    unsigned plo[IPT], phi[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      plo[i] = (unsigned)__shfl(lo, i * OPI + wocc);
      phi[i] = (unsigned)__shfl(hi, i * OPI + wocc);
    }
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const unsigned long long p = ((unsigned long long)phi[i] << 32) | plo[i];
      d[i] = *reinterpret_cast<gu32x4*>(p + (unsigned long long)vcol * ES);
    }
  };
  u32x4 data[S][IPT];
  unsigned long long next[S];
  {  // every address of the first 2S tiles lands before any data load: in the loop a
     // tile's addresses then always come after the data loads they must not drain
    unsigned long long first[S];
#pragma unroll
    for (int k = 0; k < S; ++k) {
      first[k] = addr(k);
      next[k] = addr(S + k);
    }
#pragma unroll
    for (int k = 0; k < S; ++k) asm volatile("" ::"v"(first[k]), "v"(next[k]));
#pragma unroll
    for (int k = 0; k < S; ++k) {
      issue(data[k], first[k]);
      __builtin_amdgcn_sched_barrier(0);  // stage order as in the loop (the waits depend on it)
    }
  }
  float acc = 0.f;
  unsigned char* wbase = ES == 2 ? img + wocc * ROWB + (lane % LPO) * 16 : img + wv * ROWB + wocc * ES;
  const unsigned char* rbase =
      ES == 2 ? img + ((lane & 15) >> 2) * ROWB + (((lane >> 4) % (SLICE / 16)) * 16 + (lane & 3) * 4) * 2
              : img + lane * ROWB;
  for (int t0 = 0; t0 < ntiles; t0 += S) {
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const int t = t0 + k;
#pragma unroll
      for (int i = 0; i < IPT; ++i) {
        const u32x4 v = data[k][i];
        if constexpr (ES == 2) {
          *reinterpret_cast<u32x4*>(wbase + i * OPI * ROWB) = v;
        } else {
#pragma unroll
          for (int e = 0; e < EPV; ++e) *reinterpret_cast<unsigned*>(wbase + e * ROWB + i * OPI * ES) = v[e];
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      issue(data[k], next[k]);          // tile t + S (clamped addresses past the row's end)
      next[k] = addr(t + 2 * S);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_wave_barrier();
      const int m = t < ntiles ? min(TILE, eu - su - t * TILE) : 0;
      if constexpr (ES == 2) {
        // every lane joins each transposing read (EXEC must be full); adds stop at m
        typedef short s16x4 __attribute__((ext_vector_type(4)));
        typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
        s16x4 w[TILE / 4];
#pragma unroll
        for (int q = 0; q < TILE / 4; ++q)
          w[q] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(rbase + 4 * q * ROWB));
        if (m == TILE) {
#pragma unroll
          for (int q = 0; q < TILE / 4; ++q)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc += __uint_as_float((unsigned)(unsigned short)w[q][e] << 16);
        } else {
#pragma unroll
          for (int q = 0; q < TILE / 4; ++q)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (4 * q + e < m) acc += __uint_as_float((unsigned)(unsigned short)w[q][e] << 16);
        }
      } else if (m == TILE) {  // whole tile: all LDS reads in flight ahead of the in-order adds
        uint2 w[TILE / EPR];
#pragma unroll
        for (int q = 0; q < TILE / EPR; ++q) w[q] = *reinterpret_cast<const uint2*>(rbase + q * 8);
#pragma unroll
        for (int q = 0; q < TILE / EPR; ++q) {
          acc += __uint_as_float(w[q].x);
          acc += __uint_as_float(w[q].y);
        }
      } else {
        for (int j = 0; j < m; ++j) acc += Elem<G>::load(reinterpret_cast<const G*>(rbase) + j);
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (lane < cols) {
    if (dense_out) dense_out[(int64_t)key * dim + c0 + lane] = acc;
    if (uniq_rows) uniq_rows[(int64_t)u * dim + c0 + lane] = acc;
  }
  if (row_slot && by == 0 && lane == 0) row_slot[key] = (int32_t)u;
}

template <typename G>
__global__ void __launch_bounds__(64) k_seg_hot(const unsigned* __restrict__ keys,
                                                const unsigned long long* __restrict__ gptr,
                                                const int* __restrict__ pos, const int* __restrict__ seg_start,
                                                const int* __restrict__ seg_end, int64_t n, unsigned sentinel, int dim,
                                                float* __restrict__ dense_out, float* __restrict__ uniq_rows,
                                                int32_t* __restrict__ row_slot) {
  __shared__ __attribute__((aligned(16))) unsigned char img[kHotImgBytes<G>()];
  seg_hot_body<G>(blockIdx.x, blockIdx.y, threadIdx.x, img, keys, gptr, pos, seg_start, seg_end, n, sentinel, dim,
                  dense_out, uniq_rows, row_slot);
}

// One launch for the wave path: waves [0, nhot) are the hot-row items
// (edge, slice) of k_seg_hot, the next nchunks the chunks of
// k_seg_chunks_wave, the rest the edges of k_seg_combine_edges.  The hot
// rows' sequential chains (tens of us, a few waves) then run beside the other
// waves instead of after them; the three write disjoint rows (a row is
// finished by exactly one of them).
template <typename G, int LW, int CH>
__global__ void __launch_bounds__(256) k_seg_wave_fused(int64_t nhot, int nslices, int64_t nchunks,
                                                        const unsigned* __restrict__ keys,
                                                        const unsigned long long* __restrict__ gptr,
                                                        const int* __restrict__ pos,
                                                        const int* __restrict__ seg_start,
                                                        const int* __restrict__ seg_end, int64_t n,
                                                        unsigned sentinel, int dim, float* __restrict__ dense_out,
                                                        float* __restrict__ uniq_rows,
                                                        int32_t* __restrict__ row_slot) {
  __shared__ __attribute__((aligned(16))) unsigned char img[4][kHotImgBytes<G>()];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t item = (int64_t)blockIdx.x * 4 + wave;
  if (item < nhot)
    seg_hot_body<G, CH>(item / nslices, (int)(item % nslices), lane, img[wave], keys, gptr, pos, seg_start, seg_end, n,
                    sentinel, dim, dense_out, uniq_rows, row_slot);
  else if (item < nhot + nchunks)
    seg_chunks_wave_body<G, LW, CH>(item - nhot, lane, keys, gptr, pos, seg_start, seg_end, n, sentinel, dim, dense_out,
                                uniq_rows, row_slot);
  else
    seg_edge_body<G, LW, CH>(item - nhot - nchunks, lane, keys, gptr, pos, seg_start, seg_end, n, sentinel, dim,
                         dense_out, uniq_rows, row_slot);
}

// ----------------------------------------------------- one-workgroup calls ----
// A call of at most kTinyN occurrences (the user table at BASELINE config 2: one
// user token per sequence, 128 occurrences) in ONE launch instead of ~14: keys
// built into LDS, stable ranks by counting (rank = smaller keys + equal keys
// earlier in occurrence order: the stable sort's permutation), segment heads by
// wave ballots, then one wave per unique row summing its occurrences in
// occurrence order -- the ordered mode's arithmetic (fp32 adds from 0, row by
// row in occurrence order), so the outputs equal the general path's bit for bit.
// Sparse outputs only (uniq_ids / uniq_rows / uniq_count / row_slot).
constexpr int kTinyN = 2048;
constexpr int kTinyThreads = 1024;

template <typename G, typename I, int LW>
__global__ void __launch_bounds__(kTinyThreads) k_bwd_tiny(LookupArgs la, int esize, const int32_t* __restrict__ token_type,
                                                          int32_t T_len, int64_t num_rows, int64_t padding_idx, int dim,
                                                          int64_t* __restrict__ uniq_ids, float* __restrict__ uniq_rows,
                                                          int32_t* __restrict__ uniq_count,
                                                          int32_t* __restrict__ row_slot, int32_t* err_flag) {
  __shared__ unsigned key[kTinyN];
  __shared__ unsigned long long ptr[kTinyN];
  __shared__ unsigned short ord[kTinyN];
  __shared__ int seg[kTinyN + 1];
  __shared__ int wtot[kTinyThreads / 64 + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NW = kTinyThreads / 64;
  const int64_t base = la.occ_off[0];
  const int n = (int)(la.occ_off[la.num] - base);
  const unsigned sentinel = (unsigned)num_rows;
  for (int o = tid; o < n; o += kTinyThreads) {
    const int64_t oa = base + o;
    int l = 0;
    while (l + 1 < la.num && oa >= la.occ_off[l + 1]) ++l;
    const grk_lookup& L = la.l[l];
    const int64_t rel = oa - la.occ_off[l];
    const int64_t t = rel / L.bag;
    const int a = (int)(rel - t * L.bag);
    const int64_t row = resolve_row(reinterpret_cast<const I*>(L.idx), t, a, L.idx_ld, L.idx_mode, token_type, T_len);
    unsigned k = sentinel;
    if (row < 0 || row >= L.table_rows || L.row_offset + row >= num_rows) {
      if (err_flag) *err_flag = 1;
    } else if (row != padding_idx) {
      k = (unsigned)(L.row_offset + row);
    }
    key[o] = k;
    ptr[o] = (unsigned long long)((const char*)L.grad + (t * L.grad_ld + L.grad_col) * esize);
  }
  __syncthreads();
  for (int i = tid; i < n; i += kTinyThreads) {
    const unsigned ki = key[i];
    int r = 0;
    for (int j = 0; j < n; ++j) {
      const unsigned kj = key[j];
      r += (kj < ki) | ((kj == ki) & (j < i));
    }
    ord[r] = (unsigned short)i;
  }
  __syncthreads();
  // segment heads in sorted order: each wave takes 2 x 64 consecutive positions
  constexpr int PER = kTinyN / kTinyThreads;   // positions per thread (2)
  int cnt = 0;
  bool hd[PER];
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const int pidx = (wave * PER + e) * 64 + lane;
    bool h = false;
    if (pidx < n) {
      const unsigned k = key[ord[pidx]];
      h = k != sentinel && (pidx == 0 || key[ord[pidx - 1]] != k);
    }
    hd[e] = h;
    cnt += __popcll(__ballot(h));
  }
  if (lane == 0) wtot[wave] = cnt;
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int w = 0; w < NW; ++w) {
      const int c = wtot[w];
      wtot[w] = acc;
      acc += c;
    }
    wtot[NW] = acc;
  }
  __syncthreads();
  int u0 = wtot[wave];
  const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const unsigned long long m = __ballot(hd[e]);
    if (hd[e]) seg[u0 + __popcll(m & below)] = (wave * PER + e) * 64 + lane;
    u0 += __popcll(m);
  }
  const int nseg = wtot[NW];
  if (tid == 0) {
    // one past the last real occurrence: the first sentinel position (sentinels sort last)
    int end = n;
    while (end > 0 && key[ord[end - 1]] == sentinel) --end;
    seg[nseg] = end;
    *uniq_count = nseg;
  }
  __syncthreads();
  const int c = lane * LW;
  for (int u = wave; u < nseg; u += NW) {
    const int s0 = seg[u], s1 = seg[u + 1];
    const unsigned k = key[ord[s0]];
    WaveAcc<LW> acc;
    acc.zero();
    for (int p = s0; p < s1; ++p) {
      WaveVec<G, LW> r;
      r.load(ptr[ord[p]], c);
#pragma unroll
      for (int x = 0; x < LW; ++x) acc.v[x] += r.get(x);
    }
    store_final(acc, k, u, dim, c, (float*)nullptr, uniq_rows, row_slot);
    if (uniq_ids && lane == 0) uniq_ids[u] = (int64_t)k;
  }
}

// ------------------------------------------------------------ workspace ----
// Stable radix sort of (row key, gradient-row address) pairs (grk_sort.hip).
size_t sort_pairs_workspace(int64_t n);
unsigned* sort_pairs_hist0(void* ws);
int sort_digit_bits(int end_bit);
int sort_pairs(unsigned* k0, unsigned long long* v0, unsigned* k1, unsigned long long* v1, int64_t n, int end_bit,
               void* ws, unsigned** kres, unsigned long long** vres, hipStream_t s, bool hist0_ready);
// Segment index of every sorted entry (inclusive count of row heads).
size_t head_positions_workspace(int64_t n);
int head_positions(const unsigned* keys, int64_t n, unsigned sentinel, int* pos, void* ws, hipStream_t s);

struct BwdWs {
  unsigned *keys_in, *keys_out, *seg_key;
  int *flags, *pos, *seg_start, *seg_end;
  unsigned long long *gptr_in, *gptr_out;
  float* partials;  // chunked mode: [chunks][2][dim] piece sums
  void* sort_tmp;
  size_t sort_bytes;
  void* scan_tmp;
  size_t scan_bytes;
  size_t total;
};

static inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

static int plan_ws(int64_t n, int64_t num_rows, int dim, char* base, BwdWs* ws) {
  size_t off = 0;
  auto take = [&](size_t bytes) -> char* {
    char* p = base ? base + off : nullptr;
    off += align256(bytes);
    return p;
  };
  ws->keys_in = (unsigned*)take(n * 4);
  ws->keys_out = (unsigned*)take(n * 4);
  ws->seg_key = (unsigned*)take(n * 4);
  ws->flags = (int*)take(n * 4);
  ws->pos = (int*)take(n * 4);
  ws->seg_start = (int*)take(n * 4);
  ws->seg_end = (int*)take(n * 4);
  ws->gptr_in = (unsigned long long*)take(n * 8);
  ws->gptr_out = (unsigned long long*)take(n * 8);
  ws->partials = (float*)take((size_t)((n + kPartialChunk - 1) / kPartialChunk) * 2 * dim * sizeof(float));
  unsigned end_bit = 1;
  while (end_bit < 32 && ((uint64_t)1 << end_bit) <= (uint64_t)num_rows) ++end_bit;
  size_t sb = 0, cb = 0;
  if (n > 0) {
    sb = sort_pairs_workspace(n);
    cb = head_positions_workspace(n);
  }
  ws->sort_bytes = sb;
  ws->sort_tmp = take(sb);
  ws->scan_bytes = cb;
  ws->scan_tmp = take(cb);
  ws->total = off;
  return GRK_OK;
}

// Ordered-mode wave path with CH-entry chunks: hot-row items, chunks and edges
// in one launch (k_seg_wave_fused) when rows longer than 2 CH can exist.
constexpr int64_t kSmallChunkLimit = 1 << 17;

template <typename G, int LW, int CH>
static int wave_ordered(const BwdWs& ws, int64_t total, unsigned sentinel, int dim, float* dense_out,
                        float* uniq_rows, int32_t* row_slot, hipStream_t s) {
  const int64_t chunks = (total + CH - 1) / CH;
  if (total > 2 * CH) {
    const int nsl = (dim + kHotSlice<G>() - 1) / kHotSlice<G>();
    const int64_t nhot = (chunks - 1) * nsl;
    const unsigned gf = (unsigned)((nhot + chunks + (chunks - 1) + 3) / 4);
    k_seg_wave_fused<G, LW, CH><<<gf, 256, 0, s>>>(nhot, nsl, chunks, ws.keys_out, ws.gptr_out, ws.pos, ws.seg_start,
                                                   ws.seg_end, total, sentinel, dim, dense_out, uniq_rows, row_slot);
    GRK_LAUNCH_CHECK();
    return GRK_OK;
  }
  k_seg_chunks_wave<G, LW, CH><<<(unsigned)((chunks + 3) / 4), 256, 0, s>>>(
      ws.keys_out, ws.gptr_out, ws.pos, ws.seg_start, ws.seg_end, total, sentinel, dim, dense_out, uniq_rows, row_slot);
  GRK_LAUNCH_CHECK();
  if (chunks > 1) {
    k_seg_combine_edges<G, LW, CH><<<(unsigned)((chunks - 1 + 3) / 4), 256, 0, s>>>(
        ws.keys_out, ws.gptr_out, ws.pos, ws.seg_start, ws.seg_end, total, sentinel, dim, dense_out, uniq_rows,
        row_slot);
    GRK_LAUNCH_CHECK();
  }
  return GRK_OK;
}

}  // namespace grk

using namespace grk;

extern "C" int grk_embedding_gather(const grk_feature* features, int num_features, int dim, int dtype, int itype,
                                    int64_t num_tokens, const int32_t* token_type, int32_t seq_len, void* out,
                                    int64_t out_ld, int32_t* err_flag, void* stream) {
  clear_error();
  GRK_CHECK_ARG(features && num_features > 0 && num_features <= GRK_MAX_FEATURES,
                "num_features must be in [1, %d]", GRK_MAX_FEATURES);
  GRK_CHECK_ARG(dtype == GRK_F32 || dtype == GRK_BF16, "dtype must be GRK_F32 or GRK_BF16");
  GRK_CHECK_ARG(itype == GRK_I32 || itype == GRK_I64, "itype must be GRK_I32 or GRK_I64");
  const int vec = dtype == GRK_F32 ? 4 : 8;
  GRK_CHECK_ARG(dim > 0 && dim % vec == 0, "dim (%d) must be a positive multiple of %d", dim, vec);
  GRK_CHECK_ARG(num_tokens >= 0 && (out != nullptr || num_tokens == 0), "bad output");
  GRK_CHECK_ARG(out_ld % vec == 0 && ((uintptr_t)out % 16) == 0, "output must be 16-byte aligned per row");
  FeatArgs fa;
  memset(&fa, 0, sizeof(fa));
  for (int i = 0; i < num_features; ++i) {
    const grk_feature& f = features[i];
    GRK_CHECK_ARG(f.table && (f.idx || num_tokens == 0) && f.bag >= 1 && f.num_rows > 0,
                  "feature %d: bad table/idx/bag", i);
    GRK_CHECK_ARG(f.out_col >= 0 && f.out_col + dim <= out_ld && f.out_col % vec == 0,
                  "feature %d: out_col %d out of range / misaligned", i, f.out_col);
    GRK_CHECK_ARG(((uintptr_t)f.table % 16) == 0, "feature %d: table must be 16-byte aligned", i);
    GRK_CHECK_ARG(f.idx_mode >= 0 && f.idx_mode <= 3, "feature %d: bad idx_mode", i);
    GRK_CHECK_ARG(f.idx_mode == GRK_IDX_PLAIN || f.idx_mode == GRK_IDX_POSITION || token_type,
                  "feature %d: masked mode needs token_type", i);
    GRK_CHECK_ARG(f.idx_mode != GRK_IDX_POSITION || seq_len > 0, "position mode needs seq_len");
    fa.f[i] = f;
  }
  if (num_tokens == 0) return GRK_OK;
  hipStream_t s = (hipStream_t)stream;
  if (dim / vec == 64) {
    const dim3 gw((unsigned)((num_tokens + 4 * kGatherRows - 1) / (4 * kGatherRows)), num_features);
#define GRK_GATHERW(T, I) \
  k_gather_wave<T, I><<<gw, 256, 0, s>>>(fa, num_tokens, token_type, seq_len, (T*)out, out_ld, err_flag)
    if (dtype == GRK_BF16) {
      if (itype == GRK_I64) GRK_GATHERW(bf16_t, int64_t);
      else GRK_GATHERW(bf16_t, int32_t);
    } else {
      if (itype == GRK_I64) GRK_GATHERW(float, int64_t);
      else GRK_GATHERW(float, int32_t);
    }
#undef GRK_GATHERW
    GRK_LAUNCH_CHECK();
    return GRK_OK;
  }
  const int64_t units = num_tokens * (dim / vec);
  // One (row, chunk) unit per lane over a wide grid: measured faster than 4 units
  // per lane both for cold random rows (scripts/microbench/gather.hip: 19 vs 32 us
  // for 41k rows of 1 KiB) and for the bag sums of the fused seq-side lookup (97 vs 115 us).
  const int nf = num_features > 8 ? 8 : num_features;
  dim3 grid(grid_for(units, 256, 8192 / nf + 1), num_features);
#define GRK_GATHER(T, I) \
  k_gather<T, I, 1><<<grid, 256, 0, s>>>(fa, dim, num_tokens, token_type, seq_len, (T*)out, out_ld, err_flag)
  if (dtype == GRK_BF16) {
    if (itype == GRK_I64) GRK_GATHER(bf16_t, int64_t);
    else GRK_GATHER(bf16_t, int32_t);
  } else {
    if (itype == GRK_I64) GRK_GATHER(float, int64_t);
    else GRK_GATHER(float, int32_t);
  }
#undef GRK_GATHER
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

extern "C" int grk_embedding_chunked_size(void) { return kPartialChunk; }

extern "C" size_t grk_embedding_backward_workspace(int64_t num_occurrences, int64_t num_rows, int dim) {
  BwdWs ws;
  if (plan_ws(num_occurrences, num_rows, dim, nullptr, &ws) != GRK_OK) return 0;
  return ws.total + 256;
}

extern "C" int grk_embedding_backward(const grk_lookup* lookups, int num_lookups, int dim, int grad_dtype,
                                      int itype, const int32_t* token_type, int32_t seq_len, int64_t num_rows,
                                      int64_t padding_idx, void* dense_out_, int64_t* uniq_ids, float* uniq_rows,
                                      int32_t* uniq_count, int32_t* row_slot, int flags, void* workspace,
                                      size_t workspace_bytes, int32_t* err_flag, void* stream) {
  clear_error();
  const bool dense_bf16 = (flags & GRK_BWD_DENSE_BF16) != 0;
  flags &= ~GRK_BWD_DENSE_BF16;
  GRK_CHECK_ARG(flags == GRK_BWD_ORDERED || flags == GRK_BWD_CHUNKED, "bad flags %d", flags);
  GRK_CHECK_ARG(!dense_bf16 || (flags == GRK_BWD_CHUNKED && grad_dtype == GRK_BF16 && dim == 512),
                "GRK_BWD_DENSE_BF16 needs GRK_BWD_CHUNKED with bf16 gradients of 512 columns");
  float* dense_out = dense_bf16 ? nullptr : (float*)dense_out_;
  bf16_t* dense_out16 = dense_bf16 ? (bf16_t*)dense_out_ : nullptr;
  GRK_CHECK_ARG(lookups && num_lookups > 0, "need at least one lookup");
  GRK_CHECK_ARG(grad_dtype == GRK_F32 || grad_dtype == GRK_BF16, "grad_dtype must be GRK_F32 or GRK_BF16");
  GRK_CHECK_ARG(itype == GRK_I32 || itype == GRK_I64, "bad itype");
  const int vec_req = grad_dtype == GRK_BF16 ? 8 : 4;
  GRK_CHECK_ARG(dim > 0 && dim % vec_req == 0 && dim / vec_req <= 256, "dim (%d) must be a multiple of %d and <= %d",
                dim, vec_req, 256 * vec_req);
  GRK_CHECK_ARG(num_rows > 0 && num_rows < 0xFFFFFFFFLL, "num_rows out of range");
  GRK_CHECK_ARG(uniq_count != nullptr, "uniq_count is required");
  int64_t total = 0;
  for (int i = 0; i < num_lookups; ++i) {
    const grk_lookup& L = lookups[i];
    GRK_CHECK_ARG(L.bag >= 1 && L.num_tokens >= 0 && ((L.idx && L.grad) || L.num_tokens == 0),
                  "lookup %d: bad idx/grad/bag", i);
    GRK_CHECK_ARG(L.idx_mode >= 0 && L.idx_mode <= 3, "lookup %d: bad idx_mode", i);
    GRK_CHECK_ARG(L.idx_mode == GRK_IDX_PLAIN || L.idx_mode == GRK_IDX_POSITION || token_type,
                  "lookup %d: masked mode needs token_type", i);
    GRK_CHECK_ARG(L.row_offset >= 0 && L.table_rows > 0 && L.row_offset + L.table_rows <= num_rows,
                  "lookup %d: rows [%lld, +%lld) outside the group's %lld rows", i, (long long)L.row_offset,
                  (long long)L.table_rows, (long long)num_rows);
    GRK_CHECK_ARG(L.grad_col >= 0 && L.grad_col + dim <= L.grad_ld, "lookup %d: grad_col out of range", i);
    total += L.num_tokens * L.bag;
  }
  GRK_CHECK_ARG(total < 0x7FFFFFFFLL, "too many occurrences");
  BwdWs ws;
  if (plan_ws(total, num_rows, dim, nullptr, &ws) != GRK_OK) {
    set_error("workspace query failed");
    return GRK_EHIP;
  }
  GRK_CHECK_ARG(workspace_bytes >= ws.total + 256 && workspace, "workspace too small (%zu < %zu)", workspace_bytes,
                ws.total + 256);
  char* base = (char*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
  plan_ws(total, num_rows, dim, base, &ws);
  hipStream_t s = (hipStream_t)stream;
  void* dense_any = dense_out ? (void*)dense_out : (void*)dense_out16;
  const size_t dense_bytes = (size_t)num_rows * dim * (dense_out ? sizeof(float) : sizeof(bf16_t));
  // the zero fill rides on the first key-build launch (16-byte aligned outputs; else a fill kernel)
  const bool fused_zero = total > 0 && (!dense_any || ((uintptr_t)dense_any % 16 == 0 && dense_bytes % 16 == 0));
  if (!fused_zero) {
    GRK_CHECK_HIP(zero_async(uniq_count, sizeof(int32_t), s));
    if (dense_any) GRK_CHECK_HIP(zero_async(dense_any, dense_bytes, s));
  }
  if (total == 0) return GRK_OK;
  const int B = 256;
  const int esize = grad_dtype == GRK_F32 ? 4 : 2;
  const unsigned sentinel = (unsigned)num_rows;
  {
    // a small sparse call in one launch (k_bwd_tiny): ordered mode, sparse outputs only
    const int lwt = dim % 64 == 0 ? dim / 64 : 0;
    const bool tiny_ok = total <= kTinyN && num_lookups <= kLookupsPerLaunch && flags == GRK_BWD_ORDERED &&
                         !dense_any && (uniq_rows || row_slot || uniq_ids) &&
                         ((grad_dtype == GRK_BF16 && lwt == 8) || (grad_dtype != GRK_BF16 && (lwt == 4 || lwt == 8)));
    if (tiny_ok) {
      LookupArgs la;
      memset(&la, 0, sizeof(la));
      la.num = num_lookups;
      int64_t occ = 0;
      for (int i = 0; i < num_lookups; ++i) {
        la.l[i] = lookups[i];
        la.occ_off[i] = occ;
        occ += lookups[i].num_tokens * lookups[i].bag;
      }
      la.occ_off[num_lookups] = occ;
#define GRK_TINY(G, I, LW)                                                                                          \
  k_bwd_tiny<G, I, LW><<<1, kTinyThreads, 0, s>>>(la, esize, token_type, seq_len, num_rows, padding_idx, dim,    \
                                                  uniq_ids, uniq_rows, uniq_count, row_slot, err_flag)
      if (itype == GRK_I64) {
        if (grad_dtype == GRK_BF16) GRK_TINY(bf16_t, int64_t, 8);
        else if (lwt == 8) GRK_TINY(float, int64_t, 8);
        else GRK_TINY(float, int64_t, 4);
      } else {
        if (grad_dtype == GRK_BF16) GRK_TINY(bf16_t, int32_t, 8);
        else if (lwt == 8) GRK_TINY(float, int32_t, 8);
        else GRK_TINY(float, int32_t, 4);
      }
#undef GRK_TINY
      GRK_LAUNCH_CHECK();
      return GRK_OK;
    }
  }
  // chunked mode writing only the dense rows: segment bounds by row (k_segments_key),
  // no segment numbering (head positions) at all
  const int lw0 = dim % 64 == 0 ? dim / 64 : 0;
  const bool wave_path = (grad_dtype == GRK_BF16 && lw0 == 8) || (grad_dtype != GRK_BF16 && (lw0 == 4 || lw0 == 8));
  const bool by_key = wave_path && flags == GRK_BWD_CHUNKED && !uniq_ids && !uniq_rows && !row_slot &&
                      num_rows <= total;
  // one key-build launch (<= kLookupsPerLaunch lookups): it also counts the sort's first digit
  const bool one_launch = num_lookups <= kLookupsPerLaunch;
  const int ntiles = (int)((total + kKeyTile - 1) / kKeyTile);
  unsigned end_bit = 1;
  while (end_bit < 32 && ((uint64_t)1 << end_bit) <= (uint64_t)num_rows) ++end_bit;
  const int bits0 = sort_digit_bits((int)end_bit);
  int64_t occ = 0;
  bool first_launch = true;
  for (int first = 0; first < num_lookups; first += kLookupsPerLaunch) {
    LookupArgs la;
    memset(&la, 0, sizeof(la));
    la.num = num_lookups - first < kLookupsPerLaunch ? num_lookups - first : kLookupsPerLaunch;
    for (int i = 0; i < la.num; ++i) {
      la.l[i] = lookups[first + i];
      la.occ_off[i] = occ;
      occ += la.l[i].num_tokens * la.l[i].bag;
    }
    la.occ_off[la.num] = occ;
    const int64_t cnt = occ - la.occ_off[0];
    if (cnt == 0) continue;
    const unsigned g = (unsigned)((cnt + kKeyTile - 1) / kKeyTile);
    const bool fill_here = first_launch;
    KeyFill fill;
    memset(&fill, 0, sizeof(fill));
    if (fill_here) {
      fill.zero_vecs = fused_zero && dense_any ? (int64_t)(dense_bytes / 16) : 0;
      fill.zero_dst = fill.zero_vecs ? (uint4*)dense_any : nullptr;
      fill.zero_count = fused_zero ? uniq_count : nullptr;
    }
    const unsigned gz = fill_here ? (unsigned)grid_for(fill.zero_vecs > 0 ? fill.zero_vecs : 1, B, 2048) : 0;
    unsigned* h0 = one_launch ? sort_pairs_hist0(ws.sort_tmp) : nullptr;
    if (itype == GRK_I64)
      k_build_keys<int64_t><<<g + gz, B, 0, s>>>(la, esize, token_type, seq_len, num_rows, padding_idx, ws.keys_in,
                                                 ws.gptr_in, err_flag, g, h0, ntiles, bits0, fill);
    else
      k_build_keys<int32_t><<<g + gz, B, 0, s>>>(la, esize, token_type, seq_len, num_rows, padding_idx, ws.keys_in,
                                                 ws.gptr_in, err_flag, g, h0, ntiles, bits0, fill);
    GRK_LAUNCH_CHECK();
    first_launch = false;
  }
  const int g = (int)((total + B - 1) / B);
  unsigned* skeys;
  unsigned long long* sgptr;
  {
    const int rc = sort_pairs(ws.keys_in, ws.gptr_in, ws.keys_out, ws.gptr_out, total, (int)end_bit, ws.sort_tmp, &skeys,
                              &sgptr, s, one_launch);
    if (rc) return rc;
  }
  ws.keys_out = skeys;  // the sorted pairs (either buffer of the ping-pong)
  ws.gptr_out = sgptr;
  if (by_key) {
    k_segments_key<<<g < kSegKeyBlocks ? g : kSegKeyBlocks, B, 0, s>>>(ws.keys_out, total, sentinel, ws.seg_start,
                                                                       ws.seg_end, uniq_count);
    GRK_LAUNCH_CHECK();
    ws.pos = nullptr;
  } else {
    const int rc = head_positions(ws.keys_out, total, sentinel, ws.pos, ws.scan_tmp, s);
    if (rc) return rc;
    k_segments<<<g, B, 0, s>>>(ws.keys_out, ws.pos, total, sentinel, ws.seg_start, ws.seg_end, ws.seg_key, uniq_ids,
                               uniq_count);
    GRK_LAUNCH_CHECK();
  }
  const int vec = grad_dtype == GRK_BF16 ? 8 : 4;
  const int tpr = dim / vec;
  const int groups = tpr >= 256 ? 1 : 256 / tpr;
  const int block = tpr >= 256 ? tpr : groups * tpr;
  const int64_t chunks = (total + kRedChunk - 1) / kRedChunk;
  const int lw = dim % 64 == 0 ? dim / 64 : 0;  // elements per lane with one wave per row
  if ((grad_dtype == GRK_BF16 && lw == 8) || (grad_dtype != GRK_BF16 && (lw == 4 || lw == 8))) {
    if (flags == GRK_BWD_CHUNKED) {
      const int64_t pchunks = (total + kPartialChunk - 1) / kPartialChunk;
      const unsigned gw = (unsigned)((pchunks + 3) / 4);
      const unsigned ge = (unsigned)(pchunks > 1 ? (pchunks - 1 + 3) / 4 : 0);
#define GRK_SEGP(G, LW)                                                                                          \
  k_seg_chunks_partial<G, LW, kPartialChunk><<<gw, 256, 0, s>>>(ws.keys_out, ws.gptr_out, ws.pos, ws.seg_start,  \
                                                                ws.seg_end, total, sentinel, dim, dense_out,     \
                                                                uniq_rows, row_slot, ws.partials);               \
  GRK_LAUNCH_CHECK();                                                                                            \
  if (ge)                                                                                                        \
    k_seg_partials_combine<LW, kPartialChunk><<<ge, 256, 0, s>>>(ws.keys_out, ws.pos, ws.seg_start, ws.seg_end,  \
                                                                 total, sentinel, dim, ws.partials, dense_out,    \
                                                                 uniq_rows, row_slot)
      const bool cols = grad_dtype == GRK_BF16 && dim == 512 && !ws.pos && !uniq_rows && !row_slot;
      if (cols) {   // column-sliced by XCD: same pieces and adds, an eighth of the rows' bytes per XCD
        const unsigned gc = (unsigned)(8 * ((pchunks + 31) / 32));
        if (dense_out16)
          k_seg_chunks_cols<kPartialChunk, bf16_t><<<gc, 256, 0, s>>>(ws.keys_out, ws.gptr_out, total, sentinel,
                                                                      dense_out16, ws.partials);
        else
          k_seg_chunks_cols<kPartialChunk, float><<<gc, 256, 0, s>>>(ws.keys_out, ws.gptr_out, total, sentinel,
                                                                     dense_out, ws.partials);
        GRK_LAUNCH_CHECK();
        if (ge) {
          if (dense_out16)
            k_seg_partials_combine<8, kPartialChunk, bf16_t><<<ge, 256, 0, s>>>(
                ws.keys_out, ws.pos, ws.seg_start, ws.seg_end, total, sentinel, dim, ws.partials, dense_out16,
                uniq_rows, row_slot);
          else
            k_seg_partials_combine<8, kPartialChunk><<<ge, 256, 0, s>>>(ws.keys_out, ws.pos, ws.seg_start,
                                                                       ws.seg_end, total, sentinel, dim, ws.partials,
                                                                       dense_out, uniq_rows, row_slot);
        }
      } else if (dense_out16) {
        k_seg_chunks_partial<bf16_t, 8, kPartialChunk, bf16_t><<<gw, 256, 0, s>>>(
            ws.keys_out, ws.gptr_out, ws.pos, ws.seg_start, ws.seg_end, total, sentinel, dim, dense_out16, uniq_rows,
            row_slot, ws.partials);
        GRK_LAUNCH_CHECK();
        if (ge)
          k_seg_partials_combine<8, kPartialChunk, bf16_t><<<ge, 256, 0, s>>>(
              ws.keys_out, ws.pos, ws.seg_start, ws.seg_end, total, sentinel, dim, ws.partials, dense_out16, uniq_rows,
              row_slot);
      } else if (grad_dtype == GRK_BF16) { GRK_SEGP(bf16_t, 8); }
      else if (lw == 8) { GRK_SEGP(float, 8); }
      else { GRK_SEGP(float, 4); }
#undef GRK_SEGP
      GRK_LAUNCH_CHECK();
      return GRK_OK;
    }
    // occurrence-order mode: chunks of 64 for short lists (more waves in flight
    // on calls of a few 10k mostly-distinct rows: the item / user tables),
    // 256 otherwise
    int rc;
    if (total <= kSmallChunkLimit) {
      if (grad_dtype == GRK_BF16) rc = wave_ordered<bf16_t, 8, 64>(ws, total, sentinel, dim, dense_out, uniq_rows, row_slot, s);
      else if (lw == 8) rc = wave_ordered<float, 8, 64>(ws, total, sentinel, dim, dense_out, uniq_rows, row_slot, s);
      else rc = wave_ordered<float, 4, 64>(ws, total, sentinel, dim, dense_out, uniq_rows, row_slot, s);
    } else {
      if (grad_dtype == GRK_BF16) rc = wave_ordered<bf16_t, 8, kRedChunk>(ws, total, sentinel, dim, dense_out, uniq_rows, row_slot, s);
      else if (lw == 8) rc = wave_ordered<float, 8, kRedChunk>(ws, total, sentinel, dim, dense_out, uniq_rows, row_slot, s);
      else rc = wave_ordered<float, 4, kRedChunk>(ws, total, sentinel, dim, dense_out, uniq_rows, row_slot, s);
    }
    return rc;
  } else {
    const unsigned gc = (unsigned)((chunks + groups - 1) / groups);
    const unsigned gu = (unsigned)((total + groups - 1) / groups);
    if (grad_dtype == GRK_BF16) {
      k_seg_chunks<bf16_t><<<gc, block, 0, s>>>(ws.keys_out, ws.gptr_out, ws.pos, ws.seg_start, ws.seg_end, total,
                                                sentinel, dim, dense_out, uniq_rows, row_slot);
      GRK_LAUNCH_CHECK();
      k_seg_combine<bf16_t><<<gu, block, 0, s>>>(ws.gptr_out, ws.seg_start, ws.seg_end, ws.seg_key, uniq_count, total,
                                                 dim, dense_out, uniq_rows, row_slot);
    } else {
      k_seg_chunks<float><<<gc, block, 0, s>>>(ws.keys_out, ws.gptr_out, ws.pos, ws.seg_start, ws.seg_end, total,
                                               sentinel, dim, dense_out, uniq_rows, row_slot);
      GRK_LAUNCH_CHECK();
      k_seg_combine<float><<<gu, block, 0, s>>>(ws.gptr_out, ws.seg_start, ws.seg_end, ws.seg_key, uniq_count, total,
                                                dim, dense_out, uniq_rows, row_slot);
    }
    GRK_LAUNCH_CHECK();
  }
  if (total > 2 * kRedChunk) {  // rows longer than 2 * kRedChunk exist only then
    const dim3 gh((unsigned)(chunks - 1), (unsigned)((dim + kHotSlice<bf16_t>() - 1) / kHotSlice<bf16_t>()));
    const dim3 gf((unsigned)(chunks - 1), (unsigned)((dim + kHotSlice<float>() - 1) / kHotSlice<float>()));
    if (grad_dtype == GRK_BF16)
      k_seg_hot<bf16_t><<<gh, 64, 0, s>>>(ws.keys_out, ws.gptr_out, ws.pos, ws.seg_start, ws.seg_end, total, sentinel,
                                          dim, dense_out, uniq_rows, row_slot);
    else
      k_seg_hot<float><<<gf, 64, 0, s>>>(ws.keys_out, ws.gptr_out, ws.pos, ws.seg_start, ws.seg_end, total, sentinel,
                                         dim, dense_out, uniq_rows, row_slot);
    GRK_LAUNCH_CHECK();
  }
  return GRK_OK;
}
