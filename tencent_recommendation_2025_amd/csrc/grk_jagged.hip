// Jagged (valid-token) layout of a training batch.
//
// The reference left-pads every sequence to T = maxlen + 1 and runs every
// token-wise op over all B*T rows (model/BaseLine/model.py:331-350,379-384);
// rows before a sequence's first valid token are dead: they are no key of any
// query (key padding mask), their logits are masked (next_token_type != 1), so
// nothing reaches the loss from them and their gradients are exact zeros.  At
// BASELINE config 2 they are ~47 % of the rows.  The fused trainer therefore
// runs the token-wise part of the step over each sequence's span
// [start_b, T) only, packed back to back:
//
//   row_map[r]  = b * T + t  for the r-th span token (b ascending, t ascending),
//                 -1 for the dead capacity rows r in [n, cap);
//   row_base[b] = (rows of the spans before b) - start_b, so token (b, t) is
//                 row row_base[b] + t (the attention kernels' jagged addressing);
//   seq_range   = grk_seq_ranges' [B, 3] (start, contiguous flag, longest-first).
//
// grk_gather_rows then copies the batch's per-token tensors (ids, features,
// token types) into that order in one launch.  Integer / byte work of a few MB:
// launch-bound.
#include "grk_common.h"

namespace grk {
namespace {

// exclusive scan of the spans (T - start_b) over b -> row_base, total -> *n_rows;
// one workgroup, chunks of 1024 sequences.  Spans that would end past `cap`
// (the caller under-stated the batch's rows) are dropped, never addressed out of
// bounds: their start becomes T (an empty sequence for every kernel that reads
// the ranges: no rows read or written), row_base -T, and err bit 2 is raised.
// The kept spans are a prefix (the inclusive scan is monotone), so *n_rows <= cap.
__global__ void __launch_bounds__(1024) k_jagged_base(int32_t* __restrict__ ranges, int B, int T, int64_t cap,
                                                      int64_t* __restrict__ row_base, int64_t* __restrict__ n_rows,
                                                      int32_t* __restrict__ err) {
  __shared__ int64_t part[1024];
  __shared__ int dropped;
  __shared__ unsigned long long kept;   // largest inclusive span sum <= cap
  if (threadIdx.x == 0) {
    dropped = 0;
    kept = 0;
  }
  int64_t carry = 0;
  for (int b0 = 0; b0 < B; b0 += 1024) {
    const int b = b0 + (int)threadIdx.x;
    const int st = b < B ? min(max(ranges[3 * b], 0), T) : T;
    const int64_t span = b < B ? (int64_t)(T - st) : 0;
    part[threadIdx.x] = span;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // inclusive Hillis-Steele scan
      const int64_t v = (int)threadIdx.x >= off ? part[threadIdx.x - off] : 0;
      __syncthreads();
      part[threadIdx.x] += v;
      __syncthreads();
    }
    const int64_t incl = carry + part[threadIdx.x];
    if (b < B) {
      if (incl <= cap) {
        row_base[b] = incl - span - st;
        atomicMax(&kept, (unsigned long long)incl);
      } else {
        row_base[b] = -(int64_t)T;
        ranges[3 * b] = T;
        ranges[3 * b + 1] = 1;
        dropped = 1;
      }
    }
    carry += part[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    *n_rows = (int64_t)kept;
    if (dropped && err) atomicOr(err, 2);
  }
}

// row_map over max(B*T, cap) indices: span tokens at their rows, -1 past n.
// err bit 1: a token before its sequence's span has next_token_type == 1 (its
// logit would be dropped; this includes every labelled token of a span that
// k_jagged_base dropped); bit 2 (k_jagged_base): the spans hold more rows than
// cap -- the trailing spans were dropped.
__global__ void __launch_bounds__(256) k_jagged_map(const int32_t* __restrict__ ranges, const int64_t* __restrict__ row_base,
                                                    const int64_t* __restrict__ n_rows, int B, int T, int64_t cap,
                                                    const int32_t* __restrict__ ntt, int32_t* __restrict__ row_map,
                                                    int32_t* __restrict__ err) {
  const int64_t total = (int64_t)B * T > cap ? (int64_t)B * T : cap;
  const int64_t n = *n_rows;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    if (i < (int64_t)B * T) {
      const int b = (int)(i / T), t = (int)(i % T);
      const int st = min(max(ranges[3 * b], 0), T);
      if (t >= st) {
        const int64_t r = row_base[b] + t;
        if (r < cap) row_map[r] = (int32_t)i;
        else if (err) atomicOr(err, 2);
      } else if (ntt && err && ntt[i] == 1) {
        atomicOr(err, 1);
      }
    }
    if (i >= n && i < cap) row_map[i] = -1;
  }
}

constexpr int kMaxRowCopies = 64;
constexpr int kRowUnitsPerBlock = 1024;   // 4 units per thread
struct RowCopies {
  grk_row_copy c[kMaxRowCopies];
  int32_t bend[kMaxRowCopies];   // workgroups of copies [0, i]
  int32_t meta[kMaxRowCopies];   // units per row << 2 | (log2(unit bytes) - 2)
  int n;
};

template <int SH>
struct RowUnit;
template <>
struct RowUnit<2> { typedef uint32_t T; };
template <>
struct RowUnit<3> { typedef uint2 T; };
template <>
struct RowUnit<4> { typedef uint4 T; };

template <int SH>
__device__ __forceinline__ void copy_units(const grk_row_copy& c, const int32_t* __restrict__ row_map, int64_t u0,
                                           int64_t units, int upr, bool div32) {
  typedef typename RowUnit<SH>::T U;
  U v[4];
  int64_t dst_off[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t u = u0 + k * 256 + threadIdx.x;
    dst_off[k] = -1;
    if (u >= units) continue;
    const int64_t r = upr == 1 ? u : div32 ? (int64_t)((uint32_t)u / (uint32_t)upr) : u / upr;
    const int64_t w = u - r * upr;
    const int32_t src_row = row_map[r];
    v[k] = src_row >= 0 ? *reinterpret_cast<const U*>((const char*)c.src + src_row * c.src_ld + (w << SH)) : U{};
    dst_off[k] = r * c.dst_ld + (w << SH);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (dst_off[k] >= 0) *reinterpret_cast<U*>((char*)c.dst + dst_off[k]) = v[k];
}

// dst row r <- src row row_map[r] (zeros for -1), every copy at once.  Each
// copy moves rows in the widest unit (16 / 8 / 4 bytes) its row size, strides
// and pointers allow, over its own run of workgroups (1024 consecutive units
// each: the copy is workgroup-uniform, loads of 4 units in flight per lane).
// Was one 4-byte word per thread with a 64-bit division and a fixed grid per
// copy (mostly empty workgroups): 107 us for the bench batch's 60 copies,
// ~28 MB moved.
__global__ void __launch_bounds__(256) k_gather_rows(RowCopies rc, const int32_t* __restrict__ row_map, int64_t rows) {
  const int bx = blockIdx.x;
  int lo = 0, hi = rc.n - 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (rc.bend[mid] <= bx) lo = mid + 1;
    else hi = mid;
  }
  const grk_row_copy& c = rc.c[lo];
  const int64_t u0 = (int64_t)(bx - (lo ? rc.bend[lo - 1] : 0)) * kRowUnitsPerBlock;
  const int upr = rc.meta[lo] >> 2;
  const int64_t units = rows * upr;
  const bool div32 = units < ((int64_t)1 << 32);
  switch (rc.meta[lo] & 3) {
    case 2: copy_units<4>(c, row_map, u0, units, upr, div32); break;
    case 1: copy_units<3>(c, row_map, u0, units, upr, div32); break;
    default: copy_units<2>(c, row_map, u0, units, upr, div32); break;
  }
}

}  // namespace

bool seq_ranges_jagged(const uint8_t* key_valid, int batch, int seq_len, int64_t cap, int32_t* ranges,
                       int64_t* row_base, int64_t* n_rows, int32_t* err, hipStream_t s);   // grk_attention_seq.hip
}  // namespace grk

using namespace grk;

extern "C" int grk_jagged_layout(const uint8_t* key_valid, int batch, int seq_len, int64_t capacity,
                                 const int32_t* next_token_type, int32_t* ranges, int64_t* row_base, int32_t* row_map,
                                 int64_t* num_rows, int32_t* err_flag, void* stream) {
  clear_error();
  GRK_CHECK_ARG(batch > 0 && seq_len > 0 && capacity > 0, "batch, seq_len and capacity must be > 0");
  GRK_CHECK_ARG(capacity < ((int64_t)1 << 31) && (int64_t)batch * seq_len < ((int64_t)1 << 31),
                "rows must fit int32");
  GRK_CHECK_ARG(key_valid && ranges && row_base && row_map && num_rows, "key_valid, ranges, row_base, row_map, num_rows required");
  hipStream_t s = (hipStream_t)stream;
  if (seq_ranges_jagged(key_valid, batch, seq_len, capacity, ranges, row_base, num_rows, err_flag, s)) {
    GRK_LAUNCH_CHECK();
  } else {
    const int rc = grk_seq_ranges(key_valid, batch, seq_len, ranges, stream);
    if (rc) return rc;
    k_jagged_base<<<1, 1024, 0, s>>>(ranges, batch, seq_len, capacity, row_base, num_rows, err_flag);
    GRK_LAUNCH_CHECK();
  }
  const int64_t total = (int64_t)batch * seq_len > capacity ? (int64_t)batch * seq_len : capacity;
  k_jagged_map<<<grid_for(total, 256), 256, 0, s>>>(ranges, row_base, num_rows, batch, seq_len, capacity,
                                                    next_token_type, row_map, err_flag);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

extern "C" int grk_gather_rows(const grk_row_copy* copies, int num_copies, const int32_t* row_map, int64_t rows,
                               void* stream) {
  clear_error();
  GRK_CHECK_ARG(num_copies >= 0 && num_copies <= kMaxRowCopies, "num_copies must be in [0, %d]", kMaxRowCopies);
  GRK_CHECK_ARG(rows >= 0, "rows must be >= 0");
  if (num_copies == 0 || rows == 0) return GRK_OK;
  GRK_CHECK_ARG(copies && row_map, "copies and row_map required");
  RowCopies rc;
  memset(&rc, 0, sizeof(rc));
  rc.n = num_copies;
  int64_t blocks = 0;
  for (int i = 0; i < num_copies; ++i) {
    const grk_row_copy& c = copies[i];
    GRK_CHECK_ARG(c.src && c.dst, "copy %d: src / dst required", i);
    GRK_CHECK_ARG(c.row_bytes > 0 && c.row_bytes % 4 == 0 && c.src_ld >= c.row_bytes && c.dst_ld >= c.row_bytes &&
                      c.src_ld % 4 == 0 && c.dst_ld % 4 == 0,
                  "copy %d: row_bytes must be a positive multiple of 4, strides >= row_bytes and multiples of 4", i);
    GRK_CHECK_ARG(((uintptr_t)c.src | (uintptr_t)c.dst) % 4 == 0, "copy %d: 4-byte aligned buffers required", i);
    GRK_CHECK_ARG(c.row_bytes / 4 < (1 << 29), "copy %d: rows too wide", i);
    int sh = 4;   // widest unit dividing the row, both strides and both pointers
    while (sh > 2 && ((c.row_bytes | c.src_ld | c.dst_ld | (int64_t)(uintptr_t)c.src | (int64_t)(uintptr_t)c.dst) &
                      ((1 << sh) - 1)))
      --sh;
    const int64_t upr = c.row_bytes >> sh;
    rc.c[i] = c;
    rc.meta[i] = (int32_t)(upr << 2 | (sh - 2));
    blocks += (rows * upr + kRowUnitsPerBlock - 1) / kRowUnitsPerBlock;
    GRK_CHECK_ARG(blocks < ((int64_t)1 << 31), "gather_rows: too many rows for one launch");
    rc.bend[i] = (int32_t)blocks;
  }
  k_gather_rows<<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(rc, row_map, rows);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}
