// Stable LSD radix sort of (uint32 key, uint64 value) pairs for the embedding
// backward's occurrence grouping (grk_embedding.hip): keys are table rows
// (< 2^end_bit, end_bit = bits of the group's row count), values the
// occurrences' gradient-row addresses, and the output must keep occurrence
// order within a row -- the reference's CPU embedding_dense_backward sums a
// row's occurrences sequentially in that order.
//
// rocprim::radix_sort_pairs took ~15 launches per call at these sizes (73
// launches, ~0.5 ms per C2 training step over five calls).  Here a pass per
// digit is three launches:
//   k_sort_hist    per 1024-key tile: digit counts -> hist[digit][tile]
//   k_sort_scan    one workgroup per digit: exclusive scan of the digit's
//                  tile counts, and the digit's total (the scatter's prologue
//                  prefixes the totals)
//   k_sort_scatter per tile, 4 rounds of 256 keys in index order: a key's
//                  slot = its (digit, tile) base + the keys of its digit in
//                  earlier rounds, earlier waves of this round, and lower
//                  lanes of its wave (wave ballots over the digit bits)
// so the order among equal digits is the input order: stable, deterministic,
// and (a stable sort being unique) the same output as rocprim's.
//
// Digits are up to 11 bits wide, as few passes as the key width allows
// (sort_digit_bits): the 1M-row tables' 20-bit keys take two passes of 10
// bits where 8-bit digits took three (round 4: one pass = 3 launches less
// per call).  Per-wave digit counts of a round live in LDS tagged with the
// round, so no per-round clearing of 4 x 2048 counters.
//
// The first pass's histogram can come from the caller (the embedding
// backward counts digit 0 inside its key-build kernel: hist0_ready).  Round 4
// also tried counting each next digit inside the scatter (global atomics per
// (digit, output tile), wave-aggregated): 0.34 ms per C2 step against 0.06 for
// these histogram launches -- runs of equal keys contend on one counter.
#include "grk_common.h"

namespace grk {

// Width of every digit of a sort of end_bit-bit keys: as few passes of <= 11
// bits as cover them, split evenly.
int sort_digit_bits(int end_bit) {
  if (end_bit <= 8) return end_bit < 1 ? 1 : end_bit;
  const int passes = (end_bit + 10) / 11;
  return (end_bit + passes - 1) / passes;
}

namespace {

constexpr int kSortMaxBits = 11, kSortMaxBins = 1 << kSortMaxBits;
constexpr int kSortThreads = 256, kSortRounds = 4, kSortTile = kSortThreads * kSortRounds;

__global__ void __launch_bounds__(kSortThreads) k_sort_hist(const unsigned* __restrict__ keys, int64_t n, int shift,
                                                            int bits, unsigned* __restrict__ hist, int ntiles) {
  __shared__ unsigned cnt[kSortMaxBins];
  const int tid = threadIdx.x, tile = blockIdx.x, nbins = 1 << bits;
  const unsigned mask = (unsigned)nbins - 1u;
  for (int d = tid; d < nbins; d += kSortThreads) cnt[d] = 0;
  __syncthreads();
  const int64_t t0 = (int64_t)tile * kSortTile;
#pragma unroll 4
  for (int r = 0; r < kSortRounds; ++r) {
    const int64_t i = t0 + r * kSortThreads + tid;
    if (i < n) atomicAdd(&cnt[(keys[i] >> shift) & mask], 1u);
  }
  __syncthreads();
  for (int d = tid; d < nbins; d += kSortThreads) hist[(int64_t)d * ntiles + tile] = cnt[d];
}

// Per digit (one workgroup each): in-place exclusive scan of the digit's tile
// counts hist[d][0 .. ntiles) and the digit's total -> tot[d].
__global__ void __launch_bounds__(kSortThreads) k_sort_scan(unsigned* __restrict__ hist, int ntiles,
                                                            unsigned* __restrict__ tot) {
  __shared__ unsigned part[kSortThreads];
  const int t = threadIdx.x;
  unsigned* row = hist + (int64_t)blockIdx.x * ntiles;
  unsigned carry = 0;
  for (int c0 = 0; c0 < ntiles; c0 += kSortThreads) {
    const int i = c0 + t;
    const unsigned v = i < ntiles ? row[i] : 0u;
    part[t] = v;
    __syncthreads();
    for (int off = 1; off < kSortThreads; off <<= 1) {  // inclusive scan of this chunk
      const unsigned u = t >= off ? part[t - off] : 0u;
      __syncthreads();
      part[t] += u;
      __syncthreads();
    }
    if (i < ntiles) row[i] = carry + part[t] - v;
    carry += part[kSortThreads - 1];
    __syncthreads();
  }
  if (t == 0) tot[blockIdx.x] = carry;
}

// Exclusive scan of v[0 .. nbins) in LDS in place (nbins a power of two
// <= kSortMaxBins; each thread owns nbins / 256 consecutive entries, or one).
__device__ __forceinline__ void block_exclusive_scan(unsigned* v, int nbins, unsigned* part) {
  const int tid = threadIdx.x;
  const int per = nbins > kSortThreads ? nbins / kSortThreads : 1;
  const int b0 = tid * per;
  unsigned s = 0;
  if (b0 < nbins)
    for (int j = 0; j < per; ++j) s += v[b0 + j];
  part[tid] = s;
  __syncthreads();
  for (int off = 1; off < kSortThreads; off <<= 1) {
    const unsigned u = tid >= off ? part[tid - off] : 0u;
    __syncthreads();
    part[tid] += u;
    __syncthreads();
  }
  unsigned run = part[tid] - s;
  if (b0 < nbins)
    for (int j = 0; j < per; ++j) {
      const unsigned x = v[b0 + j];
      v[b0 + j] = run;
      run += x;
    }
  __syncthreads();
}

__global__ void __launch_bounds__(kSortThreads) k_sort_scatter(const unsigned* __restrict__ kin,
                                                               const unsigned long long* __restrict__ vin,
                                                               unsigned* __restrict__ kout,
                                                               unsigned long long* __restrict__ vout, int64_t n,
                                                               int shift, int bits, const unsigned* __restrict__ hist,
                                                               int ntiles, const unsigned* __restrict__ tot) {
  constexpr int NW = kSortThreads / 64;
  __shared__ unsigned base[kSortMaxBins];
  __shared__ unsigned part[kSortThreads];
  // wcnt[q][d] = (round + 1) << 24 | keys of digit d in wave q this round; other tags read as 0
  __shared__ unsigned wcnt[NW][kSortMaxBins];
  const int tid = threadIdx.x, tile = blockIdx.x, w = tid >> 6, lane = tid & 63, nbins = 1 << bits;
  const unsigned mask = (unsigned)nbins - 1u;
  // base[d] = keys of smaller digits (exclusive scan of the totals) + this digit in earlier tiles
  for (int d = tid; d < nbins; d += kSortThreads) {
    base[d] = tot[d];
#pragma unroll
    for (int q = 0; q < NW; ++q) wcnt[q][d] = 0;
  }
  __syncthreads();
  block_exclusive_scan(base, nbins, part);
  for (int d = tid; d < nbins; d += kSortThreads) base[d] += hist[(int64_t)d * ntiles + tile];
  const unsigned long long lt = (1ull << lane) - 1ull;
  const int64_t t0 = (int64_t)tile * kSortTile;
  for (int r = 0; r < kSortRounds; ++r) {
    const int64_t i = t0 + r * kSortThreads + tid;
    const bool ok = i < n;
    unsigned key = 0;
    unsigned long long val = 0;
    if (ok) {
      key = kin[i];
      val = vin[i];
    }
    const unsigned d = (key >> shift) & mask;
    // lanes of this wave holding a valid key with the same digit
    unsigned long long peers = __ballot(ok);
    for (int bit = 0; bit < bits; ++bit) {
      const bool set = (d >> bit) & 1u;
      const unsigned long long m = __ballot(set);
      peers &= set ? m : ~m;
    }
    const unsigned tag = (unsigned)(r + 1) << 24;
    const bool leader = ok && (peers & lt) == 0;  // the digit's lowest lane in this wave
    const unsigned cnt = (unsigned)__popcll(peers);
    if (leader) wcnt[w][d] = tag | cnt;
    __syncthreads();  // this round's counts (and the previous round's base update) visible
    if (ok) {
      unsigned pos = base[d] + (unsigned)__popcll(peers & lt);
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        const unsigned c = wcnt[q][d];
        if (q < w && (c & 0xFF000000u) == tag) pos += c & 0x00FFFFFFu;
      }
      kout[pos] = key;
      vout[pos] = val;
    }
    __syncthreads();  // every slot of this round computed from the old base
    if (leader) atomicAdd(&base[d], cnt);
  }
}

// Head positions of a sorted key list (the segment index of every entry):
// pos[i] = #{j <= i : key[j] != sentinel and (j == 0 or key[j-1] != key[j])}.
// Per 1024-entry tile (4 consecutive entries per thread): head counts, one
// scan over the tiles (k_sort_scan with one row), then in-tile prefix sums.
__device__ __forceinline__ void head_flags(const unsigned* __restrict__ keys, int64_t n, unsigned sentinel,
                                           int64_t i0, int* f) {
  unsigned prev = i0 > 0 && i0 - 1 < n ? keys[i0 - 1] : 0u;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int64_t i = i0 + e;
    const unsigned k = i < n ? keys[i] : sentinel;
    f[e] = (i < n && k != sentinel && (i == 0 || prev != k)) ? 1 : 0;
    prev = k;
  }
}

__global__ void __launch_bounds__(kSortThreads) k_head_count(const unsigned* __restrict__ keys, int64_t n,
                                                             unsigned sentinel, unsigned* __restrict__ cnt) {
  __shared__ unsigned red[kSortThreads / 64];
  const int t = threadIdx.x;
  int f[4];
  head_flags(keys, n, sentinel, (int64_t)blockIdx.x * kSortTile + 4 * t, f);
  unsigned c = f[0] + f[1] + f[2] + f[3];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
  if ((t & 63) == 0) red[t >> 6] = c;
  __syncthreads();
  if (t == 0) {
    unsigned sum = 0;
#pragma unroll
    for (int w = 0; w < kSortThreads / 64; ++w) sum += red[w];
    cnt[blockIdx.x] = sum;
  }
}

__global__ void __launch_bounds__(kSortThreads) k_head_pos(const unsigned* __restrict__ keys, int64_t n,
                                                           unsigned sentinel, const unsigned* __restrict__ off,
                                                           int* __restrict__ pos) {
  __shared__ unsigned part[kSortThreads];
  const int t = threadIdx.x;
  const int64_t i0 = (int64_t)blockIdx.x * kSortTile + 4 * t;
  int f[4];
  head_flags(keys, n, sentinel, i0, f);
  const unsigned c = f[0] + f[1] + f[2] + f[3];
  part[t] = c;
  __syncthreads();
  for (int o = 1; o < kSortThreads; o <<= 1) {
    const unsigned u = t >= o ? part[t - o] : 0u;
    __syncthreads();
    part[t] += u;
    __syncthreads();
  }
  unsigned run = off[blockIdx.x] + part[t] - c;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    run += f[e];
    if (i0 + e < n) pos[i0 + e] = (int)run;
  }
}

}  // namespace

// Workspace of head_positions: one count per tile + the total.
size_t head_positions_workspace(int64_t n) {
  return ((size_t)((n + kSortTile - 1) / kSortTile) + 1) * sizeof(unsigned);
}

int head_positions(const unsigned* keys, int64_t n, unsigned sentinel, int* pos, void* ws, hipStream_t s) {
  if (n <= 0) return GRK_OK;
  GRK_CHECK_ARG(n < ((int64_t)1 << 31), "too many keys");
  const int ntiles = (int)((n + kSortTile - 1) / kSortTile);
  unsigned* cnt = (unsigned*)ws;
  k_head_count<<<ntiles, kSortThreads, 0, s>>>(keys, n, sentinel, cnt);
  GRK_LAUNCH_CHECK();
  k_sort_scan<<<1, kSortThreads, 0, s>>>(cnt, ntiles, cnt + ntiles);
  GRK_LAUNCH_CHECK();
  k_head_pos<<<ntiles, kSortThreads, 0, s>>>(keys, n, sentinel, cnt, pos);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

// Workspace of sort_pairs: the digit histogram (digit-major) and the digit totals.
size_t sort_pairs_workspace(int64_t n) {
  const int64_t ntiles = (n + kSortTile - 1) / kSortTile;
  return ((size_t)kSortMaxBins * (size_t)(ntiles > 0 ? ntiles : 1) + kSortMaxBins) * sizeof(unsigned);
}

// The first pass's histogram buffer inside a sort_pairs workspace (a caller
// that counts digit 0 itself -- the low sort_digit_bits(end_bit) bits --
// writes hist[digit][tile] there, kSortTile keys per tile).
unsigned* sort_pairs_hist0(void* ws) { return (unsigned*)ws; }

// Sorts (k0, v0) by the low end_bit bits of the keys, stably, ping-ponging
// through (k1, v1); returns in *kres / *vres which pair of buffers holds the
// result.  end_bit <= 32.  hist0_ready: sort_pairs_hist0(ws) already holds the
// first digit's tile counts.
int sort_pairs(unsigned* k0, unsigned long long* v0, unsigned* k1, unsigned long long* v1, int64_t n, int end_bit,
               void* ws, unsigned** kres, unsigned long long** vres, hipStream_t s, bool hist0_ready) {
  *kres = k0;
  *vres = v0;
  if (n <= 0) return GRK_OK;
  GRK_CHECK_ARG(end_bit >= 1 && end_bit <= 32, "end_bit must be in [1, 32]");
  GRK_CHECK_ARG(n < ((int64_t)1 << 31), "too many keys");
  const int64_t ntiles64 = (n + kSortTile - 1) / kSortTile;
  GRK_CHECK_ARG(ntiles64 < (1 << 24), "too many tiles");
  const int ntiles = (int)ntiles64;
  const int bits = sort_digit_bits(end_bit), nbins = 1 << bits;
  unsigned* hist = (unsigned*)ws;
  unsigned* tot = hist + (size_t)kSortMaxBins * ntiles;
  unsigned* kin = k0;
  unsigned* kout = k1;
  unsigned long long* vin = v0;
  unsigned long long* vout = v1;
  int pass = 0;
  for (int shift = 0; shift < end_bit; shift += bits, ++pass) {
    if (pass > 0 || !hist0_ready) {
      k_sort_hist<<<ntiles, kSortThreads, 0, s>>>(kin, n, shift, bits, hist, ntiles);
      GRK_LAUNCH_CHECK();
    }
    k_sort_scan<<<nbins, kSortThreads, 0, s>>>(hist, ntiles, tot);
    GRK_LAUNCH_CHECK();
    k_sort_scatter<<<ntiles, kSortThreads, 0, s>>>(kin, vin, kout, vout, n, shift, bits, hist, ntiles, tot);
    GRK_LAUNCH_CHECK();
    unsigned* tk = kin;
    kin = kout;
    kout = tk;
    unsigned long long* tv = vin;
    vin = vout;
    vout = tv;
  }
  *kres = kin;
  *vres = vin;
  return GRK_OK;
}

}  // namespace grk

using namespace grk;

extern "C" size_t grk_sort_pairs_workspace(int64_t n) { return sort_pairs_workspace(n); }

extern "C" int grk_sort_pairs(const uint32_t* keys_in, const uint64_t* vals_in, uint32_t* keys_out, uint64_t* vals_out,
                              uint32_t* keys_tmp, uint64_t* vals_tmp, int64_t n, int end_bit, void* workspace,
                              size_t workspace_bytes, void* stream) {
  clear_error();
  GRK_CHECK_ARG(n >= 0, "n must be >= 0");
  if (n == 0) return GRK_OK;
  GRK_CHECK_ARG(keys_in && vals_in && keys_out && vals_out && keys_tmp && vals_tmp, "buffers are required");
  GRK_CHECK_ARG(workspace && workspace_bytes >= sort_pairs_workspace(n), "workspace smaller than grk_sort_pairs_workspace()");
  hipStream_t s = (hipStream_t)stream;
  // passes alternate out <-> tmp, starting from the caller's input: the pass
  // count's parity decides which buffer starts, so the result lands in out
  GRK_CHECK_ARG(end_bit >= 1 && end_bit <= 32, "end_bit must be in [1, 32]");
  const int bits = sort_digit_bits(end_bit);
  const int passes = (end_bit + bits - 1) / bits;
  unsigned* a = (unsigned*)(passes % 2 ? keys_tmp : keys_out);
  unsigned long long* va = (unsigned long long*)(passes % 2 ? vals_tmp : vals_out);
  unsigned* b = (unsigned*)(passes % 2 ? keys_out : keys_tmp);
  unsigned long long* vb = (unsigned long long*)(passes % 2 ? vals_out : vals_tmp);
  GRK_CHECK_HIP(hipMemcpyAsync(a, keys_in, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
  GRK_CHECK_HIP(hipMemcpyAsync(va, vals_in, (size_t)n * 8, hipMemcpyDeviceToDevice, s));
  unsigned* kr;
  unsigned long long* vr;
  return sort_pairs(a, va, b, vb, n, end_bit, workspace, &kr, &vr, s, false);
}
