// Whole-sequence causal attention for gfx950 (short sequences, the
// TencentGR regime: T <= 256 at head_dim 64).  Same math, operand
// conventions and outputs as the chunked kernels of grk_attention.hip
// (softmax MHA and HSTU), restructured for a
// latency-bound problem:
//
//  * one workgroup (4 waves) per (batch, head): the sequence's K/V (forward,
//    dQ) or Q/dO (dK/dV) are staged into LDS ONCE, from the first valid key
//    on (left padding is never loaded), behind a single barrier -- the
//    chunked kernels wait on a load + barrier per 64-row chunk;
//  * causal 32-row tiles are dealt to the waves in (j, n-1-j) pairs so every
//    wave gets the same number of 32x32 sub-tiles;
//  * the relative-position bias is staged as a clamped window rabx[d] so each
//    score reads it at a compile-time offset from one per-lane base;
//  * sub-tiles strictly below the diagonal and past the padding skip all
//    masking (contiguous key validity = the dataset's left padding; any
//    other key_valid pattern takes the per-key masked path);
//  * the precise (hi/lo probability) mode is a template parameter.
#include <stdlib.h>

#include <type_traits>

#include "grk_attention.h"

namespace grk {

constexpr int kSeqWaves = 4;

// Phase timestamps for scripts/microbench/attn_stamps.hip (compiled only there).
#ifdef GRK_ATTN_STAMPS
__device__ unsigned long long g_attn_stamps[1 << 16][8];
#define GRK_STAMP(k) \
  if ((threadIdx.x & 63) == 0) g_attn_stamps[(blockIdx.x * kSeqWaves + (threadIdx.x >> 6)) & 0xFFFF][k] = __builtin_amdgcn_s_memtime()
#else
#define GRK_STAMP(k)
#endif
// dK/dV phase timestamps (100 MHz s_memrealtime) for scripts/microbench/attn_dkdv_stamps.hip.
#ifdef GRK_DKDV_STAMPS
__device__ unsigned long long g_dkdv_rt[1 << 16][8];
#define GRK_RT(k) \
  if ((threadIdx.x & 63) == 0) g_dkdv_rt[(blockIdx.x * kSeqWaves + (threadIdx.x >> 6)) & 0xFFFF][k] = __builtin_amdgcn_s_memrealtime()
#else
#define GRK_RT(k)
#endif
constexpr int kRabPad = 32;             // rabx[kRabPad + d], d >= -31 inside a sub-tile
constexpr float kCausalBias = -1.0e30f;
constexpr int kDqBinArrays = 2;         // dQ kernel: drab bins as int64 fixed point (2 float slots each)
constexpr int kSeqLdsMax = 80 * 1024;   // LDS per workgroup: 2 per CU fit gfx950's 160 KiB

struct SeqInfo {
  int start;   // first valid key
  int contig;  // valid keys are exactly [start, T)
};

__device__ __forceinline__ SeqInfo seq_info(const AttnParams& p, int b, int T, int* sh) {
  if (p.seq_range)  // uniform scalar load; clamped so a bad range can never address outside [0, T)
    return {min(max(p.seq_range[3 * b], 0), T), p.seq_range[3 * b + 1] != 0};
  const uint8_t* kv = p.key_valid;
  if (!kv) return {0, 1};
  int first = T, cnt = 0;
  for (int j = threadIdx.x; j < T; j += blockDim.x)
    if (kv[(int64_t)b * T + j]) {
      first = min(first, j);
      ++cnt;
    }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    first = min(first, __shfl_xor(first, off));
    cnt += __shfl_xor(cnt, off);
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh[wave] = first;
    sh[kSeqWaves + wave] = cnt;
  }
  __syncthreads();
  int f = T, c = 0;
#pragma unroll
  for (int w = 0; w < kSeqWaves; ++w) {
    f = min(f, sh[w]);
    c += sh[kSeqWaves + w];
  }
  return {f, c == T - f};
}

// Sequence b of workgroup row bi: with precomputed ranges the workgroups take
// the sequences longest first (column 2: k_seq_order), so the long ones never
// start last and run alone at the end of the grid (lengths are ragged).
__device__ __forceinline__ int seq_of_block(const AttnParams& p, int bi) {
  if (!p.seq_range) return bi;
  const int b = p.seq_range[3 * bi + 2];
  return min(max(b, 0), p.B - 1);
}

// grk_seq_ranges: one wave per sequence.
__global__ void __launch_bounds__(256) k_seq_ranges(const uint8_t* __restrict__ kv, int B, int T,
                                                    int* __restrict__ out) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (b >= B) return;
  int first = T, cnt = 0;
  for (int j = lane; j < T; j += 64)
    if (kv[(int64_t)b * T + j]) {
      first = min(first, j);
      ++cnt;
    }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    first = min(first, __shfl_xor(first, off));
    cnt += __shfl_xor(cnt, off);
  }
  if (lane == 0) {
    out[3 * b] = first;
    out[3 * b + 1] = cnt == T - first;
  }
}

// out[3 i + 2] = the sequence with the i-th most keys from its first valid one
// (T - first descending, ties by index): a rank count, one workgroup.  The
// key counts are staged in LDS first when B <= kSeqOrderLds (read from memory
// in the rank loop they cost 84 us at B = 128, nearly all load latency).
constexpr int kSeqOrderLds = 8192;
__global__ void __launch_bounds__(1024) k_seq_order(int B, int T, int* __restrict__ out) {
  __shared__ int len[kSeqOrderLds];
  const bool lds = B <= kSeqOrderLds;
  if (lds)
    for (int b = threadIdx.x; b < B; b += blockDim.x) len[b] = T - out[3 * b];
  __syncthreads();
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const int lb = lds ? len[b] : T - out[3 * b];
    int rank = 0;
    for (int c = 0; c < B; ++c) {
      const int lc = lds ? len[c] : T - out[3 * c];
      rank += (lc > lb) | ((lc == lb) & (c < b));
    }
    out[3 * rank + 2] = b;
  }
}

// Both columns in ONE workgroup for B <= kSeqFused and B * T <= kSeqFusedBytes:
// the key-valid bytes are staged into LDS with 16-byte loads by every thread
// (the per-sequence byte scans then read LDS, not memory -- with byte loads
// from memory the workgroup ran 38 us at B = 128, T = 201), 16 waves scan the
// sequences, the key counts T - first go to LDS, and the rank count reads them
// there.  Same output as k_seq_ranges + k_seq_order, one launch instead of two.
constexpr int kSeqFused = 1024;
constexpr int kSeqFusedBytes = 48 * 1024;
// JAG: also the jagged layout's row bases (k_jagged_base of grk_jagged.hip, the
// same drop rule for spans past `cap`), from the counts already in LDS.
template <bool JAG>
__global__ void __launch_bounds__(1024) k_seq_ranges_order(const uint8_t* __restrict__ kv, int B, int T,
                                                           int* __restrict__ out, int64_t cap,
                                                           int64_t* __restrict__ row_base,
                                                           int64_t* __restrict__ n_rows, int32_t* __restrict__ err) {
  __shared__ int len[kSeqFused];
  __shared__ __attribute__((aligned(16))) uint8_t kvs[kSeqFusedBytes];
  const int n = B * T;
  if (((uintptr_t)kv & 15) == 0) {
    for (int i = threadIdx.x; i < n / 16; i += blockDim.x)
      reinterpret_cast<uint4*>(kvs)[i] = reinterpret_cast<const uint4*>(kv)[i];
    for (int i = n / 16 * 16 + threadIdx.x; i < n; i += blockDim.x) kvs[i] = kv[i];
  } else {
    for (int i = threadIdx.x; i < n; i += blockDim.x) kvs[i] = kv[i];
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int b = w; b < B; b += 16) {
    int first = T, cnt = 0;
    for (int j = lane; j < T; j += 64)
      if (kvs[b * T + j]) {
        first = min(first, j);
        ++cnt;
      }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      first = min(first, __shfl_xor(first, off));
      cnt += __shfl_xor(cnt, off);
    }
    if (lane == 0) {
      out[3 * b] = first;
      out[3 * b + 1] = cnt == T - first;
      len[b] = T - first;
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const int lb = len[b];
    int rank = 0;
    for (int c = 0; c < B; ++c) {
      const int lc = len[c];
      rank += (lc > lb) | ((lc == lb) & (c < b));
    }
    out[3 * rank + 2] = b;
  }
  if constexpr (JAG) {
    // inclusive scan of the spans (B * T <= kSeqFusedBytes: int32), then the row bases;
    // a span ending past cap is dropped (start T, row base -T, err bit 2) -- the kept
    // spans are a prefix, so n_rows <= cap
    __shared__ int part[kSeqFused];
    const int tid = threadIdx.x;
    const int span = tid < B ? len[tid] : 0;
    part[tid] = span;
    __syncthreads();
    for (int off = 1; off < kSeqFused; off <<= 1) {
      const int v = tid >= off ? part[tid - off] : 0;
      __syncthreads();
      part[tid] += v;
      __syncthreads();
    }
    const int incl = part[tid];
    bool drop = false;
    if (tid < B) {
      const int st = T - span;
      if (incl <= cap) {
        row_base[tid] = (int64_t)incl - span - st;
      } else {
        row_base[tid] = -(int64_t)T;
        out[3 * tid] = T;
        out[3 * tid + 1] = 1;
        drop = true;
      }
    }
    // kept = the largest inclusive sum <= cap: the last kept sequence's (a prefix)
    const bool last_kept = tid < B && !drop && (tid + 1 >= B || part[tid + 1] > cap);
    if (last_kept) *n_rows = incl;
    if (tid == 0 && (B == 0 || part[0] > cap)) *n_rows = 0;
    if (drop && err && (tid == 0 || part[tid - 1] <= cap)) atomicOr(err, 2);   // the first dropped one
  }
}

// KS 8-wide fragments of row `row` of a head slice (lane hh picks 8hh..8hh+7 of each 16)
// Row addressing: token (b, t) of a head slice is row rbase + t, rbase = b * T
// (padded [B*T] layout) or row_base[b] (jagged layout: only the rows
// [start_b, T) of each sequence exist, packed back to back -- AttnParams).
// Rows outside [lo, T) are never read (zero fragments) nor written.
template <int HD>
__device__ __forceinline__ void load_frag(bf16x8* f, const bf16_t* base, int64_t ld, int64_t rbase, int lo, int T,
                                          int h, int row, int hh) {
  const bool ok = row >= lo && row < T;
  const bf16_t* src = base + (ok ? rbase + row : 0) * ld + h * HD + 8 * hh;
#pragma unroll
  for (int ks = 0; ks < HD / 16; ++ks) f[ks] = gload8(src + 16 * ks, ok);
}

template <int HD>
__device__ __forceinline__ void load_frag_any(bf16x8* f, const void* base, int64_t ld, bool f32, int64_t rbase, int lo,
                                              int T, int h, int row, int hh) {
  const bool ok = row >= lo && row < T;
  const int64_t off = (ok ? rbase + row : 0) * ld + h * HD + 8 * hh;
#pragma unroll
  for (int ks = 0; ks < HD / 16; ++ks) f[ks] = gload8_any(base, off + 16 * ks, f32, ok);
}

template <int HD>
__device__ __forceinline__ void act_frag(bf16x8* f, bool act) {
  if (act)
#pragma unroll
    for (int ks = 0; ks < HD / 16; ++ks) f[ks] = silu8(f[ks]);
}

// LDS carve-up shared by the three kernels: two row images of Tp x HD,
// then per-row floats (rabx / lse / delta), key-valid bytes, scratch ints.
// NIMG = 4 (fp32-fidelity mode): img0lo / img1lo hold the bf16 residuals
// x - bf16(x) of the two staged operands.
template <int HD, int NIMG = 2>
struct SeqLds {
  char* img0;
  char* img1;
  char* img0lo;
  char* img1lo;
  float* f0;  // Tp + kRabPad floats
  float* f1;  // F1 x (Tp + kRabPad) floats (dQ: private drab bins per (wave, half-wave); dK/dV: delta)
  uint8_t* kvs;
  int* sh;
  // time bias: times relative to the first valid event, the head's table, dQ's fixed-point bins
  unsigned long long* tbins;
  int* tss;
  float* rtab;
  __device__ SeqLds(char* smem, int Tp, int F1 = 1) {
    img0 = smem;
    img1 = smem + Tp * HD * 2;
    img0lo = smem + 2 * Tp * HD * 2;
    img1lo = smem + 3 * Tp * HD * 2;
    f0 = reinterpret_cast<float*>(smem + NIMG * Tp * HD * 2);
    f1 = f0 + Tp + kRabPad;
    kvs = reinterpret_cast<uint8_t*>(f1 + F1 * (Tp + kRabPad));
    sh = reinterpret_cast<int*>(kvs + Tp);
    tbins = reinterpret_cast<unsigned long long*>(sh + 16);  // 8-byte aligned: Tp % 32 == 0
    tss = reinterpret_cast<int*>(tbins + kMaxTimeBuckets);
    rtab = reinterpret_cast<float*>(tss + Tp);
  }
  static size_t bytes(int Tp, int F1 = 1) {
    return (size_t)NIMG * Tp * HD * 2 + (size_t)((1 + F1) * (Tp + kRabPad)) * 4 + Tp + 16 * 4 +
           kMaxTimeBuckets * 8 + (size_t)Tp * 4 + kMaxTimeBuckets * 4;
  }
};

// Time-bias staging: tss[j] = ts[b, j] - ts[b, start] clamped to +-(2^30 - 1)
// (0 past T), the head's rab_t row, and (dQ) zeroed gradient bins.
__device__ __forceinline__ void stage_time(const AttnParams& p, int b, int h, int T, int Tp, int start, int* tss,
                                           float* rtab, unsigned long long* tbins) {
  const int64_t base = start < T ? p.ts[(int64_t)b * T + start] : 0;
  const int64_t lim = (1 << 30) - 1;
  for (int j = threadIdx.x; j < Tp; j += blockDim.x) {
    int64_t d = j < T ? p.ts[(int64_t)b * T + j] - base : 0;
    d = d > lim ? lim : (d < -lim ? -lim : d);
    tss[j] = (int)d;
  }
  for (int j = threadIdx.x; j < p.nbt; j += blockDim.x) {
    rtab[j] = p.rab_t[h * p.nbt + j];
    if (tbins) tbins[j] = 0ull;
  }
}

// Fidelity mode: fragments of row `row` split into bf16 hi + lo (SiLU applied in fp32 first when act).
template <int HD>
__device__ __forceinline__ void load_frag_split(bf16x8* fh, bf16x8* fl, const void* base, int64_t ld, int dt,
                                                bool act, int64_t rbase, int lo, int T, int h, int row, int hh) {
  const bool ok = row >= lo && row < T;
  const int64_t off = (ok ? rbase + row : 0) * ld + h * HD + 8 * hh;
#pragma unroll
  for (int ks = 0; ks < HD / 16; ++ks) {
    float f[8];
    gload8f(base, off + 16 * ks, dt, ok, f);
    if (act)
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = silu(f[j]);
    split8(f, fh[ks], fl[ks]);
  }
}

// Fidelity mode staging: rows [r0, Tp) of two head slices as hi and lo images.
template <int HD>
__device__ __forceinline__ void stage_pair_split(char* h0, char* l0, const void* src0, int64_t ld0, int dt0, bool act0,
                                                 char* h1, char* l1, const void* src1, int64_t ld1, int dt1,
                                                 bool act1, int64_t rbase, int lo, int T, int h, int r0, int Tp) {
  constexpr int NCH = HD / 8, BATCH = 4;
  const int nvec = (Tp - r0) * NCH;
  for (int base = threadIdx.x; base < nvec; base += BATCH * blockDim.x) {
    float v0[BATCH][8], v1[BATCH][8];
#pragma unroll
    for (int k = 0; k < BATCH; ++k) {
      const int u = base + k * blockDim.x;
      const int t = r0 + u / NCH, c = u % NCH;
      const bool ok = u < nvec && t < T && t >= lo;
      const int64_t row = ok ? rbase + t : 0;
      gload8f(src0, row * ld0 + h * HD + c * 8, dt0, ok, v0[k]);
      gload8f(src1, row * ld1 + h * HD + c * 8, dt1, ok, v1[k]);
    }
#pragma unroll
    for (int k = 0; k < BATCH; ++k) {
      const int u = base + k * blockDim.x;
      if (u < nvec) {
        const int row = r0 + u / NCH, c = u % NCH;
        if (act0)
#pragma unroll
          for (int j = 0; j < 8; ++j) v0[k][j] = silu(v0[k][j]);
        if (act1)
#pragma unroll
          for (int j = 0; j < 8; ++j) v1[k][j] = silu(v1[k][j]);
        bf16x8 a, al, bb, bl;
        split8(v0[k], a, al);
        split8(v1[k], bb, bl);
        const int o = lds_off<HD>(row, c * 8);
        *reinterpret_cast<uint4*>(h0 + o) = __builtin_bit_cast(uint4, a);
        *reinterpret_cast<uint4*>(l0 + o) = __builtin_bit_cast(uint4, al);
        *reinterpret_cast<uint4*>(h1 + o) = __builtin_bit_cast(uint4, bb);
        *reinterpret_cast<uint4*>(l1 + o) = __builtin_bit_cast(uint4, bl);
      }
    }
  }
}

// Stage rows [r0, Tp) of two [B*T, ld] head slices into the images at the
// same rows: every load of a batch is in flight before the first use (a
// load -> SiLU -> ds_write chain per element serialises on HBM latency).
template <int HD>
__device__ __forceinline__ void stage_pair(char* img0, const void* src0, int64_t ld0, bool f32_0, bool act0,
                                           char* img1, const void* src1, int64_t ld1, bool f32_1, bool act1,
                                           int64_t rbase, int lo, int T, int h, int r0, int Tp) {
  constexpr int NCH = HD / 8, BATCH = 8;
  const int nvec = (Tp - r0) * NCH;
  for (int base = threadIdx.x; base < nvec; base += BATCH * blockDim.x) {
    bf16x8 v0[BATCH], v1[BATCH];
#pragma unroll
    for (int k = 0; k < BATCH; ++k) {
      const int u = base + k * blockDim.x;
      const int t = r0 + u / NCH, c = u % NCH;
      const bool ok = u < nvec && t < T && t >= lo;
      const int64_t row = ok ? rbase + t : 0;
      v0[k] = gload8_any(src0, row * ld0 + h * HD + c * 8, f32_0, ok);
      v1[k] = gload8_any(src1, row * ld1 + h * HD + c * 8, f32_1, ok);
    }
#pragma unroll
    for (int k = 0; k < BATCH; ++k) {
      const int u = base + k * blockDim.x;
      if (u < nvec) {
        const int row = r0 + u / NCH, c = u % NCH;
        const bf16x8 a = act0 ? silu8(v0[k]) : v0[k];
        const bf16x8 bb = act1 ? silu8(v1[k]) : v1[k];
        *reinterpret_cast<uint4*>(img0 + lds_off<HD>(row, c * 8)) = __builtin_bit_cast(uint4, a);
        *reinterpret_cast<uint4*>(img1 + lds_off<HD>(row, c * 8)) = __builtin_bit_cast(uint4, bb);
      }
    }
  }
}

// rabx[kRabPad + d] = rab[h, min(d, nb - 1)] for d >= 0, kCausalBias for d < 0:
// a key after its query gets x = -1e30, SiLU(x) = dSiLU(x) = 0 exactly (the
// sigmoid underflows to 0, every product stays finite) -- the HSTU kernels'
// causal mask without a per-score select.
// Tp + kRabPad <= 2 * blockDim for every shape the seq kernels take.
struct RabRegs {
  float v[2];
};
__device__ __forceinline__ RabRegs load_rab(const AttnParams& p, int h, int Tp) {
  RabRegs r;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int j = threadIdx.x + k * blockDim.x;
    const int d = j - kRabPad;
    r.v[k] = d < 0 ? kCausalBias : (j >= Tp + kRabPad ? 0.f : p.rab[h * p.nb + min(d, p.nb - 1)]);
  }
  return r;
}
__device__ __forceinline__ void store_rab(float* rabx, const RabRegs& r, int Tp) {
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int j = threadIdx.x + k * blockDim.x;
    if (j < Tp + kRabPad) rabx[j] = r.v[k];
  }
}

__device__ __forceinline__ void stage_kvs(uint8_t* kvs, const uint8_t* kv, int b, int T, int Tp) {
  for (int j = threadIdx.x; j < Tp; j += blockDim.x) kvs[j] = j < T && (!kv || kv[(int64_t)b * T + j]);
}

// HSTU forward / dQ: kbias[key] = 0 for a valid key, kCausalBias for padding,
// invalid or past-T keys -- added to the score's pre-activation, it masks the
// key exactly like the rab window masks the future (no per-score select).
__device__ __forceinline__ void stage_key_bias(float* kbias, const uint8_t* kv, const SeqInfo& si, int b, int T,
                                               int Tp) {
  for (int j = threadIdx.x; j < Tp; j += blockDim.x) {
    const bool ok = j >= si.start && j < T && (si.contig || kv[(int64_t)b * T + j]);
    kbias[j] = ok ? 0.f : kCausalBias;
  }
}


// relative-position bias of the 16 scores of lane (r, hh) in the sub-tile of
// keys [kb, kb+32) for query myq: rabx[kRabPad + myq - key], key = kb + acc_row(i, hh)
__device__ __forceinline__ void rab16(const float* rabx, int myq, int kb, int hh, float* rb) {
  const float* base = rabx + kRabPad + (myq - kb - 4 * hh) - 27;
#pragma unroll
  for (int i = 0; i < 16; ++i) rb[i] = base[27 - ((i & 3) + 8 * (i >> 2))];
}

// Branch-free mask of the 16 scores of lane (r, hh) in a sub-tile: row index
// kb + acc_row(i, hh) valid iff in [lo, hi] (and kvs[row] != 0 when the key
// validity is not one contiguous run).  A 16-bit mask; each select is then one
// v_cndmask.  The contiguous case never touches LDS.
// acc_row(i, hh) = (i & 3) + 8 (i >> 2) + 4 hh increases with i, so the scores
// whose row lies in [lo, hi] are the contiguous index range [n_le(lo - 1), n_le(hi)).
__device__ __forceinline__ int n_le(int c, int hh) {  // #{i : acc_row(i, hh) <= c}
  const int d = c - 4 * hh;
  return d < 0 ? 0 : min(4 * (d >> 3) + min((d & 7) + 1, 4), 16);
}
__device__ __forceinline__ unsigned mask16_range(int kb, int hh, int lo, int hi) {
  const int a = n_le(lo - 1 - kb, hh), b = n_le(hi - kb, hh);
  return b > a ? ((0xFFFFu >> (16 - b)) & ~((1u << a) - 1u)) : 0u;
}
__device__ __forceinline__ unsigned mask16(int kb, int hh, int lo, int hi, bool contig, const uint8_t* kvs) {
  unsigned m = mask16_range(kb, hh, lo, hi);
  if (!contig) {
    unsigned v = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) v |= (unsigned)(kvs[kb + acc_row(i, hh)] != 0) << i;
    m &= v;
  }
  return m;
}

// Causal tiles are dealt in pairs {u, n-1-u} (work u+1 and n-u sub-tiles:
// n+1 per pair); wave w takes pairs w, w + kSeqWaves, ...

// Tile list of one wave: pairs {u, n-1-u} for u = wave, wave + kSeqWaves, ...
// The fragments of the wave's first tile are loaded in the prologue, beside
// the staging loads, so no tile starts with a global round trip.
__device__ __forceinline__ int pair_tile(int u, int ps, int n) { return ps == 0 ? u : n - 1 - u; }
__device__ __forceinline__ bool pair_has(int u, int ps, int n) { return ps == 0 || n - 1 - u != u; }

// Jagged layout: the dead capacity rows [n, cap) past the spans hold no token,
// but the row-wise ops and weight gradients around the attention read every
// row of its outputs, so each launch zeroes them there: workgroup w clears its
// share of the tail (8-byte stores), beside its real work.
__device__ __forceinline__ void zero_tail_rows(const AttnParams& p, void* out, int64_t ld, int hd) {
  if (!p.row_base || !out) return;
  const int64_t n = p.jag_n[0];
  const int per = p.out_f32 ? 2 : 4;            // elements per 8-byte store
  const int64_t upr = (int64_t)p.H * hd / per;  // stores per row
  const int64_t units = (p.jag_cap - n) * upr;
  if (units <= 0) return;
  const int64_t chunk = (units + gridDim.x - 1) / gridDim.x;
  const int64_t u0 = (int64_t)blockIdx.x * chunk, u1 = min(units, u0 + chunk);
  for (int64_t u = u0 + threadIdx.x; u < u1; u += blockDim.x) {
    const int64_t r = n + u / upr, c = (u % upr) * per;
    void* dst = p.out_f32 ? (void*)((float*)out + r * ld + c) : (void*)((bf16_t*)out + r * ld + c);
    *reinterpret_cast<uint2*>(dst) = make_uint2(0u, 0u);
  }
}

// ================================================================ forward ====
template <int HD, int KIND, int PREC>
__global__ void __launch_bounds__(64 * kSeqWaves) k_attn_fwd_seq(AttnParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int KS = HD / 16, NDT = (HD + 31) / 32;
  const int T = p.T, nq = (T + 31) / 32, Tp = nq * 32;
  SeqLds<HD, PREC == 2 ? 4 : 2> L(smem, Tp);
  GRK_STAMP(0);
  const int b = seq_of_block(p, blockIdx.x / p.H), h = blockIdx.x % p.H;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const SeqInfo si = seq_info(p, b, T, L.sh);
  const int start = si.start, first = start / 32, kbeg = first * 32;
  const int ntiles = nq - first, npairs = (ntiles + 1) / 2;
  const int64_t rbase = p.row_base ? p.row_base[b] : (int64_t)b * T;
  const int lo = p.row_base ? start : 0;  // jagged rows: only [start, T) exist
  zero_tail_rows(p, p.out, p.ldo, HD);
  GRK_STAMP(1);
  // prologue: every independent load in flight before the first wait
  bf16x8 qpre[KS];
  if (PREC < 2 && wave < npairs) load_frag<HD>(qpre, p.q, p.ldq, rbase, lo, T, h, (first + wave) * 32 + r, hh);
  RabRegs rr;
  if (KIND == 1) rr = load_rab(p, h, Tp);
  if constexpr (PREC == 2)
    stage_pair_split<HD>(L.img0, L.img0lo, p.k, p.ldk, p.in_dt, p.act, L.img1, L.img1lo, p.v, p.ldv, p.in_dt, p.act,
                         rbase, lo, T, h, kbeg, Tp);
  else
    stage_pair<HD>(L.img0, p.k, p.ldk, false, p.act, L.img1, p.v, p.ldv, false, p.act, rbase, lo, T, h, kbeg, Tp);
  if (KIND == 1) {
    store_rab(L.f0, rr, Tp);
    stage_key_bias(L.f1, p.key_valid, si, b, T, Tp);
    if (p.nbt) stage_time(p, b, h, T, Tp, start, L.tss, L.rtab, nullptr);
  }
  if (!si.contig) stage_kvs(L.kvs, p.key_valid, b, T, Tp);
  GRK_STAMP(2);
  __syncthreads();
  GRK_STAMP(3);

  const float sl2 = p.scale * kLog2e;
  const float rdrop = 1.0f / (1.0f - p.dropout_p);
  const bool drop = KIND == 0 && p.dropout_p > 0.f;
  const unsigned long long seed = drop ? attn_seed(p) : 0ull;
  const int bh = b * p.H + h;

  // query tiles before the first valid key: every row fully masked -> 0
  for (int qt = wave; qt < first; qt += kSeqWaves) {
    const int myq = qt * 32 + r;
    f32x16 z[NDT];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) z[dt] = f32x16{};
    if (KIND == 0 && hh == 0 && myq < T && p.lse) p.lse[(int64_t)bh * T + myq] = -INFINITY;
    store_rows<HD, NDT>(p.out, p.ldo, p.out_f32, rbase + myq, h, hh, z, 0.f, myq < T && myq >= lo);
  }

  for (int pu = wave; pu < npairs; pu += kSeqWaves)
#pragma unroll
    for (int ps = 0; ps < 2; ++ps) {
      if (!pair_has(pu, ps, ntiles)) break;
      const int q0 = (first + pair_tile(pu, ps, ntiles)) * 32, myq = q0 + r;
      const bool qok = myq < T;
      bf16x8 qf[KS], ql[KS];
      if constexpr (PREC == 2) {
        load_frag_split<HD>(qf, ql, p.q, p.ldq, p.in_dt, p.act, rbase, lo, T, h, myq, hh);
      } else {
        if (pu == wave && ps == 0) {
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) qf[ks] = qpre[ks];
        } else {
          load_frag<HD>(qf, p.q, p.ldq, rbase, lo, T, h, myq, hh);
        }
        act_frag<HD>(qf, p.act);
      }
      f32x16 o[NDT];
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) o[dt] = f32x16{};
      float m = -INFINITY, l = 0.f;
      for (int kb = kbeg; kb <= q0; kb += 32) {
        f32x16 s = acc_zero();
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const bf16x8 ka = lds_row8<HD>(L.img0, kb + r, 16 * ks + 8 * hh);
          s = mfma(ka, qf[ks], s);
          if constexpr (PREC == 2) {
            s = mfma(ka, ql[ks], s);
            s = mfma(lds_row8<HD>(L.img0lo, kb + r, 16 * ks + 8 * hh), qf[ks], s);
          }
        }
        // strictly below the diagonal and past the padding: nothing to mask
        const bool fast = si.contig && kb < q0 && kb >= start;
        float pd[16];
        if (KIND == 0) {
          float x[16], tmax = -INFINITY;
#pragma unroll
          for (int i = 0; i < 16; ++i) x[i] = s[i] * sl2;
          if (!fast) {
            const unsigned mk = qok ? mask16(kb, hh, start, myq, si.contig, L.kvs) : 0u;
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] = ((mk >> i) & 1) ? x[i] : -INFINITY;
          }
#pragma unroll
          for (int i = 0; i < 16; ++i) tmax = fmaxf(tmax, x[i]);
          tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
          const float mn = fmaxf(m, tmax);
          const float alpha = (mn == -INFINITY) ? 1.f : exp2f(m - mn);
          const float mref = (mn == -INFINITY) ? 0.f : mn;  // exp2(-inf - 0) = 0 for masked scores
          float rs = 0.f;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            pd[i] = exp2f(x[i] - mref);
            rs += pd[i];
          }
          rs += __shfl_xor(rs, 32);
          l = l * alpha + rs;
          m = mn;
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt) o[dt] *= alpha;
          if (drop) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int key = kb + acc_row(i, hh);
              pd[i] = drop_keep(seed, bh, myq, key, T, p.dropout_p) ? pd[i] * rdrop : 0.f;
            }
          }
        } else {
          // causal mask in the rab window, key mask in kbias: no select
          float rb[16];
          rab16(L.f0, myq, kb, hh, rb);
          const float* kbb = L.f1 + kb + 4 * hh;
          if (p.nbt) {  // time bias: rab_t[h, bucket(t_q - t_k)]
            const int tq = L.tss[myq < Tp ? myq : Tp - 1];
#pragma unroll
            for (int i = 0; i < 16; ++i) rb[i] += L.rtab[time_bucket(tq - L.tss[kb + acc_row(i, hh)], p.nbt)];
          }
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const float x = fmaf(s[i], p.scale, rb[i]) + kbb[(i & 3) + 8 * (i >> 2)];
            pd[i] = x * sigmoid_fast(x);
          }
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          bf16x8 ph, pl;
          pack_acc(pd, s2, ph, pl);
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt) {
            const bf16x8 vf = lds_tr8<HD>(L.img1, kb + 16 * s2, dt * 32, lane);
            o[dt] = mfma(vf, ph, o[dt]);
            if (PREC) o[dt] = mfma(vf, pl, o[dt]);
            if constexpr (PREC == 2) o[dt] = mfma(lds_tr8<HD>(L.img1lo, kb + 16 * s2, dt * 32, lane), ph, o[dt]);
          }
        }
      }
      float mul = p.inv_n;
      if (KIND == 0) {
        mul = l > 0.f ? 1.0f / l : 0.f;
        if (hh == 0 && qok && p.lse) p.lse[(int64_t)bh * T + myq] = l > 0.f ? (m + log2f(l)) * kLn2 : -INFINITY;
      }
      store_rows<HD, NDT>(p.out, p.ldo, p.out_f32, rbase + myq, h, hh, o, mul, qok && myq >= lo);
      GRK_STAMP(4 + ps);
    }
  GRK_STAMP(6);
}

// ================================================================ dQ =========
template <int HD, int KIND, int PREC>
__global__ void __launch_bounds__(64 * kSeqWaves) k_attn_dq_seq(AttnParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int KS = HD / 16, NDT = (HD + 31) / 32;
  const int T = p.T, nq = (T + 31) / 32, Tp = nq * 32;
  SeqLds<HD, PREC == 2 ? 4 : 2> L(smem, Tp, kDqBinArrays + 1);
  // drab by distance d in [-kRabPad, Tp): bins[kRabPad + d], int64 fixed point
  unsigned long long* bins = reinterpret_cast<unsigned long long*>(L.f1);
  float* kbias = L.f1 + kDqBinArrays * (Tp + kRabPad);
  const int b = seq_of_block(p, blockIdx.x / p.H), h = blockIdx.x % p.H;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const SeqInfo si = seq_info(p, b, T, L.sh);
  const int start = si.start, first = start / 32, kbeg = first * 32;
  const int ntiles = nq - first, npairs = (ntiles + 1) / 2;
  const int bh = b * p.H + h;
  const int64_t rbase = p.row_base ? p.row_base[b] : (int64_t)b * T;
  const int lo = p.row_base ? start : 0;  // jagged rows: only [start, T) exist
  zero_tail_rows(p, p.dq, p.lddq, HD);
  bf16x8 qpre[KS], dpre[KS];
  if (PREC < 2 && wave < npairs) {
    const int row = (first + wave) * 32 + r;
    load_frag<HD>(qpre, p.q, p.ldq, rbase, lo, T, h, row, hh);
    load_frag_any<HD>(dpre, p.dout, p.lddo, p.dout_f32, rbase, lo, T, h, row, hh);
  }
  RabRegs rr;
  if (KIND == 1) rr = load_rab(p, h, Tp);
  if constexpr (PREC == 2)
    stage_pair_split<HD>(L.img0, L.img0lo, p.k, p.ldk, p.in_dt, p.act, L.img1, L.img1lo, p.v, p.ldv, p.in_dt, p.act,
                         rbase, lo, T, h, kbeg, Tp);
  else
    stage_pair<HD>(L.img0, p.k, p.ldk, false, p.act, L.img1, p.v, p.ldv, false, p.act, rbase, lo, T, h, kbeg, Tp);
  if (KIND == 1) {
    store_rab(L.f0, rr, Tp);
    for (int j = threadIdx.x; j < Tp + kRabPad; j += blockDim.x) bins[j] = 0ull;
    stage_key_bias(kbias, p.key_valid, si, b, T, Tp);
    if (p.nbt) stage_time(p, b, h, T, Tp, start, L.tss, L.rtab, L.tbins);
  }
  if (!si.contig) stage_kvs(L.kvs, p.key_valid, b, T, Tp);
  __syncthreads();

  const float sl2 = p.scale * kLog2e;
  const float rdrop = 1.0f / (1.0f - p.dropout_p);
  const bool drop = KIND == 0 && p.dropout_p > 0.f;
  const unsigned long long seed = drop ? attn_seed(p) : 0ull;

  for (int qt = wave; qt < first; qt += kSeqWaves) {  // fully masked query rows: dq = 0
    const int myq = qt * 32 + r;
    f32x16 z[NDT];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) z[dt] = f32x16{};
    store_rows<HD, NDT>(p.dq, p.lddq, p.out_f32, rbase + myq, h, hh, z, 0.f, myq < T && myq >= lo);
  }

  for (int pu = wave; pu < npairs; pu += kSeqWaves)
#pragma unroll
    for (int ps = 0; ps < 2; ++ps) {
      if (!pair_has(pu, ps, ntiles)) break;
      const int q0 = (first + pair_tile(pu, ps, ntiles)) * 32, myq = q0 + r;
      const bool qok = myq < T;
      bf16x8 qf[KS], dof[KS], ql[KS], dol[KS];
      if constexpr (PREC == 2) {
        load_frag_split<HD>(qf, ql, p.q, p.ldq, p.in_dt, p.act, rbase, lo, T, h, myq, hh);
        load_frag_split<HD>(dof, dol, p.dout, p.lddo, p.dout_f32 ? 0 : 1, false, rbase, lo, T, h, myq, hh);
      } else {
        if (pu == wave && ps == 0) {
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            qf[ks] = qpre[ks];
            dof[ks] = dpre[ks];
          }
        } else {
          load_frag<HD>(qf, p.q, p.ldq, rbase, lo, T, h, myq, hh);
          load_frag_any<HD>(dof, p.dout, p.lddo, p.dout_f32, rbase, lo, T, h, myq, hh);
        }
        act_frag<HD>(qf, p.act);
      }
      float lse2 = 0.f, dlt = 0.f;
      if (KIND == 0 && qok) {
        lse2 = p.lse[(int64_t)bh * T + myq] * kLog2e;
        dlt = p.delta[(int64_t)bh * T + myq];
      }
      const bool row_live = KIND == 1 || lse2 != -INFINITY;
      f32x16 acc[NDT];
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) acc[dt] = f32x16{};
      for (int kb = kbeg; kb <= q0; kb += 32) {
        f32x16 s = acc_zero(), dp = acc_zero();
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const bf16x8 ka = lds_row8<HD>(L.img0, kb + r, 16 * ks + 8 * hh);
          const bf16x8 va = lds_row8<HD>(L.img1, kb + r, 16 * ks + 8 * hh);
          s = mfma(ka, qf[ks], s);
          dp = mfma(va, dof[ks], dp);
          if constexpr (PREC == 2) {
            s = mfma(ka, ql[ks], s);
            s = mfma(lds_row8<HD>(L.img0lo, kb + r, 16 * ks + 8 * hh), qf[ks], s);
            dp = mfma(va, dol[ks], dp);
            dp = mfma(lds_row8<HD>(L.img1lo, kb + r, 16 * ks + 8 * hh), dof[ks], dp);
          }
        }
        const bool fast = si.contig && kb < q0 && kb >= start;
        float ds[16];
        const unsigned mk = (KIND == 1 || fast) ? 0xFFFFu
                                                : ((qok && row_live) ? mask16(kb, hh, start, myq, si.contig, L.kvs) : 0u);
        if (KIND == 0) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const float pv = ((mk >> i) & 1) ? exp2f(s[i] * sl2 - lse2) : 0.f;
            float dpv = dp[i];
            if (drop) dpv = drop_keep(seed, bh, myq, kb + acc_row(i, hh), T, p.dropout_p) ? dpv * rdrop : 0.f;
            ds[i] = pv * (dpv - dlt);
          }
        } else {
          // causal mask in the rab window, key mask in kbias: no select
          float rb[16];
          rab16(L.f0, myq, kb, hh, rb);
          const float* kbb = kbias + kb + 4 * hh;
          int tb[16];
          if (p.nbt) {  // time bias: rab_t[h, bucket(t_q - t_k)]
            const int tq = L.tss[myq < Tp ? myq : Tp - 1];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              tb[i] = time_bucket(tq - L.tss[kb + acc_row(i, hh)], p.nbt);
              rb[i] += L.rtab[tb[i]];
            }
          }
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const float x = fmaf(s[i], p.scale, rb[i]) + kbb[(i & 3) + 8 * (i >> 2)];
            const float sg = sigmoid_fast(x), sgn = sg * p.inv_n;
            ds[i] = dp[i] * fmaf(fmaf(-x, sg, x), sgn, sgn);  // dp * dSiLU(x) / n
          }
          if (p.drab_t) {  // fixed-point bins per bucket (masked scores have ds == 0 exactly)
#pragma unroll
            for (int i = 0; i < 16; ++i)
              if (ds[i] != 0.f) atomicAdd(&L.tbins[tb[i]], to_fix(ds[i]));
          }
          if (p.drab) {
            // drab bins by distance d = query - key.  The sub-tile's 1024 scores lie on
            // 63 diagonals: lane r of each half gathers score (key k, query (r + k) & 31)
            // of each of its 16 keys (one ds_bpermute each), whose distance is
            // q0 - kb + r (no wrap) or q0 - kb + r - 32 (wrap); the halves are added
            // and one lane per distance adds the two sums -- 2 LDS atomics per lane
            // of the first half instead of 16 per lane.  Fixed order: deterministic.
            float dhi = 0.f, dlo = 0.f;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int k = acc_row(i, hh);
              const float v = __shfl(ds[i], ((r + k) & 31) | (hh << 5));
              if (r + k < 32) dhi += v;
              else dlo += v;
            }
            dhi += __shfl_xor(dhi, 32);
            dlo += __shfl_xor(dlo, 32);
            if (hh == 0) {
              unsigned long long* bd = bins + kRabPad + (q0 - kb) + r;
              if (dhi != 0.f) atomicAdd(bd, to_fix(dhi));
              if (dlo != 0.f) atomicAdd(bd - 32, to_fix(dlo));
            }
          }
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          bf16x8 dh, dl;
          pack_acc(ds, s2, dh, dl);
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt) {
            const bf16x8 kf = lds_tr8<HD>(L.img0, kb + 16 * s2, dt * 32, lane);
            acc[dt] = mfma(kf, dh, acc[dt]);
            if (PREC) acc[dt] = mfma(kf, dl, acc[dt]);
            if constexpr (PREC == 2) acc[dt] = mfma(lds_tr8<HD>(L.img0lo, kb + 16 * s2, dt * 32, lane), dh, acc[dt]);
          }
        }
      }
      store_rows<HD, NDT>(p.dq, p.lddq, p.out_f32, rbase + myq, h, hh, acc, p.scale, qok && myq >= lo,
                          p.act ? p.q : nullptr, p.ldq, p.in_dt);
    }
  if (KIND == 1 && (p.drab || p.drab_t)) {
    __syncthreads();
    // returning atomics (their old values are folded into chk): once chk is computed,
    // this thread's adds are performed -- the order the last-workgroup finalize needs,
    // without __threadfence (an agent-scope fence writes back / invalidates the XCD's
    // L2 on gfx950: with one per workgroup, dq ran 61 -> 185 us)
    unsigned long long chk = 0ull;
    if (p.drab)
      for (int d = threadIdx.x; d < Tp; d += blockDim.x) {
        const unsigned long long q = bins[kRabPad + d];
        if (q != 0) chk ^= atomicAdd(&p.drab_fix[h * p.nb + min(d, p.nb - 1)], q);
      }
    if (p.drab_t)
      for (int j = threadIdx.x; j < p.nbt; j += blockDim.x)
        if (L.tbins[j] != 0ull) chk ^= atomicAdd(&p.drab_t_fix[h * p.nbt + j], L.tbins[j]);
    if (p.fin_count) {
      // the last workgroup to finish finalizes drab / drab_t and leaves the bins and the
      // counter zero (GRK_ATTN_BWD_WS_CLEAN): no reset and no finalize launch per call.
      // The flag lives in the bins' LDS, read out above.
      int* last = reinterpret_cast<int*>(bins);
      __syncthreads();
      if (chk == 0x9E3779B97F4A7C15ull) last[1] = 1;   // keeps chk (and the wait on the adds) alive
      if (threadIdx.x == 0) *last = atomicAdd(p.fin_count, 1u) == gridDim.x - 1;
      __syncthreads();
      if (*last) {
        if (p.drab)
          for (int i = threadIdx.x; i < p.H * p.nb; i += blockDim.x)
            drab_finalize_elem(p.drab, p.drab_fix, i, p.drab_set);
        if (p.drab_t)
          for (int i = threadIdx.x; i < p.H * p.nbt; i += blockDim.x)
            drab_finalize_elem(p.drab_t, p.drab_t_fix, i, p.drab_set);
        if (threadIdx.x == 0) atomicExch(p.fin_count, 0u);
      }
    }
  }
}

// ============================================================== dK / dV =====
// A/B build constants (scripts/build_variant.sh; both 0 in the product build):
//   GRK_ATTN_FOLD_INVN  HSTU dK/dV: P and dS without the 1/n factor, folded into
//                       the dK / dV store scales instead (one VALU per score);
//   GRK_ATTN_TB_SPLIT   HSTU dK/dV without the time bias instantiated apart
//                       (TBK = false: no per-score add of a zero bias).
#ifndef GRK_ATTN_FOLD_INVN
#define GRK_ATTN_FOLD_INVN 0
#endif
#ifndef GRK_ATTN_TB_SPLIT
#define GRK_ATTN_TB_SPLIT 0
#endif
//   GRK_DKDV_WAVES      dK/dV (hd <= 64, PREC < 2): the waves-per-SIMD register target
//   GRK_DKDV_PREFETCH   dK/dV: the first key tile's K / V fragments loaded before the
//                       Q / dO staging (1) or at the tile (0, product since round 5:
//                       218 VGPRs instead of 251, dK/dV 65-67 vs 67-70 us, step 4.03
//                       vs 4.03-4.14 ms over three same-box pairs, gpurun_out/r5v)
#ifndef GRK_DKDV_PREFETCH
#define GRK_DKDV_PREFETCH 0
#endif

template <int HD, int KIND, int PREC, bool TBK = true>
#ifndef GRK_DKDV_WAVES
#define GRK_DKDV_WAVES 2
#endif
__global__ void __launch_bounds__(64 * kSeqWaves)
__attribute__((amdgpu_waves_per_eu(PREC < 2 && HD <= 64 ? GRK_DKDV_WAVES : 1)))
k_attn_dkdv_seq(AttnParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int KS = HD / 16, NDT = (HD + 31) / 32;
  const int T = p.T, nq = (T + 31) / 32, Tp = nq * 32;
  SeqLds<HD, PREC == 2 ? 4 : 2> L(smem, Tp);
  float* lses = L.f0;  // softmax: per-query log2-domain lse, delta
  float* dlts = L.f1;
  const int b = seq_of_block(p, blockIdx.x / p.H), h = blockIdx.x % p.H;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const SeqInfo si = seq_info(p, b, T, L.sh);
  const int start = si.start, first = start / 32, kbeg = first * 32;
  const int ntiles = nq - first, npairs = (ntiles + 1) / 2;
  const int bh = b * p.H + h;
  const int64_t rbase = p.row_base ? p.row_base[b] : (int64_t)b * T;
  const int lo = p.row_base ? start : 0;  // jagged rows: only [start, T) exist
  GRK_RT(0);
  zero_tail_rows(p, p.dk, p.lddk, HD);
  zero_tail_rows(p, p.dv, p.lddv, HD);
  // key tile j (absolute first + j) visits query tiles j .. ntiles-1
  bf16x8 kpre[KS], vpre[KS];
  if (GRK_DKDV_PREFETCH && PREC < 2 && wave < npairs) {
    const int row = (first + wave) * 32 + r;
    load_frag<HD>(kpre, p.k, p.ldk, rbase, lo, T, h, row, hh);
    load_frag<HD>(vpre, p.v, p.ldv, rbase, lo, T, h, row, hh);
  }
  RabRegs rr;
  float lv[2], dl[2];
  if (KIND == 1) {
    rr = load_rab(p, h, Tp);
  } else {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      // fully masked query rows (lse = -inf) and rows past T are staged as 0:
      // every (query, key) pair they form with a valid key is masked or has dO = 0
      const int j = threadIdx.x + k * blockDim.x;
      lv[k] = 0.f;
      dl[k] = 0.f;
      if (j < T) {
        const float l = p.lse[(int64_t)bh * T + j];
        lv[k] = l == -INFINITY ? 0.f : l * kLog2e;
        dl[k] = p.delta[(int64_t)bh * T + j];
      }
    }
  }
  if constexpr (PREC == 2)
    stage_pair_split<HD>(L.img0, L.img0lo, p.q, p.ldq, p.in_dt, p.act, L.img1, L.img1lo, p.dout, p.lddo,
                         p.dout_f32 ? 0 : 1, false, rbase, lo, T, h, kbeg, Tp);
  else
    stage_pair<HD>(L.img0, p.q, p.ldq, false, p.act, L.img1, p.dout, p.lddo, p.dout_f32, false, rbase, lo, T, h, kbeg, Tp);
  if (KIND == 1) {
    store_rab(L.f0, rr, Tp);
    if (p.nbt) stage_time(p, b, h, T, Tp, start, L.tss, L.rtab, nullptr);
  } else {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int j = threadIdx.x + k * blockDim.x;
      if (j < Tp) {
        lses[j] = lv[k];
        dlts[j] = dl[k];
      }
    }
  }
  if (!si.contig) stage_kvs(L.kvs, p.key_valid, b, T, Tp);
  GRK_RT(1);
  __syncthreads();
  GRK_RT(2);

  const float sl2 = p.scale * kLog2e;
  const float rdrop = 1.0f / (1.0f - p.dropout_p);
  const bool drop = KIND == 0 && p.dropout_p > 0.f;
  const unsigned long long seed = drop ? attn_seed(p) : 0ull;
  constexpr bool fold = GRK_ATTN_FOLD_INVN && KIND == 1;
  const float pscale = fold ? p.inv_n : 1.f;  // the 1/n factor of P and dS (HSTU)
  const float sn = fold ? 1.f : p.inv_n;
#ifdef GRK_DKDV_STAMPS
  int ntile_done = 0;
#endif

  for (int kt = wave; kt < first; kt += kSeqWaves) {  // keys before the first valid one: no gradient
    const int myk = kt * 32 + r;
    f32x16 z[NDT];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) z[dt] = f32x16{};
    store_rows<HD, NDT>(p.dk, p.lddk, p.out_f32, rbase + myk, h, hh, z, 0.f, myk < T && myk >= lo);
    store_rows<HD, NDT>(p.dv, p.lddv, p.out_f32, rbase + myk, h, hh, z, 0.f, myk < T && myk >= lo);
  }

  for (int pu = wave; pu < npairs; pu += kSeqWaves)
#pragma unroll
    for (int ps = 0; ps < 2; ++ps) {
      if (!pair_has(pu, ps, ntiles)) break;
      const int k0 = (first + pair_tile(pu, ps, ntiles)) * 32, myk = k0 + r;
      const bool kin = myk < T;
      const bool kok = kin && myk >= start && (si.contig || L.kvs[myk]);
      bf16x8 kf[KS], vf[KS], kl[KS], vl[KS];
      if constexpr (PREC == 2) {
        load_frag_split<HD>(kf, kl, p.k, p.ldk, p.in_dt, p.act, rbase, lo, T, h, myk, hh);
        load_frag_split<HD>(vf, vl, p.v, p.ldv, p.in_dt, p.act, rbase, lo, T, h, myk, hh);
      } else {
        if (GRK_DKDV_PREFETCH && pu == wave && ps == 0) {
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            kf[ks] = kpre[ks];
            vf[ks] = vpre[ks];
          }
        } else {
          load_frag<HD>(kf, p.k, p.ldk, rbase, lo, T, h, myk, hh);
          load_frag<HD>(vf, p.v, p.ldv, rbase, lo, T, h, myk, hh);
        }
        act_frag<HD>(kf, p.act);
        act_frag<HD>(vf, p.act);
      }
      if (!kok) {  // padding / invalid key: S = dP = 0 keep every product finite; stored as 0
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          kf[ks] = vf[ks] = kl[ks] = vl[ks] = __builtin_bit_cast(bf16x8, make_uint4(0, 0, 0, 0));
        }
      }
      f32x16 dk[NDT], dv[NDT];
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        dk[dt] = acc_zero();
        dv[dt] = acc_zero();
      }
      for (int qb = k0; qb < Tp; qb += 32) {
        f32x16 s = acc_zero(), dp = acc_zero();
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const bf16x8 qa = lds_row8<HD>(L.img0, qb + r, 16 * ks + 8 * hh);
          const bf16x8 da = lds_row8<HD>(L.img1, qb + r, 16 * ks + 8 * hh);
          s = mfma(qa, kf[ks], s);
          dp = mfma(da, vf[ks], dp);
          if constexpr (PREC == 2) {
            s = mfma(qa, kl[ks], s);
            s = mfma(lds_row8<HD>(L.img0lo, qb + r, 16 * ks + 8 * hh), kf[ks], s);
            dp = mfma(da, vl[ks], dp);
            dp = mfma(lds_row8<HD>(L.img1lo, qb + r, 16 * ks + 8 * hh), vf[ks], dp);
          }
        }
        // Invalid keys have zeroed fragments and are stored as 0; queries past T
        // have zero Q / dO rows (their terms vanish) and a finite staged lse.
        // HSTU: the causal mask is in the rab window (kCausalBias), so no score
        // is selected; softmax: only the diagonal tile (or a non-contiguous
        // key set) is masked.
        const bool fast = si.contig && qb != k0;
        const unsigned mk = fast ? 0xFFFFu : (kok ? mask16_range(qb, hh, myk, T - 1) : 0u);
        // Per half tile (elements 8 s2 .. 8 s2 + 7): P and dS as bf16 hi / lo words,
        // then that half's dV / dK MFMAs (the second half's VALU overlaps the first
        // half's MFMAs).  Instantiated unmasked and masked behind one wave-uniform branch.
        auto half = [&](auto masked, int s2) {
        uint32_t pw[4], plw[4], dw[4], dlw[4];
        if (KIND == 0) {
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const int j = 4 * s2 + jj;
            float pd2[2], ds2[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              const int i = 2 * j + u, q = qb + acc_row(i, hh);
              const float pv = __builtin_amdgcn_exp2f(fmaf(s[i], sl2, -lses[q]));
              float dpv = dp[i];
              pd2[u] = pv;
              if (drop) {
                const bool keep = drop_keep(seed, bh, q, myk, T, p.dropout_p);
                pd2[u] = keep ? pv * rdrop : 0.f;
                dpv = keep ? dpv * rdrop : 0.f;
              }
              ds2[u] = pv * (dpv - dlts[q]);
            }
            if constexpr (decltype(masked)::value) {
              const bool m0 = (mk >> (2 * j)) & 1, m1 = (mk >> (2 * j + 1)) & 1;
              pd2[0] = m0 ? pd2[0] : 0.f; ds2[0] = m0 ? ds2[0] : 0.f;
              pd2[1] = m1 ? pd2[1] : 0.f; ds2[1] = m1 ? ds2[1] : 0.f;
            }
            split2(f32x2{pd2[0], pd2[1]}, pw[jj], plw[jj]);
            split2(f32x2{ds2[0], ds2[1]}, dw[jj], dlw[jj]);
          }
        } else {
          // bias of (query qb + acc_row(i, hh), key myk): rabx[kRabPad + q - myk]
          const float* rbase = L.f0 + kRabPad + (qb - myk + 4 * hh);
          // time bias of this half's 8 scores, behind ONE wave-uniform branch (a
          // branch per score split the loop body into 16 blocks the scheduler
          // could not interleave: MFMA and VALU work then ran back to back)
          float tbv[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) tbv[e] = 0.f;
          if (TBK && p.nbt) {
            const int tk = L.tss[myk < Tp ? myk : Tp - 1];
#pragma unroll
            for (int e = 0; e < 8; ++e)
              tbv[e] = L.rtab[time_bucket(L.tss[qb + acc_row(8 * s2 + e, hh)] - tk, p.nbt)];
          }
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const int j = 4 * s2 + jj;
            float pd2[2], ds2[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              const int i = 2 * j + u;
              const float bias = TBK ? rbase[(i & 3) + 8 * (i >> 2)] + tbv[2 * jj + u] : rbase[(i & 3) + 8 * (i >> 2)];
              const float x = fmaf(s[i], p.scale, bias);
              const float sg = sigmoid_fast(x), sgn = fold ? sg : sg * sn;
              pd2[u] = x * sgn;                                   // SiLU(x) / n
              ds2[u] = dp[i] * fmaf(fmaf(-x, sg, x), sgn, sgn);   // dp * dSiLU(x) / n
            }
            if constexpr (decltype(masked)::value) {
              const bool m0 = (mk >> (2 * j)) & 1, m1 = (mk >> (2 * j + 1)) & 1;
              pd2[0] = m0 ? pd2[0] : 0.f; ds2[0] = m0 ? ds2[0] : 0.f;
              pd2[1] = m1 ? pd2[1] : 0.f; ds2[1] = m1 ? ds2[1] : 0.f;
            }
            split2(f32x2{pd2[0], pd2[1]}, pw[jj], plw[jj]);
            split2(f32x2{ds2[0], ds2[1]}, dw[jj], dlw[jj]);
          }
        }
          const bf16x8 ph = words8(pw), pl = words8(plw);
          const bf16x8 dh = words8(dw), dl2 = words8(dlw);
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt) {
            const bf16x8 dof = lds_tr8<HD>(L.img1, qb + 16 * s2, dt * 32, lane);
            const bf16x8 qf = lds_tr8<HD>(L.img0, qb + 16 * s2, dt * 32, lane);
            dv[dt] = mfma(dof, ph, dv[dt]);
            dk[dt] = mfma(qf, dh, dk[dt]);
            if (PREC) {
              dv[dt] = mfma(dof, pl, dv[dt]);
              dk[dt] = mfma(qf, dl2, dk[dt]);
            }
            if constexpr (PREC == 2) {
              dv[dt] = mfma(lds_tr8<HD>(L.img1lo, qb + 16 * s2, dt * 32, lane), ph, dv[dt]);
              dk[dt] = mfma(lds_tr8<HD>(L.img0lo, qb + 16 * s2, dt * 32, lane), dh, dk[dt]);
            }
          }
        };
        half(std::integral_constant<bool, KIND == 0>{}, 0);
        half(std::integral_constant<bool, KIND == 0>{}, 1);
      }
      const int64_t otok = rbase + myk;
      const bool kst = kin && myk >= lo;
      store_rows<HD, NDT>(p.dk, p.lddk, p.out_f32, otok, h, hh, dk, kok ? (fold ? p.scale * pscale : p.scale) : 0.f,
                          kst, p.act ? p.k : nullptr, p.ldk, p.in_dt);
      store_rows<HD, NDT>(p.dv, p.lddv, p.out_f32, otok, h, hh, dv, kok ? pscale : 0.f, kst, p.act ? p.v : nullptr,
                          p.ldv, p.in_dt);
#ifdef GRK_DKDV_STAMPS
      if (ntile_done < 3) GRK_RT(3 + ntile_done);
      ++ntile_done;
#endif
    }
  GRK_RT(6);
}

template <int HD>
static bool seq_launch_hd(const AttnParams& p, int which, hipStream_t s) {
  const int Tp = (p.T + 31) / 32 * 32;
  const int f1 = which == 2 ? kDqBinArrays + 1 : 1;
  // fidelity mode: four images, one workgroup per CU (up to 160 KiB)
  const size_t lds = p.precise == 2 ? SeqLds<HD, 4>::bytes(Tp, f1) : SeqLds<HD, 2>::bytes(Tp, f1);
  const size_t cap = p.precise == 2 ? (size_t)160 * 1024 : (size_t)kSeqLdsMax;
  if (lds > cap || Tp + kRabPad > 2 * 64 * kSeqWaves) return false;
  const dim3 grid(p.B * p.H);
  const int threads = 64 * kSeqWaves;
#define GRK_SEQ(KERNEL)                                                                                  \
  do {                                                                                                   \
    if (p.kind == GRK_ATTN_SOFTMAX) {                                                                    \
      if (p.precise == 2) launch_lds(KERNEL<HD, 0, 2>, grid, threads, lds, s, p);                        \
      else if (p.precise) launch_lds(KERNEL<HD, 0, 1>, grid, threads, lds, s, p);                        \
      else launch_lds(KERNEL<HD, 0, 0>, grid, threads, lds, s, p);                                       \
    } else {                                                                                             \
      if (p.precise == 2) launch_lds(KERNEL<HD, 1, 2>, grid, threads, lds, s, p);                        \
      else if (p.precise) launch_lds(KERNEL<HD, 1, 1>, grid, threads, lds, s, p);                        \
      else launch_lds(KERNEL<HD, 1, 0>, grid, threads, lds, s, p);                                       \
    }                                                                                                    \
  } while (0)
  if (which == 0) GRK_SEQ(k_attn_fwd_seq);
  else if (which == 2) GRK_SEQ(k_attn_dq_seq);
#if GRK_ATTN_TB_SPLIT
  else if (p.kind != GRK_ATTN_SOFTMAX && p.nbt == 0) {
    if (p.precise == 2) launch_lds(k_attn_dkdv_seq<HD, 1, 2, false>, grid, threads, lds, s, p);
    else if (p.precise) launch_lds(k_attn_dkdv_seq<HD, 1, 1, false>, grid, threads, lds, s, p);
    else launch_lds(k_attn_dkdv_seq<HD, 1, 0, false>, grid, threads, lds, s, p);
  }
#endif
  else GRK_SEQ(k_attn_dkdv_seq);
#undef GRK_SEQ
  return true;
}

template <int HD>
static bool fidelity_fits(int T) {
  const int Tp = (T + 31) / 32 * 32;
  return SeqLds<HD, 4>::bytes(Tp, kDqBinArrays + 1) <= (size_t)160 * 1024 && Tp + kRabPad <= 2 * 64 * kSeqWaves;
}

bool attn_seq_launch(const AttnParams& p, int hd, int which, hipStream_t s) {
  static const bool chunked = getenv("GRK_ATTN_CHUNKED") != nullptr;  // force the chunked kernels (A/B tests)
  if (chunked) return false;
  switch (hd) {
    case 16: return seq_launch_hd<16>(p, which, s);
    case 32: return seq_launch_hd<32>(p, which, s);
    case 64: return seq_launch_hd<64>(p, which, s);
    case 128: return seq_launch_hd<128>(p, which, s);
  }
  return false;
}

}  // namespace grk

using namespace grk;

extern "C" int grk_attention_fidelity_supported(int seq_len, int head_dim) {
  if (seq_len <= 0 || getenv("GRK_ATTN_CHUNKED")) return 0;
  switch (head_dim) {
    case 16: return fidelity_fits<16>(seq_len);
    case 32: return fidelity_fits<32>(seq_len);
    case 64: return fidelity_fits<64>(seq_len);
    case 128: return fidelity_fits<128>(seq_len);
    case 256:
    case 512: return wide_fidelity_enabled(head_dim) ? 1 : 0;  // the wide-head kernels (any T)
  }
  return 0;
}

namespace grk {
// grk_jagged_layout's ranges + row bases in one launch when the batch fits the fused
// workgroup (false: the caller runs grk_seq_ranges and k_jagged_base)
bool seq_ranges_jagged(const uint8_t* key_valid, int batch, int seq_len, int64_t cap, int32_t* ranges,
                       int64_t* row_base, int64_t* n_rows, int32_t* err, hipStream_t s) {
  if (batch <= 0 || batch > kSeqFused || (int64_t)batch * seq_len > kSeqFusedBytes) return false;
  k_seq_ranges_order<true><<<1, 1024, 0, s>>>(key_valid, batch, seq_len, ranges, cap, row_base, n_rows, err);
  return true;
}
}  // namespace grk

extern "C" int grk_seq_ranges(const uint8_t* key_valid, int batch, int seq_len, int32_t* ranges, void* stream) {
  clear_error();
  GRK_CHECK_ARG(batch >= 0 && seq_len > 0, "batch must be >= 0 and seq_len > 0");
  if (batch == 0) return GRK_OK;
  GRK_CHECK_ARG(key_valid && ranges, "key_valid and ranges required");
  if (batch <= kSeqFused && (int64_t)batch * seq_len <= kSeqFusedBytes) {
    k_seq_ranges_order<false><<<1, 1024, 0, (hipStream_t)stream>>>(key_valid, batch, seq_len, ranges, 0, nullptr,
                                                                    nullptr, nullptr);
    GRK_LAUNCH_CHECK();
    return GRK_OK;
  }
  k_seq_ranges<<<(batch + 3) / 4, 256, 0, (hipStream_t)stream>>>(key_valid, batch, seq_len, ranges);
  GRK_LAUNCH_CHECK();
  k_seq_order<<<1, 1024, 0, (hipStream_t)stream>>>(batch, seq_len, ranges);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}
