// Shared pieces of the gfx950 attention kernels (grk_attention.hip: the
// chunked kernels for any length; grk_attention_seq.hip: whole-sequence
// kernels for short sequences).  See grk_attention.hip for the conventions.
#pragma once
#include "grk_common.h"
#include "grk_mfma.h"

namespace grk {

constexpr int kChunk = 64;      // rows staged per LDS chunk
constexpr int kBlockRows = 128; // queries (fwd/dQ) or keys (dKdV) per workgroup
constexpr int kRabMax = 2048;

struct AttnParams {
  int kind, B, H, T;
  const bf16_t *q, *k, *v;
  int64_t ldq, ldk, ldv;
  const uint8_t* key_valid;
  float scale, inv_n, dropout_p;
  unsigned long long seed;
  const unsigned long long* seed_dev;  // optional: seed read at kernel time (graph replay)
  const float* rab;
  int nb;
  int precise;      // 0 fast, 1 hi/lo P and dS, 2 + hi/lo Q/K/V/dO (fp32 fidelity)
  int in_dt;        // precise == 2: dtype of q/k/v (GRK_F32 / GRK_F16 / GRK_BF16)
  int out_f32;
  int act;  // GRK_ACT_SILU: q/k/v are pre-activations
  int qkv_f8;  // q/k/v are OCP fp8 e4m3 (chunked kernels, head_dim 64 / 128)
  const int* seq_range;  // optional [B, 3] (first valid key, contiguous flag; longest-first order)
  // optional jagged layout (whole-sequence kernels + delta): token (b, t) of q/k/v/out/dO/dq/dk/dv
  // is row row_base[b] + t and only t in [seq_range[3 b], T) exist; NULL = padded rows b * T + t
  const int64_t* row_base;
  const int64_t* jag_n;  // jagged: span rows (device); rows [*jag_n, jag_cap) of every output are zeroed
  int64_t jag_cap;
  unsigned long long* drab_fix;  // [H, nb] int64 fixed-point drab accumulator (deterministic)
  // HSTU time bias (whole-sequence kernels): S += rab_t[h, time_bucket(ts_q - ts_k)]
  const int64_t* ts;
  const float* rab_t;
  int nbt;                           // 0 = off
  float* drab_t;
  unsigned long long* drab_t_fix;    // [H, nbt] fixed point
  // forward
  void* out; int64_t ldo; float* lse;
  // backward
  const void* dout; int64_t lddo; int dout_f32;
  const float* delta;
  void *dq, *dk, *dv; int64_t lddq, lddk, lddv;
  float* drab;
  unsigned* fin_count;   // non-null: the whole-sequence dq kernel's last workgroup finalizes
                         // drab / drab_t from the fixed-point bins and leaves bins + counter zero
  int drab_set;          // finalize writes drab / drab_t (1) or adds to them (0)
};



// Eight consecutive elements of a q/k/v/dO row as exact fp32 (dtype GRK_F32 /
// GRK_F16 / GRK_BF16), zero when !ok.
__device__ __forceinline__ void gload8f(const void* base, int64_t off, int dt, bool ok, float* f) {
  if (!ok) {
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = 0.f;
    return;
  }
  if (dt == 0) {  // GRK_F32
    const float4* fp = reinterpret_cast<const float4*>((const float*)base + off);
    const float4 a = fp[0], b = fp[1];
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  } else if (dt == 2) {  // GRK_F16
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    const h8 v = *reinterpret_cast<const h8*>((const _Float16*)base + off);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (float)v[j];
  } else {
    const bf16x8 v = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>((const bf16_t*)base + off));
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (float)v[j];
  }
}

// x = hi + lo with hi = bf16(x), lo = bf16(x - hi): 16 significant bits (fp16
// values exactly; fp32 to ~2^-17 relative).
__device__ __forceinline__ void split8(const float* f, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 h = static_cast<__bf16>(f[j]);
    hi[j] = h;
    lo[j] = static_cast<__bf16>(f[j] - static_cast<float>(h));
  }
}

// The dropout seed of a launch: the device value when one is given.
__device__ __forceinline__ unsigned long long attn_seed(const AttnParams& p) {
  return p.seed_dev ? *p.seed_dev : p.seed;
}

// Counter-based dropout keep decision for element (b*H+h, q, k): identical
// in forward and backward.
__device__ __forceinline__ bool drop_keep(unsigned long long seed, int bh, int q, int k, int T, float p) {
  unsigned long long x = seed ^ (((unsigned long long)bh * (unsigned)T + (unsigned)q) * (unsigned)T + (unsigned)k) *
                                    0x9E3779B97F4A7C15ull;
  x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27; x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  const float u = (float)(x >> 40) * (1.0f / 16777216.0f);
  return u >= p;
}

// Stage rows [r0, r0+kChunk) of a [B*T, ld] head slice into a swizzled LDS
// image (zeros outside [0, T)).
// Stage rows [r0, r0 + nrows) of a [B*T, ld] head slice into image rows
// [dst0, dst0 + nrows) of a swizzled LDS image (zeros outside [0, T));
// act: apply SiLU on the way (pre-activation inputs).
// src: 0 bf16, 1 fp32, 2 fp8 e4m3 (gload8_src).
template <int HD>
__device__ __forceinline__ void stage_rows_at(char* dst, const void* src, int64_t ld, int b, int T, int h, int r0,
                                              int nrows, int dst0, int src_dt, bool act) {
  constexpr int NCH = HD / 8;
  for (int u = threadIdx.x; u < nrows * NCH; u += blockDim.x) {
    const int row = u / NCH, c = u % NCH;
    const int t = r0 + row;
    const bool ok = t >= 0 && t < T;
    bf16x8 v = gload8_src(src, ((int64_t)b * T + (ok ? t : 0)) * ld + h * HD + c * 8, src_dt, ok);
    if (act) v = silu8(v);
    *reinterpret_cast<uint4*>(dst + lds_off<HD>(dst0 + row, c * 8)) = __builtin_bit_cast(uint4, v);
  }
}

template <int HD>
__device__ __forceinline__ void stage_rows(char* dst, const void* src, int64_t ld, int b, int T, int h, int r0,
                                           int src_dt, bool act = false) {
  stage_rows_at<HD>(dst, src, ld, b, T, h, r0, kChunk, 0, src_dt, act);
}

// fp8 row image (the A operand rows of the fp8 QK^T MFMA): row of HD bytes =
// HD/8 8-byte granules; granule g of row r at position g ^ (r & MASK), so the
// 32 rows a wave reads at one column spread over the banks.
template <int HD>
__device__ __forceinline__ int lds8_off(int row, int col) {
  constexpr int NG = HD / 8;
  constexpr int MASK = NG >= 16 ? 15 : NG - 1;
  return row * HD + (((col >> 3) ^ (row & MASK)) << 3);
}

template <int HD>
__device__ __forceinline__ f8x8 lds_row8_f8(const char* base, int row, int col) {
  return *reinterpret_cast<const f8x8*>(base + lds8_off<HD>(row, col));
}

// Rows [r0, r0 + kChunk) of an fp8 [B*T, ld] head slice into an fp8 row image.
template <int HD>
__device__ __forceinline__ void stage_rows_f8(char* dst, const void* src, int64_t ld, int b, int T, int h, int r0) {
  constexpr int NG = HD / 8;
  for (int u = threadIdx.x; u < kChunk * NG; u += blockDim.x) {
    const int row = u / NG, g = u % NG;
    const int t = r0 + row;
    const bool ok = t >= 0 && t < T;
    const uint2 w = ok ? *reinterpret_cast<const uint2*>((const uint8_t*)src + ((int64_t)b * T + t) * ld + h * HD + g * 8)
                       : make_uint2(0, 0);
    *reinterpret_cast<uint2*>(dst + lds8_off<HD>(row, g * 8)) = w;
  }
}

__device__ __forceinline__ int seq_start(const uint8_t* kv, int b, int T, int* s_start) {
  if (!kv) return 0;
  if (threadIdx.x == 0) *s_start = T;
  __syncthreads();
  for (int j = threadIdx.x; j < T; j += blockDim.x)
    if (kv[(int64_t)b * T + j]) atomicMin(s_start, j);
  __syncthreads();
  return *s_start;
}

template <typename OutT>
__device__ __forceinline__ void store4(OutT* p, const float* v);
template <>
__device__ __forceinline__ void store4<float>(float* p, const float* v) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
template <>
__device__ __forceinline__ void store4<bf16_t>(bf16_t* p, const float* v) {
  uint2 t;
  t.x = (unsigned)f32_to_bf16(v[0]) | ((unsigned)f32_to_bf16(v[1]) << 16);
  t.y = (unsigned)f32_to_bf16(v[2]) | ((unsigned)f32_to_bf16(v[3]) << 16);
  *reinterpret_cast<uint2*>(p) = t;
}

// Store an accumulated D^T tile set acc[NDT] (rows = feature d, lane = token)
// to row `tok` of a [B*T, ld] output: lane holds d = dt*32 + 8g + 4hh + 0..3.
// With dsrc (GRK_ACT_SILU) the value is the gradient w.r.t. the activation
// and is multiplied by dSiLU(pre) read from the same position of dsrc.
template <int HD, int NDT>
__device__ __forceinline__ void store_rows(void* out, int64_t ld, bool f32, int64_t tok, int h, int hh,
                                           const f32x16* acc, float mul, bool ok, const void* dsrc = nullptr,
                                           int64_t ldsrc = 0, int dsrc_dt = 1) {
  if (!ok) return;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = dt * 32 + 8 * g + 4 * hh;
      if (d >= HD) continue;
      float v[4] = {acc[dt][4 * g] * mul, acc[dt][4 * g + 1] * mul, acc[dt][4 * g + 2] * mul, acc[dt][4 * g + 3] * mul};
      if (dsrc && dsrc_dt == 1) {
        const uint2 pw = *reinterpret_cast<const uint2*>((const bf16_t*)dsrc + tok * ldsrc + h * HD + d);
        v[0] *= dsilu(__uint_as_float(pw.x << 16));
        v[1] *= dsilu(__uint_as_float(pw.x & 0xFFFF0000u));
        v[2] *= dsilu(__uint_as_float(pw.y << 16));
        v[3] *= dsilu(__uint_as_float(pw.y & 0xFFFF0000u));
      } else if (dsrc) {  // fp32 / fp16 pre-activations (fidelity mode)
        const int64_t o4 = tok * ldsrc + h * HD + d;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          v[e] *= dsilu(dsrc_dt == 0 ? ((const float*)dsrc)[o4 + e] : (float)((const _Float16*)dsrc)[o4 + e]);
      }
      const int64_t off = tok * ld + h * HD + d;
      if (f32) store4<float>((float*)out + off, v);
      else store4<bf16_t>((bf16_t*)out + off, v);
    }
}

// drab is accumulated as 64-bit fixed point (value * 2^32) with integer
// atomics, in LDS and across workgroups: integer sums do not depend on the
// order of the adds (deterministic), and ds_add_u64 costs ~93 cycles per
// wave-instruction on gfx950 against ~1150 for ds_add_f32
// (scripts/microbench/lds_ops.hip).  Range +-2^31, resolution 2^-32.
constexpr double kFixScale = 4294967296.0;
__device__ __forceinline__ unsigned long long to_fix(float v) {
  const double d = fmin(fmax((double)v * kFixScale, -9.0e18), 9.0e18);
  return (unsigned long long)(long long)d;
}

// drab[i] (+)= fix[i] / 2^32, fix[i] = 0: the fixed-point finalize, by the threads of
// one workgroup (the last dq workgroup) or a grid.
__device__ __forceinline__ void drab_finalize_elem(float* drab, unsigned long long* fix, int i, bool set) {
  const unsigned long long v = atomicExch(&fix[i], 0ull);
  const float x = (float)((double)(long long)v * (1.0 / kFixScale));
  drab[i] = set ? x : drab[i] + x;
}

// Launch with `lds` bytes of dynamic LDS; above 64 KiB the kernel's limit is
// raised first (once per device, kernel and size; gfx950 allows up to 160 KiB).
inline void launch_lds(void (*kernel)(AttnParams), dim3 grid, int threads, size_t lds, hipStream_t s,
                       const AttnParams& p) {
  if (lds > 64 * 1024) (void)ensure_dynamic_lds((const void*)kernel, lds);
  kernel<<<grid, threads, lds, s>>>(p);
}

constexpr int kMaxTimeBuckets = 64;

// Half-octave bucket of a time gap (grk.h, grk_attn_args.timestamps).
__device__ __forceinline__ int time_bucket(int d, int nbt) {
  const unsigned x = (unsigned)(d < 0 ? -d : d) + 1u;
  const int l = 31 - __clz(x);
  const int h1 = l > 0 ? (int)((x >> (l - 1)) & 1u) : 0;
  return min(2 * l + h1, nbt - 1);
}

// Time bias of the chunked / wide kernels (TB instantiations): a stamp relative
// to the sequence's first valid key, clamped to +-(2^30 - 1), 0 past T -- the
// whole-sequence kernels' stage_time convention, so every path buckets alike.
__device__ __forceinline__ int rel_stamp(const AttnParams& p, int b, int T, int start, int j) {
  const int64_t base = start < T ? p.ts[(int64_t)b * T + start] : 0;
  const int64_t lim = (1 << 30) - 1;
  const int64_t d = j < T ? p.ts[(int64_t)b * T + j] - base : 0;
  return (int)(d > lim ? lim : (d < -lim ? -lim : d));
}

// Whole-sequence kernels (grk_attention_seq.hip): one workgroup per
// (batch, head) with the sequence's K/V (or Q/dO) resident in LDS.
// Returns true and launches when the shape fits; false = use the chunked path.
bool attn_seq_launch(const AttnParams& p, int hd, int which, hipStream_t s);

// Wide-head kernels (grk_attention_wide.hip): head_dim 256 / 512, the head's
// columns split over a workgroup's waves (which: 0 forward, 2 dQ, 3 dK/dV).
int attn_wide_launch(const AttnParams& p, int hd, int which, hipStream_t s);
// Whether the wide-head kernels take precise = 2 at this head_dim (256, opt-in).
bool wide_fidelity_enabled(int hd);

}  // namespace grk
