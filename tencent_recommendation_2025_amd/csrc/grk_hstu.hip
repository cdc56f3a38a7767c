// HSTU output gate for gfx950: y = dropout(LayerNorm(o) * SiLU(u)), its
// backward, and the deterministic dgamma/dbeta column sums.
//
// Replaces (north star; no reference -- oracle/hstu.py):
//   y = out_linear(dropout(attn_norm(HSTU-attn(q, k, v)) * u)),  u = SiLU(pre_u)
// which in eager PyTorch is a silu, a dtype cast, a LayerNorm, a multiply and
// a dropout (forward) and ~10 elementwise/reduction kernels (backward), each
// a full [N, D] HBM round trip.  Here: one pass over o / u / y forward, one
// pass over gy / o / u / do / du backward.
//
// Layout: o, u, y, gy, do, du are bf16 rows of length D with row strides
// (u and du are the first D columns of the [N, 4D] pre-activation / its grad).
// One 64-lane wave per row; lane owns the 16-byte vectors c = lane + 64 j.
// LayerNorm statistics (mean, rstd) are saved per row by the forward.
#include "grk_common.h"

namespace grk {

constexpr int kNgWaves = 4;        // waves per workgroup
// fixed backward grid -> fixed reduction order (GRK_NG_BWD_BLOCKS: A/B builds)
#ifndef GRK_NG_BWD_BLOCKS
#define GRK_NG_BWD_BLOCKS 512
#endif
constexpr int kNgBwdBlocks = GRK_NG_BWD_BLOCKS;

struct NGParams {
  const bf16_t* o; int64_t ldo;
  const bf16_t* u; int64_t ldu;
  const float* gamma; const float* beta;
  float eps;
  int64_t rows; int dim;
  float dropout_p; unsigned long long seed;
  const unsigned long long* seed_dev;  // optional: seed read at kernel time (graph replay)
  bf16_t* y; int64_t ldy;
  float* stats;  // [rows, 2] = mean, rstd
  // backward
  const bf16_t* gy; int64_t ldgy;
  bf16_t* dout; int64_t lddo;
  bf16_t* du; int64_t lddu;
  float* partial;  // [gridDim.x, 2, dim]
  float* dgamma; float* dbeta;
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// Dropout decisions of the norm gate and the embedding combine: element
// (row, col) of a [rows, dim] activation is dropped iff its 16-bit uniform is
// below thr16 = ceil(p * 65536) (the drop probability is p to within 2^-16).
// The uniforms of the flattened elements 4j .. 4j+3 are the four 16-bit fields
// of ONE splitmix64 finalisation of (seed, j) -- a quarter of the 64-bit
// multiplies of one mix per element, which left the gate kernels VALU-bound
// (k_ng_fwd 540 VALU per row-lane, 84 of them quarter-rate integer multiplies).
// Forward and backward draw the same decisions; dim % 8 == 0, so a lane's 8
// elements are two whole groups.
__device__ __forceinline__ unsigned long long drop_mix(unsigned long long seed, unsigned long long j) {
  unsigned long long x = seed ^ (j * 0x9E3779B97F4A7C15ull);
  x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27; x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return x;
}

__device__ __forceinline__ void drop8(unsigned long long seed, float p, int64_t row, int c8, int dim, float* m) {
  const float rk = 1.0f / (1.0f - p);
  const unsigned thr = (unsigned)ceilf(p * 65536.0f);
  const unsigned long long j = (unsigned long long)(row * dim + c8) >> 2;
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const unsigned long long x = drop_mix(seed, j + g);
#pragma unroll
    for (int e = 0; e < 4; ++e) m[4 * g + e] = ((unsigned)(x >> (16 * e)) & 0xFFFFu) >= thr ? rk : 0.f;
  }
}

__device__ __forceinline__ void load8(const bf16_t* p, float* f) {
  const uint4 w = *reinterpret_cast<const uint4*>(p);
  const unsigned ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(ws[i] << 16);
    f[2 * i + 1] = __uint_as_float(ws[i] & 0xFFFF0000u);
  }
}

__device__ __forceinline__ void store8(bf16_t* p, const float* f) {
  uint4 w;
  unsigned* ws = &w.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) ws[i] = (unsigned)f32_to_bf16(f[2 * i]) | ((unsigned)f32_to_bf16(f[2 * i + 1]) << 16);
  *reinterpret_cast<uint4*>(p) = w;
}

__device__ __forceinline__ void load8f(const float* p, float* f) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

// dropout multiplier of the 8 elements starting at column c8
__device__ __forceinline__ void keep8(const NGParams& p, int64_t row, int c8, float* m) {
  if (p.dropout_p <= 0.f) {
#pragma unroll
    for (int e = 0; e < 8; ++e) m[e] = 1.f;
    return;
  }
  drop8(p.seed_dev ? *p.seed_dev : p.seed, p.dropout_p, row, c8, p.dim, m);
}

// ------------------------------------------------------------------ forward --
template <int VPL>
__global__ void __launch_bounds__(64 * kNgWaves) k_ng_fwd(NGParams p) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kNgWaves + (threadIdx.x >> 6);
  if (row >= p.rows) return;
  const int nv = p.dim >> 3;
  float x[VPL][8];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + 64 * j;
    if (c < nv) {
      load8(p.o + row * p.ldo + 8 * c, x[j]);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += x[j][e];
    }
  }
  const float inv_d = 1.0f / (float)p.dim;
  const float mean = wave_sum(s) * inv_d;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j)
    if (lane + 64 * j < nv)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = x[j][e] - mean;
        q += d * d;
      }
  const float rstd = rsqrtf(wave_sum(q) * inv_d + p.eps);
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + 64 * j;
    if (c >= nv) continue;
    float u[8], g[8], b[8], m[8], y[8];
    load8(p.u + row * p.ldu + 8 * c, u);
    load8f(p.gamma + 8 * c, g);
    load8f(p.beta + 8 * c, b);
    keep8(p, row, 8 * c, m);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      // SiLU(u) rounded to bf16 first: u is the bf16 activation of the reference formulation
      const float su = bf16_to_f32(f32_to_bf16(silu(u[e])));
      y[e] = ((x[j][e] - mean) * rstd * g[e] + b[e]) * su * m[e];
    }
    store8(p.y + row * p.ldy + 8 * c, y);
  }
  if (lane == 0 && p.stats) {
    p.stats[2 * row] = mean;
    p.stats[2 * row + 1] = rstd;
  }
}

// ----------------------------------------------------------------- backward --
// zhat = (o - mean) rstd, z = zhat g + b, su = SiLU(u), m = dropout multiplier
//   gz = gy su m          du = gy z m dSiLU(u)
//   dgamma += gz zhat     dbeta += gz
//   do = rstd (gz g - mean(gz g) - zhat mean(gz g zhat))
template <int VPL>
__global__ void __launch_bounds__(64 * kNgWaves) k_ng_bwd(NGParams p) {
  __shared__ float red[2 * 64 * VPL * 8];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nv = p.dim >> 3;
  const float inv_d = 1.0f / (float)p.dim;
  float dg[VPL][8], db[VPL][8], g[VPL][8];
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + 64 * j;
#pragma unroll
    for (int e = 0; e < 8; ++e) { dg[j][e] = 0.f; db[j][e] = 0.f; g[j][e] = 0.f; }
    if (c < nv) load8f(p.gamma + 8 * c, g[j]);
  }
  const int64_t stride = (int64_t)gridDim.x * kNgWaves;
  for (int64_t row = (int64_t)blockIdx.x * kNgWaves + wave; row < p.rows; row += stride) {
    const float mean = p.stats[2 * row], rstd = p.stats[2 * row + 1];
    float zh[VPL][8], gzg[VPL][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int c = lane + 64 * j;
      if (c >= nv) continue;
      float o[8], u[8], gy[8], b[8], m[8], du[8];
      load8(p.o + row * p.ldo + 8 * c, o);
      load8(p.u + row * p.ldu + 8 * c, u);
      load8(p.gy + row * p.ldgy + 8 * c, gy);
      load8f(p.beta + 8 * c, b);
      keep8(p, row, 8 * c, m);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float su = bf16_to_f32(f32_to_bf16(silu(u[e])));
        zh[j][e] = (o[e] - mean) * rstd;
        const float z = zh[j][e] * g[j][e] + b[e];
        const float gm = gy[e] * m[e];
        const float gz = gm * su;
        du[e] = gm * z * dsilu(u[e]);
        dg[j][e] += gz * zh[j][e];
        db[j][e] += gz;
        gzg[j][e] = gz * g[j][e];
        s1 += gzg[j][e];
        s2 += gzg[j][e] * zh[j][e];
      }
      store8(p.du + row * p.lddu + 8 * c, du);
    }
    s1 = wave_sum(s1) * inv_d;
    s2 = wave_sum(s2) * inv_d;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int c = lane + 64 * j;
      if (c >= nv) continue;
      float d[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] = rstd * (gzg[j][e] - s1 - zh[j][e] * s2);
      store8(p.dout + row * p.lddo + 8 * c, d);
    }
  }
  // block partials: waves add in fixed order
  for (int w = 0; w < kNgWaves; ++w) {
    if (wave == w)
#pragma unroll
      for (int j = 0; j < VPL; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int i = (lane + 64 * j) * 8 + e;
          red[i] = (w == 0 ? 0.f : red[i]) + dg[j][e];
          red[64 * VPL * 8 + i] = (w == 0 ? 0.f : red[64 * VPL * 8 + i]) + db[j][e];
        }
    __syncthreads();
  }
  float* part = p.partial + (int64_t)blockIdx.x * 2 * p.dim;
  for (int i = threadIdx.x; i < p.dim; i += blockDim.x) {
    part[i] = red[i];
    part[p.dim + i] = red[64 * VPL * 8 + i];
  }
}

// dgamma | dbeta = column sums of the block partials in a fixed order: 64
// columns per workgroup, 16 row groups each summing a strided subset of the
// blocks, then the 16 group sums added in order.
constexpr int kColGroups = 16;
__global__ void __launch_bounds__(64 * kColGroups) k_ng_colsum(NGParams p, int nblocks) {
  __shared__ float part[kColGroups][64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + cl;
  float acc = 0.f;
  if (i < 2 * p.dim) {
#pragma unroll 8
    for (int bk = grp; bk < nblocks; bk += kColGroups) acc += p.partial[(int64_t)bk * 2 * p.dim + i];
  }
  part[grp][cl] = acc;
  __syncthreads();
  if (grp == 0 && i < 2 * p.dim) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < kColGroups; ++g) t += part[g][cl];
    if (i < p.dim) p.dgamma[i] = t;
    else p.dbeta[i - p.dim] = t;
  }
}

// ------------------------------------------------- residual add + LayerNorm --
// The HSTU block's residual stream (model/BaseLine/model.py:330-345 with the
// HSTU block): s_{i+1} = s_i + y_i, x_{i+1} = LayerNorm_{i+1}(s_{i+1}), which
// eager autocast runs as a bf16 add, an fp32 LayerNorm of the bf16 sum and a
// cast of its output for the next GEMM (backward: LayerNorm input grad,
// gamma/beta reductions, casts and a bf16 add of the two residual grads).
// Forward: one wave per row, s_new = bf16(s + y) (y may be absent), x =
// LN(s_new) g + b stored as bf16 or fp32, (mean, rstd) saved.  Backward:
// ds = gs + rstd (gx g - mean(gx g) - zhat mean(gx g zhat)) rounded once to
// bf16 (gs may be absent), dgamma/dbeta through fixed-order block partials.
struct ANParams {
  const bf16_t* s; int64_t lds;
  const bf16_t* y; int64_t ldy;
  const float* gamma; const float* beta;
  float eps;
  int64_t rows; int dim;
  bf16_t* s_out; int64_t ldso;
  void* x; int64_t ldx; int x_f32;
  float* stats;
  // backward
  const void* gx; int64_t ldgx; int gx_f32;
  const bf16_t* gs; int64_t ldgs;
  bf16_t* ds; int64_t ldds;
  float* partial;
};

__device__ __forceinline__ void load8_any(const void* base, int64_t off, bool f32, float* f) {
  if (f32) load8f(reinterpret_cast<const float*>(base) + off, f);
  else load8(reinterpret_cast<const bf16_t*>(base) + off, f);
}

template <int VPL>
__global__ void __launch_bounds__(64 * kNgWaves) k_an_fwd(ANParams p) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kNgWaves + (threadIdx.x >> 6);
  if (row >= p.rows) return;
  const int nv = p.dim >> 3;
  float v[VPL][8];
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + 64 * j;
    if (c >= nv) continue;
    load8(p.s + row * p.lds + 8 * c, v[j]);
    if (p.y) {
      float t[8];
      load8(p.y + row * p.ldy + 8 * c, t);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[j][e] = bf16_to_f32(f32_to_bf16(v[j][e] + t[e]));  // the bf16 residual sum
      store8(p.s_out + row * p.ldso + 8 * c, v[j]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) sum += v[j][e];
  }
  const float inv_d = 1.0f / (float)p.dim;
  const float mean = wave_sum(sum) * inv_d;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j)
    if (lane + 64 * j < nv)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = v[j][e] - mean;
        q += d * d;
      }
  const float rstd = rsqrtf(wave_sum(q) * inv_d + p.eps);
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + 64 * j;
    if (c >= nv) continue;
    float g[8], b[8], x[8];
    load8f(p.gamma + 8 * c, g);
    load8f(p.beta + 8 * c, b);
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = (v[j][e] - mean) * rstd * g[e] + b[e];
    if (p.x_f32) {
      float* dst = reinterpret_cast<float*>(p.x) + row * p.ldx + 8 * c;
      reinterpret_cast<float4*>(dst)[0] = make_float4(x[0], x[1], x[2], x[3]);
      reinterpret_cast<float4*>(dst)[1] = make_float4(x[4], x[5], x[6], x[7]);
    } else {
      store8(reinterpret_cast<bf16_t*>(p.x) + row * p.ldx + 8 * c, x);
    }
  }
  if (lane == 0) {
    p.stats[2 * row] = mean;
    p.stats[2 * row + 1] = rstd;
  }
}

template <int VPL>
__global__ void __launch_bounds__(64 * kNgWaves) k_an_bwd(ANParams p) {
  __shared__ float red[2 * 64 * VPL * 8];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nv = p.dim >> 3;
  const float inv_d = 1.0f / (float)p.dim;
  float dg[VPL][8], db[VPL][8], g[VPL][8];
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + 64 * j;
#pragma unroll
    for (int e = 0; e < 8; ++e) { dg[j][e] = 0.f; db[j][e] = 0.f; g[j][e] = 0.f; }
    if (c < nv) load8f(p.gamma + 8 * c, g[j]);
  }
  const int64_t stride = (int64_t)gridDim.x * kNgWaves;
  for (int64_t row = (int64_t)blockIdx.x * kNgWaves + wave; row < p.rows; row += stride) {
    const float mean = p.stats[2 * row], rstd = p.stats[2 * row + 1];
    float zh[VPL][8], gzg[VPL][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int c = lane + 64 * j;
      if (c >= nv) continue;
      float sv[8], gx[8];
      load8(p.s + row * p.lds + 8 * c, sv);
      load8_any(p.gx, row * p.ldgx + 8 * c, p.gx_f32, gx);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        zh[j][e] = (sv[e] - mean) * rstd;
        dg[j][e] += gx[e] * zh[j][e];
        db[j][e] += gx[e];
        gzg[j][e] = gx[e] * g[j][e];
        s1 += gzg[j][e];
        s2 += gzg[j][e] * zh[j][e];
      }
    }
    s1 = wave_sum(s1) * inv_d;
    s2 = wave_sum(s2) * inv_d;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int c = lane + 64 * j;
      if (c >= nv) continue;
      float d[8], gs[8];
      if (p.gs) load8(p.gs + row * p.ldgs + 8 * c, gs);
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] = rstd * (gzg[j][e] - s1 - zh[j][e] * s2) + (p.gs ? gs[e] : 0.f);
      store8(p.ds + row * p.ldds + 8 * c, d);
    }
  }
  for (int w = 0; w < kNgWaves; ++w) {
    if (wave == w)
#pragma unroll
      for (int j = 0; j < VPL; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int i = (lane + 64 * j) * 8 + e;
          red[i] = (w == 0 ? 0.f : red[i]) + dg[j][e];
          red[64 * VPL * 8 + i] = (w == 0 ? 0.f : red[64 * VPL * 8 + i]) + db[j][e];
        }
    __syncthreads();
  }
  float* part = p.partial + (int64_t)blockIdx.x * 2 * p.dim;
  for (int i = threadIdx.x; i < p.dim; i += blockDim.x) {
    part[i] = red[i];
    part[p.dim + i] = red[64 * VPL * 8 + i];
  }
}

static int ng_blocks_bwd(int64_t rows) {
  int64_t need = (rows + kNgWaves - 1) / kNgWaves;
  return (int)(need < kNgBwdBlocks ? (need < 1 ? 1 : need) : kNgBwdBlocks);
}

static int ng_check(const NGParams& p) {
  GRK_CHECK_ARG(p.rows >= 0, "rows must be >= 0");
  GRK_CHECK_ARG(p.dim > 0 && p.dim % 8 == 0 && p.dim <= 2048, "dim must be a multiple of 8 in [8, 2048]");
  GRK_CHECK_ARG(p.gamma && p.beta, "gamma/beta required");
  GRK_CHECK_ARG(p.dropout_p >= 0.f && p.dropout_p < 1.f, "dropout_p must be in [0, 1)");
  GRK_CHECK_ARG(p.rows == 0 || (p.o && p.u), "o/u required");
  GRK_CHECK_ARG(p.ldo >= p.dim && p.ldu >= p.dim && p.ldo % 8 == 0 && p.ldu % 8 == 0,
                "row strides must be >= dim and multiples of 8");
  GRK_CHECK_ARG(((uintptr_t)p.o | (uintptr_t)p.u | (uintptr_t)p.gamma | (uintptr_t)p.beta) % 16 == 0,
                "o/u/gamma/beta must be 16-byte aligned");
  return GRK_OK;
}

// ----------------------------------------------- fp8 q/k/v (config C5) ----
// The fp8 HSTU layer quantises its SiLU'd v|q|k once per step: out[n, c] =
// e4m3(SiLU(pre[n, c])) (fp32 SiLU, round to nearest even, clamped to the
// e4m3 range +-448), 8 elements per lane; the backward is straight-through:
// the attention's gradients w.r.t. those fp8 values times dSiLU(pre), in place.
__global__ void __launch_bounds__(256) k_silu_fp8(const bf16_t* __restrict__ pre, int64_t ldp, int64_t rows,
                                                  int cols, unsigned char* __restrict__ out, int64_t ldo) {
  const int per_row = cols / 8;
  const int64_t units = rows * per_row;
  const bool div32 = units < ((int64_t)1 << 32);   // 32-bit division where the units allow
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < units; u += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = div32 ? (int64_t)((uint32_t)u / (uint32_t)per_row) : u / per_row;
    const int c = (int)(u - r * per_row) * 8;
    const uint4 w = *reinterpret_cast<const uint4*>(pre + r * ldp + c);
    const unsigned ws[4] = {w.x, w.y, w.z, w.w};
    float f[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f[2 * k] = silu(__uint_as_float(ws[k] << 16));
      f[2 * k + 1] = silu(__uint_as_float(ws[k] & 0xFFFF0000u));
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] = fminf(fmaxf(f[k], -448.f), 448.f);
    int lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], lo, true);
    int hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], 0, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], hi, true);
    *reinterpret_cast<uint2*>(out + r * ldo + c) = make_uint2((unsigned)lo, (unsigned)hi);
  }
}

__global__ void __launch_bounds__(256) k_dsilu_mul(bf16_t* __restrict__ g, int64_t ldg,
                                                   const bf16_t* __restrict__ pre, int64_t ldp, int64_t rows,
                                                   int cols) {
  const int per_row = cols / 8;
  const int64_t units = rows * per_row;
  const bool div32 = units < ((int64_t)1 << 32);   // 32-bit division where the units allow
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < units; u += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = div32 ? (int64_t)((uint32_t)u / (uint32_t)per_row) : u / per_row;
    const int c = (int)(u - r * per_row) * 8;
    uint4* gp = reinterpret_cast<uint4*>(g + r * ldg + c);
    const uint4 gw = *gp, pw = *reinterpret_cast<const uint4*>(pre + r * ldp + c);
    const unsigned gs[4] = {gw.x, gw.y, gw.z, gw.w}, ps[4] = {pw.x, pw.y, pw.z, pw.w};
    unsigned o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float a = __uint_as_float(gs[k] << 16) * dsilu(__uint_as_float(ps[k] << 16));
      const float b = __uint_as_float(gs[k] & 0xFFFF0000u) * dsilu(__uint_as_float(ps[k] & 0xFFFF0000u));
      o[k] = (unsigned)f32_to_bf16(a) | ((unsigned)f32_to_bf16(b) << 16);
    }
    *gp = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// ----------------------------------------- embedding combine (log2feats) ----
// The input of the first block (model/BaseLine/model.py:313-321):
//   seqs = dropout((act(a) + act(b)) * scale + pos),  act = ReLU or identity
// where a / b are the itemdnn / userdnn GEMM outputs (pre-activation with
// relu) and pos the position-embedding rows.  Eager: two ReLUs, an add, a
// mul, an add and a dropout forward; masking, scaling and two ReLU masks
// backward.  Here one pass each way, 8 elements per lane, rounded to bf16
// once.  Backward: g = gy m, gpos = g, ga = g scale [a > 0], gb likewise.
struct ECParams {
  const bf16_t* a; int64_t lda;
  const bf16_t* b; int64_t ldb;  // optional
  const bf16_t* pos; int64_t ldp;  // optional
  float scale; int relu;
  int64_t rows; int dim;
  float dropout_p; unsigned long long seed;
  const unsigned long long* seed_dev;
  bf16_t* y; int64_t ldy;
  const bf16_t* gy; int64_t ldgy;
  bf16_t* ga; int64_t ldga;
  bf16_t* gb; int64_t ldgb;
  bf16_t* gpos; int64_t ldgp;
};

__device__ __forceinline__ void ec_keep8(const ECParams& p, int64_t row, int c8, float* m) {
  if (p.dropout_p <= 0.f) {
#pragma unroll
    for (int e = 0; e < 8; ++e) m[e] = 1.f;
    return;
  }
  drop8(p.seed_dev ? *p.seed_dev : p.seed, p.dropout_p, row, c8, p.dim, m);
}

__global__ void __launch_bounds__(256) k_emb_combine(ECParams p) {
  const int per_row = p.dim >> 3;
  const int64_t units = p.rows * per_row;
  const bool div32 = units < ((int64_t)1 << 32);   // 32-bit division where the units allow
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < units; u += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = div32 ? (int64_t)((uint32_t)u / (uint32_t)per_row) : u / per_row;
    const int c = (int)(u - r * per_row) * 8;
    float a[8], b[8], q[8], m[8], y[8];
    load8(p.a + r * p.lda + c, a);
    if (p.b) load8(p.b + r * p.ldb + c, b);
    if (p.pos) load8(p.pos + r * p.ldp + c, q);
    ec_keep8(p, r, c, m);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float s = p.relu ? fmaxf(a[e], 0.f) : a[e];
      if (p.b) s += p.relu ? fmaxf(b[e], 0.f) : b[e];
      s *= p.scale;
      if (p.pos) s += q[e];
      y[e] = s * m[e];
    }
    store8(p.y + r * p.ldy + c, y);
  }
}

__global__ void __launch_bounds__(256) k_emb_combine_bwd(ECParams p) {
  const int per_row = p.dim >> 3;
  const int64_t units = p.rows * per_row;
  const bool div32 = units < ((int64_t)1 << 32);   // 32-bit division where the units allow
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < units; u += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = div32 ? (int64_t)((uint32_t)u / (uint32_t)per_row) : u / per_row;
    const int c = (int)(u - r * per_row) * 8;
    float g[8], m[8], t[8];
    load8(p.gy + r * p.ldgy + c, g);
    ec_keep8(p, r, c, m);
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] *= m[e];
    if (p.gpos) store8(p.gpos + r * p.ldgp + c, g);
    if (p.ga) {
      if (p.relu) load8(p.a + r * p.lda + c, t);
#pragma unroll
      for (int e = 0; e < 8; ++e) t[e] = (!p.relu || t[e] > 0.f) ? g[e] * p.scale : 0.f;
      store8(p.ga + r * p.ldga + c, t);
    }
    if (p.gb) {
      if (p.relu) load8(p.b + r * p.ldb + c, t);
#pragma unroll
      for (int e = 0; e < 8; ++e) t[e] = (!p.relu || t[e] > 0.f) ? g[e] * p.scale : 0.f;
      store8(p.gb + r * p.ldgb + c, t);
    }
  }
}

static unsigned ec_grid(int64_t rows, int dim) {
  const int64_t units = rows * (dim / 8);
  const int64_t want = (units + 255) / 256;
  return (unsigned)(want < 4096 ? (want < 1 ? 1 : want) : 4096);
}

static int ec_check_rows(const void* t, int64_t ld, int dim, const char* name) {
  if (!t) return GRK_OK;
  if (ld < dim || ld % 8 != 0 || (uintptr_t)t % 16 != 0) {
    set_error("%s: row stride must be >= dim and a multiple of 8, 16-byte aligned", name);
    return GRK_EINVAL;
  }
  return GRK_OK;
}

}  // namespace grk

using namespace grk;

extern "C" int grk_emb_combine_fwd(const void* a, int64_t lda, const void* b, int64_t ldb, const void* pos,
                                   int64_t ldp, float scale, int relu, int64_t rows, int dim, float dropout_p,
                                   uint64_t seed, const uint64_t* seed_dev, void* y, int64_t ldy, void* stream) {
  clear_error();
  GRK_CHECK_ARG(rows >= 0 && dim > 0 && dim % 8 == 0, "dim must be a positive multiple of 8");
  GRK_CHECK_ARG(dropout_p >= 0.f && dropout_p < 1.f, "dropout_p must be in [0, 1)");
  if (rows == 0) return GRK_OK;
  GRK_CHECK_ARG(a && y, "a and y required");
  int rc;
  if ((rc = ec_check_rows(a, lda, dim, "a")) || (rc = ec_check_rows(b, ldb, dim, "b")) ||
      (rc = ec_check_rows(pos, ldp, dim, "pos")) || (rc = ec_check_rows(y, ldy, dim, "y")))
    return rc;
  ECParams p;
  memset(&p, 0, sizeof(p));
  p.a = (const bf16_t*)a; p.lda = lda; p.b = (const bf16_t*)b; p.ldb = ldb; p.pos = (const bf16_t*)pos; p.ldp = ldp;
  p.scale = scale; p.relu = relu != 0; p.rows = rows; p.dim = dim;
  p.dropout_p = dropout_p; p.seed = seed; p.seed_dev = (const unsigned long long*)seed_dev;
  p.y = (bf16_t*)y; p.ldy = ldy;
  k_emb_combine<<<ec_grid(rows, dim), 256, 0, (hipStream_t)stream>>>(p);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

extern "C" int grk_emb_combine_bwd(const void* gy, int64_t ldgy, const void* a, int64_t lda, const void* b,
                                   int64_t ldb, float scale, int relu, int64_t rows, int dim, float dropout_p,
                                   uint64_t seed, const uint64_t* seed_dev, void* ga, int64_t ldga, void* gb,
                                   int64_t ldgb, void* gpos, int64_t ldgp, void* stream) {
  clear_error();
  GRK_CHECK_ARG(rows >= 0 && dim > 0 && dim % 8 == 0, "dim must be a positive multiple of 8");
  GRK_CHECK_ARG(dropout_p >= 0.f && dropout_p < 1.f, "dropout_p must be in [0, 1)");
  if (rows == 0) return GRK_OK;
  GRK_CHECK_ARG(gy, "gy required");
  GRK_CHECK_ARG(!relu || ((!ga || a) && (!gb || b)), "relu: ga / gb need the forward's a / b");
  int rc;
  if ((rc = ec_check_rows(gy, ldgy, dim, "gy")) || (rc = ec_check_rows(a, lda, dim, "a")) ||
      (rc = ec_check_rows(b, ldb, dim, "b")) || (rc = ec_check_rows(ga, ldga, dim, "ga")) ||
      (rc = ec_check_rows(gb, ldgb, dim, "gb")) || (rc = ec_check_rows(gpos, ldgp, dim, "gpos")))
    return rc;
  ECParams p;
  memset(&p, 0, sizeof(p));
  p.a = (const bf16_t*)a; p.lda = lda; p.b = (const bf16_t*)b; p.ldb = ldb;
  p.scale = scale; p.relu = relu != 0; p.rows = rows; p.dim = dim;
  p.dropout_p = dropout_p; p.seed = seed; p.seed_dev = (const unsigned long long*)seed_dev;
  p.gy = (const bf16_t*)gy; p.ldgy = ldgy; p.ga = (bf16_t*)ga; p.ldga = ldga; p.gb = (bf16_t*)gb; p.ldgb = ldgb;
  p.gpos = (bf16_t*)gpos; p.ldgp = ldgp;
  k_emb_combine_bwd<<<ec_grid(rows, dim), 256, 0, (hipStream_t)stream>>>(p);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

extern "C" int grk_norm_gate_fwd(const void* o, int64_t ldo, const void* u, int64_t ldu, const float* gamma,
                                 const float* beta, float eps, int64_t rows, int dim, float dropout_p, uint64_t seed,
                                 const uint64_t* seed_dev,
                                 void* y, int64_t ldy, float* stats, void* stream) {
  clear_error();
  NGParams p;
  memset(&p, 0, sizeof(p));
  p.o = (const bf16_t*)o; p.ldo = ldo; p.u = (const bf16_t*)u; p.ldu = ldu;
  p.gamma = gamma; p.beta = beta; p.eps = eps; p.rows = rows; p.dim = dim;
  p.dropout_p = dropout_p; p.seed = seed; p.seed_dev = (const unsigned long long*)seed_dev; p.y = (bf16_t*)y; p.ldy = ldy; p.stats = stats;
  int rc = ng_check(p);
  if (rc) return rc;
  GRK_CHECK_ARG(rows == 0 || (y && ldy >= dim && ldy % 8 == 0 && (uintptr_t)y % 16 == 0), "bad y / ldy");
  if (rows == 0) return GRK_OK;
  const unsigned grid = (unsigned)((rows + kNgWaves - 1) / kNgWaves);
  hipStream_t s = (hipStream_t)stream;
  const int vpl = (dim / 8 + 63) / 64;
  if (vpl == 1) k_ng_fwd<1><<<grid, 64 * kNgWaves, 0, s>>>(p);
  else if (vpl == 2) k_ng_fwd<2><<<grid, 64 * kNgWaves, 0, s>>>(p);
  else k_ng_fwd<4><<<grid, 64 * kNgWaves, 0, s>>>(p);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

extern "C" size_t grk_norm_gate_bwd_workspace(int64_t rows, int dim) {
  return (size_t)ng_blocks_bwd(rows) * 2 * (size_t)(dim > 0 ? dim : 0) * sizeof(float);
}

extern "C" int grk_norm_gate_bwd(const void* gy, int64_t ldgy, const void* o, int64_t ldo, const void* u,
                                 int64_t ldu, const float* gamma, const float* beta, const float* stats, int64_t rows,
                                 int dim, float dropout_p, uint64_t seed, const uint64_t* seed_dev, void* dout,
                                 int64_t lddo, void* du,
                                 int64_t lddu, float* dgamma, float* dbeta, void* ws, size_t ws_bytes, void* stream) {
  clear_error();
  NGParams p;
  memset(&p, 0, sizeof(p));
  p.o = (const bf16_t*)o; p.ldo = ldo; p.u = (const bf16_t*)u; p.ldu = ldu;
  p.gamma = gamma; p.beta = beta; p.rows = rows; p.dim = dim;
  p.dropout_p = dropout_p; p.seed = seed; p.seed_dev = (const unsigned long long*)seed_dev; p.stats = const_cast<float*>(stats);
  p.gy = (const bf16_t*)gy; p.ldgy = ldgy; p.dout = (bf16_t*)dout; p.lddo = lddo; p.du = (bf16_t*)du; p.lddu = lddu;
  p.partial = (float*)ws; p.dgamma = dgamma; p.dbeta = dbeta;
  int rc = ng_check(p);
  if (rc) return rc;
  GRK_CHECK_ARG(dgamma && dbeta, "dgamma/dbeta required");
  GRK_CHECK_ARG(ws && ws_bytes >= grk_norm_gate_bwd_workspace(rows, dim), "workspace too small");
  GRK_CHECK_ARG(rows == 0 || (gy && dout && du && stats), "gy/dout/du/stats required");
  GRK_CHECK_ARG(ldgy >= dim && lddo >= dim && lddu >= dim && ldgy % 8 == 0 && lddo % 8 == 0 && lddu % 8 == 0,
                "row strides must be >= dim and multiples of 8");
  GRK_CHECK_ARG(((uintptr_t)gy | (uintptr_t)dout | (uintptr_t)du) % 16 == 0, "gy/dout/du must be 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  const int nb = ng_blocks_bwd(rows);
  if (rows > 0) {
    const int vpl = (dim / 8 + 63) / 64;
    if (vpl == 1) k_ng_bwd<1><<<nb, 64 * kNgWaves, 0, s>>>(p);
    else if (vpl == 2) k_ng_bwd<2><<<nb, 64 * kNgWaves, 0, s>>>(p);
    else k_ng_bwd<4><<<nb, 64 * kNgWaves, 0, s>>>(p);
    GRK_LAUNCH_CHECK();
  } else {
    GRK_CHECK_HIP(zero_async(ws, grk_norm_gate_bwd_workspace(rows, dim), s));
  }
  k_ng_colsum<<<(2 * dim + 63) / 64, 64 * kColGroups, 0, s>>>(p, nb);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

extern "C" int grk_add_norm_fwd(const void* s, int64_t lds, const void* y, int64_t ldy, const float* gamma,
                                const float* beta, float eps, int64_t rows, int dim, void* s_out, int64_t ldso,
                                void* x, int64_t ldx, int x_dtype, float* stats, void* stream) {
  clear_error();
  GRK_CHECK_ARG(rows >= 0 && dim > 0 && dim % 8 == 0 && dim <= 2048, "dim must be a multiple of 8 in [8, 2048]");
  if (rows == 0) return GRK_OK;
  GRK_CHECK_ARG(s && gamma && beta && x && stats, "s / gamma / beta / x / stats required");
  GRK_CHECK_ARG(!y || s_out, "y needs s_out (the residual sum)");
  GRK_CHECK_ARG(x_dtype == GRK_BF16 || x_dtype == GRK_F32, "x must be bf16 or fp32");
  GRK_CHECK_ARG(lds >= dim && lds % 8 == 0 && ldx >= dim && ldx % 8 == 0 && (!y || (ldy >= dim && ldy % 8 == 0 &&
                ldso >= dim && ldso % 8 == 0)), "row strides must be >= dim and multiples of 8");
  GRK_CHECK_ARG(((uintptr_t)s | (uintptr_t)y | (uintptr_t)s_out | (uintptr_t)x | (uintptr_t)gamma |
                 (uintptr_t)beta) % 16 == 0, "operands must be 16-byte aligned");
  ANParams p;
  memset(&p, 0, sizeof(p));
  p.s = (const bf16_t*)s; p.lds = lds; p.y = (const bf16_t*)y; p.ldy = ldy;
  p.gamma = gamma; p.beta = beta; p.eps = eps; p.rows = rows; p.dim = dim;
  p.s_out = (bf16_t*)s_out; p.ldso = ldso; p.x = x; p.ldx = ldx; p.x_f32 = x_dtype == GRK_F32; p.stats = stats;
  const unsigned grid = (unsigned)((rows + kNgWaves - 1) / kNgWaves);
  hipStream_t st = (hipStream_t)stream;
  const int vpl = (dim / 8 + 63) / 64;
  if (vpl == 1) k_an_fwd<1><<<grid, 64 * kNgWaves, 0, st>>>(p);
  else if (vpl == 2) k_an_fwd<2><<<grid, 64 * kNgWaves, 0, st>>>(p);
  else k_an_fwd<4><<<grid, 64 * kNgWaves, 0, st>>>(p);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

extern "C" size_t grk_add_norm_bwd_workspace(int64_t rows, int dim) { return grk_norm_gate_bwd_workspace(rows, dim); }

extern "C" int grk_add_norm_bwd(const void* gx, int64_t ldgx, int gx_dtype, const void* gs, int64_t ldgs,
                                const void* s_new, int64_t lds, const float* gamma, const float* stats, int64_t rows,
                                int dim, void* ds, int64_t ldds, float* dgamma, float* dbeta, void* ws,
                                size_t ws_bytes, void* stream) {
  clear_error();
  GRK_CHECK_ARG(rows >= 0 && dim > 0 && dim % 8 == 0 && dim <= 2048, "dim must be a multiple of 8 in [8, 2048]");
  GRK_CHECK_ARG(gamma && dgamma && dbeta, "gamma / dgamma / dbeta required");
  GRK_CHECK_ARG(ws && ws_bytes >= grk_add_norm_bwd_workspace(rows, dim), "workspace too small");
  GRK_CHECK_ARG(gx_dtype == GRK_BF16 || gx_dtype == GRK_F32, "gx must be bf16 or fp32");
  GRK_CHECK_ARG(rows == 0 || (gx && s_new && stats && ds), "gx / s_new / stats / ds required");
  GRK_CHECK_ARG(ldgx >= dim && ldgx % 8 == 0 && lds >= dim && lds % 8 == 0 && ldds >= dim && ldds % 8 == 0 &&
                (!gs || (ldgs >= dim && ldgs % 8 == 0)), "row strides must be >= dim and multiples of 8");
  GRK_CHECK_ARG(((uintptr_t)gx | (uintptr_t)gs | (uintptr_t)s_new | (uintptr_t)ds | (uintptr_t)gamma) % 16 == 0,
                "operands must be 16-byte aligned");
  ANParams p;
  memset(&p, 0, sizeof(p));
  p.s = (const bf16_t*)s_new; p.lds = lds; p.gamma = gamma; p.rows = rows; p.dim = dim;
  p.stats = const_cast<float*>(stats);
  p.gx = gx; p.ldgx = ldgx; p.gx_f32 = gx_dtype == GRK_F32; p.gs = (const bf16_t*)gs; p.ldgs = ldgs;
  p.ds = (bf16_t*)ds; p.ldds = ldds; p.partial = (float*)ws;
  hipStream_t st = (hipStream_t)stream;
  const int nb = ng_blocks_bwd(rows);
  if (rows > 0) {
    const int vpl = (dim / 8 + 63) / 64;
    if (vpl == 1) k_an_bwd<1><<<nb, 64 * kNgWaves, 0, st>>>(p);
    else if (vpl == 2) k_an_bwd<2><<<nb, 64 * kNgWaves, 0, st>>>(p);
    else k_an_bwd<4><<<nb, 64 * kNgWaves, 0, st>>>(p);
    GRK_LAUNCH_CHECK();
  } else {
    GRK_CHECK_HIP(zero_async(ws, grk_add_norm_bwd_workspace(rows, dim), st));
  }
  NGParams q;
  memset(&q, 0, sizeof(q));
  q.dim = dim; q.partial = (float*)ws; q.dgamma = dgamma; q.dbeta = dbeta;
  k_ng_colsum<<<(2 * dim + 63) / 64, 64 * kColGroups, 0, st>>>(q, nb);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

extern "C" int grk_silu_fp8(const void* pre, int64_t ldpre, int64_t rows, int cols, void* out, int64_t ldout,
                            void* stream) {
  clear_error();
  GRK_CHECK_ARG(rows >= 0 && cols > 0 && cols % 8 == 0, "rows >= 0 and cols a positive multiple of 8");
  GRK_CHECK_ARG(rows == 0 || (pre && out), "pre / out are required");
  GRK_CHECK_ARG(ldpre >= cols && ldpre % 8 == 0 && (uintptr_t)pre % 16 == 0, "pre: 16-byte aligned rows");
  GRK_CHECK_ARG(ldout >= cols && ldout % 8 == 0 && (uintptr_t)out % 8 == 0, "out: 8-byte aligned rows");
  if (rows == 0) return GRK_OK;
  const int64_t units = rows * (cols / 8);
  k_silu_fp8<<<grid_for(units, 256, 8192), 256, 0, (hipStream_t)stream>>>((const bf16_t*)pre, ldpre, rows, cols,
                                                                          (unsigned char*)out, ldout);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

extern "C" int grk_dsilu_mul(void* g, int64_t ldg, const void* pre, int64_t ldpre, int64_t rows, int cols,
                             void* stream) {
  clear_error();
  GRK_CHECK_ARG(rows >= 0 && cols > 0 && cols % 8 == 0, "rows >= 0 and cols a positive multiple of 8");
  GRK_CHECK_ARG(rows == 0 || (g && pre), "g / pre are required");
  GRK_CHECK_ARG(ldg >= cols && ldg % 8 == 0 && (uintptr_t)g % 16 == 0, "g: 16-byte aligned rows");
  GRK_CHECK_ARG(ldpre >= cols && ldpre % 8 == 0 && (uintptr_t)pre % 16 == 0, "pre: 16-byte aligned rows");
  if (rows == 0) return GRK_OK;
  const int64_t units = rows * (cols / 8);
  k_dsilu_mul<<<grid_for(units, 256, 8192), 256, 0, (hipStream_t)stream>>>((bf16_t*)g, ldg, (const bf16_t*)pre,
                                                                           ldpre, rows, cols);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}
