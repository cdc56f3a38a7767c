// Table AdamW for gfx950.
//
// Replaces torch.optim.AdamW's update of the embedding tables
// (model/BaseLine/main.py:131,189; model/BaseLineO1/main.py:174,249) in the
// torch single-tensor order:
//   p *= 1 - lr*wd;  m = m + (1-b1)(g - m);  v = v*b2 + (1-b2) g g;
//   p -= step_size * m / (sqrt(v)/sqrt(1-b2^t) + eps)
// Dense mode streams every row (reference semantics, HBM-bound:
// 10 B/elem read + 10 B/elem written for bf16 params + fp32 moments); the
// gradient is row-sparse and found through row_slot.  Lazy mode touches only
// rows with a gradient.
#include "grk_common.h"

namespace grk {

// Per-step constants of the update (uniform across a launch or a replayed
// step): 1/sqrt(1-b2^t) is taken once here so the element update has no
// IEEE division.
struct AdamStep {
  float decay, w1, beta2, w2, inv_bc2, eps, step_size;
};
__device__ __forceinline__ AdamStep adam_step(const grk_adamw_hparams& hp) {
  AdamStep s;
  s.decay = 1.0f - hp.lr * hp.weight_decay;
  s.w1 = 1.0f - hp.beta1;
  s.beta2 = hp.beta2;
  s.w2 = 1.0f - hp.beta2;
  s.inv_bc2 = 1.0f / hp.bias_corr2_sqrt;
  s.eps = hp.eps;
  s.step_size = hp.step_size;
  return s;
}

// Hyper-parameters of a launch: by value (eager callers), or -- for launches
// captured once in a HIP graph and replayed every step -- read on the device
// at kernel start from hp_ring[*t % ring_len] with the step counter *t in
// device memory (the *_dev entry points).  Uniform scalar loads.
struct HpArg {
  grk_adamw_hparams hp;
  const grk_adamw_hparams* ring;
  const int32_t* t;
  int ring_len;
  // optional (dense mode): g += (*l2coef) * p -- the gradient of l2 * ||W||_F
  // (model/BaseLine/main.py:184-185) with *l2coef = l2 / ||W|| from grk_table_l2_norm
  const float* l2coef;
};
__device__ __forceinline__ grk_adamw_hparams resolve(const HpArg& a) {
  if (a.ring) return a.ring[*a.t % a.ring_len];
  return a.hp;
}
__device__ __forceinline__ int resolve_t(int t, const int32_t* t_dev) { return t_dev ? *t_dev : t; }

// One element of the torch single-tensor AdamW step.  Every update path (dense,
// lazy, dense-gradient, catch-up replay) goes through this function, so a
// replayed g = 0 step is bit-identical to the step the dense pass would run.
// sqrt and the reciprocal are the hardware v_sqrt_f32 / v_rcp_f32 (1 ulp
// each): the correctly rounded library forms cost ~30 VALU ops per element
// (scaling, refinement FMAs, denorm-mode switches), which made replayed steps
// VALU-bound; the difference from torch's rounding is a few ulp of the
// ~lr-sized update term, far inside the parity tolerances (tests/).
// Every rounding is spelled out (explicit fmaf, contraction off): the
// compiler's own contraction choices depend on the calling context (a gradient
// loaded from memory vs a literal 0 in the catch-up replay), and deferred ==
// dense bit-identity needs the same operation sequence in every kernel.
__device__ __forceinline__ void adam1(float& p, float& m, float& v, float g, const AdamStep& s) {
#pragma clang fp contract(off)
  const float pe = p * s.decay;
  const float me = __builtin_fmaf(s.w1, g - m, m);
  const float ve = __builtin_fmaf(s.w2 * g, g, v * s.beta2);
  const float denom = __builtin_fmaf(__builtin_amdgcn_sqrtf(ve), s.inv_bc2, s.eps);
  p = __builtin_fmaf(-s.step_size, me * __builtin_amdgcn_rcpf(denom), pe);
  m = me;
  v = ve;
}

// adam1 with g = 0 (the catch-up replay), the same bits with fewer operations:
//   g - m = -m and fma(w1, -m, m) == fma(-w1, m, m) for every m (signed zeros
//   included: both give +0 for m = +-0);  fma(w2 * 0, 0, v * b2) == v * b2
//   (v >= 0 is never -0, so adding +0 changes nothing).
__device__ __forceinline__ void adam1_g0(float& p, float& m, float& v, const AdamStep& s) {
#pragma clang fp contract(off)
  const float pe = p * s.decay;
  const float me = __builtin_fmaf(-s.w1, m, m);
  const float ve = v * s.beta2;
  const float denom = __builtin_fmaf(__builtin_amdgcn_sqrtf(ve), s.inv_bc2, s.eps);
  p = __builtin_fmaf(-s.step_size, me * __builtin_amdgcn_rcpf(denom), pe);
  m = me;
  v = ve;
}

// adam1_g0 on two elements at once, written on 2-vectors so every multiply / FMA
// is one packed v_pk_*_f32 (the denominator's FMA included, which the compiler
// left unpacked behind the two sqrts): per element the same IEEE operations in the
// same order -- the same bits as adam1_g0 (the replay loop of k_adamw_catchup).
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void adam2_g0(f2v& p, f2v& m, f2v& v, const AdamStep& s) {
#pragma clang fp contract(off)
  const f2v pe = p * s.decay;
  const f2v me = __builtin_elementwise_fma((f2v)(-s.w1), m, m);
  const f2v ve = v * s.beta2;
  f2v sq;
  sq.x = __builtin_amdgcn_sqrtf(ve.x);
  sq.y = __builtin_amdgcn_sqrtf(ve.y);
  const f2v den = __builtin_elementwise_fma(sq, (f2v)(s.inv_bc2), (f2v)(s.eps));
  f2v r;
  r.x = __builtin_amdgcn_rcpf(den.x);
  r.y = __builtin_amdgcn_rcpf(den.y);
  p = __builtin_elementwise_fma((f2v)(-s.step_size), me * r, pe);
  m = me;
  v = ve;
}

// NV consecutive elements (NV = 4 or 8) of param / exp_avg / exp_avg_sq in
// registers: param via one 8/16-byte access (bf16) or NV/4 float4s, moments
// via NV/4 float4s each.
template <typename P, int NV>
__device__ __forceinline__ void load_pmv(const P* p, const float* m, const float* v, float* pv, float* mv, float* vv) {
  if constexpr (sizeof(P) == 4) {
#pragma unroll
    for (int k = 0; k < NV / 4; ++k) {
      const float4 t = reinterpret_cast<const float4*>(p)[k];
      pv[4 * k] = t.x; pv[4 * k + 1] = t.y; pv[4 * k + 2] = t.z; pv[4 * k + 3] = t.w;
    }
  } else {
    unsigned w[NV / 2];
    if constexpr (NV == 8) {
      const uint4 t = *reinterpret_cast<const uint4*>(p);
      w[0] = t.x; w[1] = t.y; w[2] = t.z; w[3] = t.w;
    } else {
      const uint2 t = *reinterpret_cast<const uint2*>(p);
      w[0] = t.x; w[1] = t.y;
    }
#pragma unroll
    for (int k = 0; k < NV / 2; ++k) {
      pv[2 * k] = __uint_as_float(w[k] << 16);
      pv[2 * k + 1] = __uint_as_float(w[k] & 0xFFFF0000u);
    }
  }
#pragma unroll
  for (int k = 0; k < NV / 4; ++k) {
    const float4 a = reinterpret_cast<const float4*>(m)[k], b = reinterpret_cast<const float4*>(v)[k];
    mv[4 * k] = a.x; mv[4 * k + 1] = a.y; mv[4 * k + 2] = a.z; mv[4 * k + 3] = a.w;
    vv[4 * k] = b.x; vv[4 * k + 1] = b.y; vv[4 * k + 2] = b.z; vv[4 * k + 3] = b.w;
  }
}

template <typename P, int NV>
__device__ __forceinline__ void store_pmv(P* p, float* m, float* v, const float* pv, const float* mv, const float* vv) {
  if constexpr (sizeof(P) == 4) {
#pragma unroll
    for (int k = 0; k < NV / 4; ++k)
      reinterpret_cast<float4*>(p)[k] = make_float4(pv[4 * k], pv[4 * k + 1], pv[4 * k + 2], pv[4 * k + 3]);
  } else {
    unsigned w[NV / 2];
#pragma unroll
    for (int k = 0; k < NV / 2; ++k)
      w[k] = (unsigned)f32_to_bf16(pv[2 * k]) | ((unsigned)f32_to_bf16(pv[2 * k + 1]) << 16);
    if constexpr (NV == 8) *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
    else *reinterpret_cast<uint2*>(p) = make_uint2(w[0], w[1]);
  }
#pragma unroll
  for (int k = 0; k < NV / 4; ++k) {
    reinterpret_cast<float4*>(m)[k] = make_float4(mv[4 * k], mv[4 * k + 1], mv[4 * k + 2], mv[4 * k + 3]);
    reinterpret_cast<float4*>(v)[k] = make_float4(vv[4 * k], vv[4 * k + 1], vv[4 * k + 2], vv[4 * k + 3]);
  }
}

// AdamW on NV consecutive elements.
template <typename P, int NV>
__device__ __forceinline__ void adam_vec(P* p, float* m, float* v, const float* g, const AdamStep& s) {
  float pv[NV], mv[NV], vv[NV];
  load_pmv<P, NV>(p, m, v, pv, mv, vv);
#pragma unroll
  for (int e = 0; e < NV; ++e) adam1(pv[e], mv[e], vv[e], g[e], s);
  store_pmv<P, NV>(p, m, v, pv, mv, vv);
}

template <int NV>
__device__ __forceinline__ void load_grad(const float* src, float* g) {
#pragma unroll
  for (int k = 0; k < NV / 4; ++k) {
    const float4 t = reinterpret_cast<const float4*>(src)[k];
    g[4 * k] = t.x; g[4 * k + 1] = t.y; g[4 * k + 2] = t.z; g[4 * k + 3] = t.w;
  }
}

// Dense mode: one NV-vector per thread and a grid covering the whole table
// (no grid-stride loop): measured fastest for this read+write stream on
// gfx950 (scripts/microbench/adamw_dense.hip: 6.09 TB/s vs 5.66 for a
// 4-wide grid-stride loop; nontemporal hints were slower).
template <typename P, int NV>
__global__ void __launch_bounds__(256) k_adamw_dense(P* __restrict__ param, float* __restrict__ m,
                                                     float* __restrict__ v, int64_t num_rows, int dim,
                                                     const float* __restrict__ uniq_rows,
                                                     const int32_t* __restrict__ row_slot, HpArg hpa) {
  const int q = dim / NV;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= num_rows * q) return;
  const int64_t row = i / q;
  const int c = (int)(i - row * q) * NV;
  const int32_t slot = row_slot ? row_slot[row] : -1;
  float g[NV];
#pragma unroll
  for (int e = 0; e < NV; ++e) g[e] = 0.f;
  if (slot >= 0) load_grad<NV>(uniq_rows + (int64_t)slot * dim + c, g);
  const int64_t off = row * dim + c;
  const AdamStep st = adam_step(resolve(hpa));
  float pv[NV], mv[NV], vv[NV];
  load_pmv<P, NV>(param + off, m + off, v + off, pv, mv, vv);
  if (hpa.l2coef) {  // + d(l2 ||W||)/dp at the parameters the loss saw (before this step's decay)
    const float k = *hpa.l2coef;
#pragma unroll
    for (int e = 0; e < NV; ++e) g[e] += k * pv[e];
  }
#pragma unroll
  for (int e = 0; e < NV; ++e) adam1(pv[e], mv[e], vv[e], g[e], st);
  store_pmv<P, NV>(param + off, m + off, v + off, pv, mv, vv);
}

// ||W||_F of a table (l2_emb term, model/BaseLine/main.py:184-185): per-block
// fp64 partial sums of squares over a fixed grid, then one block sums the
// partials in block order -- deterministic, independent of scheduling.
constexpr int kNormBlocks = 1024;
template <typename P>
__global__ void __launch_bounds__(256) k_table_sumsq(const P* __restrict__ p, int64_t n, double* __restrict__ part) {
  __shared__ double red[256];
  double acc = 0.0;
  constexpr int NV = Vec16<P>::N;                  // 16-byte loads (the table is 16-byte aligned)
  const int64_t nv = n / NV;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += (int64_t)kNormBlocks * 256) {
    Vec16<P> x;
    x.load(p + i * NV);
    float sq = 0.f;                                  // 8 squares in fp32 (exact for bf16 inputs), then fp64
#pragma unroll
    for (int e = 0; e < NV; ++e) sq = fmaf(x.get(e), x.get(e), sq);
    acc += (double)sq;
  }
  for (int64_t i = nv * NV + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)kNormBlocks * 256) {
    const double x = (double)Elem<P>::load(p + i);
    acc += x * x;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(256) k_table_norm_final(const double* __restrict__ part, float l2,
                                                          float* __restrict__ norm, float* __restrict__ coef) {
  __shared__ double red[256];
  double acc = 0.0;
  for (int i = threadIdx.x; i < kNormBlocks; i += 256) acc += part[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float nr = (float)sqrt(red[0]);
    norm[0] = nr;
    if (coef) coef[0] = nr > 0.f ? l2 / nr : 0.f;   // torch's norm backward at 0 gives 0 too
  }
}

// Dense gradient of any dtype ([rows, grad_ld], GT = float or bf16): every
// row moves; one NV-vector per thread over a full grid as k_adamw_dense.
template <typename P, typename GT, int NV>
__global__ void __launch_bounds__(256) k_adamw_dense_grad(P* __restrict__ param, float* __restrict__ m,
                                                          float* __restrict__ v, int64_t num_rows, int dim,
                                                          const GT* __restrict__ grad, int64_t grad_ld,
                                                          HpArg hpa) {
  const int q = dim / NV;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= num_rows * q) return;
  const int64_t row = i / q;
  const int c = (int)(i - row * q) * NV;
  float g[NV];
  const GT* src = grad + row * grad_ld + c;
  if constexpr (sizeof(GT) == 4) {
    load_grad<NV>(reinterpret_cast<const float*>(src), g);
  } else {
#pragma unroll
    for (int e = 0; e < NV; ++e) g[e] = bf16_to_f32(reinterpret_cast<const bf16_t*>(src)[e]);
  }
  const int64_t off = row * dim + c;
  adam_vec<P, NV>(param + off, m + off, v + off, g, adam_step(resolve(hpa)));
}

// Several dense gradients over row ranges of one table in ONE launch (the
// feature tables of the `small` group get their gradients as dense [rows, D]
// blocks through the dnn projections): rows covered by a range take its
// gradient (bf16 or fp32, own row stride), rows between ranges g = 0 -- the
// update of k_adamw_dense_grad / k_adamw_dense per row, one launch instead of
// one per range (each ~5 us of launch in a captured step).
constexpr int kMaxGradRanges = 64;
struct GradRanges {
  grk_grad_range r[kMaxGradRanges];
  int n;
};

// shadow (fp32 params only, may be null): the updated parameters also written
// as bf16 in the same [num_rows, dim] layout -- the bf16 GEMM operand of the
// dense layers, so the forward reads it instead of casting every weight per step.
template <typename P, int NV>
__global__ void __launch_bounds__(256) k_adamw_ranges(P* __restrict__ param, float* __restrict__ m,
                                                      float* __restrict__ v, int64_t num_rows, int dim, GradRanges gr,
                                                      HpArg hpa, bf16_t* __restrict__ shadow) {
  const int q = dim / NV;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= num_rows * q) return;
  const int64_t row = i / q;
  const int c = (int)(i - row * q) * NV;
  int lo = 0, hi = gr.n;  // first range whose end is past row (ranges sorted, disjoint)
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (gr.r[mid].row_end <= row) lo = mid + 1;
    else hi = mid;
  }
  float g[NV];
#pragma unroll
  for (int e = 0; e < NV; ++e) g[e] = 0.f;
  if (lo < gr.n && gr.r[lo].row_start <= row) {
    const grk_grad_range& rr = gr.r[lo];
    const int64_t off = (row - rr.row_start) * rr.grad_ld + c;
    if (rr.grad_dtype == GRK_F32) {
      load_grad<NV>(reinterpret_cast<const float*>(rr.grad) + off, g);
    } else {
#pragma unroll
      for (int e = 0; e < NV; ++e) g[e] = bf16_to_f32(reinterpret_cast<const bf16_t*>(rr.grad)[off + e]);
    }
  }
  const int64_t off = row * dim + c;
  float pv[NV], mv[NV], vv[NV];
  load_pmv<P, NV>(param + off, m + off, v + off, pv, mv, vv);
  const AdamStep st = adam_step(resolve(hpa));
#pragma unroll
  for (int e = 0; e < NV; ++e) adam1(pv[e], mv[e], vv[e], g[e], st);
  store_pmv<P, NV>(param + off, m + off, v + off, pv, mv, vv);
  if (shadow) {
    unsigned w[NV / 2];
#pragma unroll
    for (int k = 0; k < NV / 2; ++k)
      w[k] = (unsigned)f32_to_bf16(pv[2 * k]) | ((unsigned)f32_to_bf16(pv[2 * k + 1]) << 16);
    if constexpr (NV == 8) *reinterpret_cast<uint4*>(shadow + off) = make_uint4(w[0], w[1], w[2], w[3]);
    else *reinterpret_cast<uint2*>(shadow + off) = make_uint2(w[0], w[1]);
  }
}

// Catch-up (deferred dense-parity updates): one wave per row; lane 0 claims
// the row (last[row] <- t) so duplicate ids replay it once; the skipped g = 0
// steps (last, t] are replayed in registers with each step's hyper-parameters,
// rounding bf16 parameters after every step exactly as a store/load would.
// The replayed step range is wave-uniform; the per-step constants of the whole
// ring are computed once per workgroup into LDS (the replay loop then waits on
// no scalar load per step) and the slot advances without a per-step modulo.
// Full flush (ids == null): every row once, so the claim is a plain read and
// store (no atomic) and the row's first vector is loaded before it.
// Rolling flush (ids == null, num_slices > 1): only slice (t mod num_slices) of
// the rows, [s * per, (s + 1) * per) with per = ceil(num_rows / num_slices) --
// one launch per step, captured once in the step's HIP graph, brings every row
// up at least every num_slices steps at a constant per-step cost (the full
// flush's spike of every row once per segment, spread evenly).
constexpr int kCatchupLds = 64;
#ifndef GRK_CATCHUP_PACKED
#define GRK_CATCHUP_PACKED 1
#endif
template <typename P, int NV>
__global__ void __launch_bounds__(256) k_adamw_catchup(P* __restrict__ param, float* __restrict__ m,
                                                       float* __restrict__ v, int64_t num_rows, int dim,
                                                       int32_t* __restrict__ last, const int64_t* __restrict__ ids,
                                                       int64_t num_ids, const grk_adamw_hparams* __restrict__ ring,
                                                       int ring_len, int t_host, const int32_t* __restrict__ t_dev,
                                                       int num_slices) {
  __shared__ AdamStep steps[kCatchupLds];
  const bool staged = ring_len <= kCatchupLds;
  if (staged) {
    for (int i = threadIdx.x; i < ring_len; i += blockDim.x) steps[i] = adam_step(ring[i]);
    __syncthreads();
  }
  const int t = resolve_t(t_host, t_dev);
  const int lane = threadIdx.x & 63;
  // one wave per row; a grid smaller than the rows' waves (the rolling slice under
  // GRK_SLICE_WGS) walks them grid-stride
  const int64_t per = num_slices > 1 ? (num_rows + num_slices - 1) / num_slices : num_rows;
  const int64_t nw = ids ? num_ids : per;
  for (int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); w < nw; w += (int64_t)gridDim.x * 4) {
    const int64_t row = ids ? ids[w] : (num_slices > 1 ? (int64_t)(t % num_slices) * per + w : w);
    if (row < 0 || row >= num_rows) continue;
    float pv[NV], mv[NV], vv[NV];
    int c = lane * NV;
    int from = 0;
    if (ids) {
      // A plain read first: later duplicates of a hot row see the claim without
      // queueing on the atomic; the exchange still decides who replays.
      if (__builtin_nontemporal_load(&last[row]) >= t) continue;
      if (lane == 0) from = atomicExch(&last[row], t);
      from = __builtin_amdgcn_readfirstlane(__shfl(from, 0));
      if (from >= t) continue;
      if (c < dim) load_pmv<P, NV>(param + row * dim + c, m + row * dim + c, v + row * dim + c, pv, mv, vv);
    } else {
      if (c < dim) load_pmv<P, NV>(param + row * dim + c, m + row * dim + c, v + row * dim + c, pv, mv, vv);
      from = __builtin_amdgcn_readfirstlane(last[row]);
      if (from >= t) continue;
      if (lane == 0) last[row] = t;
    }
    const int slot0 = (from + 1) % ring_len;
    for (bool first = true; c < dim; c += 64 * NV, first = false) {
      const int64_t off = row * dim + c;
      if (!first) load_pmv<P, NV>(param + off, m + off, v + off, pv, mv, vv);
      int slot = slot0;
      for (int st = from + 1; st <= t; ++st) {
        const AdamStep s = staged ? steps[slot] : adam_step(ring[slot]);
        slot = slot + 1 == ring_len ? 0 : slot + 1;
#if GRK_CATCHUP_PACKED
#pragma unroll
        for (int e = 0; e < NV; e += 2) {
          f2v p2 = {pv[e], pv[e + 1]}, m2 = {mv[e], mv[e + 1]}, v2 = {vv[e], vv[e + 1]};
          adam2_g0(p2, m2, v2, s);
          pv[e] = p2.x; pv[e + 1] = p2.y; mv[e] = m2.x; mv[e + 1] = m2.y; vv[e] = v2.x; vv[e + 1] = v2.y;
          if constexpr (sizeof(P) == 2) {   // one v_cvt_pk_bf16_f32 per pair, then the two halves back
            typedef __bf16 bf2v __attribute__((ext_vector_type(2)));
            const unsigned w2 = __builtin_bit_cast(unsigned, __builtin_convertvector(p2, bf2v));
            pv[e] = __uint_as_float(w2 << 16);
            pv[e + 1] = __uint_as_float(w2 & 0xFFFF0000u);
          }
        }
#else
#pragma unroll
        for (int e = 0; e < NV; ++e) {
          adam1_g0(pv[e], mv[e], vv[e], s);
          if constexpr (sizeof(P) == 2) pv[e] = bf16_to_f32(f32_to_bf16(pv[e]));
        }
#endif
      }
      store_pmv<P, NV>(param + off, m + off, v + off, pv, mv, vv);
    }
  }
}

__global__ void k_stamp_rows(int32_t* __restrict__ last, const int64_t* __restrict__ ids,
                             const int32_t* __restrict__ count, int64_t max_uniq, int t_host,
                             const int32_t* __restrict__ t_dev) {
  const int t = resolve_t(t_host, t_dev);
  const int64_t n = *count < max_uniq ? *count : max_uniq;
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n; u += (int64_t)gridDim.x * blockDim.x)
    last[ids[u]] = t;
}

template <typename P, int NV>
__global__ void __launch_bounds__(256) k_adamw_lazy(P* __restrict__ param, float* __restrict__ m,
                                                    float* __restrict__ v, int dim,
                                                    const int64_t* __restrict__ uniq_ids,
                                                    const float* __restrict__ uniq_rows,
                                                    const int32_t* __restrict__ count, int64_t max_uniq,
                                                    HpArg hpa) {
  const int q = dim / NV;
  const AdamStep st = adam_step(resolve(hpa));
  const int64_t n = *count;
  const int64_t total = (n < max_uniq ? n : max_uniq) * q;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t u = i / q;
    const int c = (int)(i - u * q) * NV;
    float g[NV];
    load_grad<NV>(uniq_rows + u * dim + c, g);
    const int64_t off = uniq_ids[u] * dim + c;
    adam_vec<P, NV>(param + off, m + off, v + off, g, st);
  }
}

__global__ void k_reset_slots(int32_t* __restrict__ row_slot, const int64_t* __restrict__ uniq_ids,
                              const int32_t* __restrict__ count, int64_t max_uniq) {
  const int64_t n = *count < max_uniq ? *count : max_uniq;
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n; u += (int64_t)gridDim.x * blockDim.x)
    row_slot[uniq_ids[u]] = -1;
}

}  // namespace grk

using namespace grk;

static int table_adamw(void* param, int param_dtype, float* exp_avg, float* exp_avg_sq, int64_t num_rows, int dim,
                       const int64_t* uniq_ids, const float* uniq_rows, const int32_t* uniq_count, int64_t max_uniq,
                       int32_t* row_slot, HpArg hp, int mode, void* stream) {
  clear_error();
  GRK_CHECK_ARG(param && exp_avg && exp_avg_sq, "param / exp_avg / exp_avg_sq required");
  GRK_CHECK_ARG(param_dtype == GRK_F32 || param_dtype == GRK_BF16, "bad param dtype");
  GRK_CHECK_ARG(dim > 0 && dim % 4 == 0, "dim must be a multiple of 4");
  GRK_CHECK_ARG(mode == GRK_ADAM_DENSE || mode == GRK_ADAM_LAZY, "bad mode");
  GRK_CHECK_ARG(mode == GRK_ADAM_DENSE || (uniq_ids && uniq_rows && uniq_count), "lazy mode needs uniq_* inputs");
  GRK_CHECK_ARG(mode == GRK_ADAM_LAZY || !row_slot || uniq_rows, "dense mode with row_slot needs uniq_rows");
  GRK_CHECK_ARG(hp.ring ? (hp.t && hp.ring_len > 0) : hp.hp.bias_corr2_sqrt > 0.f,
                "bias_corr2_sqrt must be > 0 (or a device ring and step)");
  hipStream_t s = (hipStream_t)stream;
  const bool v8 = dim % 8 == 0;
  if (mode == GRK_ADAM_DENSE) {
    const int64_t work = num_rows * (dim / (v8 ? 8 : 4));
    if (work == 0) return GRK_OK;
    GRK_CHECK_ARG((work + 255) / 256 < (int64_t)1 << 31, "table too large for one launch");
    const unsigned g = (unsigned)((work + 255) / 256);
#define GRK_DENSE(P, NV) k_adamw_dense<P, NV><<<g, 256, 0, s>>>((P*)param, exp_avg, exp_avg_sq, num_rows, dim, \
                                                              uniq_rows, row_slot, hp)
    if (param_dtype == GRK_BF16) { if (v8) GRK_DENSE(bf16_t, 8); else GRK_DENSE(bf16_t, 4); }
    else { if (v8) GRK_DENSE(float, 8); else GRK_DENSE(float, 4); }
#undef GRK_DENSE
  } else {
    const int g = grid_for(max_uniq * (dim / (v8 ? 8 : 4)), 256, 256 * 32);
#define GRK_LAZY(P, NV) k_adamw_lazy<P, NV><<<g, 256, 0, s>>>((P*)param, exp_avg, exp_avg_sq, dim, uniq_ids, \
                                                            uniq_rows, uniq_count, max_uniq, hp)
    if (param_dtype == GRK_BF16) { if (v8) GRK_LAZY(bf16_t, 8); else GRK_LAZY(bf16_t, 4); }
    else { if (v8) GRK_LAZY(float, 8); else GRK_LAZY(float, 4); }
#undef GRK_LAZY
  }
  GRK_LAUNCH_CHECK();
  if (row_slot && uniq_ids && uniq_count) {  // without uniq_ids row_slot is a fixed map (e.g. identity)
    k_reset_slots<<<grid_for(max_uniq, 256, 1024), 256, 0, s>>>(row_slot, uniq_ids, uniq_count, max_uniq);
    GRK_LAUNCH_CHECK();
  }
  return GRK_OK;
}

static int table_adamw_dense(void* param, int param_dtype, float* exp_avg, float* exp_avg_sq, int64_t num_rows,
                             int dim, const void* grad, int grad_dtype, int64_t grad_ld, HpArg hp, void* stream) {
  clear_error();
  GRK_CHECK_ARG(num_rows >= 0, "num_rows must be >= 0");
  if (num_rows == 0) return GRK_OK;
  GRK_CHECK_ARG(param && exp_avg && exp_avg_sq && grad, "param / exp_avg / exp_avg_sq / grad required");
  GRK_CHECK_ARG(param_dtype == GRK_F32 || param_dtype == GRK_BF16, "bad param dtype");
  GRK_CHECK_ARG(grad_dtype == GRK_F32 || grad_dtype == GRK_BF16, "bad grad dtype");
  GRK_CHECK_ARG(dim > 0 && dim % 4 == 0 && grad_ld >= dim && grad_ld % 4 == 0, "dim / grad_ld must be multiples of 4");
  GRK_CHECK_ARG(hp.ring ? (hp.t && hp.ring_len > 0) : hp.hp.bias_corr2_sqrt > 0.f,
                "bias_corr2_sqrt must be > 0 (or a device ring and step)");
  const bool v8 = dim % 8 == 0 && grad_ld % 8 == 0;
  const int64_t work = num_rows * (dim / (v8 ? 8 : 4));
  GRK_CHECK_ARG((work + 255) / 256 < (int64_t)1 << 31, "table too large for one launch");
  const unsigned g = (unsigned)((work + 255) / 256);
  hipStream_t s = (hipStream_t)stream;
#define GRK_DG(P, GT, NV) k_adamw_dense_grad<P, GT, NV><<<g, 256, 0, s>>>((P*)param, exp_avg, exp_avg_sq, num_rows, \
                                                                         dim, (const GT*)grad, grad_ld, hp)
  if (param_dtype == GRK_BF16) {
    if (grad_dtype == GRK_BF16) { if (v8) GRK_DG(bf16_t, bf16_t, 8); else GRK_DG(bf16_t, bf16_t, 4); }
    else { if (v8) GRK_DG(bf16_t, float, 8); else GRK_DG(bf16_t, float, 4); }
  } else {
    if (grad_dtype == GRK_BF16) { if (v8) GRK_DG(float, bf16_t, 8); else GRK_DG(float, bf16_t, 4); }
    else { if (v8) GRK_DG(float, float, 8); else GRK_DG(float, float, 4); }
  }
#undef GRK_DG
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}


static int table_adamw_catchup(void* param, int param_dtype, float* exp_avg, float* exp_avg_sq, int64_t num_rows,
                               int dim, int32_t* last, const int64_t* ids, int64_t num_ids,
                               const grk_adamw_hparams* hp_ring, int32_t ring_len, int32_t t, const int32_t* t_dev,
                               void* stream, int32_t num_slices = 1) {
  clear_error();
  GRK_CHECK_ARG(num_rows >= 0 && num_ids >= 0, "num_rows / num_ids must be >= 0");
  GRK_CHECK_ARG(num_slices >= 1 && (num_slices == 1 || !ids), "num_slices >= 1 (and > 1 only without ids)");
  const int64_t waves = ids ? num_ids : (num_rows + num_slices - 1) / num_slices;
  if (waves == 0) return GRK_OK;
  GRK_CHECK_ARG(param && exp_avg && exp_avg_sq && last && hp_ring, "param / moments / last / hp_ring required");
  GRK_CHECK_ARG(param_dtype == GRK_F32 || param_dtype == GRK_BF16, "bad param dtype");
  GRK_CHECK_ARG(dim > 0 && dim % 4 == 0, "dim must be a multiple of 4");
  GRK_CHECK_ARG(ring_len > 0 && t >= 0, "ring_len must be > 0 and t >= 0");
  GRK_CHECK_ARG((waves + 3) / 4 < (int64_t)1 << 31, "too many rows for one launch");
  unsigned g = (unsigned)((waves + 3) / 4);
  // rolling slice: at most kSliceWgs workgroups, walking the slice's rows grid-stride --
  // the slice then holds a bounded share of the CUs while it runs beside the step on its
  // side stream, instead of flooding every CU at launch (512 = two per CU, measured best:
  // 3.99 vs 4.04 ms/step with the full grid, 4.11 at 256)
  constexpr unsigned kSliceWgs = 512;
  if (!ids && num_slices > 1 && g > kSliceWgs) g = kSliceWgs;
  hipStream_t s = (hipStream_t)stream;
  const bool v8 = dim % 8 == 0;
#define GRK_CU(P, NV) k_adamw_catchup<P, NV><<<g, 256, 0, s>>>((P*)param, exp_avg, exp_avg_sq, num_rows, dim, last, \
                                                               ids, num_ids, hp_ring, ring_len, t, t_dev, \
                                                               num_slices)
  if (param_dtype == GRK_BF16) { if (v8) GRK_CU(bf16_t, 8); else GRK_CU(bf16_t, 4); }
  else { if (v8) GRK_CU(float, 8); else GRK_CU(float, 4); }
#undef GRK_CU
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

static int stamp_rows(int32_t* last, const int64_t* uniq_ids, const int32_t* uniq_count, int64_t max_uniq,
                      int32_t t, const int32_t* t_dev, void* stream) {
  clear_error();
  if (max_uniq <= 0) return GRK_OK;
  GRK_CHECK_ARG(last && uniq_ids && uniq_count, "last / uniq_ids / uniq_count required");
  k_stamp_rows<<<grid_for(max_uniq, 256, 1024), 256, 0, (hipStream_t)stream>>>(last, uniq_ids, uniq_count, max_uniq, t,
                                                                               t_dev);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

static HpArg by_value(grk_adamw_hparams hp) { return HpArg{hp, nullptr, nullptr, 0, nullptr}; }
static HpArg on_device(const grk_adamw_hparams* ring, int32_t ring_len, const int32_t* t) {
  HpArg a{};
  a.ring = ring;
  a.t = t;
  a.ring_len = ring_len;
  return a;
}

extern "C" int grk_table_adamw(void* param, int param_dtype, float* exp_avg, float* exp_avg_sq, int64_t num_rows,
                               int dim, const int64_t* uniq_ids, const float* uniq_rows, const int32_t* uniq_count,
                               int64_t max_uniq, int32_t* row_slot, grk_adamw_hparams hp, int mode, void* stream) {
  return table_adamw(param, param_dtype, exp_avg, exp_avg_sq, num_rows, dim, uniq_ids, uniq_rows, uniq_count,
                     max_uniq, row_slot, by_value(hp), mode, stream);
}

extern "C" int grk_table_adamw_dev(void* param, int param_dtype, float* exp_avg, float* exp_avg_sq, int64_t num_rows,
                                   int dim, const int64_t* uniq_ids, const float* uniq_rows, const int32_t* uniq_count,
                                   int64_t max_uniq, int32_t* row_slot, const grk_adamw_hparams* hp_ring,
                                   int32_t ring_len, const int32_t* t_dev, int mode, void* stream) {
  if (!hp_ring || !t_dev || ring_len <= 0) { set_error("hp_ring / t_dev / ring_len required"); return GRK_EINVAL; }
  return table_adamw(param, param_dtype, exp_avg, exp_avg_sq, num_rows, dim, uniq_ids, uniq_rows, uniq_count,
                     max_uniq, row_slot, on_device(hp_ring, ring_len, t_dev), mode, stream);
}

extern "C" int grk_table_adamw_dense(void* param, int param_dtype, float* exp_avg, float* exp_avg_sq,
                                     int64_t num_rows, int dim, const void* grad, int grad_dtype, int64_t grad_ld,
                                     grk_adamw_hparams hp, void* stream) {
  return table_adamw_dense(param, param_dtype, exp_avg, exp_avg_sq, num_rows, dim, grad, grad_dtype, grad_ld,
                           by_value(hp), stream);
}

extern "C" int grk_table_adamw_dense_dev(void* param, int param_dtype, float* exp_avg, float* exp_avg_sq,
                                         int64_t num_rows, int dim, const void* grad, int grad_dtype, int64_t grad_ld,
                                         const grk_adamw_hparams* hp_ring, int32_t ring_len, const int32_t* t_dev,
                                         void* stream) {
  if (!hp_ring || !t_dev || ring_len <= 0) { set_error("hp_ring / t_dev / ring_len required"); return GRK_EINVAL; }
  return table_adamw_dense(param, param_dtype, exp_avg, exp_avg_sq, num_rows, dim, grad, grad_dtype, grad_ld,
                           on_device(hp_ring, ring_len, t_dev), stream);
}

extern "C" int grk_table_adamw_catchup(void* param, int param_dtype, float* exp_avg, float* exp_avg_sq,
                                       int64_t num_rows, int dim, int32_t* last, const int64_t* ids, int64_t num_ids,
                                       const grk_adamw_hparams* hp_ring, int32_t ring_len, int32_t t, void* stream) {
  return table_adamw_catchup(param, param_dtype, exp_avg, exp_avg_sq, num_rows, dim, last, ids, num_ids, hp_ring,
                             ring_len, t, nullptr, stream);
}

extern "C" int grk_table_adamw_catchup_dev(void* param, int param_dtype, float* exp_avg, float* exp_avg_sq,
                                           int64_t num_rows, int dim, int32_t* last, const int64_t* ids,
                                           int64_t num_ids, const grk_adamw_hparams* hp_ring, int32_t ring_len,
                                           const int32_t* t_dev, void* stream) {
  if (!t_dev) { set_error("t_dev required"); return GRK_EINVAL; }
  return table_adamw_catchup(param, param_dtype, exp_avg, exp_avg_sq, num_rows, dim, last, ids, num_ids, hp_ring,
                             ring_len, 0, t_dev, stream);
}

extern "C" int grk_table_adamw_catchup_slice_dev(void* param, int param_dtype, float* exp_avg, float* exp_avg_sq,
                                                 int64_t num_rows, int dim, int32_t* last,
                                                 const grk_adamw_hparams* hp_ring, int32_t ring_len,
                                                 const int32_t* t_dev, int32_t num_slices, void* stream) {
  if (!t_dev) { set_error("t_dev required"); return GRK_EINVAL; }
  return table_adamw_catchup(param, param_dtype, exp_avg, exp_avg_sq, num_rows, dim, last, nullptr, 0, hp_ring,
                             ring_len, 0, t_dev, stream, num_slices);
}

extern "C" int grk_stamp_rows(int32_t* last, const int64_t* uniq_ids, const int32_t* uniq_count, int64_t max_uniq,
                              int32_t t, void* stream) {
  return stamp_rows(last, uniq_ids, uniq_count, max_uniq, t, nullptr, stream);
}

extern "C" int grk_stamp_rows_dev(int32_t* last, const int64_t* uniq_ids, const int32_t* uniq_count, int64_t max_uniq,
                                  const int32_t* t_dev, void* stream) {
  if (!t_dev) { set_error("t_dev required"); return GRK_EINVAL; }
  return stamp_rows(last, uniq_ids, uniq_count, max_uniq, 0, t_dev, stream);
}

extern "C" int grk_table_adamw_l2_dev(void* param, int param_dtype, float* exp_avg, float* exp_avg_sq,
                                      int64_t num_rows, int dim, const int64_t* uniq_ids, const float* uniq_rows,
                                      const int32_t* uniq_count, int64_t max_uniq, int32_t* row_slot,
                                      const grk_adamw_hparams* hp_ring, int32_t ring_len, const int32_t* t_dev,
                                      const float* l2_coef, void* stream) {
  if (!hp_ring || !t_dev || ring_len <= 0) { set_error("hp_ring / t_dev / ring_len required"); return GRK_EINVAL; }
  if (!l2_coef) { set_error("l2_coef required"); return GRK_EINVAL; }
  HpArg hp = on_device(hp_ring, ring_len, t_dev);
  hp.l2coef = l2_coef;
  return table_adamw(param, param_dtype, exp_avg, exp_avg_sq, num_rows, dim, uniq_ids, uniq_rows, uniq_count,
                     max_uniq, row_slot, hp, GRK_ADAM_DENSE, stream);
}

extern "C" size_t grk_table_l2_norm_workspace(void) { return (size_t)kNormBlocks * sizeof(double); }

extern "C" int grk_table_l2_norm(const void* param, int param_dtype, int64_t num_rows, int dim, float l2, float* norm,
                                 float* l2_coef, void* workspace, size_t workspace_bytes, void* stream) {
  clear_error();
  GRK_CHECK_ARG(num_rows >= 0 && dim > 0, "bad table shape");
  GRK_CHECK_ARG(param_dtype == GRK_F32 || param_dtype == GRK_BF16, "bad param dtype");
  GRK_CHECK_ARG(norm && workspace, "norm / workspace required");
  GRK_CHECK_ARG(workspace_bytes >= grk_table_l2_norm_workspace(), "workspace too small");
  GRK_CHECK_ARG(num_rows == 0 || param, "param required");
  GRK_CHECK_ARG((uintptr_t)param % 16 == 0, "param must be 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  const int64_t n = num_rows * (int64_t)dim;
  double* part = (double*)workspace;
  if (param_dtype == GRK_BF16) k_table_sumsq<bf16_t><<<kNormBlocks, 256, 0, s>>>((const bf16_t*)param, n, part);
  else k_table_sumsq<float><<<kNormBlocks, 256, 0, s>>>((const float*)param, n, part);
  GRK_LAUNCH_CHECK();
  k_table_norm_final<<<1, 256, 0, s>>>(part, l2, norm, l2_coef);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

extern "C" int grk_table_adamw_ranges_dev(void* param, int param_dtype, float* exp_avg, float* exp_avg_sq,
                                          int64_t num_rows, int dim, const grk_grad_range* ranges, int num_ranges,
                                          const grk_adamw_hparams* hp_ring, int32_t ring_len, const int32_t* t_dev,
                                          void* shadow, void* stream) {
  clear_error();
  GRK_CHECK_ARG(num_rows >= 0, "num_rows must be >= 0");
  if (num_rows == 0) return GRK_OK;
  GRK_CHECK_ARG(param && exp_avg && exp_avg_sq, "param / exp_avg / exp_avg_sq required");
  GRK_CHECK_ARG(param_dtype == GRK_F32 || param_dtype == GRK_BF16, "bad param dtype");
  GRK_CHECK_ARG(!shadow || (param_dtype == GRK_F32 && (uintptr_t)shadow % 16 == 0),
                "shadow: fp32 params only, 16-byte aligned");
  GRK_CHECK_ARG(dim > 0 && dim % 4 == 0, "dim must be a multiple of 4");
  GRK_CHECK_ARG(hp_ring && t_dev && ring_len > 0, "hp_ring / t_dev / ring_len required");
  GRK_CHECK_ARG(num_ranges >= 0 && num_ranges <= kMaxGradRanges, "num_ranges must be in [0, %d]", kMaxGradRanges);
  GradRanges gr;
  memset(&gr, 0, sizeof(gr));
  gr.n = num_ranges;
  bool v8 = dim % 8 == 0;
  int64_t prev_end = 0;
  for (int i = 0; i < num_ranges; ++i) {
    const grk_grad_range& r = ranges[i];
    GRK_CHECK_ARG(r.grad && r.row_start >= prev_end && r.row_end > r.row_start && r.row_end <= num_rows,
                  "range %d: rows [%lld, %lld) must be sorted, disjoint, non-empty and inside the table", i,
                  (long long)r.row_start, (long long)r.row_end);
    GRK_CHECK_ARG(r.grad_dtype == GRK_F32 || r.grad_dtype == GRK_BF16, "range %d: bad grad dtype", i);
    GRK_CHECK_ARG(r.grad_ld >= dim && r.grad_ld % 4 == 0, "range %d: grad_ld must be >= dim, multiple of 4", i);
    v8 = v8 && r.grad_ld % 8 == 0;
    prev_end = r.row_end;
    gr.r[i] = r;
  }
  const int64_t work = num_rows * (dim / (v8 ? 8 : 4));
  GRK_CHECK_ARG((work + 255) / 256 < (int64_t)1 << 31, "table too large for one launch");
  const unsigned g = (unsigned)((work + 255) / 256);
  hipStream_t s = (hipStream_t)stream;
  const HpArg hp = on_device(hp_ring, ring_len, t_dev);
#define GRK_RG(P, NV) \
  k_adamw_ranges<P, NV><<<g, 256, 0, s>>>((P*)param, exp_avg, exp_avg_sq, num_rows, dim, gr, hp, (bf16_t*)shadow)
  if (param_dtype == GRK_BF16) { if (v8) GRK_RG(bf16_t, 8); else GRK_RG(bf16_t, 4); }
  else { if (v8) GRK_RG(float, 8); else GRK_RG(float, 4); }
#undef GRK_RG
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}
