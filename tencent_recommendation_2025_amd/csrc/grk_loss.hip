// Pair logits + BCE loss for gfx950.
//
// Replaces, in one pass over h / e_pos / e_neg:
//   pos_logits = (log_feats * pos_embs).sum(-1) * loss_mask     model/BaseLine/model.py:379-382
//   neg_logits = (log_feats * neg_embs).sum(-1) * loss_mask
//   loss = BCEWithLogits(pos[idx], 1) + BCEWithLogits(neg[idx], 0),
//          idx = np.where(next_token_type == 1)                   model/BaseLine/main.py:177-182
// The index set is never materialised on the host: the count lives on the
// device, so the step has no host sync.  The loss is reduced in a fixed
// order (per-block partials, then one block), so it is deterministic.
// HBM-bound: 3 x N x D elements read forward, 3 read + 3 written backward.
// h and the item embeddings may differ in dtype (GRK_F32_BF16: fp32 h from the
// last LayerNorm, bf16 e_pos / e_neg from the item dnn under autocast): read as
// they are, with the fp32 path's chunking and summation order, so the logits
// equal those of promoting e to fp32 first, bitwise -- without the casts.
#include "grk_common.h"

namespace grk {

template <typename T, int N> struct VecN;
template <> struct VecN<float, 4> : Vec16<float> {};
template <> struct VecN<bf16_t, 8> : Vec16<bf16_t> {};
template <> struct VecN<bf16_t, 4> {  // 4 bf16 (8 bytes)
  uint2 v;
  __device__ __forceinline__ void load(const bf16_t* p) { v = *reinterpret_cast<const uint2*>(p); }
  __device__ __forceinline__ void store(bf16_t* p) const { *reinterpret_cast<uint2*>(p) = v; }
  __device__ __forceinline__ float get(int i) const {
    const unsigned w = (&v.x)[i >> 1];
    return __uint_as_float((i & 1) ? (w & 0xFFFF0000u) : (w << 16));
  }
  __device__ __forceinline__ void set(int i, float f) {
    const unsigned b = f32_to_bf16(f);
    unsigned& w = (&v.x)[i >> 1];
    w = (i & 1) ? ((w & 0x0000FFFFu) | (b << 16)) : ((w & 0xFFFF0000u) | b);
  }
};
template <typename TH, typename TE>
constexpr int pair_vec() { return (sizeof(TH) == 4 || sizeof(TE) == 4) ? 4 : 8; }

__device__ __forceinline__ float softplus(float x) { return fmaxf(x, 0.f) + log1pf(__expf(-fabsf(x))); }
__device__ __forceinline__ float sigmoidf(float x) { return 1.0f / (1.0f + __expf(-x)); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// One wave per row; lanes stride over 16-byte chunks of the row.
template <typename TH, typename TE>
__global__ void __launch_bounds__(256) k_pair_logits(const TH* __restrict__ h, int64_t ldh, const TE* __restrict__ ep,
                                                     int64_t ldp, const TE* __restrict__ en, int64_t ldn,
                                                     const int32_t* __restrict__ ntt, int64_t N, int D,
                                                     float* __restrict__ pos_out, float* __restrict__ neg_out,
                                                     float* __restrict__ partials) {
  constexpr int VEC = pair_vec<TH, TE>();
  __shared__ float red[3][4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t n = (int64_t)blockIdx.x * 4 + wave;
  float lp = 0.f, ln = 0.f, cnt = 0.f;
  if (n < N) {
    float sp = 0.f, sn = 0.f;
    for (int c = lane * VEC; c < D; c += 64 * VEC) {
      VecN<TH, VEC> a;
      VecN<TE, VEC> b, d;
      a.load(h + n * ldh + c);
      b.load(ep + n * ldp + c);
      d.load(en + n * ldn + c);
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        sp = fmaf(a.get(e), b.get(e), sp);
        sn = fmaf(a.get(e), d.get(e), sn);
      }
    }
    sp = wave_sum(sp);
    sn = wave_sum(sn);
    const bool valid = ntt ? ntt[n] == 1 : true;
    const float pl = valid ? sp : 0.f, nl = valid ? sn : 0.f;
    if (lane == 0) {
      if (pos_out) pos_out[n] = pl;
      if (neg_out) neg_out[n] = nl;
    }
    if (valid) {
      lp = softplus(-pl);
      ln = softplus(nl);
      cnt = 1.f;
    }
  }
  if (partials) {
    if (lane == 0) { red[0][wave] = lp; red[1][wave] = ln; red[2][wave] = cnt; }
    __syncthreads();
    if (threadIdx.x < 3) {
      const int k = threadIdx.x;
      partials[(int64_t)blockIdx.x * 3 + k] = ((red[k][0] + red[k][1]) + red[k][2]) + red[k][3];
    }
  }
}

// Fixed-order reduction of the per-block partials -> loss, count.
__global__ void __launch_bounds__(1024) k_bce_finalize(const float* __restrict__ partials, int64_t nblocks,
                                                       float* __restrict__ loss, int32_t* __restrict__ count) {
  __shared__ double red[3][1024];
  double a[3] = {0.0, 0.0, 0.0};
  for (int64_t i = threadIdx.x; i < nblocks; i += blockDim.x)
#pragma unroll
    for (int k = 0; k < 3; ++k) a[k] += (double)partials[i * 3 + k];
#pragma unroll
  for (int k = 0; k < 3; ++k) red[k][threadIdx.x] = a[k];
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s)
#pragma unroll
      for (int k = 0; k < 3; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double c = red[2][0];
    const double cc = c > 0 ? c : 1.0;
    loss[0] = (float)(red[0][0] / cc + red[1][0] / cc);
    count[0] = (int32_t)c;
  }
}

// dh = gp*e_pos + gn*e_neg ; de_pos = gp*h ; de_neg = gn*h.
// mode 0: gp, gn given per row.  mode 1: BCE coefficients from the logits:
//   gp = g*(sigmoid(pos)-1)/cnt, gn = g*sigmoid(neg)/cnt on valid rows.
template <typename TH, typename TE>
__global__ void __launch_bounds__(256) k_pair_logits_bwd(const TH* __restrict__ h, int64_t ldh,
                                                         const TE* __restrict__ ep, int64_t ldp,
                                                         const TE* __restrict__ en, int64_t ldn, int64_t N, int D,
                                                         int mode, const float* __restrict__ gpos,
                                                         const float* __restrict__ gneg,
                                                         const float* __restrict__ pos_logits,
                                                         const float* __restrict__ neg_logits,
                                                         const int32_t* __restrict__ ntt,
                                                         const int32_t* __restrict__ count,
                                                         const float* __restrict__ grad_loss, TH* __restrict__ dh,
                                                         int64_t lddh, TE* __restrict__ dep, int64_t lddp,
                                                         TE* __restrict__ den, int64_t lddn) {
  constexpr int VEC = pair_vec<TH, TE>();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t n = (int64_t)blockIdx.x * 4 + wave;
  if (n >= N) return;
  float gp, gn;
  if (mode == 0) {
    const bool valid = ntt ? ntt[n] == 1 : true;  // the forward zeroed masked logits
    gp = (gpos && valid) ? gpos[n] : 0.f;
    gn = (gneg && valid) ? gneg[n] : 0.f;
  } else {
    const bool valid = ntt ? ntt[n] == 1 : true;
    const float c = (float)max(*count, 1);
    const float g = grad_loss ? *grad_loss : 1.f;
    gp = valid ? g * (sigmoidf(pos_logits[n]) - 1.0f) / c : 0.f;
    gn = valid ? g * sigmoidf(neg_logits[n]) / c : 0.f;
  }
  for (int c = lane * VEC; c < D; c += 64 * VEC) {
    VecN<TH, VEC> a, oh;
    VecN<TE, VEC> b, d, op, on;
    a.load(h + n * ldh + c);
    b.load(ep + n * ldp + c);
    d.load(en + n * ldn + c);
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      const float hv = a.get(e);
      oh.set(e, fmaf(gp, b.get(e), gn * d.get(e)));  // explicit: the same rounding in every dtype instantiation
      op.set(e, gp * hv);
      on.set(e, gn * hv);
    }
    if (dh) oh.store(dh + n * lddh + c);
    if (dep) op.store(dep + n * lddp + c);
    if (den) on.store(den + n * lddn + c);
  }
}

}  // namespace grk

using namespace grk;

static int check_rows(const void* p, int64_t ld, int D, int vec, const char* name) {
  GRK_CHECK_ARG(p && ld >= D && ld % vec == 0 && ((uintptr_t)p % 16) == 0,
                "%s: needs a 16-byte aligned row-major matrix with ld >= D (multiple of %d)", name, vec);
  return GRK_OK;
}

extern "C" size_t grk_pair_logits_partials(int64_t num_rows) { return (size_t)((num_rows + 3) / 4) * 3; }

extern "C" int grk_pair_logits_fwd(const void* h, int64_t ldh, const void* e_pos, int64_t ldp, const void* e_neg,
                                   int64_t ldn, const int32_t* next_token_type, int64_t num_rows, int dim, int dtype,
                                   float* pos_logits, float* neg_logits, float* partials, float* loss,
                                   int32_t* count, void* stream) {
  clear_error();
  GRK_CHECK_ARG(dtype == GRK_F32 || dtype == GRK_BF16 || dtype == GRK_F32_BF16, "bad dtype");
  const int vec = dtype == GRK_BF16 ? 8 : 4;
  GRK_CHECK_ARG(dim > 0 && dim % vec == 0, "dim must be a positive multiple of %d", vec);
  GRK_CHECK_ARG(num_rows >= 0, "num_rows < 0");
  GRK_CHECK_ARG(!loss || (partials && count), "loss needs partials and count");
  if (num_rows == 0) {
    if (loss) {
      GRK_CHECK_HIP(zero_async(loss, 4, (hipStream_t)stream));
      GRK_CHECK_HIP(zero_async(count, 4, (hipStream_t)stream));
    }
    return GRK_OK;
  }
  int rc;
  if ((rc = check_rows(h, ldh, dim, vec, "h")) || (rc = check_rows(e_pos, ldp, dim, vec, "e_pos")) ||
      (rc = check_rows(e_neg, ldn, dim, vec, "e_neg")))
    return rc;
  hipStream_t s = (hipStream_t)stream;
  const int64_t blocks = (num_rows + 3) / 4;
  if (dtype == GRK_BF16)
    k_pair_logits<bf16_t, bf16_t><<<(unsigned)blocks, 256, 0, s>>>((const bf16_t*)h, ldh, (const bf16_t*)e_pos, ldp,
                                                                   (const bf16_t*)e_neg, ldn, next_token_type,
                                                                   num_rows, dim, pos_logits, neg_logits, partials);
  else if (dtype == GRK_F32_BF16)
    k_pair_logits<float, bf16_t><<<(unsigned)blocks, 256, 0, s>>>((const float*)h, ldh, (const bf16_t*)e_pos, ldp,
                                                                  (const bf16_t*)e_neg, ldn, next_token_type,
                                                                  num_rows, dim, pos_logits, neg_logits, partials);
  else
    k_pair_logits<float, float><<<(unsigned)blocks, 256, 0, s>>>((const float*)h, ldh, (const float*)e_pos, ldp,
                                                                 (const float*)e_neg, ldn, next_token_type, num_rows,
                                                                 dim, pos_logits, neg_logits, partials);
  GRK_LAUNCH_CHECK();
  if (loss) {
    k_bce_finalize<<<1, 1024, 0, s>>>(partials, blocks, loss, count);
    GRK_LAUNCH_CHECK();
  }
  return GRK_OK;
}

extern "C" int grk_pair_logits_bwd(const void* h, int64_t ldh, const void* e_pos, int64_t ldp, const void* e_neg,
                                   int64_t ldn, int64_t num_rows, int dim, int dtype, const float* gpos,
                                   const float* gneg, const float* pos_logits, const float* neg_logits,
                                   const int32_t* next_token_type, const int32_t* count, const float* grad_loss,
                                   void* dh, int64_t lddh, void* de_pos, int64_t lddp, void* de_neg, int64_t lddn,
                                   void* stream) {
  clear_error();
  GRK_CHECK_ARG(dtype == GRK_F32 || dtype == GRK_BF16 || dtype == GRK_F32_BF16, "bad dtype");
  const int vec = dtype == GRK_BF16 ? 8 : 4;
  GRK_CHECK_ARG(dim > 0 && dim % vec == 0, "dim must be a positive multiple of %d", vec);
  const int mode = (pos_logits || neg_logits) ? 1 : 0;
  GRK_CHECK_ARG(mode == 0 || (pos_logits && neg_logits && count), "BCE mode needs pos/neg logits and count");
  if (num_rows == 0) return GRK_OK;
  int rc;
  if ((rc = check_rows(h, ldh, dim, vec, "h")) || (rc = check_rows(e_pos, ldp, dim, vec, "e_pos")) ||
      (rc = check_rows(e_neg, ldn, dim, vec, "e_neg")))
    return rc;
  if (dh && (rc = check_rows(dh, lddh, dim, vec, "dh"))) return rc;
  if (de_pos && (rc = check_rows(de_pos, lddp, dim, vec, "de_pos"))) return rc;
  if (de_neg && (rc = check_rows(de_neg, lddn, dim, vec, "de_neg"))) return rc;
  hipStream_t s = (hipStream_t)stream;
  const int64_t blocks = (num_rows + 3) / 4;
  if (dtype == GRK_F32_BF16)
    k_pair_logits_bwd<float, bf16_t><<<(unsigned)blocks, 256, 0, s>>>(
        (const float*)h, ldh, (const bf16_t*)e_pos, ldp, (const bf16_t*)e_neg, ldn, num_rows, dim, mode, gpos, gneg,
        pos_logits, neg_logits, next_token_type, count, grad_loss, (float*)dh, lddh, (bf16_t*)de_pos, lddp,
        (bf16_t*)de_neg, lddn);
  else if (dtype == GRK_BF16)
    k_pair_logits_bwd<bf16_t, bf16_t><<<(unsigned)blocks, 256, 0, s>>>(
        (const bf16_t*)h, ldh, (const bf16_t*)e_pos, ldp, (const bf16_t*)e_neg, ldn, num_rows, dim, mode, gpos, gneg,
        pos_logits, neg_logits, next_token_type, count, grad_loss, (bf16_t*)dh, lddh, (bf16_t*)de_pos, lddp,
        (bf16_t*)de_neg, lddn);
  else
    k_pair_logits_bwd<float, float><<<(unsigned)blocks, 256, 0, s>>>(
        (const float*)h, ldh, (const float*)e_pos, ldp, (const float*)e_neg, ldn, num_rows, dim, mode, gpos, gneg,
        pos_logits, neg_logits, next_token_type, count, grad_loss, (float*)dh, lddh, (float*)de_pos, lddp,
        (float*)de_neg, lddn);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}
