// Causal attention for wide heads (head_dim 256 / 512) on gfx950.
//
// The O1 baseline runs one head over the whole hidden width
// (model/BaseLineO1/main.py:45 num_heads=1, hidden_units up to 512 in
// BASELINE config 4); the chunked kernels of grk_attention.hip keep a whole
// head row per lane in registers, which stops at head_dim 128.  Here a
// workgroup owns 32 rows -- queries (forward, dQ) or keys (dK/dV) of one
// (batch, head) -- and its HD/64 waves split the head's columns into 64-wide
// slices (4 waves at 256, 8 at 512): every wave forms the partial 32x32
// score (and dP) product of its slice, the partials are exchanged through LDS and summed in wave order
// (every wave then holds bitwise the same S / dP, so the softmax state and
// the element math agree without further traffic), and each wave multiplies
// P / dS into its own column slice of O / dQ / dK / dV.  K/V (or Q/dO) tiles
// of 32 rows x HD are staged through the same swizzled LDS image as the
// chunked kernels.  Element math, masks, dropout and the HSTU pointwise form
// are those of grk_attention.hip (same drop_keep stream, same lse / delta
// conventions), so the backward of either path reads the other's forward.
// fp32-fidelity (precise = 2) is not offered for these widths.
#include "grk_attention.h"

namespace grk {
namespace {

constexpr int kWRows = 32;   // queries (fwd, dQ) or keys (dK/dV) per workgroup
constexpr int kWTail = 304;  // kvs[32] | s_start | lses[32] | dlts[32], then rab (+ drab bins)

template <int HD>
struct Wide {
  static constexpr int NW = HD / 64, NT = 64 * NW;  // column slices = waves
  static constexpr int DQ = 64, KSQ = DQ / 16, NDT = DQ / 32;
  static constexpr int IMG = kWRows * HD * 2;   // one 32-row bf16 image
  static constexpr int RED = NW * 4 * 64 * 16;  // one f32x16 per lane per wave
};

__device__ __forceinline__ void red_put(float4* red, int w, int lane, const f32x16& x) {
#pragma unroll
  for (int q = 0; q < 4; ++q) red[(w * 4 + q) * 64 + lane] = make_float4(x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]);
}

// Sum of the NW waves' partials, in wave order (identical in every wave).
template <int NW>
__device__ __forceinline__ f32x16 red_sum(const float4* red, int lane) {
  f32x16 s;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 a = red[q * 64 + lane];
    s[4 * q] = a.x; s[4 * q + 1] = a.y; s[4 * q + 2] = a.z; s[4 * q + 3] = a.w;
  }
#pragma unroll 1
  for (int w = 1; w < NW; ++w)  // streamed: 8 waves' partials at once would not fit the registers
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 a = red[(w * 4 + q) * 64 + lane];
      s[4 * q] += a.x; s[4 * q + 1] += a.y; s[4 * q + 2] += a.z; s[4 * q + 3] += a.w;
    }
  return s;
}

__device__ __forceinline__ void* shift(void* p, bool f32, int n) { return (char*)p + (size_t)n * (f32 ? 4 : 2); }

// ================================================================ forward ====
template <int HD, int KIND>
__global__ void __launch_bounds__(HD) k_attn_fwd_wide(AttnParams p) {
  using W = Wide<HD>;
  constexpr int KSQ = W::KSQ, NDT = W::NDT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Ks = smem;
  char* Vs = smem + W::IMG;
  float4* red = reinterpret_cast<float4*>(smem + 2 * W::IMG);
  char* tail = smem + 2 * W::IMG + W::RED;
  uint8_t* kvs = reinterpret_cast<uint8_t*>(tail);
  int* s_start = reinterpret_cast<int*>(tail + 32);
  float* rabs = reinterpret_cast<float*>(tail + kWTail);

  const int b = blockIdx.z, h = blockIdx.y, T = p.T;
  const int ws = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int q0 = blockIdx.x * kWRows, myq = q0 + r;
  const bool qok = myq < T;
  const int start = seq_start(p.key_valid, b, T, s_start);
  if (KIND == 1)
    for (int j = threadIdx.x; j < p.nb; j += blockDim.x) rabs[j] = p.rab[h * p.nb + j];
  const int c0 = ws * W::DQ;  // this wave's columns within the head

  bf16x8 qf[KSQ];
  const bf16_t* qrow = p.q + ((int64_t)b * T + (qok ? myq : 0)) * p.ldq + h * HD + c0;
#pragma unroll
  for (int ks = 0; ks < KSQ; ++ks) {
    qf[ks] = gload8(qrow + 16 * ks + 8 * hh, qok);
    if (p.act) qf[ks] = silu8(qf[ks]);
  }
  f32x16 o[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) o[dt] = f32x16{};
  float m = -INFINITY, l = 0.f;
  const float sl2 = p.scale * kLog2e;
  const float rdrop = 1.0f / (1.0f - p.dropout_p);
  const bool drop = KIND == 0 && p.dropout_p > 0.f;
  const unsigned long long seed = drop ? attn_seed(p) : 0ull;
  const int bh = b * p.H + h;

  const int kend = min(T, q0 + kWRows);
  for (int kb = (start / 32) * 32; kb < kend; kb += 32) {
    __syncthreads();
    stage_rows_at<HD>(Ks, p.k, p.ldk, b, T, h, kb, 32, 0, false, p.act);
    stage_rows_at<HD>(Vs, p.v, p.ldv, b, T, h, kb, 32, 0, false, p.act);
    if (threadIdx.x < 32) {
      const int t = kb + threadIdx.x;
      kvs[threadIdx.x] = (t < T) && (!p.key_valid || p.key_valid[(int64_t)b * T + t]);
    }
    __syncthreads();
    f32x16 s = f32x16{};
#pragma unroll
    for (int ks = 0; ks < KSQ; ++ks) s = mfma(lds_row8<HD>(Ks, r, c0 + 16 * ks + 8 * hh), qf[ks], s);
    red_put(red, ws, lane, s);
    __syncthreads();
    s = red_sum<W::NW>(red, lane);
    float pd[16];
    if (KIND == 0) {
      float x[16], pr[16], tmax = -INFINITY;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int kr = acc_row(i, hh), key = kb + kr;
        const bool ok = qok && key <= myq && kvs[kr];
        x[i] = ok ? s[i] * sl2 : -INFINITY;
        tmax = fmaxf(tmax, x[i]);
      }
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
      const float mn = fmaxf(m, tmax);
      const float alpha = (mn == -INFINITY) ? 1.f : exp2f(m - mn);
      float rs = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        pr[i] = (x[i] == -INFINITY) ? 0.f : exp2f(x[i] - mn);
        rs += pr[i];
      }
      rs += __shfl_xor(rs, 32);
      l = l * alpha + rs;
      m = mn;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) o[dt] *= alpha;
#pragma unroll
      for (int i = 0; i < 16; ++i)
        pd[i] = !drop ? pr[i]
                      : (drop_keep(seed, bh, myq, kb + acc_row(i, hh), T, p.dropout_p) ? pr[i] * rdrop : 0.f);
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int kr = acc_row(i, hh), key = kb + kr;
        const bool ok = qok && key <= myq && kvs[kr];
        const float sp = s[i] * p.scale + rabs[ok ? min(myq - key, p.nb - 1) : 0];
        pd[i] = ok ? silu(sp) * p.inv_n : 0.f;
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      bf16x8 ph, pl;
      pack_acc(pd, s2, ph, pl);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const bf16x8 vf = lds_tr8<HD>(Vs, 16 * s2, c0 + 32 * dt, lane);
        o[dt] = mfma(vf, ph, o[dt]);
        if (p.precise) o[dt] = mfma(vf, pl, o[dt]);
      }
    }
  }
  float mul = 1.f;
  if (KIND == 0) {
    mul = l > 0.f ? 1.0f / l : 0.f;
    if (ws == 0 && hh == 0 && qok && p.lse) p.lse[(int64_t)bh * T + myq] = l > 0.f ? (m + log2f(l)) * kLn2 : -INFINITY;
  }
  store_rows<HD, NDT>(shift(p.out, p.out_f32, c0), p.ldo, p.out_f32, (int64_t)b * T + myq, h, hh, o, mul, qok);
}

// ================================================================ dQ =========
template <int HD, int KIND>
__global__ void __launch_bounds__(HD) k_attn_dq_wide(AttnParams p) {
  using W = Wide<HD>;
  constexpr int KSQ = W::KSQ, NDT = W::NDT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Ks = smem;
  char* Vs = smem + W::IMG;
  float4* red = reinterpret_cast<float4*>(smem + 2 * W::IMG);
  float4* red2 = red + W::RED / 16;
  char* tail = smem + 2 * W::IMG + 2 * W::RED;
  uint8_t* kvs = reinterpret_cast<uint8_t*>(tail);
  int* s_start = reinterpret_cast<int*>(tail + 32);
  float* rabs = reinterpret_cast<float*>(tail + kWTail);
  unsigned long long* bins = reinterpret_cast<unsigned long long*>(rabs + (p.nb + 1) / 2 * 2);

  const int b = blockIdx.z, h = blockIdx.y, T = p.T;
  const int ws = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int q0 = blockIdx.x * kWRows, myq = q0 + r;
  const bool qok = myq < T;
  const int start = seq_start(p.key_valid, b, T, s_start);
  if (KIND == 1)
    for (int j = threadIdx.x; j < p.nb; j += blockDim.x) {
      rabs[j] = p.rab[h * p.nb + j];
      bins[j] = 0ull;
    }
  const int bh = b * p.H + h;
  const int c0 = ws * W::DQ;
  const int64_t tok = (int64_t)b * T + (qok ? myq : 0);

  bf16x8 qf[KSQ], dof[KSQ];
#pragma unroll
  for (int ks = 0; ks < KSQ; ++ks) {
    qf[ks] = gload8(p.q + tok * p.ldq + h * HD + c0 + 16 * ks + 8 * hh, qok);
    if (p.act) qf[ks] = silu8(qf[ks]);
    dof[ks] = gload8_any(p.dout, tok * p.lddo + h * HD + c0 + 16 * ks + 8 * hh, p.dout_f32, qok);
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
  const float sl2 = p.scale * kLog2e;
  const float rdrop = 1.0f / (1.0f - p.dropout_p);
  const bool drop = KIND == 0 && p.dropout_p > 0.f;
  const unsigned long long seed = drop ? attn_seed(p) : 0ull;

  const int kend = min(T, q0 + kWRows);
  for (int kb = (start / 32) * 32; kb < kend; kb += 32) {
    __syncthreads();
    stage_rows_at<HD>(Ks, p.k, p.ldk, b, T, h, kb, 32, 0, false, p.act);
    stage_rows_at<HD>(Vs, p.v, p.ldv, b, T, h, kb, 32, 0, false, p.act);
    if (threadIdx.x < 32) {
      const int t = kb + threadIdx.x;
      kvs[threadIdx.x] = (t < T) && (!p.key_valid || p.key_valid[(int64_t)b * T + t]);
    }
    __syncthreads();
    f32x16 s = f32x16{}, dp = f32x16{};
#pragma unroll
    for (int ks = 0; ks < KSQ; ++ks) {
      s = mfma(lds_row8<HD>(Ks, r, c0 + 16 * ks + 8 * hh), qf[ks], s);
      dp = mfma(lds_row8<HD>(Vs, r, c0 + 16 * ks + 8 * hh), dof[ks], dp);
    }
    red_put(red, ws, lane, s);
    red_put(red2, ws, lane, dp);
    __syncthreads();
    s = red_sum<W::NW>(red, lane);
    dp = red_sum<W::NW>(red2, lane);
    float ds[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int kr = acc_row(i, hh), key = kb + kr;
      const bool ok = qok && row_live && key <= myq && kvs[kr];
      if (KIND == 0) {
        const float pv = ok ? exp2f(s[i] * sl2 - lse2) : 0.f;
        float dpv = dp[i];
        if (drop) dpv = drop_keep(seed, bh, myq, key, T, p.dropout_p) ? dpv * rdrop : 0.f;
        ds[i] = pv * (dpv - dlt);
      } else {
        const int bk = min(myq - key, p.nb - 1);
        const float sp = s[i] * p.scale + rabs[ok ? bk : 0];
        ds[i] = ok ? dp[i] * dsilu(sp) * p.inv_n : 0.f;
        // every wave holds the same dS: wave 0 alone adds it to the bins
        if (ws == 0 && ok && ds[i] != 0.f && p.drab) atomicAdd(&bins[bk], to_fix(ds[i]));
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      bf16x8 dh, dl;
      pack_acc(ds, s2, dh, dl);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const bf16x8 kf = lds_tr8<HD>(Ks, 16 * s2, c0 + 32 * dt, lane);
        acc[dt] = mfma(kf, dh, acc[dt]);
        if (p.precise) acc[dt] = mfma(kf, dl, acc[dt]);
      }
    }
  }
  store_rows<HD, NDT>(shift(p.dq, p.out_f32, c0), p.lddq, p.out_f32, (int64_t)b * T + myq, h, hh, acc, p.scale, qok,
                      p.act ? (const void*)(p.q + c0) : nullptr, p.ldq);
  if (KIND == 1 && p.drab) {
    __syncthreads();
    for (int j = threadIdx.x; j < p.nb; j += blockDim.x)
      if (bins[j] != 0ull) atomicAdd(&p.drab_fix[h * p.nb + j], bins[j]);
  }
}

// ============================================================== dK / dV =====
template <int HD, int KIND>
__global__ void __launch_bounds__(HD) k_attn_dkdv_wide(AttnParams p) {
  using W = Wide<HD>;
  constexpr int KSQ = W::KSQ, NDT = W::NDT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Qs = smem;
  char* Ds = smem + W::IMG;
  float4* red = reinterpret_cast<float4*>(smem + 2 * W::IMG);
  float4* red2 = red + W::RED / 16;
  char* tail = smem + 2 * W::IMG + 2 * W::RED;
  int* s_start = reinterpret_cast<int*>(tail + 32);
  float* lses = reinterpret_cast<float*>(tail + 48);
  float* dlts = lses + 32;
  float* rabs = reinterpret_cast<float*>(tail + kWTail);

  const int b = blockIdx.z, h = blockIdx.y, T = p.T;
  const int ws = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int k0 = blockIdx.x * kWRows, myk = k0 + r;
  const int start = seq_start(p.key_valid, b, T, s_start);
  const bool kok = myk < T && myk >= start && (!p.key_valid || p.key_valid[(int64_t)b * T + myk]);
  if (KIND == 1)
    for (int j = threadIdx.x; j < p.nb; j += blockDim.x) rabs[j] = p.rab[h * p.nb + j];
  const int bh = b * p.H + h;
  const int c0 = ws * W::DQ;
  const int64_t tok = (int64_t)b * T + (myk < T ? myk : 0);

  bf16x8 kf[KSQ], vf[KSQ];
#pragma unroll
  for (int ks = 0; ks < KSQ; ++ks) {
    kf[ks] = gload8(p.k + tok * p.ldk + h * HD + c0 + 16 * ks + 8 * hh, myk < T);
    vf[ks] = gload8(p.v + tok * p.ldv + h * HD + c0 + 16 * ks + 8 * hh, myk < T);
    if (p.act) {
      kf[ks] = silu8(kf[ks]);
      vf[ks] = silu8(vf[ks]);
    }
  }
  f32x16 dk[NDT], dv[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) { dk[dt] = f32x16{}; dv[dt] = f32x16{}; }
  const float sl2 = p.scale * kLog2e;
  const float rdrop = 1.0f / (1.0f - p.dropout_p);
  const bool drop = KIND == 0 && p.dropout_p > 0.f;
  const unsigned long long seed = drop ? attn_seed(p) : 0ull;

  // queries that can see this block's keys: q >= k0 and q >= start
  for (int qb = (max(k0, start) / 32) * 32; qb < T; qb += 32) {
    __syncthreads();
    stage_rows_at<HD>(Qs, p.q, p.ldq, b, T, h, qb, 32, 0, false, p.act);
    stage_rows_at<HD>(Ds, p.dout, p.lddo, b, T, h, qb, 32, 0, p.dout_f32, false);
    if (threadIdx.x < 32) {
      const int t = qb + threadIdx.x;
      float lv = -INFINITY, dl = 0.f;
      if (KIND == 0 && t < T) {
        lv = p.lse[(int64_t)bh * T + t] * kLog2e;
        dl = p.delta[(int64_t)bh * T + t];
      }
      lses[threadIdx.x] = lv;
      dlts[threadIdx.x] = dl;
    }
    __syncthreads();
    f32x16 s = f32x16{}, dp = f32x16{};
#pragma unroll
    for (int ks = 0; ks < KSQ; ++ks) {
      s = mfma(lds_row8<HD>(Qs, r, c0 + 16 * ks + 8 * hh), kf[ks], s);
      dp = mfma(lds_row8<HD>(Ds, r, c0 + 16 * ks + 8 * hh), vf[ks], dp);
    }
    red_put(red, ws, lane, s);
    red_put(red2, ws, lane, dp);
    __syncthreads();
    s = red_sum<W::NW>(red, lane);
    dp = red_sum<W::NW>(red2, lane);
    float pd[16], ds[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int qr = acc_row(i, hh), q = qb + qr;
      const bool ok = kok && q < T && myk <= q;
      if (KIND == 0) {
        const float lv = lses[qr];
        const float pv = (ok && lv != -INFINITY) ? exp2f(s[i] * sl2 - lv) : 0.f;
        float dpv = dp[i];
        pd[i] = pv;
        if (drop) {
          const bool keep = drop_keep(seed, bh, q, myk, T, p.dropout_p);
          pd[i] = keep ? pv * rdrop : 0.f;
          dpv = keep ? dpv * rdrop : 0.f;
        }
        ds[i] = pv * (dpv - dlts[qr]);
      } else {
        const float sp = s[i] * p.scale + rabs[ok ? min(q - myk, p.nb - 1) : 0];
        pd[i] = ok ? silu(sp) * p.inv_n : 0.f;
        ds[i] = ok ? dp[i] * dsilu(sp) * p.inv_n : 0.f;
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      bf16x8 ph, pl, dh, dl;
      pack_acc(pd, s2, ph, pl);
      pack_acc(ds, s2, dh, dl);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const bf16x8 dof = lds_tr8<HD>(Ds, 16 * s2, c0 + 32 * dt, lane);
        const bf16x8 qf = lds_tr8<HD>(Qs, 16 * s2, c0 + 32 * dt, lane);
        dv[dt] = mfma(dof, ph, dv[dt]);
        dk[dt] = mfma(qf, dh, dk[dt]);
        if (p.precise) {
          dv[dt] = mfma(dof, pl, dv[dt]);
          dk[dt] = mfma(qf, dl, dk[dt]);
        }
      }
    }
  }
  const int64_t otok = (int64_t)b * T + myk;
  store_rows<HD, NDT>(shift(p.dk, p.out_f32, c0), p.lddk, p.out_f32, otok, h, hh, dk, p.scale, myk < T,
                      p.act ? (const void*)(p.k + c0) : nullptr, p.ldk);
  store_rows<HD, NDT>(shift(p.dv, p.out_f32, c0), p.lddv, p.out_f32, otok, h, hh, dv, 1.f, myk < T,
                      p.act ? (const void*)(p.v + c0) : nullptr, p.ldv);
}

template <int HD>
int wide_hd(const AttnParams& p, int which, hipStream_t s) {
  using W = Wide<HD>;
  const dim3 grid((p.T + kWRows - 1) / kWRows, p.H, p.B);
  const bool hstu = p.kind == GRK_ATTN_HSTU;
  const size_t rab = hstu ? (size_t)(p.nb + 1) / 2 * 2 * 4 : 0;
  if (which == 0) {
    const size_t lds = 2 * W::IMG + W::RED + kWTail + rab;
    launch_lds(hstu ? k_attn_fwd_wide<HD, 1> : k_attn_fwd_wide<HD, 0>, grid, W::NT, lds, s, p);
  } else if (which == 2) {
    const size_t lds = 2 * W::IMG + 2 * W::RED + kWTail + rab + (hstu ? (size_t)p.nb * 8 : 0);
    launch_lds(hstu ? k_attn_dq_wide<HD, 1> : k_attn_dq_wide<HD, 0>, grid, W::NT, lds, s, p);
  } else {
    const size_t lds = 2 * W::IMG + 2 * W::RED + kWTail + rab;
    launch_lds(hstu ? k_attn_dkdv_wide<HD, 1> : k_attn_dkdv_wide<HD, 0>, grid, W::NT, lds, s, p);
  }
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

}  // namespace

int attn_wide_launch(const AttnParams& p, int hd, int which, hipStream_t s) {
  if (p.precise == 2) {
    set_error("fp32-fidelity attention (precise = 2) is not offered for head_dim %d", hd);
    return GRK_EUNSUPPORTED;
  }
  switch (hd) {
    case 256: return wide_hd<256>(p, which, s);
    case 512: return wide_hd<512>(p, which, s);
  }
  set_error("head_dim %d unsupported (16, 32, 64, 128, 256, 512)", hd);
  return GRK_EUNSUPPORTED;
}

}  // namespace grk
