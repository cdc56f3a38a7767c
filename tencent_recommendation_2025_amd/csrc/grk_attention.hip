// Causal attention for gfx950 with MFMA 32x32x16 bf16: the reference's
// softmax MHA core and the north-star HSTU pointwise attention.
//
// Replaces:
//   softmax: F.scaled_dot_product_attention(Q, K, V, dropout_p, attn_mask)
//            with log2feats' mask (causal AND key-not-padding)
//            (model/BaseLine/model.py:39-43,331-335;
//             model/BaseLineO1/model.py:73-77,443-447)
//   hstu:    A = SiLU(alpha QK^T + rab[i-j]) * inv_n * mask ; O = A V
//            (no reference; oracle/hstu.py)
//
// Layout: Q/K/V/O/dO are [B*T, ld] row-major with head h at columns
// [h*HD, (h+1)*HD) -- the natural output of the fused projection GEMM, no
// transposes.  One workgroup = 4 waves = 128 consecutive queries (forward,
// dQ) or keys (dK/dV) of one (batch, head); K/V (or Q/dO) chunks of 64 rows
// are staged through LDS with an XOR-swizzled row image that serves both the
// row reads (ds_read_b128) and the transposed reads (ds_read_b64_tr_b16).
//
// MFMA operand conventions (lane l: r = l&31, hh = l>>5):
//   A[r][8hh+j], B[8hh+j][r], D[(i&3)+8(i>>2)+4hh][r].
// The forward computes S^T = K Q^T so a lane owns one query column; P^T is
// then directly the B operand of O^T = V^T P^T (permuted k order, see
// cdna_hip_programming.md §3).  Backward = dQ kernel (S^T, dP^T, dQ^T) +
// dK/dV kernel (S, dP, dV^T, dK^T): no atomics on dQ/dK/dV, deterministic.
#include "grk_attention.h"

namespace grk {

// LDS of the TB instantiations: kChunk staged stamps, the head's rab_t row and
// (dQ) the drab_t fixed-point bins.
constexpr int kTimeLds = kChunk * 4 + kMaxTimeBuckets * 4 + kMaxTimeBuckets * 8;

// ================================================================ forward ====
// F8: q/k/v are fp8 e4m3 (post-activation): S^T = K Q^T on the fp8 MFMA from
// an fp8 K image and fp8 Q fragments; V staged as (exact) bf16 for P V.
// TB: with the HSTU time bias rab_t[h, time_bucket(t_q - t_k)] (KIND 1, not F8).
template <int HD, int KIND, bool F8, bool TB = false>
__global__ void __launch_bounds__(256) k_attn_fwd(AttnParams p) {
  constexpr int KS = HD / 16, NDT = (HD + 31) / 32;
  constexpr int IMG = kChunk * HD * 2;
  constexpr int RAB = KIND == 1 ? kRabMax : 4;
  __shared__ __attribute__((aligned(16))) char smem[2 * IMG + 64 + RAB * 4 + 16 + (TB ? kTimeLds : 0)];
  char* Ks = smem;
  char* Vs = smem + IMG;
  uint8_t* kvs = reinterpret_cast<uint8_t*>(smem + 2 * IMG);
  float* rabs = reinterpret_cast<float*>(smem + 2 * IMG + 64);
  int* s_start = reinterpret_cast<int*>(smem + 2 * IMG + 64 + RAB * 4);
  int* tsk = reinterpret_cast<int*>(smem + 2 * IMG + 64 + RAB * 4 + 16);  // TB: key stamps of the chunk
  float* rtab = reinterpret_cast<float*>(tsk + kChunk);                    // TB: rab_t[h, :]

  const int b = blockIdx.z, h = blockIdx.y, T = p.T;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int q0 = blockIdx.x * kBlockRows, qw = q0 + wave * 32, myq = qw + r;
  const bool qok = myq < T;
  const int start = seq_start(p.key_valid, b, T, s_start);
  if (KIND == 1)
    for (int j = threadIdx.x; j < p.nb; j += blockDim.x) rabs[j] = p.rab[h * p.nb + j];
  int tq = 0;
  if constexpr (TB) {
    for (int j = threadIdx.x; j < p.nbt; j += blockDim.x) rtab[j] = p.rab_t[h * p.nbt + j];
    tq = rel_stamp(p, b, T, start, myq);
  }

  bf16x8 qf[F8 ? 1 : KS];
  f8x8 qf8[F8 ? KS : 1];
  const int64_t qoff = ((int64_t)b * T + (qok ? myq : 0)) * p.ldq + h * HD;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    if constexpr (F8) {
      qf8[ks] = qok ? *reinterpret_cast<const f8x8*>((const uint8_t*)p.q + qoff + 16 * ks + 8 * hh) : 0;
    } else {
      qf[ks] = gload8(p.q + qoff + 16 * ks + 8 * hh, qok);
      if (p.act) qf[ks] = silu8(qf[ks]);
    }
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

  const int kbeg = (start / 32) * 32;
  const int kend = min(T, q0 + kBlockRows);
  for (int kc = kbeg; kc < kend; kc += kChunk) {
    __syncthreads();
    if constexpr (F8) {
      stage_rows_f8<HD>(Ks, p.k, p.ldk, b, T, h, kc);
      stage_rows<HD>(Vs, p.v, p.ldv, b, T, h, kc, 2);
    } else {
      stage_rows<HD>(Ks, p.k, p.ldk, b, T, h, kc, 0, p.act);
      stage_rows<HD>(Vs, p.v, p.ldv, b, T, h, kc, 0, p.act);
    }
    if (threadIdx.x < kChunk) {
      const int t = kc + threadIdx.x;
      kvs[threadIdx.x] = (t < T) && (!p.key_valid || p.key_valid[(int64_t)b * T + t]);
      if constexpr (TB) tsk[threadIdx.x] = rel_stamp(p, b, T, start, t);
    }
    __syncthreads();
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int kb = kc + 32 * sub;
      if (kb > qw + 31 || kb >= kend || kb + 32 <= start) continue;  // wave-uniform causal/padding skip
      f32x16 s = acc_zero();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if constexpr (F8) s = mfma8(lds_row8_f8<HD>(Ks, 32 * sub + r, 16 * ks + 8 * hh), qf8[ks], s);
        else s = mfma(lds_row8<HD>(Ks, 32 * sub + r, 16 * ks + 8 * hh), qf[ks], s);
      }
      float pr[16], pd[16];
      if (KIND == 0) {
        float x[16], tmax = -INFINITY;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int kr = 32 * sub + acc_row(i, hh), key = kc + kr;
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
        for (int i = 0; i < 16; ++i) {
          pd[i] = pr[i];
          if (drop) {
            const int key = kc + 32 * sub + acc_row(i, hh);
            pd[i] = drop_keep(seed, bh, myq, key, T, p.dropout_p) ? pr[i] * rdrop : 0.f;
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int kr = 32 * sub + acc_row(i, hh), key = kc + kr;
          const bool ok = qok && key <= myq && kvs[kr];
          float sp = s[i] * p.scale + rabs[ok ? min(myq - key, p.nb - 1) : 0];
          if constexpr (TB) sp += rtab[time_bucket(tq - tsk[kr], p.nbt)];
          pd[i] = ok ? silu(sp) * p.inv_n : 0.f;
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        bf16x8 ph, pl;
        pack_acc(pd, s2, ph, pl);
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          bf16x8 vf = lds_tr8<HD>(Vs, 32 * sub + 16 * s2, dt * 32, lane);
          o[dt] = mfma(vf, ph, o[dt]);
          if (p.precise) o[dt] = mfma(vf, pl, o[dt]);
        }
      }
    }
  }
  float mul = 1.f;
  if (KIND == 0) {
    mul = l > 0.f ? 1.0f / l : 0.f;
    if (hh == 0 && qok && p.lse) p.lse[(int64_t)bh * T + myq] = l > 0.f ? (m + log2f(l)) * kLn2 : -INFINITY;
  }
  store_rows<HD, NDT>(p.out, p.ldo, p.out_f32, (int64_t)b * T + myq, h, hh, o, mul, qok);
}

// ========================================================== delta (softmax) ==
// delta[bh, t] = sum_d dO[t, d] * O[t, d]  (fp32), one wave per (b, t, h).
template <int HD>
__global__ void __launch_bounds__(256) k_attn_delta(AttnParams p) {
  const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const int64_t total = (int64_t)p.B * p.T * p.H;
  if (wid >= total) return;
  const int h = (int)(wid % p.H);
  int64_t tok = wid / p.H;
  const int b = (int)(tok / p.T), t = (int)(tok % p.T);
  if (p.row_base) {  // jagged rows: only [start_b, T) exist; earlier (fully masked) queries get delta 0
    if (t < p.seq_range[3 * b]) {
      if ((threadIdx.x & 63) == 0) const_cast<float*>(p.delta)[((int64_t)b * p.H + h) * p.T + t] = 0.f;
      return;
    }
    tok = p.row_base[b] + t;
  }
  float acc = 0.f;
  for (int d = lane; d < HD; d += 64) {
    const int64_t oo = tok * p.ldo + h * HD + d, od = tok * p.lddo + h * HD + d;
    const float ov = p.out_f32 ? ((const float*)p.out)[oo] : bf16_to_f32(((const bf16_t*)p.out)[oo]);
    const float dv = p.dout_f32 ? ((const float*)p.dout)[od] : bf16_to_f32(((const bf16_t*)p.dout)[od]);
    acc += ov * dv;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  if (lane == 0) const_cast<float*>(p.delta)[((int64_t)b * p.H + h) * p.T + t] = acc;
}

// ================================================================ dQ =========
// F8: fp8 q/k/v read as (exact) bf16; all products on the bf16 MFMA.
template <int HD, int KIND, bool F8, bool TB = false>
__global__ void __launch_bounds__(256) k_attn_bwd_dq(AttnParams p) {
  constexpr int KS = HD / 16, NDT = (HD + 31) / 32;
  constexpr int IMG = kChunk * HD * 2;
  constexpr int RAB = KIND == 1 ? kRabMax : 4;
  __shared__ __attribute__((aligned(16))) char smem[2 * IMG + 64 + 3 * RAB * 4 + 16 + (TB ? kTimeLds : 0)];
  char* Ks = smem;
  char* Vs = smem + IMG;
  uint8_t* kvs = reinterpret_cast<uint8_t*>(smem + 2 * IMG);
  float* rabs = reinterpret_cast<float*>(smem + 2 * IMG + 64);
  unsigned long long* bins = reinterpret_cast<unsigned long long*>(rabs + RAB);  // int64 fixed point
  int* s_start = reinterpret_cast<int*>(smem + 2 * IMG + 64 + 3 * RAB * 4);
  int* tsk = reinterpret_cast<int*>(smem + 2 * IMG + 64 + 3 * RAB * 4 + 16);  // TB: key stamps of the chunk
  float* rtab = reinterpret_cast<float*>(tsk + kChunk);                        // TB: rab_t[h, :]
  unsigned long long* tbins = reinterpret_cast<unsigned long long*>(rtab + kMaxTimeBuckets);  // TB: drab_t bins

  const int b = blockIdx.z, h = blockIdx.y, T = p.T;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int q0 = blockIdx.x * kBlockRows, qw = q0 + wave * 32, myq = qw + r;
  const bool qok = myq < T;
  const int start = seq_start(p.key_valid, b, T, s_start);
  if (KIND == 1)
    for (int j = threadIdx.x; j < p.nb; j += blockDim.x) {
      rabs[j] = p.rab[h * p.nb + j];
      bins[j] = 0ull;
    }
  int tq = 0;
  if constexpr (TB) {
    for (int j = threadIdx.x; j < p.nbt; j += blockDim.x) {
      rtab[j] = p.rab_t[h * p.nbt + j];
      tbins[j] = 0ull;
    }
    tq = rel_stamp(p, b, T, start, myq);
  }
  const int bh = b * p.H + h;
  const int64_t tok = (int64_t)b * T + (qok ? myq : 0);

  bf16x8 qf[KS], dof[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    qf[ks] = gload8_src(p.q, tok * p.ldq + h * HD + 16 * ks + 8 * hh, F8 ? 2 : 0, qok);
    if (p.act) qf[ks] = silu8(qf[ks]);
    dof[ks] = gload8_any(p.dout, tok * p.lddo + h * HD + 16 * ks + 8 * hh, p.dout_f32, qok);
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

  const int kbeg = (start / 32) * 32;
  const int kend = min(T, q0 + kBlockRows);
  for (int kc = kbeg; kc < kend; kc += kChunk) {
    __syncthreads();
    stage_rows<HD>(Ks, p.k, p.ldk, b, T, h, kc, F8 ? 2 : 0, p.act);
    stage_rows<HD>(Vs, p.v, p.ldv, b, T, h, kc, F8 ? 2 : 0, p.act);
    if (threadIdx.x < kChunk) {
      const int t = kc + threadIdx.x;
      kvs[threadIdx.x] = (t < T) && (!p.key_valid || p.key_valid[(int64_t)b * T + t]);
      if constexpr (TB) tsk[threadIdx.x] = rel_stamp(p, b, T, start, t);
    }
    __syncthreads();
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int kb = kc + 32 * sub;
      if (kb > qw + 31 || kb >= kend || kb + 32 <= start) continue;
      f32x16 s = acc_zero(), dp = acc_zero();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        s = mfma(lds_row8<HD>(Ks, 32 * sub + r, 16 * ks + 8 * hh), qf[ks], s);
        dp = mfma(lds_row8<HD>(Vs, 32 * sub + r, 16 * ks + 8 * hh), dof[ks], dp);
      }
      float ds[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int kr = 32 * sub + acc_row(i, hh), key = kc + kr;
        const bool ok = qok && row_live && key <= myq && kvs[kr];
        if (KIND == 0) {
          const float pv = ok ? exp2f(s[i] * sl2 - lse2) : 0.f;
          float dpv = dp[i];
          if (drop) dpv = drop_keep(seed, bh, myq, key, T, p.dropout_p) ? dpv * rdrop : 0.f;
          ds[i] = pv * (dpv - dlt);
        } else {
          const int bk = min(myq - key, p.nb - 1);
          float sp = s[i] * p.scale + rabs[ok ? bk : 0];
          int tbk = 0;
          if constexpr (TB) {
            tbk = time_bucket(tq - tsk[kr], p.nbt);
            sp += rtab[tbk];
          }
          ds[i] = ok ? dp[i] * dsilu(sp) * p.inv_n : 0.f;
          if (ok && ds[i] != 0.f && p.drab) atomicAdd(&bins[bk], to_fix(ds[i]));
          if constexpr (TB)
            if (ok && ds[i] != 0.f && p.drab_t) atomicAdd(&tbins[tbk], to_fix(ds[i]));
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        bf16x8 dh, dl;
        pack_acc(ds, s2, dh, dl);
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          bf16x8 kf = lds_tr8<HD>(Ks, 32 * sub + 16 * s2, dt * 32, lane);
          acc[dt] = mfma(kf, dh, acc[dt]);
          if (p.precise) acc[dt] = mfma(kf, dl, acc[dt]);
        }
      }
    }
  }
  store_rows<HD, NDT>(p.dq, p.lddq, p.out_f32, (int64_t)b * T + myq, h, hh, acc, p.scale, qok,
                      p.act ? p.q : nullptr, p.ldq);
  if (KIND == 1 && (p.drab || (TB && p.drab_t))) {
    __syncthreads();
    if (p.drab)
      for (int j = threadIdx.x; j < p.nb; j += blockDim.x)
        if (bins[j] != 0ull) atomicAdd(&p.drab_fix[h * p.nb + j], bins[j]);
    if constexpr (TB)
      if (p.drab_t)
        for (int j = threadIdx.x; j < p.nbt; j += blockDim.x)
          if (tbins[j] != 0ull) atomicAdd(&p.drab_t_fix[h * p.nbt + j], tbins[j]);
  }
}

// ============================================================== dK / dV =====
// F8: S = Q K^T on the fp8 MFMA (fp8 Q image + fp8 K fragments); Q also
// staged as (exact) bf16 for dK = dS^T Q, V fragments as bf16 for dP.
template <int HD, int KIND, bool F8, bool TB = false>
__global__ void __launch_bounds__(256) k_attn_bwd_dkdv(AttnParams p) {
  constexpr int KS = HD / 16, NDT = (HD + 31) / 32;
  constexpr int IMG = kChunk * HD * 2;
  constexpr int IMG8 = F8 ? kChunk * HD : 0;
  constexpr int RAB = KIND == 1 ? kRabMax : 4;
  __shared__ __attribute__((aligned(16))) char smem[2 * IMG + IMG8 + 2 * kChunk * 4 + RAB * 4 + 16 +
                                                    (TB ? kTimeLds : 0)];
  char* Qs = smem;
  char* Ds = smem + IMG;
  char* Q8s = smem + 2 * IMG + 2 * kChunk * 4 + RAB * 4 + 16;
  float* lses = reinterpret_cast<float*>(smem + 2 * IMG);
  float* dlts = lses + kChunk;
  float* rabs = dlts + kChunk;
  int* s_start = reinterpret_cast<int*>(smem + 2 * IMG + 2 * kChunk * 4 + RAB * 4);
  int* tsq = reinterpret_cast<int*>(smem + 2 * IMG + IMG8 + 2 * kChunk * 4 + RAB * 4 + 16);  // TB: query stamps
  float* rtab = reinterpret_cast<float*>(tsq + kChunk);                                      // TB: rab_t[h, :]

  const int b = blockIdx.z, h = blockIdx.y, T = p.T;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int k0 = blockIdx.x * kBlockRows, kw = k0 + wave * 32, myk = kw + r;
  const int start = seq_start(p.key_valid, b, T, s_start);
  const bool kok = myk < T && myk >= start && (!p.key_valid || p.key_valid[(int64_t)b * T + myk]);
  if (KIND == 1)
    for (int j = threadIdx.x; j < p.nb; j += blockDim.x) rabs[j] = p.rab[h * p.nb + j];
  int tk = 0;
  if constexpr (TB) {
    for (int j = threadIdx.x; j < p.nbt; j += blockDim.x) rtab[j] = p.rab_t[h * p.nbt + j];
    tk = rel_stamp(p, b, T, start, myk);
  }
  const int bh = b * p.H + h;
  const int64_t tok = (int64_t)b * T + (myk < T ? myk : 0);

  bf16x8 kf[F8 ? 1 : KS], vf[KS];
  f8x8 kf8[F8 ? KS : 1];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int64_t ko = tok * p.ldk + h * HD + 16 * ks + 8 * hh;
    if constexpr (F8) {
      kf8[ks] = myk < T ? *reinterpret_cast<const f8x8*>((const uint8_t*)p.k + ko) : 0;
      vf[ks] = gload8_src(p.v, tok * p.ldv + h * HD + 16 * ks + 8 * hh, 2, myk < T);
    } else {
      kf[ks] = gload8(p.k + ko, myk < T);
      vf[ks] = gload8(p.v + tok * p.ldv + h * HD + 16 * ks + 8 * hh, myk < T);
      if (p.act) {
        kf[ks] = silu8(kf[ks]);
        vf[ks] = silu8(vf[ks]);
      }
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
  const int qbeg = (max(k0, start) / 32) * 32;
  for (int qc = qbeg; qc < T; qc += kChunk) {
    __syncthreads();
    stage_rows<HD>(Qs, p.q, p.ldq, b, T, h, qc, F8 ? 2 : 0, p.act);
    if constexpr (F8) stage_rows_f8<HD>(Q8s, p.q, p.ldq, b, T, h, qc);
    stage_rows<HD>(Ds, p.dout, p.lddo, b, T, h, qc, p.dout_f32 ? 1 : 0);
    if (threadIdx.x < kChunk) {
      const int t = qc + threadIdx.x;
      float lv = -INFINITY, dl = 0.f;
      if (KIND == 0 && t < T) {
        lv = p.lse[(int64_t)bh * T + t] * kLog2e;
        dl = p.delta[(int64_t)bh * T + t];
      }
      lses[threadIdx.x] = lv;
      dlts[threadIdx.x] = dl;
      if constexpr (TB) tsq[threadIdx.x] = rel_stamp(p, b, T, start, t);
    }
    __syncthreads();
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int qb = qc + 32 * sub;
      if (qb + 31 < kw || qb >= T) continue;  // wave-uniform: every query precedes this wave's keys
      f32x16 s = acc_zero(), dp = acc_zero();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if constexpr (F8) s = mfma8(lds_row8_f8<HD>(Q8s, 32 * sub + r, 16 * ks + 8 * hh), kf8[ks], s);
        else s = mfma(lds_row8<HD>(Qs, 32 * sub + r, 16 * ks + 8 * hh), kf[ks], s);
        dp = mfma(lds_row8<HD>(Ds, 32 * sub + r, 16 * ks + 8 * hh), vf[ks], dp);
      }
      float pd[16], ds[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qr = 32 * sub + acc_row(i, hh), q = qc + qr;
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
          float sp = s[i] * p.scale + rabs[ok ? min(q - myk, p.nb - 1) : 0];
          if constexpr (TB) sp += rtab[time_bucket(tsq[qr] - tk, p.nbt)];
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
          bf16x8 dof = lds_tr8<HD>(Ds, 32 * sub + 16 * s2, dt * 32, lane);
          bf16x8 qf = lds_tr8<HD>(Qs, 32 * sub + 16 * s2, dt * 32, lane);
          dv[dt] = mfma(dof, ph, dv[dt]);
          dk[dt] = mfma(qf, dh, dk[dt]);
          if (p.precise) {
            dv[dt] = mfma(dof, pl, dv[dt]);
            dk[dt] = mfma(qf, dl, dk[dt]);
          }
        }
      }
    }
  }
  const int64_t otok = (int64_t)b * T + myk;
  store_rows<HD, NDT>(p.dk, p.lddk, p.out_f32, otok, h, hh, dk, p.scale, myk < T, p.act ? p.k : nullptr, p.ldk);
  store_rows<HD, NDT>(p.dv, p.lddv, p.out_f32, otok, h, hh, dv, 1.f, myk < T, p.act ? p.v : nullptr, p.ldv);
}

template <int HD, bool F8 = false>
static int launch_hd(const AttnParams& p, int which, hipStream_t s) {
  dim3 grid((p.T + kBlockRows - 1) / kBlockRows, p.H, p.B);
  const bool tb = !F8 && p.kind == GRK_ATTN_HSTU && p.nbt > 0;  // fill_params: fp8 q/k/v take no time bias
  if (which == 0) {
    if (p.kind == GRK_ATTN_SOFTMAX) k_attn_fwd<HD, 0, F8><<<grid, 256, 0, s>>>(p);
    else if (tb) k_attn_fwd<HD, 1, false, true><<<grid, 256, 0, s>>>(p);
    else k_attn_fwd<HD, 1, F8><<<grid, 256, 0, s>>>(p);
  } else if (which == 1) {
    const int64_t waves = (int64_t)p.B * p.T * p.H;
    k_attn_delta<HD><<<(unsigned)((waves + 3) / 4), 256, 0, s>>>(p);
  } else if (which == 2) {
    if (p.kind == GRK_ATTN_SOFTMAX) k_attn_bwd_dq<HD, 0, F8><<<grid, 256, 0, s>>>(p);
    else if (tb) k_attn_bwd_dq<HD, 1, false, true><<<grid, 256, 0, s>>>(p);
    else k_attn_bwd_dq<HD, 1, F8><<<grid, 256, 0, s>>>(p);
  } else {
    if (p.kind == GRK_ATTN_SOFTMAX) k_attn_bwd_dkdv<HD, 0, F8><<<grid, 256, 0, s>>>(p);
    else if (tb) k_attn_bwd_dkdv<HD, 1, false, true><<<grid, 256, 0, s>>>(p);
    else k_attn_bwd_dkdv<HD, 1, F8><<<grid, 256, 0, s>>>(p);
  }
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

// drab[i] += fixed-point accumulator (after the dQ kernels)
__global__ void k_drab_finalize(float* __restrict__ drab, const unsigned long long* __restrict__ fix, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) drab[i] += (float)((double)(long long)fix[i] * (1.0 / kFixScale));
}
// GRK_ATTN_BWD_WS_CLEAN when the dq kernel was not the whole-sequence one: finalize
// (set or add) and leave the bins zero.
__global__ void k_drab_finalize_clean(float* __restrict__ drab, unsigned long long* __restrict__ fix, int n, int set) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) drab_finalize_elem(drab, fix, i, set);
}

static int launch(const AttnParams& p, int hd, int which, hipStream_t s) {
  if (p.qkv_f8 && p.row_base) {
    set_error("fp8 q/k/v run the chunked kernels, which take the padded layout only (row_base must be NULL)");
    return GRK_EUNSUPPORTED;
  }
  if (p.qkv_f8) {  // fp8 q/k/v: the chunked kernels (C5: T = 1025), head_dim 64 / 128
    if (hd == 64) return launch_hd<64, true>(p, which, s);
    if (hd == 128) return launch_hd<128, true>(p, which, s);
    set_error("fp8 q/k/v attention supports head_dim 64 / 128, not %d", hd);
    return GRK_EUNSUPPORTED;
  }
  if (which != 1 && attn_seq_launch(p, hd, which, s)) {
    GRK_LAUNCH_CHECK();
    return GRK_OK;
  }
  if (p.row_base && (which != 1 || hd > 128)) {
    set_error("the jagged layout (row_base) runs in the whole-sequence kernels only: T = %d x head_dim %d does not "
              "fit them", p.T, hd);
    return GRK_EUNSUPPORTED;
  }
  if (p.precise == 2 && which != 1 && hd <= 128) {
    set_error("fp32-fidelity attention (precise = 2) runs in the whole-sequence kernels only: T = %d x head_dim %d "
              "does not fit their LDS", p.T, hd);
    return GRK_EUNSUPPORTED;
  }
  switch (hd) {
    case 16: return launch_hd<16>(p, which, s);
    case 32: return launch_hd<32>(p, which, s);
    case 64: return launch_hd<64>(p, which, s);
    case 128: return launch_hd<128>(p, which, s);
    case 256:
    case 512:
      if (which != 1) return attn_wide_launch(p, hd, which, s);
      {
        const int64_t waves = (int64_t)p.B * p.T * p.H;
        if (hd == 256) k_attn_delta<256><<<(unsigned)((waves + 3) / 4), 256, 0, s>>>(p);
        else k_attn_delta<512><<<(unsigned)((waves + 3) / 4), 256, 0, s>>>(p);
        GRK_LAUNCH_CHECK();
        return GRK_OK;
      }
  }
  set_error("head_dim %d unsupported (16, 32, 64, 128, 256, 512)", hd);
  return GRK_EUNSUPPORTED;
}

static int fill_params(const grk_attn_args* a, AttnParams* p) {
  GRK_CHECK_ARG(a != nullptr, "args is NULL");
  GRK_CHECK_ARG(a->kind == GRK_ATTN_SOFTMAX || a->kind == GRK_ATTN_HSTU, "bad kind");
  GRK_CHECK_ARG(a->batch > 0 && a->heads > 0 && a->seq_len > 0, "batch/heads/seq_len must be > 0");
  GRK_CHECK_ARG(a->head_dim == 16 || a->head_dim == 32 || a->head_dim == 64 || a->head_dim == 128 ||
                    a->head_dim == 256 || a->head_dim == 512,
                "head_dim %d unsupported (16, 32, 64, 128, 256, 512)", a->head_dim);
  GRK_CHECK_ARG(a->q && a->k && a->v, "q/k/v required");
  const int64_t need = (int64_t)a->heads * a->head_dim;
  GRK_CHECK_ARG(a->ldq >= need && a->ldk >= need && a->ldv >= need, "row strides smaller than heads*head_dim");
  GRK_CHECK_ARG(a->ldq % 8 == 0 && a->ldk % 8 == 0 && a->ldv % 8 == 0, "row strides must be multiples of 8");
  GRK_CHECK_ARG(((uintptr_t)a->q | (uintptr_t)a->k | (uintptr_t)a->v) % 16 == 0, "q/k/v must be 16-byte aligned");
  GRK_CHECK_ARG(a->kind == GRK_ATTN_SOFTMAX || (a->rab && a->num_buckets > 0 && a->num_buckets <= kRabMax),
                "hstu needs rab with 1..%d buckets", kRabMax);
  GRK_CHECK_ARG(a->dropout_p >= 0.f && a->dropout_p < 1.f, "dropout_p must be in [0, 1)");
  GRK_CHECK_ARG(a->kind == GRK_ATTN_SOFTMAX || a->dropout_p == 0.f, "hstu attention has no dropout");
  GRK_CHECK_ARG(a->out_dtype == GRK_F32 || a->out_dtype == GRK_BF16, "out_dtype must be GRK_F32 / GRK_BF16");
  GRK_CHECK_ARG(a->act == GRK_ACT_NONE || a->act == GRK_ACT_SILU, "act must be GRK_ACT_NONE / GRK_ACT_SILU");
  GRK_CHECK_ARG(a->precise >= 0 && a->precise <= 2, "precise must be 0, 1 or 2");
  GRK_CHECK_ARG(a->precise != 2 || a->qkv_dtype == GRK_F32 || a->qkv_dtype == GRK_F16 || a->qkv_dtype == GRK_BF16,
                "qkv_dtype must be GRK_F32 / GRK_F16 / GRK_BF16");
  const bool f8 = a->precise != 2 && a->qkv_dtype == GRK_FP8_E4M3;
  GRK_CHECK_ARG(!f8 || a->act == GRK_ACT_NONE, "fp8 q/k/v hold activations: act must be GRK_ACT_NONE");
  GRK_CHECK_ARG(!f8 || a->num_time_buckets == 0, "fp8 q/k/v: no time bias (whole-sequence kernels only)");
  GRK_CHECK_ARG(!f8 || ((uintptr_t)a->q | (uintptr_t)a->k | (uintptr_t)a->v) % 8 == 0, "fp8 q/k/v: 8-byte aligned");
  GRK_CHECK_ARG(a->num_time_buckets >= 0 && a->num_time_buckets <= kMaxTimeBuckets,
                "num_time_buckets must be in [0, %d]", kMaxTimeBuckets);
  GRK_CHECK_ARG(a->num_time_buckets == 0 || (a->kind == GRK_ATTN_HSTU && a->timestamps && a->rab_t),
                "the time bias is an HSTU feature and needs timestamps and rab_t");
  memset(p, 0, sizeof(*p));
  p->kind = a->kind; p->B = a->batch; p->H = a->heads; p->T = a->seq_len;
  if (a->num_time_buckets > 0) {
    p->ts = a->timestamps; p->rab_t = a->rab_t; p->nbt = a->num_time_buckets;
  }
  p->q = (const bf16_t*)a->q; p->k = (const bf16_t*)a->k; p->v = (const bf16_t*)a->v;
  p->ldq = a->ldq; p->ldk = a->ldk; p->ldv = a->ldv;
  p->key_valid = a->key_valid;
  p->scale = a->scale; p->inv_n = a->inv_n; p->dropout_p = a->dropout_p; p->seed = a->seed; p->seed_dev = (const unsigned long long*)a->seed_dev;
  p->rab = a->rab; p->nb = a->num_buckets;
  p->precise = a->precise; p->out_f32 = a->out_dtype == GRK_F32;
  p->in_dt = a->precise == 2 ? a->qkv_dtype : GRK_BF16;
  p->act = a->act;
  p->qkv_f8 = f8;
  p->seq_range = a->seq_range;
  GRK_CHECK_ARG(!a->row_base || (a->seq_range && a->num_rows && a->capacity > 0),
                "the jagged layout (row_base) needs seq_range, num_rows and capacity");
  p->row_base = a->row_base;
  p->jag_n = a->num_rows;
  p->jag_cap = a->capacity;
  return GRK_OK;
}

}  // namespace grk

using namespace grk;

extern "C" int grk_attention_fwd(const grk_attn_args* a, void* out, int64_t ldo, float* lse, void* stream) {
  clear_error();
  AttnParams p;
  int rc = fill_params(a, &p);
  if (rc) return rc;
  GRK_CHECK_ARG(out && ldo >= (int64_t)a->heads * a->head_dim, "bad out / ldo");
  GRK_CHECK_ARG(a->kind == GRK_ATTN_HSTU || lse, "softmax forward needs lse [B, H, T]");
  p.out = out; p.ldo = ldo; p.lse = lse;
  return launch(p, a->head_dim, 0, (hipStream_t)stream);
}

extern "C" int grk_attention_bwd_parts(const grk_attn_args* a, const void* out, int64_t ldo, const void* dout,
                                       int64_t lddo, int dout_dtype, const float* lse, float* delta_ws, void* dq,
                                       int64_t lddq, void* dk, int64_t lddk, void* dv, int64_t lddv, float* drab,
                                       int64_t* drab_ws, int parts, void* stream) {
  clear_error();
  AttnParams p;
  int rc = fill_params(a, &p);
  if (rc) return rc;
  GRK_CHECK_ARG((parts & 3) >= 1 && parts <= 15, "bad parts (%d)", parts);
  const bool do_dq = parts & GRK_ATTN_BWD_DQ, do_dkdv = parts & GRK_ATTN_BWD_DKDV;
  const bool clean = parts & GRK_ATTN_BWD_WS_CLEAN, dset = parts & GRK_ATTN_BWD_DRAB_SET;
  const int64_t need = (int64_t)a->heads * a->head_dim;
  GRK_CHECK_ARG(dout && lddo >= need && lddo % 8 == 0, "bad dout / lddo");
  GRK_CHECK_ARG(dout_dtype == GRK_F32 || dout_dtype == GRK_BF16, "bad dout dtype");
  GRK_CHECK_ARG(!do_dq || (dq && lddq >= need), "bad dq");
  GRK_CHECK_ARG(!do_dkdv || (dk && dv && lddk >= need && lddv >= need), "bad dk/dv");
  GRK_CHECK_ARG(a->kind == GRK_ATTN_HSTU || (out && lse && delta_ws && ldo >= need),
                "softmax backward needs out, lse and delta_ws [B, H, T]");
  p.out = const_cast<void*>(out); p.ldo = ldo;
  p.dout = dout; p.lddo = lddo; p.dout_f32 = dout_dtype == GRK_F32;
  p.lse = const_cast<float*>(lse); p.delta = delta_ws;
  p.dq = dq; p.lddq = lddq; p.dk = dk; p.lddk = lddk; p.dv = dv; p.lddv = lddv;
  GRK_CHECK_ARG(!do_dq || !drab || drab_ws, "drab needs drab_ws (int64 [H, nb] scratch)");
  p.drab = (a->kind == GRK_ATTN_HSTU && do_dq) ? drab : nullptr;
  p.drab_fix = reinterpret_cast<unsigned long long*>(drab_ws);
  GRK_CHECK_ARG(!do_dq || p.nbt == 0 || !a->drab_t || a->drab_t_ws, "drab_t needs drab_t_ws (int64 [H, nbt] scratch)");
  p.drab_t = (p.nbt > 0 && do_dq) ? a->drab_t : nullptr;
  p.drab_t_fix = reinterpret_cast<unsigned long long*>(a->drab_t_ws);
  hipStream_t s = (hipStream_t)stream;
  if (do_dq) {
    const int nfix = a->heads * a->num_buckets;
    GRK_CHECK_ARG(!clean || a->kind != GRK_ATTN_HSTU || p.drab, "GRK_ATTN_BWD_WS_CLEAN needs drab and drab_ws");
    if (clean && p.drab) {
      // scratch zero on entry, left zero; the counter is the extra slot after the bins
      bool fused = false;
      if (!p.qkv_f8) {
        AttnParams pf = p;
        pf.fin_count = reinterpret_cast<unsigned*>(drab_ws + nfix);
        pf.drab_set = dset;
        fused = attn_seq_launch(pf, a->head_dim, 2, s);
        if (fused) GRK_LAUNCH_CHECK();
      }
      if (!fused) {
        rc = launch(p, a->head_dim, 2, s);
        if (rc) return rc;
        k_drab_finalize_clean<<<(nfix + 255) / 256, 256, 0, s>>>(p.drab, p.drab_fix, nfix, dset);
        GRK_LAUNCH_CHECK();
        if (p.drab_t) {
          const int nt = a->heads * p.nbt;
          k_drab_finalize_clean<<<(nt + 255) / 256, 256, 0, s>>>(p.drab_t, p.drab_t_fix, nt, dset);
          GRK_LAUNCH_CHECK();
        }
      }
    } else {
      if (p.drab) GRK_CHECK_HIP(zero_async(drab_ws, (size_t)nfix * 8, s));
      if (p.drab_t) GRK_CHECK_HIP(zero_async(a->drab_t_ws, (size_t)a->heads * p.nbt * 8, s));
      if (dset && p.drab) GRK_CHECK_HIP(zero_async(p.drab, (size_t)nfix * 4, s));
      if (dset && p.drab_t) GRK_CHECK_HIP(zero_async(p.drab_t, (size_t)a->heads * p.nbt * 4, s));
      if (a->kind == GRK_ATTN_SOFTMAX) {
        // out dtype of the forward output equals out_dtype of these args
        rc = launch(p, a->head_dim, 1, s);
        if (rc) return rc;
      }
      rc = launch(p, a->head_dim, 2, s);
      if (rc) return rc;
      if (p.drab) {
        k_drab_finalize<<<(nfix + 255) / 256, 256, 0, s>>>(p.drab, p.drab_fix, nfix);
        GRK_LAUNCH_CHECK();
      }
      if (p.drab_t) {
        const int nt = a->heads * p.nbt;
        k_drab_finalize<<<(nt + 255) / 256, 256, 0, s>>>(p.drab_t, p.drab_t_fix, nt);
        GRK_LAUNCH_CHECK();
      }
    }
  }
  return do_dkdv ? launch(p, a->head_dim, 3, s) : GRK_OK;
}

extern "C" int grk_attention_bwd(const grk_attn_args* a, const void* out, int64_t ldo, const void* dout,
                                 int64_t lddo, int dout_dtype, const float* lse, float* delta_ws, void* dq,
                                 int64_t lddq, void* dk, int64_t lddk, void* dv, int64_t lddv, float* drab,
                                 int64_t* drab_ws, void* stream) {
  return grk_attention_bwd_parts(a, out, ldo, dout, lddo, dout_dtype, lse, delta_ws, dq, lddq, dk, lddk, dv, lddv,
                                 drab, drab_ws, GRK_ATTN_BWD_DQ | GRK_ATTN_BWD_DKDV, stream);
}
