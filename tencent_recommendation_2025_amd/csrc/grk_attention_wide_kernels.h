// Wide-head attention kernels (head_dim 256 / 512) and their launcher
// template -- included by grk_attention_wide.hip (every product
// instantiation) and grk_attention_wide_fid.hip (the fp32-fidelity ones, a
// translation unit of their own: instantiated beside the others they
// perturbed the other kernels' register allocation, checked on the
// disassembly).  Design notes: grk_attention_wide.hip.
#pragma once
#include "grk_attention.h"

namespace grk {
namespace {


constexpr int kWRows = 32;   // queries (fwd, dQ) or keys (dK/dV) per workgroup
constexpr int kWTail = 304;  // kvs[32] | s_start | lses[32] | dlts[32], then rab (+ drab bins)
// TB (time bias) instantiations, after those: stamps[32] | rab_t[64] | drab_t bins[64] (dQ)
constexpr int kWTime = kWRows * 4 + kMaxTimeBuckets * 4 + kMaxTimeBuckets * 8;

template <int HD>
struct Wide {
  static constexpr int NW = HD / 64, NT = 64 * NW;  // column slices = waves
  static constexpr int DQ = 64, KSQ = DQ / 16, NDT = DQ / 32;
  static constexpr int EPW = 16 / NW;               // tile elements per lane each wave turns into P / dS
  static constexpr int IMG = kWRows * HD * 2;       // one 32-row bf16 image
  static constexpr int RED = NW * 8 * 64 * 8;       // partial products: [wave][element pair][lane] float2
  static constexpr int GX = NW * 64 * EPW * 4;      // P or dS as bf16 hi / lo words: [wave][lane][EPW]
};

// fp32 fidelity at head_dim 512: the hi + lo images (4 x 32 KiB) leave no room
// for whole-tile partial products, so the partials meet in RR rounds of 8 / RR
// element pairs (red_rounds) -- the same additions in the same order, 1 / RR of
// the LDS -- and the next tile is fetched at the top of the loop instead of
// under the current tile's products (its registers would spill).
template <int HD, bool FID>
struct WideF {
  static constexpr int RR = (FID && HD == 512) ? 4 : 1;
  static constexpr int RED = Wide<HD>::RED / RR;    // one partial-product buffer
  static constexpr bool PREFETCH = RR == 1;
};
constexpr size_t kMaxWideLds = 160 * 1024;

// This wave's partial 32x32 product (over its column slice) to LDS.
__device__ __forceinline__ void red_put(float2* red, int ws, int lane, const f32x16& x) {
#pragma unroll
  for (int pr = 0; pr < 8; ++pr) red[(ws * 8 + pr) * 64 + lane] = make_float2(x[2 * pr], x[2 * pr + 1]);
}

// The EPW elements k in [ws*EPW, (ws+1)*EPW) this wave owns, summed over the
// waves' partials in wave order.
template <int NW>
__device__ __forceinline__ void red_own(const float2* red, int ws, int lane, float* e) {
  constexpr int EPW = 16 / NW;
#pragma unroll
  for (int q = 0; q < EPW / 2; ++q) {
    const int pr = ws * (EPW / 2) + q;
    float2 t = red[pr * 64 + lane];
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      const float2 u = red[(w * 8 + pr) * 64 + lane];
      t.x += u.x;
      t.y += u.y;
    }
    e[2 * q] = t.x;
    e[2 * q + 1] = t.y;
  }
}

// Own elements -> bf16 hi / lo words (hi = bf16(x), lo = bf16(x - hi)).
template <int EPW>
__device__ __forceinline__ void put_words(uint32_t* gx, int ws, int lane, const float* g) {
  uint32_t* dst = gx + (ws * 64 + lane) * EPW;
#pragma unroll
  for (int e2 = 0; e2 < EPW / 2; ++e2) {
    const __bf16 h0 = static_cast<__bf16>(g[2 * e2]), h1 = static_cast<__bf16>(g[2 * e2 + 1]);
    const __bf16 l0 = static_cast<__bf16>(g[2 * e2] - static_cast<float>(h0));
    const __bf16 l1 = static_cast<__bf16>(g[2 * e2 + 1] - static_cast<float>(h1));
    dst[e2] = (uint32_t)__builtin_bit_cast(bf16_t, h0) | ((uint32_t)__builtin_bit_cast(bf16_t, h1) << 16);
    dst[EPW / 2 + e2] = (uint32_t)__builtin_bit_cast(bf16_t, l0) | ((uint32_t)__builtin_bit_cast(bf16_t, l1) << 16);
  }
}

// Elements 8 s2 .. 8 s2 + 7 of the whole tile (the MFMA B operand, as
// pack_acc forms it) from the owners' words.
template <int EPW>
__device__ __forceinline__ void get_words(const uint32_t* gx, int lane, int s2, bf16x8& hi, bf16x8& lo) {
  uint32_t hw[4], lw[4];
#pragma unroll
  for (int pp = 0; pp < 4; ++pp) {
    const int k = 8 * s2 + 2 * pp, w = k / EPW, kk = k % EPW;
    const uint32_t* src = gx + (w * 64 + lane) * EPW;
    hw[pp] = src[kk / 2];
    lw[pp] = src[EPW / 2 + kk / 2];
  }
  hi = __builtin_bit_cast(bf16x8, make_uint4(hw[0], hw[1], hw[2], hw[3]));
  lo = __builtin_bit_cast(bf16x8, make_uint4(lw[0], lw[1], lw[2], lw[3]));
}

// Tile row of element k (acc_row with k not a compile-time constant).
__device__ __forceinline__ int elem_row(int k, int hh) { return (k & 3) + 8 * (k >> 2) + 4 * hh; }

__device__ __forceinline__ void* shift(void* p, bool f32, int n) { return (char*)p + (size_t)n * (f32 ? 4 : 2); }

// Workgroup barrier for LDS hand-offs only (waits for LDS operations, not for
// the next tile's global loads, which __syncthreads()' fence would drain).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// red_put + barrier + red_own (of one or, TWO, two products) in RR rounds: in
// round rd every wave writes pairs [rd PR, (rd + 1) PR) of its partials and the
// waves owning one of those pairs sum them, wave 0 first, as red_own does.
template <int NW, int RR, bool TWO>
__device__ __forceinline__ void red_rounds(float2* red, float2* red2, int ws, int lane, const f32x16& x,
                                           const f32x16& x2, float* e, float* e2) {
  constexpr int PR = 8 / RR, OWN = 16 / NW / 2;  // pairs per round; pairs a wave owns
#pragma unroll
  for (int rd = 0; rd < RR; ++rd) {
    if (rd > 0) lds_barrier();  // the previous round's partials have been read
#pragma unroll
    for (int q = 0; q < PR; ++q) {
      const int pr = rd * PR + q;
      red[(ws * PR + q) * 64 + lane] = make_float2(x[2 * pr], x[2 * pr + 1]);
      if (TWO) red2[(ws * PR + q) * 64 + lane] = make_float2(x2[2 * pr], x2[2 * pr + 1]);
    }
    lds_barrier();
#pragma unroll
    for (int q = 0; q < OWN; ++q) {
      const int lp = ws * OWN + q - rd * PR;  // the owned pair's slot in this round (wave-uniform)
      if (lp < 0 || lp >= PR) continue;
      float2 t = red[lp * 64 + lane], t2 = TWO ? red2[lp * 64 + lane] : make_float2(0.f, 0.f);
#pragma unroll
      for (int w = 1; w < NW; ++w) {
        const float2 u = red[(w * PR + lp) * 64 + lane];
        t.x += u.x;
        t.y += u.y;
        if (TWO) {
          const float2 u2 = red2[(w * PR + lp) * 64 + lane];
          t2.x += u2.x;
          t2.y += u2.y;
        }
      }
      e[2 * q] = t.x;
      e[2 * q + 1] = t.y;
      if (TWO) {
        e2[2 * q] = t2.x;
        e2[2 * q + 1] = t2.y;
      }
    }
  }
}

// 32 rows x HD of a [B*T, ld] head slice (bf16, or fp32 when F32), zero past
// T: fetch() into registers under the previous tile's work, put() into the
// swizzled LDS image (rounded to bf16, SiLU on the way when act) between two
// barriers.
template <int HD, int NT, bool F32>
struct WRows {
  static constexpr int NCH = HD / 8, PER = kWRows * NCH / NT;  // 16-byte chunks per thread
  uint4 v[F32 ? 2 * PER : PER];
  __device__ __forceinline__ void fetch(const void* src, int64_t ld, int b, int T, int h, int r0) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = threadIdx.x + j * NT, row = u / NCH, c = u % NCH, t = r0 + row;
      const int64_t off = ((int64_t)b * T + t) * ld + h * HD + c * 8;
      if (F32) {
        v[2 * j] = v[2 * j + 1] = make_uint4(0, 0, 0, 0);
        if (t < T) {
          v[2 * j] = reinterpret_cast<const uint4*>((const float*)src + off)[0];
          v[2 * j + 1] = reinterpret_cast<const uint4*>((const float*)src + off)[1];
        }
      } else {
        v[j] = make_uint4(0, 0, 0, 0);
        if (t < T) v[j] = *reinterpret_cast<const uint4*>((const bf16_t*)src + off);
      }
    }
  }
  __device__ __forceinline__ void put(char* img, bool act) const {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = threadIdx.x + j * NT, row = u / NCH, c = u % NCH;
      bf16x8 x;
      if (F32) {
        const float4 a = __builtin_bit_cast(float4, v[2 * j]), d = __builtin_bit_cast(float4, v[2 * j + 1]);
        x[0] = (__bf16)a.x; x[1] = (__bf16)a.y; x[2] = (__bf16)a.z; x[3] = (__bf16)a.w;
        x[4] = (__bf16)d.x; x[5] = (__bf16)d.y; x[6] = (__bf16)d.z; x[7] = (__bf16)d.w;
      } else {
        x = __builtin_bit_cast(bf16x8, v[j]);
      }
      if (act) x = silu8(x);
      *reinterpret_cast<uint4*>(img + lds_off<HD>(row, c * 8)) = __builtin_bit_cast(uint4, x);
    }
  }
};

// fp32-fidelity (FID) tiles: 32 rows x HD read exactly (dt: GRK_F32 / GRK_F16 /
// GRK_BF16, gload8f), SiLU in fp32 when act, put() as a bf16 hi image and a
// bf16 lo (= x - hi) image -- the whole-sequence kernels' stage_pair_split.
template <int HD, int NT>
struct WRowsF {
  static constexpr int NCH = HD / 8, PER = kWRows * NCH / NT;
  float v[PER][8];
  __device__ __forceinline__ void fetch(const void* src, int64_t ld, int dt, int b, int T, int h, int r0) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = threadIdx.x + j * NT, row = u / NCH, c = u % NCH, t = r0 + row;
      gload8f(src, ((int64_t)b * T + (t < T ? t : 0)) * ld + h * HD + c * 8, dt, t < T, v[j]);
    }
  }
  __device__ __forceinline__ void put(char* hi, char* lo, bool act) const {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = threadIdx.x + j * NT, row = u / NCH, c = u % NCH;
      float f[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = act ? silu(v[j][e]) : v[j][e];
      bf16x8 xh, xl;
      split8(f, xh, xl);
      const int o = lds_off<HD>(row, c * 8);
      *reinterpret_cast<uint4*>(hi + o) = __builtin_bit_cast(uint4, xh);
      *reinterpret_cast<uint4*>(lo + o) = __builtin_bit_cast(uint4, xl);
    }
  }
};

// FID register fragments: this wave's KSQ 8-wide pieces of row `row` as hi + lo.
template <int KSQ>
__device__ __forceinline__ void frag_split(bf16x8* fh, bf16x8* fl, const void* base, int64_t off, int dt, bool act,
                                           bool ok) {
#pragma unroll
  for (int ks = 0; ks < KSQ; ++ks) {
    float f[8];
    gload8f(base, off + 16 * ks, dt, ok, f);
    if (act)
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = silu(f[e]);
    split8(f, fh[ks], fl[ks]);
  }
}

// Element n past a raw q/k/v pointer of dtype dt (the dSiLU source of a store).
__device__ __forceinline__ const void* at_dt(const void* p, int dt, int n) {
  return (const char*)p + (size_t)n * (dt == 0 ? 4 : 2);
}

__device__ __forceinline__ uint8_t key_ok(const AttnParams& p, int b, int t) {
  return (t < p.T) && (!p.key_valid || p.key_valid[(int64_t)b * p.T + t]);
}

// ================================================================ forward ====
// TB: with the HSTU time bias rab_t[h, time_bucket(t_q - t_k)] (KIND 1).
// FID: fp32 fidelity (precise = 2): q/k/v read exactly and split into bf16
// hi + lo; every product hi*hi + hi*lo + lo*hi; the lo images sit in front.
template <int HD, int KIND, bool TB = false, bool FID = false>
__global__ void __launch_bounds__(HD) k_attn_fwd_wide(AttnParams p) {
  using W = Wide<HD>;
  using WF = WideF<HD, FID>;
  constexpr int KSQ = W::KSQ, NDT = W::NDT, NW = W::NW, EPW = W::EPW;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  char* smem = smem_raw + (FID ? 2 * W::IMG : 0);
  char* Kl = smem_raw;           // FID: lo images
  char* Vl = smem_raw + W::IMG;
  char* Ks = smem;
  char* Vs = smem + W::IMG;
  float2* red = reinterpret_cast<float2*>(smem + 2 * W::IMG);
  uint32_t* gxp = reinterpret_cast<uint32_t*>(smem + 2 * W::IMG + WF::RED);
  float* mx = reinterpret_cast<float*>(smem + 2 * W::IMG + WF::RED + W::GX);  // [wave][lane]
  char* tail = smem + 2 * W::IMG + WF::RED + W::GX + NW * 64 * 4;
  uint8_t* kvs = reinterpret_cast<uint8_t*>(tail);
  int* s_start = reinterpret_cast<int*>(tail + 32);
  float* rabs = reinterpret_cast<float*>(tail + kWTail);
  int* tsk = reinterpret_cast<int*>(rabs + (p.nb + 1) / 2 * 2);  // TB: the key tile's stamps
  float* rtab = reinterpret_cast<float*>(tsk + kWRows);          // TB: rab_t[h, :]

  const int b = blockIdx.z, h = blockIdx.y, T = p.T;
  const int ws = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int q0 = blockIdx.x * kWRows, myq = q0 + r;
  const bool qok = myq < T;
  const int start = seq_start(p.key_valid, b, T, s_start);
  if (KIND == 1)
    for (int j = threadIdx.x; j < p.nb; j += blockDim.x) rabs[j] = p.rab[h * p.nb + j];
  int tq = 0;
  if constexpr (TB) {
    for (int j = threadIdx.x; j < p.nbt; j += blockDim.x) rtab[j] = p.rab_t[h * p.nbt + j];
    tq = rel_stamp(p, b, T, start, myq);
  }
  const int c0 = ws * W::DQ;  // this wave's columns within the head

  bf16x8 qf[KSQ], ql[FID ? KSQ : 1];
  if constexpr (FID) {
    frag_split<KSQ>(qf, ql, p.q, ((int64_t)b * T + (qok ? myq : 0)) * p.ldq + h * HD + c0 + 8 * hh, p.in_dt, p.act,
                    qok);
  } else {
    const bf16_t* qrow = p.q + ((int64_t)b * T + (qok ? myq : 0)) * p.ldq + h * HD + c0;
#pragma unroll
    for (int ks = 0; ks < KSQ; ++ks) {
      qf[ks] = gload8(qrow + 16 * ks + 8 * hh, qok);
      if (p.act) qf[ks] = silu8(qf[ks]);
    }
  }
  f32x16 o[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) o[dt] = acc_zero();
  float m = -INFINITY, lw = 0.f;  // running max (same in every wave); this wave's share of the row sum
  const float sl2 = p.scale * kLog2e;
  const float rdrop = 1.0f / (1.0f - p.dropout_p);
  const bool drop = KIND == 0 && p.dropout_p > 0.f;
  const unsigned long long seed = drop ? attn_seed(p) : 0ull;
  const int bh = b * p.H + h;

  const int kend = min(T, q0 + kWRows), kbeg = (start / 32) * 32;
  WRows<HD, W::NT, false> kt, vt;
  WRowsF<HD, W::NT> ktf, vtf;
  uint8_t kvb = 0;
  if (kbeg < kend) {
    if constexpr (FID) {
      if (WF::PREFETCH) {
        ktf.fetch(p.k, p.ldk, p.in_dt, b, T, h, kbeg);
        vtf.fetch(p.v, p.ldv, p.in_dt, b, T, h, kbeg);
      }
    } else {
      kt.fetch(p.k, p.ldk, b, T, h, kbeg);
      vt.fetch(p.v, p.ldv, b, T, h, kbeg);
    }
    if (threadIdx.x < 32) kvb = key_ok(p, b, kbeg + threadIdx.x);
  }
  for (int kb = kbeg; kb < kend; kb += 32) {
    if (!WF::PREFETCH) {  // FID at 512: this tile fetched here, not under the previous one
      ktf.fetch(p.k, p.ldk, p.in_dt, b, T, h, kb);
      vtf.fetch(p.v, p.ldv, p.in_dt, b, T, h, kb);
    }
    __syncthreads();
    if constexpr (FID) {
      ktf.put(Ks, Kl, p.act);
      vtf.put(Vs, Vl, p.act);
    } else {
      kt.put(Ks, p.act);
      vt.put(Vs, p.act);
    }
    if (threadIdx.x < 32) {
      kvs[threadIdx.x] = kvb;
      if constexpr (TB) tsk[threadIdx.x] = rel_stamp(p, b, T, start, kb + threadIdx.x);
    }
    lds_barrier();
    if (kb + 32 < kend) {  // in flight under this tile's work
      if constexpr (FID) {
        if (WF::PREFETCH) {
          ktf.fetch(p.k, p.ldk, p.in_dt, b, T, h, kb + 32);
          vtf.fetch(p.v, p.ldv, p.in_dt, b, T, h, kb + 32);
        }
      } else {
        kt.fetch(p.k, p.ldk, b, T, h, kb + 32);
        vt.fetch(p.v, p.ldv, b, T, h, kb + 32);
      }
      if (threadIdx.x < 32) kvb = key_ok(p, b, kb + 32 + threadIdx.x);
    }
    f32x16 s = acc_zero();
    if constexpr (FID) {
#pragma unroll
      for (int ks = 0; ks < KSQ; ++ks) {
        const bf16x8 kh = lds_row8<HD>(Ks, r, c0 + 16 * ks + 8 * hh);
        s = mfma(kh, qf[ks], s);
        s = mfma(kh, ql[ks], s);
        s = mfma(lds_row8<HD>(Kl, r, c0 + 16 * ks + 8 * hh), qf[ks], s);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < KSQ; ++ks) s = mfma(lds_row8<HD>(Ks, r, c0 + 16 * ks + 8 * hh), qf[ks], s);
    }
    float se[EPW], pd[EPW];
    if constexpr (WF::RR > 1) {
      red_rounds<NW, WF::RR, false>(red, red, ws, lane, s, s, se, se);
    } else {
      red_put(red, ws, lane, s);
      lds_barrier();
      red_own<NW>(red, ws, lane, se);
    }
    if (KIND == 0) {
      float x[EPW], tmax = -INFINITY;
#pragma unroll
      for (int e = 0; e < EPW; ++e) {
        const int kr = elem_row(ws * EPW + e, hh), key = kb + kr;
        const bool ok = qok && key <= myq && kvs[kr];
        x[e] = ok ? se[e] * sl2 : -INFINITY;
        tmax = fmaxf(tmax, x[e]);
      }
      mx[ws * 64 + lane] = fmaxf(tmax, __shfl_xor(tmax, 32));
      lds_barrier();
#pragma unroll
      for (int w = 0; w < NW; ++w) tmax = fmaxf(tmax, mx[w * 64 + lane]);
      const float mn = fmaxf(m, tmax);
      const float alpha = (mn == -INFINITY) ? 1.f : exp2f(m - mn);
      float rs = 0.f;
#pragma unroll
      for (int e = 0; e < EPW; ++e) {
        const float pr = (x[e] == -INFINITY) ? 0.f : exp2f(x[e] - mn);
        rs += pr;
        pd[e] = pr;
        if (drop) {
          const int key = kb + elem_row(ws * EPW + e, hh);
          pd[e] = drop_keep(seed, bh, myq, key, T, p.dropout_p) ? pr * rdrop : 0.f;
        }
      }
      lw = lw * alpha + rs;
      m = mn;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) o[dt] *= alpha;
    } else {
#pragma unroll
      for (int e = 0; e < EPW; ++e) {
        const int kr = elem_row(ws * EPW + e, hh), key = kb + kr;
        const bool ok = qok && key <= myq && kvs[kr];
        float sp = se[e] * p.scale + rabs[ok ? min(myq - key, p.nb - 1) : 0];
        if constexpr (TB) sp += rtab[time_bucket(tq - tsk[kr], p.nbt)];
        pd[e] = ok ? silu(sp) * p.inv_n : 0.f;
      }
    }
    put_words<EPW>(gxp, ws, lane, pd);
    lds_barrier();
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      bf16x8 ph, pl;
      get_words<EPW>(gxp, lane, s2, ph, pl);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const bf16x8 vf = lds_tr8<HD>(Vs, 16 * s2, c0 + 32 * dt, lane);
        o[dt] = mfma(vf, ph, o[dt]);
        if (p.precise) o[dt] = mfma(vf, pl, o[dt]);
        if constexpr (FID) o[dt] = mfma(lds_tr8<HD>(Vl, 16 * s2, c0 + 32 * dt, lane), ph, o[dt]);
      }
    }
  }
  float mul = 1.f;
  if (KIND == 0) {
    // row sum = every wave's share, both half-waves, in a fixed order
    mx[ws * 64 + lane] = lw;
    lds_barrier();
    float l = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) l += mx[w * 64 + r] + mx[w * 64 + 32 + r];
    mul = l > 0.f ? 1.0f / l : 0.f;
    if (ws == 0 && hh == 0 && qok && p.lse) p.lse[(int64_t)bh * T + myq] = l > 0.f ? (m + log2f(l)) * kLn2 : -INFINITY;
  }
  store_rows<HD, NDT>(shift(p.out, p.out_f32, c0), p.ldo, p.out_f32, (int64_t)b * T + myq, h, hh, o, mul, qok);
}

// ================================================================ dQ =========
template <int HD, int KIND, bool TB = false, bool FID = false>
__global__ void __launch_bounds__(HD) k_attn_dq_wide(AttnParams p) {
  using W = Wide<HD>;
  using WF = WideF<HD, FID>;
  constexpr int KSQ = W::KSQ, NDT = W::NDT, NW = W::NW, EPW = W::EPW;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  char* smem = smem_raw + (FID ? 2 * W::IMG : 0);
  char* Kl = smem_raw;           // FID: lo images
  char* Vl = smem_raw + W::IMG;
  char* Ks = smem;
  char* Vs = smem + W::IMG;
  float2* red = reinterpret_cast<float2*>(smem + 2 * W::IMG);
  float2* red2 = reinterpret_cast<float2*>(smem + 2 * W::IMG + WF::RED);
  uint32_t* gxd = reinterpret_cast<uint32_t*>(smem + 2 * W::IMG + 2 * WF::RED);
  char* tail = smem + 2 * W::IMG + 2 * WF::RED + W::GX;
  uint8_t* kvs = reinterpret_cast<uint8_t*>(tail);
  int* s_start = reinterpret_cast<int*>(tail + 32);
  float* rabs = reinterpret_cast<float*>(tail + kWTail);
  unsigned long long* bins = reinterpret_cast<unsigned long long*>(rabs + (p.nb + 1) / 2 * 2);
  int* tsk = reinterpret_cast<int*>(bins + p.nb);                                   // TB: key tile stamps
  float* rtab = reinterpret_cast<float*>(tsk + kWRows);                             // TB: rab_t[h, :]
  unsigned long long* tbins = reinterpret_cast<unsigned long long*>(rtab + kMaxTimeBuckets);  // TB: drab_t

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
  int tq = 0;
  if constexpr (TB) {
    for (int j = threadIdx.x; j < p.nbt; j += blockDim.x) {
      rtab[j] = p.rab_t[h * p.nbt + j];
      tbins[j] = 0ull;
    }
    tq = rel_stamp(p, b, T, start, myq);
  }
  const int bh = b * p.H + h;
  const int c0 = ws * W::DQ;
  const int64_t tok = (int64_t)b * T + (qok ? myq : 0);

  bf16x8 qf[KSQ], dof[KSQ], ql[FID ? KSQ : 1], dol[FID ? KSQ : 1];
  if constexpr (FID) {
    frag_split<KSQ>(qf, ql, p.q, tok * p.ldq + h * HD + c0 + 8 * hh, p.in_dt, p.act, qok);
    frag_split<KSQ>(dof, dol, p.dout, tok * p.lddo + h * HD + c0 + 8 * hh, p.dout_f32 ? 0 : 1, false, qok);
  } else {
#pragma unroll
    for (int ks = 0; ks < KSQ; ++ks) {
      qf[ks] = gload8(p.q + tok * p.ldq + h * HD + c0 + 16 * ks + 8 * hh, qok);
      if (p.act) qf[ks] = silu8(qf[ks]);
      dof[ks] = gload8_any(p.dout, tok * p.lddo + h * HD + c0 + 16 * ks + 8 * hh, p.dout_f32, qok);
    }
  }
  float lse2 = 0.f, dlt = 0.f;
  if (KIND == 0 && qok) {
    lse2 = p.lse[(int64_t)bh * T + myq] * kLog2e;
    dlt = p.delta[(int64_t)bh * T + myq];
  }
  const bool row_live = KIND == 1 || lse2 != -INFINITY;
  f32x16 acc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) acc[dt] = acc_zero();
  const float sl2 = p.scale * kLog2e;
  const float rdrop = 1.0f / (1.0f - p.dropout_p);
  const bool drop = KIND == 0 && p.dropout_p > 0.f;
  const unsigned long long seed = drop ? attn_seed(p) : 0ull;

  const int kend = min(T, q0 + kWRows), kbeg = (start / 32) * 32;
  WRows<HD, W::NT, false> kt, vt;
  WRowsF<HD, W::NT> ktf, vtf;
  uint8_t kvb = 0;
  if (kbeg < kend) {
    if constexpr (FID) {
      if (WF::PREFETCH) {
        ktf.fetch(p.k, p.ldk, p.in_dt, b, T, h, kbeg);
        vtf.fetch(p.v, p.ldv, p.in_dt, b, T, h, kbeg);
      }
    } else {
      kt.fetch(p.k, p.ldk, b, T, h, kbeg);
      vt.fetch(p.v, p.ldv, b, T, h, kbeg);
    }
    if (threadIdx.x < 32) kvb = key_ok(p, b, kbeg + threadIdx.x);
  }
  for (int kb = kbeg; kb < kend; kb += 32) {
    if (!WF::PREFETCH) {  // FID at 512: this tile fetched here, not under the previous one
      ktf.fetch(p.k, p.ldk, p.in_dt, b, T, h, kb);
      vtf.fetch(p.v, p.ldv, p.in_dt, b, T, h, kb);
    }
    __syncthreads();
    if constexpr (FID) {
      ktf.put(Ks, Kl, p.act);
      vtf.put(Vs, Vl, p.act);
    } else {
      kt.put(Ks, p.act);
      vt.put(Vs, p.act);
    }
    if (threadIdx.x < 32) {
      kvs[threadIdx.x] = kvb;
      if constexpr (TB) tsk[threadIdx.x] = rel_stamp(p, b, T, start, kb + threadIdx.x);
    }
    lds_barrier();
    if (kb + 32 < kend) {  // in flight under this tile's work
      if constexpr (FID) {
        if (WF::PREFETCH) {
          ktf.fetch(p.k, p.ldk, p.in_dt, b, T, h, kb + 32);
          vtf.fetch(p.v, p.ldv, p.in_dt, b, T, h, kb + 32);
        }
      } else {
        kt.fetch(p.k, p.ldk, b, T, h, kb + 32);
        vt.fetch(p.v, p.ldv, b, T, h, kb + 32);
      }
      if (threadIdx.x < 32) kvb = key_ok(p, b, kb + 32 + threadIdx.x);
    }
    f32x16 s = acc_zero(), dp = acc_zero();
    if constexpr (FID) {
#pragma unroll
      for (int ks = 0; ks < KSQ; ++ks) {
        const bf16x8 kh = lds_row8<HD>(Ks, r, c0 + 16 * ks + 8 * hh);
        const bf16x8 vh = lds_row8<HD>(Vs, r, c0 + 16 * ks + 8 * hh);
        s = mfma(kh, qf[ks], s);
        dp = mfma(vh, dof[ks], dp);
        s = mfma(kh, ql[ks], s);
        s = mfma(lds_row8<HD>(Kl, r, c0 + 16 * ks + 8 * hh), qf[ks], s);
        dp = mfma(vh, dol[ks], dp);
        dp = mfma(lds_row8<HD>(Vl, r, c0 + 16 * ks + 8 * hh), dof[ks], dp);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < KSQ; ++ks) {
        s = mfma(lds_row8<HD>(Ks, r, c0 + 16 * ks + 8 * hh), qf[ks], s);
        dp = mfma(lds_row8<HD>(Vs, r, c0 + 16 * ks + 8 * hh), dof[ks], dp);
      }
    }
    float se[EPW], de[EPW], ds[EPW];
    if constexpr (WF::RR > 1) {
      red_rounds<NW, WF::RR, true>(red, red2, ws, lane, s, dp, se, de);
    } else {
      red_put(red, ws, lane, s);
      red_put(red2, ws, lane, dp);
      lds_barrier();
      red_own<NW>(red, ws, lane, se);
      red_own<NW>(red2, ws, lane, de);
    }
#pragma unroll
    for (int e = 0; e < EPW; ++e) {
      const int kr = elem_row(ws * EPW + e, hh), key = kb + kr;
      const bool ok = qok && row_live && key <= myq && kvs[kr];
      if (KIND == 0) {
        const float pv = ok ? exp2f(se[e] * sl2 - lse2) : 0.f;
        float dpv = de[e];
        if (drop) dpv = drop_keep(seed, bh, myq, key, T, p.dropout_p) ? dpv * rdrop : 0.f;
        ds[e] = pv * (dpv - dlt);
      } else {
        const int bk = min(myq - key, p.nb - 1);
        float sp = se[e] * p.scale + rabs[ok ? bk : 0];
        int tbk = 0;
        if constexpr (TB) {
          tbk = time_bucket(tq - tsk[kr], p.nbt);
          sp += rtab[tbk];
        }
        ds[e] = ok ? de[e] * dsilu(sp) * p.inv_n : 0.f;
        if (ok && ds[e] != 0.f && p.drab) atomicAdd(&bins[bk], to_fix(ds[e]));
        if constexpr (TB)
          if (ok && ds[e] != 0.f && p.drab_t) atomicAdd(&tbins[tbk], to_fix(ds[e]));
      }
    }
    put_words<EPW>(gxd, ws, lane, ds);
    lds_barrier();
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      bf16x8 dh, dl;
      get_words<EPW>(gxd, lane, s2, dh, dl);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const bf16x8 kf = lds_tr8<HD>(Ks, 16 * s2, c0 + 32 * dt, lane);
        acc[dt] = mfma(kf, dh, acc[dt]);
        if (p.precise) acc[dt] = mfma(kf, dl, acc[dt]);
        if constexpr (FID) acc[dt] = mfma(lds_tr8<HD>(Kl, 16 * s2, c0 + 32 * dt, lane), dh, acc[dt]);
      }
    }
  }
  if constexpr (FID)
    store_rows<HD, NDT>(shift(p.dq, p.out_f32, c0), p.lddq, p.out_f32, (int64_t)b * T + myq, h, hh, acc, p.scale, qok,
                        p.act ? at_dt(p.q, p.in_dt, c0) : nullptr, p.ldq, p.in_dt);
  else
    store_rows<HD, NDT>(shift(p.dq, p.out_f32, c0), p.lddq, p.out_f32, (int64_t)b * T + myq, h, hh, acc, p.scale, qok,
                        p.act ? (const void*)(p.q + c0) : nullptr, p.ldq);
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
template <int HD, int KIND, bool DF32, bool TB = false, bool FID = false>
__global__ void __launch_bounds__(HD) k_attn_dkdv_wide(AttnParams p) {
  using W = Wide<HD>;
  using WF = WideF<HD, FID>;
  constexpr int KSQ = W::KSQ, NDT = W::NDT, NW = W::NW, EPW = W::EPW;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  char* smem = smem_raw + (FID ? 2 * W::IMG : 0);
  char* Ql = smem_raw;           // FID: lo images
  char* Dl = smem_raw + W::IMG;
  char* Qs = smem;
  char* Ds = smem + W::IMG;
  float2* red = reinterpret_cast<float2*>(smem + 2 * W::IMG);
  float2* red2 = reinterpret_cast<float2*>(smem + 2 * W::IMG + WF::RED);
  uint32_t* gxp = reinterpret_cast<uint32_t*>(smem + 2 * W::IMG + 2 * WF::RED);
  uint32_t* gxd = gxp + W::GX / 4;
  char* tail = smem + 2 * W::IMG + 2 * WF::RED + 2 * W::GX;
  int* s_start = reinterpret_cast<int*>(tail + 32);
  float* lses = reinterpret_cast<float*>(tail + 48);
  float* dlts = lses + 32;
  float* rabs = reinterpret_cast<float*>(tail + kWTail);
  int* tsq = reinterpret_cast<int*>(rabs + (p.nb + 1) / 2 * 2);  // TB: the query tile's stamps
  float* rtab = reinterpret_cast<float*>(tsq + kWRows);          // TB: rab_t[h, :]

  const int b = blockIdx.z, h = blockIdx.y, T = p.T;
  const int ws = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int k0 = blockIdx.x * kWRows, myk = k0 + r;
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
  const int c0 = ws * W::DQ;
  const int64_t tok = (int64_t)b * T + (myk < T ? myk : 0);

  bf16x8 kf[KSQ], vf[KSQ], kl[FID ? KSQ : 1], vl[FID ? KSQ : 1];
  if constexpr (FID) {
    frag_split<KSQ>(kf, kl, p.k, tok * p.ldk + h * HD + c0 + 8 * hh, p.in_dt, p.act, myk < T);
    frag_split<KSQ>(vf, vl, p.v, tok * p.ldv + h * HD + c0 + 8 * hh, p.in_dt, p.act, myk < T);
  } else {
#pragma unroll
    for (int ks = 0; ks < KSQ; ++ks) {
      kf[ks] = gload8(p.k + tok * p.ldk + h * HD + c0 + 16 * ks + 8 * hh, myk < T);
      vf[ks] = gload8(p.v + tok * p.ldv + h * HD + c0 + 16 * ks + 8 * hh, myk < T);
      if (p.act) {
        kf[ks] = silu8(kf[ks]);
        vf[ks] = silu8(vf[ks]);
      }
    }
  }
  f32x16 dk[NDT], dv[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) { dk[dt] = acc_zero(); dv[dt] = acc_zero(); }
  const float sl2 = p.scale * kLog2e;
  const float rdrop = 1.0f / (1.0f - p.dropout_p);
  const bool drop = KIND == 0 && p.dropout_p > 0.f;
  const unsigned long long seed = drop ? attn_seed(p) : 0ull;

  // queries that can see this block's keys: q >= k0 and q >= start
  const int qbeg = (max(k0, start) / 32) * 32;
  WRows<HD, W::NT, false> qt;
  WRows<HD, W::NT, DF32> dt_;
  WRowsF<HD, W::NT> qtf, dtf;
  float lv = -INFINITY, dl = 0.f;
  auto fetch = [&](int qb) {
    if constexpr (FID) {
      qtf.fetch(p.q, p.ldq, p.in_dt, b, T, h, qb);
      dtf.fetch(p.dout, p.lddo, DF32 ? 0 : 1, b, T, h, qb);
    } else {
      qt.fetch(p.q, p.ldq, b, T, h, qb);
      dt_.fetch(p.dout, p.lddo, b, T, h, qb);
    }
    const int t = qb + (int)threadIdx.x;
    lv = -INFINITY;
    dl = 0.f;
    if (KIND == 0 && threadIdx.x < 32 && t < T) {
      lv = p.lse[(int64_t)bh * T + t];
      dl = p.delta[(int64_t)bh * T + t];
    }
  };
  if (WF::PREFETCH && qbeg < T) fetch(qbeg);
  for (int qb = qbeg; qb < T; qb += 32) {
    if (!WF::PREFETCH) fetch(qb);  // FID at 512: this tile fetched here, not under the previous one
    __syncthreads();
    if constexpr (FID) {
      qtf.put(Qs, Ql, p.act);
      dtf.put(Ds, Dl, false);
    } else {
      qt.put(Qs, p.act);
      dt_.put(Ds, false);
    }
    if (threadIdx.x < 32) {
      lses[threadIdx.x] = lv * kLog2e;
      dlts[threadIdx.x] = dl;
      if constexpr (TB) tsq[threadIdx.x] = rel_stamp(p, b, T, start, qb + threadIdx.x);
    }
    lds_barrier();
    if (WF::PREFETCH && qb + 32 < T) fetch(qb + 32);  // in flight under this tile's work
    f32x16 s = acc_zero(), dp = acc_zero();
    if constexpr (FID) {
#pragma unroll
      for (int ks = 0; ks < KSQ; ++ks) {
        const bf16x8 qh = lds_row8<HD>(Qs, r, c0 + 16 * ks + 8 * hh);
        const bf16x8 dh = lds_row8<HD>(Ds, r, c0 + 16 * ks + 8 * hh);
        s = mfma(qh, kf[ks], s);
        dp = mfma(dh, vf[ks], dp);
        s = mfma(qh, kl[ks], s);
        s = mfma(lds_row8<HD>(Ql, r, c0 + 16 * ks + 8 * hh), kf[ks], s);
        dp = mfma(dh, vl[ks], dp);
        dp = mfma(lds_row8<HD>(Dl, r, c0 + 16 * ks + 8 * hh), vf[ks], dp);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < KSQ; ++ks) {
        s = mfma(lds_row8<HD>(Qs, r, c0 + 16 * ks + 8 * hh), kf[ks], s);
        dp = mfma(lds_row8<HD>(Ds, r, c0 + 16 * ks + 8 * hh), vf[ks], dp);
      }
    }
    float se[EPW], de[EPW], pd[EPW], ds[EPW];
    if constexpr (WF::RR > 1) {
      red_rounds<NW, WF::RR, true>(red, red2, ws, lane, s, dp, se, de);
    } else {
      red_put(red, ws, lane, s);
      red_put(red2, ws, lane, dp);
      lds_barrier();
      red_own<NW>(red, ws, lane, se);
      red_own<NW>(red2, ws, lane, de);
    }
#pragma unroll
    for (int e = 0; e < EPW; ++e) {
      const int qr = elem_row(ws * EPW + e, hh), q = qb + qr;
      const bool ok = kok && q < T && myk <= q;
      if (KIND == 0) {
        const float lq = lses[qr];
        const float pv = (ok && lq != -INFINITY) ? exp2f(se[e] * sl2 - lq) : 0.f;
        float dpv = de[e];
        pd[e] = pv;
        if (drop) {
          const bool keep = drop_keep(seed, bh, q, myk, T, p.dropout_p);
          pd[e] = keep ? pv * rdrop : 0.f;
          dpv = keep ? dpv * rdrop : 0.f;
        }
        ds[e] = pv * (dpv - dlts[qr]);
      } else {
        float sp = se[e] * p.scale + rabs[ok ? min(q - myk, p.nb - 1) : 0];
        if constexpr (TB) sp += rtab[time_bucket(tsq[qr] - tk, p.nbt)];
        pd[e] = ok ? silu(sp) * p.inv_n : 0.f;
        ds[e] = ok ? de[e] * dsilu(sp) * p.inv_n : 0.f;
      }
    }
    put_words<EPW>(gxp, ws, lane, pd);
    put_words<EPW>(gxd, ws, lane, ds);
    lds_barrier();
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      bf16x8 ph, pl, dh, dl2;
      get_words<EPW>(gxp, lane, s2, ph, pl);
      get_words<EPW>(gxd, lane, s2, dh, dl2);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const bf16x8 dof = lds_tr8<HD>(Ds, 16 * s2, c0 + 32 * dt, lane);
        const bf16x8 qf = lds_tr8<HD>(Qs, 16 * s2, c0 + 32 * dt, lane);
        dv[dt] = mfma(dof, ph, dv[dt]);
        dk[dt] = mfma(qf, dh, dk[dt]);
        if (p.precise) {
          dv[dt] = mfma(dof, pl, dv[dt]);
          dk[dt] = mfma(qf, dl2, dk[dt]);
        }
        if constexpr (FID) {
          dv[dt] = mfma(lds_tr8<HD>(Dl, 16 * s2, c0 + 32 * dt, lane), ph, dv[dt]);
          dk[dt] = mfma(lds_tr8<HD>(Ql, 16 * s2, c0 + 32 * dt, lane), dh, dk[dt]);
        }
      }
    }
  }
  const int64_t otok = (int64_t)b * T + myk;
  if constexpr (FID) {
    store_rows<HD, NDT>(shift(p.dk, p.out_f32, c0), p.lddk, p.out_f32, otok, h, hh, dk, p.scale, myk < T,
                        p.act ? at_dt(p.k, p.in_dt, c0) : nullptr, p.ldk, p.in_dt);
    store_rows<HD, NDT>(shift(p.dv, p.out_f32, c0), p.lddv, p.out_f32, otok, h, hh, dv, 1.f, myk < T,
                        p.act ? at_dt(p.v, p.in_dt, c0) : nullptr, p.ldv, p.in_dt);
  } else {
    store_rows<HD, NDT>(shift(p.dk, p.out_f32, c0), p.lddk, p.out_f32, otok, h, hh, dk, p.scale, myk < T,
                        p.act ? (const void*)(p.k + c0) : nullptr, p.ldk);
    store_rows<HD, NDT>(shift(p.dv, p.out_f32, c0), p.lddv, p.out_f32, otok, h, hh, dv, 1.f, myk < T,
                        p.act ? (const void*)(p.v + c0) : nullptr, p.ldv);
  }
}

inline int wide_lds_refused(size_t lds) {
  set_error("wide-head attention needs %zu bytes of LDS (at most %zu: fewer relative-position buckets)", lds,
            kMaxWideLds);
  return GRK_EUNSUPPORTED;
}

template <int HD, bool FID = false>
int wide_hd(const AttnParams& p, int which, hipStream_t s) {
  using W = Wide<HD>;
  constexpr size_t RED = WideF<HD, FID>::RED;
  const dim3 grid((p.T + kWRows - 1) / kWRows, p.H, p.B);
  const bool hstu = p.kind == GRK_ATTN_HSTU;
  const bool tb = hstu && p.nbt > 0;
  const size_t rab = hstu ? (size_t)(p.nb + 1) / 2 * 2 * 4 : 0;
  const size_t tlds = (tb ? (size_t)kWTime : 0) + (FID ? (size_t)2 * W::IMG : 0);  // + FID's lo images
  if (which == 0) {
    const size_t lds = 2 * W::IMG + RED + W::GX + W::NW * 64 * 4 + kWTail + rab + tlds;
    if (lds > kMaxWideLds) return wide_lds_refused(lds);
    launch_lds(tb     ? k_attn_fwd_wide<HD, 1, true, FID>
               : hstu ? k_attn_fwd_wide<HD, 1, false, FID>
                      : k_attn_fwd_wide<HD, 0, false, FID>,
               grid, W::NT, lds, s, p);
  } else if (which == 2) {
    const size_t lds = 2 * W::IMG + 2 * RED + W::GX + kWTail + rab + (hstu ? (size_t)p.nb * 8 : 0) + tlds;
    if (lds > kMaxWideLds) return wide_lds_refused(lds);
    launch_lds(tb     ? k_attn_dq_wide<HD, 1, true, FID>
               : hstu ? k_attn_dq_wide<HD, 1, false, FID>
                      : k_attn_dq_wide<HD, 0, false, FID>,
               grid, W::NT, lds, s, p);
  } else {
    const size_t lds = 2 * W::IMG + 2 * RED + 2 * W::GX + kWTail + rab + tlds;
    if (lds > kMaxWideLds) return wide_lds_refused(lds);
    if (p.dout_f32)
      launch_lds(tb     ? k_attn_dkdv_wide<HD, 1, true, true, FID>
                 : hstu ? k_attn_dkdv_wide<HD, 1, true, false, FID>
                        : k_attn_dkdv_wide<HD, 0, true, false, FID>,
                 grid, W::NT, lds, s, p);
    else
      launch_lds(tb     ? k_attn_dkdv_wide<HD, 1, false, true, FID>
                 : hstu ? k_attn_dkdv_wide<HD, 1, false, false, FID>
                        : k_attn_dkdv_wide<HD, 0, false, false, FID>,
                 grid, W::NT, lds, s, p);
  }
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

}  // namespace
}  // namespace grk
