// Weight gradients of the dense layers on MFMA (gfx950).
//
//   dW[M, N] = dY^T X          db[M] = sum_k dY[k, m]
//   dY [K, M], X [K, N]: bf16 row-major, K = tokens (25,728 - 51,456 at
//   BASELINE config 2), M, N = 512 - 2048 features; dW fp32 (the master
//   weights' dtype) or bf16.
//
// Replaces the weight-gradient GEMM autograd runs for every nn.Linear /
// Conv1d(k=1) of the model under bf16 autocast (model/BaseLine/model.py:65-78,
// 129-139, 302-309; the HSTU uvqk / output projections) and the bias-gradient
// column sum beside it.  hipBLASLt tiles this shape (small output, long
// reduction) with one workgroup per 256-wide output tile: 4 to 16 workgroups
// for 256 CUs, 140-410 TF/s in the bench step.  Here the reduction is split
// into S slices so that a launch has ~512 workgroups:
//  * one 256-thread workgroup = one 128x128 output tile of one K slice; each
//    wave accumulates a 64x64 quarter in registers (2x2 MFMA 32x32x16 tiles);
//  * both operands are K-major in memory: 32-row K steps of dY and X are
//    staged as they lie (coalesced 256-B rows, XOR-swizzled) into a double
//    LDS buffer (the next step's global loads in flight under the MFMAs) and read as MFMA fragments with ds_read_b64_tr_b16 (the same
//    k permutation for both operands, so the product still sums over k);
//  * every slice writes its fp32 partial tile with plain stores and
//    k_wgrad_reduce sums the slices in slice order -- deterministic, no
//    atomics; db comes from the dY tiles the n = 0 workgroups stage anyway.
#include <algorithm>

#include "grk_common.h"
#include "grk_mfma.h"
#include "grk_ring.h"

namespace grk {
namespace {

constexpr int kWgTile = 128;                    // output rows / cols per workgroup
constexpr int kWgImg = kWgK * kWgTile * 2;      // one staged [32][128] bf16 image (8 KiB)

// 256-byte rows; the XOR keeps the 16-B row writes and the transposed
// 32x32x16 fragment reads conflict-free (cdna_hip_programming.md T10, layout (b)).
__device__ __forceinline__ int wg_off(int row, int ch) {
  return row * (kWgTile * 2) + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

// Fragment over the 16 k rows [k0, k0+16) for output index c0 + r:
// element j of lane (r, h) = img[k0 + 8(j>>2) + 4h + (j&3)][c0 + r].
__device__ __forceinline__ bf16x8 wg_frag(const char* img, int k0, int c0, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int col = c0 + 16 * (g & 1) + 4 * (i & 3);
  const int row = k0 + 4 * (g >> 1) + (i >> 2);
  const int sub = 2 * (col & 7);
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + wg_off(row, col >> 3) + sub));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + wg_off(row + 8, col >> 3) + sub));
  const bf16x4 l4 = __builtin_bit_cast(bf16x4, lo), h4 = __builtin_bit_cast(bf16x4, hi);
  bf16x8 f;
  f[0] = l4[0]; f[1] = l4[1]; f[2] = l4[2]; f[3] = l4[3];
  f[4] = h4[0]; f[5] = h4[1]; f[6] = h4[2]; f[7] = h4[3];
  return f;
}

template <bool DB>
__global__ void __launch_bounds__(256) k_wgrad(const bf16_t* __restrict__ A, int64_t lda,
                                               const bf16_t* __restrict__ B, int64_t ldb, int K, int M, int N,
                                               int kchunk, float* __restrict__ part, float* __restrict__ dbpart) {
  __shared__ __attribute__((aligned(16))) char smem[4 * kWgImg];  // [buffer 0 / 1][dY, X]: 32 KiB
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w & 1, wn = w >> 1, r = lane & 31, hh = lane >> 5;
  // XCD-aware tile order: workgroups are dealt round-robin to the 8 XCDs
  // (physical id % 8), so logical tile ids are laid out XCD-major -- the n-tiles
  // sharing one dY block and the m-tiles sharing one X block of a K-slice run
  // on the same XCD and read them through its L2 once (PMC: 546 -> see DESIGN).
  const unsigned nx = gridDim.x, my = gridDim.y;
  const unsigned total = nx * my * gridDim.z;
  const unsigned phys = blockIdx.x + nx * (blockIdx.y + my * blockIdx.z);
  const unsigned logical = total % 8 == 0 ? (phys % 8) * (total / 8) + phys / 8 : phys;
  const int bx = (int)(logical % nx), by = (int)((logical / nx) % my), s = (int)(logical / (nx * my));
  const int n0 = bx * kWgTile, m0 = by * kWgTile;
  const int kb = s * kchunk, ke = min(K, kb + kchunk);
  const int nsteps = ke > kb ? (ke - kb + kWgK - 1) / kWgK : 0;
  const bool do_db = DB && bx == 0;
  const int ch = tid & 15, row0 = tid >> 4;  // this thread's 16-B column chunk and first staged row
  const bool mok = m0 + 8 * ch < M, nok = n0 + 8 * ch < N;
  const bf16_t* pa = A + m0 + 8 * ch;
  const bf16_t* pb = B + n0 + 8 * ch;
  constexpr int NC = kWgK / 16;  // staged rows per thread per step
  uint4 ra[NC], rb[NC];
  float cs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) cs[e] = 0.f;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  auto load = [&](int step, uint4* xa, uint4* xb) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int k = kb + step * kWgK + row0 + 16 * c;
      const bool ok = k < ke;
      xa[c] = ok && mok ? *reinterpret_cast<const uint4*>(pa + (int64_t)k * lda) : make_uint4(0, 0, 0, 0);
      xb[c] = ok && nok ? *reinterpret_cast<const uint4*>(pb + (int64_t)k * ldb) : make_uint4(0, 0, 0, 0);
    }
  };
  auto stage = [&](int buf, const uint4* xa, const uint4* xb) {
    char* ia = smem + buf * 2 * kWgImg;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      *reinterpret_cast<uint4*>(ia + wg_off(row0 + 16 * c, ch)) = xa[c];
      *reinterpret_cast<uint4*>(ia + kWgImg + wg_off(row0 + 16 * c, ch)) = xb[c];
      if (do_db) {
        const unsigned u[4] = {xa[c].x, xa[c].y, xa[c].z, xa[c].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          cs[2 * e] += __uint_as_float(u[e] << 16);
          cs[2 * e + 1] += __uint_as_float(u[e] & 0xFFFF0000u);
        }
      }
    }
  };

  if (nsteps > 0) {
    load(0, ra, rb);
    stage(0, ra, rb);
  }
  __syncthreads();
  for (int step = 0; step < nsteps; ++step) {
    const int cur = step & 1;
    if (step + 1 < nsteps) load(step + 1, ra, rb);
    const char* ia = smem + cur * 2 * kWgImg;
    const char* ib = ia + kWgImg;
#pragma unroll
    for (int ks = 0; ks < kWgK / 16; ++ks) {
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = wg_frag(ia, 16 * ks, 64 * wm + 32 * i, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = wg_frag(ib, 16 * ks, 64 * wn + 32 * j, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma(fa[i], fb[j], acc[i][j]);
    }
    if (step + 1 < nsteps) stage(cur ^ 1, ra, rb);
    __syncthreads();
  }

  // partial tile of slice s: lane (r, hh) holds rows m = ... + acc_row(e, hh), column n = ... + r
  float* out = part + (int64_t)s * M * N;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + 64 * wn + 32 * j + r;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + 64 * wm + 32 * i + acc_row(e, hh);
        if (m < M && n < N) out[(int64_t)m * N + n] = acc[i][j][e];
      }
    }
  if (do_db) {  // the 16 threads of one column chunk hold staged rows row0 = 0..15: summed in row order
    float* red = reinterpret_cast<float*>(smem);  // [16][128], free after the loop's last barrier
#pragma unroll
    for (int e = 0; e < 8; ++e) red[row0 * kWgTile + 8 * ch + e] = cs[e];
    __syncthreads();
    if (tid < kWgTile && m0 + tid < M) {
      float t = 0.f;
      for (int q = 0; q < 16; ++q) t += red[q * kWgTile + tid];
      dbpart[(int64_t)s * M + m0 + tid] = t;
    }
  }
}

// ---------------------------------------------------------------------------
// The same tile and K split with the operands staged by LDS-DMA
// (global_load_lds_dwordx4) in a 4-deep ring: the 32-row steps t+1..t+3 are in
// flight while step t is multiplied.  Measured on the register-staged kernel
// above (round 3): each step waited ~1.5k cycles for its loads behind 256
// cycles of MFMA per wave (one step of prefetch), ~10x the MFMA time per
// launch.  Here nothing is staged through VGPRs:
//   * a wave-instruction writes 1 KiB = 4 rows of the [32][128] image at
//     wave-uniform base + lane * 16, so the XOR swizzle of wg_off is applied
//     to the SOURCE: lane l of row group g loads global chunk (l & 15) ^ f(row)
//     into LDS slot l & 15 (wg_frag reads slot ch ^ f(row) for chunk ch);
//   * per step each wave issues 2 + 2 instructions (dY, X); step t is retired
//     by `s_waitcnt vmcnt(8)` (steps t+1, t+2 stay in flight) and a raw
//     s_barrier (a __syncthreads() would drain every DMA: vmcnt(0));
//   * the slot refilled with step t+3 is the one step t-1 read: every wave
//     has passed this step's barrier, so its reads of it are done;
//   * db from the dY fragments the wn = 0 waves hold anyway: each lane sums
//     its 8 k values per fragment (column m = c0 + (lane & 31)), the two
//     k halves (lanes l, l + 32) are added once at the end.
//   * columns past M / N read a valid column instead (their outputs are
//     never stored); K must be a multiple of 32 (no partial steps: the
//     slices are whole steps) -- else the register-staged kernel runs.
// SUB: 32-row k steps per ring stage (one barrier per SUB steps; the slice length
// is then a multiple of 32 SUB rows).
template <bool DB, int WM, int WN, int NST, int SUB = 1>
__global__ void __launch_bounds__(64 * WM * WN) k_wgrad_lds(const bf16_t* __restrict__ A, int64_t lda,
                                                            const bf16_t* __restrict__ B, int64_t ldb, int K, int M,
                                                            int N, int kchunk, float* __restrict__ part,
                                                            float* __restrict__ dbpart) {
  using G = WgRing<WM, WN, NST>;
  __shared__ __attribute__((aligned(16))) char smem[NST * SUB * G::STAGE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w % WM, wn = w / WM, r = lane & 31, hh = lane >> 5;
  const unsigned nx = gridDim.x, my = gridDim.y;
  const unsigned total = nx * my * gridDim.z;
  const unsigned phys = blockIdx.x + nx * (blockIdx.y + my * blockIdx.z);
  const unsigned logical = total % 8 == 0 ? (phys % 8) * (total / 8) + phys / 8 : phys;
  const int bx = (int)(logical % nx), by = (int)((logical / nx) % my), s = (int)(logical / (nx * my));
  const int n0 = bx * G::TN, m0 = by * G::TM;
  const int kb = s * kchunk, ke = min(K, kb + kchunk);
  const int nsteps = ke > kb ? (ke - kb) / (kWgK * SUB) : 0;   // ring stages of SUB steps
  const bool do_db = DB && bx == 0 && wn == 0;
  // this lane's source rows: DMA instruction q of an image covers rows [q * 1024 / RB, ...)
  const bf16_t* pa[G::PWA];
  const bf16_t* pb[G::PWB];
#pragma unroll
  for (int i = 0; i < G::PWA; ++i) {
    constexpr int CPR = G::RBA / 16;   // 16-byte chunks per row
    const int q = w * G::PWA + i, row = q * (1024 / G::RBA) + lane / CPR;
    const int ma = m0 + 8 * ((lane % CPR) ^ wg_swz(row));
    pa[i] = A + (int64_t)(kb + row) * lda + (ma < M ? ma : 0);
  }
#pragma unroll
  for (int i = 0; i < G::PWB; ++i) {
    constexpr int CPR = G::RBB / 16;
    const int q = w * G::PWB + i, row = q * (1024 / G::RBB) + lane / CPR;
    const int nb = n0 + 8 * ((lane % CPR) ^ wg_swz(row));
    pb[i] = B + (int64_t)(kb + row) * ldb + (nb < N ? nb : 0);
  }
  // wave-uniform LDS byte address of stage 0
  const unsigned lds0 = (unsigned)__builtin_amdgcn_readfirstlane(
      (int)((unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem));
  const unsigned wu = (unsigned)__builtin_amdgcn_readfirstlane(w);   // wave-uniform: the DMA base is an SGPR
  auto issue = [&](int step, int buf) {
#pragma unroll
    for (int u = 0; u < SUB; ++u) {
      const unsigned base = lds0 + (buf * SUB + u) * G::STAGE;
      const int64_t ka = (int64_t)(step * SUB + u) * kWgK * lda, kbb = (int64_t)(step * SUB + u) * kWgK * ldb;
#pragma unroll
      for (int i = 0; i < G::PWA; ++i) wg_dma16(pa[i] + ka, base + (wu * G::PWA + i) * 1024);
#pragma unroll
      for (int i = 0; i < G::PWB; ++i) wg_dma16(pb[i] + kbb, base + G::IMGA + (wu * G::PWB + i) * 1024);
    }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
  float cs[2] = {0.f, 0.f};
  // ring_frag's addresses, hoisted: per lane the byte offsets (within a stage) of the
  // lo / hi halves of fragments i (A) and j (B) at k rows 0..15; rows 16..31 have the
  // same swizzle, so k step 1 is an immediate offset (16 RB) on the same registers.
  // Every fragment read of a step is issued before its MFMAs, so the second half's
  // reads run under the first half's MFMAs (SQ: 34 % of wave cycles waited on
  // instruction dependencies with a read -> wait -> MFMA sequence per k step, and
  // ~15 VALU address ops per k step).
  unsigned oa[2][2], ob[2][2];
  {
    const int g = lane >> 4, ii = lane & 15;
    const int row = 4 * (g >> 1) + (ii >> 2);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ca = 64 * wm + 32 * i + 16 * (g & 1) + 4 * (ii & 3);
      const int cb = 64 * wn + 32 * i + 16 * (g & 1) + 4 * (ii & 3);
      oa[i][0] = row * G::RBA + 16 * ((ca >> 3) ^ wg_swz(row)) + 2 * (ca & 7);
      oa[i][1] = (row + 8) * G::RBA + 16 * ((ca >> 3) ^ wg_swz(row + 8)) + 2 * (ca & 7);
      ob[i][0] = G::IMGA + row * G::RBB + 16 * ((cb >> 3) ^ wg_swz(row)) + 2 * (cb & 7);
      ob[i][1] = G::IMGA + (row + 8) * G::RBB + 16 * ((cb >> 3) ^ wg_swz(row + 8)) + 2 * (cb & 7);
    }
  }
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  typedef __attribute__((address_space(3))) char lds_char;
  auto frag = [&](const lds_char* st, unsigned lo, unsigned hi, int koff) {
    const s16x4 l = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(st + lo + koff));
    const s16x4 h = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(st + hi + koff));
    const bf16x4 l4 = __builtin_bit_cast(bf16x4, l), h4 = __builtin_bit_cast(bf16x4, h);
    bf16x8 f;
    f[0] = l4[0]; f[1] = l4[1]; f[2] = l4[2]; f[3] = l4[3];
    f[4] = h4[0]; f[5] = h4[1]; f[6] = h4[2]; f[7] = h4[3];
    return f;
  };

  for (int t = 0; t < NST - 1 && t < nsteps; ++t) issue(t, t);
  for (int t = 0; t < nsteps; ++t) {
    ring_wait<G::P * SUB, NST>(nsteps - 1 - t);
    if (t + NST - 1 < nsteps) issue(t + NST - 1, (t + NST - 1) % NST);
#pragma unroll
    for (int u = 0; u < SUB; ++u) {
    const lds_char* st = (const lds_char*)smem + ((t % NST) * SUB + u) * G::STAGE;
    bf16x8 fa[2][2], fb[2][2];   // [k step][i / j]
#pragma unroll
    for (int ks = 0; ks < kWgK / 16; ++ks) {
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[ks][i] = frag(st, oa[i][0], oa[i][1], ks * 16 * G::RBA);
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[ks][j] = frag(st, ob[j][0], ob[j][1], ks * 16 * G::RBB);
    }
#pragma unroll
    for (int ks = 0; ks < kWgK / 16; ++ks) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma(fa[ks][i], fb[ks][j], acc[i][j]);
      if (do_db) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          float q = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) q += static_cast<float>(fa[ks][i][e]);
          cs[i] += q;
        }
      }
    }
    }
  }
  float* out = part + (int64_t)s * M * N;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + 64 * wn + 32 * j + r;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + 64 * wm + 32 * i + acc_row(e, hh);
        if (m < M && n < N) out[(int64_t)m * N + n] = acc[i][j][e];
      }
    }
  if (do_db) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float other = __shfl_xor(cs[i], 32);   // the other k half of column r
      const int m = m0 + 64 * wm + 32 * i + r;
      if (hh == 0 && m < M) dbpart[(int64_t)s * M + m] = cs[i] + other;
    }
  }
}

__device__ __forceinline__ void wg_store4(float* p, const float4& v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ void wg_store4(bf16_t* p, const float4& v) {
  uint2 t;
  t.x = (unsigned)f32_to_bf16(v.x) | ((unsigned)f32_to_bf16(v.y) << 16);
  t.y = (unsigned)f32_to_bf16(v.z) | ((unsigned)f32_to_bf16(v.w) << 16);
  *reinterpret_cast<uint2*>(p) = t;
}

// out[m][n] = sum over slices s = 0, 1, ... of part[s][m][n]; db[m] likewise.
template <typename OT>
__global__ void __launch_bounds__(256) k_wgrad_reduce(const float* __restrict__ part, int S, int M, int N,
                                                      OT* __restrict__ out, int64_t ldo,
                                                      const float* __restrict__ dbpart, float* __restrict__ db) {
  const int64_t n4 = N / 4, total = (int64_t)M * n4, mn = (int64_t)M * N;
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < total; u += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = u / n4;
    const int64_t n = (u - m * n4) * 4;
    const float* p = part + m * N + n;
    // up to eight slices' loads in flight at once (the whole reduction at S <= 8:
    // one memory latency per output chunk), added in slice order
    const int c = S < 8 ? S : 8;
    float4 v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (q < c) v[q] = *reinterpret_cast<const float4*>(p + q * mn);
    float4 a = v[0];
#pragma unroll
    for (int q = 1; q < 8; ++q)
      if (q < c) {
        a.x += v[q].x;
        a.y += v[q].y;
        a.z += v[q].z;
        a.w += v[q].w;
      }
    int s = c;
    for (; s + 8 <= S; s += 8) {
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = *reinterpret_cast<const float4*>(p + (s + q) * mn);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        a.x += v[q].x;
        a.y += v[q].y;
        a.z += v[q].z;
        a.w += v[q].w;
      }
    }
    for (; s < S; ++s) {
      const float4 w = *reinterpret_cast<const float4*>(p + s * mn);
      a.x += w.x;
      a.y += w.y;
      a.z += w.z;
      a.w += w.w;
    }
    wg_store4(out + m * ldo + n, a);
  }
  // db: spread over the grid (one column per thread), slices' loads in flight
  // together, summed in slice order (a single workgroup walking all M columns
  // with one dependent load per slice was the reduce kernel's critical path)
  if (db)
    for (int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; m < M; m += (int64_t)gridDim.x * blockDim.x) {
      const int c = S < 8 ? S : 8;
      float v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (q < c) v[q] = dbpart[(int64_t)q * M + m];
      float t = v[0];
#pragma unroll
      for (int q = 1; q < 8; ++q)
        if (q < c) t += v[q];
      for (int s = c; s < S; ++s) t += dbpart[(int64_t)s * M + m];
      db[m] = t;
    }
}

// K slices: about two workgroups per CU (latency hiding), slices of >= kSliceRows rows.
// Measured (round 5): 256- and 128-row slices slower than 512.
constexpr int kSliceRows = 512;
#ifndef GRK_WGRAD_SUB2
#define GRK_WGRAD_SUB2 1   // A/B builds: 0 = one barrier per 32-row step in the 256 x 128 ring
#endif
constexpr bool kWgSub2 = GRK_WGRAD_SUB2;
int wgrad_splits(int64_t K, int64_t M, int64_t N) {
  const int64_t tiles = ((M + kWgTile - 1) / kWgTile) * ((N + kWgTile - 1) / kWgTile);
  int S = 1;
  while (S < 64 && tiles * S < 512 && K >= (int64_t)S * 2 * kSliceRows) S *= 2;
  return S;
}

// Kernel plan of a shape: which ring (kind 0: the register-staged kernel, K not a
// multiple of 32; 1: 128 x 128 tiles, two workgroups per CU; 2: 256 x 128 tiles, one
// 8-wave workgroup per CU, for M >= 1024 -- the uvqk weight gradients), the tile and
// the K split.  grk_mgemm's K-major split-K mode was measured slower (round 5) and removed.
struct WgPlan {
  int kind, tm, tn, S;
};
WgPlan wgrad_plan(int64_t K, int64_t M, int64_t N) {
  WgPlan p{0, kWgTile, kWgTile, wgrad_splits(K, M, N)};
  if (K % kWgK) return p;
  if (M < 1024) {
    p.kind = 1;
    return p;
  }
  p = WgPlan{2, 256, 128, 1};
  const int64_t tiles = ((M + 255) / 256) * ((N + 127) / 128);
  while (p.S < 64 && tiles * p.S < 256 && K >= (int64_t)p.S * 2 * kSliceRows) p.S *= 2;   // one workgroup per CU
  return p;
}

}  // namespace

}  // namespace grk

using namespace grk;

extern "C" size_t grk_wgrad_workspace(int64_t k, int64_t m, int64_t n) {
  if (k < 0 || m <= 0 || n <= 0) return 0;
  const int S = wgrad_plan(k, m, n).S;
  return ((size_t)S * m * n + (size_t)S * m) * sizeof(float);
}

extern "C" int grk_wgrad(const void* dy, int64_t ld_dy, const void* x, int64_t ld_x, int64_t k, int64_t m, int64_t n,
                         void* dw, int64_t ld_dw, int dw_dtype, float* db, void* workspace, size_t workspace_bytes,
                         void* stream) {
  clear_error();
  GRK_CHECK_ARG(k >= 0 && m > 0 && n > 0, "sizes must be k >= 0, m > 0, n > 0");
  GRK_CHECK_ARG(m % 8 == 0 && n % 8 == 0, "m and n must be multiples of 8");
  GRK_CHECK_ARG(k < ((int64_t)1 << 31) && m < (1 << 24) && n < (1 << 24), "GEMM too large");
  GRK_CHECK_ARG(k == 0 || (dy && x), "dy and x are required");
  GRK_CHECK_ARG(dw && workspace, "dw and workspace are required");
  GRK_CHECK_ARG(ld_dy >= m && ld_x >= n && ld_dy % 8 == 0 && ld_x % 8 == 0,
                "row strides must cover the rows and be multiples of 8");
  GRK_CHECK_ARG((uintptr_t)dy % 16 == 0 && (uintptr_t)x % 16 == 0, "dy / x must be 16-byte aligned");
  GRK_CHECK_ARG(dw_dtype == GRK_F32 || dw_dtype == GRK_BF16, "dw must be fp32 or bf16");
  GRK_CHECK_ARG(ld_dw >= n && ld_dw % 4 == 0, "ld_dw must be >= n and a multiple of 4");
  GRK_CHECK_ARG(workspace_bytes >= grk_wgrad_workspace(k, m, n), "workspace smaller than grk_wgrad_workspace()");
  const WgPlan pl = wgrad_plan(k, m, n);
  const int S = pl.S;
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)workspace;
  float* dbp = part + (size_t)S * m * n;
  // slices of whole ring stages (64 rows for the two-step 256 x 128 ring)
  const int kq = (pl.kind == 2 && kWgSub2 && k % 64 == 0) ? 64 : kWgK;
  const int kchunk = (int)(((k + S - 1) / S + kq - 1) / kq * kq);
  const dim3 grid((unsigned)((n + pl.tn - 1) / pl.tn), (unsigned)((m + pl.tm - 1) / pl.tm), (unsigned)S);
  const bf16_t *A = (const bf16_t*)dy, *Bx = (const bf16_t*)x;
#define GRK_WG(KERN, THREADS)                                                                               \
  do {                                                                                                     \
    if (db) KERN<true><<<grid, THREADS, 0, s>>>(A, ld_dy, Bx, ld_x, (int)k, (int)m, (int)n, kchunk, part, dbp); \
    else KERN<false><<<grid, THREADS, 0, s>>>(A, ld_dy, Bx, ld_x, (int)k, (int)m, (int)n, kchunk, part, nullptr); \
  } while (0)
  if (pl.kind == 2 && kWgSub2 && k % 64 == 0 && kchunk % 64 == 0) {
    if (db) k_wgrad_lds<true, 4, 2, 3, 2><<<grid, 512, 0, s>>>(A, ld_dy, Bx, ld_x, (int)k, (int)m, (int)n, kchunk, part,
                                                              dbp);
    else k_wgrad_lds<false, 4, 2, 3, 2><<<grid, 512, 0, s>>>(A, ld_dy, Bx, ld_x, (int)k, (int)m, (int)n, kchunk,
                                                             part, nullptr);
  } else if (pl.kind == 2) {
    if (db) k_wgrad_lds<true, 4, 2, 6><<<grid, 512, 0, s>>>(A, ld_dy, Bx, ld_x, (int)k, (int)m, (int)n, kchunk, part, dbp);
    else k_wgrad_lds<false, 4, 2, 6><<<grid, 512, 0, s>>>(A, ld_dy, Bx, ld_x, (int)k, (int)m, (int)n, kchunk, part,
                                                          nullptr);
  } else if (pl.kind == 1) {
    if (db) k_wgrad_lds<true, 2, 2, 4><<<grid, 256, 0, s>>>(A, ld_dy, Bx, ld_x, (int)k, (int)m, (int)n, kchunk, part, dbp);
    else k_wgrad_lds<false, 2, 2, 4><<<grid, 256, 0, s>>>(A, ld_dy, Bx, ld_x, (int)k, (int)m, (int)n, kchunk, part,
                                                          nullptr);
  } else {
    GRK_WG(k_wgrad, 256);
  }
#undef GRK_WG
  GRK_LAUNCH_CHECK();
  const int64_t work = m * n / 4;
  const unsigned g = (unsigned)std::min<int64_t>((work + 255) / 256, 4096);
  if (dw_dtype == GRK_F32)
    k_wgrad_reduce<float><<<g, 256, 0, s>>>(part, S, (int)m, (int)n, (float*)dw, ld_dw, db ? dbp : nullptr, db);
  else
    k_wgrad_reduce<bf16_t><<<g, 256, 0, s>>>(part, S, (int)m, (int)n, (bf16_t*)dw, ld_dw, db ? dbp : nullptr, db);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}
