// Forward / input-gradient GEMMs of the dense layers on MFMA (gfx950): the
// nn.Linear products of the HSTU blocks (uvqk / out_linear) and of the item /
// user dnns under bf16 autocast (model/BaseLine/model.py:129-139,302-309;
// model/BaseLineO1/model.py uvqk restatement), with the layer's epilogue fused
// into the store:
//
//   C[m, n] = act( A[m, :] . op(B)[:, n] + bias[n] + beta * C_in[m, n] )
//
//   A [M, K] K-contiguous bf16 (the token rows);
//   B [N, K] K-contiguous (b_layout 0: C = A B^T, the forward x W^T) or
//     [K, N] N-contiguous (b_layout 1: C = A B, the input gradient dY W);
//   act = identity or ReLU; beta in {0, 1}; C bf16 or fp32, fp32 accumulation,
//   one rounding at the store.
//
// Shapes at BASELINE config 2 (jagged capacity M ~ 14k rows): uvqk forward
// N = 2048, K = 512; its input gradient N = 512, K = 2048; out_linear and the
// dnn layers N = 512, K = 512 - 552.
//
// Structure (cdna_hip_programming.md §5):
//  * one workgroup of 8 waves per CU owns a BM x BN output tile; each wave a
//    (BM/WM) x (BN/WN) sub-tile of 32 x 32 MFMA tiles (v_mfma_f32_32x32x16_bf16,
//    accumulators in registers);
//  * 64-deep K steps staged by LDS-DMA (global_load_lds_dwordx4, grk_ring.h
//    wg_dma16) into an NST-stage ring retired by counted vmcnt + raw s_barrier:
//    K-contiguous images are [rows][64 k] with 128-B rows, 16-B chunk c of row r
//    at slot c ^ ((r >> 1) & 7) (conflict-free ds_read_b128 fragment reads over the
//    ds_read_b128 lane groups); the N-contiguous B image is [64 k][BN] read with
//    ds_read_b64_tr_b16 (grk_ring.h ring_frag; A then in ring_frag's k order);
//  * the K tail (K % 64, a multiple of 8) is masked per 16-B chunk in the last
//    step's fragments, so operands may be column blocks of wider buffers;
//  * XCD-aware tile order: consecutive logical tiles (the column tiles of one row
//    block, sharing its A rows) run on one XCD and meet in its L2;
//  * epilogue through LDS: each wave's fp32 tile rows are restaged so a lane owns
//    8 consecutive columns -- bias / C_in reads and the bf16 stores are 16-byte
//    vectors over whole 128-B row segments (from registers they would be 2-byte
//    scattered stores).
#include <type_traits>

#include "grk_common.h"
#include "grk_mfma.h"
#include "grk_ring.h"

namespace grk {
namespace {

// K-contiguous images: rows of BK k (RB = 2 BK bytes), 16-byte chunk c of row r at
// slot c ^ mg_swz<RB>(r) -- conflict-free for the fragment reads (lane l reads row
// l & 31, so each ds_read_b128 lane group, {0-3, 12-15, 20-27}-shaped, covers 16
// rows whose (bank row, slot) pairs the swizzle makes distinct).
template <int RB>
__device__ __forceinline__ int mg_swz(int row) {
  if constexpr (RB == 128) return (row >> 1) & 7;
  else return (row >> 2) & 3;
}

template <int BM, int BN, int WM, int WN, int NST, bool BNC, int BK>
struct MgGeo {
  static constexpr int NW = WM * WN, NT = 64 * NW;
  static constexpr int RBA = 2 * BK;                          // A image row bytes ([BM][BK])
  static constexpr int IMGA = BM * RBA;
  static constexpr int RBB = BNC ? 2 * BN : 2 * BK;           // B image row bytes
  static constexpr int IMGB = BNC ? BK * RBB : BN * RBA;      // [BK][BN] or [BN][BK]
  static constexpr int STAGE = IMGA + IMGB;
  static constexpr int PWA = IMGA / 1024 / NW, PWB = IMGB / 1024 / NW;
  static constexpr int P = PWA + PWB;                         // DMA instructions per wave and stage
  static constexpr int WTM = BM / WM, WTN = BN / WN;          // wave sub-tile
  static constexpr int TI = WTM / 32, TJ = WTN / 32;
  static constexpr int SROW = WTN + 4;                        // epilogue stage row (fp32 elements)
  static_assert(IMGA % (1024 * NW) == 0 && IMGB % (1024 * NW) == 0, "images must split evenly over the waves");
  static_assert(NST >= 2 && NST * STAGE <= 160 * 1024, "ring too large for the LDS");
  static_assert(NW * 32 * SROW * 4 <= NST * STAGE, "epilogue stage must fit in the ring");
  static_assert(WTN % 32 == 0 && WTM % 32 == 0 && (WTN / 8) <= 64, "wave tile");
  static_assert(BK == 32 || BK == 64, "BK: 32 or 64");
};

// Natural k order (B K-contiguous): element j of lane (r, h) = img[row][k0 + 8h + j].
template <int RB>
__device__ __forceinline__ uint4 mg_chunk(const char* img, int row, int c) {
  return *reinterpret_cast<const uint4*>(img + row * RB + 16 * (c ^ mg_swz<RB>(row)));
}

// ring_frag's k order (beside an N-contiguous B): element j of lane (r, h) =
// img[row][k0 + 8(j >> 2) + 4h + (j & 3)]: two 8-byte halves of chunks c0, c0 + 1.
template <int RB>
__device__ __forceinline__ uint4 mg_chunk_perm(const char* img, int row, int c0, int h) {
  const uint2 lo = *reinterpret_cast<const uint2*>(img + row * RB + 16 * (c0 ^ mg_swz<RB>(row)) + 8 * h);
  const uint2 hi = *reinterpret_cast<const uint2*>(img + row * RB + 16 * ((c0 + 1) ^ mg_swz<RB>(row)) + 8 * h);
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}

template <typename T> struct MgOut;
template <> struct MgOut<bf16_t> {
  static __device__ __forceinline__ void load8(const bf16_t* p, float* v) {
    const uint4 t = *reinterpret_cast<const uint4*>(p);
    const unsigned w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[2 * e] = __uint_as_float(w[e] << 16);
      v[2 * e + 1] = __uint_as_float(w[e] & 0xFFFF0000u);
    }
  }
  static __device__ __forceinline__ void store8(bf16_t* p, const float* v) {
    unsigned w[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) w[e] = (unsigned)f32_to_bf16(v[2 * e]) | ((unsigned)f32_to_bf16(v[2 * e + 1]) << 16);
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
};
template <> struct MgOut<float> {
  static __device__ __forceinline__ void load8(const float* p, float* v) {
    const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  static __device__ __forceinline__ void store8(float* p, const float* v) {
    reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
};

struct MgArgs {
  const bf16_t* a;
  int64_t lda;
  const bf16_t* b;
  int64_t ldb;
  void* c;
  int64_t ldc;
  const void* c_in;     // beta = 1: C_in (same dtype / ldc as C; may alias C), else null
  const void* bias;     // [N] fp32 or bf16, or null
  int bias_f32;
  int relu;
  int M, N, K;
  int tiles_n;          // column tiles
  int total;            // tiles of the launch
};

// Waves per SIMD the register budget is cut for: 2 for 8-wave (and 4-wave, two per
// CU) workgroups, 4 for 16-wave ones; with 4 the fragment reads of the next 16-deep
// k slice are not hoisted over the current slice's MFMAs (sched_barrier), which
// keeps the kernel inside 128 VGPRs (the other waves of the SIMD cover the latency).
template <int WM, int WN> constexpr int mg_waves_per_simd() { return WM * WN >= 16 ? 4 : 2; }

template <int BM, int BN, int WM, int WN, int NST, bool BNC, int BK, typename OT>
__global__ void __launch_bounds__(64 * WM * WN, (mg_waves_per_simd<WM, WN>())) k_mgemm(MgArgs g) {
  using G = MgGeo<BM, BN, WM, WN, NST, BNC, BK>;
  constexpr int RBA = G::RBA, CPR = RBA / 16, RPI = 1024 / RBA;   // chunks per row, rows per DMA instruction
  __shared__ __attribute__((aligned(16))) char smem[NST * G::STAGE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w % WM, wn = w / WM, r = lane & 31, hh = lane >> 5;
  // bijective XCD remap (cdna_hip_programming.md §5): blocks b, b + 8, ... share an XCD
  const unsigned phys = blockIdx.x, total = (unsigned)g.total;
  const unsigned q8 = total / 8, r8 = total % 8, xcd = phys % 8;
  const unsigned logical = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + phys / 8;
  const int tile = (int)logical;
  const int m0 = (tile / g.tiles_n) * BM, n0 = (tile % g.tiles_n) * BN;
  const int M = g.M, N = g.N;
  const int K = g.K;
  const int nsteps = K > 0 ? (K + BK - 1) / BK : 0;
  // DMA sources of this lane (rows clamped into the matrices: their outputs are not stored)
  // (K-contiguous images: row base + this lane's chunk column; a chunk past K -- the
  // last step's tail -- reads the row's last chunk instead, never past the row's end,
  // and is masked in the fragments)
  const bf16_t* pa[G::PWA];
  const bf16_t* pb[G::PWB];
  int acol[G::PWA], bcol[G::PWB];
#pragma unroll
  for (int i = 0; i < G::PWA; ++i) {
    const int q = w * G::PWA + i, row = RPI * q + lane / CPR;     // RPI rows of RBA bytes per instruction
    const int ma = min(m0 + row, M - 1);
    pa[i] = g.a + (int64_t)ma * g.lda;
    acol[i] = 8 * ((lane % CPR) ^ mg_swz<RBA>(row));
  }
#pragma unroll
  for (int i = 0; i < G::PWB; ++i) {
    const int q = w * G::PWB + i;
    if constexpr (BNC) {
      constexpr int CPB = G::RBB / 16;                            // chunks per k row
      const int row = q * (1024 / G::RBB) + lane / CPB;
      const int nb = n0 + 8 * ((lane % CPB) ^ wg_swz(row));
      bcol[i] = row;                                              // the image row (k) of this lane
      pb[i] = g.b + (nb < N ? nb : 0);
    } else {
      const int row = RPI * q + lane / CPR;
      const int nb = min(n0 + row, N - 1);
      pb[i] = g.b + (int64_t)nb * g.ldb;
      bcol[i] = 8 * ((lane % CPR) ^ mg_swz<RBA>(row));
    }
  }
  const unsigned lds0 = (unsigned)__builtin_amdgcn_readfirstlane(
      (int)((unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem));
  const unsigned wu = (unsigned)__builtin_amdgcn_readfirstlane(w);
  auto issue = [&](int step, int buf) {
    const unsigned base = lds0 + buf * G::STAGE;
    const int k0 = step * BK;
#pragma unroll
    for (int i = 0; i < G::PWA; ++i) wg_dma16(pa[i] + min(k0 + acol[i], K - 8), base + (wu * G::PWA + i) * 1024);
#pragma unroll
    for (int i = 0; i < G::PWB; ++i) {
      if constexpr (BNC) {
        const int k = min(k0 + bcol[i], K - 1);                   // rows past K: a real row, times A's zeros
        wg_dma16(pb[i] + (int64_t)k * g.ldb, base + G::IMGA + (wu * G::PWB + i) * 1024);
      } else {
        wg_dma16(pb[i] + min(k0 + bcol[i], K - 8), base + G::IMGA + (wu * G::PWB + i) * 1024);
      }
    }
  };
  f32x16 acc[G::TI][G::TJ];
#pragma unroll
  for (int i = 0; i < G::TI; ++i)
#pragma unroll
    for (int j = 0; j < G::TJ; ++j) acc[i][j] = acc_zero();

  // one BK-deep step; MASK: the K tail (chunks at k >= K read as zeros)
  auto compute = [&](const char* ia, const char* ib, int kvalid, auto mask_tag) {
    constexpr bool MASK = decltype(mask_tag)::value;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 fa[G::TI], fb[G::TJ];
#pragma unroll
      for (int i = 0; i < G::TI; ++i) {
        const int row = wm * G::WTM + 32 * i + r;
        uint4 v;
        if constexpr (BNC) {
          v = mg_chunk_perm<RBA>(ia, row, 2 * ks, hh);
          if (MASK) {
            if (8 * (2 * ks) >= kvalid) v.x = v.y = 0u;
            if (8 * (2 * ks + 1) >= kvalid) v.z = v.w = 0u;
          }
        } else {
          v = mg_chunk<RBA>(ia, row, 2 * ks + hh);
          if (MASK && 8 * (2 * ks + hh) >= kvalid) v = make_uint4(0u, 0u, 0u, 0u);
        }
        fa[i] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int j = 0; j < G::TJ; ++j) {
        if constexpr (BNC) {
          fb[j] = ring_frag<G::RBB>(ib, 16 * ks, wn * G::WTN + 32 * j, lane);
        } else {
          uint4 v = mg_chunk<RBA>(ib, wn * G::WTN + 32 * j + r, 2 * ks + hh);
          if (MASK && 8 * (2 * ks + hh) >= kvalid) v = make_uint4(0u, 0u, 0u, 0u);
          fb[j] = __builtin_bit_cast(bf16x8, v);
        }
      }
#pragma unroll
      for (int i = 0; i < G::TI; ++i)
#pragma unroll
        for (int j = 0; j < G::TJ; ++j) acc[i][j] = mfma(fa[i], fb[j], acc[i][j]);
      if constexpr (mg_waves_per_simd<WM, WN>() >= 4 || G::TI * G::TJ >= 8) __builtin_amdgcn_sched_barrier(0);
    }
  };

  for (int t = 0; t < NST - 1 && t < nsteps; ++t) issue(t, t);
  // full steps in the loop, the K tail (if any) peeled after it: one compute body
  // in the loop keeps the accumulators in fixed registers
  const int nfull = K / BK;
  for (int t = 0; t < nfull; ++t) {
    ring_wait<G::P, NST>(nsteps - 1 - t);
    if (t + NST - 1 < nsteps) issue(t + NST - 1, (t + NST - 1) % NST);
    const char* ia = smem + (t % NST) * G::STAGE;
    compute(ia, ia + G::IMGA, BK, std::false_type{});
  }
  if (nfull < nsteps) {
    ring_wait<G::P, NST>(0);
    const char* ia = smem + (nfull % NST) * G::STAGE;
    compute(ia, ia + G::IMGA, K - nfull * BK, std::true_type{});
  }
  __syncthreads();   // every wave is done reading the ring: its LDS holds the epilogue stages

  // ---- epilogue: per 32-row band i, the wave's [32][WTN] fp32 rows through LDS ----
  float* stg = reinterpret_cast<float*>(smem) + w * 32 * G::SROW;
  constexpr int LPR = G::WTN / 8;          // lanes per row (8 columns each)
  constexpr int RPP = 64 / LPR;            // rows per pass
  const int lrow = lane / LPR, lc = 8 * (lane % LPR);
  const int ncol = n0 + wn * G::WTN + lc;
  const bool nok = ncol < N;               // N % 8 == 0: a lane's 8 columns are all in or all out
  float bias[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bias[e] = 0.f;
  if (g.bias && nok) {
    if (g.bias_f32) MgOut<float>::load8(reinterpret_cast<const float*>(g.bias) + ncol, bias);
    else MgOut<bf16_t>::load8(reinterpret_cast<const bf16_t*>(g.bias) + ncol, bias);
  }
  OT* C = reinterpret_cast<OT*>(g.c);
  const OT* Cin = reinterpret_cast<const OT*>(g.c_in);
#pragma unroll
  for (int i = 0; i < G::TI; ++i) {
#pragma unroll
    for (int j = 0; j < G::TJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) stg[acc_row(e, hh) * G::SROW + 32 * j + r] = acc[i][j][e];
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's stage writes done (LDS is in order per wave)
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int p = 0; p < 32 / RPP; ++p) {
      const int rr = p * RPP + lrow;
      const int64_t m = (int64_t)m0 + wm * G::WTM + 32 * i + rr;
      float v[8];
      const float4 a = *reinterpret_cast<const float4*>(stg + rr * G::SROW + lc);
      const float4 b = *reinterpret_cast<const float4*>(stg + rr * G::SROW + lc + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
      if (m < M && nok) {
        float cin[8];
        if (Cin) MgOut<OT>::load8(Cin + m * g.ldc + ncol, cin);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float x = v[e] + bias[e];
          if (Cin) x += cin[e];
          v[e] = g.relu ? fmaxf(x, 0.f) : x;
        }
        MgOut<OT>::store8(C + m * g.ldc + ncol, v);
      }
    }
    __builtin_amdgcn_wave_barrier();   // reads of this band done before the next band's writes
  }
}

// Tile configuration: 256 x 128 tiles of 8 waves (each wave 64 x 64 = 2 x 2 MFMA
// tiles), 64-deep K steps in a 3-stage ring -- the fastest of the round-5 sweep
// (256 x 128 / 256 x 256 / 128 x 128 tiles, 32-deep steps in 4-6 stages) on every
// step shape.
template <bool BNC, typename OT>
hipError_t launch(const MgArgs& a0, hipStream_t s) {
  MgArgs a = a0;
  a.tiles_n = (a.N + 127) / 128;
  a.total = ((a.M + 255) / 256) * a.tiles_n;
  k_mgemm<256, 128, 4, 2, 3, BNC, 64, OT><<<(unsigned)a.total, 512, 0, s>>>(a);
  return hipGetLastError();
}

}  // namespace

}  // namespace grk

using namespace grk;

extern "C" int grk_gemm_mfma_supported(int trans_a, int b_layout, int64_t m, int64_t n, int64_t k, int64_t lda,
                                       int64_t ldb, int64_t ldc, int c_dtype, float alpha, float beta) {
  return trans_a == 0 && (b_layout == 0 || b_layout == 1) && m > 0 && n > 0 && k > 0 && n % 8 == 0 && k % 8 == 0 &&
         lda % 8 == 0 && ldb % 8 == 0 && ldc % 8 == 0 && m < (1 << 30) && n < (1 << 24) && k < (1 << 24) &&
         (c_dtype == GRK_BF16 || c_dtype == GRK_F32) && alpha == 1.0f && (beta == 0.0f || beta == 1.0f);
}

extern "C" int grk_gemm_mfma(int b_layout, int64_t m, int64_t n, int64_t k, const void* a, int64_t lda, const void* b,
                             int64_t ldb, void* c, int64_t ldc, int c_dtype, const void* c_in, const void* bias,
                             int bias_dtype, int epilogue, void* stream) {
  clear_error();
  GRK_CHECK_ARG(grk_gemm_mfma_supported(0, b_layout, m, n, k, lda, ldb, ldc, c_dtype, 1.0f, c_in ? 1.0f : 0.0f),
                "grk_gemm_mfma: unsupported shape (m=%lld n=%lld k=%lld lda=%lld ldb=%lld ldc=%lld)", (long long)m,
                (long long)n, (long long)k, (long long)lda, (long long)ldb, (long long)ldc);
  GRK_CHECK_ARG(a && b && c, "a, b and c are required");
  GRK_CHECK_ARG(lda >= k && ldb >= (b_layout ? n : k) && ldc >= n, "leading dimension too small");
  GRK_CHECK_ARG(((uintptr_t)a | (uintptr_t)b | (uintptr_t)c | (uintptr_t)c_in) % 16 == 0,
                "a / b / c / c_in must be 16-byte aligned");
  GRK_CHECK_ARG(!bias || ((uintptr_t)bias % 16 == 0 && (bias_dtype == GRK_F32 || bias_dtype == GRK_BF16)),
                "bias: 16-byte aligned fp32 or bf16");
  GRK_CHECK_ARG(epilogue == GRK_GEMM_EP_NONE || epilogue == GRK_GEMM_EP_RELU, "bad epilogue %d", epilogue);
  MgArgs g{};
  g.a = (const bf16_t*)a;
  g.lda = lda;
  g.b = (const bf16_t*)b;
  g.ldb = ldb;
  g.c = c;
  g.ldc = ldc;
  g.c_in = c_in;
  g.bias = bias;
  g.bias_f32 = bias_dtype == GRK_F32;
  g.relu = epilogue == GRK_GEMM_EP_RELU;
  g.M = (int)m;
  g.N = (int)n;
  g.K = (int)k;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  if (b_layout) e = c_dtype == GRK_BF16 ? launch<true, bf16_t>(g, s) : launch<true, float>(g, s);
  else e = c_dtype == GRK_BF16 ? launch<false, bf16_t>(g, s) : launch<false, float>(g, s);
  GRK_CHECK_HIP(e);
  return GRK_OK;
}
