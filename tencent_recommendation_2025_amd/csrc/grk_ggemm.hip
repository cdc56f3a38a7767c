// Grouped GEMMs of the projected feature tables (gfx950 MFMA, LDS-DMA ring).
//
// The fused model looks its item / user feature tables up through projections
// P_f = E_f W_f^T (model._projection: the reference's per-feature embedding
// lookups feeding itemdnn / userdnn, model/BaseLine/model.py:254-310, restated
// so that the dnn GEMM runs over table rows instead of tokens).  Per table f:
//   forward   P_f  [rows_f, d_out] = E_f [rows_f, d_in] . W_f^T     (W_f = W[:, cols_f])
//   backward  dE_f [rows_f, d_in]  = dP_f [rows_f, d_out] . W_f
//             dW_f [d_out, d_in]   = dP_f^T . E_f                   (into W's gradient, columns cols_f)
// 22 tables of 11 - 10,001 rows at BASELINE config 2: torch.bmm over the
// equal-row-count stacks took ~280 us a step in 15 launches (plus the stacking
// copies); here each of the three is ONE launch over all tables (the weight
// gradient plus one reduction of its split-K slices).
//
// grk_grouped_gemm: C_g = A_g . op(B_g), A_g [rows_g, K] K-contiguous, B_g either
// [N, K] K-contiguous (b_layout 0: C = A B^T) or [K, N] N-contiguous (b_layout 1:
// C = A B).  128 x 128 tiles, 4 waves of 64 x 64 (2 x 2 MFMA 32x32x16), 32-row K
// steps staged by LDS-DMA in a 4-stage ring (grk_ring.h), K = 512 at C2.
//   * K-contiguous images hold [128 rows][32 k] (64-byte rows; chunk c of row r at
//     slot c ^ ((r >> 1) & 3), conflict-free 16-B reads), read as MFMA fragments
//     with ds_read_b128 -- or, beside an N-contiguous B (read with
//     ds_read_b64_tr_b16, whose k order is permuted: grk_ring.h ring_frag), with
//     two ds_read_b64 in the same permuted k order, so the product still sums
//     every k once;
//   * rows past a group's end read its last row (their outputs are not stored).
// grk_grouped_wgrad: C_g [M, N] = A_g^T B_g over K_g rows (both K-major, the
// k_wgrad_lds layout), fp32; K_g a multiple of 32 (the projected tables' P rows are
// padded to 32 with zero gradient rows), B rows past b_rows read its last row
// (multiplied by A's zero rows there: exact zeros).  Groups of more than
// kGwSliceRows rows are split over K; their slices are summed in slice order by
// k_gwgrad_reduce (deterministic), the others store C directly.
#include <algorithm>

#include "grk_common.h"
#include "grk_mfma.h"
#include "grk_ring.h"

namespace grk {
namespace {

constexpr int kGgMax = 32;              // groups per launch
constexpr int kGgTile = 128;
constexpr int kGgNst = 4;
constexpr int kGgImg = kWgK * kGgTile * 2;   // one staged image: 8 KiB
constexpr int kGgStage = 2 * kGgImg;
constexpr int kGwSliceRows = 1024;      // wgrad: K rows per slice (about)

struct GgGroup {
  const bf16_t* a;
  int64_t lda;
  const bf16_t* b;
  int64_t ldb;
  void* c;
  int64_t ldc;
  int64_t rows;     // gemm: rows of A / C; wgrad: K rows
  int64_t b_rows;   // wgrad: rows of B that exist
  int tile0;        // first tile of the group in the launch
  int slices;       // wgrad: K slices
  int kchunk;       // wgrad: K rows per slice (multiple of 32)
  int part0;        // wgrad: first partial buffer of the group (-1: stores C directly)
};
struct GgArgs {
  GgGroup g[kGgMax];
  int n;
  int total;        // tiles of the launch
};

// K-contiguous images: 64-byte rows of 32 k, 16-byte chunk c of row r at slot c ^ kc_swz(r)
__device__ __forceinline__ int kc_swz(int row) { return (row >> 1) & 3; }

// natural k order: element j of lane (r, h) = img[row][k0 + 8h + j]
__device__ __forceinline__ bf16x8 kc_frag(const char* img, int row, int k0, int h) {
  const int c = (k0 >> 3) + h;
  return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(img + row * 64 + 16 * (c ^ kc_swz(row))));
}

// ring_frag's k order: element j of lane (r, h) = img[row][k0 + 8(j >> 2) + 4h + (j & 3)]
__device__ __forceinline__ bf16x8 kc_frag_perm(const char* img, int row, int k0, int h) {
  const int c0 = k0 >> 3;
  const uint2 lo = *reinterpret_cast<const uint2*>(img + row * 64 + 16 * (c0 ^ kc_swz(row)) + 8 * h);
  const uint2 hi = *reinterpret_cast<const uint2*>(img + row * 64 + 16 * ((c0 + 1) ^ kc_swz(row)) + 8 * h);
  return __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
}

// The launch's tile t -> (group, tile within the group); tiles are dealt XCD-major
// (workgroup i runs on XCD i % 8): consecutive logical tiles -- the column tiles of
// one row block, sharing its A rows -- run on one XCD and meet in its L2.
__device__ __forceinline__ int gg_tile(const GgArgs& ga, int& grp) {
  const unsigned phys = blockIdx.x, total = (unsigned)ga.total;
  const unsigned t = total % 8 == 0 ? (phys % 8) * (total / 8) + phys / 8 : phys;
  int g = 0;
  while (g + 1 < ga.n && (int)t >= ga.g[g + 1].tile0) ++g;
  grp = g;
  return (int)t - ga.g[g].tile0;
}

__device__ __forceinline__ void gg_store(float* p, float v) { *p = v; }
__device__ __forceinline__ void gg_store(bf16_t* p, float v) { *p = f32_to_bf16(v); }

template <bool BNC, typename OT>
__global__ void __launch_bounds__(256) k_ggemm(GgArgs ga, int N, int K) {
  __shared__ __attribute__((aligned(16))) char smem[kGgNst * kGgStage];
  int gi;
  const int local = gg_tile(ga, gi);
  const GgGroup& G = ga.g[gi];
  const int ntn = (N + kGgTile - 1) / kGgTile;
  const int m0 = (local / ntn) * kGgTile, n0 = (local % ntn) * kGgTile;
  const int64_t M = G.rows;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w & 1, wn = w >> 1, r = lane & 31, hh = lane >> 5;
  // DMA sources: each wave issues 2 instructions per image and step (1 KiB each)
  const bf16_t* pa[2];
  const bf16_t* pb[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = 2 * w + i;
    const int row = 16 * q + (lane >> 2);                       // K-contiguous: 16 rows of 64 B
    const int64_t ma = min<int64_t>(m0 + row, M - 1);
    pa[i] = G.a + ma * G.lda + 8 * ((lane & 3) ^ kc_swz(row));
    if constexpr (BNC) {
      const int krow = 4 * q + (lane >> 4);                     // K rows: 4 rows of 256 B
      const int nb = n0 + 8 * ((lane & 15) ^ wg_swz(krow));
      pb[i] = G.b + (int64_t)krow * G.ldb + (nb < N ? nb : 0);
    } else {
      const int64_t nbr = min(n0 + row, N - 1);
      pb[i] = G.b + nbr * G.ldb + 8 * ((lane & 3) ^ kc_swz(row));
    }
  }
  const unsigned lds0 = (unsigned)__builtin_amdgcn_readfirstlane(
      (int)((unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem));
  const unsigned wu = (unsigned)__builtin_amdgcn_readfirstlane(w);
  auto issue = [&](int step, int buf) {
    const unsigned base = lds0 + buf * kGgStage;
    const int64_t kb = (int64_t)step * kWgK * (BNC ? G.ldb : 1);
#pragma unroll
    for (int i = 0; i < 2; ++i) wg_dma16(pa[i] + step * kWgK, base + (wu * 2 + i) * 1024);
#pragma unroll
    for (int i = 0; i < 2; ++i) wg_dma16(pb[i] + kb, base + kGgImg + (wu * 2 + i) * 1024);
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
  const int nsteps = K / kWgK;
  for (int t = 0; t < kGgNst - 1 && t < nsteps; ++t) issue(t, t);
  for (int t = 0; t < nsteps; ++t) {
    ring_wait<4, kGgNst>(nsteps - 1 - t);
    if (t + kGgNst - 1 < nsteps) issue(t + kGgNst - 1, (t + kGgNst - 1) % kGgNst);
    const char* ia = smem + (t % kGgNst) * kGgStage;
    const char* ib = ia + kGgImg;
#pragma unroll
    for (int ks = 0; ks < kWgK / 16; ++ks) {
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = 64 * wm + 32 * i + r;
        fa[i] = BNC ? kc_frag_perm(ia, row, 16 * ks, hh) : kc_frag(ia, row, 16 * ks, hh);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
        fb[j] = BNC ? ring_frag<2 * kGgTile>(ib, 16 * ks, 64 * wn + 32 * j, lane)
                    : kc_frag(ib, 64 * wn + 32 * j + r, 16 * ks, hh);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma(fa[i], fb[j], acc[i][j]);
    }
  }
  OT* C = reinterpret_cast<OT*>(G.c);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + 64 * wn + 32 * j + r;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t m = m0 + 64 * wm + 32 * i + acc_row(e, hh);
        if (m < M && n < N) gg_store(C + m * G.ldc + n, acc[i][j][e]);
      }
    }
}

// Grouped weight gradient: the k_wgrad_lds<false, 2, 2, 4> tile over a group's K slice.
__global__ void __launch_bounds__(256) k_gwgrad(GgArgs ga, int M, int N, float* __restrict__ part) {
  using R = WgRing<2, 2, kGgNst>;
  __shared__ __attribute__((aligned(16))) char smem[kGgNst * R::STAGE];
  int gi;
  const int local = gg_tile(ga, gi);
  const GgGroup& G = ga.g[gi];
  const int ntn = (N + R::TN - 1) / R::TN, ntm = (M + R::TM - 1) / R::TM;
  const int s = local / (ntn * ntm), mn = local % (ntn * ntm);
  const int m0 = (mn / ntn) * R::TM, n0 = (mn % ntn) * R::TN;
  const int64_t kb = (int64_t)s * G.kchunk, ke = min<int64_t>(G.rows, kb + G.kchunk);
  const int nsteps = ke > kb ? (int)((ke - kb) / kWgK) : 0;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w & 1, wn = w >> 1, r = lane & 31, hh = lane >> 5;
  // per-lane source row of each DMA instruction (rows advance by 32 per step: the
  // B clamp to b_rows is per step, through the row index)
  int arow[R::PWA], brow[R::PWB];
  int acol[R::PWA], bcol[R::PWB];
#pragma unroll
  for (int i = 0; i < R::PWA; ++i) {
    constexpr int CPR = R::RBA / 16;
    const int q = w * R::PWA + i, row = q * (1024 / R::RBA) + lane / CPR;
    const int ma = m0 + 8 * ((lane % CPR) ^ wg_swz(row));
    arow[i] = row;
    acol[i] = ma < M ? ma : 0;
  }
#pragma unroll
  for (int i = 0; i < R::PWB; ++i) {
    constexpr int CPR = R::RBB / 16;
    const int q = w * R::PWB + i, row = q * (1024 / R::RBB) + lane / CPR;
    const int nb = n0 + 8 * ((lane % CPR) ^ wg_swz(row));
    brow[i] = row;
    bcol[i] = nb < N ? nb : 0;
  }
  const unsigned lds0 = (unsigned)__builtin_amdgcn_readfirstlane(
      (int)((unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem));
  const unsigned wu = (unsigned)__builtin_amdgcn_readfirstlane(w);
  const int64_t alast = G.rows - 1, blast = G.b_rows - 1;
  auto issue = [&](int step, int buf) {
    const unsigned base = lds0 + buf * R::STAGE;
    const int64_t k0 = kb + (int64_t)step * kWgK;
#pragma unroll
    for (int i = 0; i < R::PWA; ++i)
      wg_dma16(G.a + min(k0 + arow[i], alast) * G.lda + acol[i], base + (wu * R::PWA + i) * 1024);
#pragma unroll
    for (int i = 0; i < R::PWB; ++i)
      wg_dma16(G.b + min(k0 + brow[i], blast) * G.ldb + bcol[i], base + R::IMGA + (wu * R::PWB + i) * 1024);
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
  for (int t = 0; t < kGgNst - 1 && t < nsteps; ++t) issue(t, t);
  for (int t = 0; t < nsteps; ++t) {
    ring_wait<R::P, kGgNst>(nsteps - 1 - t);
    if (t + kGgNst - 1 < nsteps) issue(t + kGgNst - 1, (t + kGgNst - 1) % kGgNst);
    const char* ia = smem + (t % kGgNst) * R::STAGE;
    const char* ib = ia + R::IMGA;
#pragma unroll
    for (int ks = 0; ks < kWgK / 16; ++ks) {
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = ring_frag<R::RBA>(ia, 16 * ks, 64 * wm + 32 * i, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = ring_frag<R::RBB>(ib, 16 * ks, 64 * wn + 32 * j, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma(fa[i], fb[j], acc[i][j]);
    }
  }
  float* out;
  int64_t ldo;
  if (G.part0 >= 0) {
    out = part + (int64_t)(G.part0 + s) * M * N;
    ldo = N;
  } else {
    out = reinterpret_cast<float*>(G.c);
    ldo = G.ldc;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + 64 * wn + 32 * j + r;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + 64 * wm + 32 * i + acc_row(e, hh);
        if (m < M && n < N) out[(int64_t)m * ldo + n] = acc[i][j][e];
      }
    }
}

// C_g = sum over the group's slices, in slice order (split groups only); grid:
// blockIdx.y = the split group's index in `split`, blockIdx.x over M x N / 4.
struct GwSplit {
  int g[kGgMax];
  int n;
};
__global__ void __launch_bounds__(256) k_gwgrad_reduce(GgArgs ga, GwSplit sp, int M, int N,
                                                       const float* __restrict__ part) {
  const GgGroup& G = ga.g[sp.g[blockIdx.y]];
  const int64_t n4 = N / 4, total = (int64_t)M * n4, mn = (int64_t)M * N;
  float* C = reinterpret_cast<float*>(G.c);
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < total; u += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = u / n4, n = (u - m * n4) * 4;
    const float* p = part + (int64_t)G.part0 * mn + m * N + n;
    float4 a = *reinterpret_cast<const float4*>(p);
    for (int s = 1; s < G.slices; ++s) {
      const float4 v = *reinterpret_cast<const float4*>(p + s * mn);
      a.x += v.x;
      a.y += v.y;
      a.z += v.z;
      a.w += v.w;
    }
    *reinterpret_cast<float4*>(C + m * G.ldc + n) = a;
  }
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

int fill_args(const grk_gemm_group* groups, int num_groups, GgArgs* ga) {
  GRK_CHECK_ARG(groups && num_groups >= 1 && num_groups <= kGgMax, "num_groups must be in [1, %d]", kGgMax);
  memset(ga, 0, sizeof(*ga));
  ga->n = num_groups;
  for (int i = 0; i < num_groups; ++i) {
    const grk_gemm_group& q = groups[i];
    GRK_CHECK_ARG(q.a && q.b && q.c && q.rows >= 1, "group %d: a / b / c and rows >= 1 required", i);
    GRK_CHECK_ARG(aligned16(q.a) && aligned16(q.b) && q.lda % 8 == 0 && q.ldb % 8 == 0,
                  "group %d: a / b must be 16-byte aligned with row strides multiples of 8", i);
    GgGroup& g = ga->g[i];
    g.a = (const bf16_t*)q.a;
    g.lda = q.lda;
    g.b = (const bf16_t*)q.b;
    g.ldb = q.ldb;
    g.c = q.c;
    g.ldc = q.ldc;
    g.rows = q.rows;
    g.b_rows = q.b_rows;
    g.part0 = -1;
    g.slices = 1;
  }
  return GRK_OK;
}

}  // namespace
}  // namespace grk

using namespace grk;

extern "C" int grk_grouped_gemm(const grk_gemm_group* groups, int num_groups, int b_layout, int64_t n, int64_t k,
                                int c_dtype, void* stream) {
  clear_error();
  GgArgs ga;
  const int rc = fill_args(groups, num_groups, &ga);
  if (rc) return rc;
  GRK_CHECK_ARG(b_layout == 0 || b_layout == 1, "b_layout must be 0 (B [N, K]) or 1 (B [K, N])");
  GRK_CHECK_ARG(n >= 8 && n % 8 == 0 && n < (1 << 24), "n must be a positive multiple of 8");
  GRK_CHECK_ARG(k >= kWgK && k % kWgK == 0 && k < (1 << 24), "k must be a positive multiple of %d", kWgK);
  GRK_CHECK_ARG(c_dtype == GRK_F32 || c_dtype == GRK_BF16, "c must be fp32 or bf16");
  int64_t tiles = 0;
  const int64_t ntn = (n + kGgTile - 1) / kGgTile;
  for (int i = 0; i < num_groups; ++i) {
    const GgGroup& g = ga.g[i];
    GRK_CHECK_ARG(g.lda >= k && g.ldb >= (b_layout ? n : k) && g.ldc >= n,
                  "group %d: row strides must cover k (A), %s (B) and n (C)", i, b_layout ? "n" : "k");
    ga.g[i].tile0 = (int)tiles;
    tiles += (g.rows + kGgTile - 1) / kGgTile * ntn;
    GRK_CHECK_ARG(tiles < (1 << 30), "too many tiles");
  }
  ga.total = (int)tiles;
  hipStream_t s = (hipStream_t)stream;
  const unsigned g = (unsigned)tiles;
  if (b_layout == 1) {
    if (c_dtype == GRK_BF16) k_ggemm<true, bf16_t><<<g, 256, 0, s>>>(ga, (int)n, (int)k);
    else k_ggemm<true, float><<<g, 256, 0, s>>>(ga, (int)n, (int)k);
  } else {
    if (c_dtype == GRK_BF16) k_ggemm<false, bf16_t><<<g, 256, 0, s>>>(ga, (int)n, (int)k);
    else k_ggemm<false, float><<<g, 256, 0, s>>>(ga, (int)n, (int)k);
  }
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

namespace {
// K split of a weight-gradient group: slices of about kGwSliceRows rows, whole steps
void gw_split(int64_t rows, int* slices, int* kchunk) {
  const int64_t steps = rows / kWgK;
  int S = (int)std::min<int64_t>(16, std::max<int64_t>(1, (rows + kGwSliceRows / 2) / kGwSliceRows));
  const int64_t per = (steps + S - 1) / S;
  S = (int)((steps + per - 1) / per);
  *slices = S;
  *kchunk = (int)(per * kWgK);
}
}  // namespace

extern "C" size_t grk_grouped_wgrad_workspace(const grk_gemm_group* groups, int num_groups, int64_t m, int64_t n) {
  if (!groups || num_groups < 1 || num_groups > kGgMax || m <= 0 || n <= 0) return 0;
  size_t parts = 0;
  for (int i = 0; i < num_groups; ++i) {
    if (groups[i].rows < kWgK || groups[i].rows % kWgK) return 0;
    int S, kc;
    gw_split(groups[i].rows, &S, &kc);
    if (S > 1) parts += (size_t)S;
  }
  return std::max<size_t>(parts * (size_t)m * (size_t)n * sizeof(float), 16);
}

extern "C" int grk_grouped_wgrad(const grk_gemm_group* groups, int num_groups, int64_t m, int64_t n, void* workspace,
                                 size_t workspace_bytes, void* stream) {
  clear_error();
  GgArgs ga;
  const int rc = fill_args(groups, num_groups, &ga);
  if (rc) return rc;
  GRK_CHECK_ARG(m >= 8 && n >= 8 && m % 8 == 0 && n % 8 == 0 && m < (1 << 16) && n < (1 << 16),
                "m and n must be positive multiples of 8");
  GRK_CHECK_ARG(workspace && workspace_bytes >= grk_grouped_wgrad_workspace(groups, num_groups, m, n),
                "workspace smaller than grk_grouped_wgrad_workspace()");
  using R = WgRing<2, 2, kGgNst>;
  const int64_t tiles_mn = ((m + R::TM - 1) / R::TM) * ((n + R::TN - 1) / R::TN);
  int64_t tiles = 0;
  int parts = 0;
  GwSplit sp;
  memset(&sp, 0, sizeof(sp));
  for (int i = 0; i < num_groups; ++i) {
    GgGroup& g = ga.g[i];
    GRK_CHECK_ARG(g.rows >= kWgK && g.rows % kWgK == 0, "group %d: K rows must be a positive multiple of %d", i, kWgK);
    GRK_CHECK_ARG(g.b_rows >= 1 && g.b_rows <= g.rows, "group %d: b_rows must be in [1, rows]", i);
    GRK_CHECK_ARG(g.lda >= m && g.ldb >= n && g.ldc >= n && g.ldc % 4 == 0 && aligned16(g.c),
                  "group %d: row strides must cover m (A) / n (B, C); C 16-byte aligned, ldc a multiple of 4", i);
    gw_split(g.rows, &g.slices, &g.kchunk);
    if (g.slices > 1) {
      g.part0 = parts;
      parts += g.slices;
      sp.g[sp.n++] = i;
    }
    g.tile0 = (int)tiles;
    tiles += tiles_mn * g.slices;
  }
  ga.total = (int)tiles;
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)workspace;
  k_gwgrad<<<(unsigned)tiles, 256, 0, s>>>(ga, (int)m, (int)n, part);
  GRK_LAUNCH_CHECK();
  if (sp.n) {
    const int64_t work = m * n / 4;
    const dim3 grid((unsigned)std::min<int64_t>((work + 255) / 256, 256), (unsigned)sp.n);
    k_gwgrad_reduce<<<grid, 256, 0, s>>>(ga, sp, (int)m, (int)n, part);
    GRK_LAUNCH_CHECK();
  }
  return GRK_OK;
}
