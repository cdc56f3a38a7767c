// Exact maximum-inner-product top-k retrieval (gfx950): the ANN step of the
// reference's inference (model/BaseLine/infer.py:213-225, an external faiss
// HNSW binary, inner-product metric, top-10), done by brute force.
//
// Pass 1 (k_mips_scan): one workgroup = 4 waves x 32 queries; the query rows
// live in registers as bf16 MFMA A-fragments for the whole scan; the item
// slice of the workgroup's split streams through in tiles of 64 items
// (B-fragments straight from global memory -- the 4 waves walk the same tiles
// in step, so 3 of 4 reads are cache hits).  Each 32x64 score tile goes
// through a padded LDS window so lane (q, half) sees the 32 scores of one
// query and keeps a sorted register list of its 16 best (score desc, item
// index asc).  Output: 16 candidate item indices per (query, split, half).
//
// Pass 2 (k_mips_rerank): one wave per query re-scores every candidate in
// fp32 (lane-strided products, fixed xor-butterfly sum: the same order for
// every candidate, deterministic) and selects the k best by the same total
// order.  bf16 scoring in pass 1 only decides which 16 items per slice reach
// pass 2; the returned scores and order are fp32's.
#include "grk_mfma.h"

#include <math.h>

namespace grk {
namespace {

constexpr int kQPerWave = 32;
constexpr int kQPerBlock = 4 * kQPerWave;
constexpr int kItemTile = 64;
constexpr int kCand = 16;           // candidates per (query, split, half) = max k
constexpr int kMaxSplits = 32;
constexpr int kSPitch = kItemTile + 1;  // padded LDS row: conflict-free column reads

__device__ __forceinline__ bool better(float a, int ia, float b, int ib) {
  return a > b || (a == b && ia < ib);
}

template <int KS>  // KS = 16-wide k-steps held in registers (dim <= 16 KS)
__global__ void __launch_bounds__(256) k_mips_scan(const void* __restrict__ queries, int64_t ld_q,
                                                   const void* __restrict__ items, int64_t ld_i, int f32,
                                                   int64_t nq, int64_t ni, int dim, int splits,
                                                   int64_t tiles_per_split, int32_t* __restrict__ cand) {
  __shared__ float sh[4][kQPerWave * kSPitch];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, hh = lane >> 5;
  const int64_t q0 = (int64_t)blockIdx.x * kQPerBlock + wave * kQPerWave;
  const int split = blockIdx.y;
  const bool isf = f32 != 0;

  bf16x8 qf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int col = 16 * ks + 8 * hh;
    qf[ks] = gload8_any(queries, (q0 + r) * ld_q + col, isf, q0 + r < nq && col < dim);
  }

  float ts[kCand];
  int ti[kCand];
#pragma unroll
  for (int j = 0; j < kCand; ++j) { ts[j] = -INFINITY; ti[j] = -1; }

  float* S = sh[wave];
  const int myq = lane & 31, half = lane >> 5;
  const int64_t tiles = (ni + kItemTile - 1) / kItemTile;
  const int64_t t_begin = split * tiles_per_split;
  const int64_t t_end = t_begin + tiles_per_split < tiles ? t_begin + tiles_per_split : tiles;
  for (int64_t t = t_begin; t < t_end; ++t) {
    const int64_t n0 = t * kItemTile;
    f32x16 acc0 = {}, acc1 = {};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int col = 16 * ks + 8 * hh;
      const bool kok = col < dim;
      const bf16x8 b0 = gload8_any(items, (n0 + r) * ld_i + col, isf, kok && n0 + r < ni);
      const bf16x8 b1 = gload8_any(items, (n0 + 32 + r) * ld_i + col, isf, kok && n0 + 32 + r < ni);
      acc0 = mfma(qf[ks], b0, acc0);
      acc1 = mfma(qf[ks], b1, acc1);
    }
    // D[query][item]: lane (r, hh) holds item column r, query rows acc_row(i, hh)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = acc_row(i, hh);
      S[row * kSPitch + r] = n0 + r < ni ? acc0[i] : -INFINITY;
      S[row * kSPitch + 32 + r] = n0 + 32 + r < ni ? acc1[i] : -INFINITY;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int64_t base = n0 + 32 * half;
#pragma unroll 4
    for (int j = 0; j < 32; ++j) {
      const float v = S[myq * kSPitch + 32 * half + j];
      if (v > ts[kCand - 1]) {  // items arrive in index order: equal scores keep the earlier item
        ts[kCand - 1] = v;
        ti[kCand - 1] = (int)(base + j);
#pragma unroll
        for (int m = kCand - 1; m > 0; --m) {
          if (ts[m] > ts[m - 1]) {
            const float a = ts[m]; ts[m] = ts[m - 1]; ts[m - 1] = a;
            const int b = ti[m]; ti[m] = ti[m - 1]; ti[m - 1] = b;
          }
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  const int64_t q = q0 + myq;
  if (q < nq) {
    int32_t* out = cand + ((q * splits + split) * 2 + half) * kCand;
#pragma unroll
    for (int j = 0; j < kCand; ++j) out[j] = ti[j];
  }
}

__device__ __forceinline__ float load_any(const void* base, int64_t off, bool f32) {
  return f32 ? reinterpret_cast<const float*>(base)[off] : bf16_to_f32(reinterpret_cast<const bf16_t*>(base)[off]);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

// one wave per query; ncand = splits * 2 * kCand candidates
template <int M>  // M = ceil(dim / 64) elements per lane
__global__ void __launch_bounds__(256) k_mips_rerank(const void* __restrict__ queries, int64_t ld_q,
                                                     const void* __restrict__ items, int64_t ld_i, int f32,
                                                     int64_t nq, int dim, int ncand, int k,
                                                     const int32_t* __restrict__ cand,
                                                     const uint64_t* __restrict__ item_ids,
                                                     float* __restrict__ out_scores, int64_t* __restrict__ out_ids) {
  __shared__ float sc_all[4][2 * kMaxSplits * kCand];
  __shared__ int id_all[4][2 * kMaxSplits * kCand];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 4 + wave;
  if (q >= nq) return;
  const bool isf = f32 != 0;
  float* sc = sc_all[wave];
  int* id = id_all[wave];
  float qv[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int e = lane + 64 * m;
    qv[m] = e < dim ? load_any(queries, q * ld_q + e, isf) : 0.f;
  }
  const int32_t* cq = cand + q * ncand;
  for (int c0 = 0; c0 < ncand; c0 += 4) {
    int ic[4];
    float part[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      ic[u] = c0 + u < ncand ? cq[c0 + u] : -1;
      part[u] = 0.f;
      if (ic[u] >= 0) {
#pragma unroll
        for (int m = 0; m < M; ++m) {
          const int e = lane + 64 * m;
          if (e < dim) part[u] = fmaf(qv[m], load_any(items, (int64_t)ic[u] * ld_i + e, isf), part[u]);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float s = wave_sum(part[u]);
      if (lane == 0 && c0 + u < ncand) {
        sc[c0 + u] = ic[u] >= 0 ? s : -INFINITY;
        id[c0 + u] = ic[u] >= 0 ? ic[u] : INT32_MAX;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  for (int j = 0; j < k; ++j) {
    float bs = -INFINITY;
    int bi = INT32_MAX, bc = -1;
    for (int c = lane; c < ncand; c += 64) {
      const float s = sc[c];
      const int i = id[c];
      if (bc < 0 || better(s, i, bs, bi)) { bs = s; bi = i; bc = c; }
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      const float os = __shfl_xor(bs, m, 64);
      const int oi = __shfl_xor(bi, m, 64), oc = __shfl_xor(bc, m, 64);
      if (oc >= 0 && (bc < 0 || better(os, oi, bs, bi))) { bs = os; bi = oi; bc = oc; }
    }
    const bool real = bc >= 0 && bi != INT32_MAX;
    if (lane == 0) {
      out_scores[q * k + j] = real ? bs : -INFINITY;
      out_ids[q * k + j] = real ? (item_ids ? (int64_t)item_ids[bi] : (int64_t)bi) : -1;
      if (bc >= 0) { sc[bc] = -INFINITY; id[bc] = INT32_MAX; }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

int mips_splits(int64_t nq, int64_t ni) {
  const int64_t qtiles = (nq + kQPerBlock - 1) / kQPerBlock;
  const int64_t tiles = (ni + kItemTile - 1) / kItemTile;
  int64_t s = (1024 + qtiles - 1) / (qtiles > 0 ? qtiles : 1);
  if (s > kMaxSplits) s = kMaxSplits;
  if (s > tiles) s = tiles;
  return (int)(s < 1 ? 1 : s);
}

}  // namespace
}  // namespace grk

using namespace grk;

extern "C" size_t grk_mips_topk_workspace(int64_t num_queries, int64_t num_items) {
  if (num_queries <= 0 || num_items <= 0) return 256;
  return (size_t)num_queries * mips_splits(num_queries, num_items) * 2 * kCand * sizeof(int32_t) + 256;
}

extern "C" int grk_mips_topk(const void* queries, int64_t ld_q, const void* items, int64_t ld_i, int dtype,
                             int64_t num_queries, int64_t num_items, int dim, int k, const uint64_t* item_ids,
                             float* out_scores, int64_t* out_ids, void* workspace, size_t workspace_bytes,
                             void* stream) {
  clear_error();
  GRK_CHECK_ARG(dtype == GRK_F32 || dtype == GRK_BF16, "dtype must be GRK_F32 or GRK_BF16");
  GRK_CHECK_ARG(dim > 0 && dim % 8 == 0 && dim <= 512, "dim (%d) must be a positive multiple of 8, <= 512", dim);
  GRK_CHECK_ARG(k >= 1 && k <= kCand, "k (%d) must be in [1, %d]", k, kCand);
  GRK_CHECK_ARG(num_queries >= 0 && num_items >= 0, "negative sizes");
  GRK_CHECK_ARG(num_items < INT32_MAX, "num_items must be < 2^31");
  GRK_CHECK_ARG(ld_q >= dim && ld_i >= dim, "row strides must be >= dim");
  const size_t es = dtype == GRK_F32 ? 4 : 2;
  GRK_CHECK_ARG((ld_q * es) % 16 == 0 && (ld_i * es) % 16 == 0, "row strides must be multiples of 16 bytes");
  GRK_CHECK_ARG(((uintptr_t)queries % 16) == 0 && ((uintptr_t)items % 16) == 0, "rows must be 16-byte aligned");
  if (num_queries == 0) return GRK_OK;
  GRK_CHECK_ARG(out_scores && out_ids, "null output");
  hipStream_t s = (hipStream_t)stream;
  const int f32 = dtype == GRK_F32;
  if (num_items == 0) {
    const int64_t n = num_queries * k;
    // -inf / -1 fill through the rerank kernel's empty-candidate path: no candidates
    k_mips_rerank<1><<<(unsigned)((num_queries + 3) / 4), 256, 0, s>>>(queries, ld_q, queries, ld_q, f32,
                                                                        num_queries, dim, 0, k, nullptr, nullptr,
                                                                        out_scores, out_ids);
    GRK_LAUNCH_CHECK();
    (void)n;
    return GRK_OK;
  }
  const int splits = mips_splits(num_queries, num_items);
  const size_t need = (size_t)num_queries * splits * 2 * kCand * sizeof(int32_t);
  GRK_CHECK_ARG(workspace && workspace_bytes >= need, "workspace too small (%zu < %zu bytes)", workspace_bytes, need);
  int32_t* cand = (int32_t*)workspace;
  const int64_t tiles = (num_items + kItemTile - 1) / kItemTile;
  const int64_t tps = (tiles + splits - 1) / splits;
  dim3 g1((unsigned)((num_queries + kQPerBlock - 1) / kQPerBlock), (unsigned)splits);
  const int ks = (dim + 15) / 16;
#define GRK_SCAN(KS)                                                                                        \
  k_mips_scan<KS><<<g1, 256, 0, s>>>(queries, ld_q, items, ld_i, f32, num_queries, num_items, dim, splits, \
                                     tps, cand)
  if (ks <= 4) GRK_SCAN(4);
  else if (ks <= 8) GRK_SCAN(8);
  else if (ks <= 16) GRK_SCAN(16);
  else GRK_SCAN(32);
#undef GRK_SCAN
  GRK_LAUNCH_CHECK();
  const int ncand = splits * 2 * kCand;
  const unsigned g2 = (unsigned)((num_queries + 3) / 4);
  const int m = (dim + 63) / 64;
#define GRK_RERANK(M)                                                                                          \
  k_mips_rerank<M><<<g2, 256, 0, s>>>(queries, ld_q, items, ld_i, f32, num_queries, dim, ncand, k, cand, item_ids, \
                                      out_scores, out_ids)
  switch (m) {
    case 1: GRK_RERANK(1); break;
    case 2: GRK_RERANK(2); break;
    case 3: case 4: GRK_RERANK(4); break;
    default: GRK_RERANK(8); break;
  }
#undef GRK_RERANK
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}
