// Residual quantisation: the code search of config 4's RQ-VAE semantic-ID
// tokenizer (BASELINE.json configs[3]; the reference has no tokenizer -- its
// anchor is the item side of model/BaseLineO1/model.py:167-555, where the
// semantic ids enter as extra item_sparse features).
//
// For every row z of the latent matrix and every level l (codebooks C_l):
//   r_0 = z
//   code_l = argmin_k  sum_j (r_l[j] - C_l[k][j])^2     (lowest k on ties)
//   r_{l+1} = r_l - C_l[code_l]
//   quant   = C_0[code_0] + C_1[code_1] + ...           (level order)
// The distance is the direct squared difference in fp32: each difference,
// square and partial sum rounded, j ascending (this file is compiled with
// -ffp-contract=off, so no FMA fuses the square into the sum).  The codes are
// therefore a pure function of the fp32 inputs and oracle/rqvae.py restates
// them bit-exactly with numpy -- the ||r||^2 - 2 r.c + ||c||^2 GEMM form would
// put MFMA rounding into the argmin and flip near-ties.
//
// Work is 3 * levels * codes * dim flops per row (~1.5e5 at 3 x 256 x 64) and
// reads each row once.  A workgroup of 256 threads owns 32 row slots; 8 threads
// per slot split the codes and keep the residuals in registers.  A level's
// codebook is staged into LDS in chunks (rows padded by 4 floats: the code
// rows one ds_read_b128 of a wave touches land in disjoint banks) and the 8
// partial minima meet in LDS in a fixed order.  Packed fp32 (v_pk_add /
// v_pk_mul: element-wise IEEE, per-code order unchanged) does two distances
// per op: two ROWS per thread against one code, so every LDS read serves two
// rows (a one-row form packing two codes was bound by LDS read bandwidth: a
// ds_read_b128 delivers 16 B to every lane, broadcast or not; 4.83 vs 3.46 ms
// at latent 64, 17.8 vs 11.2 ms at 128).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "grk.h"
#include "grk_common.h"

namespace grk {
namespace {

constexpr int kRqRows = 32;                    // rows per workgroup
constexpr int kRqGroups = 8;                   // threads per row (code groups)
constexpr int kRqBlock = kRqRows * kRqGroups;  // 256
constexpr int kRqMaxLevels = 8;
constexpr int kRqLdsBytes = 76 * 1024;         // two workgroups per CU

typedef float f2 __attribute__((ext_vector_type(2)));

__host__ __device__ constexpr int rq_stride(int d) { return d + 4; }

int rq_chunk(int d, int codes) {
  int c = (kRqLdsBytes / (rq_stride(d) * 4)) & ~(2 * kRqGroups - 1);
  return codes < c ? codes : c;
}

// Two rows per thread, packed over the rows: lane pair (row a, row b) of one
// register pair meets one code per packed op, so every codebook element read
// from LDS serves two rows -- the one-row form is bound by the LDS read
// bandwidth (each ds_read_b128 delivers 16 B to every lane, broadcast or not).
// Threads take codes g, g + 8, ... in ascending order (strict < keeps the
// lowest code of equal distances).
template <int D>
__global__ __launch_bounds__(kRqBlock) void k_rq_assign(const float* __restrict__ z, int64_t ld_z,
                                                         const float* __restrict__ cb, int64_t n, int K,
                                                         int levels, int chunk, int32_t* __restrict__ codes_out,
                                                         float* __restrict__ quant, float* __restrict__ dist_out,
                                                         float* __restrict__ resid) {
  constexpr int ROWS = 2 * kRqRows;
  extern __shared__ float4 rq_smem[];
  float* sc = reinterpret_cast<float*>(rq_smem);
  __shared__ float red_d[kRqGroups][ROWS];
  __shared__ int red_k[kRqGroups][ROWS];
  __shared__ int code_sh[kRqMaxLevels][ROWS];
  constexpr int S = rq_stride(D);

  const int tid = threadIdx.x;
  const int slot = tid % kRqRows;
  const int g = tid / kRqRows;
  const int64_t ga = (int64_t)blockIdx.x * ROWS + slot, gb = ga + kRqRows;

  f2 r[D];  // r[j] = (row a, row b)
#pragma unroll
  for (int j = 0; j < D; ++j) r[j] = f2{0.f, 0.f};
  if (ga < n) {
    const float4* zp = reinterpret_cast<const float4*>(z + ga * ld_z);
#pragma unroll
    for (int j = 0; j < D / 4; ++j) {
      const float4 v = zp[j];
      r[4 * j].x = v.x; r[4 * j + 1].x = v.y; r[4 * j + 2].x = v.z; r[4 * j + 3].x = v.w;
    }
  }
  if (gb < n) {
    const float4* zp = reinterpret_cast<const float4*>(z + gb * ld_z);
#pragma unroll
    for (int j = 0; j < D / 4; ++j) {
      const float4 v = zp[j];
      r[4 * j].y = v.x; r[4 * j + 1].y = v.y; r[4 * j + 2].y = v.z; r[4 * j + 3].y = v.w;
    }
  }

  for (int l = 0; l < levels; ++l) {
    const float* C = cb + (int64_t)l * K * D;
    float bda = INFINITY, bdb = INFINITY;
    int bka = 0x7fffffff, bkb = 0x7fffffff;
    for (int c0 = 0; c0 < K; c0 += chunk) {
      const int cn = min(chunk, K - c0);
      __syncthreads();  // previous chunk / level fully read
      for (int i = tid; i < cn * (D / 4); i += kRqBlock) {
        const int k = i / (D / 4), q = i % (D / 4);
        *reinterpret_cast<float4*>(sc + k * S + 4 * q) =
            *reinterpret_cast<const float4*>(C + (int64_t)(c0 + k) * D + 4 * q);
      }
      __syncthreads();
      // codes k and k + 8 side by side: two independent dependent-add chains
      // interleave (one chain alone stalls on every packed result)
      for (int k = g; k < cn; k += 2 * kRqGroups) {
        const bool two = k + kRqGroups < cn;
        const float* a = sc + k * S;
        const float* b = sc + (two ? k + kRqGroups : k) * S;
        f2 acc = {0.f, 0.f}, acc2 = {0.f, 0.f};
#pragma unroll
        for (int j = 0; j < D; j += 4) {
          const float4 c = *reinterpret_cast<const float4*>(a + j);
          const float4 e = *reinterpret_cast<const float4*>(b + j);
          f2 d, d2;
          d = r[j] - f2{c.x, c.x};         d2 = r[j] - f2{e.x, e.x};
          acc = acc + d * d;               acc2 = acc2 + d2 * d2;
          d = r[j + 1] - f2{c.y, c.y};     d2 = r[j + 1] - f2{e.y, e.y};
          acc = acc + d * d;               acc2 = acc2 + d2 * d2;
          d = r[j + 2] - f2{c.z, c.z};     d2 = r[j + 2] - f2{e.z, e.z};
          acc = acc + d * d;               acc2 = acc2 + d2 * d2;
          d = r[j + 3] - f2{c.w, c.w};     d2 = r[j + 3] - f2{e.w, e.w};
          acc = acc + d * d;               acc2 = acc2 + d2 * d2;
        }
        if (acc.x < bda) { bda = acc.x; bka = c0 + k; }
        if (acc.y < bdb) { bdb = acc.y; bkb = c0 + k; }
        if (two && acc2.x < bda) { bda = acc2.x; bka = c0 + k + kRqGroups; }
        if (two && acc2.y < bdb) { bdb = acc2.y; bkb = c0 + k + kRqGroups; }
      }
    }
    red_d[g][slot] = bda;
    red_k[g][slot] = bka;
    red_d[g][slot + kRqRows] = bdb;
    red_k[g][slot + kRqRows] = bkb;
    __syncthreads();
    int mk2[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int row = slot + u * kRqRows;
      float md = red_d[0][row];
      int mk = red_k[0][row];
#pragma unroll
      for (int q = 1; q < kRqGroups; ++q) {
        const float d = red_d[q][row];
        const int kk = red_k[q][row];
        if (d < md || (d == md && kk < mk)) { md = d; mk = kk; }
      }
      if (mk >= K) mk = 0;  // every distance NaN
      mk2[u] = mk;
      const int64_t gr = u ? gb : ga;
      if (g == 0) {
        code_sh[l][row] = mk;
        if (gr < n) {
          codes_out[gr * levels + l] = mk;
          if (dist_out) dist_out[gr * levels + l] = md;
        }
      }
    }
    const float4* ca = reinterpret_cast<const float4*>(C + (int64_t)mk2[0] * D);
    const float4* cbw = reinterpret_cast<const float4*>(C + (int64_t)mk2[1] * D);
#pragma unroll
    for (int j = 0; j < D / 4; ++j) {
      const float4 va = ca[j], vb = cbw[j];
      r[4 * j] = r[4 * j] - f2{va.x, vb.x};
      r[4 * j + 1] = r[4 * j + 1] - f2{va.y, vb.y};
      r[4 * j + 2] = r[4 * j + 2] - f2{va.z, vb.z};
      r[4 * j + 3] = r[4 * j + 3] - f2{va.w, vb.w};
    }
  }
  __syncthreads();
  constexpr int W = D / kRqGroups;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int row = slot + u * kRqRows;
    const int64_t gr = u ? gb : ga;
    if (gr >= n) continue;
#pragma unroll
    for (int j = 0; j < D; ++j) {
      if (j / W != g) continue;
      if (quant) {
        float q = cb[(int64_t)code_sh[0][row] * D + j];
        for (int l = 1; l < levels; ++l) q = q + cb[((int64_t)l * K + code_sh[l][row]) * D + j];
        quant[gr * D + j] = q;
      }
      if (resid) resid[gr * D + j] = u ? r[j].y : r[j].x;
    }
  }
}

template <int D>
int launch_rq(const float* z, int64_t ld_z, const float* cb, int64_t n, int K, int levels, int32_t* codes,
              float* quant, float* dist, float* resid, hipStream_t s) {
  const int chunk = rq_chunk(D, K);
  const size_t lds = (size_t)chunk * rq_stride(D) * sizeof(float);
  GRK_CHECK_HIP(ensure_dynamic_lds((const void*)k_rq_assign<D>, kRqLdsBytes));
  const int64_t blocks = (n + 2 * kRqRows - 1) / (2 * kRqRows);
  k_rq_assign<D><<<dim3((unsigned)blocks), kRqBlock, lds, s>>>(z, ld_z, cb, n, K, levels, chunk, codes, quant,
                                                                 dist, resid);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

}  // namespace
}  // namespace grk

using namespace grk;

extern "C" int grk_rq_assign(const float* z, int64_t ld_z, const float* codebooks, int64_t n, int dim,
                             int codes, int levels, int32_t* out_codes, float* out_quant, float* out_dist,
                             float* out_resid, void* stream) {
  clear_error();
  GRK_CHECK_ARG(n >= 0, "n must be >= 0");
  GRK_CHECK_ARG(dim == 16 || dim == 32 || dim == 64 || dim == 128, "dim (%d) must be 16, 32, 64 or 128", dim);
  GRK_CHECK_ARG(codes >= 1 && codes <= 65536, "codes (%d) must be in [1, 65536]", codes);
  GRK_CHECK_ARG(levels >= 1 && levels <= kRqMaxLevels, "levels (%d) must be in [1, %d]", levels, kRqMaxLevels);
  GRK_CHECK_ARG(ld_z >= dim && ld_z % 4 == 0, "ld_z (%lld) must be >= dim and a multiple of 4", (long long)ld_z);
  GRK_CHECK_ARG(n < (int64_t)0x7FFFFFFF * kRqRows, "n too large");  // grid.x
  if (n == 0) return GRK_OK;
  GRK_CHECK_ARG(z && codebooks && out_codes, "NULL z / codebooks / out_codes");
  GRK_CHECK_ARG(((uintptr_t)z & 15) == 0 && ((uintptr_t)codebooks & 15) == 0, "z / codebooks must be 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  switch (dim) {
    case 16: return launch_rq<16>(z, ld_z, codebooks, n, codes, levels, out_codes, out_quant, out_dist, out_resid, s);
    case 32: return launch_rq<32>(z, ld_z, codebooks, n, codes, levels, out_codes, out_quant, out_dist, out_resid, s);
    case 64: return launch_rq<64>(z, ld_z, codebooks, n, codes, levels, out_codes, out_quant, out_dist, out_resid, s);
    default: return launch_rq<128>(z, ld_z, codebooks, n, codes, levels, out_codes, out_quant, out_dist, out_resid, s);
  }
}
