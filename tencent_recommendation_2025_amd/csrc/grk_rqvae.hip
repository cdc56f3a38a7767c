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
// Work is VALU-bound (3 * levels * codes * dim flops per row, ~1.5e5 at
// 3 x 256 x 64) and reads each row once: one workgroup of 256 threads owns 32
// rows; 8 threads per row split the codes and keep the row's residual in
// registers.  A level's codebook is staged into LDS in chunks (rows padded by
// 4 floats: the four code rows one ds_read_b128 of a wave touches land in
// disjoint banks), every thread scores two codes at once with packed fp32
// (v_pk_add/v_pk_mul: element-wise IEEE, so the per-code order is unchanged),
// and the 8 partial minima meet in LDS in a fixed order.
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

template <int D>
__global__ __launch_bounds__(kRqBlock) void k_rq_assign(const float* __restrict__ z, int64_t ld_z,
                                                        const float* __restrict__ cb, int64_t n, int K,
                                                        int levels, int chunk, int32_t* __restrict__ codes_out,
                                                        float* __restrict__ quant, float* __restrict__ dist_out,
                                                        float* __restrict__ resid) {
  extern __shared__ float4 rq_smem[];
  float* sc = reinterpret_cast<float*>(rq_smem);
  __shared__ float red_d[kRqGroups][kRqRows];
  __shared__ int red_k[kRqGroups][kRqRows];
  __shared__ int code_sh[kRqMaxLevels][kRqRows];
  constexpr int S = rq_stride(D);

  const int tid = threadIdx.x;
  const int row = tid % kRqRows;
  const int g = tid / kRqRows;
  const int64_t gr = (int64_t)blockIdx.x * kRqRows + row;
  const bool valid = gr < n;

  float r[D];
  if (valid) {
    const float4* zp = reinterpret_cast<const float4*>(z + gr * ld_z);
#pragma unroll
    for (int j = 0; j < D / 4; ++j) {
      const float4 v = zp[j];
      r[4 * j] = v.x; r[4 * j + 1] = v.y; r[4 * j + 2] = v.z; r[4 * j + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < D; ++j) r[j] = 0.f;
  }

  for (int l = 0; l < levels; ++l) {
    const float* C = cb + (int64_t)l * K * D;
    float bd = INFINITY;
    int bk = 0x7fffffff;
    for (int c0 = 0; c0 < K; c0 += chunk) {
      const int cn = min(chunk, K - c0);
      __syncthreads();  // previous chunk / level fully read
      for (int i = tid; i < cn * (D / 4); i += kRqBlock) {
        const int k = i / (D / 4), q = i % (D / 4);
        *reinterpret_cast<float4*>(sc + k * S + 4 * q) =
            *reinterpret_cast<const float4*>(C + (int64_t)(c0 + k) * D + 4 * q);
      }
      __syncthreads();
      // this thread scores local codes k, k+1 for k = 2g, 2g + 16, ...: its
      // codes ascend, so strict < keeps the lowest k of equal distances
      for (int k = 2 * g; k < cn; k += 2 * kRqGroups) {
        const bool two = k + 1 < cn;
        const float* a = sc + k * S;
        const float* b = sc + (two ? k + 1 : k) * S;
        f2 acc = {0.f, 0.f};
#pragma unroll
        for (int j = 0; j < D; j += 4) {
          const float4 ca = *reinterpret_cast<const float4*>(a + j);
          const float4 cv = *reinterpret_cast<const float4*>(b + j);
          f2 d;
          d = f2{r[j], r[j]} - f2{ca.x, cv.x};         acc = acc + d * d;
          d = f2{r[j + 1], r[j + 1]} - f2{ca.y, cv.y}; acc = acc + d * d;
          d = f2{r[j + 2], r[j + 2]} - f2{ca.z, cv.z}; acc = acc + d * d;
          d = f2{r[j + 3], r[j + 3]} - f2{ca.w, cv.w}; acc = acc + d * d;
        }
        if (acc.x < bd) { bd = acc.x; bk = c0 + k; }
        if (two && acc.y < bd) { bd = acc.y; bk = c0 + k + 1; }
      }
    }
    red_d[g][row] = bd;
    red_k[g][row] = bk;
    __syncthreads();
    // every thread of the row reduces the 8 partial minima in the same order
    float md = red_d[0][row];
    int mk = red_k[0][row];
#pragma unroll
    for (int q = 1; q < kRqGroups; ++q) {
      const float d = red_d[q][row];
      const int kk = red_k[q][row];
      if (d < md || (d == md && kk < mk)) { md = d; mk = kk; }
    }
    if (mk >= K) mk = 0;  // every distance NaN
    const float4* cw = reinterpret_cast<const float4*>(C + (int64_t)mk * D);
#pragma unroll
    for (int j = 0; j < D / 4; ++j) {
      const float4 v = cw[j];
      r[4 * j] = r[4 * j] - v.x; r[4 * j + 1] = r[4 * j + 1] - v.y;
      r[4 * j + 2] = r[4 * j + 2] - v.z; r[4 * j + 3] = r[4 * j + 3] - v.w;
    }
    if (g == 0) {
      code_sh[l][row] = mk;
      if (valid) {
        codes_out[gr * levels + l] = mk;
        if (dist_out) dist_out[gr * levels + l] = md;
      }
    }
  }
  __syncthreads();
  if (!valid) return;
  // group g writes columns [g*D/8, (g+1)*D/8) of quant / resid (compile-time
  // column loop with a predicate: no dynamic register indexing)
  constexpr int W = D / kRqGroups;
#pragma unroll
  for (int j = 0; j < D; ++j) {
    if (j / W != g) continue;
    if (quant) {
      float q = cb[(int64_t)code_sh[0][row] * D + j];
      for (int l = 1; l < levels; ++l) q = q + cb[((int64_t)l * K + code_sh[l][row]) * D + j];
      quant[gr * D + j] = q;
    }
    if (resid) resid[gr * D + j] = r[j];
  }
}

template <int D>
int launch_rq(const float* z, int64_t ld_z, const float* cb, int64_t n, int K, int levels, int32_t* codes,
              float* quant, float* dist, float* resid, hipStream_t s) {
  const int chunk = rq_chunk(D, K);
  const size_t lds = (size_t)chunk * rq_stride(D) * sizeof(float);
  static bool attr_set = false;
  if (!attr_set) {
    GRK_CHECK_HIP(hipFuncSetAttribute((const void*)k_rq_assign<D>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      kRqLdsBytes));
    attr_set = true;
  }
  const int64_t blocks = (n + kRqRows - 1) / kRqRows;
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
  GRK_CHECK_ARG(n < (int64_t)0x7FFFFFFF * kRqRows, "n too large");
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
