// The composed itemdnn / userdnn weight of the projection restatement
// (model._dnn_weight, functional.dnn_weight) in one launch each way.
//
//   W = [ B_0 | B_1 .. (direct features) | W_k Wt_k (mm features) | b + sum_k W_k bt_k | 0 ]
//
// B_j / W_k are column blocks of the dnn weight (fp32 views with the weight's
// row stride), [Wt_k | bt_k] the feature's emb_transform (kk x w weight, kk
// bias).  The reference runs itemdnn(cat(item_emb, feature embs,
// emb_transform(mm))) (model/BaseLine/model.py:129-139, 242-277); the
// restatement folds emb_transform into the weight so one GEMM reads the mm
// values directly.  Eager torch composed it with a cat per feature, a GEMM per
// feature, an add, a cat of every block and a cast (backward: a cast, a cat and
// two GEMMs per feature) -- ~12 launches of a few microseconds per step.  Here:
//   forward : one launch, a workgroup per 8 output rows with W_k's rows and
//             [Wt | bt] in LDS (the K = kk products of the mm columns and the bias
//             column summed in k order, fp32);
//   backward: g32 = fp32(g) and dW_k = dM [Wt | bt]^T (a workgroup per 8 rows),
//             [dWt | dbt] = W_k^T dM (a workgroup per 16 columns of W_k, those and
//             all of dM in LDS), dM = [g(mm columns) | g(bias column)]; fixed-order
//             sums.  Shapes whose tiles do not fit LDS run per-output kernels.
#include <algorithm>

#include "grk_common.h"

namespace grk {
namespace {

constexpr int kMaxDnnBlocks = 16;
constexpr int kMaxDnnMms = 4;

struct DnnCols {
  grk_dnnw_block b[kMaxDnnBlocks];
  grk_dnnw_mm m[kMaxDnnMms];
  int nb, nm;
};

__device__ __forceinline__ float ld_any(const void* p, int64_t i, int dt) {
  return dt == GRK_BF16 ? bf16_to_f32(reinterpret_cast<const bf16_t*>(p)[i]) : reinterpret_cast<const float*>(p)[i];
}

__global__ void __launch_bounds__(256) k_dnnw_fwd(DnnCols cs, const float* __restrict__ bias, int d, int bias_col,
                                                  int width, void* __restrict__ out, int out_dt) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)d * width) return;
  const int i = (int)(e / width), c = (int)(e - (int64_t)i * width);
  float v = 0.f;
  if (c == bias_col) {
    v = bias[i];
    for (int f = 0; f < cs.nm; ++f) {
      const grk_dnnw_mm& m = cs.m[f];
      float acc = 0.f;
      for (int k = 0; k < m.kk; ++k) acc = fmaf(m.wk[(int64_t)i * m.ldk + k], m.bt[k], acc);
      v += acc;
    }
  } else {
    bool done = false;
    for (int j = 0; j < cs.nb && !done; ++j) {
      const grk_dnnw_block& b = cs.b[j];
      if (c >= b.col && c < b.col + b.width) {
        v = ld_any(b.src, (int64_t)i * b.ld + (c - b.col), b.dtype);
        done = true;
      }
    }
    for (int f = 0; f < cs.nm && !done; ++f) {
      const grk_dnnw_mm& m = cs.m[f];
      if (c >= m.col && c < m.col + m.w) {
        const int jj = c - m.col;
        float acc = 0.f;
        for (int k = 0; k < m.kk; ++k) acc = fmaf(m.wk[(int64_t)i * m.ldk + k], m.wt[(int64_t)k * m.ldt + jj], acc);
        v = acc;
        done = true;
      }
    }
  }
  if (out_dt == GRK_BF16) reinterpret_cast<bf16_t*>(out)[e] = f32_to_bf16(v);
  else reinterpret_cast<float*>(out)[e] = v;
}

// g32 (blocks [0, g_blocks)) and dW_k of every mm feature (the following blocks):
// dW_k[i, k] = sum_{j < w} g[i, col + j] Wt[k, j] + g[i, bias_col] bt[k]
struct DnnBwd {
  DnnCols cs;
  int64_t dwk_off[kMaxDnnMms];    // element offset of feature f's dW_k in dwk
  int dwk_blocks[kMaxDnnMms + 1]; // first workgroup of each feature's dW_k
};

__global__ void __launch_bounds__(256) k_dnnw_bwd_a(DnnBwd p, const void* __restrict__ g, int g_dt, int64_t ldg,
                                                    int d, int width, int bias_col, float* __restrict__ g32,
                                                    float* __restrict__ dwk) {
  const int bx = blockIdx.x;
  if (bx < p.dwk_blocks[0]) {
    const int64_t e = (int64_t)bx * blockDim.x + threadIdx.x;
    if (e >= (int64_t)d * width) return;
    const int i = (int)(e / width), c = (int)(e - (int64_t)i * width);
    g32[e] = ld_any(g, (int64_t)i * ldg + c, g_dt);
    return;
  }
  int f = 0;
  while (f + 1 < p.cs.nm && bx >= p.dwk_blocks[f + 1]) ++f;
  const grk_dnnw_mm& m = p.cs.m[f];
  const int64_t e = (int64_t)(bx - p.dwk_blocks[f]) * blockDim.x + threadIdx.x;
  if (e >= (int64_t)d * m.kk) return;
  const int i = (int)(e / m.kk), k = (int)(e - (int64_t)i * m.kk);
  float acc = 0.f;
  for (int j = 0; j < m.w; ++j) acc = fmaf(ld_any(g, (int64_t)i * ldg + m.col + j, g_dt), m.wt[(int64_t)k * m.ldt + j], acc);
  acc = fmaf(ld_any(g, (int64_t)i * ldg + bias_col, g_dt), m.bt[k], acc);
  dwk[p.dwk_off[f] + e] = acc;
}

// [dWt | dbt][k, j] = sum_{i < d} W_k[i, k] dM[i, j], dM[:, j] = g[:, col + j] (j < w),
// g[:, bias_col] (j = w); one thread per (k, j), lanes along k (coalesced W_k rows)
__global__ void __launch_bounds__(256) k_dnnw_bwd_b(DnnBwd p, const void* __restrict__ g, int g_dt, int64_t ldg,
                                                    int d, int bias_col, float* __restrict__ det, int f,
                                                    int64_t det_off) {
  const grk_dnnw_mm& m = p.cs.m[f];
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)m.kk * (m.w + 1)) return;
  const int j = (int)(e / m.kk), k = (int)(e - (int64_t)j * m.kk);
  const int gc = j < m.w ? m.col + j : bias_col;
  float acc = 0.f;
  for (int i = 0; i < d; ++i) acc = fmaf(m.wk[(int64_t)i * m.ldk + k], ld_any(g, (int64_t)i * ldg + gc, g_dt), acc);
  det[det_off + (int64_t)k * (m.w + 1) + j] = acc;
}

// ---- LDS-tiled forms (the default where their LDS fits): the K = kk products read
// [Wt | bt] and the W_k rows / dM columns from LDS instead of serial global loads
// (the per-output kernels above ran ~1000 waves of 512 dependent-latency iterations
// each way: the step 0.3 ms slower than the torch composition).
constexpr int kDnnRows = 8;    // output rows per workgroup (forward, backward rows kernel)
constexpr int kDnnKc = 16;     // W_k columns per workgroup (backward columns kernel)
constexpr size_t kDnnLdsMax = 150 * 1024;

// dst[o] = load(o) for o < n by the workgroup, 8 independent loads in flight per
// thread before their LDS stores (a load-then-store loop waits one memory latency
// per element: the staging then dominated these small kernels)
template <typename F>
__device__ __forceinline__ void stage_lds(float* dst, int n, F load) {
  for (int base = threadIdx.x; base < n; base += 8 * blockDim.x) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int o = base + u * blockDim.x;
      v[u] = o < n ? load(o) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int o = base + u * blockDim.x;
      if (o < n) dst[o] = v[u];
    }
  }
}

// forward: workgroup = kDnnRows rows of the output.  Per mm feature f: W_k rows and
// [Wt | bt] staged, the rows' w + 1 products summed in k order into mmL; then one pass
// writes every column of the rows (blocks copied, mm columns from mmL, the bias column
// bias + sum_f the features' bt products in f order, zeros elsewhere).
__global__ void __launch_bounds__(256) k_dnnw_fwd_t(DnnCols cs, const float* __restrict__ bias, int d, int bias_col,
                                                    int width, void* __restrict__ out, int out_dt, int kkmax,
                                                    int msum) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* mmL = lds;                         // [kDnnRows][msum]
  float* wkL = mmL + kDnnRows * msum;       // [kDnnRows][kk]
  float* etL = wkL + kDnnRows * kkmax;      // [kk][w + 1]
  const int i0 = blockIdx.x * kDnnRows, rows = min(kDnnRows, d - i0), tid = threadIdx.x;
  int moff = 0;
  for (int f = 0; f < cs.nm; ++f) {
    const grk_dnnw_mm& m = cs.m[f];
    const int W1 = m.w + 1;
    __syncthreads();
    stage_lds(wkL, rows * m.kk, [&](int o) {
      const int r = o / m.kk, k = o - r * m.kk;
      return m.wk[(int64_t)(i0 + r) * m.ldk + k];
    });
    stage_lds(etL, m.kk * W1, [&](int o) {
      const int k = o / W1, j = o - k * W1;
      return j < m.w ? m.wt[(int64_t)k * m.ldt + j] : m.bt[k];
    });
    __syncthreads();
    for (int o = tid; o < rows * W1; o += blockDim.x) {
      const int r = o / W1, j = o - r * W1;
      const float* wr = wkL + r * m.kk;
      float acc = 0.f;
#pragma unroll 16   // LDS reads of 16 k in flight ahead of the (k-ordered) FMA chain
      for (int k = 0; k < m.kk; ++k) acc = fmaf(wr[k], etL[k * W1 + j], acc);
      mmL[r * msum + moff + j] = acc;
    }
    moff += W1;
  }
  __syncthreads();
#pragma unroll 4
  for (int o = tid; o < rows * width; o += blockDim.x) {   // unrolled: block loads of 4 columns in flight
    const int r = o / width, c = o - r * width, i = i0 + r;
    float v = 0.f;
    if (c == bias_col) {
      v = bias[i];
      int mo = 0;
      for (int f = 0; f < cs.nm; ++f) {
        v += mmL[r * msum + mo + cs.m[f].w];
        mo += cs.m[f].w + 1;
      }
    } else {
      bool done = false;
      for (int j = 0; j < cs.nb && !done; ++j) {
        const grk_dnnw_block& b = cs.b[j];
        if (c >= b.col && c < b.col + b.width) {
          v = ld_any(b.src, (int64_t)i * b.ld + (c - b.col), b.dtype);
          done = true;
        }
      }
      int mo = 0;
      for (int f = 0; f < cs.nm && !done; ++f) {
        const grk_dnnw_mm& m = cs.m[f];
        if (c >= m.col && c < m.col + m.w) {
          v = mmL[r * msum + mo + (c - m.col)];
          done = true;
        }
        mo += m.w + 1;
      }
    }
    const int64_t e = (int64_t)i * width + c;
    if (out_dt == GRK_BF16) reinterpret_cast<bf16_t*>(out)[e] = f32_to_bf16(v);
    else reinterpret_cast<float*>(out)[e] = v;
  }
}

// backward, rows: workgroup = kDnnRows rows: g32 of the rows, and per feature dM's rows
// and [Wt | bt] staged, dW_k[i, k] = sum_j dM[i, j] [Wt | bt][k, j] in j order
__global__ void __launch_bounds__(256) k_dnnw_bwd_rows(DnnBwd p, const void* __restrict__ g, int g_dt, int64_t ldg,
                                                       int d, int width, int bias_col, float* __restrict__ g32,
                                                       float* __restrict__ dwk, int kkmax) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* dML = lds;                         // [kDnnRows][w + 1]
  float* etL = dML + kDnnRows * 64;         // [kk][w + 1]  (w + 1 <= 64)
  const int i0 = blockIdx.x * kDnnRows, rows = min(kDnnRows, d - i0), tid = threadIdx.x;
  for (int base = tid; base < rows * width; base += 8 * blockDim.x) {   // 8 loads in flight per thread
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int o = base + u * blockDim.x, r = o / width, c = o - r * width;
      v[u] = o < rows * width ? ld_any(g, (int64_t)(i0 + r) * ldg + c, g_dt) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int o = base + u * blockDim.x, r = o / width, c = o - r * width;
      if (o < rows * width) g32[(int64_t)(i0 + r) * width + c] = v[u];
    }
  }
  for (int f = 0; f < p.cs.nm; ++f) {
    const grk_dnnw_mm& m = p.cs.m[f];
    const int W1 = m.w + 1;
    __syncthreads();
    stage_lds(dML, rows * W1, [&](int o) {
      const int r = o / W1, j = o - r * W1;
      return ld_any(g, (int64_t)(i0 + r) * ldg + (j < m.w ? m.col + j : bias_col), g_dt);
    });
    stage_lds(etL, m.kk * W1, [&](int o) {
      const int k = o / W1, j = o - k * W1;
      return j < m.w ? m.wt[(int64_t)k * m.ldt + j] : m.bt[k];
    });
    __syncthreads();
    for (int o = tid; o < rows * m.kk; o += blockDim.x) {
      const int r = o / m.kk, k = o - r * m.kk;
      const float* dr = dML + r * W1;
      const float* er = etL + k * W1;
      float acc = 0.f;
#pragma unroll 16
      for (int j = 0; j < W1; ++j) acc = fmaf(dr[j], er[j], acc);
      dwk[p.dwk_off[f] + (int64_t)(i0 + r) * m.kk + k] = acc;
    }
  }
}

// backward, columns of feature f: workgroup = kDnnKc columns of W_k, with those columns
// and all of dM staged: [dWt | dbt][k, j] = sum_i W_k[i, k] dM[i, j] in i order
__global__ void __launch_bounds__(256) k_dnnw_bwd_cols(DnnBwd p, const void* __restrict__ g, int g_dt, int64_t ldg,
                                                       int d, int bias_col, float* __restrict__ det, int f,
                                                       int64_t det_off) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const grk_dnnw_mm& m = p.cs.m[f];
  const int W1 = m.w + 1, k0 = blockIdx.x * kDnnKc, kc_n = min(kDnnKc, m.kk - k0), tid = threadIdx.x;
  float* wkL = lds;                         // [d][kDnnKc]
  float* dML = wkL + (int64_t)d * kDnnKc;   // [d][w + 1]
  stage_lds(wkL, d * kDnnKc, [&](int o) {
    const int i = o / kDnnKc, kc = o - i * kDnnKc;
    return kc < kc_n ? m.wk[(int64_t)i * m.ldk + k0 + kc] : 0.f;
  });
  stage_lds(dML, d * W1, [&](int o) {
    const int i = o / W1, j = o - i * W1;
    return ld_any(g, (int64_t)i * ldg + (j < m.w ? m.col + j : bias_col), g_dt);
  });
  __syncthreads();
  for (int o = tid; o < kc_n * W1; o += blockDim.x) {
    const int kc = o / W1, j = o - kc * W1;
    float acc = 0.f;
#pragma unroll 16
    for (int i = 0; i < d; ++i) acc = fmaf(wkL[i * kDnnKc + kc], dML[i * W1 + j], acc);
    det[det_off + (int64_t)(k0 + kc) * W1 + j] = acc;
  }
}

int dnn_cols(DnnCols& cs, const grk_dnnw_block* blocks, int nblocks, const grk_dnnw_mm* mms, int nmm, int d,
             int width, int bias_col) {
  GRK_CHECK_ARG(nblocks >= 0 && nblocks <= kMaxDnnBlocks, "at most %d blocks", kMaxDnnBlocks);
  GRK_CHECK_ARG(nmm >= 0 && nmm <= kMaxDnnMms, "at most %d mm features", kMaxDnnMms);
  GRK_CHECK_ARG(d > 0 && width > 0 && bias_col >= 0 && bias_col < width, "bad d / width / bias_col");
  GRK_CHECK_ARG((int64_t)d * width < ((int64_t)1 << 31), "weight too large");
  memset(&cs, 0, sizeof(cs));
  cs.nb = nblocks;
  cs.nm = nmm;
  for (int j = 0; j < nblocks; ++j) {
    const grk_dnnw_block& b = blocks[j];
    GRK_CHECK_ARG(b.src && (b.dtype == GRK_F32 || b.dtype == GRK_BF16), "block %d: src and an fp32 / bf16 dtype", j);
    GRK_CHECK_ARG(b.width > 0 && b.col >= 0 && b.col + b.width <= width && b.ld >= b.width, "block %d: bad columns",
                  j);
    GRK_CHECK_ARG(bias_col < b.col || bias_col >= b.col + b.width, "block %d covers the bias column", j);
    cs.b[j] = b;
  }
  for (int f = 0; f < nmm; ++f) {
    const grk_dnnw_mm& m = mms[f];
    GRK_CHECK_ARG(m.wk && m.wt && m.bt, "mm %d: wk / wt / bt required", f);
    GRK_CHECK_ARG(m.kk > 0 && m.w > 0 && m.col >= 0 && m.col + m.w <= width && m.ldk >= m.kk && m.ldt >= m.w,
                  "mm %d: bad shape", f);
    GRK_CHECK_ARG(bias_col < m.col || bias_col >= m.col + m.w, "mm %d covers the bias column", f);
    cs.m[f] = m;
  }
  return GRK_OK;
}

}  // namespace
}  // namespace grk

using namespace grk;

extern "C" int grk_dnn_weight_fwd(const grk_dnnw_block* blocks, int nblocks, const grk_dnnw_mm* mms, int nmm,
                                  const float* bias, int d, int width, int bias_col, void* out, int out_dtype,
                                  void* stream) {
  clear_error();
  DnnCols cs;
  const int rc = dnn_cols(cs, blocks, nblocks, mms, nmm, d, width, bias_col);
  if (rc) return rc;
  GRK_CHECK_ARG(bias && out && (out_dtype == GRK_F32 || out_dtype == GRK_BF16), "bias, out (fp32 / bf16) required");
  const int64_t n = (int64_t)d * width;
  int kkmax = 0, wmax = 0, msum = 0;
  for (int f = 0; f < nmm; ++f) {
    kkmax = std::max(kkmax, mms[f].kk);
    wmax = std::max(wmax, mms[f].w);
    msum += mms[f].w + 1;
  }
  const size_t lds = ((size_t)kDnnRows * msum + (size_t)kDnnRows * kkmax + (size_t)kkmax * (wmax + 1)) * 4;
  if (lds <= kDnnLdsMax) {
    if (lds > 64 * 1024) GRK_CHECK_HIP(ensure_dynamic_lds((const void*)k_dnnw_fwd_t, lds));
    k_dnnw_fwd_t<<<(unsigned)((d + kDnnRows - 1) / kDnnRows), 256, lds, (hipStream_t)stream>>>(
        cs, bias, d, bias_col, width, out, out_dtype, kkmax, msum);
  } else {
    k_dnnw_fwd<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(cs, bias, d, bias_col, width, out,
                                                                              out_dtype);
  }
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

extern "C" int grk_dnn_weight_bwd(const void* g, int g_dtype, int64_t ldg, const grk_dnnw_mm* mms, int nmm, int d,
                                  int width, int bias_col, float* g32, float* dwk, float* det, void* stream) {
  clear_error();
  DnnBwd p;
  memset(&p, 0, sizeof(p));
  const int rc = dnn_cols(p.cs, nullptr, 0, mms, nmm, d, width, bias_col);
  if (rc) return rc;
  GRK_CHECK_ARG(g && g32 && (g_dtype == GRK_F32 || g_dtype == GRK_BF16) && ldg >= width, "g (fp32 / bf16), g32 required");
  GRK_CHECK_ARG(nmm == 0 || (dwk && det), "dwk / det required with mm features");
  hipStream_t s = (hipStream_t)stream;
  const int64_t n = (int64_t)d * width;
  int blocks = (int)((n + 255) / 256);
  int64_t off = 0;
  for (int f = 0; f < nmm; ++f) {
    p.dwk_blocks[f] = blocks;
    p.dwk_off[f] = off;
    const int64_t e = (int64_t)d * mms[f].kk;
    blocks += (int)((e + 255) / 256);
    off += e;
  }
  p.dwk_blocks[nmm] = blocks;
  if (nmm == 0) p.dwk_blocks[0] = blocks;
  int kkmax = 0, wmax = 0;
  for (int f = 0; f < nmm; ++f) {
    kkmax = std::max(kkmax, mms[f].kk);
    wmax = std::max(wmax, mms[f].w);
  }
  const size_t lds_rows = ((size_t)kDnnRows * 64 + (size_t)kkmax * (wmax + 1)) * 4;
  const size_t lds_cols = ((size_t)d * kDnnKc + (size_t)d * (wmax + 1)) * 4;
  const bool tiled = wmax + 1 <= 64 && lds_rows <= kDnnLdsMax && lds_cols <= kDnnLdsMax;
  if (tiled) {
    if (lds_rows > 64 * 1024) GRK_CHECK_HIP(ensure_dynamic_lds((const void*)k_dnnw_bwd_rows, lds_rows));
    k_dnnw_bwd_rows<<<(unsigned)((d + kDnnRows - 1) / kDnnRows), 256, lds_rows, s>>>(p, g, g_dtype, ldg, d, width,
                                                                                     bias_col, g32, dwk, kkmax);
  } else {
    k_dnnw_bwd_a<<<(unsigned)blocks, 256, 0, s>>>(p, g, g_dtype, ldg, d, width, bias_col, g32, dwk);
  }
  GRK_LAUNCH_CHECK();
  if (tiled && lds_cols > 64 * 1024) GRK_CHECK_HIP(ensure_dynamic_lds((const void*)k_dnnw_bwd_cols, lds_cols));
  int64_t doff = 0;
  for (int f = 0; f < nmm; ++f) {
    const int64_t e = (int64_t)mms[f].kk * (mms[f].w + 1);
    if (tiled)
      k_dnnw_bwd_cols<<<(unsigned)((mms[f].kk + kDnnKc - 1) / kDnnKc), 256, lds_cols, s>>>(p, g, g_dtype, ldg, d,
                                                                                            bias_col, det, f, doff);
    else
      k_dnnw_bwd_b<<<(unsigned)((e + 255) / 256), 256, 0, s>>>(p, g, g_dtype, ldg, d, bias_col, det, f, doff);
    GRK_LAUNCH_CHECK();
    doff += e;
  }
  return GRK_OK;
}
