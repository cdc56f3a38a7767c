// In-batch sampled softmax for gfx950 (north star, no
// reference implementation -- oracle/loss.py::sampled_softmax).
//
//   z_ij = <h_i, e_j> / tau over valid columns j, with j != i masked when
//          item_id[j] == item_id[i] (the same item is not its own negative);
//   loss = mean over valid rows of (logsumexp_j z_ij - z_ii).
//
// Forward: flash-style online logsumexp, never materialising the M x M logits.
// A workgroup = 4 waves x 32 rows; the row block's H fragments stay in
// registers, candidate tiles of 32 rows of E are staged through LDS
// (swizzled row image), S^T = E H^T on MFMA 32x32x16 bf16 so a lane owns one
// row i.  The columns are split into slices over workgroups (row blocks alone
// would leave most CUs idle); a combine kernel merges the slices' (max, sum)
// and reduces the loss in a fixed order.
// Backward: a second pass recomputes the tiles and writes
//   G_ij = (softmax_ij - [i == j]) * grad_loss / (count * tau)   (bf16)
// so that dH = G E and dE = G^T H are two plain GEMMs (hipBLASLt).
#include "grk_common.h"
#include "grk_mfma.h"

namespace grk {

constexpr int kSSRows = 128;  // rows per workgroup (4 waves x 32)

struct SSParams {
  const bf16_t* h; int64_t ldh;
  const bf16_t* e; int64_t lde;
  const int64_t* ids;
  const uint8_t* valid;
  int M;
  float sl2;            // log2(e) / tau
  int slice_cols;       // columns per slice (multiple of 32)
  float *pm, *pl;       // [nslices, M] partial max / sum (log2 domain)
  float* diag;          // [M] z_ii in log2 units
  float* lse2;          // [M] log2-domain logsumexp
  float* partials;      // [nblocks * 2]
  float* loss; int32_t* count;
  const float* grad_loss;
  bf16_t* G; int64_t ldg;
  int col_tiles;        // tiles per workgroup in the gradient kernel
};

template <int D>
__device__ __forceinline__ void ss_stage(char* Es, int64_t* cid, uint8_t* cval, const SSParams& p, int jb) {
  constexpr int NCH = D / 8;
  for (int u = threadIdx.x; u < 32 * NCH; u += blockDim.x) {
    const int row = u / NCH, c = u % NCH;
    const int j = jb + row;
    const bool ok = j < p.M;
    uint4 v = ok ? *reinterpret_cast<const uint4*>(p.e + (int64_t)j * p.lde + c * 8) : make_uint4(0, 0, 0, 0);
    *reinterpret_cast<uint4*>(Es + lds_off<D>(row, c * 8)) = v;
  }
  if (threadIdx.x < 32) {
    const int j = jb + threadIdx.x;
    const bool ok = j < p.M;
    cid[threadIdx.x] = ok ? p.ids[j] : -1;
    cval[threadIdx.x] = ok ? p.valid[j] : 0;
  }
}

template <int D>
__device__ __forceinline__ f32x16 ss_tile(const char* Es, const bf16x8* hf, int r, int hh) {
  constexpr int KS = D / 16;
  f32x16 s = f32x16{};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) s = mfma(lds_row8<D>(Es, r, 16 * ks + 8 * hh), hf[ks], s);
  return s;
}

template <int D>
__global__ void __launch_bounds__(256) k_ss_fwd(SSParams p) {
  constexpr int KS = D / 16;
  __shared__ __attribute__((aligned(16))) char smem[32 * D * 2 + 32 * 8 + 32];
  char* Es = smem;
  int64_t* cid = reinterpret_cast<int64_t*>(smem + 32 * D * 2);
  uint8_t* cval = reinterpret_cast<uint8_t*>(smem + 32 * D * 2 + 32 * 8);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int i = blockIdx.x * kSSRows + wave * 32 + r;
  const bool iok = i < p.M && p.valid[i];
  const bool wave_live = __ballot(iok) != 0;
  const int64_t myid = iok ? p.ids[i] : -2;
  bf16x8 hf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) hf[ks] = gload8(p.h + (int64_t)(iok ? i : 0) * p.ldh + 16 * ks + 8 * hh, iok);
  float m = -INFINITY, l = 0.f;
  const int c0 = blockIdx.y * p.slice_cols;
  const int c1 = min(p.M, c0 + p.slice_cols);
  for (int jb = c0; jb < c1; jb += 32) {
    __syncthreads();
    ss_stage<D>(Es, cid, cval, p, jb);
    __syncthreads();
    if (!wave_live) continue;
    f32x16 s = ss_tile<D>(Es, hf, r, hh);
    float x[16], tmax = -INFINITY;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int jr = acc_row(k, hh), j = jb + jr;
      const bool ok = iok && cval[jr] && (j == i || cid[jr] != myid);
      x[k] = ok ? s[k] * p.sl2 : -INFINITY;
      if (j == i && iok) p.diag[i] = s[k] * p.sl2;
      tmax = fmaxf(tmax, x[k]);
    }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
    const float mn = fmaxf(m, tmax);
    float rs = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) rs += (x[k] == -INFINITY) ? 0.f : exp2f(x[k] - mn);
    rs += __shfl_xor(rs, 32);
    l = (mn == -INFINITY) ? 0.f : l * exp2f(m - mn) + rs;
    m = mn;
  }
  if (hh == 0 && i < p.M) {
    p.pm[(int64_t)blockIdx.y * p.M + i] = m;
    p.pl[(int64_t)blockIdx.y * p.M + i] = l;
  }
}

// Merge slices -> lse2[i]; per-block (loss, count) partials in fixed order.
__global__ void __launch_bounds__(256) k_ss_combine(SSParams p, int nslices) {
  __shared__ float red[2][256];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float li = 0.f, ci = 0.f;
  if (i < p.M && p.valid[i]) {
    float mx = -INFINITY;
    for (int s = 0; s < nslices; ++s) mx = fmaxf(mx, p.pm[(int64_t)s * p.M + i]);
    float sum = 0.f;
    for (int s = 0; s < nslices; ++s) {
      const float ms = p.pm[(int64_t)s * p.M + i];
      if (ms != -INFINITY) sum += p.pl[(int64_t)s * p.M + i] * exp2f(ms - mx);
    }
    const float l2 = mx + log2f(sum);
    p.lse2[i] = l2;
    li = (l2 - p.diag[i]) * kLn2;
    ci = 1.f;
  } else if (i < p.M) {
    p.lse2[i] = -INFINITY;
  }
  red[0][threadIdx.x] = li;
  red[1][threadIdx.x] = ci;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      red[0][threadIdx.x] += red[0][threadIdx.x + s];
      red[1][threadIdx.x] += red[1][threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    p.partials[2 * blockIdx.x] = red[0][0];
    p.partials[2 * blockIdx.x + 1] = red[1][0];
  }
}

__global__ void __launch_bounds__(1024) k_ss_finalize(SSParams p, int nblocks) {
  __shared__ double red[2][1024];
  double a = 0.0, c = 0.0;
  for (int b = threadIdx.x; b < nblocks; b += blockDim.x) {
    a += p.partials[2 * b];
    c += p.partials[2 * b + 1];
  }
  red[0][threadIdx.x] = a;
  red[1][threadIdx.x] = c;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      red[0][threadIdx.x] += red[0][threadIdx.x + s];
      red[1][threadIdx.x] += red[1][threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double cnt = red[1][0];
    p.loss[0] = (float)(red[0][0] / (cnt > 0 ? cnt : 1.0));
    p.count[0] = (int32_t)cnt;
  }
}

// G tile writer: every (i, j) in [0, M)^2 is written (zeros where masked).
template <int D>
__global__ void __launch_bounds__(256) k_ss_grad(SSParams p) {
  constexpr int KS = D / 16;
  __shared__ __attribute__((aligned(16))) char smem[32 * D * 2 + 32 * 8 + 32];
  char* Es = smem;
  int64_t* cid = reinterpret_cast<int64_t*>(smem + 32 * D * 2);
  uint8_t* cval = reinterpret_cast<uint8_t*>(smem + 32 * D * 2 + 32 * 8);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int i = blockIdx.x * kSSRows + wave * 32 + r;
  const bool irow = i < p.M;
  const bool iok = irow && p.valid[i];
  const bool wave_live = __ballot(iok) != 0;
  const int64_t myid = iok ? p.ids[i] : -2;
  const float l2 = iok ? p.lse2[i] : 0.f;
  const float coef = (p.grad_loss ? *p.grad_loss : 1.f) / (float)max(*p.count, 1) * (p.sl2 / kLog2e);
  bf16x8 hf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) hf[ks] = gload8(p.h + (int64_t)(iok ? i : 0) * p.ldh + 16 * ks + 8 * hh, iok);
  const int jb0 = blockIdx.y * p.col_tiles * 32;
  for (int t = 0; t < p.col_tiles; ++t) {
    const int jb = jb0 + 32 * t;
    if (jb >= p.M) break;
    __syncthreads();
    ss_stage<D>(Es, cid, cval, p, jb);
    __syncthreads();
    f32x16 s = f32x16{};
    if (wave_live) s = ss_tile<D>(Es, hf, r, hh);
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k = 4 * g4 + q;
        const int jr = acc_row(k, hh), j = jb + jr;
        const bool ok = iok && j < p.M && cval[jr] && (j == i || cid[jr] != myid);
        const float pr = ok ? exp2f(s[k] * p.sl2 - l2) : 0.f;
        v[q] = ok ? (pr - (j == i ? 1.f : 0.f)) * coef : 0.f;
      }
      const int j0 = jb + 8 * g4 + 4 * hh;
      if (!irow) continue;
      bf16_t* dst = p.G + (int64_t)i * p.ldg + j0;
      if (j0 + 3 < p.M) {
        uint2 w;
        w.x = (unsigned)f32_to_bf16(v[0]) | ((unsigned)f32_to_bf16(v[1]) << 16);
        w.y = (unsigned)f32_to_bf16(v[2]) | ((unsigned)f32_to_bf16(v[3]) << 16);
        *reinterpret_cast<uint2*>(dst) = w;
      } else {
        for (int q = 0; q < 4; ++q)
          if (j0 + q < p.M) dst[q] = f32_to_bf16(v[q]);
      }
    }
  }
}

template <int D>
static int ss_launch(const SSParams& p, int which, int nslices, hipStream_t s) {
  const unsigned rb = (unsigned)((p.M + kSSRows - 1) / kSSRows);
  if (which == 0) {
    k_ss_fwd<D><<<dim3(rb, nslices), 256, 0, s>>>(p);
  } else {
    const int tiles = (p.M + 31) / 32;
    k_ss_grad<D><<<dim3(rb, (tiles + p.col_tiles - 1) / p.col_tiles), 256, 0, s>>>(p);
  }
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

static int ss_dispatch(const SSParams& p, int dim, int which, int nslices, hipStream_t s) {
  switch (dim) {
    case 32: return ss_launch<32>(p, which, nslices, s);
    case 64: return ss_launch<64>(p, which, nslices, s);
    case 128: return ss_launch<128>(p, which, nslices, s);
    case 256: return ss_launch<256>(p, which, nslices, s);
    case 512: return ss_launch<512>(p, which, nslices, s);
  }
  set_error("dim %d unsupported (32, 64, 128, 256, 512)", dim);
  return GRK_EUNSUPPORTED;
}

static int ss_slices(int M) {
  // enough workgroups to cover the chip: row blocks x slices >= ~2 per CU
  const int rb = (M + kSSRows - 1) / kSSRows;
  int ns = (512 + rb - 1) / rb;
  const int tiles = (M + 31) / 32;
  if (ns > tiles) ns = tiles;
  return ns < 1 ? 1 : ns;
}

}  // namespace grk

using namespace grk;

extern "C" size_t grk_sampled_softmax_workspace(int64_t num_rows) {
  const int M = (int)num_rows;
  const int ns = ss_slices(M);
  const int nb = (M + 255) / 256;
  return ((size_t)2 * ns * M + 2 * (size_t)M + 2 * (size_t)nb + 64) * sizeof(float);
}

static int ss_fill(const void* h, int64_t ldh, const void* e, int64_t lde, const int64_t* ids, const uint8_t* valid,
                   int64_t num_rows, int dim, float tau, SSParams* p) {
  GRK_CHECK_ARG(h && e && ids && valid, "h, e, item_ids and valid are required");
  GRK_CHECK_ARG(num_rows > 0 && num_rows < (1LL << 30), "num_rows out of range");
  GRK_CHECK_ARG(dim == 32 || dim == 64 || dim == 128 || dim == 256 || dim == 512, "dim %d unsupported", dim);
  GRK_CHECK_ARG(ldh >= dim && lde >= dim && ldh % 8 == 0 && lde % 8 == 0, "row strides must be >= dim, multiple of 8");
  GRK_CHECK_ARG(((uintptr_t)h | (uintptr_t)e) % 16 == 0, "h / e must be 16-byte aligned");
  GRK_CHECK_ARG(tau > 0.f, "temperature must be > 0");
  memset(p, 0, sizeof(*p));
  p->h = (const bf16_t*)h; p->ldh = ldh; p->e = (const bf16_t*)e; p->lde = lde;
  p->ids = ids; p->valid = valid; p->M = (int)num_rows; p->sl2 = kLog2e / tau;
  return GRK_OK;
}

extern "C" int grk_sampled_softmax_fwd(const void* h, int64_t ldh, const void* e, int64_t lde, const int64_t* item_ids,
                                       const uint8_t* valid, int64_t num_rows, int dim, float tau, float* lse2,
                                       float* loss, int32_t* count, void* workspace, size_t workspace_bytes,
                                       void* stream) {
  clear_error();
  SSParams p;
  int rc = ss_fill(h, ldh, e, lde, item_ids, valid, num_rows, dim, tau, &p);
  if (rc) return rc;
  GRK_CHECK_ARG(lse2 && loss && count && workspace, "lse2, loss, count and workspace are required");
  GRK_CHECK_ARG(workspace_bytes >= grk_sampled_softmax_workspace(num_rows), "workspace too small");
  const int M = p.M;
  const int ns = ss_slices(M);
  const int nb = (M + 255) / 256;
  float* ws = (float*)workspace;
  p.pm = ws; p.pl = ws + (size_t)ns * M; p.diag = ws + (size_t)2 * ns * M;
  p.partials = p.diag + M;
  p.lse2 = lse2; p.loss = loss; p.count = count;
  const int tiles = (M + 31) / 32;
  p.slice_cols = ((tiles + ns - 1) / ns) * 32;
  hipStream_t s = (hipStream_t)stream;
  rc = ss_dispatch(p, dim, 0, ns, s);
  if (rc) return rc;
  k_ss_combine<<<nb, 256, 0, s>>>(p, ns);
  GRK_LAUNCH_CHECK();
  k_ss_finalize<<<1, 1024, 0, s>>>(p, nb);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

extern "C" int grk_sampled_softmax_grad(const void* h, int64_t ldh, const void* e, int64_t lde,
                                        const int64_t* item_ids, const uint8_t* valid, int64_t num_rows, int dim,
                                        float tau, const float* lse2, const int32_t* count, const float* grad_loss,
                                        void* G, int64_t ldg, void* stream) {
  clear_error();
  SSParams p;
  int rc = ss_fill(h, ldh, e, lde, item_ids, valid, num_rows, dim, tau, &p);
  if (rc) return rc;
  GRK_CHECK_ARG(lse2 && count && G, "lse2, count and G are required");
  GRK_CHECK_ARG(ldg >= num_rows && ldg % 4 == 0, "ldg must be >= num_rows and a multiple of 4");
  p.lse2 = const_cast<float*>(lse2); p.count = const_cast<int32_t*>(count); p.grad_loss = grad_loss;
  p.G = (bf16_t*)G; p.ldg = ldg; p.col_tiles = 8;
  return ss_dispatch(p, dim, 1, 0, (hipStream_t)stream);
}
