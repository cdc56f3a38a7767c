// Validate every hipBLASLt heuristic candidate grk_gemm may pick for a shape:
// for each candidate, run it, run a DIFFERENT GEMM that shares the workspace,
// run it again, and compare both results against a naive fp32 reference and
// against each other.  Found (round 2): some candidates (e.g. the
// "Custom_..._UserArgs" kernels) are right on their first call and wrong on
// later ones once another GEMM has used the workspace.
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 -x hip -o build/gemm_validate \
//     scripts/microbench/gemm_validate.hip -lhipblaslt && build/gemm_validate
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt-ext.hpp>
#include <hipblaslt/hipblaslt.h>

#include <cmath>
#include <cstdio>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
#define CB(x) do { hipblasStatus_t s = (x); if (s != HIPBLAS_STATUS_SUCCESS) { printf("%s: %d\n", #x, (int)s); exit(1); } } while (0)

typedef __hip_bfloat16 bf16;

// y[m, n] = sum_k x[m, k] w[n, k] (row-major), fp32
__global__ void k_ref(const bf16* x, const bf16* w, float* y, int M, int N, int K) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * N) return;
  const int m = i / N, n = i % N;
  float acc = 0.f;
  for (int k = 0; k < K; ++k) acc += (float)x[(size_t)m * K + k] * (float)w[(size_t)n * K + k];
  y[i] = acc;
}

__global__ void k_fill(bf16* p, size_t n, unsigned seed) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned x = (unsigned)i * 2654435761u ^ seed;
  x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
  p[i] = (bf16)(((int)(x & 0xFFFF) - 32768) / 32768.0f);
}

struct Gemm {  // row-major y[M, N] = x[M, K] w[N, K]^T as grk_gemm issues it (col-major C'[N, M])
  int64_t M, N, K;
  hipblasLtMatmulDesc_t op;
  hipblasLtMatrixLayout_t A, B, C;
  bf16 *x, *w, *y;
  void init(int64_t m, int64_t n, int64_t k, unsigned seed) {
    M = m; N = n; K = k;
    CB(hipblasLtMatmulDescCreate(&op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
    hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
    CB(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
    CB(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
    CB(hipblasLtMatrixLayoutCreate(&A, HIP_R_16BF, K, N, K));
    CB(hipblasLtMatrixLayoutCreate(&B, HIP_R_16BF, K, M, K));
    CB(hipblasLtMatrixLayoutCreate(&C, HIP_R_16BF, N, M, N));
    CK(hipMalloc(&x, M * K * 2)); CK(hipMalloc(&w, N * K * 2)); CK(hipMalloc(&y, M * N * 2));
    k_fill<<<(M * K + 255) / 256, 256>>>(x, M * K, seed);
    k_fill<<<(N * K + 255) / 256, 256>>>(w, N * K, seed * 7 + 1);
  }
  bool run(hipblasLtHandle_t h, const hipblasLtMatmulAlgo_t* algo, void* ws, size_t wsb, bf16* out) {
    float alpha = 1.f, beta = 0.f;
    return hipblasLtMatmul(h, op, &alpha, w, A, x, B, &beta, out, C, out, C, algo, ws, wsb, 0) ==
           HIPBLAS_STATUS_SUCCESS;
  }
};

static double rel_err(const std::vector<bf16>& got, const std::vector<float>& ref) {
  double num = 0, den = 0;
  for (size_t i = 0; i < ref.size(); ++i) {
    const double d = (double)(float)got[i] - ref[i];
    num += d * d;
    den += (double)ref[i] * ref[i];
  }
  return std::sqrt(num / (den > 0 ? den : 1));
}

int main(int argc, char** argv) {
  hipblasLtHandle_t h;
  CB(hipblasLtCreate(&h));
  const size_t wsb = 256ull << 20;
  void* ws;
  CK(hipMalloc(&ws, wsb));
  Gemm other;
  other.init(248, 64, 256, 99);
  std::vector<hipblasLtMatmulHeuristicResult_t> ores(256);
  int n_other = 0;
  {
    hipblasLtMatmulPreference_t pref;
    CB(hipblasLtMatmulPreferenceCreate(&pref));
    uint64_t wmax = wsb;
    CB(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wmax, sizeof(wmax)));
    CB(hipblasLtMatmulAlgoGetHeuristic(h, other.op, other.A, other.B, other.C, other.C, pref, 256, ores.data(),
                                       &n_other));
  }
  const int64_t shapes[][3] = {{248, 512, 64}, {25728, 2048, 512}};
  for (auto& s : shapes) {
    Gemm g;
    g.init(s[0], s[1], s[2], 5);
    float* yref;
    CK(hipMalloc(&yref, g.M * g.N * 4));
    k_ref<<<(g.M * g.N + 255) / 256, 256>>>(g.x, g.w, yref, g.M, g.N, g.K);
    std::vector<float> ref(g.M * g.N);
    CK(hipMemcpy(ref.data(), yref, ref.size() * 4, hipMemcpyDeviceToHost));
    hipblasLtMatmulPreference_t pref;
    CB(hipblasLtMatmulPreferenceCreate(&pref));
    uint64_t wmax = wsb;
    CB(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wmax, sizeof(wmax)));
    std::vector<hipblasLtMatmulHeuristicResult_t> res(256);
    int n = 0;
    CB(hipblasLtMatmulAlgoGetHeuristic(h, g.op, g.A, g.B, g.C, g.C, pref, 256, res.data(), &n));
    int bad = 0;
    bf16 *o1, *o2;
    CK(hipMalloc(&o1, g.M * g.N * 2)); CK(hipMalloc(&o2, g.M * g.N * 2));
    std::vector<bf16> h1(g.M * g.N), h2(g.M * g.N);
    for (int i = 0; i < n; ++i) {
      CK(hipMemset(o1, 0, g.M * g.N * 2)); CK(hipMemset(o2, 0, g.M * g.N * 2));
      if (!g.run(h, &res[i].algo, ws, wsb, o1)) continue;
      // every candidate of another shape on the same workspace (what grk_gemm's timing of a new shape does)
      for (int j = 0; j < n_other; ++j) other.run(h, &ores[j].algo, ws, wsb, other.y);
      if (!g.run(h, &res[i].algo, ws, wsb, o2)) continue;
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(h1.data(), o1, h1.size() * 2, hipMemcpyDeviceToHost));
      CK(hipMemcpy(h2.data(), o2, h2.size() * 2, hipMemcpyDeviceToHost));
      const double e1 = rel_err(h1, ref), e2 = rel_err(h2, ref);
      const bool same = memcmp(h1.data(), h2.data(), h1.size() * 2) == 0;
      if (e1 > 1e-2 || e2 > 1e-2 || !same) {
        ++bad;
        printf("  M=%lld N=%lld K=%lld cand %3d ws=%zu: first err %.2e, second err %.2e, repeat-equal %d: %s\n",
               (long long)g.M, (long long)g.N, (long long)g.K, i, (size_t)res[i].workspaceSize, e1, e2, (int)same,
               hipblaslt_ext::getKernelNameFromAlgo(h, res[i].algo).substr(0, 90).c_str());
      }
    }
    printf("M=%lld N=%lld K=%lld: %d candidates, %d bad\n", (long long)g.M, (long long)g.N, (long long)g.K, n, bad);
    fflush(stdout);
  }
  return 0;
}
