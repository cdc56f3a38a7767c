// Exhaustive hipBLASLt algorithm timing for the bench step's GEMM shapes
// (bf16 inputs, fp32 compute), against the heuristic's first choice (what
// torch runs).  Column-major problem: C[m,n] = op(A)[m,k] op(B)[k,n].
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 -o build/hipblaslt_search \
//     scripts/microbench/hipblaslt_search.cpp -lhipblaslt && build/hipblaslt_search
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt-ext.hpp>
#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <cstdio>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
#define CB(x) do { hipblasStatus_t s = (x); if (s != HIPBLAS_STATUS_SUCCESS) { printf("%s: %d\n", #x, (int)s); exit(1); } } while (0)

struct Prob {
  const char* name;
  hipblasOperation_t opA, opB;
  int64_t m, n, k, lda, ldb, ldc;
  hipDataType tD;
};

static float time_algo(hipblasLtHandle_t h, hipblasLtMatmulDesc_t op, hipblasLtMatrixLayout_t A, hipblasLtMatrixLayout_t B,
                       hipblasLtMatrixLayout_t C, hipblasLtMatmulAlgo_t* algo, void* a, void* b, void* c, void* ws,
                       size_t wsb, hipStream_t s, int reps) {
  float alpha = 1.f, beta = 0.f;
  for (int i = 0; i < 2; ++i)
    if (hipblasLtMatmul(h, op, &alpha, a, A, b, B, &beta, c, C, c, C, algo, ws, wsb, s) != HIPBLAS_STATUS_SUCCESS)
      return -1.f;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < reps; ++i) hipblasLtMatmul(h, op, &alpha, a, A, b, B, &beta, c, C, c, C, algo, ws, wsb, s);
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
  return ms * 1e3f / reps;
}

int main() {
  const int64_t M = 128 * 201, M2 = 2 * M, d = 512;
  const Prob probs[] = {
      // dW[N,K] = gy^T x  ->  col-major C[K,N] = x_cm[K,M] (N) * gy_cm[N,M]^T (T)
      {"uvqk dW  (K=512,N=2048,red M)", HIPBLAS_OP_N, HIPBLAS_OP_T, d, 4 * d, M, d, 4 * d, d, HIP_R_16BF},
      {"uvqk dW fp32 out", HIPBLAS_OP_N, HIPBLAS_OP_T, d, 4 * d, M, d, 4 * d, d, HIP_R_32F},
      {"out_linear dW (512x512, red M)", HIPBLAS_OP_N, HIPBLAS_OP_T, d, d, M, d, d, d, HIP_R_16BF},
      {"out_linear dW fp32 out", HIPBLAS_OP_N, HIPBLAS_OP_T, d, d, M, d, d, d, HIP_R_32F},
      {"itemdnn dW (552x512, red 2M)", HIPBLAS_OP_N, HIPBLAS_OP_T, d + 40, d, M2, d + 40, d, d + 40, HIP_R_16BF},
      // fwd y[M,N] = x W^T -> col-major C[N,M] = W_cm[K,N]^T (T) * x_cm[K,M] (N)
      {"uvqk fwd (N=2048,K=512)", HIPBLAS_OP_T, HIPBLAS_OP_N, 4 * d, M, d, d, d, 4 * d, HIP_R_16BF},
      {"out_linear fwd", HIPBLAS_OP_T, HIPBLAS_OP_N, d, M, d, d, d, d, HIP_R_16BF},
      // dX[M,K] = gy W -> col-major C[K,M] = W_cm[K,N] (N) * gy_cm[N,M] (N)
      {"uvqk dX (K=512, red N=2048)", HIPBLAS_OP_N, HIPBLAS_OP_N, d, M, 4 * d, d, 4 * d, d, HIP_R_16BF},
      {"itemdnn dX (2M rows)", HIPBLAS_OP_N, HIPBLAS_OP_N, d + 40, M2, d, d + 40, d, d + 40, HIP_R_16BF},
  };
  hipblasLtHandle_t h;
  CB(hipblasLtCreate(&h));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const size_t wsb = 128ull << 20;
  void *a, *b, *c, *ws;
  CK(hipMalloc(&a, 256ull << 20)); CK(hipMalloc(&b, 256ull << 20)); CK(hipMalloc(&c, 256ull << 20));
  CK(hipMalloc(&ws, wsb));
  CK(hipMemset(a, 0x3c, 256ull << 20)); CK(hipMemset(b, 0x3c, 256ull << 20));
  for (const Prob& p : probs) {
    hipblasLtMatmulDesc_t op;
    CB(hipblasLtMatmulDescCreate(&op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
    CB(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_TRANSA, &p.opA, sizeof(p.opA)));
    CB(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_TRANSB, &p.opB, sizeof(p.opB)));
    hipblasLtMatrixLayout_t A, B, C;
    const int64_t ar = p.opA == HIPBLAS_OP_N ? p.m : p.k, ac = p.opA == HIPBLAS_OP_N ? p.k : p.m;
    const int64_t br = p.opB == HIPBLAS_OP_N ? p.k : p.n, bc = p.opB == HIPBLAS_OP_N ? p.n : p.k;
    CB(hipblasLtMatrixLayoutCreate(&A, HIP_R_16BF, ar, ac, p.lda));
    CB(hipblasLtMatrixLayoutCreate(&B, HIP_R_16BF, br, bc, p.ldb));
    CB(hipblasLtMatrixLayoutCreate(&C, p.tD, p.m, p.n, p.ldc));
    hipblasLtMatmulPreference_t pref;
    CB(hipblasLtMatmulPreferenceCreate(&pref));
    uint64_t wmax = wsb;
    CB(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wmax, sizeof(wmax)));
    hipblasLtMatmulHeuristicResult_t top[1];
    int ntop = 0;
    hipblasLtMatmulAlgoGetHeuristic(h, op, A, B, C, C, pref, 1, top, &ntop);
    const double flops = 2.0 * p.m * p.n * p.k;
    float t_heur = ntop ? time_algo(h, op, A, B, C, &top[0].algo, a, b, c, ws, wsb, s, 10) : -1.f;
    std::vector<hipblasLtMatmulHeuristicResult_t> all;
    hipblaslt_ext::getAllAlgos(h, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, p.opA, p.opB, HIP_R_16BF, HIP_R_16BF, p.tD,
                               p.tD, HIPBLAS_COMPUTE_32F, all);
    std::vector<std::pair<float, int>> res;
    float alpha = 1.f, beta = 0.f;
    for (int i = 0; i < (int)all.size(); ++i) {
      size_t need = 0;
      if (hipblaslt_ext::matmulIsAlgoSupported(h, op, &alpha, A, B, &beta, C, C, all[i].algo, need) !=
          HIPBLAS_STATUS_SUCCESS || need > wsb)
        continue;
      float t = time_algo(h, op, A, B, C, &all[i].algo, a, b, c, ws, wsb, s, 5);
      if (t > 0) res.push_back({t, i});
    }
    std::sort(res.begin(), res.end());
    printf("%-34s heuristic %7.1f us (%6.1f TF/s); %zu algos, %zu supported\n", p.name, t_heur,
           flops / t_heur / 1e6, all.size(), res.size());
    for (int j = 0; j < (int)res.size() && j < 4; ++j) {
      auto& r = all[res[j].second];
      float t = time_algo(h, op, A, B, C, &r.algo, a, b, c, ws, wsb, s, 20);
      printf("    %7.1f us (%6.1f TF/s) idx %d  %s\n", t, flops / t / 1e6, hipblaslt_ext::getIndexFromAlgo(r.algo),
             hipblaslt_ext::getKernelNameFromAlgo(h, r.algo).c_str());
    }
    fflush(stdout);
  }
  return 0;
}
