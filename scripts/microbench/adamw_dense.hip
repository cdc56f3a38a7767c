// Microbenchmark: dense-parity table AdamW variants on a [rows, dim] bf16
// table with fp32 moments (the bench's 1M x 512 item table).  Prints
// GB/s of algorithmic traffic (20 B/element) per variant.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mb_adamw scripts/microbench/adamw_dense.hip && /tmp/mb_adamw
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

struct HP { float lr, b1, b2, eps, wd, step, bc2; };

__device__ __forceinline__ float bf(unsigned short x) { return __uint_as_float(((unsigned)x) << 16); }
__device__ __forceinline__ unsigned short tobf(float f) { __bf16 b = (__bf16)f; return __builtin_bit_cast(unsigned short, b); }

__device__ __forceinline__ void upd(float& p, float& m, float& v, float g, const HP& h) {
  p *= 1.0f - h.lr * h.wd;
  m = m + (1.0f - h.b1) * (g - m);
  v = v * h.b2 + (1.0f - h.b2) * g * g;
  p = p - h.step * (m / (sqrtf(v) / h.bc2 + h.eps));
}

// A: 4 elements / thread, flat grid-stride (current libgrk)
__global__ void __launch_bounds__(256) kA(unsigned short* P, float* M, float* V, int64_t rows, int dim,
                                          const float* U, const int* slot, HP h) {
  const int q = dim / 4;
  const int64_t total = rows * q;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / q;
    const int c = (int)(i - row * q) * 4;
    const int s = slot[row];
    float g[4] = {0, 0, 0, 0};
    if (s >= 0) { float4 t = *(const float4*)(U + (int64_t)s * dim + c); g[0] = t.x; g[1] = t.y; g[2] = t.z; g[3] = t.w; }
    const int64_t o = row * dim + c;
    uint2 pt = *(uint2*)(P + o);
    float4 mt = *(float4*)(M + o), vt = *(float4*)(V + o);
    float p[4] = {__uint_as_float(pt.x << 16), __uint_as_float(pt.x & 0xFFFF0000u), __uint_as_float(pt.y << 16), __uint_as_float(pt.y & 0xFFFF0000u)};
    float m[4] = {mt.x, mt.y, mt.z, mt.w}, v[4] = {vt.x, vt.y, vt.z, vt.w};
    for (int e = 0; e < 4; ++e) upd(p[e], m[e], v[e], g[e], h);
    pt.x = tobf(p[0]) | ((unsigned)tobf(p[1]) << 16); pt.y = tobf(p[2]) | ((unsigned)tobf(p[3]) << 16);
    *(uint2*)(P + o) = pt;
    *(float4*)(M + o) = make_float4(m[0], m[1], m[2], m[3]);
    *(float4*)(V + o) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ float4 ld4(const float* p) {
  if (NT) { f4 t = __builtin_nontemporal_load((const f4*)p); return make_float4(t.x, t.y, t.z, t.w); }
  return *(const float4*)p;
}
template <bool NT>
__device__ __forceinline__ void st4(float* p, float4 v) {
  if (NT) { f4 t = {v.x, v.y, v.z, v.w}; __builtin_nontemporal_store(t, (f4*)p); }
  else *(float4*)p = v;
}
template <bool NT>
__device__ __forceinline__ uint4 ldu4(const unsigned short* p) {
  if (NT) { u4 t = __builtin_nontemporal_load((const u4*)p); return make_uint4(t.x, t.y, t.z, t.w); }
  return *(const uint4*)p;
}
template <bool NT>
__device__ __forceinline__ void stu4(unsigned short* p, uint4 v) {
  if (NT) { u4 t = {v.x, v.y, v.z, v.w}; __builtin_nontemporal_store(t, (u4*)p); }
  else *(uint4*)p = v;
}

template <bool NT>
__device__ __forceinline__ void vec8(unsigned short* P, float* M, float* V, int64_t o, const float* gsrc, const HP& h) {
  uint4 pt = ldu4<NT>(P + o);
  float4 m0 = ld4<NT>(M + o), m1 = ld4<NT>(M + o + 4), v0 = ld4<NT>(V + o), v1 = ld4<NT>(V + o + 4);
  float g[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (gsrc) { float4 a = *(const float4*)gsrc, b = *(const float4*)(gsrc + 4); g[0] = a.x; g[1] = a.y; g[2] = a.z; g[3] = a.w; g[4] = b.x; g[5] = b.y; g[6] = b.z; g[7] = b.w; }
  unsigned w[4] = {pt.x, pt.y, pt.z, pt.w};
  float p[8], m[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w}, v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
  for (int i = 0; i < 4; ++i) { p[2 * i] = __uint_as_float(w[i] << 16); p[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u); }
  for (int e = 0; e < 8; ++e) upd(p[e], m[e], v[e], g[e], h);
  for (int i = 0; i < 4; ++i) w[i] = tobf(p[2 * i]) | ((unsigned)tobf(p[2 * i + 1]) << 16);
  stu4<NT>(P + o, make_uint4(w[0], w[1], w[2], w[3]));
  st4<NT>(M + o, make_float4(m[0], m[1], m[2], m[3])); st4<NT>(M + o + 4, make_float4(m[4], m[5], m[6], m[7]));
  st4<NT>(V + o, make_float4(v[0], v[1], v[2], v[3])); st4<NT>(V + o + 4, make_float4(v[4], v[5], v[6], v[7]));
}

// B/C: 8 elements / thread, flat grid-stride (NT = nontemporal)
template <bool NT>
__global__ void __launch_bounds__(256) kB(unsigned short* P, float* M, float* V, int64_t rows, int dim,
                                          const float* U, const int* slot, HP h) {
  const int q = dim / 8;
  const int64_t total = rows * q;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / q;
    const int c = (int)(i - row * q) * 8;
    const int s = slot[row];
    vec8<NT>(P, M, V, row * dim + c, s >= 0 ? U + (int64_t)s * dim + c : nullptr, h);
  }
}

// D/E: one wave per row (dim = 512 -> 64 lanes x 8), grid-stride over rows, UNR rows per iteration
template <bool NT, int UNR>
__global__ void __launch_bounds__(256) kD(unsigned short* P, float* M, float* V, int64_t rows, int dim,
                                          const float* U, const int* slot, HP h) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r0 = wave * UNR; r0 < rows; r0 += nw * UNR) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t row = r0 + u;
      if (row < rows) {
        const int s = slot[row];
        for (int c = lane * 8; c < dim; c += 512)
          vec8<NT>(P, M, V, row * dim + c, s >= 0 ? U + (int64_t)s * dim + c : nullptr, h);
      }
    }
  }
}

// F: one vector per thread, no loop (grid covers the table)
template <bool NT>
__global__ void __launch_bounds__(256) kF(unsigned short* P, float* M, float* V, int64_t rows, int dim,
                                          const float* U, const int* slot, HP h) {
  const int q = dim / 8;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * q) return;
  const int64_t row = i / q;
  const int c = (int)(i - row * q) * 8;
  const int s = slot[row];
  vec8<NT>(P, M, V, row * dim + c, s >= 0 ? U + (int64_t)s * dim + c : nullptr, h);
}

int main() {
  const int64_t rows = 1000001;
  const int dim = 512;
  const int64_t n = rows * dim;
  unsigned short* P; float *M, *V, *U; int* slot;
  const int64_t nu = 45000;
  CK(hipMalloc(&P, n * 2)); CK(hipMalloc(&M, n * 4)); CK(hipMalloc(&V, n * 4));
  CK(hipMalloc(&U, nu * dim * 4)); CK(hipMalloc(&slot, rows * 4));
  CK(hipMemset(P, 0x3c, n * 2)); CK(hipMemset(M, 0, n * 4)); CK(hipMemset(V, 0, n * 4)); CK(hipMemset(U, 0, nu * dim * 4));
  int* hs = (int*)malloc(rows * 4);
  for (int64_t r = 0; r < rows; ++r) hs[r] = -1;
  for (int64_t u = 0; u < nu; ++u) hs[(u * 2654435761ull) % rows] = (int)u;
  CK(hipMemcpy(slot, hs, rows * 4, hipMemcpyHostToDevice));
  HP h = {1e-3f, 0.9f, 0.98f, 1e-8f, 0.01f, 1e-3f, 0.2f};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const double bytes = 20.0 * n;
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    const int reps = 20;
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-44s %8.1f us  %7.1f GB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
  };
  for (int g : {2048, 8192, 32768}) {
    char nm[64];
    snprintf(nm, 64, "A 4/thr grid-stride g=%d", g);
    run(nm, [&] { kA<<<g, 256>>>(P, M, V, rows, dim, U, slot, h); });
    snprintf(nm, 64, "B 8/thr grid-stride g=%d", g);
    run(nm, [&] { kB<false><<<g, 256>>>(P, M, V, rows, dim, U, slot, h); });
    snprintf(nm, 64, "C 8/thr grid-stride NT g=%d", g);
    run(nm, [&] { kB<true><<<g, 256>>>(P, M, V, rows, dim, U, slot, h); });
    snprintf(nm, 64, "D wave/row unr1 g=%d", g);
    run(nm, [&] { kD<false, 1><<<g, 256>>>(P, M, V, rows, dim, U, slot, h); });
    snprintf(nm, 64, "D wave/row unr2 g=%d", g);
    run(nm, [&] { kD<false, 2><<<g, 256>>>(P, M, V, rows, dim, U, slot, h); });
    snprintf(nm, 64, "E wave/row unr2 NT g=%d", g);
    run(nm, [&] { kD<true, 2><<<g, 256>>>(P, M, V, rows, dim, U, slot, h); });
  }
  const int gf = (int)((n / 8 + 255) / 256);
  run("F one vec/thread (full grid)", [&] { kF<false><<<gf, 256>>>(P, M, V, rows, dim, U, slot, h); });
  run("F one vec/thread (full grid) NT", [&] { kF<true><<<gf, 256>>>(P, M, V, rows, dim, U, slot, h); });
  CK(hipDeviceSynchronize());
  printf("done\n");
  return 0;
}
