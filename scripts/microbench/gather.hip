// Microbenchmark: cold random-row gather from the bench's 1M x 512 bf16 item
// table (the bench's item_gather_roofline workload: ~60k random rows), with
// variants of the lane mapping, rows in flight and store policy.  Every timed
// launch follows a 512 MiB fill that evicts the Infinity Cache.  Prints GB/s
// of algorithmic traffic (row read + row write + 8 B index).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mb_gather scripts/microbench/gather.hip && /tmp/mb_gather
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int D = 512;        // bf16 elements per row (1 KiB)
constexpr int CH = D / 8;     // 16-byte chunks per row

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void nt_store(uint4 v, uint4* p) {
  u32x4 x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(p));
}

// A: (row, chunk) units strided over the grid, UNROLL units per lane (libgrk's k_gather)
template <int UNROLL, bool NT>
__global__ void __launch_bounds__(256) kA(const uint4* __restrict__ table, const int64_t* __restrict__ idx,
                                          int64_t n, uint4* __restrict__ out) {
  const int64_t units = n * CH;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; base < units; base += stride * UNROLL) {
    uint4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t unit = base + u * stride;
      if (unit < units) v[u] = table[idx[unit / CH] * CH + unit % CH];
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t unit = base + u * stride;
      if (unit >= units) continue;
      if (NT) nt_store(v[u], out + unit);
      else out[unit] = v[u];
    }
  }
}

// A1: one (row, chunk) unit per lane, grid-stride, BS threads per block
template <int BS>
__global__ void __launch_bounds__(BS) kA1(const uint4* __restrict__ table, const int64_t* __restrict__ idx,
                                          int64_t n, uint4* __restrict__ out) {
  const int64_t units = n * CH;
  const int64_t stride = (int64_t)gridDim.x * BS;
  for (int64_t u = (int64_t)blockIdx.x * BS + threadIdx.x; u < units; u += stride)
    out[u] = table[idx[u / CH] * CH + u % CH];
}

// B: each wave owns R consecutive output rows: one index load per lane (lane r<R
// loads idx[r]), broadcast with readlane, then R independent 1 KiB row loads.
template <int R, bool NT>
__global__ void __launch_bounds__(256) kB(const uint4* __restrict__ table, const int64_t* __restrict__ idx,
                                          int64_t n, uint4* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r0 = wave * R; r0 < n; r0 += waves * R) {
    const int64_t my = lane < R && r0 + lane < n ? idx[r0 + lane] : 0;
    uint4 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int64_t row = __builtin_amdgcn_readlane((int)my, r) | ((int64_t)__builtin_amdgcn_readlane((int)(my >> 32), r) << 32);
      if (r0 + r < n) v[r] = table[row * CH + lane];
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (r0 + r >= n) continue;
      if (NT) nt_store(v[r], out + (r0 + r) * CH + lane);
      else out[(r0 + r) * CH + lane] = v[r];
    }
  }
}

// C: persistent waves (a capped grid), R rows per wave and pass; the next pass's
// indices are loaded while the current rows are in flight
template <int R, bool NT>
__global__ void __launch_bounds__(256) kC(const uint4* __restrict__ table, const int64_t* __restrict__ idx,
                                          int64_t n, uint4* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  int64_t r0 = wave * R;
  int64_t my = lane < R && r0 + lane < n ? idx[r0 + lane] : 0;
  for (; r0 < n; r0 += waves * R) {
    uint4 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int64_t row = __builtin_amdgcn_readlane((int)my, r) | ((int64_t)__builtin_amdgcn_readlane((int)(my >> 32), r) << 32);
      if (r0 + r < n) v[r] = table[row * CH + lane];
    }
    const int64_t r1 = r0 + waves * R;
    my = lane < R && r1 + lane < n ? idx[r1 + lane] : 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (r0 + r >= n) continue;
      if (NT) nt_store(v[r], out + (r0 + r) * CH + lane);
      else out[(r0 + r) * CH + lane] = v[r];
    }
  }
}

// contiguous copy of the same bytes (ceiling for one launch of this size)
__global__ void __launch_bounds__(256) kCopy(const uint4* __restrict__ src, int64_t units, uint4* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < units; i += stride) out[i] = src[i];
}

// eviction by READING 512 MiB: the caches end full of clean lines, so the timed
// launch pays no write-back of the flush buffer
__global__ void kTouch(const uint4* p, int64_t n, unsigned* sink) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  unsigned acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) acc ^= p[i].x ^ p[i].w;
  if (acc == 0x12345679u) sink[0] = acc;
}

__global__ void kFill(uint4* p, int64_t n, unsigned v) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = make_uint4(v, v, v, v);
}

static unsigned* g_sink;
static bool g_read_flush = true;
template <typename F>
static void run(const char* name, F launch, double bytes, uint4* flush, int64_t flush_units) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  launch();
  CK(hipDeviceSynchronize());
  double cold = 0, warm = 0;
  const int reps = 20;
  for (int i = 0; i < reps; ++i) {
    if (g_read_flush) kTouch<<<4096, 256>>>(flush, flush_units, g_sink);
    else kFill<<<4096, 256>>>(flush, flush_units, i);
    CK(hipEventRecord(a));
    launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    cold += ms;
  }
  for (int i = 0; i < reps; ++i) {
    CK(hipEventRecord(a));
    launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    warm += ms;
  }
  cold /= reps;
  warm /= reps;
  printf("%-28s cold %7.2f us %7.1f GB/s (%.3f of 8000) | warm %7.2f us %7.1f GB/s\n", name, cold * 1e3,
         bytes / (cold * 1e-3) / 1e9, bytes / (cold * 1e-3) / 1e9 / 8000.0, warm * 1e3, bytes / (warm * 1e-3) / 1e9);
}

int main(int argc, char** argv) {
  const int64_t rows = 1000000;
  const int64_t n = argc > 1 ? atoll(argv[1]) : 60000;
  g_read_flush = argc > 2 ? atoi(argv[2]) != 0 : true;
  CK(hipMalloc(&g_sink, 4));
  uint4 *table, *out, *flush, *src;
  int64_t* idx;
  CK(hipMalloc(&table, rows * D * 2));
  CK(hipMalloc(&out, n * D * 2));
  CK(hipMalloc(&src, n * D * 2));
  const int64_t flush_units = (512ll << 20) / 16;
  CK(hipMalloc(&flush, flush_units * 16));
  CK(hipMalloc(&idx, n * 8));
  kFill<<<4096, 256>>>(table, rows * CH, 0x3f803f80u);
  kFill<<<4096, 256>>>(src, n * CH, 1u);
  std::vector<int64_t> h(n);
  uint64_t s = 88172645463325252ull;
  for (int64_t i = 0; i < n; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    h[i] = 1 + (int64_t)(s % (uint64_t)(rows - 1));
  }
  CK(hipMemcpy(idx, h.data(), n * 8, hipMemcpyHostToDevice));
  const double bytes = 2.0 * n * D * 2 + 8.0 * n;
  kFill<<<4096, 256>>>(flush, flush_units, 7u);
  printf("rows %lld of %lld, %.1f MB algorithmic, eviction by %s 512 MiB\n", (long long)n, (long long)rows,
         bytes / 1e6, g_read_flush ? "reading" : "writing");
  auto grid = [&](int64_t work, int cap) { int64_t g = (work + 255) / 256; return (unsigned)(g < cap ? g : cap); };
  run("copy (contiguous)", [&] { kCopy<<<grid(n * CH, 8192), 256>>>(src, n * CH, out); }, bytes, flush, flush_units);
  run("A unroll4 cap4097", [&] { kA<4, false><<<grid((n * CH + 3) / 4, 4097), 256>>>(table, idx, n, out); }, bytes, flush, flush_units);
  run("A unroll4 cap4097 NT", [&] { kA<4, true><<<grid((n * CH + 3) / 4, 4097), 256>>>(table, idx, n, out); }, bytes, flush, flush_units);
  run("A unroll1 nocap", [&] { kA<1, false><<<grid(n * CH, 1 << 20), 256>>>(table, idx, n, out); }, bytes, flush, flush_units);
  run("A unroll1 nocap NT", [&] { kA<1, true><<<grid(n * CH, 1 << 20), 256>>>(table, idx, n, out); }, bytes, flush, flush_units);
  run("A unroll1 cap8192", [&] { kA<1, false><<<grid(n * CH, 8192), 256>>>(table, idx, n, out); }, bytes, flush, flush_units);
  run("A unroll2 nocap", [&] { kA<2, false><<<grid((n * CH + 1) / 2, 1 << 20), 256>>>(table, idx, n, out); }, bytes, flush, flush_units);
  run("A unroll8 nocap", [&] { kA<8, false><<<grid((n * CH + 7) / 8, 1 << 20), 256>>>(table, idx, n, out); }, bytes, flush, flush_units);
  run("B R=2", [&] { kB<2, false><<<grid((n + 1) / 2 * 64, 1 << 20), 256>>>(table, idx, n, out); }, bytes, flush, flush_units);
  run("B R=4", [&] { kB<4, false><<<grid((n + 3) / 4 * 64, 1 << 20), 256>>>(table, idx, n, out); }, bytes, flush, flush_units);
  run("B R=4 NT", [&] { kB<4, true><<<grid((n + 3) / 4 * 64, 1 << 20), 256>>>(table, idx, n, out); }, bytes, flush, flush_units);
  run("B R=8", [&] { kB<8, false><<<grid((n + 7) / 8 * 64, 1 << 20), 256>>>(table, idx, n, out); }, bytes, flush, flush_units);
  run("B R=8 NT", [&] { kB<8, true><<<grid((n + 7) / 8 * 64, 1 << 20), 256>>>(table, idx, n, out); }, bytes, flush, flush_units);
  run("B R=16", [&] { kB<16, false><<<grid((n + 15) / 16 * 64, 1 << 20), 256>>>(table, idx, n, out); }, bytes, flush, flush_units);
  run("B R=4 half grid", [&] { kB<4, false><<<grid((n + 7) / 8 * 64, 1 << 20), 256>>>(table, idx, n, out); }, bytes, flush, flush_units);
  if (argc > 3) {   // round-6 second sweep: the one-unit-per-lane form around its best grid
    for (int cap : {2048, 4096, 6144, 8192, 12288, 16384, 1 << 20}) {
      char nm[64];
      snprintf(nm, sizeof nm, "A1 256 cap %d", cap);
      run(nm, [&] { kA1<256><<<grid(n * CH, cap), 256>>>(table, idx, n, out); }, bytes, flush, flush_units);
    }
    auto grid2 = [&](int64_t work, int bs, int cap) { int64_t g = (work + bs - 1) / bs; return (unsigned)(g < cap ? g : cap); };
    for (int cap : {1024, 2048, 4096, 1 << 20}) {
      char nm[64];
      snprintf(nm, sizeof nm, "A1 512 cap %d", cap);
      run(nm, [&] { kA1<512><<<grid2(n * CH, 512, cap), 512>>>(table, idx, n, out); }, bytes, flush, flush_units);
      snprintf(nm, sizeof nm, "A1 1024 cap %d", cap);
      run(nm, [&] { kA1<1024><<<grid2(n * CH, 1024, cap), 1024>>>(table, idx, n, out); }, bytes, flush, flush_units);
    }
    run("copy (contiguous) again", [&] { kCopy<<<grid(n * CH, 8192), 256>>>(src, n * CH, out); }, bytes, flush, flush_units);
    CK(hipDeviceSynchronize());
    return 0;
  }
  for (int cap : {512, 1024, 2048, 4096}) {
    char nm[64];
    snprintf(nm, sizeof nm, "C R=4 grid %d", cap);
    run(nm, [&] { kC<4, false><<<cap, 256>>>(table, idx, n, out); }, bytes, flush, flush_units);
    snprintf(nm, sizeof nm, "C R=4 NT grid %d", cap);
    run(nm, [&] { kC<4, true><<<cap, 256>>>(table, idx, n, out); }, bytes, flush, flush_units);
    snprintf(nm, sizeof nm, "C R=2 grid %d", cap);
    run(nm, [&] { kC<2, false><<<cap, 256>>>(table, idx, n, out); }, bytes, flush, flush_units);
    snprintf(nm, sizeof nm, "C R=8 grid %d", cap);
    run(nm, [&] { kC<8, false><<<cap, 256>>>(table, idx, n, out); }, bytes, flush, flush_units);
  }
  run("B R=1", [&] { kB<1, false><<<grid(n * 64, 1 << 20), 256>>>(table, idx, n, out); }, bytes, flush, flush_units);
  run("B R=1 NT", [&] { kB<1, true><<<grid(n * 64, 1 << 20), 256>>>(table, idx, n, out); }, bytes, flush, flush_units);
  CK(hipDeviceSynchronize());
  return 0;
}
