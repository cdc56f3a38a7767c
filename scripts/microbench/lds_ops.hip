// LDS primitive costs on gfx950 for the attention drab reduction design:
// cycles per wave-instruction (s_memtime per wave), 256-thread workgroups,
// 2 workgroups per CU, 16 operations per "sub-tile", 64 sub-tiles.
//   hipcc --offload-arch=gfx950 -O3 -o build/lds_ops scripts/microbench/lds_ops.hip && build/lds_ops
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int kIters = 64;

// MODE 0: ds_add_f32, 64 distinct addresses per instruction (per-wave private bins)
// MODE 1: ds_add_f32, lanes r and r+36 collide (the attention's hh pattern), bins shared by the 4 waves
// MODE 2: ds_read_b32 + v_add + ds_write_b32 on private distinct addresses (16 reads, then 16 writes)
// MODE 3: ds_write_b32 only (distinct addresses)
// MODE 4: ds_bpermute_b32 (random permutation)
// MODE 5: DPP row_shl:1 v_add chain (VALU reference)
// MODE 6: ds_add_f32, 32 active lanes (half wave), distinct addresses
// MODE 7: ds_add_u32 (integer), hh pairs collide, bins shared by 4 waves
// MODE 8: ds_add_u64 (integer), hh pairs collide, bins shared by 4 waves
// MODE 9: ds_add_u32, per-wave bins, distinct addresses
template <int MODE>
__global__ void __launch_bounds__(256) k(float* out, unsigned long long* cyc, int salt) {
  __shared__ float bins[4 * 2 * 320 + 64];
  __shared__ unsigned long long bins64[2 * 320 + 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 31, hh = lane >> 5;
  for (int j = threadIdx.x; j < 4 * 2 * 320; j += 256) bins[j] = 0.f;
  __syncthreads();
  float v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = (float)(lane * 16 + i + salt) * 1e-3f;
  float acc = 0.f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIters; ++it) {
    const int base = 32 + (it & 7) * 8;
    if (MODE == 0) {
      float* b = bins + (wave * 2 + hh) * 320 + base + r;
#pragma unroll
      for (int i = 0; i < 16; ++i) atomicAdd(&b[-((i & 3) + 8 * (i >> 2))], v[i]);
    } else if (MODE == 1) {
      float* b = bins + base + r - 4 * hh;
#pragma unroll
      for (int i = 0; i < 16; ++i) atomicAdd(&b[-((i & 3) + 8 * (i >> 2))], v[i]);
    } else if (MODE == 2) {
      float* b = bins + (wave * 2 + hh) * 320 + base + r;
      float t[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) t[i] = b[-((i & 3) + 8 * (i >> 2))];
#pragma unroll
      for (int i = 0; i < 16; ++i) b[-((i & 3) + 8 * (i >> 2))] = t[i] + v[i];
    } else if (MODE == 3) {
      float* b = bins + (wave * 2 + hh) * 320 + base + r;
#pragma unroll
      for (int i = 0; i < 16; ++i) b[-((i & 3) + 8 * (i >> 2))] = v[i];
    } else if (MODE == 4) {
#pragma unroll
      for (int i = 0; i < 16; ++i) acc += __int_as_float(__builtin_amdgcn_ds_bpermute(((lane * 7 + i) & 63) * 4, __float_as_int(v[i])));
    } else if (MODE == 5) {
#pragma unroll
      for (int i = 0; i < 16; ++i)
        acc += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v[i] + acc), 0x101, 0xf, 0xf, true));
    } else if (MODE == 7) {
      unsigned* b = reinterpret_cast<unsigned*>(bins) + base + r - 4 * hh;
#pragma unroll
      for (int i = 0; i < 16; ++i) atomicAdd(&b[-((i & 3) + 8 * (i >> 2))], (unsigned)(v[i] * 65536.f));
    } else if (MODE == 8) {
      unsigned long long* b = bins64 + base + r - 4 * hh;
#pragma unroll
      for (int i = 0; i < 16; ++i) atomicAdd(&b[-((i & 3) + 8 * (i >> 2))], (unsigned long long)(long long)(v[i] * 4294967296.f));
    } else if (MODE == 9) {
      unsigned* b = reinterpret_cast<unsigned*>(bins) + (wave * 2 + hh) * 320 + base + r;
#pragma unroll
      for (int i = 0; i < 16; ++i) atomicAdd(&b[-((i & 3) + 8 * (i >> 2))], (unsigned)(v[i] * 65536.f));
    } else if (MODE == 6) {
      if (hh == 0) {
        float* b = bins + wave * 320 + base + r;
#pragma unroll
        for (int i = 0; i < 16; ++i) atomicAdd(&b[-((i & 3) + 8 * (i >> 2))], v[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = v[i] * 1.0001f + 1e-6f;
  }
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  __syncthreads();
  if (lane == 0) cyc[blockIdx.x * 4 + wave] = t1 - t0;
  if (threadIdx.x == 0) out[blockIdx.x] = bins[40 + salt] + acc + (float)bins64[40 + salt];
}

template <int MODE>
int run(const char* name, int blocks, float* out, unsigned long long* cyc) {
  k<MODE><<<blocks, 256>>>(out, cyc, 0);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  k<MODE><<<blocks, 256>>>(out, cyc, 1);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long* h = new unsigned long long[blocks * 4];
  CK(hipMemcpy(h, cyc, blocks * 4 * 8, hipMemcpyDeviceToHost));
  double s = 0;
  for (int i = 0; i < blocks * 4; ++i) s += h[i];
  delete[] h;
  const double per = s / (blocks * 4) / (kIters * 16.0);
  printf("%-58s %7.1f cycles per wave-instruction (%.1f us kernel)\n", name, per, ms * 1e3);
  return 0;
}

int main() {
  const int blocks = 512;  // 2 per CU
  float* out; unsigned long long* cyc;
  CK(hipMalloc(&out, blocks * 4)); CK(hipMalloc(&cyc, blocks * 4 * 8));
  run<0>("ds_add_f32, 64 distinct addrs, per-wave bins", blocks, out, cyc);
  run<1>("ds_add_f32, hh pairs collide, bins shared by 4 waves", blocks, out, cyc);
  run<6>("ds_add_f32, 32 active lanes, per-wave bins", blocks, out, cyc);
  run<7>("ds_add_u32, hh pairs collide, shared bins", blocks, out, cyc);
  run<8>("ds_add_u64, hh pairs collide, shared bins", blocks, out, cyc);
  run<9>("ds_add_u32, per-wave bins, distinct addrs", blocks, out, cyc);
  run<2>("ds_read_b32 + add + ds_write_b32 (per element pair)", blocks, out, cyc);
  run<3>("ds_write_b32, distinct addrs", blocks, out, cyc);
  run<4>("ds_bpermute_b32", blocks, out, cyc);
  run<5>("v_add_f32 with DPP row_shl:1 (dependent chain)", blocks, out, cyc);
  return 0;
}
