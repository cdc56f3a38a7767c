// Shared helpers for the grk HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/grk.h"

namespace grk {

// ---------------------------------------------------------------- errors ----
// Thread-local message returned by grk_last_error(); every C-ABI entry point
// returns 0 on success or a non-zero GRK_E* code after calling set_error().
void set_error(const char* fmt, ...);
void clear_error();
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) per (device, kernel), thread-safe (grk_util.cpp).
hipError_t ensure_dynamic_lds(const void* kernel, size_t bytes);

#define GRK_CHECK_ARG(cond, ...)                   \
  do {                                             \
    if (!(cond)) {                                 \
      ::grk::set_error(__VA_ARGS__);               \
      return GRK_EINVAL;                           \
    }                                              \
  } while (0)

#define GRK_CHECK_HIP(expr)                                                     \
  do {                                                                          \
    hipError_t _e = (expr);                                                     \
    if (_e != hipSuccess) {                                                     \
      ::grk::set_error("%s failed: %s", #expr, hipGetErrorString(_e));          \
      return GRK_EHIP;                                                          \
    }                                                                           \
  } while (0)

#define GRK_LAUNCH_CHECK()                                                      \
  do {                                                                          \
    hipError_t _e = hipGetLastError();                                          \
    if (_e != hipSuccess) {                                                     \
      ::grk::set_error("kernel launch failed: %s", hipGetErrorString(_e));      \
      return GRK_EHIP;                                                          \
    }                                                                           \
  } while (0)

// ------------------------------------------------------------- numerics ----
typedef unsigned short bf16_t;  // raw bf16 storage

__device__ __forceinline__ float bf16_to_f32(bf16_t x) {
  return __uint_as_float(((unsigned)x) << 16);
}
// Round-to-nearest-even, NaN stays NaN (hipcc emits v_cvt_pk_bf16_f32).
__device__ __forceinline__ bf16_t f32_to_bf16(float f) {
  __bf16 b = static_cast<__bf16>(f);
  return __builtin_bit_cast(bf16_t, b);
}

// sigmoid via the hardware exp2 / reciprocal (v_exp_f32, v_rcp_f32: ~1 ulp),
// no IEEE division; saturates cleanly to 0 / 1 for large |x|.
__device__ __forceinline__ float sigmoid_fast(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.4426950408889634f));
}
__device__ __forceinline__ float silu(float x) { return x * sigmoid_fast(x); }
__device__ __forceinline__ float dsilu(float x) {
  const float sg = sigmoid_fast(x);
  return sg * (1.0f + x * (1.0f - sg));
}

template <typename T> struct Elem;
template <> struct Elem<float> {
  static __device__ __forceinline__ float load(const float* p) { return *p; }
  static __device__ __forceinline__ void store(float* p, float v) { *p = v; }
};
template <> struct Elem<bf16_t> {
  static __device__ __forceinline__ float load(const bf16_t* p) { return bf16_to_f32(*p); }
  static __device__ __forceinline__ void store(bf16_t* p, float v) { *p = f32_to_bf16(v); }
};

// 16-byte vector of T: 4 fp32 or 8 bf16.
template <typename T> struct Vec16;
template <> struct Vec16<float> {
  static constexpr int N = 4;
  float4 v;
  __device__ __forceinline__ void load(const float* p) { v = *reinterpret_cast<const float4*>(p); }
  __device__ __forceinline__ void store(float* p) const { *reinterpret_cast<float4*>(p) = v; }
  __device__ __forceinline__ float get(int i) const { return (&v.x)[i]; }
  __device__ __forceinline__ void set(int i, float f) { (&v.x)[i] = f; }
};
template <> struct Vec16<bf16_t> {
  static constexpr int N = 8;
  uint4 v;
  __device__ __forceinline__ void load(const bf16_t* p) { v = *reinterpret_cast<const uint4*>(p); }
  __device__ __forceinline__ void store(bf16_t* p) const { *reinterpret_cast<uint4*>(p) = v; }
  __device__ __forceinline__ float get(int i) const {
    unsigned w = (&v.x)[i >> 1];
    return __uint_as_float((i & 1) ? (w & 0xFFFF0000u) : (w << 16));
  }
  __device__ __forceinline__ void set(int i, float f) {
    unsigned b = f32_to_bf16(f);
    unsigned& w = (&v.x)[i >> 1];
    w = (i & 1) ? ((w & 0x0000FFFFu) | (b << 16)) : ((w & 0xFFFF0000u) | b);
  }
};

inline size_t dtype_size(int dt) { return dt == GRK_F32 ? 4 : 2; }

namespace {
// Zero-fill as a kernel (16-byte stores when aligned, 4-byte stores otherwise).
// Used instead of hipMemsetAsync for every buffer that must be zero at a
// kernel's start: a hipMemsetAsync captured into a HIP graph does not zero its
// buffer on the second and later replays (ROCm 7.2; any size above 4 bytes --
// scripts/graph_memset_check.py), so nothing in a step that may
// be captured uses one.
__global__ void k_zero_fill(uint32_t* __restrict__ p, size_t words, size_t vecs) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const size_t t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (size_t i = t0; i < vecs; i += stride) reinterpret_cast<uint4*>(p)[i] = make_uint4(0u, 0u, 0u, 0u);
  for (size_t i = vecs * 4 + t0; i < words; i += stride) p[i] = 0u;
}
}  // namespace

// bytes: a multiple of 4.  Never a hipMemsetAsync (see k_zero_fill).
inline hipError_t zero_async(void* p, size_t bytes, hipStream_t s) {
  const size_t words = bytes / 4;
  if (words == 0) return hipSuccess;
  const bool aligned = (uintptr_t)p % 16 == 0;
  const size_t vecs = aligned ? words / 4 : 0;
  const size_t work = aligned ? (vecs > 0 ? vecs : 1) : words;
  const size_t blocks = (work + 255) / 256;
  k_zero_fill<<<(unsigned)(blocks < 4096 ? blocks : 4096), 256, 0, s>>>((uint32_t*)p, words, vecs);
  return hipGetLastError();
}

inline int grid_for(int64_t work, int block, int max_blocks = 256 * 16) {
  int64_t g = (work + block - 1) / block;
  if (g < 1) g = 1;
  if (g > max_blocks) g = max_blocks;
  return (int)g;
}

}  // namespace grk
