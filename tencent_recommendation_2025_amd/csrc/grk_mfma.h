// MFMA 32x32x16 bf16 fragment helpers shared by the attention and
// sampled-softmax kernels (gfx950).  Lane l: r = l & 31, hh = l >> 5;
//   A[r][8hh + j], B[8hh + j][r], D[(i&3) + 8(i>>2) + 4hh][r].
#pragma once
#include "grk_common.h"

namespace grk {

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));


__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// A zero accumulator for the FIRST MFMA of a chain, opaque to the compiler.
// With a literal zero srcC the 32x32 MFMA's destination is untied, and in the
// VGPR form (grk_attention_seq, -amdgpu-mfma-vgpr-form) the register allocator
// may hand it the registers of a srcA/srcB that dies at that MFMA.  A multi-pass
// MFMA whose vdst overlaps its srcA/srcB is outside the ISA's rules; on gfx950 it
// produced timing-dependent wrong rows whenever two workgroups shared a CU
// (DESIGN.md §5b).  Through this value srcC is a live register tied to vdst, so
// vdst can never alias a source.  scripts/check_mfma_overlap.py (run by `make`)
// rejects any library whose code object still has such an MFMA.
__device__ __forceinline__ f32x16 acc_zero() {
  float z;
  asm("v_mov_b32 %0, 0" : "=v"(z));
  f32x16 r;
#pragma unroll
  for (int i = 0; i < 16; ++i) r[i] = z;
  return r;
}

// Swizzled LDS row image: row of HD bf16 = HD/8 16-byte chunks; chunk c of
// row r lives at chunk position c ^ (r & MASK).
template <int HD>
__device__ __forceinline__ int lds_off(int row, int col) {
  constexpr int NCH = HD / 8;
  constexpr int MASK = NCH >= 8 ? 7 : NCH - 1;
  const int c = col >> 3;
  return row * (HD * 2) + ((c ^ (row & MASK)) << 4) + ((col & 7) << 1);
}

template <int HD>
__device__ __forceinline__ bf16x8 lds_row8(const char* base, int row, int col) {
  return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(base + lds_off<HD>(row, col)));
}

// Transposed fragment: element j of lane (r, hh) = M[row0 + 8(j>>2) + 4hh + (j&3)][col0 + r].
template <int HD>
__device__ __forceinline__ bf16x8 lds_tr8(const char* base, int row0, int col0, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int q4 = i >> 2, p = i & 3;
  const int hh = g >> 1;
  const int col = col0 + 16 * (g & 1) + 4 * p;
  const int ra = row0 + 4 * hh + q4;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + lds_off<HD>(ra, col)));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + lds_off<HD>(ra + 8, col)));
  bf16x4 l4 = __builtin_bit_cast(bf16x4, lo), h4 = __builtin_bit_cast(bf16x4, hi);
  bf16x8 r;
  r[0] = l4[0]; r[1] = l4[1]; r[2] = l4[2]; r[3] = l4[3];
  r[4] = h4[0]; r[5] = h4[1]; r[6] = h4[2]; r[7] = h4[3];
  return r;
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// Two values as packed bf16 words: hi = bf16(x) (round to nearest even),
// lo = bf16(x - hi) -- one v_cvt_pk_bf16_f32 per word.  Scalar f32 math only:
// packed f32 VALU (v_pk_*_f32) costs more than two scalar ops between MFMAs
// (MI355X_MICROARCH.md), and packed SiLU sequences in the forward gave
// run-to-run different outputs.
__device__ __forceinline__ void split2(f32x2 x, uint32_t& hi, uint32_t& lo) {
  const uint32_t h = __builtin_bit_cast(uint32_t, __builtin_convertvector(x, bf16x2));
  const float r0 = x.x - __uint_as_float(h << 16), r1 = x.y - __uint_as_float(h & 0xFFFF0000u);
  hi = h;
  lo = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{r0, r1}, bf16x2));
}

__device__ __forceinline__ bf16x8 words8(const uint32_t* w) {
  return __builtin_bit_cast(bf16x8, make_uint4(w[0], w[1], w[2], w[3]));
}

// Accumulator registers 8s..8s+7 as a bf16 operand (hi part, and the
// residual lo part for the precise mode).
__device__ __forceinline__ void pack_acc(const float* x, int s, bf16x8& hi, bf16x8& lo) {
  uint32_t h[4], l[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) split2(f32x2{x[8 * s + 2 * j], x[8 * s + 2 * j + 1]}, h[j], l[j]);
  hi = words8(h);
  lo = words8(l);
}

__device__ __forceinline__ int acc_row(int i, int hh) { return (i & 3) + 8 * (i >> 2) + 4 * hh; }

// Load a [HD] bf16 row slice as an 8-wide fragment from global; zero if !ok.
__device__ __forceinline__ bf16x8 gload8(const bf16_t* p, bool ok) {
  uint4 v = ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0, 0, 0, 0);
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ bf16x8 gload8_any(const void* base, int64_t off, bool f32, bool ok) {
  if (!ok) return __builtin_bit_cast(bf16x8, make_uint4(0, 0, 0, 0));
  if (!f32) return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>((const bf16_t*)base + off));
  const float4* fp = reinterpret_cast<const float4*>((const float*)base + off);
  float4 a = fp[0], b = fp[1];
  bf16x8 r;
  r[0] = (__bf16)a.x; r[1] = (__bf16)a.y; r[2] = (__bf16)a.z; r[3] = (__bf16)a.w;
  r[4] = (__bf16)b.x; r[5] = (__bf16)b.y; r[6] = (__bf16)b.z; r[7] = (__bf16)b.w;
  return r;
}

// ---- OCP fp8 e4m3 (gfx950's fp8 format) ----
// Eight e4m3 values in one 64-bit fragment: the A / B operand of the fp8
// 32x32x16 MFMA, same lane map as the bf16 form (element j of lane (r, hh) is
// k = 8hh + j) and the bf16 form's rate; products of fp8 values are exact in
// its fp32 accumulation.
typedef long f8x8;

__device__ __forceinline__ f32x16 mfma8(f8x8 a, f8x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_fp8_fp8(a, b, c, 0, 0, 0);
}

// Eight e4m3 values (bytes of w, element 0 in the lowest byte) as bf16.  Exact:
// every e4m3 value is a bf16 value (3 mantissa bits, exponents 2^-9 .. 2^8),
// so the fp32 result of v_cvt_pk_f32_fp8 truncates to bf16 without rounding.
__device__ __forceinline__ bf16x8 f8x8_to_bf16(uint2 w) {
  const f32x2 a = __builtin_amdgcn_cvt_pk_f32_fp8((int)w.x, false), b = __builtin_amdgcn_cvt_pk_f32_fp8((int)w.x, true);
  const f32x2 c = __builtin_amdgcn_cvt_pk_f32_fp8((int)w.y, false), d = __builtin_amdgcn_cvt_pk_f32_fp8((int)w.y, true);
  const uint32_t words[4] = {(__float_as_uint(a.x) >> 16) | (__float_as_uint(a.y) & 0xFFFF0000u),
                             (__float_as_uint(b.x) >> 16) | (__float_as_uint(b.y) & 0xFFFF0000u),
                             (__float_as_uint(c.x) >> 16) | (__float_as_uint(c.y) & 0xFFFF0000u),
                             (__float_as_uint(d.x) >> 16) | (__float_as_uint(d.y) & 0xFFFF0000u)};
  return words8(words);
}

// Eight consecutive elements from global as bf16: src 0 = bf16, 1 = fp32
// (rounded), 2 = fp8 e4m3 (exact); zero when !ok.
__device__ __forceinline__ bf16x8 gload8_src(const void* base, int64_t off, int src, bool ok) {
  if (src == 2) {
    const uint2 w = ok ? *reinterpret_cast<const uint2*>((const uint8_t*)base + off) : make_uint2(0, 0);
    return f8x8_to_bf16(w);
  }
  return gload8_any(base, off, src == 1, ok);
}

// SiLU of each element, computed in fp32 and rounded to bf16 (= F.silu on bf16).
__device__ __forceinline__ bf16x8 silu8(bf16x8 x) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = static_cast<__bf16>(silu(static_cast<float>(x[j])));
  return r;
}

}  // namespace grk
