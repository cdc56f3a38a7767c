// LDS-DMA ring helpers shared by the MFMA GEMM kernels (grk_wgrad.hip,
// grk_ggemm.hip): 32-row K steps staged by global_load_lds_dwordx4 into a ring of
// LDS stages, retired by counted s_waitcnt vmcnt + s_barrier.  Images with K
// rows ("K-major": 32 rows x (64 WM | 64 WN) columns, RB-byte rows) are read as
// MFMA fragments with ds_read_b64_tr_b16 (ring_frag).
#pragma once
#include "grk_common.h"
#include "grk_mfma.h"

namespace grk {

constexpr int kWgK = 32;                        // K rows per step

__device__ __forceinline__ int wg_swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

// One 16-byte-per-lane LDS-DMA (global_load_lds_dwordx4) to the wave-uniform LDS
// address lds.  In asm, so hipcc does not count it: its alias tracking of
// LDS-DMA stores otherwise puts s_waitcnt vmcnt(0) before the step's first
// ds_read (seen in the ISA), draining the ring; the counted waits below are
// the only ones (cdna_hip_programming.md §5.7: M0 set and restored inside).
__device__ __forceinline__ void wg_dma16(const bf16_t* src, unsigned lds) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds)
      : "memory");
}

template <int N>
__device__ __forceinline__ void wg_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// Ring geometry: WM x WN waves, each owning a 64 x 64 quarter-tile of the output
// (2 x 2 MFMA 32x32x16 tiles), so a workgroup owns a (64 WM) x (64 WN) tile; NST
// LDS stages of one 32-row step each (dY image [32][64 WM], X image [32][64 WN]),
// NST - 1 steps issued ahead.  <2, 2, 4>: 128 x 128 tiles, 64 KiB, two
// workgroups per CU; <4, 2, 6>: 256 x 128 tiles, 144 KiB, one workgroup of 8
// waves per CU -- a third fewer operand bytes per FLOP and 4 steps in flight
// (an LDS-DMA lands ~1.1 us after issue, MI355X_MICROARCH.md).
template <int WM, int WN, int NST>
struct WgRing {
  static constexpr int TM = 64 * WM, TN = 64 * WN;   // output tile rows (M) / columns (N)
  static constexpr int RBA = 2 * TM, RBB = 2 * TN;   // image row bytes
  static constexpr int IMGA = kWgK * RBA, IMGB = kWgK * RBB;
  static constexpr int STAGE = IMGA + IMGB;
  static constexpr int NW = WM * WN, NT = 64 * NW;
  static constexpr int PWA = IMGA / 1024 / NW, PWB = IMGB / 1024 / NW;   // DMA instructions per wave and stage
  static constexpr int P = PWA + PWB;
  static_assert(IMGA % (1024 * NW) == 0 && IMGB % (1024 * NW) == 0, "images must split evenly over the waves");
  static_assert(NST >= 3 && NST * STAGE <= 160 * 1024, "ring too large for the LDS");
};

// Fragment over k rows [k0, k0+16) of an image with RB-byte rows (wg_frag's map).
template <int RB>
__device__ __forceinline__ bf16x8 ring_frag(const char* img, int k0, int c0, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int col = c0 + 16 * (g & 1) + 4 * (i & 3);
  const int row = k0 + 4 * (g >> 1) + (i >> 2);
  const int sub = 2 * (col & 7);
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4*)(img + row * RB + 16 * ((col >> 3) ^ wg_swz(row)) + sub));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4*)(img + (row + 8) * RB + 16 * ((col >> 3) ^ wg_swz(row + 8)) + sub));
  const bf16x4 l4 = __builtin_bit_cast(bf16x4, lo), h4 = __builtin_bit_cast(bf16x4, hi);
  bf16x8 f;
  f[0] = l4[0]; f[1] = l4[1]; f[2] = l4[2]; f[3] = l4[3];
  f[4] = h4[0]; f[5] = h4[1]; f[6] = h4[2]; f[7] = h4[3];
  return f;
}

// Retire the oldest step in flight: at most `ahead` later stages (P DMA instructions
// each) may stay outstanding.
template <int P, int NST>
__device__ __forceinline__ void ring_wait(int ahead) {
  static_assert(NST - 2 <= 5, "ring_wait covers at most 5 stages ahead");
  if (ahead >= NST - 2) ahead = NST - 2;
  switch (ahead) {
    case 5: wg_wait_barrier<5 * P>(); break;
    case 4: wg_wait_barrier<4 * P>(); break;
    case 3: wg_wait_barrier<3 * P>(); break;
    case 2: wg_wait_barrier<2 * P>(); break;
    case 1: wg_wait_barrier<1 * P>(); break;
    default: wg_wait_barrier<0>(); break;
  }
}

}  // namespace grk
