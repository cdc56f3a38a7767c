// In-batch sampled softmax for gfx950 (north star, no
// reference implementation -- oracle/loss.py::sampled_softmax).
//
//   z_ij = <h_i, e_j> / tau - log q_j over valid columns j, with j != i masked
//          when item_id[j] == item_id[i] (the same item is not its own negative);
//   loss = mean over valid rows of (logsumexp_j z_ij - z_ii).
// log q_j (optional, per position): the logQ correction of sampled softmax
// (Yi et al., RecSys 2019) -- the log sampling probability of column j's item,
// subtracted from every logit of that column (positive and negatives alike);
// without it log q = 0.
//
// Only valid positions (next token an item) take part, ~half of a C2 batch, so
// every kernel works on the COMPACT index space: k_ss_compact lists the valid
// positions in order (vidx, count nv on the device -- no host sync: the grids
// are sized for all positions and idle blocks leave at once) and k_ss_gather
// copies their h / e rows and ids into contiguous compact buffers, so the
// tile loops below stream plain rows.
//
// Every pass has one shape: a workgroup owns 32 compact rows of one side,
// keeps their fragments in registers and walks 32-row tiles of the other side
// staged through LDS (swizzled row image; the next tile is loaded into
// registers under the current tile's MFMAs).  The D columns are split over the
// workgroup's waves (D = 512: 4 waves x 128); each wave's partial scores over
// its D slice are summed through LDS in a fixed order, so every wave holds the
// full 32 x 32 score tile S^T (MFMA 32x32x16 bf16, a lane owns one row).
//   forward: flash-style online logsumexp over column slices (never the
//            nv x nv logits); a combine kernel merges the slices' (max, sum)
//            and reduces the loss in a fixed order;
//   backward, fused (no G matrix): with G_ij = (softmax_ij - [i == j]) * g /
//            (nv * tau),  dH = G E  (workgroups owning rows of H) and
//            dE = G^T H  (owning rows of E) in one grid, each wave
//            accumulating its D slice; G enters the MFMA as bf16 hi + lo
//            (G = hi + lo to ~2^-16 relative): fp32-level gradients.
// Deterministic: no atomics, fixed reduction orders.
#include "grk_common.h"
#include "grk_mfma.h"
#include "grk_ring.h"

namespace grk {

struct SSParams {
  const bf16_t* h; int64_t ldh;
  const bf16_t* e; int64_t lde;
  const int64_t* ids;
  const float* logq;    // optional [M] log q per position (natural log)
  float* lqc;           // [M] log2(e) * log q of the compact rows (0 without logq)
  int* vidx;            // compact index -> position (valid positions, ascending)
  int* nvp;             // number of valid positions (device)
  bf16_t *hc, *ec;      // [M, D] compact copies of the valid rows of h, e
  int64_t* idc;         // [M] their item ids
  int M;                // positions (upper bound of nv)
  float sl2;            // log2(e) / tau
  int nslices;          // forward column slices
  float *pm, *pl;       // [nslices, M] partial max / sum (log2 domain), compact rows
  float* diag;          // [M] z_ii in log2 units, compact rows
  float* lse2;          // [M] log2-domain logsumexp, compact rows
  float* lsec;          // backward at D = 512: lse2 copied into the workspace ([M + kSS2Pad])
  float* part;          // backward at D = 512: [kSSBGrid][2][64][512] partial gradients (k_ss_bwd2)
  float* partials;      // [nblocks]
  float* loss;
  const float* grad_loss;
  float* dh; int64_t lddh;  // fp32 gradients, by position
  float* de; int64_t ldde;
};

// valid positions in order -> vidx[0 .. nv), nv -> *nv and *count (one workgroup)
__global__ void __launch_bounds__(1024) k_ss_compact(const uint8_t* __restrict__ valid, int M, int* __restrict__ vidx,
                                                     int* __restrict__ nv, int32_t* __restrict__ count) {
  __shared__ int part[1024];
  const int per = (M + 1023) / 1024;
  const int b0 = min(M, (int)threadIdx.x * per), b1 = min(M, b0 + per);
  int c = 0;
  for (int i = b0; i < b1; ++i) c += valid[i] != 0;
  part[threadIdx.x] = c;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int v = (int)threadIdx.x >= off ? part[threadIdx.x - off] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  int o = part[threadIdx.x] - c;
  for (int i = b0; i < b1; ++i)
    if (valid[i]) vidx[o++] = i;
  if (threadIdx.x == 1023) {
    *nv = part[1023];
    if (count) *count = part[1023];
  }
}

// compact copies: hc[c] = h[vidx[c]], ec[c] = e[vidx[c]], idc[c] = ids[vidx[c]]
template <int D>
__global__ void __launch_bounds__(256) k_ss_gather(SSParams p) {
  constexpr int NCH = D / 8;
  const int64_t units = (int64_t)(*p.nvp) * NCH;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < units; u += stride) {
    const int c = (int)(u / NCH), ch = (int)(u % NCH);
    const int i = p.vidx[c];
    *reinterpret_cast<uint4*>(p.hc + (int64_t)c * D + ch * 8) =
        *reinterpret_cast<const uint4*>(p.h + (int64_t)i * p.ldh + ch * 8);
    *reinterpret_cast<uint4*>(p.ec + (int64_t)c * D + ch * 8) =
        *reinterpret_cast<const uint4*>(p.e + (int64_t)i * p.lde + ch * 8);
    if (ch == 0) {
      p.idc[c] = p.ids[i];
      p.lqc[c] = p.logq ? p.logq[i] * kLog2e : 0.f;
      if (p.lsec) p.lsec[c] = p.lse2[c];
    }
  }
}

// Workgroup shape: NR row groups of 32 owned rows x NW slices of the D
// columns, one wave each.  Every staged tile serves 32 * NR owned rows (the
// tiles stream from L2 / the Infinity Cache once per workgroup).
template <int D>
struct SSB {
  static constexpr int NW = D >= 128 ? 4 : D / 32;  // D slices
  static constexpr int NR = NW == 4 ? 2 : 4;        // row groups (<= 512 threads)
  static constexpr int NT = 64 * NW * NR;
  static constexpr int ROWS = 32 * NR;
  static constexpr int DQ = D / NW;                  // columns per wave (multiple of 32)
  static constexpr int KSQ = DQ / 16;
  static constexpr int NDT = DQ / 32;
};

// A tile = 32 compact rows [t0, t0 + 32) of src (zero past nv) with their ids
// (and, when lse_in, their lse2): fetch() into registers under the previous
// tile's work, put() into the swizzled LDS image between two barriers.
template <int D, int NT>
struct SSTile {
  static constexpr int NCH = D / 8;
  static constexpr int PER = (32 * NCH + NT - 1) / NT;  // 16-byte vectors per thread
  uint4 v[PER];
  int64_t id;
  float lse;
  __device__ __forceinline__ void fetch(const bf16_t* src, const int64_t* idsrc, const float* lse_in, int t0,
                                        int nv) {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int x = threadIdx.x + u * NT, row = x / NCH, c = x % NCH;
      const int tc = t0 + row;
      v[u] = make_uint4(0, 0, 0, 0);
      if (x < 32 * NCH && tc < nv) v[u] = *reinterpret_cast<const uint4*>(src + (int64_t)tc * D + c * 8);
    }
    if (threadIdx.x < 32) {
      const int tc = t0 + threadIdx.x;
      const bool ok = tc < nv;
      id = ok ? idsrc[tc] : -1;
      lse = (ok && lse_in) ? lse_in[tc] : 0.f;
    }
  }
  __device__ __forceinline__ void put(char* img, int64_t* tid, float* tlse) const {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int x = threadIdx.x + u * NT, row = x / NCH, c = x % NCH;
      if (x < 32 * NCH) *reinterpret_cast<uint4*>(img + lds_off<D>(row, c * 8)) = v[u];
    }
    if (threadIdx.x < 32) {
      tid[threadIdx.x] = id;
      tlse[threadIdx.x] = lse;
    }
  }
};

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS
// operations, not for its global loads.  __syncthreads() is a release fence +
// s_barrier, and the fence waits vmcnt(0) -- it would drain the next tile's
// prefetch at every exchange.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Forward: 4 waves x 32 compact rows of h (full-D fragments in registers, no
// cross-wave exchange) walk a slice of e's tiles.
constexpr int kSSFwdRows = 128;

template <int D, bool LQ>
__global__ void __launch_bounds__(256) k_ss_fwd(SSParams p) {
  constexpr int KS = D / 16;
  __shared__ __attribute__((aligned(16))) char img[32 * D * 2];
  __shared__ int64_t tid[32];
  __shared__ float tlse[32];
  const int nv = *p.nvp;
  const int oc0 = blockIdx.x * kSSFwdRows;
  if (oc0 >= nv) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int oc = oc0 + wave * 32 + r;
  const bool ook = oc < nv;
  const bool wave_live = oc0 + wave * 32 < nv;
  const int64_t oid = ook ? p.idc[oc] : -2;
  bf16x8 of[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) of[ks] = gload8(p.hc + (int64_t)oc * D + 16 * ks + 8 * hh, ook);
  float m = -INFINITY, l = 0.f;
  const int tiles = (nv + 31) / 32, per = (tiles + p.nslices - 1) / p.nslices;
  const int c0 = blockIdx.y * per * 32, c1 = min(nv, c0 + per * 32);
  SSTile<D, 256> tile;
  const float* lq_in = LQ ? p.lqc : nullptr;  // the tile's per-column log2 q rides in its lse slot
  if (c0 < c1) tile.fetch(p.ec, p.idc, lq_in, c0, nv);
  for (int jb = c0; jb < c1; jb += 32) {
    __syncthreads();
    tile.put(img, tid, tlse);
    __syncthreads();
    if (jb + 32 < c1) tile.fetch(p.ec, p.idc, lq_in, jb + 32, nv);  // in flight under this tile's work
    if (!wave_live) continue;
    f32x16 s = acc_zero();
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) s = mfma(lds_row8<D>(img, r, 16 * ks + 8 * hh), of[ks], s);
    const bool full = jb + 32 <= nv;
    float x[16], tmax = -INFINITY;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int jr = acc_row(k, hh), jc = jb + jr;
      const bool ok = (full || jc < nv) && (jc == oc || tid[jr] != oid);
      x[k] = ok ? (LQ ? s[k] * p.sl2 - tlse[jr] : s[k] * p.sl2) : -INFINITY;
      tmax = fmaxf(tmax, x[k]);
    }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
    const float mn = fmaxf(m, tmax);
    if (mn == -INFINITY) continue;
    float rs = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) rs += __builtin_amdgcn_exp2f(x[k] - mn);  // exp2(-inf) = 0
    rs += __shfl_xor(rs, 32);
    l = l * __builtin_amdgcn_exp2f(m - mn) + rs;
    m = mn;
  }
  if (hh == 0 && ook) {
    p.pm[(int64_t)blockIdx.y * p.M + oc] = m;
    p.pl[(int64_t)blockIdx.y * p.M + oc] = l;
  }
}

// Forward at D = 512 (BASELINE config 2; round 6): the E tiles stream through an
// LDS-DMA ring instead of being staged through registers.
//  * 8 waves x 32 compact rows of h = 256 rows per workgroup, each wave holding its
//    rows' full-D fragments (128 VGPRs) for the whole column walk, so a staged
//    32-row E tile serves 256 rows (the round-2 kernel: 128, behind two barriers
//    and a register round trip per tile);
//  * E tiles (32 rows x 1 KiB at the padded stride below, one global_load_lds_dwordx4
//    per row) plus the tile's ids and log2 q (one more DMA) land in a kSS2Nst-stage
//    ring; one barrier per tile (ring_wait);
//  * persistent workgroups, the columns cut into one slice per XCD (SS2Split below).
// Per tile a wave runs 32 MFMAs (32 ds_read_b128 of the E image) and the online
// logsumexp update of its 16 scores per lane -- the math of k_ss_fwd.
// The D = 512 tile images: 32 rows of 1 KiB at a padded stride of kSS2Row = 1040 B, so
// row r starts 4 banks after row r - 1: a fragment read (ds_read_b128, lane (r, hh)
// reads 16 bytes of row r) spreads each group of 16 lanes over all 64 banks, and
// every fragment of a tile is one lane base plus an immediate offset (an XOR swizzle
// would need an address register per fragment: the backward's accumulators and own-row
// fragments leave none).  A row lands as one contiguous 1 KiB LDS-DMA.
constexpr int kSS2Row = 1040;
__device__ __forceinline__ int ss_off(int row, int col) { return row * kSS2Row + col * 2; }
__device__ __forceinline__ bf16x8 ss_row8(const char* img, int row, int col) {
  return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(img + ss_off(row, col)));
}
// lds_tr8's transposed fragment over the ss_off image
__device__ __forceinline__ bf16x8 ss_tr8(const char* img, int row0, int col0, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int q4 = i >> 2, pp = i & 3;
  const int hh = g >> 1;
  const int col = col0 + 16 * (g & 1) + 4 * pp;
  const int ra = row0 + 4 * hh + q4;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + ss_off(ra, col)));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + ss_off(ra + 8, col)));
  bf16x4 l4 = __builtin_bit_cast(bf16x4, lo), h4 = __builtin_bit_cast(bf16x4, hi);
  bf16x8 f;
  f[0] = l4[0]; f[1] = l4[1]; f[2] = l4[2]; f[3] = l4[3];
  f[4] = h4[0]; f[5] = h4[1]; f[6] = h4[2]; f[7] = h4[3];
  return f;
}

constexpr int kSSPre = 4;                    // fragment reads in flight ahead of their MFMA
constexpr int kSS2Rows = 256;
constexpr int kSS2Nst = 4;
constexpr int kSS2Img = 32 * kSS2Row;
constexpr int kSS2Stage = kSS2Img + 1024;   // + the tile's ids (256 B) and log2 q (128 B)
constexpr int kSS2Pad = 64;                 // idc / lqc rows past M the meta DMA may read

// Work split (stream-K, XCD-sliced): the columns are cut into 8 slices, slice x is
// the work of XCD x's kSS2PerXcd persistent workgroups (blockIdx % 8 = x), so an XCD
// streams only its 1/8 of E (~1.7 MB at C2) through its own 4 MiB L2; within the slice
// the RB x tx units (256-row blocks x the slice's tiles) are cut evenly over the XCD's
// workgroups, so no CU idles through a partial last wave of workgroups (864 fixed
// workgroups on 256 CUs ran 4 rounds for 3.4 rounds of work).  A block's part of the
// slice wholly inside one workgroup leaves its (max, sum) in slot F[x][block]; a part
// cut between workgroups leaves one per piece in W[workgroup][first / last] --
// k_ss_combine merges the pieces of every slice in a fixed order.
#ifndef GRK_SS_FWD_PAIRS
#define GRK_SS_FWD_PAIRS 1   // A/B builds: 0 = one barrier per tile
#endif
constexpr int kSS2PerXcd = 32;
constexpr int kSS2Grid = 8 * kSS2PerXcd;

struct SS2Split {
  int rb, nt, tb, tx;
  int64_t units;
  __device__ SS2Split(int nv, int x) : rb((nv + kSS2Rows - 1) / kSS2Rows), nt((nv + 31) / 32) {
    tb = (int)((int64_t)x * nt / 8);
    tx = (int)((int64_t)(x + 1) * nt / 8) - tb;
    units = (int64_t)rb * tx;
  }
  __device__ int64_t start(int j) const { return (int64_t)j * units / kSS2PerXcd; }
  __device__ int owner(int64_t u) const {
    int j = (int)(u * kSS2PerXcd / max(units, (int64_t)1));
    while (j + 1 < kSS2PerXcd && start(j + 1) <= u) ++j;
    while (j > 0 && start(j) > u) --j;
    return j;
  }
};
// (max, sum) slots: F [8][rbmax * 256] then W [kSS2Grid][2][256], each as pm / pl
__device__ __forceinline__ int64_t ss2_fslot(int x, int b, int rbmax) { return ((int64_t)x * rbmax + b) * kSS2Rows; }
__device__ __forceinline__ int64_t ss2_wslot(int g, int last, int rbmax) {
  return ((int64_t)8 * rbmax + 2 * g + last) * kSS2Rows;
}

template <bool LQ>
__global__ void __launch_bounds__(512) k_ss_fwd2(SSParams p, int rbmax) {
  constexpr int D = 512, KS = D / 16, NST = kSS2Nst, P = 5;
  __shared__ __attribute__((aligned(16))) char smem[NST * kSS2Stage];
  const int nv = *p.nvp;
  const int g = blockIdx.x, x = g & 7, j = g >> 3;
  const SS2Split sp(nv, x);
  const int64_t u0 = sp.start(j), u1 = sp.start(j + 1);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const unsigned lds0 = (unsigned)__builtin_amdgcn_readfirstlane(
      (int)((unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem));
  // this lane's DMA sources: E rows 4 wave .. 4 wave + 3 of a tile (16-byte chunk
  // lane of each: rows land whole at the padded stride), and one 16-byte piece of the meta
  auto issue = [&](int t, int buf) {
    const unsigned base = lds0 + buf * kSS2Stage;
    const int t0 = t * 32;
    const int wu = __builtin_amdgcn_readfirstlane(wave);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wu * 4 + i;
      const int srow = min(t0 + row, nv - 1);
      wg_dma16(p.ec + (int64_t)srow * D + 8 * lane, base + row * kSS2Row);
    }
    const bf16_t* meta = lane >= 16 && lane < 24 ? (const bf16_t*)(p.lqc + t0 + 4 * (lane - 16))
                                                 : (const bf16_t*)(p.idc + t0 + 2 * (lane & 15));
    wg_dma16(meta, base + kSS2Img);
  };
  for (int64_t u = u0; u < u1;) {
    const int b = (int)(u / sp.tx);
    const int t0 = sp.tb + (int)(u - (int64_t)b * sp.tx);
    const int64_t ue = min(u1, (int64_t)(b + 1) * sp.tx);
    const int nt = (int)(ue - u);
    const bool whole = nt == sp.tx, first = u == u0;
    u = ue;
    const int oc0 = b * kSS2Rows;
    const int oc = oc0 + wave * 32 + r;
    const bool ook = oc < nv;
    const bool wave_live = oc0 + wave * 32 < nv;
    const int64_t oid = ook ? p.idc[oc] : -2;
    bf16x8 of[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) of[ks] = gload8(p.hc + (int64_t)oc * D + 16 * ks + 8 * hh, ook);
    lds_barrier();   // every wave is past the previous piece's reads of the ring
    float m = -INFINITY, l = 0.f;
#if GRK_SS_FWD_PAIRS
    // tile pairs: the NST = 4 slots as 2 stages of 2 tiles, one barrier per pair (the
    // next pair loads under this pair's MFMAs); an odd piece's last pair loads its
    // last tile twice (a constant DMA count per stage)
    static_assert(NST == 4, "pairs of the 4 ring slots");
    auto issue2 = [&](int st, int bf) {
      issue(t0 + 2 * st, 2 * bf);
      issue(t0 + min(2 * st + 1, nt - 1), 2 * bf + 1);
    };
    issue2(0, 0);
    const int npair = (nt + 1) / 2;
    for (int st = 0; st < npair; ++st) {
      wg_wait_barrier<0>();   // this pair landed; every wave is past the previous pair
      if (st + 1 < npair) issue2(st + 1, (st + 1) & 1);
      for (int h2 = 0; h2 < 2; ++h2) {
      const int i = 2 * st + h2;
      if (i >= nt) break;
      if (!wave_live) continue;
      const char* img = smem + (2 * (st & 1) + h2) * kSS2Stage;
#else
    for (int i = 0; i < NST - 1 && i < nt; ++i) issue(t0 + i, i);
    for (int i = 0; i < nt; ++i) {
      ring_wait<P, NST>(nt - 1 - i);
      if (i + NST - 1 < nt) issue(t0 + i + NST - 1, (i + NST - 1) % NST);
      if (!wave_live) continue;
      const char* img = smem + (i % NST) * kSS2Stage;
#endif
      const int64_t* tid = reinterpret_cast<const int64_t*>(img + kSS2Img);
      const float* tlq = reinterpret_cast<const float*>(img + kSS2Img + 256);
      // the E fragments kSSPre k-steps ahead of their MFMA (a read issued right before its
      // MFMA exposes the LDS latency on every k-step)
      f32x16 s = acc_zero();
      bf16x8 af[kSSPre];
#pragma unroll
      for (int ks = 0; ks < kSSPre; ++ks) af[ks] = ss_row8(img, r, 16 * ks + 8 * hh);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 a = af[ks % kSSPre];
        if (ks + kSSPre < KS) af[ks % kSSPre] = ss_row8(img, r, 16 * (ks + kSSPre) + 8 * hh);
        s = mfma(a, of[ks], s);
      }
      const int jb = (t0 + i) * 32;
      const bool full = jb + 32 <= nv;
      float xs[16], tmax = -INFINITY;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int jr = acc_row(k, hh), jc = jb + jr;
        // branch-free (the id is read whatever the other terms: no per-score branch)
        const int64_t tj = tid[jr];
        const bool ok = (full | (jc < nv)) & ((jc == oc) | (tj != oid));
        xs[k] = ok ? (LQ ? s[k] * p.sl2 - tlq[jr] : s[k] * p.sl2) : -INFINITY;
        tmax = fmaxf(tmax, xs[k]);
      }
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
      const float mn = fmaxf(m, tmax);
      if (mn == -INFINITY) continue;
      float rs = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) rs += __builtin_amdgcn_exp2f(xs[k] - mn);  // exp2(-inf) = 0
      rs += __shfl_xor(rs, 32);
      l = l * __builtin_amdgcn_exp2f(m - mn) + rs;
      m = mn;
    }
#if GRK_SS_FWD_PAIRS
    }
#endif
    if (hh == 0 && ook) {
      const int64_t at = (whole ? ss2_fslot(x, b, rbmax) : ss2_wslot(g, first ? 0 : 1, rbmax)) + wave * 32 + r;
      p.pm[at] = m;
      p.pl[at] = l;
    }
  }
}

// z_ii (log2 units) of every compact row: one wave per row, fixed lane order.
template <int D>
__global__ void __launch_bounds__(256) k_ss_diag(SSParams p) {
  const int nv = *p.nvp;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (c >= nv) return;
  float acc = 0.f;
  for (int d = lane; d < D; d += 64)
    acc += bf16_to_f32(p.hc[(int64_t)c * D + d]) * bf16_to_f32(p.ec[(int64_t)c * D + d]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if (lane == 0) p.diag[c] = acc * p.sl2 - p.lqc[c];
}

// Merge slices -> lse2[ic]; per-block loss partials in a fixed order.
__device__ __forceinline__ void ss_lse_add(float& mx, float& sum, float ms, float ls) {
  if (ms == -INFINITY) return;
  if (ms > mx) { sum = sum * exp2f(mx - ms) + ls; mx = ms; }
  else sum += ls * exp2f(ms - mx);
}

template <bool SPLIT>
__global__ void __launch_bounds__(256) k_ss_combine(SSParams p, int rbmax) {
  __shared__ float red[256];
  const int nv = *p.nvp;
  const int ic = blockIdx.x * blockDim.x + threadIdx.x;
  float li = 0.f;
  if (ic < nv) {
    float mx = -INFINITY, sum = 0.f;
    if constexpr (SPLIT) {   // k_ss_fwd2's slots: per slice, its piece(s) in workgroup order
      const int b = ic / kSS2Rows, row = ic % kSS2Rows;
      for (int x = 0; x < 8; ++x) {
        const SS2Split sp(nv, x);
        if (sp.tx == 0) continue;
        const int64_t x0 = (int64_t)b * sp.tx;
        const int ja = sp.owner(x0), jb = sp.owner(x0 + sp.tx - 1);
        if (ja == jb) {
          const int64_t at = ss2_fslot(x, b, rbmax) + row;
          ss_lse_add(mx, sum, p.pm[at], p.pl[at]);
          continue;
        }
        for (int jj = ja; jj <= jb; ++jj) {
          if (sp.start(jj + 1) == sp.start(jj)) continue;   // an empty range
          const int64_t at = ss2_wslot(x + 8 * jj, sp.start(jj) >= x0 ? 0 : 1, rbmax) + row;
          ss_lse_add(mx, sum, p.pm[at], p.pl[at]);
        }
      }
    } else {
      for (int s = 0; s < p.nslices; ++s) mx = fmaxf(mx, p.pm[(int64_t)s * p.M + ic]);
      for (int s = 0; s < p.nslices; ++s) {
        const float ms = p.pm[(int64_t)s * p.M + ic];
        if (ms != -INFINITY) sum += p.pl[(int64_t)s * p.M + ic] * exp2f(ms - mx);
      }
    }
    const float l2 = mx + log2f(sum);
    p.lse2[ic] = l2;
    li = (l2 - p.diag[ic]) * kLn2;
  }
  red[threadIdx.x] = li;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) p.partials[blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(1024) k_ss_finalize(SSParams p, int nblocks) {
  __shared__ double red[1024];
  double a = 0.0;
  for (int b = threadIdx.x; b < nblocks; b += blockDim.x) a += p.partials[b];
  red[threadIdx.x] = a;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const int nv = *p.nvp;
    p.loss[0] = (float)(red[0] / (nv > 0 ? nv : 1));
  }
}

// Backward: blockIdx.y = 0 owns compact rows of h (dH = G E, walking e's
// tiles), 1 owns compact rows of e (dE = G^T H, walking h's tiles).  Per tile
// and row group: each D-slice wave's 16 partial scores go to LDS; wave ws sums
// (in slice order) and turns into G the EPW = 16 / NW elements it owns, and
// hands them back as bf16 hi / lo words; every wave then multiplies the whole
// G tile into its D slice of the gradient.  The softmax math runs once per
// element, not once per wave.
template <int D>
struct SSBwdLds {
  static constexpr int NW = SSB<D>::NW, NR = SSB<D>::NR, EPW = 16 / NW;
  char img[32 * D * 2];
  float4 red[NW > 1 ? NR * NW * 4 * 64 : 1];  // partial scores [rg][wave][quad][lane]
  uint32_t gx[NR * NW * 64 * EPW];             // G words [rg][wave][lane][EPW/2 hi, EPW/2 lo]
  int64_t tid[32];
  float tlse[32];
};

template <int D>
__global__ void __launch_bounds__(SSB<D>::NT) k_ss_bwd(SSParams p) {
  constexpr int NW = SSB<D>::NW, DQ = SSB<D>::DQ, KSQ = SSB<D>::KSQ, NDT = SSB<D>::NDT;
  constexpr int EPW = 16 / NW;
  __shared__ __attribute__((aligned(16))) SSBwdLds<D> L;
  const int nv = *p.nvp;
  const int oc0 = blockIdx.x * SSB<D>::ROWS;
  if (oc0 >= nv) return;
  const bool rows = blockIdx.y == 0;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int rg = wave / NW, ws = wave % NW;
  const int oc = oc0 + rg * 32 + r;
  const bool ook = oc < nv;
  const int64_t oid = ook ? p.idc[oc] : -2;
  // exponent offset of element (row i, column j) = lse2_i + log2 q_j: the own row's part
  // here, the tile row's part staged with the tile (lse2 of h rows, or log2 q of e rows)
  const float olse = ook ? (rows ? p.lse2[oc] : (p.logq ? p.lqc[oc] : 0.f)) : 0.f;
  const bf16_t* own = rows ? p.hc : p.ec;
  const bf16_t* tsrc = rows ? p.ec : p.hc;
  const float* lse_in = rows ? (p.logq ? p.lqc : nullptr) : p.lse2;
  const int col0 = ws * DQ;
  bf16x8 of[KSQ];
#pragma unroll
  for (int ks = 0; ks < KSQ; ++ks) of[ks] = gload8(own + (int64_t)oc * D + col0 + 16 * ks + 8 * hh, ook);
  const float coef = (p.grad_loss ? *p.grad_loss : 1.f) / (float)max(nv, 1) * (p.sl2 / kLog2e);
  f32x16 acc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) acc[dt] = acc_zero();
  uint32_t* gx_mine = L.gx + ((rg * NW + ws) * 64 + lane) * EPW;
  SSTile<D, SSB<D>::NT> tile;
  tile.fetch(tsrc, p.idc, lse_in, 0, nv);
  for (int tb = 0; tb < nv; tb += 32) {
    __syncthreads();
    tile.put(L.img, L.tid, L.tlse);
    __syncthreads();
    if (tb + 32 < nv) tile.fetch(tsrc, p.idc, lse_in, tb + 32, nv);  // in flight under this tile's work
    f32x16 s = acc_zero();
#pragma unroll
    for (int ks = 0; ks < KSQ; ++ks) s = mfma(lds_row8<D>(L.img, r, col0 + 16 * ks + 8 * hh), of[ks], s);
    // this wave's elements k in [ws * EPW, (ws + 1) * EPW): full scores, slice order
    float se[EPW];
    if constexpr (NW > 1) {
      float4* red = L.red + rg * NW * 4 * 64;
#pragma unroll
      for (int q = 0; q < 4; ++q) red[(ws * 4 + q) * 64 + lane] = make_float4(s[4 * q], s[4 * q + 1], s[4 * q + 2], s[4 * q + 3]);
      lds_barrier();
#pragma unroll
      for (int q = 0; q < EPW / 4; ++q) {
        float4 t = red[(0 * 4 + ws * (EPW / 4) + q) * 64 + lane];
#pragma unroll 1
        for (int w = 1; w < NW; ++w) {
          const float4 u = red[(w * 4 + ws * (EPW / 4) + q) * 64 + lane];
          t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
        }
        se[4 * q] = t.x; se[4 * q + 1] = t.y; se[4 * q + 2] = t.z; se[4 * q + 3] = t.w;
      }
    } else {
#pragma unroll
      for (int k = 0; k < 16; ++k) se[k] = s[k];
    }
    const bool full = tb + 32 <= nv;
    float g[EPW];
#pragma unroll
    for (int e = 0; e < EPW; ++e) {
      const int k = ws * EPW + e;  // not a compile-time constant across waves: acc_row by formula
      const int tr = (k & 3) + 8 * (k >> 2) + 4 * hh, tc = tb + tr;
      const bool ok = ook && (full || tc < nv) && (tc == oc || L.tid[tr] != oid);
      const float pr = __builtin_amdgcn_exp2f(fmaf(se[e], p.sl2, -(olse + L.tlse[tr])));
      g[e] = ok ? (tc == oc ? pr - 1.f : pr) * coef : 0.f;
    }
#pragma unroll
    for (int e2 = 0; e2 < EPW / 2; ++e2) {
      const __bf16 h0 = static_cast<__bf16>(g[2 * e2]), h1 = static_cast<__bf16>(g[2 * e2 + 1]);
      const __bf16 l0 = static_cast<__bf16>(g[2 * e2] - static_cast<float>(h0));
      const __bf16 l1 = static_cast<__bf16>(g[2 * e2 + 1] - static_cast<float>(h1));
      gx_mine[e2] = (uint32_t)__builtin_bit_cast(bf16_t, h0) | ((uint32_t)__builtin_bit_cast(bf16_t, h1) << 16);
      gx_mine[EPW / 2 + e2] = (uint32_t)__builtin_bit_cast(bf16_t, l0) | ((uint32_t)__builtin_bit_cast(bf16_t, l1) << 16);
    }
    lds_barrier();
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      uint32_t hw[4], lw[4];
#pragma unroll
      for (int pp = 0; pp < 4; ++pp) {  // element pair 8 s2 + 2 pp .. + 1
        const int k = 8 * s2 + 2 * pp, w = k / EPW, kk = k % EPW;
        const uint32_t* src = L.gx + ((rg * NW + w) * 64 + lane) * EPW;
        hw[pp] = src[kk / 2];
        lw[pp] = src[EPW / 2 + kk / 2];
      }
      const bf16x8 gh = __builtin_bit_cast(bf16x8, make_uint4(hw[0], hw[1], hw[2], hw[3]));
      const bf16x8 gl = __builtin_bit_cast(bf16x8, make_uint4(lw[0], lw[1], lw[2], lw[3]));
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const bf16x8 tf = lds_tr8<D>(L.img, 16 * s2, col0 + 32 * dt, lane);
        acc[dt] = mfma(tf, gh, acc[dt]);
        acc[dt] = mfma(tf, gl, acc[dt]);
      }
    }
  }
  if (!ook) return;
  const int pos = p.vidx[oc];
  float* out = rows ? p.dh + (int64_t)pos * p.lddh : p.de + (int64_t)pos * p.ldde;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4)
      *reinterpret_cast<float4*>(out + col0 + 32 * dt + 8 * g4 + 4 * hh) =
          make_float4(acc[dt][4 * g4], acc[dt][4 * g4 + 1], acc[dt][4 * g4 + 2], acc[dt][4 * g4 + 3]);
}

// Backward at D = 512 (round 6): k_ss_bwd's decomposition -- 2 row groups of 32 own rows
// x 4 D quarters = 8 waves; per tile each wave's partial scores (8 MFMAs) go to LDS, wave
// q sums the four quarters of the EPW = 4 scores it owns (in D order), turns them into G
// (bf16 hi + lo words) and hands them back; every wave then multiplies the whole G tile
// into its 4 column blocks (16 MFMAs) -- the softmax VALU runs once per score.  What
// changed from round 2: the other side's 32-row tiles stream through a 3-stage LDS-DMA
// ring (k_ss_fwd2's padded image + meta) instead of a register round trip one tile
// ahead behind two barriers; the hand-off buffers are laid out lane-minor (conflict-free
// 16-byte accesses); the masks are branch-free; the fragment reads run ahead of their
// MFMAs.
constexpr int kSSBRg = 2;                       // row groups
constexpr int kSSBNw = 4;                       // D quarters
constexpr int kSSBEpw = 16 / kSSBNw;            // scores per lane each wave turns into G
constexpr int kSSBRows = 32 * kSSBRg;
constexpr int kSSBNst = 3;
constexpr int kSSBRed = kSSBRg * kSSBNw * 4 * 64 * 16;          // float4 partials [wave][quad][lane]
constexpr int kSSBGx = kSSBRg * kSSBNw * (kSSBEpw / 2) * 2 * 64 * 4;   // G words [wave][word][lane]

// Work split (stream-K): the 2 x RB row blocks (RB = ceil(nv / 64) per direction) times
// nt column tiles are one linear range of "units" cut evenly over kSSBGrid persistent
// workgroups (one per CU; the LDS holds one), so no CU idles through a second, partial
// wave of workgroups (426 blocks on 256 CUs at C2 ran 2 rounds for 1.66 rounds of work).
// A workgroup's range crosses at most two block boundaries: a block wholly inside it is
// written out directly; a block cut between workgroups leaves one partial per piece in
// the workspace (slot 0 = the workgroup's first piece, 1 = its last) and k_ss_bwd_fix
// sums them in workgroup order.
constexpr int kSSBGrid = 256;
constexpr int kSSBPart = kSSBRows * 512;        // floats per partial slot

struct SSBSplit {
  int rb, nt;
  int64_t units;
  __device__ SSBSplit(int nv) : rb((nv + kSSBRows - 1) / kSSBRows), nt((nv + 31) / 32) { units = (int64_t)2 * rb * nt; }
  __device__ int64_t start(int g) const { return (int64_t)g * units / kSSBGrid; }
  __device__ int owner(int64_t x) const {   // the workgroup whose range holds unit x
    int g = (int)(x * kSSBGrid / max(units, (int64_t)1));
    while (g + 1 < kSSBGrid && start(g + 1) <= x) ++g;
    while (g > 0 && start(g) > x) --g;
    return g;
  }
};

__global__ void __launch_bounds__(512) k_ss_bwd2(SSParams p) {
  constexpr int D = 512, NW = kSSBNw, DQ = D / NW, KSQ = DQ / 16, NDT = DQ / 32, NST = kSSBNst, EPW = kSSBEpw, P = 5;
  __shared__ __attribute__((aligned(16))) char smem[NST * kSS2Stage + kSSBRed + kSSBGx];
  float4* red = reinterpret_cast<float4*>(smem + NST * kSS2Stage);
  uint32_t* gx = reinterpret_cast<uint32_t*>(smem + NST * kSS2Stage + kSSBRed);
  const int nv = *p.nvp;
  const SSBSplit sp(nv);
  const int g = blockIdx.x;
  const int64_t u0 = sp.start(g), u1 = sp.start(g + 1);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int rg = wave / NW, ws = wave % NW;
  const int col0 = ws * DQ;
  const float coef = (p.grad_loss ? *p.grad_loss : 1.f) / (float)max(nv, 1) * (p.sl2 / kLog2e);
  const unsigned lds0 = (unsigned)__builtin_amdgcn_readfirstlane(
      (int)((unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem));
  const int wu = __builtin_amdgcn_readfirstlane(wave);
  float4* red_mine = red + wave * 4 * 64 + lane;                 // [wave][quad][lane]
  const float4* red_q = red + (rg * NW) * 4 * 64 + ws * 64 + lane;   // quad ws of this row group's waves
  uint32_t* gx_mine = gx + wave * EPW * 64 + lane;               // [wave][word][lane]: EPW/2 hi, EPW/2 lo
  const uint32_t* gx_grp = gx + (rg * NW) * EPW * 64 + lane;
  // The range is walked from its first block boundary on ([bnd, u1), then [u0, bnd)):
  // the blocks a workgroup starts at tile 0 then run in step with the other workgroups
  // of its XCD, which stream the same tiles at the same time through their shared L2
  // (walked from u0, every workgroup sat at its own tile offset: PMC 3.3 GB per launch).
  const int64_t bnd = u0 % sp.nt == 0 ? u0 : min(u1, (u0 / sp.nt + 1) * sp.nt);
  for (int64_t q = 0; q < u1 - u0;) {
    const int64_t u = q < u1 - bnd ? bnd + q : u0 + (q - (u1 - bnd));
    const int64_t uend = q < u1 - bnd ? u1 : bnd;
    const int blk = (int)(u / sp.nt);
    const int t0 = (int)(u - (int64_t)blk * sp.nt);
    const int64_t ue = min(uend, (int64_t)(blk + 1) * sp.nt);
    const int n = (int)(ue - u);
    const bool first = u == u0;   // slot 0: the piece holding the range's first unit
    q += n;
    const bool rows = blk < sp.rb;
    const int oc0 = (rows ? blk : blk - sp.rb) * kSSBRows;
    const int oc = oc0 + rg * 32 + r;
    const bool ook = oc < nv;
    const int64_t oid = ook ? p.idc[oc] : -2;
    const uint32_t olo = (uint32_t)oid;
    // exponent offset of element (row i, column j) = lse2_i + log2 q_j: the own row's part
    // here, the tile row's part in the tile's meta (log2 q of e rows, or lse2 of h rows)
    const float olse = ook ? (rows ? p.lsec[oc] : p.lqc[oc]) : 0.f;
    const bf16_t* own = rows ? p.hc : p.ec;
    const bf16_t* tsrc = rows ? p.ec : p.hc;
    const float* tmeta = rows ? p.lqc : p.lsec;
    bf16x8 of[KSQ];
#pragma unroll
    for (int ks = 0; ks < KSQ; ++ks) of[ks] = gload8(own + (int64_t)oc * D + col0 + 16 * ks + 8 * hh, ook);
    f32x16 acc[NDT];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) acc[dt] = acc_zero();
    auto issue = [&](int t, int buf) {   // 4 tile rows per wave + the meta (every wave, same bytes)
      const unsigned base = lds0 + buf * kSS2Stage;
      const int tr0 = t * 32;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wu * 4 + i;
        const int srow = min(tr0 + row, nv - 1);
        wg_dma16(tsrc + (int64_t)srow * D + 8 * lane, base + row * kSS2Row);
      }
      const bf16_t* meta = lane >= 16 && lane < 24 ? (const bf16_t*)(tmeta + tr0 + 4 * (lane - 16))
                                                   : (const bf16_t*)(p.idc + tr0 + 2 * (lane & 15));
      wg_dma16(meta, base + kSS2Img);
    };
    // every wave is past the previous piece's reads of the ring and hand-off buffers
    lds_barrier();
    issue(t0, 0);
    if (n > 1) issue(t0 + 1, 1);
    if (n > 1) wg_wait_barrier<P>();
    else wg_wait_barrier<0>();
    for (int i = 0; i < n; ++i) {
      const char* img = smem + (i % NST) * kSS2Stage;
      const int64_t* tid = reinterpret_cast<const int64_t*>(img + kSS2Img);
      const uint32_t* tid32 = reinterpret_cast<const uint32_t*>(img + kSS2Img);
      const float* tlse = reinterpret_cast<const float*>(img + kSS2Img + 256);
      const int tb = (t0 + i) * 32;
      f32x16 s = acc_zero();
      bf16x8 af[kSSPre];
#pragma unroll
      for (int ks = 0; ks < kSSPre; ++ks) af[ks] = ss_row8(img, r, col0 + 16 * ks + 8 * hh);
#pragma unroll
      for (int ks = 0; ks < KSQ; ++ks) {
        const bf16x8 a = af[ks % kSSPre];
        if (ks + kSSPre < KSQ) af[ks % kSSPre] = ss_row8(img, r, col0 + 16 * (ks + kSSPre) + 8 * hh);
        s = mfma(a, of[ks], s);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) red_mine[64 * q] = make_float4(s[4 * q], s[4 * q + 1], s[4 * q + 2], s[4 * q + 3]);
      // the product's fragments of the first half tile, read while the partials travel
      bf16x8 tfs[NDT];
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) tfs[dt] = ss_tr8(img, 0, col0 + 32 * dt, lane);
      lds_barrier();
      // every wave is past tile i - 1's product: its stage takes tile i + 2
      if (i + 2 < n) issue(t0 + i + 2, (i + 2) % NST);
      // this wave's EPW scores (elements 4 ws .. 4 ws + 3 = quad ws), the quarters in D order
      float se[EPW];
      {
        float4 t = red_q[0];
#pragma unroll
        for (int w = 1; w < NW; ++w) {
          const float4 v = red_q[w * 4 * 64];
          t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
        }
        se[0] = t.x; se[1] = t.y; se[2] = t.z; se[3] = t.w;
      }
      const bool full = tb + 32 <= nv;
      float gv[EPW];
      bool lodup = false;
#pragma unroll
      for (int e = 0; e < EPW; ++e) {
        // element k = 4 ws + e: acc_row = (k & 3) + 8 (k >> 2) + 4 hh = e + 8 ws + 4 hh
        const int tr = e + 8 * ws + 4 * hh, tc = tb + tr;
        const bool same = tid32[2 * tr] == olo;   // ids compared on their low words (one register)
        const bool ok = ook & (full | (tc < nv)) & ((tc == oc) | !same);
        lodup |= ook & same & (tc != oc);
        const float pr = __builtin_amdgcn_exp2f(fmaf(se[e], p.sl2, -(olse + tlse[tr])));
        gv[e] = ok ? (tc == oc ? pr - 1.f : pr) * coef : 0.f;
      }
      if (__builtin_expect(__ballot(lodup) != 0, 0)) {   // a low-word match: the full ids decide (rare)
#pragma unroll
        for (int e = 0; e < EPW; ++e) {
          const int tr = e + 8 * ws + 4 * hh, tc = tb + tr;
          const bool ok = ook & (full | (tc < nv)) & ((tc == oc) | (tid[tr] != oid));
          const float pr = __builtin_amdgcn_exp2f(fmaf(se[e], p.sl2, -(olse + tlse[tr])));
          gv[e] = ok ? (tc == oc ? pr - 1.f : pr) * coef : 0.f;
        }
      }
#pragma unroll
      for (int e2 = 0; e2 < EPW / 2; ++e2) {
        uint32_t hw, lw;
        split2(f32x2{gv[2 * e2], gv[2 * e2 + 1]}, hw, lw);
        gx_mine[64 * e2] = hw;
        gx_mine[64 * (EPW / 2 + e2)] = lw;
      }
      // tile i + 1 landed (tile i + 2 may stay in flight) and every G word is written
      if (i + 2 < n) wg_wait_barrier<P>();
      else wg_wait_barrier<0>();
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        // G words of elements 8 s2 .. 8 s2 + 7: pairs 2 pp of wave w = k / EPW
        uint32_t hw[4], lw[4];
#pragma unroll
        for (int pp = 0; pp < 4; ++pp) {
          const int k = 8 * s2 + 2 * pp, w = k / EPW, kk = k % EPW;
          hw[pp] = gx_grp[(w * EPW + kk / 2) * 64];
          lw[pp] = gx_grp[(w * EPW + EPW / 2 + kk / 2) * 64];
        }
        const bf16x8 gh = words8(hw), gl = words8(lw);
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const bf16x8 tf = tfs[dt];
          if (s2 == 0) tfs[dt] = ss_tr8(img, 16, col0 + 32 * dt, lane);   // the second half's, under these MFMAs
          acc[dt] = mfma(tf, gh, acc[dt]);
          acc[dt] = mfma(tf, gl, acc[dt]);
        }
      }
    }
    if (!ook) continue;
    float* out;
    if (t0 == 0 && n == sp.nt) {   // the whole block in this workgroup: final rows
      const int pos = p.vidx[oc];
      out = rows ? p.dh + (int64_t)pos * p.lddh : p.de + (int64_t)pos * p.ldde;
    } else {
      out = p.part + (int64_t)(2 * g + (first ? 0 : 1)) * kSSBPart + (int64_t)(rg * 32 + r) * D;
    }
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4)
        *reinterpret_cast<float4*>(out + col0 + 32 * dt + 8 * g4 + 4 * hh) =
            make_float4(acc[dt][4 * g4], acc[dt][4 * g4 + 1], acc[dt][4 * g4 + 2], acc[dt][4 * g4 + 3]);
  }
}

// The blocks k_ss_bwd2 cut between workgroups: their pieces summed in workgroup order.
// Grid: 2 x ceil(M / 64) blocks (rows, then columns), 256 threads.
__global__ void __launch_bounds__(256) k_ss_bwd_fix(SSParams p, int rbmax) {
  const int nv = *p.nvp;
  const SSBSplit sp(nv);
  const bool rows = (int)blockIdx.x < rbmax;
  const int rb = rows ? blockIdx.x : blockIdx.x - rbmax;
  if (rb >= sp.rb) return;
  const int blk = rows ? rb : sp.rb + rb;
  const int64_t x0 = (int64_t)blk * sp.nt, x1 = x0 + sp.nt - 1;
  const int ga = sp.owner(x0), gb = sp.owner(x1);
  if (ga == gb) return;   // written by its workgroup
  for (int c = threadIdx.x; c < kSSBRows * 128; c += 256) {
    const int row = c >> 7, c4 = c & 127;
    const int oc = rb * kSSBRows + row;
    if (oc >= nv) break;   // rows ascend with c
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int w = ga; w <= gb; ++w) {
      if (sp.start(w + 1) == sp.start(w)) continue;   // an empty range (units < workgroups)
      const int slot = sp.start(w) >= x0 ? 0 : 1;
      const float4 v = reinterpret_cast<const float4*>(p.part + (int64_t)(2 * w + slot) * kSSBPart + (int64_t)row * 512)[c4];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    const int pos = p.vidx[oc];
    float* out = rows ? p.dh + (int64_t)pos * p.lddh : p.de + (int64_t)pos * p.ldde;
    reinterpret_cast<float4*>(out)[c4] = t;
  }
}

// which: 0 = compaction gather + forward, 1 = compaction gather + backward
template <int D>
static int ss_launch(const SSParams& p, int which, hipStream_t s) {
  k_ss_gather<D><<<grid_for((int64_t)p.M * (D / 8), 256), 256, 0, s>>>(p);
  GRK_LAUNCH_CHECK();
  if (which == 0) {
    k_ss_diag<D><<<(unsigned)((p.M + 3) / 4), 256, 0, s>>>(p);
    GRK_LAUNCH_CHECK();
    if constexpr (D == 512) {
      const int rbmax = (p.M + kSS2Rows - 1) / kSS2Rows;
      if (p.logq) k_ss_fwd2<true><<<kSS2Grid, 512, 0, s>>>(p, rbmax);
      else k_ss_fwd2<false><<<kSS2Grid, 512, 0, s>>>(p, rbmax);
    } else {
      const dim3 grid((unsigned)((p.M + kSSFwdRows - 1) / kSSFwdRows), p.nslices);
      if (p.logq) k_ss_fwd<D, true><<<grid, 256, 0, s>>>(p);
      else k_ss_fwd<D, false><<<grid, 256, 0, s>>>(p);
    }
  } else if constexpr (D == 512) {
    k_ss_bwd2<<<kSSBGrid, 512, 0, s>>>(p);
    GRK_LAUNCH_CHECK();
    const int rbmax = (p.M + kSSBRows - 1) / kSSBRows;
    k_ss_bwd_fix<<<(unsigned)(2 * rbmax), 256, 0, s>>>(p, rbmax);
  } else {
    k_ss_bwd<D><<<dim3((unsigned)((p.M + SSB<D>::ROWS - 1) / SSB<D>::ROWS), 2), SSB<D>::NT, 0, s>>>(p);
  }
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

static int ss_dispatch(const SSParams& p, int dim, int which, hipStream_t s) {
  switch (dim) {
    case 32: return ss_launch<32>(p, which, s);
    case 64: return ss_launch<64>(p, which, s);
    case 128: return ss_launch<128>(p, which, s);
    case 256: return ss_launch<256>(p, which, s);
    case 512: return ss_launch<512>(p, which, s);
  }
  set_error("dim %d unsupported (32, 64, 128, 256, 512)", dim);
  return GRK_EUNSUPPORTED;
}

static int ss_slices(int M, int D) {
  if (D == 512) return 8;   // k_ss_fwd2: one column slice per XCD
  // forward column slices: ~1k workgroups when every position is valid
  // (half of them, ~2 per CU, at C2's ~53 % valid)
  const int rb = (M + kSSFwdRows - 1) / kSSFwdRows;
  int ns = (1024 + rb - 1) / rb;
  const int tiles = (M + 31) / 32;
  if (ns > tiles) ns = tiles;
  return ns < 1 ? 1 : ns;
}

struct SSWs {
  int* vidx;
  int* nv;
  bf16_t *hc, *ec;
  int64_t* idc;
  float *lqc, *lsec, *pm, *pl, *diag, *partials, *part;
  size_t bytes;
};

static SSWs ss_ws(char* base, int M, int D) {
  SSWs w;
  const int ns = ss_slices(M, D);
  const int nb = (M + 255) / 256;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* q = base ? base + off : nullptr;
    off += (bytes + 255) & ~(size_t)255;
    return q;
  };
  w.vidx = (int*)take((size_t)M * 4);
  w.nv = (int*)take(4);
  w.hc = (bf16_t*)take((size_t)M * D * 2);
  w.ec = (bf16_t*)take((size_t)M * D * 2);
  w.idc = (int64_t*)take((size_t)(M + kSS2Pad) * 8);   // k_ss_fwd2's meta DMA reads whole 32-row tiles
  w.lqc = (float*)take((size_t)(M + kSS2Pad) * 4);
  w.lsec = (float*)take((size_t)(M + kSS2Pad) * 4);
  // (max, sum) slots: ns slices x M rows, or k_ss_fwd2's F + W slots
  const size_t nslot = D == 512 ? ((size_t)8 * ((M + kSS2Rows - 1) / kSS2Rows) + 2 * kSS2Grid) * kSS2Rows
                                : (size_t)ns * M;
  w.pm = (float*)take(nslot * 4);
  w.pl = (float*)take(nslot * 4);
  w.diag = (float*)take((size_t)M * 4);
  w.partials = (float*)take((size_t)nb * 4);
  w.part = D == 512 ? (float*)take((size_t)kSSBGrid * 2 * kSSBPart * 4) : nullptr;
  w.bytes = off;
  return w;
}

}  // namespace grk

using namespace grk;

extern "C" size_t grk_sampled_softmax_workspace(int64_t num_rows, int dim) {
  if (num_rows <= 0 || num_rows >= (1LL << 30) || dim <= 0 || dim > 512) return 0;
  return ss_ws(nullptr, (int)num_rows, dim).bytes + 256;
}

static int ss_fill(const void* h, int64_t ldh, const void* e, int64_t lde, const int64_t* ids, const uint8_t* valid,
                   int64_t num_rows, int dim, float tau, const float* log_q, void* workspace, size_t workspace_bytes,
                   SSParams* p, SSWs* w) {
  GRK_CHECK_ARG(h && e && ids && valid, "h, e, item_ids and valid are required");
  GRK_CHECK_ARG(num_rows > 0 && num_rows < (1LL << 30), "num_rows out of range");
  GRK_CHECK_ARG(dim == 32 || dim == 64 || dim == 128 || dim == 256 || dim == 512, "dim %d unsupported", dim);
  GRK_CHECK_ARG(ldh >= dim && lde >= dim && ldh % 8 == 0 && lde % 8 == 0, "row strides must be >= dim, multiple of 8");
  GRK_CHECK_ARG(((uintptr_t)h | (uintptr_t)e) % 16 == 0, "h / e must be 16-byte aligned");
  GRK_CHECK_ARG(tau > 0.f, "temperature must be > 0");
  GRK_CHECK_ARG(workspace && workspace_bytes >= grk_sampled_softmax_workspace(num_rows, dim), "workspace too small");
  memset(p, 0, sizeof(*p));
  p->h = (const bf16_t*)h; p->ldh = ldh; p->e = (const bf16_t*)e; p->lde = lde;
  p->ids = ids; p->logq = log_q; p->M = (int)num_rows; p->sl2 = kLog2e / tau;
  p->nslices = ss_slices(p->M, dim);
  *w = ss_ws((char*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255), p->M, dim);
  p->vidx = w->vidx; p->nvp = w->nv; p->hc = w->hc; p->ec = w->ec; p->idc = w->idc; p->lqc = w->lqc;
  p->pm = w->pm; p->pl = w->pl; p->diag = w->diag; p->partials = w->partials;
  return GRK_OK;
}

extern "C" int grk_sampled_softmax_fwd(const void* h, int64_t ldh, const void* e, int64_t lde, const int64_t* item_ids,
                                       const uint8_t* valid, int64_t num_rows, int dim, float tau, const float* log_q,
                                       float* lse2,
                                       float* loss, int32_t* count, void* workspace, size_t workspace_bytes,
                                       void* stream) {
  clear_error();
  SSParams p;
  SSWs w;
  int rc = ss_fill(h, ldh, e, lde, item_ids, valid, num_rows, dim, tau, log_q, workspace, workspace_bytes, &p, &w);
  if (rc) return rc;
  GRK_CHECK_ARG(lse2 && loss && count, "lse2, loss and count are required");
  p.lse2 = lse2; p.loss = loss;
  hipStream_t s = (hipStream_t)stream;
  k_ss_compact<<<1, 1024, 0, s>>>(valid, p.M, w.vidx, w.nv, count);
  GRK_LAUNCH_CHECK();
  rc = ss_dispatch(p, dim, 0, s);
  if (rc) return rc;
  const int nb = (p.M + 255) / 256;
  if (dim == 512) k_ss_combine<true><<<nb, 256, 0, s>>>(p, (p.M + kSS2Rows - 1) / kSS2Rows);
  else k_ss_combine<false><<<nb, 256, 0, s>>>(p, 0);
  GRK_LAUNCH_CHECK();
  k_ss_finalize<<<1, 1024, 0, s>>>(p, nb);
  GRK_LAUNCH_CHECK();
  return GRK_OK;
}

extern "C" int grk_sampled_softmax_bwd(const void* h, int64_t ldh, const void* e, int64_t lde, const int64_t* item_ids,
                                       const uint8_t* valid, int64_t num_rows, int dim, float tau, const float* log_q,
                                       const float* lse2,
                                       const float* grad_loss, float* dh, int64_t lddh, float* de, int64_t ldde,
                                       void* workspace, size_t workspace_bytes, void* stream) {
  clear_error();
  SSParams p;
  SSWs w;
  int rc = ss_fill(h, ldh, e, lde, item_ids, valid, num_rows, dim, tau, log_q, workspace, workspace_bytes, &p, &w);
  if (rc) return rc;
  GRK_CHECK_ARG(lse2 && dh && de, "lse2, dh and de are required");
  GRK_CHECK_ARG(lddh >= dim && ldde >= dim && lddh % 4 == 0 && ldde % 4 == 0, "lddh / ldde must be >= dim, multiple of 4");
  GRK_CHECK_ARG(((uintptr_t)dh | (uintptr_t)de) % 16 == 0, "dh / de must be 16-byte aligned");
  p.lse2 = const_cast<float*>(lse2); p.grad_loss = grad_loss;
  if (dim == 512) { p.lsec = w.lsec; p.part = w.part; }   // k_ss_bwd2 stages the tile rows' lse2 by DMA from a padded copy
  p.dh = dh; p.lddh = lddh; p.de = de; p.ldde = ldde;
  hipStream_t s = (hipStream_t)stream;
  // rows of positions that are not valid stay zero
  GRK_CHECK_HIP(zero_async(dh, (size_t)p.M * lddh * 4, s));
  GRK_CHECK_HIP(zero_async(de, (size_t)p.M * ldde * 4, s));
  k_ss_compact<<<1, 1024, 0, s>>>(valid, p.M, w.vidx, w.nv, nullptr);
  GRK_LAUNCH_CHECK();
  return ss_dispatch(p, dim, 1, s);
}
