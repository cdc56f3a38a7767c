// Causal attention for wide heads (head_dim 256 / 512) on gfx950.
//
// The O1 baseline runs one head over the whole hidden width
// (model/BaseLineO1/main.py:45 num_heads=1, hidden_units up to 512 in
// BASELINE config 4); the chunked kernels of grk_attention.hip keep a whole
// head row per lane in registers, which stops at head_dim 128.  Here a
// workgroup owns 32 rows -- queries (forward, dQ) or keys (dK/dV) of one
// (batch, head) -- and its HD/64 waves split the head's columns into 64-wide
// slices (4 waves at 256, 8 at 512).  Per 32-row tile every wave forms the
// partial 32x32 score (and dP) product of its slice; the partials meet in LDS
// and wave w sums, in wave order, only the 16/NW elements per lane it owns,
// turns them into P / dS (the softmax or pointwise math runs once per element)
// and hands them back as bf16 hi / lo words; every wave then multiplies the
// whole P / dS tile into its own column slice of O / dQ / dK / dV (the
// sampled-softmax backward's scheme, grk_sampled_softmax.hip).  The forward's
// running max is exchanged per tile, its row sums once at the end.  K/V (or
// Q/dO) tiles of 32 rows x HD are prefetched into registers under the
// previous tile's work and staged through the chunked kernels' swizzled LDS
// image.  Element math, masks, dropout and the HSTU pointwise form
// are those of grk_attention.hip (same drop_keep stream, same lse / delta
// conventions), so the backward of either path reads the other's forward.
// fp32-fidelity (precise = 2): head_dim 256 / 512, opt-in (grk_attention_wide_fid.hip).
// The kernels: grk_attention_wide_kernels.h.
#include "grk_attention_wide_kernels.h"

namespace grk {

bool wide_fidelity_enabled(int hd) {
  // head_dim 256 and 512 (512: the partial products meet in rounds, WideF);
  // parity vs the fp64 oracle verified on MI355X in round 4
  return hd == 256 || hd == 512;
}

// grk_attention_wide_fid.hip
int attn_wide_fid_launch(const AttnParams& p, int hd, int which, hipStream_t s);

int attn_wide_launch(const AttnParams& p, int hd, int which, hipStream_t s) {
  if (p.precise == 2) {
    if (wide_fidelity_enabled(hd)) return attn_wide_fid_launch(p, hd, which, s);
    set_error("fp32-fidelity attention (precise = 2) is not offered for head_dim %d", hd);
    return GRK_EUNSUPPORTED;
  }
  switch (hd) {
    case 256: return wide_hd<256>(p, which, s);
    case 512: return wide_hd<512>(p, which, s);
  }
  set_error("head_dim %d unsupported (16, 32, 64, 128, 256, 512)", hd);
  return GRK_EUNSUPPORTED;
}

}  // namespace grk
