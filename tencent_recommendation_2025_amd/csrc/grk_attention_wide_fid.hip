// fp32-fidelity (precise = 2) wide-head attention, head_dim 256 / 512: the FID
// instantiations of grk_attention_wide_kernels.h in a translation unit of
// their own (see there).  Selected by wide_fidelity_enabled (head_dim 256 / 512)
// until the parity test has run on hardware.
#include "grk_attention_wide_kernels.h"

namespace grk {

int attn_wide_fid_launch(const AttnParams& p, int hd, int which, hipStream_t s) {
  return hd == 512 ? wide_hd<512, true>(p, which, s) : wide_hd<256, true>(p, which, s);
}

}  // namespace grk
