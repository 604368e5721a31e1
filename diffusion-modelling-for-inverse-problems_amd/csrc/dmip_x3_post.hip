// fp32-accurate split-fp16 sampler instantiations: SAMPLER_POSTERIOR (dmip_x3.h).
#include "dmip_x3.h"

namespace dmip {

hipError_t launch_x3_sampler_post(const X3SamplerParams& p, int width, int xdim, int n_y, hipStream_t st, bool* ok) {
  *ok = true;
#define X(Wv, Dv) \
  if (width == Wv && xdim == Dv) return launch_x3_sampler_n<SAMPLER_POSTERIOR, Wv, Dv, 0>(p, n_y, st);
  X(64, 2) X(128, 2) X(256, 2) X(512, 2) X(64, 3) X(128, 3) X(256, 3) X(512, 3)
#undef X
  *ok = false;
  return hipSuccess;
}

}  // namespace dmip
