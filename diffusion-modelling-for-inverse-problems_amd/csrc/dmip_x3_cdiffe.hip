// fp32-accurate split-fp16 sampler instantiations: SAMPLER_CDIFFE (dmip_x3.h).
#include "dmip_x3.h"

namespace dmip {

hipError_t launch_x3_sampler_cdiffe(const X3SamplerParams& p, int width, int xdim, int ydim, int n_y, hipStream_t st,
                                    bool* ok) {
  *ok = true;
#define X(Wv, Dv, Mv) \
  if (width == Wv && xdim == Dv && ydim == Mv) return launch_x3_sampler_n<SAMPLER_CDIFFE, Wv, Dv, Mv>(p, n_y, st);
  X(64, 2, 2) X(128, 2, 2) X(256, 2, 2) X(512, 2, 2) X(64, 3, 23) X(128, 3, 23) X(256, 3, 23) X(512, 3, 23)
#undef X
  *ok = false;
  return hipSuccess;
}

}  // namespace dmip
