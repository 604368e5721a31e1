// Exact-f32 sampler instantiations: SAMPLER_CDIFFE for the two problems' (xdim, ydim) (dmip_f32.h).
#include "dmip_f32.h"

namespace dmip {

hipError_t launch_f32_sampler_cdiffe(const F32SamplerParams& p, int width, int xdim, int ydim, int n_y, hipStream_t st,
                                     bool* ok) {
  *ok = true;
#define X(Wv, Dv, Mv) \
  if (width == Wv && xdim == Dv && ydim == Mv) return launch_f32_sampler_n<SAMPLER_CDIFFE, Wv, Dv, Mv>(p, n_y, st);
  X(64, 2, 2) X(128, 2, 2) X(256, 2, 2) X(512, 2, 2) X(64, 3, 23) X(128, 3, 23) X(256, 3, 23) X(512, 3, 23)
#undef X
  *ok = false;
  return hipSuccess;
}

}  // namespace dmip
