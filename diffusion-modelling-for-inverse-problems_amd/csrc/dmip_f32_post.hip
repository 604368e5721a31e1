// Exact-f32 sampler instantiations: SAMPLER_POSTERIOR (dmip_f32.h).
#include "dmip_f32.h"

namespace dmip {

hipError_t launch_f32_sampler_post(const F32SamplerParams& p, int width, int xdim, int n_y, hipStream_t st, bool* ok) {
  *ok = true;
#define X(Wv, Dv) \
  if (width == Wv && xdim == Dv) return launch_f32_sampler_n<SAMPLER_POSTERIOR, Wv, Dv, 0>(p, n_y, st);
  X(64, 2) X(128, 2) X(256, 2) X(512, 2) X(64, 3) X(128, 3) X(256, 3) X(512, 3)
#undef X
  *ok = false;
  return hipSuccess;
}

}  // namespace dmip
