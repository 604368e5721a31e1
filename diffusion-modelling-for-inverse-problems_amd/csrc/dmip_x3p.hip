// The paired-tile 32x32 fp32x3 CDE sampler (dmip_x3p.h): instantiations and dispatch.
#include "dmip_x3p.h"

namespace dmip {

bool x3p_sampler_supported(int mode, int width, int n_hidden, int xdim) {
  return mode == SAMPLER_CDE && width == 256 && n_hidden == 3 && (xdim == 2 || xdim == 3);
}

hipError_t launch_x3p_sampler(const X3SamplerParams& p, int xdim, int n_y, hipStream_t st, bool* ok) {
  *ok = true;
  if (xdim == 2) return p.noise ? launch_x3p_sampler_t<2, true>(p, n_y, st) : launch_x3p_sampler_t<2, false>(p, n_y, st);
  if (xdim == 3) return p.noise ? launch_x3p_sampler_t<3, true>(p, n_y, st) : launch_x3p_sampler_t<3, false>(p, n_y, st);
  *ok = false;
  return hipSuccess;
}

}  // namespace dmip
