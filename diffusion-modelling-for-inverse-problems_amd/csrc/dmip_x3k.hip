// The k-major multi-tile fp32x3 CDE sampler (dmip_x3k.h): instantiations and dispatch.
#include "dmip_x3k.h"

#include <cstdlib>

namespace dmip {

// Development knob (not part of the ABI): DMIP_X3K_NT = 1 | 2 | 3 chain tiles per wave (default 3; all three are
// covered by tests/test_gpu_x3k.py).
static int x3k_nt() {
  const char* e = getenv("DMIP_X3K_NT");
  const int v = e ? atoi(e) : 3;
  return v == 1 || v == 2 ? v : 3;
}
#ifdef DMIP_DIAG
// Diagnostic library only (make diag; never the product build): DMIP_X3_DIAG = 1 runs the no-ring timing
// ablation (stale weights), 2 writes per-phase cycle stamps into the snapshot buffer (profiles/README.md).
static int x3k_diag() {
  const char* e = getenv("DMIP_X3_DIAG");
  return e ? atoi(e) : 0;
}
#endif

bool x3k_sampler_supported(int mode, int width, int n_hidden, int xdim) {
  return mode == SAMPLER_CDE && width == 256 && n_hidden == 3 && (xdim == 2 || xdim == 3);
}

hipError_t launch_x3k_sampler(const X3SamplerParams& p, int xdim, int n_y, hipStream_t st, bool* ok) {
  *ok = true;
  const int nt = x3k_nt();
#ifdef DMIP_DIAG
  if (x3k_diag() == 1 && xdim == 3 && !p.noise)
    return nt == 2 ? launch_x3k_sampler_t<3, 2, false, 1>(p, n_y, st) : launch_x3k_sampler_t<3, 3, false, 1>(p, n_y, st);
  // DMIP_X3_DIAG = 2: per-phase cycle stamps into the snapshot buffer (scripts/x3k_stamps.py)
  if (x3k_diag() == 2 && xdim == 3 && !p.noise && p.snap_out)
    return nt == 1   ? launch_x3k_sampler_t<3, 1, false, 2>(p, n_y, st)
           : nt == 2 ? launch_x3k_sampler_t<3, 2, false, 2>(p, n_y, st)
                     : launch_x3k_sampler_t<3, 3, false, 2>(p, n_y, st);
#endif
#define X(Dv, NTv)                                                                     \
  if (xdim == Dv && nt == NTv)                                                         \
    return p.noise ? launch_x3k_sampler_t<Dv, NTv, true>(p, n_y, st) : launch_x3k_sampler_t<Dv, NTv, false>(p, n_y, st);
  X(2, 1) X(3, 1) X(2, 2) X(3, 2) X(2, 3) X(3, 3)
#undef X
  *ok = false;
  return hipSuccess;
}

}  // namespace dmip
