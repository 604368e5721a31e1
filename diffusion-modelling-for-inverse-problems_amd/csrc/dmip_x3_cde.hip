// fp32-accurate split-fp16 sampler instantiations: SAMPLER_CDE (dmip_x3.h).
#include "dmip_x3.h"
#include "dmip_x3s.h"

#include <cstdlib>

namespace dmip {

#ifdef DMIP_DIAG
// Diagnostic library only (make diag; never the product build): DMIP_X3_DIAG=d (1..7, 8, 16, 24, 32, 40) runs the timing ablation
// DIAG = d of the width-256 / width-512, xdim-3 CDE kernels (dmip_x3.h XEngine); see profiles/README.md.
static int x3_diag() {
  const char* e = getenv("DMIP_X3_DIAG");
  return e ? atoi(e) : 0;
}
#endif

bool x3s_sampler_eligible(int mode, int width, int n_hidden, int xdim, long long n_chains, int n_y) {
  X3SamplerParams q{};
  q.n_chains = n_chains;
  q.n_hidden = n_hidden;
  return mode == SAMPLER_CDE && width == 64 && (xdim == 2 || xdim == 3) && x3s_eligible(q, n_y);
}

hipError_t launch_x3_sampler_cde(const X3SamplerParams& p, int width, int xdim, int n_y, hipStream_t st, bool* ok) {
  *ok = true;
#ifdef DMIP_DIAG
  if ((width == 256 || width == 512) && xdim == 3 && !p.noise) {
    switch (x3_diag()) {
#define DG(d)                                                                                   \
  case d:                                                                                       \
    return width == 256 ? launch_x3_sampler_t<SAMPLER_CDE, 256, 3, 0, false, d>(p, n_y, st)    \
                        : launch_x3_sampler_t<SAMPLER_CDE, 512, 3, 0, false, d>(p, n_y, st);
      DG(1) DG(2) DG(3) DG(4) DG(6) DG(7) DG(8) DG(16) DG(24) DG(32) DG(40)
#undef DG
      default: break;
    }
  }
#endif
  if (width == 64 && x3s_eligible(p, n_y)) {  // the latency engine (dmip_x3s.h)
    if (xdim == 2) return launch_x3s_sampler<2>(p, n_y, st);
    if (xdim == 3) return launch_x3s_sampler<3>(p, n_y, st);
  }
  if (!p.bias_y) return hipErrorInvalidValue;  // (a caller that skipped the bias prep for the latency engine)
#define X(Wv, Dv) \
  if (width == Wv && xdim == Dv) return launch_x3_sampler_n<SAMPLER_CDE, Wv, Dv, 0>(p, n_y, st);
  X(64, 2) X(128, 2) X(256, 2) X(512, 2) X(64, 3) X(128, 3) X(256, 3) X(512, 3)
#undef X
  *ok = false;
  return hipSuccess;
}

}  // namespace dmip
