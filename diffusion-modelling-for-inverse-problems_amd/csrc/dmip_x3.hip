// fp32-accurate split-fp16 networks (DMIP_PREC_F32X3): the per-y layer-1 bias prep kernel and the
// sampler dispatch. Device code: dmip_x3.h; the sampler instantiations are spread over
// dmip_x3_{cde,post,cdiffe}.hip so they compile in parallel.
#include "dmip_x3.h"

namespace dmip {
namespace x3 {

// CDE / likelihood layer-1 bias with y folded in: c (b1_u + W1_{u,y} . y), f64 accumulation, one
// rounding (the y columns do not enter the sampler's layer-1 image)
__global__ void x3_bias_prep_kernel(X3BiasPrepParams p) {
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  const int yi = blockIdx.y;
  if (u >= p.width) return;
  const float* wrow = p.w1 + (size_t)u * p.in_dim;
  double c = p.b1[u];
  for (int m = 0; m < p.ydim; ++m) c += (double)wrow[p.xdim + m] * (double)p.y[(size_t)yi * p.ydim + m];
  p.bias_y[(size_t)yi * p.width + u] = (float)((double)kTanhScale * c);
}

}  // namespace x3

hipError_t launch_x3_bias_prep(const X3BiasPrepParams& p, int n_y, hipStream_t st) {
  hipLaunchKernelGGL(x3::x3_bias_prep_kernel, dim3((unsigned)((p.width + 127) / 128), (unsigned)n_y), dim3(128), 0, st,
                     p);
  return hipGetLastError();
}

int x3_chunk_bytes(int width) {
  switch (width) {
    case 64: return x3::Shape<64>::CHUNK;
    case 128: return x3::Shape<128>::CHUNK;
    case 256: return x3::Shape<256>::CHUNK;
    case 512: return x3::Shape<512>::CHUNK;
    default: return 0;
  }
}

int x3_tiles_per_chunk(int width) {
  switch (width) {
    case 64: return x3::Shape<64>::CT;
    case 128: return x3::Shape<128>::CT;
    case 256: return x3::Shape<256>::CT;
    case 512: return x3::Shape<512>::CT;
    default: return 0;
  }
}

hipError_t launch_x3_sampler(const X3SamplerParams& p, int mode, int width, int n_hidden, int xdim, int ydim, int n_y,
                             hipStream_t st, bool* supported) {
  *supported = false;
  if (!x3_sampler_supported(mode, width, n_hidden, xdim, ydim)) return hipSuccess;
  if (mode == SAMPLER_CDE) return launch_x3_sampler_cde(p, width, xdim, n_y, st, supported);
  if (mode == SAMPLER_POSTERIOR) return launch_x3_sampler_post(p, width, xdim, n_y, st, supported);
  return launch_x3_sampler_cdiffe(p, width, xdim, ydim, n_y, st, supported);
}

// Compiled: widths 64 / 128 / 256 / 512, 1 to 3 hidden layers (a runtime count), xdim 2 or 3 (CDE,
// Posterior: any ydim -- y is folded into layer 1's bias); CDiffE for (xdim, ydim) = (2, 2) and (3, 23) at
// every width (at width 512 the 27-input layer-1 image, 96 KiB, streams through the weight ring: L1R).
bool x3_sampler_supported(int mode, int width, int n_hidden, int xdim, int ydim) {
  if (n_hidden < 1 || n_hidden > x3::kMaxHidden) return false;
  if (width != 64 && width != 128 && width != 256 && width != 512) return false;
  if (mode == SAMPLER_CDE || mode == SAMPLER_POSTERIOR) return xdim == 2 || xdim == 3;
  if (mode == SAMPLER_CDIFFE) return (xdim == 2 && ydim == 2) || (xdim == 3 && ydim == 23);
  return false;
}

}  // namespace dmip
