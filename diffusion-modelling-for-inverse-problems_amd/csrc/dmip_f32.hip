// Exact-f32 networks (DMIP_PREC_F32): the per-y layer-1 prep kernel, the network forward
// instantiations and the sampler dispatch. Device code: dmip_f32.h; the sampler instantiations are
// spread over dmip_f32_{cde,post,cdiffe}.hip so they compile in parallel.
#include "dmip_f32.h"

namespace dmip {
namespace f32 {

// ------------------------------------------------------------------- per-y layer-1 prep kernel
// CDE / likelihood layer 1 with y folded in: columns (x_0..x_{D-1}, t, c) with the bias column
// c_u = b1_u + W1_{u,y} . y in f64 (rounded once), image [n_y][ST][K1Q][64] as the engine reads it.
__global__ void f32_l1_prep_kernel(F32L1PrepParams p) {
  const int u = blockIdx.x * blockDim.x + threadIdx.x;  // hidden unit
  const int yi = blockIdx.y;
  if (u >= p.width) return;
  const float* wrow = p.w1 + (size_t)u * p.in_dim;
  double c = p.b1[u];
  for (int m = 0; m < p.ydim; ++m) c += (double)wrow[p.xdim + m] * (double)p.y[(size_t)yi * p.ydim + m];
  const int st = p.width / 16, o = u / 16, i = u % 16;
  float* img = p.l1y + (size_t)yi * st * p.k1q * 64;
  for (int s = 0; s < p.k1q; ++s)
    for (int gg = 0; gg < 4; ++gg) {
      const int col = 4 * s + gg;
      float val = 0.0f;
      if (col < p.xdim) val = wrow[col];
      else if (col == p.xdim) val = wrow[p.in_dim - 1];  // t
      else if (col == p.xdim + 1) val = (float)c;
      img[((size_t)o * p.k1q + s) * 64 + i + 16 * gg] = val;
    }
}

}  // namespace f32

hipError_t launch_f32_sampler(const F32SamplerParams& p, int mode, int width, int n_hidden, int xdim, int ydim,
                              int n_y, hipStream_t st, bool* supported) {
  *supported = false;
  if (n_hidden < 1 || n_hidden > f32::kMaxHidden || !f32_sampler_supported(mode, width, n_hidden, xdim, ydim))
    return hipSuccess;
  if (mode == SAMPLER_CDE) return launch_f32_sampler_cde(p, width, xdim, n_y, st, supported);
  if (mode == SAMPLER_POSTERIOR) return launch_f32_sampler_post(p, width, xdim, n_y, st, supported);
  return launch_f32_sampler_cdiffe(p, width, xdim, ydim, n_y, st, supported);
}

// Compiled: widths 64 / 128 / 256 / 512, 1 to 3 hidden layers (a runtime count), xdim 2 or 3 (CDE,
// Posterior: any ydim -- y is folded into layer 1); CDiffE for the two problems' (xdim, ydim) =
// (2, 2) and (3, 23).
bool f32_sampler_supported(int mode, int width, int n_hidden, int xdim, int ydim) {
  if (n_hidden < 1 || n_hidden > f32::kMaxHidden) return false;
  if (width != 64 && width != 128 && width != 256 && width != 512) return false;
  if (mode == SAMPLER_CDE || mode == SAMPLER_POSTERIOR) return xdim == 2 || xdim == 3;
  if (mode == SAMPLER_CDIFFE) return (xdim == 2 && ydim == 2) || (xdim == 3 && ydim == 23);
  return false;
}

// layer-1 k-steps: 2 (in_dim <= 7: every x,t and the linear problem's x,y,t network) or 8 (in_dim
// <= 31: the scatterometry x,y,t networks); output tiles: 1 (out_dim <= 16) or 2 (<= 32, CDiffE)
// any input width with in_dim + 1 <= 32 (layer-1 k-steps are a runtime count of the image); output
// tiles: 1 (out_dim <= 16) or 2 (<= 32: the CDiffE joint score)
hipError_t launch_f32_forward(const F32ForwardParams& p, int width, int ot, hipStream_t st, bool* supported) {
  *supported = true;
  if (p.n_hidden < 1 || p.n_hidden > f32::kMaxHidden || p.k1q < 1 || p.k1q > f32::kForwardK1Q) {
    *supported = false;
    return hipSuccess;
  }
  constexpr int K = f32::kForwardK1Q;
#define X(Wv, OTv)                                                                                    \
  if (width == Wv && ot == OTv)                                                                       \
    return p.act ? launch_f32_forward_t<Wv, K, OTv, 1>(p, st) : launch_f32_forward_t<Wv, K, OTv, 0>(p, st);
  X(64, 1) X(128, 1) X(256, 1) X(512, 1) X(64, 2) X(128, 2) X(256, 2) X(512, 2)
#undef X
  *supported = false;
  return hipSuccess;
}

hipError_t launch_f32_l1_prep(const F32L1PrepParams& p, int n_y, hipStream_t st) {
  hipLaunchKernelGGL(f32::f32_l1_prep_kernel, dim3((unsigned)((p.width + 127) / 128), (unsigned)n_y), dim3(128), 0, st,
                     p);
  return hipGetLastError();
}

}  // namespace dmip
