// Device bodies of the training step's elementwise work, shared by the stand-alone launches (dmip_step.hip) and
// the captured bf16 step's fused launches (dmip_train.hip: plan_prologue_kernel, loss_grad_reduce_adam_kernel).
#pragma once
#include "dmip_device.h"
#include "dmip_internal.h"

#include <cmath>

namespace dmip {
namespace stepdev {

// sample b's diffusion time (BaseClassDiffusionModel.sample_t, models/diffusion.py:48-58: the debiased
// inverse-CDF sampler of sdeflow-light, restated in sdes.py:sample_vp_truncated_q, or uniform) and forward-diffusion
// noise eps (base_sde.sample's randn_like, sdes.py:37-49), from the chain-keyed generator (seed, sample, step);
// with x_src set, also the sample's batch row into the captured graph's staging buffers
__device__ __forceinline__ void draw_one(const TrainDrawsParams& p, long long b) {
  if (b >= p.batch) return;
  const unsigned long long sid = p.stream_id + (p.draw_ctr ? *p.draw_ctr : 0ull);
  Rng r = rng_init(p.seed, (uint64_t)b, sid);
  const float u = (float)(rng_next(r) >> 8) * 0x1p-24f;  // [0, 1)
  float t;
  if (p.debias) {
    // q(t) ~ beta(t)/var(t) above t_eps, flat below (sdes.py sample_vp_truncated_q), then + 1e-4 and the
    // reference's t > T correction (models/diffusion.py:52-54)
    const float lower = p.te * p.r_te / p.Z;
    float tv;
    if (u <= lower) {
      tv = p.Z / p.r_te * u;
    } else {
      const float v = p.Z * u + p.A_te - p.te * p.r_te;
      const float Bu = v > 20.0f ? v : log1pf(expf(v));  // softplus
      tv = (-p.b + sqrtf(p.b * p.b + 2.0f * p.a * Bu)) / p.a;
    }
    t = tv + p.t_add;
    if (t > p.T) t -= p.t_add;
  } else {
    t = p.t_add + u * p.T;  // models/diffusion.py:55-57
    if (t > p.T) t = p.T - p.t_add;
  }
  p.t[b] = t;
  float n[4];
  rng_normals<4>(r, n);
  for (int k = 0; k < p.xdim; ++k) p.eps[b * p.xdim + k] = n[k];
  if (p.x_src) {
    for (int k = 0; k < p.xdim; ++k) p.x_dst[b * p.xdim + k] = p.x_src[b * p.xdim + k];
    for (int k = 0; k < p.ydim; ++k) p.y_dst[b * p.ydim + k] = p.y_src[b * p.ydim + k];
  }
}

// Adam's step-dependent scalars: lr / bc1 and sqrt(bc2), bc_i = 1 - beta_i^step -- torch's, in double as the host
// path forms them, when the step comes from the captured graph's device counter
struct AdamScalars {
  float step_size, bc2_sqrt;
};
__device__ __forceinline__ AdamScalars adam_scalars(const AdamParams& p) {
  if (!p.step_ctr) return AdamScalars{p.step_size, p.bc2_sqrt};
  const double step = (double)(*p.step_ctr + 1);
  return AdamScalars{(float)(p.lr_d / (1.0 - pow(p.beta1_d, step))), (float)sqrt(1.0 - pow(p.beta2_d, step))};
}

// torch.optim.Adam (_single_tensor_adam) on flat element e of the parameter list: m = lerp(m, g, 1 - beta1);
// v = beta2 v + (1 - beta2) g^2; p -= (lr / bc1) m / (sqrt(v) / sqrt(bc2) + eps).
// g: the element's gradient (the caller may have it in a register already)
__device__ __forceinline__ void adam_one(const AdamParams& p, const AdamScalars& sc, long long e, float g) {
  int k = 0;
  while (k < p.n - 1 && e >= p.off[k + 1]) ++k;
  if (e >= p.off[p.n]) return;
  const long long i = e - p.off[k];
  float m = p.m[k][i], v = p.v[k][i];
  m = p.w1 < 0.5f ? m + p.w1 * (g - m) : g - (g - m) * (1.0f - p.w1);  // torch's lerp(m, g, w1)
  v = __fmul_rn(v, p.beta2) + __fmul_rn(p.w2 * g, g);  // mul_(beta2).addcmul_(g, g, value=w2)
  p.m[k][i] = m;
  p.v[k][i] = v;
  const float denom = sqrtf(v) / sc.bc2_sqrt + p.eps;
  p.param[k][i] = p.param[k][i] - sc.step_size * (m / denom);
}

// the element's gradient as adam_kernel reads it (the flat index e into tensor k's .grad)
__device__ __forceinline__ float adam_grad(const AdamParams& p, long long e) {
  int k = 0;
  while (k < p.n - 1 && e >= p.off[k + 1]) ++k;
  return e < p.off[p.n] ? p.grad[k][e - p.off[k]] : 0.0f;
}

}  // namespace stepdev
}  // namespace dmip
