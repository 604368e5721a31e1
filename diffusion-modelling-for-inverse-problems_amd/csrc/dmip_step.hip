// The rest of a training step on the device, so one step is a handful of launches with no host work:
//  * train_draws_kernel: the batch's diffusion times (BaseClassDiffusionModel.sample_t,
//    models/diffusion.py:48-58: the debiased inverse-CDF sampler of sdeflow-light, restated in
//    sdes.py:sample_vp_truncated_q, or uniform) and the forward-diffusion noise eps (base_sde.sample's
//    randn_like, sdes.py:37-49), from the chain-keyed generator (seed, sample index, step);
//  * adam_kernel: torch.optim.Adam's update (amsgrad off, no weight decay) on the optimizer's own
//    state tensors, every parameter tensor in one launch.
#include "dmip_device.h"
#include "dmip_internal.h"

#include <cmath>

namespace dmip {
namespace step {

__global__ void train_draws_kernel(TrainDrawsParams p) {
  const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
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
}

// torch.optim.Adam (_single_tensor_adam): m = lerp(m, g, 1 - beta1); v = beta2 v + (1 - beta2) g^2;
// p -= (lr / bc1) m / (sqrt(v) / sqrt(bc2) + eps), bc_i = 1 - beta_i^step
__global__ void adam_kernel(AdamParams p) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  int k = 0;
  while (k < p.n - 1 && e >= p.off[k + 1]) ++k;
  if (e >= p.off[p.n]) return;
  const long long i = e - p.off[k];
  const float g = p.grad[k][i];
  float m = p.m[k][i], v = p.v[k][i];
  m = p.w1 < 0.5f ? m + p.w1 * (g - m) : g - (g - m) * (1.0f - p.w1);  // torch's lerp(m, g, w1)
  v = __fmul_rn(v, p.beta2) + __fmul_rn(p.w2 * g, g);  // mul_(beta2).addcmul_(g, g, value=w2)
  p.m[k][i] = m;
  p.v[k][i] = v;
  float step_size = p.step_size, bc2_sqrt = p.bc2_sqrt;
  if (p.step_ctr) {  // torch's scalars in double, as the host path forms them
    const double step = (double)(*p.step_ctr + 1);
    step_size = (float)(p.lr_d / (1.0 - pow(p.beta1_d, step)));
    bc2_sqrt = (float)sqrt(1.0 - pow(p.beta2_d, step));
  }
  const float denom = sqrtf(v) / bc2_sqrt + p.eps;
  p.param[k][i] = p.param[k][i] - step_size * (m / denom);
}

__global__ void counters_advance_kernel(StepCounters* c) {
  if (threadIdx.x == 0) {
    c->draw += 1;
    c->step += 1;
  }
}

}  // namespace step

hipError_t launch_train_draws(const TrainDrawsParams& p, hipStream_t st) {
  hipLaunchKernelGGL(step::train_draws_kernel, dim3((unsigned)((p.batch + 255) / 256)), dim3(256), 0, st, p);
  return hipGetLastError();
}

hipError_t launch_counters_advance(StepCounters* c, hipStream_t st) {
  hipLaunchKernelGGL(step::counters_advance_kernel, dim3(1), dim3(64), 0, st, c);
  return hipGetLastError();
}

hipError_t launch_adam(const AdamParams& p, hipStream_t st) {
  const long long n = p.off[p.n];
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(step::adam_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, p);
  return hipGetLastError();
}

}  // namespace dmip
