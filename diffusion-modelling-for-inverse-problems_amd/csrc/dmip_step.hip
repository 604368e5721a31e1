// The rest of a training step on the device, so one step is a handful of launches with no host work:
//  * train_draws_kernel: the batch's diffusion times (BaseClassDiffusionModel.sample_t,
//    models/diffusion.py:48-58: the debiased inverse-CDF sampler of sdeflow-light, restated in
//    sdes.py:sample_vp_truncated_q, or uniform) and the forward-diffusion noise eps (base_sde.sample's
//    randn_like, sdes.py:37-49), from the chain-keyed generator (seed, sample index, step);
//  * adam_kernel: torch.optim.Adam's update (amsgrad off, no weight decay) on the optimizer's own
//    state tensors, every parameter tensor in one launch.
#include "dmip_stepdev.h"

namespace dmip {
namespace step {

__global__ void train_draws_kernel(TrainDrawsParams p) {
  stepdev::draw_one(p, (long long)blockIdx.x * blockDim.x + threadIdx.x);
}

__global__ void adam_kernel(AdamParams p) {
  __shared__ stepdev::AdamScalars sc;  // the step's scalars once per workgroup (double pow)
  if (threadIdx.x == 0) sc = stepdev::adam_scalars(p);
  __syncthreads();
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  stepdev::adam_one(p, sc, e, stepdev::adam_grad(p, e));
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

const void* train_draws_func() { return (const void*)step::train_draws_kernel; }

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
