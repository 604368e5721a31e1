// Evaluation support: numpy.histogramdd-exact binning of samples on the device,
// feeding the histogram-KL metric of the reference's evaluate drivers
// (main_diffusion_scatterometry.py:71-102, main_diffusion_linear.py). Integer/atomic work, bound by
// the atomic rate into the (L2-resident, 75^3 x 4 B = 1.7 MB) count array; one thread per point.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dmip_internal.h"

namespace dmip {

// numpy.histogramdd(x, bins=nbins, range=(lo, hi)) per dimension: edges = linspace(lo, hi, nbins + 1)
// in float64 (edges[k] = lo + k * step, step = (hi - lo) / nbins; the last edge exactly hi); a value
// v (float32 promoted to float64) falls in bin searchsorted(edges, v, 'right') - 1, except v == hi
// which goes to the last bin; values outside [lo, hi] are dropped.
__device__ __forceinline__ int np_bin(double v, double lo, double hi, int nbins) {
  if (!(v >= lo && v <= hi)) return -1;
  if (v == hi) return nbins - 1;
  const double step = (hi - lo) / nbins;
  int k = (int)floor((v - lo) / step);
  if (k < 0) k = 0;
  if (k > nbins - 1) k = nbins - 1;
  // exact correction against the float64 edges numpy compares with
  while (k > 0 && v < lo + k * step) --k;
  while (k < nbins - 1 && v >= lo + (k + 1) * step) ++k;
  return k;
}

__global__ void histogram_kernel(const float* x, long long n, int d, int nbins, double lo, double hi,
                                 unsigned int* counts, long long hist_stride) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* p = x + ((size_t)blockIdx.y * n + i) * d;
  long long idx = 0;
  for (int k = 0; k < d; ++k) {
    const int b = np_bin((double)p[k], lo, hi, nbins);
    if (b < 0) return;
    idx = idx * nbins + b;
  }
  atomicAdd(counts + (size_t)blockIdx.y * hist_stride + idx, 1u);
}

hipError_t launch_histogram(const float* x, long long n, int d, int nbins, double lo, double hi, int n_hist,
                            unsigned int* counts, hipStream_t st) {
  long long stride = 1;
  for (int k = 0; k < d; ++k) stride *= nbins;
  dim3 grid((unsigned)((n + 255) / 256), (unsigned)n_hist);
  hipLaunchKernelGGL(histogram_kernel, grid, dim3(256), 0, st, x, n, d, nbins, lo, hi, counts, stride);
  return hipGetLastError();
}

}  // namespace dmip
