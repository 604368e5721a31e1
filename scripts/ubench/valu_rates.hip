// Microbenchmark: issue cost of the activation building blocks on gfx950 (one wave per SIMD and
// two waves per SIMD), independent chains so latency is hidden. Prints cycles per wave-instruction.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 half2_t __attribute__((ext_vector_type(2)));

#define CHAINS 8
template <int OP>
__global__ void k(float* out, int iters) {
  float v[CHAINS];
  half2_t hv[CHAINS];
  for (int c = 0; c < CHAINS; ++c) { v[c] = 0.001f * (threadIdx.x + c); hv[c] = half2_t{(_Float16)v[c], (_Float16)(v[c] * 0.5f)}; }
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      if constexpr (OP == 0) v[c] = __builtin_amdgcn_exp2f(v[c]);
      if constexpr (OP == 1) v[c] = __builtin_amdgcn_rcpf(v[c]);
      if constexpr (OP == 2) v[c] = v[c] + 1.0f;
      if constexpr (OP == 3) { float t = v[c]; asm volatile("v_cvt_pkrtz_f16_f32 %0, %1, %2" : "=v"(hv[c]) : "v"(t), "v"(t)); }
      if constexpr (OP == 4) hv[c].x = __builtin_amdgcn_rcph(hv[c].x);
      if constexpr (OP == 5) hv[c] = hv[c] + half2_t{(_Float16)1.0f, (_Float16)1.0f};
      if constexpr (OP == 6) { _Float16 x = hv[c].x; asm volatile("v_exp_f16 %0, %1" : "=v"(x) : "v"(x)); hv[c].x = x; }
      if constexpr (OP == 8) { _Float16 x = hv[c].x; asm volatile("v_rcp_f16 %0, %1" : "=v"(x) : "v"(x)); hv[c].x = x; }
      if constexpr (OP == 9) { float x = v[c]; asm volatile("v_exp_f32 %0, %1" : "=v"(x) : "v"(x)); v[c] = x; }
      if constexpr (OP == 7) v[c] = __builtin_fmaf(v[c], 1.0001f, 0.5f);
    }
  }
  long long t1 = clock64();
  float s = 0; for (int c = 0; c < CHAINS; ++c) s += v[c] + (float)hv[c].x + (float)hv[c].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) out[1 << 20] = (float)(t1 - t0);
}

template <int OP>
void run(const char* name, float* d, int threads) {
  const int iters = 4096;
  hipLaunchKernelGGL(k<OP>, dim3(256), dim3(threads), 0, 0, d, iters);
  hipDeviceSynchronize();
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL(k<OP>, dim3(256), dim3(threads), 0, 0, d, iters);
  hipEventRecord(b); hipEventSynchronize(b);
  float cyc; hipMemcpy(&cyc, d + (1 << 20), 4, hipMemcpyDeviceToHost);
  float ms; hipEventElapsedTime(&ms, a, b);
  printf("%-12s waves/SIMD=%d  clock64 cycles per wave-instr: %6.2f   (wall %.3f ms)\n", name, threads / 256, cyc / (iters * (double)CHAINS), ms);
}

int main() {
  float* d; hipMalloc(&d, (2 << 20) * sizeof(float));
  for (int t : {256, 512}) {
    run<0>("exp_f32", d, t); run<1>("rcp_f32", d, t); run<2>("add_f32", d, t); run<7>("fma_f32", d, t);
    run<6>("exp_f16asm", d, t); run<8>("rcp_f16asm", d, t); run<9>("exp_f32asm", d, t); run<4>("rcp_f16", d, t); run<5>("pk_add_f16", d, t); run<3>("cvt_pkrtz", d, t);
  }
  return 0;
}
