// Microbenchmark: do transcendentals (v_exp/v_rcp) overlap with plain VALU (fma/add) or with MFMA
// issued by the same / the other wave of a SIMD? Wall time per launch, 2 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
#define C 8
template <int OP>
__global__ void __launch_bounds__(512) k(float* out, int iters) {
  float v[C], u[C];
  for (int c = 0; c < C; ++c) { v[c] = 0.001f * (threadIdx.x + c); u[c] = v[c] * 0.3f; }
  f32x16 acc = {};
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (__bf16)(0.01f * j); b[j] = (__bf16)(0.02f * threadIdx.x); }
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
      if constexpr (OP == 0) v[c] = __builtin_amdgcn_exp2f(v[c]);                       // exp only
      if constexpr (OP == 1) { v[c] = __builtin_amdgcn_exp2f(v[c]); u[c] = __builtin_fmaf(u[c], 1.0001f, 0.3f); }  // exp + 1 fma
      if constexpr (OP == 2) { v[c] = __builtin_amdgcn_exp2f(v[c]); u[c] = __builtin_fmaf(u[c], 1.0001f, 0.3f);
                               u[c] = __builtin_fmaf(u[c], 0.9999f, 0.1f); u[c] = __builtin_fmaf(u[c], 1.0001f, 0.2f); }  // exp + 3 fma
      if constexpr (OP == 3) v[c] = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(v[c]));  // activation
      if constexpr (OP == 4) u[c] = __builtin_fmaf(u[c], 1.0001f, 0.3f);                 // fma only
    }
    if constexpr (OP >= 5) {
#pragma unroll
      for (int m = 0; m < 4; ++m) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
#pragma unroll
      for (int c = 0; c < C; ++c) {
        if constexpr (OP == 6) v[c] = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(v[c]));  // 4 MFMA + 8 act
        if constexpr (OP == 7) u[c] = __builtin_fmaf(u[c], 1.0001f, 0.3f);  // 4 MFMA + 8 fma
      }
    }
  }
  float s = 0; for (int c = 0; c < C; ++c) s += v[c] + u[c];
  for (int j = 0; j < 16; ++j) s += acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int OP>
void run(const char* name, float* d) {
  const int iters = 4096;
  hipLaunchKernelGGL(k<OP>, dim3(256), dim3(512), 0, 0, d, iters);
  (void)hipDeviceSynchronize();
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  float best = 1e9;
  for (int r = 0; r < 5; ++r) {
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k<OP>, dim3(256), dim3(512), 0, 0, d, iters);
    (void)hipEventRecord(b); (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
  }
  // per SIMD: 2 waves x iters x C "units"
  printf("%-22s %.3f ms   %.3f ns per unit per SIMD\n", name, best, best * 1e6 / (2.0 * iters * C));
}
int main() {
  float* d; (void)hipMalloc(&d, (1 << 20) * sizeof(float));
  run<0>("exp", d); run<4>("fma", d); run<1>("exp+fma", d); run<2>("exp+3fma", d); run<3>("act(exp,add,rcp)", d);
  run<5>("4mfma", d); run<6>("4mfma+8act", d); run<7>("4mfma+8fma", d);
  return 0;
}
