// Cycles per v_mfma_f32_32x32x16_f16 in a dependent accumulation chain (same accumulator), AGPR form (builtin)
// vs VGPR form (inline asm, dst/srcC in VGPRs), and with 2 independent chains interleaved; one wave per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int N = 512;

template <int MODE>
__global__ void __launch_bounds__(256, 1) k(float* out, uint64_t* cyc, float seed) {
  u32x4 a = {__float_as_uint(seed), 0x3c003c00u, 0x3c00u + threadIdx.x, 0x1234u};
  u32x4 b = {0x3c003c00u, __float_as_uint(seed * 2), 0x2222u, 0x3c00u};
  f32x16 c0 = {}, c1 = {};
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; ++i) {
    if constexpr (MODE == 0) {  // builtin, one chain
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c0, 0, 0, 0);
    } else if constexpr (MODE == 1) {  // VGPR form asm, one chain
      asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(c0) : "v"(a), "v"(b));
    } else if constexpr (MODE == 2) {  // VGPR form asm, two interleaved chains
      asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(c0) : "v"(a), "v"(b));
      asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(c1) : "v"(a), "v"(b));
    } else {  // AGPR form asm, one chain
      asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(c0) : "v"(a), "v"(b));
    }
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int r = 0; r < 16; ++r) s += c0[r] + c1[r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float* out; uint64_t* cyc;
  hipMalloc(&out, 256 * 256 * 4);
  hipMalloc(&cyc, 256 * 8);
  uint64_t h[256];
  const char* names[] = {"builtin AGPR form, 1 chain", "asm VGPR form, 1 chain", "asm VGPR form, 2 chains", "asm AGPR form, 1 chain"};
  for (int m = 0; m < 4; ++m) {
    for (int rep = 0; rep < 3; ++rep) {
      if (m == 0) hipLaunchKernelGGL(k<0>, dim3(256), dim3(256), 0, 0, out, cyc, 1.0f);
      if (m == 1) hipLaunchKernelGGL(k<1>, dim3(256), dim3(256), 0, 0, out, cyc, 1.0f);
      if (m == 2) hipLaunchKernelGGL(k<2>, dim3(256), dim3(256), 0, 0, out, cyc, 1.0f);
      if (m == 3) hipLaunchKernelGGL(k<3>, dim3(256), dim3(256), 0, 0, out, cyc, 1.0f);
      hipDeviceSynchronize();
    }
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double s = 0; for (int i = 0; i < 256; ++i) s += h[i];
    const int n = (m == 2 ? 2 : 1) * N;
    printf("%-28s %.1f cycles per MFMA\n", names[m], s / 256 / n);
  }
  return 0;
}
