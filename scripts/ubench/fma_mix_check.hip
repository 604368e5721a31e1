#include <hip/hip_runtime.h>
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
__global__ void k(const float* in, unsigned* hi_o, unsigned* lo_o) {
  int i = threadIdx.x;
  float a = in[2*i], b = in[2*i+1];
  unsigned hi = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a, b}, f16x2));
  unsigned lo;
  asm volatile("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(lo) : "v"(hi), "v"(a));
  asm volatile("v_fma_mixhi_f16 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(lo) : "v"(hi), "v"(b));
  hi_o[i] = hi;
  lo_o[i] = lo;
}
int main() {
  const int n = 64;
  float h[2*n]; unsigned ho[n], lo[n];
  srand(3);
  for (int i = 0; i < 2*n; ++i) { float r = rand() / (float)RAND_MAX; h[i] = (i % 4 == 0) ? r * 1e-3f : (i % 4 == 1 ? r * 1e-6f : r); }
  float* d; unsigned *dh, *dl;
  hipMalloc(&d, sizeof h); hipMalloc(&dh, sizeof ho); hipMalloc(&dl, sizeof lo);
  hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
  k<<<1, n>>>(d, dh, dl);
  hipMemcpy(ho, dh, sizeof ho, hipMemcpyDeviceToHost); hipMemcpy(lo, dl, sizeof lo, hipMemcpyDeviceToHost);
  int bad = 0; double worst = 0;
  for (int i = 0; i < n; ++i) for (int p = 0; p < 2; ++p) {
    _Float16 hh = __builtin_bit_cast(f16x2, ho[i])[p], ll = __builtin_bit_cast(f16x2, lo[i])[p];
    float a = h[2*i+p];
    _Float16 eh = (_Float16)a, el = (_Float16)(a - (float)eh);
    if (__builtin_bit_cast(unsigned short, hh) != __builtin_bit_cast(unsigned short, eh) ||
        __builtin_bit_cast(unsigned short, ll) != __builtin_bit_cast(unsigned short, el)) ++bad;
    double e = fabs((double)a - (double)(float)hh - (double)(float)ll);
    if (e > worst) worst = e;
  }
  printf("fma_mix split: %d mismatches vs host split of %d; worst |a - hi - lo| = %.3e\n", bad, 2*n, worst);
  return bad != 0;
}
