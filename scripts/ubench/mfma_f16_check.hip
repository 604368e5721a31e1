// Checks two facts the split-fp16 (f16x3) sampler engine relies on, on the real gfx950:
//  1. the operand lane maps of v_mfma_f32_16x16x32_f16 (lane l: A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15],
//     D[4(l>>4)+r][l&15]) -- checked with exact small-integer data and an asymmetric B;
//  2. fp16 SUBNORMAL operands are honoured (not flushed) by the f16 MFMAs (16x16x32 and 32x32x16):
//     the lo halves of split activations and weights are often below 2^-14.
// Also measures the split-product error: z = sum_k (A_hi B_hi + A_hi B_lo + A_lo B_hi) against f64.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// A [16][32], B [32][16] row-major f16 -> D [16][16] f32
__global__ void k16(const _Float16* A, const _Float16* B, float* D) {
  const int l = threadIdx.x;
  f16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = A[(l & 15) * 32 + 8 * (l >> 4) + j];
    b[j] = B[(8 * (l >> 4) + j) * 16 + (l & 15)];
  }
  f32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

// A [32][16], B [16][32] -> D [32][32]
__global__ void k32(const _Float16* A, const _Float16* B, float* D) {
  const int l = threadIdx.x;
  f16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = A[(l & 31) * 16 + 8 * (l >> 5) + j];
    b[j] = B[(8 * (l >> 5) + j) * 32 + (l & 31)];
  }
  f32x16 c = {};
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) D[((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)] = c[r];
}

// split product over K = 32 (one 16x16x32 tile, 3 MFMAs)
__global__ void ksplit(const _Float16* Ah, const _Float16* Al, const _Float16* Bh, const _Float16* Bl, float* D) {
  const int l = threadIdx.x;
  f16x8 ah, al, bh, bl;
  for (int j = 0; j < 8; ++j) {
    const int ia = (l & 15) * 32 + 8 * (l >> 4) + j, ib = (8 * (l >> 4) + j) * 16 + (l & 15);
    ah[j] = Ah[ia], al[j] = Al[ia], bh[j] = Bh[ib], bl[j] = Bl[ib];
  }
  f32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);   \
      exit(2);                                                           \
    }                                                                    \
  } while (0)

template <typename T>
T* dev(const std::vector<T>& v) {
  T* p;
  CK(hipMalloc(&p, v.size() * sizeof(T)));
  CK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return p;
}

int run16(const std::vector<_Float16>& A, const std::vector<_Float16>& B, std::vector<float>& D) {
  _Float16 *a = dev(A), *b = dev(B);
  float* d;
  CK(hipMalloc(&d, 256 * 4));
  hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, a, b, d);
  CK(hipDeviceSynchronize());
  D.resize(256);
  CK(hipMemcpy(D.data(), d, 256 * 4, hipMemcpyDeviceToHost));
  hipFree(a), hipFree(b), hipFree(d);
  return 0;
}

int run32(const std::vector<_Float16>& A, const std::vector<_Float16>& B, std::vector<float>& D) {
  _Float16 *a = dev(A), *b = dev(B);
  float* d;
  CK(hipMalloc(&d, 1024 * 4));
  hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, a, b, d);
  CK(hipDeviceSynchronize());
  D.resize(1024);
  CK(hipMemcpy(D.data(), d, 1024 * 4, hipMemcpyDeviceToHost));
  hipFree(a), hipFree(b), hipFree(d);
  return 0;
}

int main() {
  int bad = 0;
  // 1. layout: exact small integers, asymmetric B
  {
    std::vector<_Float16> A(16 * 32), B(32 * 16);
    for (int i = 0; i < 16; ++i)
      for (int k = 0; k < 32; ++k) A[i * 32 + k] = (_Float16)(float)((i * 7 + k * 3) % 11 - 5);
    for (int k = 0; k < 32; ++k)
      for (int j = 0; j < 16; ++j) B[k * 16 + j] = (_Float16)(float)((k * 5 + j * 13 + k * j) % 9 - 4);
    std::vector<float> D;
    run16(A, B, D);
    int err = 0;
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        double s = 0;
        for (int k = 0; k < 32; ++k) s += (double)(float)A[i * 32 + k] * (double)(float)B[k * 16 + j];
        if (D[i * 16 + j] != (float)s) ++err;
      }
    printf("layout 16x16x32 f16: %d mismatches of 256\n", err);
    bad += err != 0;
  }
  // 2. subnormals: A = I (rows 0..15, k = i) and B[k][j] = subnormal values
  {
    std::vector<_Float16> A(16 * 32, (_Float16)0.0f), B(32 * 16, (_Float16)0.0f);
    for (int i = 0; i < 16; ++i) A[i * 32 + i] = (_Float16)1.0f;
    int n_sub = 0, n_ok = 0;
    for (int k = 0; k < 32; ++k)
      for (int j = 0; j < 16; ++j) B[k * 16 + j] = (_Float16)(ldexpf(1.0f + (k * 16 + j) % 7, -24 + (j % 9)));
    std::vector<float> D;
    run16(A, B, D);
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        const float want = (float)B[i * 16 + j];
        if (std::fabs(want) < 6.103515625e-05f) {
          ++n_sub;
          if (D[i * 16 + j] == want) ++n_ok;
        }
      }
    printf("subnormal B (16x16x32 f16): %d of %d subnormal values exact\n", n_ok, n_sub);
    bad += n_ok != n_sub;
    // subnormal A operand too, and a product of two normals with a subnormal result
    std::vector<_Float16> A2(16 * 32, (_Float16)0.0f), B2(32 * 16, (_Float16)0.0f);
    for (int i = 0; i < 16; ++i) A2[i * 32 + i] = (_Float16)ldexpf(3.0f, -22);  // subnormal
    for (int k = 0; k < 32; ++k)
      for (int j = 0; j < 16; ++j) B2[k * 16 + j] = (_Float16)(float)(j + 1);
    run16(A2, B2, D);
    int ok2 = 0;
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) ok2 += D[i * 16 + j] == ldexpf(3.0f, -22) * (float)(j + 1);
    printf("subnormal A (16x16x32 f16): %d of 256 exact\n", ok2);
    bad += ok2 != 256;
  }
  {
    std::vector<_Float16> A(32 * 16, (_Float16)0.0f), B(16 * 32, (_Float16)0.0f);
    for (int i = 0; i < 16; ++i) A[i * 16 + i] = (_Float16)1.0f;
    for (int k = 0; k < 16; ++k)
      for (int j = 0; j < 32; ++j) B[k * 32 + j] = (_Float16)(ldexpf(1.0f + (k * 32 + j) % 5, -24 + (j % 9)));
    std::vector<float> D;
    run32(A, B, D);
    int n_sub = 0, n_ok = 0;
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 32; ++j) {
        const float want = (float)B[i * 32 + j];
        if (std::fabs(want) < 6.103515625e-05f) {
          ++n_sub;
          n_ok += D[i * 32 + j] == want;
        }
      }
    printf("subnormal B (32x32x16 f16): %d of %d subnormal values exact\n", n_ok, n_sub);
    bad += n_ok != n_sub;
  }
  // 3. split-product accuracy: random W ~ U(-0.3, 0.3), h ~ U(0, 1) (r-form activations), K = 32
  {
    srand(7);
    std::vector<double> Wd(16 * 32), Hd(32 * 16);
    std::vector<_Float16> Ah(512), Al(512), Bh(512), Bl(512);
    for (int i = 0; i < 512; ++i) {
      const float w = (float)(0.6 * rand() / (double)RAND_MAX - 0.3);
      const float h = (float)(rand() / (double)RAND_MAX) * (i % 3 == 0 ? 1e-3f : 1.0f);
      Wd[i] = w, Hd[i] = h;
      Ah[i] = (_Float16)w;
      Al[i] = (_Float16)(w - (float)Ah[i]);
      Bh[i] = (_Float16)h;
      Bl[i] = (_Float16)(h - (float)Bh[i]);
    }
    _Float16 *ah = dev(Ah), *al = dev(Al), *bh = dev(Bh), *bl = dev(Bl);
    float* d;
    CK(hipMalloc(&d, 256 * 4));
    hipLaunchKernelGGL(ksplit, dim3(1), dim3(64), 0, 0, ah, al, bh, bl, d);
    CK(hipDeviceSynchronize());
    std::vector<float> D(256);
    CK(hipMemcpy(D.data(), d, 1024, hipMemcpyDeviceToHost));
    double worst = 0, worst_f32 = 0;
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        double s = 0, sa = 0;
        float sf = 0.0f;
        for (int k = 0; k < 32; ++k) {
          s += Wd[i * 32 + k] * Hd[k * 16 + j];
          sa += std::fabs(Wd[i * 32 + k] * Hd[k * 16 + j]);
          sf = fmaf((float)Wd[i * 32 + k], (float)Hd[k * 16 + j], sf);
        }
        worst = std::fmax(worst, std::fabs(D[i * 16 + j] - s) / sa);
        worst_f32 = std::fmax(worst_f32, std::fabs(sf - s) / sa);
      }
    printf("split f16x3 product error / sum|w h|: %.3e (2^%.1f); f32 fma chain: %.3e (2^%.1f)\n", worst,
           std::log2(worst), worst_f32, std::log2(worst_f32));
  }
  printf(bad ? "FAIL\n" : "PASS\n");
  return bad ? 1 : 0;
}
