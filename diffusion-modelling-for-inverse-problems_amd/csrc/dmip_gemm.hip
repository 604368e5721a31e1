// Exact-f32 training engine on gfx950: one tiled MFMA GEMM (v_mfma_f32_16x16x4_f32, an fmaf chain)
// with fused epilogues, plus the elementwise stages of the PosteriorLoss step (A18). A network's
// training step over a batch is GEMM-shaped work and runs as GEMMs:
//   forward   Z_l = H_{l-1} W_l^T + b_l, H_l = act(Z_l), act'(Z_l) kept      (epilogue BIAS_TANH[2])
//   backward  D_{l-1} = (D_l W_l) * act'(Z_{l-1})                            (epilogue MUL_AUX)
//   gradients [dW_l | db_l] = D_l^T [H_{l-1} | 1]                              (split-K over the batch,
//             fixed-order reduction: deterministic)
// Activations are stored row-major [B][ld] with ld = width + 1 and the last column set to 1, so one
// GEMM yields a layer's weight AND bias gradient.
// Reference: nets.py:17-57 (the MLP chain, double tanh on layer 1), losses.py:293-386 (PosteriorLoss),
// models/diffusion.py:204-229 (its training loop).
#include "dmip_device.h"
#include "dmip_internal.h"

#include <algorithm>

namespace dmip {
namespace gemm {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int KB = 16;
constexpr int NT = 256;  // 4 waves: 2 x 2 wave tiles

__device__ __forceinline__ f32x4 mfma4(float a, float b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// epilogue of one output element (m, n) from the accumulated value v
template <int EPI>
__device__ __forceinline__ void epilogue_k(const GemmParams& p, long long m, int n, float v) {
  switch (EPI) {
    case GEMM_EPI_NONE:
      p.c[m * p.ldc + n] = v;
      break;
    case GEMM_EPI_BIAS:
      p.c[m * p.ldc + n] = v + p.bias[n];
      break;
    case GEMM_EPI_BIAS_TANH: {
      const float h = tanhf(v + p.bias[n]);
      p.c[m * p.ldc + n] = h;
      p.aux_out[m * p.ldaux + n] = 1.0f - h * h;
      break;
    }
    case GEMM_EPI_BIAS_TANH2: {  // the reference's first layer applies tanh twice (nets.py:21-26)
      const float t1 = tanhf(v + p.bias[n]);
      const float t2 = tanhf(t1);
      p.c[m * p.ldc + n] = t2;
      p.aux_out[m * p.ldaux + n] = (1.0f - t2 * t2) * (1.0f - t1 * t1);
      break;
    }
    case GEMM_EPI_MUL_AUX:
      p.c[m * p.ldc + n] = v * p.aux_in[m * p.ldaux + n];
      break;
    case GEMM_EPI_WGRAD:  // [dW | db]: column N-1 is the bias gradient
      if (n < p.n - 1) p.c[m * p.ldc + n] = v;
      else p.bias_out[m] = v;
      break;
    default:
      break;
  }
}

__device__ __forceinline__ void epilogue(const GemmParams& p, long long m, int n, float v) {
  switch (p.epi) {
    case GEMM_EPI_NONE: epilogue_k<GEMM_EPI_NONE>(p, m, n, v); break;
    case GEMM_EPI_BIAS: epilogue_k<GEMM_EPI_BIAS>(p, m, n, v); break;
    case GEMM_EPI_BIAS_TANH: epilogue_k<GEMM_EPI_BIAS_TANH>(p, m, n, v); break;
    case GEMM_EPI_BIAS_TANH2: epilogue_k<GEMM_EPI_BIAS_TANH2>(p, m, n, v); break;
    case GEMM_EPI_MUL_AUX: epilogue_k<GEMM_EPI_MUL_AUX>(p, m, n, v); break;
    case GEMM_EPI_WGRAD: epilogue_k<GEMM_EPI_WGRAD>(p, m, n, v); break;
    default: break;
  }
}

// C (M x N) = A (M x K) B (K x N) with A(m, k) = TA ? A[k lda + m] : A[m lda + k] and
// B(k, n) = TB ? B[n ldb + k] : B[k ldb + n]. grid.z > 1: split-K partials (raw sums) into p.part.
// Tile T x T (T = 64 or 128), 4 waves as 2 x 2 wave tiles of T/2 x T/2, i.e. (T/32)^2 MFMA tiles of
// 16 x 16 per wave; KB = 16 k per LDS slice, double-buffered with the next slice's global loads in
// flight during the MFMAs. Every output element accumulates over k in the same order whatever T, so
// both tile sizes give bit-identical results (and the split-K boundaries are multiples of KB).
// LDS rows are padded to a stride of 16 banks mod 64, so the four lane groups g of an operand read
// hit disjoint banks. T = 128 quarters the global and LDS traffic per flop of the 64 tile: the
// training GEMMs at width 512 ran at ~0.3 of the f32 MFMA peak with T = 64.
template <bool TA, bool TB, int T>
__global__ void __launch_bounds__(NT) gemm_f32_kernel(GemmParams p) {
  constexpr int TW = T / 32;         // MFMA tiles per wave per dimension
  constexpr int LDR = T + 16;        // padded LDS row (floats)
  constexpr int PER = T * KB / NT;   // elements of each operand slice loaded per thread
  __shared__ float As[2][KB][LDR];
  __shared__ float Bs[2][KB][LDR];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i = lane & 15, g = lane >> 4;
  const long long m0 = (long long)blockIdx.y * T;
  const int n0 = blockIdx.x * T;
  const int wm = (w >> 1) * (T / 2), wn = (w & 1) * (T / 2);
  // this split's k range
  const long long kchunk = ((p.k + gridDim.z - 1) / gridDim.z + KB - 1) / KB * KB;
  const long long k_lo = (long long)blockIdx.z * kchunk;
  const long long k_hi = k_lo + kchunk < p.k ? k_lo + kchunk : p.k;

  f32x4 acc[TW][TW];
#pragma unroll
  for (int a = 0; a < TW; ++a)
#pragma unroll
    for (int b = 0; b < TW; ++b) acc[a][b] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

  // global -> registers for one KB slice, PER elements of A and of B per thread. Element e = q NT + tid:
  // consecutive lanes take consecutive elements along each operand's contiguous dimension, so one
  // wave-load touches 4 rows x 64 B (k-contiguous operands) or 256 contiguous bytes
  float ra[PER], rb[PER];
  auto load = [&](long long k0) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = q * NT + tid;  // element of the T x KB slice
      int mm, kk;
      if (TA) { kk = e / T; mm = e % T; } else { mm = e / KB; kk = e % KB; }
      const long long m = m0 + mm, k = k0 + kk;
      ra[q] = (m < p.m && k < k_hi) ? (TA ? p.a[k * p.lda + m] : p.a[m * p.lda + k]) : 0.0f;
      int nn, kb;
      if (TB) { nn = e / KB; kb = e % KB; } else { kb = e / T; nn = e % T; }
      const long long n = n0 + nn, kq = k0 + kb;
      rb[q] = (n < p.n && kq < k_hi) ? (TB ? p.b[n * p.ldb + kq] : p.b[kq * p.ldb + n]) : 0.0f;
    }
  };
  auto store = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = q * NT + tid;
      int mm, kk;
      if (TA) { kk = e / T; mm = e % T; } else { mm = e / KB; kk = e % KB; }
      As[buf][kk][mm] = ra[q];
      int nn, kb;
      if (TB) { nn = e / KB; kb = e % KB; } else { kb = e / T; nn = e % T; }
      Bs[buf][kb][nn] = rb[q];
    }
  };

  int buf = 0;
  if (k_lo < k_hi) {
    load(k_lo);
    store(0);
  }
  __syncthreads();
  for (long long k0 = k_lo; k0 < k_hi; k0 += KB) {
    const bool more = k0 + KB < k_hi;
    if (more) load(k0 + KB);  // global loads of the next slice in flight during the MFMAs
#pragma unroll
    for (int ks = 0; ks < KB / 4; ++ks) {
      float av[TW], bv[TW];
#pragma unroll
      for (int a = 0; a < TW; ++a) av[a] = As[buf][ks * 4 + g][wm + a * 16 + i];
#pragma unroll
      for (int b = 0; b < TW; ++b) bv[b] = Bs[buf][ks * 4 + g][wn + b * 16 + i];
#pragma unroll
      for (int a = 0; a < TW; ++a)
#pragma unroll
        for (int b = 0; b < TW; ++b) acc[a][b] = mfma4(av[a], bv[b], acc[a][b]);
    }
    if (more) store(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }

  // lane (g, j = i) of MFMA tile (a, b) holds rows 4g + r of column j. The epilogue kind is
  // dispatched once, outside the fully unrolled element loop (a switch per element kept the loop
  // rolled and indexed the accumulators dynamically, through scratch)
  auto emit = [&](auto f) __attribute__((always_inline)) {
#pragma unroll
    for (int a = 0; a < TW; ++a)
#pragma unroll
      for (int b = 0; b < TW; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long long m = m0 + wm + a * 16 + 4 * g + r;
          const int n = n0 + wn + b * 16 + i;
          if (m < p.m && n < p.n) f(m, n, acc[a][b][r]);
        }
  };
  if (gridDim.z > 1) {
    emit([&](long long m, int n, float v) { p.part[((long long)blockIdx.z * p.m + m) * p.n + n] = v; });
    return;
  }
  switch (p.epi) {
    case GEMM_EPI_NONE: emit([&](long long m, int n, float v) { epilogue_k<GEMM_EPI_NONE>(p, m, n, v); }); break;
    case GEMM_EPI_BIAS: emit([&](long long m, int n, float v) { epilogue_k<GEMM_EPI_BIAS>(p, m, n, v); }); break;
    case GEMM_EPI_BIAS_TANH:
      emit([&](long long m, int n, float v) { epilogue_k<GEMM_EPI_BIAS_TANH>(p, m, n, v); });
      break;
    case GEMM_EPI_BIAS_TANH2:
      emit([&](long long m, int n, float v) { epilogue_k<GEMM_EPI_BIAS_TANH2>(p, m, n, v); });
      break;
    case GEMM_EPI_MUL_AUX:
      emit([&](long long m, int n, float v) { epilogue_k<GEMM_EPI_MUL_AUX>(p, m, n, v); });
      break;
    case GEMM_EPI_WGRAD: emit([&](long long m, int n, float v) { epilogue_k<GEMM_EPI_WGRAD>(p, m, n, v); }); break;
    default: break;
  }
}

// split-K: sum the partials in split order (deterministic), then the epilogue
__global__ void gemm_reduce_kernel(GemmParams p, int splits) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= p.m * p.n) return;
  float s = 0.0f;
  for (int z = 0; z < splits; ++z) s += p.part[(long long)z * p.m * p.n + e];
  epilogue(p, e / p.n, (int)(e % p.n), s);
}

// ---------------------------------------------------------------- PosteriorLoss elementwise stages
// prep: alpha, std at t (sdes.py:24-28 order), x_t = eps std + alpha x (sdes.py:37-49), the two
// network input matrices [x_t, t, 1] and [x_t, y, t, 1] (nets.py:33,54 plus the ones column)
__global__ void posterior_prep_kernel(PosteriorParams p) {
  const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= p.batch) return;
  const float t = p.t[b];
  const float al = vp_mean_weight(t, p.bmin, p.bdiff);
  const float sd = vp_std(t, p.bmin, p.bdiff);
  p.alpha[b] = al;
  p.stdv[b] = sd;
  const int D = p.xdim, M = p.ydim;
  float* pin = p.prior_in + b * (D + 2);
  float* lin = p.lik_in + b * (D + M + 2);
  for (int k = 0; k < D; ++k) {
    const float xt = __fadd_rn(__fmul_rn(p.eps[b * D + k], sd), __fmul_rn(al, p.x[b * D + k]));
    p.x_t[b * D + k] = xt;
    pin[k] = xt;
    lin[k] = xt;
  }
  for (int k = 0; k < M; ++k) lin[D + k] = p.y[b * M + k];
  pin[D] = t;
  pin[D + 1] = 1.0f;
  lin[D + M] = t;
  lin[D + M + 1] = 1.0f;
}

// x_0 = 1 / alpha * (x_t + std^2 s_prior)   (losses.py:379, the reference's operation order)
__global__ void posterior_x0_kernel(PosteriorParams p) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= p.batch * p.xdim) return;
  const long long b = e / p.xdim;
  const float sd = p.stdv[b];
  const float inv = __fdiv_rn(1.0f, p.alpha[b]);
  p.x0[e] = __fmul_rn(inv, __fadd_rn(p.x_t[e], __fmul_rn(__fmul_rn(sd, sd), p.s_prior[e])));
}

// target = u + std^2 J_s^T u (losses.py:366 with the three VJPs / VHPs combined by linearity),
// the per-row losses (losses.py:376,381) and the output adjoints of both networks
__global__ void posterior_target_kernel(PosteriorParams p) {
  const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= p.batch) return;
  const int D = p.xdim;
  const float sd = p.stdv[b], al = p.alpha[b];
  const float inv_b = 1.0f / (float)p.batch;
  float prior = 0.0f, lik = 0.0f;
  for (int k = 0; k < D; ++k) {
    const long long e = b * D + k;
    const float tgt = p.u[e] + sd * sd * p.jtu[b * (D + 1) + k];  // jtu: input gradient over [x_t, t]
    p.target[e] = tgt;
    const float rp = p.s_prior[e] * sd + p.eps[e];  // DSMLoss residual s std + eps (losses.py:42-52)
    const float rl = al * p.s_lik[e] - tgt;
    prior += rp * rp;
    lik += rl * rl;
    p.adj_prior[e] = rp * sd * inv_b;                 // d mean(0.5 |rp|^2) / d s_prior
    p.adj_lik[e] = 2.0f * p.lam * al * rl * inv_b;    // d mean(lam |rl|^2) / d s_lik
  }
  p.rows[b * 2 + 0] = 0.5f * prior;
  p.rows[b * 2 + 1] = lik;
}

// loss, PriorLoss, LikelihoodLoss: one workgroup, fixed-order tree (deterministic), f64 sums
__global__ void posterior_loss_reduce_kernel(PosteriorParams p) {
  __shared__ double sp[256], sl[256];
  double a = 0.0, c = 0.0;
  for (long long b = threadIdx.x; b < p.batch; b += 256) {
    a += p.rows[b * 2 + 0];
    c += p.rows[b * 2 + 1];
  }
  sp[threadIdx.x] = a;
  sl[threadIdx.x] = c;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      sp[threadIdx.x] += sp[threadIdx.x + s];
      sl[threadIdx.x] += sl[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double n = (double)p.batch;
    p.loss_out[1] = (float)(sp[0] / n);
    p.loss_out[2] = (float)((double)p.lam * sl[0] / n);
    p.loss_out[0] = (float)(sp[0] / n + (double)p.lam * sl[0] / n);
  }
}

// the ones column of an activation matrix [B][ld] (column ld - 1)
__global__ void ones_column_kernel(float* h, long long rows, int ld) {
  const long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < rows) h[r * ld + ld - 1] = 1.0f;
}

}  // namespace gemm

// ----------------------------------------------------------------------------------- launches
// K splits of a weight-gradient GEMM (out x (in + 1) over the n_bwd B sample rows): enough workgroups
// for ~4 per CU at any batch -- a small batch no longer runs its whole sample reduction on the few
// output tiles' workgroups -- with at least 128 rows per split; at most `cap` (the partial buffer).
int gemm_wgrad_splits(long long m, long long n, long long k, int cap) {
  const long long T = (m >= 128 && n >= 128) ? 128 : 64;
  const long long tiles = ((m + T - 1) / T) * ((n + T - 1) / T);
  long long s = (1024 + tiles - 1) / tiles;
  s = std::min(s, std::max(1LL, k / 128));
  return (int)std::max(1LL, std::min<long long>(s, cap));
}

hipError_t launch_gemm_f32(const GemmParams& p_in, bool ta, bool tb, int splits, hipStream_t st) {
  GemmParams p = p_in;
  if (p.m <= 0 || p.n <= 0) return hipSuccess;
  if (splits < 1) splits = 1;
  if (splits > 1 && !p.part) return hipErrorInvalidValue;
  // 128 x 128 tiles where both output dimensions fill them (the width-256/512 layers); 64 x 64 for the
  // narrow ones (width 64, output layers), where a 128 tile would be mostly empty
  const bool big = p.m >= 128 && p.n >= 128;
  const int T = big ? 128 : 64;
  const dim3 grid((unsigned)((p.n + T - 1) / T), (unsigned)((p.m + T - 1) / T), (unsigned)splits);
#define G(TA_, TB_)                                                                                          \
  if (ta == TA_ && tb == TB_) {                                                                              \
    if (big) hipLaunchKernelGGL((gemm::gemm_f32_kernel<TA_, TB_, 128>), grid, dim3(gemm::NT), 0, st, p);     \
    else hipLaunchKernelGGL((gemm::gemm_f32_kernel<TA_, TB_, 64>), grid, dim3(gemm::NT), 0, st, p);          \
  }
  G(false, false) G(false, true) G(true, false) G(true, true)
#undef G
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || splits == 1) return e;
  const long long n = p.m * p.n;
  hipLaunchKernelGGL(gemm::gemm_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, p, splits);
  return hipGetLastError();
}

hipError_t launch_ones_column(float* h, long long rows, int ld, hipStream_t st) {
  hipLaunchKernelGGL(gemm::ones_column_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, st, h, rows, ld);
  return hipGetLastError();
}

hipError_t launch_posterior_stage(const PosteriorParams& p, int stage, hipStream_t st) {
  const unsigned rows = (unsigned)((p.batch + 255) / 256);
  switch (stage) {
    case 0: hipLaunchKernelGGL(gemm::posterior_prep_kernel, dim3(rows), dim3(256), 0, st, p); break;
    case 1:
      hipLaunchKernelGGL(gemm::posterior_x0_kernel, dim3((unsigned)((p.batch * p.xdim + 255) / 256)), dim3(256), 0,
                         st, p);
      break;
    case 2: hipLaunchKernelGGL(gemm::posterior_target_kernel, dim3(rows), dim3(256), 0, st, p); break;
    default: hipLaunchKernelGGL(gemm::posterior_loss_reduce_kernel, dim3(1), dim3(256), 0, st, p); break;
  }
  return hipGetLastError();
}

}  // namespace dmip
