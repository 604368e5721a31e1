// Score-matching training losses of the CDE (DSMLoss / DSM_PDELoss / PINNLoss / PINNLoss2 with the
// ScoreFPE or conditional ScoreFPE residual, losses.py:42-290, as CDE.train_epoch calls them,
// models/diffusion.py:74-89) in exact f32 at any network width -- the reference configs' [512]*3
// included -- as stacked-stream MFMA GEMMs (dmip_gemm.hip) plus three elementwise kernels.
//
// Formulation (the oracle's, oracle/dmip_oracle.py:loss_grad): forward-mode jets through the MLP.
// Streams (blocks of B rows, stacked so that one GEMM per layer serves all of them):
//   P   primal at (x_t, y, t)
//   V   tangent along d/dt of (x_t(t), y, t) -- batch_gradient's total derivative (losses.py:20-26)
//   C   primal at (x, y, 0) -- the initial-condition score (losses.py:220)
//   E_a tangent along x_t,a (the exact divergence, losses.py:14-18); E_ac second order (grad_x of
//       the divergence inside the detached grad_x, losses.py:88-89)
// Reverse pass through P, V, C only (grad_x is detached in the reference): per layer one stacked
// GEMM for [dW | db] (the ones column of the input matrices is 1 for P and C rows, 0 for V) and one
// for the hidden adjoints, then zbar_P = d1 hbar_P + d2 z_V hbar_V, zbar_V = d1 hbar_V,
// zbar_C = d1c hbar_C.
#include "dmip_device.h"
#include "dmip_internal.h"

#include <algorithm>
#include <vector>

namespace dmip {
namespace jets {

// d/dt of mean_weight, std and g (sdes.py:21-35 differentiated; the oracle's _vp_terms)
struct VpT {
  float alpha, sd, beta, g, dalpha, dstd, dg;
};

__device__ __forceinline__ VpT vp_terms(float t, float bmin, float bdiff) {
  VpT v;
  v.alpha = vp_mean_weight(t, bmin, bdiff);
  v.sd = vp_std(t, bmin, bdiff);
  v.beta = __fadd_rn(bmin, __fmul_rn(bdiff, t));
  v.g = (float)__dsqrt_rn((double)v.beta);
  const float e = expf(-0.5f * t * t * bdiff - t * bmin);
  v.dalpha = v.alpha * (-0.5f * t * bdiff - 0.5f * bmin);
  v.dstd = e * (t * bdiff + bmin) / (2.0f * v.sd);
  v.dg = bdiff / (2.0f * v.g);
  return v;
}

// layer-0 input matrix of every stream: [nS B][in + 1], the last column the ones column
__global__ void jets_prep_kernel(JetsParams p) {
  const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= p.batch) return;
  const int D = p.xdim, M = p.ydim, IN = D + M + 1, ld = IN + 1;
  const float t = p.t[b];
  const VpT v = vp_terms(t, p.bmin, p.bdiff);
  p.scal[b * 8 + 0] = v.alpha;
  p.scal[b * 8 + 1] = v.sd;
  p.scal[b * 8 + 2] = v.beta;
  p.scal[b * 8 + 3] = v.g;
  p.scal[b * 8 + 4] = v.dg;
  const long long B = p.batch;
  auto row = [&](int blk) { return p.h[0] + ((long long)blk * B + b) * ld; };
  float* rp = row(0);
  for (int k = 0; k < D; ++k) {
    const float x = p.x[b * D + k], e = p.eps[b * D + k];
    const float xt = __fadd_rn(__fmul_rn(e, v.sd), __fmul_rn(v.alpha, x));  // sdes.py:37-49
    p.x_t[b * D + k] = xt;
    rp[k] = xt;
    if (p.blk_v >= 0) row(p.blk_v)[k] = v.dalpha * x + v.dstd * e;  // d x_t / dt
    if (p.blk_c >= 0) row(p.blk_c)[k] = x;
  }
  for (int k = 0; k < M; ++k) {
    rp[D + k] = p.y[b * M + k];
    if (p.blk_v >= 0) row(p.blk_v)[D + k] = 0.0f;
    if (p.blk_c >= 0) row(p.blk_c)[D + k] = p.y[b * M + k];
  }
  rp[IN - 1] = t;
  rp[IN] = 1.0f;
  if (p.blk_v >= 0) {
    row(p.blk_v)[IN - 1] = 1.0f;
    row(p.blk_v)[IN] = 0.0f;
  }
  if (p.blk_c >= 0) {
    row(p.blk_c)[IN - 1] = 0.0f;
    row(p.blk_c)[IN] = 1.0f;
  }
  for (int a = 0; a < p.n_e; ++a) {
    float* r = row(p.blk_e + a);
    for (int k = 0; k < ld; ++k) r[k] = k == a ? 1.0f : 0.0f;
  }
  for (int q = 0; q < p.n_pair; ++q) {
    float* r = row(p.blk_e + p.n_e + q);
    for (int k = 0; k < ld; ++k) r[k] = 0.0f;
  }
}

// hidden layer: Z [nS B][W] (no bias) -> H [nS B][W + 1] with the jets, and the reverse-pass factors
// aux [3][B][W]: d1 (P), d2 z_V (P's cross term), d1 of the C stream
__global__ void jets_act_kernel(JetsParams p, const float* Z, const float* bias, float* H, float* aux, int width,
                                int twice) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long B = p.batch;
  if (e >= B * width) return;
  const long long b = e / width;
  const int u = (int)(e % width);
  const int ldh = width + 1;
  auto zr = [&](int blk) { return Z[((long long)blk * B + b) * width + u]; };
  auto hw = [&](int blk, float v) { H[((long long)blk * B + b) * ldh + u] = v; };
  const float z = zr(0) + bias[u];
  float hn, d1, d2;
  if (twice) {  // tanh(tanh(z)) (nets.py:21-26)
    const float pz = tanhf(z);
    hn = tanhf(pz);
    const float q = 1.0f - pz * pz, k1 = 1.0f - hn * hn;
    d1 = k1 * q;
    d2 = -2.0f * q * (hn * d1 + pz * k1);
  } else {
    hn = tanhf(z);
    d1 = 1.0f - hn * hn;
    d2 = -2.0f * hn * d1;
  }
  hw(0, hn);
  aux[b * width + u] = d1;
  if (p.blk_v >= 0) {
    const float zv = zr(p.blk_v);
    hw(p.blk_v, d1 * zv);
    aux[(B + b) * width + u] = d2 * zv;
  }
  if (p.blk_c >= 0) {
    const float zc = zr(p.blk_c) + bias[u];
    float hc, d1c;
    if (twice) {
      const float pc = tanhf(zc);
      hc = tanhf(pc);
      d1c = (1.0f - hc * hc) * (1.0f - pc * pc);
    } else {
      hc = tanhf(zc);
      d1c = 1.0f - hc * hc;
    }
    hw(p.blk_c, hc);
    aux[(2 * B + b) * width + u] = d1c;
  }
  float ze[4];
  for (int a = 0; a < p.n_e; ++a) {
    ze[a] = zr(p.blk_e + a);
    hw(p.blk_e + a, d1 * ze[a]);
  }
  int q = 0;
  for (int a = 0; a < p.n_e; ++a)
    for (int c = a; c < p.n_e; ++c, ++q) hw(p.blk_e + p.n_e + q, d1 * zr(p.blk_e + p.n_e + q) + d2 * ze[a] * ze[c]);
  if (u == 0) {  // the ones column: 1 for the biased streams (P, C), 0 for the tangents
    for (int blk = 0; blk < p.n_streams; ++blk)
      H[((long long)blk * B + b) * ldh + width] = (blk == 0 || blk == p.blk_c) ? 1.0f : 0.0f;
  }
}

// per sample: the loss terms and the output adjoints of P, V, C (losses.py:42-242; the oracle's
// loss_grad). A [nS B][out] is the output layer without its bias.
__global__ void jets_loss_kernel(JetsParams p, const float* A, const float* bout) {
  const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long B = p.batch;
  if (b >= B) return;
  const int D = p.xdim, O = p.out_dim;
  const float* sc = p.scal + b * 8;
  const float al = sc[0], sd = sc[1], beta = sc[2], g = sc[3], dg = sc[4];
  auto ar = [&](int blk, int i) { return A[((long long)blk * B + b) * O + i]; };
  float s[4], dsdt[4], dls[4] = {0, 0, 0, 0}, dlv[4] = {0, 0, 0, 0};
  const float invB = 1.0f / (float)B;
  float dsm = 0.0f;
  float* zb = p.zbar;  // [nb][B][O]
  for (int i = 0; i < D; ++i) {
    const float aP = ar(0, i) + bout[i];
    const float si = aP / g;
    const float r = si * sd + p.eps[b * D + i];  // DSMLoss (losses.py:50-52)
    dsm += r * r;
    if (i >= 4) {  // DSMLoss only (the C-ABI admits D > 4 for no other loss): the adjoint directly
      zb[b * O + i] = r * sd * invB / g;
      continue;
    }
    s[i] = si;
    if (p.blk_v >= 0) dsdt[i] = ar(p.blk_v, i) / g - aP * dg / (g * g);
    if (p.has_dsm) dls[i] += r * sd * invB;
  }
  dsm *= 0.5f;
  float pde = 0.0f;
  if (p.pde == 1) {  // ScoreFPELoss, exact divergence (losses.py:77-98)
    float J[4][4], gx[4], u[4];
    for (int i = 0; i < D; ++i)
      for (int a = 0; a < D; ++a) J[i][a] = ar(p.blk_e + a, i) / g;
    auto hm = [&](int a, int c, int i) {  // second-order tangent (a <= c) of output i
      int q = 0;
      for (int aa = 0; aa < D; ++aa)
        for (int cc = aa; cc < D; ++cc, ++q)
          if (aa == a && cc == c) return ar(p.blk_e + D + q, i) / g;
      return 0.0f;
    };
    for (int j = 0; j < D; ++j) {
      float v = s[j];
      for (int i = 0; i < D; ++i)
        v += hm(i < j ? i : j, i < j ? j : i, i) + (2.0f * s[i] + p.x_t[b * D + i]) * J[i][j];
      gx[j] = v;
    }
    for (int j = 0; j < D; ++j) {
      u[j] = dsdt[j] - 0.5f * beta * gx[j];
      const float du = p.pde_l1 ? ((u[j] > 0.0f) - (u[j] < 0.0f)) / (float)D : 2.0f * u[j] / (float)D;
      pde += p.pde_l1 ? fabsf(u[j]) : u[j] * u[j];
      dlv[j] += p.lam * du * invB / g;
      dls[j] += p.lam * du * invB * (-dg / g);
    }
    pde /= (float)D;
  } else if (p.pde == 2) {  // ConditionalScoreFPELoss (losses.py:100-124)
    for (int j = 0; j < D; ++j) {
      const float sd3 = sd * sd * sd;
      const float u = sd3 * dsdt[j] - 0.5f * p.eps[b * D + j] * beta * al * al;
      const float du = p.pde_l1 ? (float)((u > 0.0f) - (u < 0.0f)) : 2.0f * u;
      pde += p.pde_l1 ? fabsf(u) : u * u;
      dlv[j] += p.lam * du * sd3 * invB / g;
      dls[j] += p.lam * du * sd3 * invB * (-dg / g);
    }
  }
  float ic = 0.0f;
  for (int i = 0; i < O; ++i) {
    if (i >= 4 && i < D) continue;  // written above
    zb[b * O + i] = i < D ? dls[i] / g : 0.0f;
    if (p.blk_v >= 0) zb[((long long)p.blk_v * B + b) * O + i] = i < D ? dlv[i] : 0.0f;
  }
  if (p.blk_c >= 0) {  // initial condition (losses.py:220-228), s_0 = a(x, y, 0) / g(0)
    const float g0 = (float)__dsqrt_rn((double)p.bmin);
    for (int i = 0; i < O; ++i) {
      float dd = 0.0f;
      if (i < D) {
        const float s0 = (ar(p.blk_c, i) + bout[i]) / g0;
        float tgt;
        if (p.ic_target) {
          tgt = p.ic_target[b * D + i];
        } else {  // the linear problem's posterior score -x + ((y - (A x + b)) Sinv^T) A (linear_problem.py:61-65)
          const float* x = p.x + b * D;
          const float* y = p.y + b * p.ydim;
          float res[2], w[2];
          for (int k = 0; k < 2; ++k) res[k] = y[k] - (p.icA[2 * k] * x[0] + p.icA[2 * k + 1] * x[1] + p.icb[k]);
          for (int k = 0; k < 2; ++k) w[k] = res[0] * p.icS[2 * k] + res[1] * p.icS[2 * k + 1];
          tgt = -x[i] + w[0] * p.icA[i] + w[1] * p.icA[2 + i];
        }
        const float dl = s0 - tgt;
        ic += p.ic_l1 ? fabsf(dl) : dl * dl;
        dd = p.lam2 * (p.ic_l1 ? (float)((dl > 0.0f) - (dl < 0.0f)) : 2.0f * dl) / (float)D;
      }
      zb[((long long)p.blk_c * B + b) * O + i] = dd * invB / g0;
    }
    ic = p.lam2 * ic / (float)D;
  }
  p.rows[b * 3 + 0] = dsm;
  p.rows[b * 3 + 1] = pde;
  p.rows[b * 3 + 2] = ic;
}

// hidden adjoints: hbar [nb B][W] -> zbar (same layout)
__global__ void jets_bwd_kernel(JetsParams p, const float* hbar, const float* aux, float* zbar, int width) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long B = p.batch;
  if (e >= B * width) return;
  const long long b = e / width;
  const int u = (int)(e % width);
  const float d1 = aux[b * width + u];
  const float hP = hbar[b * width + u];
  float zP = d1 * hP;
  if (p.blk_v >= 0) {
    const float hV = hbar[((long long)p.blk_v * B + b) * width + u];
    zP += aux[(B + b) * width + u] * hV;
    zbar[((long long)p.blk_v * B + b) * width + u] = d1 * hV;
  }
  zbar[b * width + u] = zP;
  if (p.blk_c >= 0) {
    const float hC = hbar[((long long)p.blk_c * B + b) * width + u];
    zbar[((long long)p.blk_c * B + b) * width + u] = aux[(2 * B + b) * width + u] * hC;
  }
}

// loss components: loss, PDE (lam mean), IC (lam2 included), DSM mean -- fixed-order f64 tree
__global__ void jets_reduce_kernel(JetsParams p) {
  __shared__ double s[3][256];
  double a[3] = {0.0, 0.0, 0.0};
  for (long long b = threadIdx.x; b < p.batch; b += 256)
    for (int k = 0; k < 3; ++k) a[k] += p.rows[b * 3 + k];
  for (int k = 0; k < 3; ++k) s[k][threadIdx.x] = a[k];
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
      for (int k = 0; k < 3; ++k) s[k][threadIdx.x] += s[k][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double n = (double)p.batch;
    const double dsm = s[0][0] / n, pde = (double)p.lam * s[1][0] / n, ic = s[2][0] / n;
    p.loss_out[0] = (float)((p.has_dsm ? dsm : 0.0) + (p.pde ? pde : 0.0) + (p.blk_c >= 0 ? ic : 0.0));
    p.loss_out[1] = (float)pde;
    p.loss_out[2] = (float)ic;
    p.loss_out[3] = (float)dsm;
  }
}

}  // namespace jets

// ------------------------------------------------------------------------------ orchestration
hipError_t launch_jets_loss_grad(const JetsParams& p_in, int n_hidden, const int* widths, const float* const* W,
                                 const float* const* bvec, float* grads, hipStream_t st) {
  JetsParams p = p_in;
  const long long B = p.batch;
  const int L = n_hidden, IN = p.xdim + p.ydim + 1, O = p.out_dim, nS = p.n_streams, nb = p.n_bwd;
  auto in_w = [&](int l) { return l == 0 ? IN : widths[l - 1]; };
  auto out_w = [&](int l) { return l == L ? O : widths[l]; };
  const unsigned rows_grid = (unsigned)((B + 255) / 256);
  hipError_t e;
  hipLaunchKernelGGL(jets::jets_prep_kernel, dim3(rows_grid), dim3(256), 0, st, p);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  // forward: one stacked GEMM per layer (no bias: P and C add theirs in the activation kernels)
  for (int l = 0; l <= L; ++l) {
    GemmParams g{};
    g.a = p.h[l];
    g.lda = in_w(l) + 1;
    g.b = W[l];
    g.ldb = in_w(l);
    g.m = (long long)nS * B;
    g.n = out_w(l);
    g.k = in_w(l);
    g.c = l == L ? p.a_out : p.z;
    g.ldc = out_w(l);
    g.epi = GEMM_EPI_NONE;
    if ((e = launch_gemm_f32(g, false, true, 1, st)) != hipSuccess) return e;
    if (l < L) {
      const long long n = B * widths[l];
      hipLaunchKernelGGL(jets::jets_act_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, p, p.z, bvec[l],
                         p.h[l + 1], p.aux[l], widths[l], l == 0 ? 1 : 0);
      if ((e = hipGetLastError()) != hipSuccess) return e;
    }
  }
  hipLaunchKernelGGL(jets::jets_loss_kernel, dim3(rows_grid), dim3(256), 0, st, p, p.a_out, bvec[L]);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  // reverse through P, V, C (the first nb blocks of every stacked matrix)
  std::vector<size_t> poff(L + 2, 0);  // reference parameter order: W_0, b_0, W_1, b_1, ...
  for (int l = 0; l <= L; ++l) poff[l + 1] = poff[l] + (size_t)out_w(l) * in_w(l) + out_w(l);
  const float* zb = p.zbar;
  float* bufs[2] = {p.zbar_a, p.zbar_b};
  for (int l = L; l >= 0; --l) {
    GemmParams g{};
    g.a = zb;
    g.lda = out_w(l);
    g.b = p.h[l];
    g.ldb = in_w(l) + 1;
    g.m = out_w(l);
    g.n = in_w(l) + 1;
    g.k = (long long)nb * B;
    g.c = grads + poff[l];
    g.ldc = in_w(l);
    g.epi = GEMM_EPI_WGRAD;
    g.bias_out = grads + poff[l] + (size_t)out_w(l) * in_w(l);
    g.part = p.part;
    if ((e = launch_gemm_f32(g, true, false, gemm_wgrad_splits(g.m, g.n, g.k, p.splits), st)) != hipSuccess) return e;
    if (l == 0) break;
    GemmParams h{};
    h.a = zb;
    h.lda = out_w(l);
    h.b = W[l];
    h.ldb = in_w(l);
    h.m = (long long)nb * B;
    h.n = in_w(l);
    h.k = out_w(l);
    h.c = p.hbar;
    h.ldc = in_w(l);
    h.epi = GEMM_EPI_NONE;
    if ((e = launch_gemm_f32(h, false, false, 1, st)) != hipSuccess) return e;
    float* nxt = bufs[l & 1];
    const long long n = B * in_w(l);
    hipLaunchKernelGGL(jets::jets_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, p, p.hbar,
                       p.aux[l - 1], nxt, in_w(l));
    if ((e = hipGetLastError()) != hipSuccess) return e;
    zb = nxt;
  }
  hipLaunchKernelGGL(jets::jets_reduce_kernel, dim3(1), dim3(256), 0, st, p);
  return hipGetLastError();
}

}  // namespace dmip
