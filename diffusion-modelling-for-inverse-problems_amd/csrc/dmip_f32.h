// Exact-f32 score networks on gfx950: the parity-precision (DMIP_PREC_F32) reverse-SDE samplers and
// network forward, arithmetic identical in kind to the reference's fp32 (nets.py:32-35,
// models/diffusion.py:38-42): every product and sum in f32, on the matrix cores.
//
// v_mfma_f32_16x16x4_f32 is an exact f32 fmaf chain (MI355X_MICROARCH.md: f32 in, f32 accumulate,
// no reduced-precision operands) at the f32 vector rate (157 TF). Layout (one wave = 16 chains):
//   * a layer's output tile is 16 units x 16 chains: lane (g = l >> 4, j = l & 15) holds units
//     4g + r (r = 0..3) of chain j. That tile is directly the B operand of 4 k-steps of the next
//     layer (k-step (q, r) takes register r of tile q), so activations stay in f32 registers.
//   * weight images (packed by dmip_capi.cpp): k-step (q, r) of output tile o, lane (i, g), holds
//     W[16 o + i][16 q + 4 g + r] -- one float4 (ds_read_b128) per lane feeds 4 MFMAs. A 16-row
//     tile of a W-input layer is one W*64-byte chunk; hidden layers and the output layer are
//     streamed from L2 through an R-slot LDS ring by LDS-DMA (the bf16 sampler's ring protocol);
//     layer 1 (every input column + a bias column) and the biases are LDS-resident.
//   * every lane group g of a chain carries an identical copy of its state (x, RNG), so the layer-1
//     operand (input column 4 s + g at k-step s) is a per-lane select, and the output rows (at
//     g = 0) are broadcast back with one shuffle per dimension.
// The RNG consumption per chain is the bf16 sampler's (x0, then per step: CDiffE's y_t normals,
// corrector normals, the EM normals), so both precisions draw identical noise chain by chain.
#pragma once
#include "dmip_device.h"
#include "dmip_internal.h"

namespace dmip {
namespace f32 {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma4(float a, float b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int W>
struct Shape {
  static constexpr int ST = W / 16;                         // 16-unit tiles per layer (= k-groups)
  static constexpr int CHUNK = W * 64;                      // one 16-row tile of a W-input layer
  static constexpr int NW = (W == 64 || W == 512) ? 4 : 8;  // W = 512: one wave per SIMD (2 x 128 VGPR activations)
  static constexpr int PPW = CHUNK / 1024 / NW;             // LDS-DMA pieces per wave per chunk
  static_assert(PPW >= 1 && CHUNK % (1024 * NW) == 0, "ring pieces");
};

constexpr int align16(int v) { return (v + 15) / 16 * 16; }
constexpr int kLdsBudget = 160 * 1024;

// LDS: layer-1 images of the networks, their biases, the observation (CDiffE), then the ring.
//   K1Q0/K1Q1: layer-1 k-steps of net 0 / net 1;  BF: bias floats staged per net;  M: observation
template <int W, int NNET, int K1Q0, int K1Q1, int BF, int M>
struct FLay {
  using S = Shape<W>;
  static constexpr int L1_0 = 0;
  static constexpr int L1_1 = L1_0 + S::ST * K1Q0 * 256;
  static constexpr int BIAS = L1_1 + (NNET > 1 ? S::ST * K1Q1 * 256 : 0);
  static constexpr int BIAS_BYTES = align16(BF * 4);
  static constexpr int YOBS = BIAS + NNET * BIAS_BYTES;
  static constexpr int RING = align16(YOBS + M * 4);
  static constexpr int R0 = (kLdsBudget - RING) / S::CHUNK;
  static constexpr int R = R0 > 4 ? 4 : R0;
  static constexpr int TOTAL = RING + R * S::CHUNK;
  static_assert(R >= 2, "LDS budget: fewer than two ring slots");
};

// the hidden activation (include/dmip.h dmip_act): ACT 0 = tanh (the reference's nn.Tanh, libm tanhf), 1 = SiLU
// (nn.SiLU: z sigmoid(z) = z / (1 + exp(-z)) with libm expf and an IEEE division). Layer 1 applies it twice
// (nets.py:26: the activation module is registered a second time as `act`, whatever it is)
template <int ACT>
__device__ __forceinline__ float act_f32(float z) {
  if constexpr (ACT == 0) return tanhf(z);
  else return z / (1.0f + expf(-z));
}

// The network engine: NNET networks of nl layers (runtime) of width W share one weight ring; each
// network evaluation streams (nl - 1) ST hidden tiles then OT output tiles, in the order of the host's
// stream image. The ring position advances incrementally (no 64-bit modulo per chunk). ACT: act_f32.
template <int W, int NNET, int OT, int R, int RING_OFF, int ACT = 0>
struct FEngine {
  using S = Shape<W>;
  static constexpr int ST = S::ST, NW = S::NW, PPW = S::PPW, CHUNK = S::CHUNK;

  char* lds;
  const char* img[2];
  int bias_off[2];
  int nl;        // hidden layers
  int ncn;       // chunks per network evaluation
  int c_issue;   // next chunk to issue, in [0, NNET ncn)
  int s_issue;   // its ring slot
  int s_read;    // ring slot of the next chunk to consume
  int w, lane, g;

  __device__ __forceinline__ void init(int n_hidden) {
    nl = n_hidden;
    ncn = (nl - 1) * ST + OT;
    c_issue = s_issue = s_read = 0;
  }

  // the next refill's source and ring slot (the stream position advances); its PPW pieces per wave go out at once
  // (ring_issue) or beside the consuming tile's MFMAs (round 5, as the fp32x3 engine: SPREAD)
  const char* dma_src;
  char* dma_dst;
  __device__ __forceinline__ void ring_target() {
    // wave-uniform by construction; say so (the divergence analysis cannot see it through the loops)
    const int c = __builtin_amdgcn_readfirstlane(c_issue);
    const int n = __builtin_amdgcn_readfirstlane(ncn);
    const uint64_t addr = (uint64_t)((c < n ? img[0] : img[1]) + (size_t)(c < n ? c : c - n) * CHUNK);
    const char* base = (const char*)(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(addr >> 32)) << 32) |
                                     (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)addr));
    asm volatile("" : "+s"(base));  // keep the per-chunk address out of the loop-invariant hoist
    dma_src = base;
    dma_dst = lds + RING_OFF + __builtin_amdgcn_readfirstlane(s_issue) * CHUNK;
    c_issue = c_issue + 1 == NNET * ncn ? 0 : c_issue + 1;
    s_issue = s_issue + 1 == R ? 0 : s_issue + 1;
  }
  __device__ __forceinline__ void ring_piece(int q) const {
    const int piece = w * PPW + q;
    glds16(dma_src + piece * 1024, dma_dst + piece * 1024, lane);
  }
  __device__ __forceinline__ void ring_issue() {  // (locals, not the members: at W = 512 that spilled less)
    const int c = __builtin_amdgcn_readfirstlane(c_issue);
    const int n = __builtin_amdgcn_readfirstlane(ncn);
    const uint64_t addr = (uint64_t)((c < n ? img[0] : img[1]) + (size_t)(c < n ? c : c - n) * CHUNK);
    const char* base = (const char*)(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(addr >> 32)) << 32) |
                                     (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)addr));
    asm volatile("" : "+s"(base));  // keep the per-chunk address out of the loop-invariant hoist
    char* dst = lds + RING_OFF + __builtin_amdgcn_readfirstlane(s_issue) * CHUNK;
#pragma unroll
    for (int q = 0; q < PPW; ++q) {
      const int piece = w * PPW + q;
      glds16(base + piece * 1024, dst + piece * 1024, lane);
    }
    c_issue = c_issue + 1 == NNET * ncn ? 0 : c_issue + 1;
    s_issue = s_issue + 1 == R ? 0 : s_issue + 1;
  }
#ifdef DMIP_X3_BURST_DMA
  static constexpr bool SPREAD = false;
#else
  // (the refill 2 chunks ahead; at W = 512 the f32 kernels are register-bound and the live refill state spilled)
  static constexpr bool SPREAD = R >= 3 && PPW <= ST && W <= 256;
#endif

  // the next chunk of the stream, landed (own pieces counted, the others' by the barrier); the
  // slot read one chunk ago is refilled R - 1 chunks ahead
  __device__ __forceinline__ const char* chunk_sync() {
    wait_vmcnt<(R - 2) * PPW>();
    lds_barrier();
    if constexpr (SPREAD) ring_target();  // pieces issued by tile_product, all within this chunk
    else ring_issue();
    const char* slot = lds + RING_OFF + s_read * CHUNK;
    s_read = s_read + 1 == R ? 0 : s_read + 1;
    return slot;
  }

  __device__ __forceinline__ void stage(char* dst, const char* src, int bytes) {
    for (int blk = w; blk < bytes / 1024; blk += NW) glds16(src + blk * 1024, dst + blk * 1024, lane);
  }

  // after the caller's staging: all landed, then prime the ring
  __device__ __forceinline__ void start() {
    wait_vmcnt<0>();
    __syncthreads();
    for (int q = 0; q < R - 1; ++q) ring_issue();
  }

  __device__ __forceinline__ void finish() { wait_vmcnt<0>(); }

  __device__ __forceinline__ f32x4 bias4(int ni, int li, int tile) const {
    return *(const f32x4*)((const float*)(lds + bias_off[ni]) + li * W + 16 * tile + 4 * g);
  }

  // acc(tile) = sum over the W inputs of a streamed chunk: two accumulation chains (even / odd
  // k-groups), the MFMA's 40-cycle dependent latency against its 32-cycle issue
  // (SPREAD: the pending refill's piece p issued beside k-group (p ST) / PPW)
  __device__ __forceinline__ f32x4 tile_product(const char* ch, const float (&H)[ST][4], f32x4 acc0) const {
    f32x4 acc1 = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int q = 0; q < ST; ++q) {
      if constexpr (SPREAD) {
#pragma unroll
        for (int p = 0; p < PPW; ++p)
          if ((p * ST) / PPW == q) ring_piece(p);
      }
      const f32x4 a = *(const f32x4*)(ch + (q * 64 + lane) * 16);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (q & 1) acc1 = mfma4(a[r], H[q][r], acc1);
        else acc0 = mfma4(a[r], H[q][r], acc0);
      }
    }
    return acc0 + acc1;
  }

  // layer 1 (every input column + the bias column, image at l1_off) and its double activation (nets.py:21-26)
  //   K1Q: k-steps compiled (the operand array), k1q: k-steps of the image (<= K1Q, wave-uniform)
  template <int K1Q>
  __device__ __forceinline__ void layer1(int l1_off, int k1q, const float (&b)[K1Q], float (&H)[ST][4]) {
    asm volatile("" ::: "memory");
    const float* l1 = (const float*)(lds + l1_off);
#pragma unroll
    for (int o = 0; o < ST; ++o) {
      f32x4 z = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int s = 0; s < K1Q; ++s)
        if (s < k1q) z = mfma4(l1[(o * k1q + s) * 64 + lane], b[s], z);
#pragma unroll
      for (int r = 0; r < 4; ++r) H[o][r] = act_f32<ACT>(act_f32<ACT>(z[r]));
    }
  }

  __device__ __forceinline__ void hidden(int ni, int li, const float (&Hin)[ST][4], float (&Hout)[ST][4]) {
#pragma unroll
    for (int o = 0; o < ST; ++o) {
      const char* ch = chunk_sync();
      const f32x4 z = tile_product(ch, Hin, bias4(ni, li, o));
#pragma unroll
      for (int r = 0; r < 4; ++r) Hout[o][r] = act_f32<ACT>(z[r]);
    }
  }

  __device__ __forceinline__ void output(int ni, const float (&Hin)[ST][4], f32x4 (&out)[OT]) {
#pragma unroll
    for (int t = 0; t < OT; ++t) {
      const char* ch = chunk_sync();
      out[t] = tile_product(ch, Hin, bias4(ni, nl - 1, t));
    }
  }

  // one network: layer 1 from the B values b, the nl - 1 hidden layers (ping-pong), the output tiles
  template <int K1Q>
  __device__ __forceinline__ void eval(int ni, int l1_off, int k1q, const float (&b)[K1Q], f32x4 (&out)[OT]) {
    float Ha[ST][4], Hb[ST][4];
    layer1<K1Q>(l1_off, k1q, b, Ha);
    for (int li = 0; li + 1 < nl; li += 2) {
      hidden(ni, li, Ha, Hb);
      if (li + 2 < nl) hidden(ni, li + 1, Hb, Ha);
    }
    if ((nl & 1) != 0) output(ni, Ha, out);  // nl - 1 even: the last hidden output is in Ha
    else output(ni, Hb, out);
  }
};

// per-lane B value of layer-1 k-step s: input column 4 s + g of the chain (v: the NV inputs, then
// the bias column 1.0, zero beyond)
template <int NV, int K1Q>
__device__ __forceinline__ void l1_operand(const float (&v)[NV], int g, float (&b)[K1Q]) {
  auto col = [&](int c) -> float { return c < NV ? v[c] : (c == NV ? 1.0f : 0.0f); };
#pragma unroll
  for (int s = 0; s < K1Q; ++s) {
    const float c0 = col(4 * s), c1 = col(4 * s + 1), c2 = col(4 * s + 2), c3 = col(4 * s + 3);
    b[s] = g == 0 ? c0 : (g == 1 ? c1 : (g == 2 ? c2 : c3));
  }
}

constexpr int k1q_of(int n_cols) { return (n_cols + 3) / 4; }
constexpr int kMaxHidden = 3;  // hidden layers compiled: 1..3 (bias staging bound)

// ---------------------------------------------------------------------------- sampler kernel
// The reverse-SDE loop (models/diffusion.py:27-46) with the networks in exact f32:
//   MODE_CDE        a = net(x, y, tau), y folded into the per-y layer-1 bias column (f64 prep)
//   MODE_POSTERIOR  a = g (lik(x, y, tau) + prior(x, tau))            (nets.py:155-157)
//   MODE_CDIFFE     y_t = eps std(tau) + mean_weight(tau) y, a = net(x, y_t, tau)[:D]   (+ Langevin
//                   corrector steps before each predictor step, as the bf16 kernel)
// then mu = g a + 0.5 beta x, x <- x + delta mu + sqrt(delta) g xi (dmip_device.h em_update).
// Work: the grid is at most one resident wave set; a y's 16-chain tiles are spread over its waves by
// the balanced WaveSchedule of dmip_device.h (equal segments of C wave-steps, split tiles handed over
// through global memory), so 100k chains cost 3.05 rounds of the GPU's capacity, not 4. Every lane
// group of a chain holds the same state, so the hand-over stores all 64 lanes like the 16-bit kernel.
template <int MODE, int W, int D, int M, int ACT = 0>
struct SamplerCfg {
  static constexpr int NNET = MODE == SAMPLER_POSTERIOR ? 2 : 1;
  static constexpr int NV0 = MODE == SAMPLER_CDIFFE ? D + M + 1 : D + 1;  // net 0 inputs (y folded for CDE)
  static constexpr int K1Q0 = k1q_of(NV0 + 1);
  static constexpr int K1Q1 = k1q_of(D + 2);                              // prior (x, t) + bias
  static constexpr int BF_MAX = (kMaxHidden - 1) * W + 16;                // hidden biases + output tile 0
  using L = FLay<W, NNET, K1Q0, K1Q1, BF_MAX, M>;
  using E = FEngine<W, NNET, 1, L::R, L::RING, ACT>;
};

template <int MODE, int W, int D, int M, bool NOISE, int ACT = 0>
__global__ void __launch_bounds__(Shape<W>::NW * 64, 1) f32_sampler_kernel(F32SamplerParams p) {
  using C = SamplerCfg<MODE, W, D, M, ACT>;
  using L = typename C::L;
  using E = typename C::E;
  constexpr int NW = Shape<W>::NW, ST = Shape<W>::ST;
  static_assert(L::TOTAL <= kLdsBudget, "LDS budget");
  static_assert(D <= 4, "output rows of a chain sit in lane group 0 (D <= 4)");
  __shared__ __attribute__((aligned(16))) char lds[L::TOTAL];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, j = lane & 15;
  const int yi = blockIdx.y;

  E eng{lds, {p.net[0].stream, p.net[1].stream}, {L::BIAS, L::BIAS + L::BIAS_BYTES}};
  eng.w = w, eng.lane = lane, eng.g = g;
  eng.init(p.n_hidden);
  const int bf = (p.n_hidden - 1) * W + 16;
  {
    const float* l10 = MODE == SAMPLER_CDIFFE ? p.net[0].l1 : p.l1y + (size_t)yi * ST * C::K1Q0 * 64;
    eng.stage(lds + L::L1_0, (const char*)l10, ST * C::K1Q0 * 256);
    if constexpr (C::NNET > 1) eng.stage(lds + L::L1_1, (const char*)p.net[1].l1, ST * C::K1Q1 * 256);
    for (int ni = 0; ni < C::NNET; ++ni) {
      float* bl = (float*)(lds + L::BIAS + ni * L::BIAS_BYTES);
      for (int i = threadIdx.x; i < bf; i += NW * 64) bl[i] = p.net[ni].bias[i];
    }
    if constexpr (MODE == SAMPLER_CDIFFE) {
      float* yo = (float*)(lds + L::YOBS);
      for (int i = threadIdx.x; i < M; i += NW * 64) yo[i] = p.y_obs[(size_t)yi * M + i];
    }
    eng.start();
  }
  const float* yobs = (const float*)(lds + L::YOBS);

  const int S = p.num_steps;
  const long long tiles_y = (p.n_chains + 15) / 16;
  const long long n_waves = (long long)gridDim.x * NW;  // waves sharing this y
  const long long gw = (long long)blockIdx.x * NW + w;  // this wave among them
  constexpr int XW = sampler_xfer_words(D);
  const WaveSchedule sched(tiles_y, S, n_waves, gw);
  const size_t noise_step = (size_t)gridDim.y * p.n_chains * D;

  for (int sgi = 0; sgi < sched.n_seg; ++sgi) {
    const Seg sg = sched.segment(sgi);
    const long long c_local = (long long)(sg.job >= 0 ? sg.job : 0) * 16 + j;
    const bool valid = sg.job >= 0 && c_local < p.n_chains;
    const long long c_rd = valid ? c_local : 0;
    Rng rng;
    float x[D];
    bool lost = false;  // the hand-over never arrived: the tile's output is poisoned and reported
    if (sg.kind == 2) {  // resume the tile the previous wave of the grid handed over
      const size_t slot = (size_t)yi * n_waves + gw - 1;
      lost = handover_wait(p.xflag + slot, p.spin_limit, p.err, kErrHandover, lane);
      const float* src = p.xfer + slot * XW;
#pragma unroll
      for (int k = 0; k < D; ++k) x[k] = lost ? __builtin_nanf("") : src[k * 64 + lane];
      rng.s0 = __float_as_uint(src[(D + 0) * 64 + lane]);
      rng.s1 = __float_as_uint(src[(D + 1) * 64 + lane]);
      rng.s2 = __float_as_uint(src[(D + 2) * 64 + lane]);
      rng.s3 = __float_as_uint(src[(D + 3) * 64 + lane]);
    } else {
      rng = rng_init(p.seed, (uint64_t)(p.chain_offset + c_local), (uint64_t)yi);
      float n0[D];
      if constexpr (NOISE) {
        const float* src = p.noise + ((size_t)yi * p.n_chains + c_rd) * D;
#pragma unroll
        for (int k = 0; k < D; ++k) n0[k] = src[k];
      } else {
        rng_normals<D>(rng, n0);
      }
#pragma unroll
      for (int k = 0; k < D; ++k) x[k] = __fadd_rn(__fmul_rn(n0[k], p.stdv), p.mean);
    }

    SnapCursor snap(p.snap_every, sg.s0);
    for (int i0 = sg.s0; i0 < sg.s1; ++i0) {
      const int i = sg.kind == 3 ? 0 : i0;  // idle steps: a dummy tile at step 0, discarded
      const StepCoef cf = step_coef(i, S, p.T, p.bmin, p.bdiff);
      float v[C::NV0];
#pragma unroll
      for (int k = 0; k < D; ++k) v[k] = x[k];
      if constexpr (MODE == SAMPLER_CDIFFE) {
        // y_t = eps * std(T-t) + mean_weight(T-t) * y  (sdes.py:37-44)
        const float mw = vp_mean_weight(cf.tau, p.bmin, p.bdiff);
        const float sd = vp_std(cf.tau, p.bmin, p.bdiff);
        float eps[M];
        rng_normals<M>(rng, eps);
#pragma unroll
        for (int k = 0; k < M; ++k) v[D + k] = __fadd_rn(__fmul_rn(eps[k], sd), __fmul_rn(mw, yobs[k]));
      }
      v[C::NV0 - 1] = cf.tau;

      // a(x) at this step's time and y_t: output rows 0..D-1 of every chain, on all its lanes
      // always inlined: an outlined call would put the activation arrays on the scratch stack
      auto score = [&](const float (&vin)[C::NV0], float (&a)[D]) __attribute__((always_inline)) {
        f32x4 out[1];
        float b0[C::K1Q0];
        l1_operand<C::NV0, C::K1Q0>(vin, g, b0);
        eng.template eval<C::K1Q0>(0, L::L1_0, C::K1Q0, b0, out);
        if constexpr (C::NNET > 1) {
          float vp[D + 1];
#pragma unroll
          for (int k = 0; k < D; ++k) vp[k] = vin[k];
          vp[D] = cf.tau;
          float b1[C::K1Q1];
          l1_operand<D + 1, C::K1Q1>(vp, g, b1);
          f32x4 out1[1];
          eng.template eval<C::K1Q1>(1, L::L1_1, C::K1Q1, b1, out1);
          out[0] = out[0] + out1[0];  // prior + likelihood, then g * (...)
        }
#pragma unroll
        for (int k = 0; k < D; ++k) a[k] = __shfl(out[0][k], j, 64);
      };

      if constexpr (MODE == SAMPLER_CDIFFE) {
        // Langevin corrector steps (the bf16 kernel's definition, dmip_kernels.hip): s = a / g,
        // eps = 2 alpha snr^2 var(T - t), x <- x + eps s + sqrt(2 eps) z, alpha = exp(-beta delta)
        for (int c = 0; c < p.n_corr; ++c) {
          float oc[D];
          score(v, oc);
          float z[D], sc[D];
          rng_normals<D>(rng, z);
#pragma unroll
          for (int k = 0; k < D; ++k) sc[k] = oc[k] / cf.g;
          const float alpha = __expf(-cf.beta * p.delta);
          const float sd = vp_std(cf.tau, p.bmin, p.bdiff);
          const float r = (p.snr * p.snr) * (sd * sd);
          const float es = 2.0f * alpha * r;
          const float ns = __fsqrt_rn(2.0f * es);
#pragma unroll
          for (int k = 0; k < D; ++k) {
            x[k] = x[k] + es * sc[k] + ns * z[k];
            v[k] = x[k];
          }
        }
      }

      float a[D];
      score(v, a);
      float xi[D];
      if constexpr (NOISE) {
        const float* src = p.noise + noise_step * (i + 1) + ((size_t)yi * p.n_chains + c_rd) * D;
#pragma unroll
        for (int k = 0; k < D; ++k) xi[k] = src[k];
      } else {
        rng_normals<D>(rng, xi);
      }
#pragma unroll
      for (int k = 0; k < D; ++k) {
        const float ak = MODE == SAMPLER_POSTERIOR ? __fmul_rn(cf.g, a[k]) : a[k];
        x[k] = em_update(x[k], ak, xi[k], cf, p.delta, p.sqrt_delta);
      }
      snap.at_step<D>(i0, p.snap_every, p.snap_out, gridDim.y, yi, p.n_chains, c_local, sg.kind != 3 && valid && g == 0, x);
    }
    if (sg.kind == 1) {  // hand the tile over to the next wave of the grid
      const size_t slot = (size_t)yi * n_waves + gw;
      float* dst = p.xfer + slot * XW;
#pragma unroll
      for (int k = 0; k < D; ++k) dst[k * 64 + lane] = x[k];
      dst[(D + 0) * 64 + lane] = __uint_as_float(rng.s0);
      dst[(D + 1) * 64 + lane] = __uint_as_float(rng.s1);
      dst[(D + 2) * 64 + lane] = __uint_as_float(rng.s2);
      dst[(D + 3) * 64 + lane] = __uint_as_float(rng.s3);
      handover_publish(p.xflag + slot, lane, p.debug_flags);
    } else if (sg.kind != 3 && valid && g == 0) {
      float* dst = p.x_out + ((size_t)yi * p.n_chains + c_local) * D;
#pragma unroll
      for (int k = 0; k < D; ++k) dst[k] = x[k];
    }
    (void)lost;
  }
  eng.finish();
}

// ------------------------------------------------------------------------------ forward kernel
// out[n] = net(cat[x, y, t]) in exact f32 (nets.py:32-35 / 52-57): layer 1 over every input column.
//   K1Q: layer-1 k-steps compiled (any image with in_dim + 1 <= 4 K1Q; the image's own count is the
//   runtime p.k1q);  OT: output tiles (out_dim <= 16 OT)
constexpr int kForwardK1Q = 8;
template <int W, int K1Q, int OT, int ACT>
struct ForwardCfg {
  static constexpr int BF_MAX = (kMaxHidden - 1) * W + 16 * OT;
  using L = FLay<W, 1, K1Q, 1, BF_MAX, 0>;
  using E = FEngine<W, 1, OT, L::R, L::RING, ACT>;
};

template <int W, int K1Q, int OT, int ACT>
__global__ void __launch_bounds__(Shape<W>::NW * 64, 1) f32_forward_kernel(F32ForwardParams p) {
  using C = ForwardCfg<W, K1Q, OT, ACT>;
  using L = typename C::L;
  constexpr int NW = Shape<W>::NW, ST = Shape<W>::ST;
  static_assert(L::TOTAL <= kLdsBudget, "LDS budget");
  __shared__ __attribute__((aligned(16))) char lds[L::TOTAL];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, j = lane & 15;
  typename C::E eng{lds, {p.net.stream, p.net.stream}, {L::BIAS, L::BIAS}};
  eng.w = w, eng.lane = lane, eng.g = g;
  eng.init(p.n_hidden);
  eng.stage(lds + L::L1_0, (const char*)p.net.l1, ST * p.k1q * 256);
  {
    float* bl = (float*)(lds + L::BIAS);
    const int bf = (p.n_hidden - 1) * W + 16 * OT;
    for (int i = threadIdx.x; i < bf; i += NW * 64) bl[i] = p.net.bias[i];
  }
  eng.start();
  const int in_dim = p.xdim + p.ydim + 1;
  const long long tiles = (p.n + 15) / 16;
  const long long per_round = (long long)gridDim.x * NW;
  const long long rounds = (tiles + per_round - 1) / per_round;
  for (long long rd = 0; rd < rounds; ++rd) {
    const long long row = ((rd * gridDim.x + blockIdx.x) * NW + w) * 16 + j;
    const bool valid = row < p.n;
    const long long rr = valid ? row : 0;
    float b[K1Q];
#pragma unroll
    for (int s = 0; s < K1Q; ++s) {
      const int c = 4 * s + g;  // this lane's input column
      float val = 0.0f;
      if (c < p.xdim) val = p.x[rr * p.xdim + c];
      else if (c < p.xdim + p.ydim) val = p.y[(p.y_stride ? rr * p.y_stride : 0) + (c - p.xdim)];
      else if (c == in_dim - 1) val = p.t[p.t_stride ? rr : 0];
      else if (c == in_dim) val = 1.0f;
      b[s] = val;
    }
    f32x4 out[OT];
    eng.template eval<K1Q>(0, L::L1_0, p.k1q, b, out);
    if (valid) {
#pragma unroll
      for (int t = 0; t < OT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int k = 16 * t + 4 * g + r;
          if (k < p.out_dim) p.out[row * p.out_dim + k] = out[t][r];
        }
    }
  }
  eng.finish();
}

}  // namespace f32

// ----------------------------------------------------------------- launch helpers (per TU)
template <int MODE, int W, int D, int M, bool NOISE, int ACT = 0>
inline hipError_t launch_f32_sampler_t(const F32SamplerParams& p, int n_y, hipStream_t st) {
  constexpr int NW = f32::Shape<W>::NW;
  auto kern = f32::f32_sampler_kernel<MODE, W, D, M, NOISE, ACT>;
  const long long tiles = (p.n_chains + 15) / 16;
  long long g = resident_slots(kern, NW * 64, st) / (n_y > 0 ? n_y : 1);
  const long long cap = (tiles + NW - 1) / NW;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  // the balanced schedule's hand-over needs every workgroup of the grid resident at once: g is
  // capped by the stream device's occupancy above
  F32SamplerParams q = p;
  char* buf = nullptr;
  hipError_t e = alloc_handover((size_t)g * n_y * NW, D, st, &buf, &q.xfer, &q.xflag);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)g, (unsigned)n_y), dim3(NW * 64), 0, st, q);
  e = hipGetLastError();
  (void)hipFreeAsync(buf, st);
  return e;
}

// the SiLU chain (p.act == DMIP_ACT_SILU_TWICE_FIRST) is compiled for the CDE sampler only; the caller
// (dmip_em_sample) refuses it for the other modes
template <int MODE, int W, int D, int M>
inline hipError_t launch_f32_sampler_n(const F32SamplerParams& p, int n_y, hipStream_t st) {
  if constexpr (MODE == SAMPLER_CDE) {
    if (p.act != 0) {
      if (p.noise) return launch_f32_sampler_t<MODE, W, D, M, true, 1>(p, n_y, st);
      return launch_f32_sampler_t<MODE, W, D, M, false, 1>(p, n_y, st);
    }
    if (p.noise) return launch_f32_sampler_t<MODE, W, D, M, true>(p, n_y, st);
  }
  return launch_f32_sampler_t<MODE, W, D, M, false>(p, n_y, st);
}

template <int W, int K1Q, int OT, int ACT>
inline hipError_t launch_f32_forward_t(const F32ForwardParams& p, hipStream_t st) {
  constexpr int NW = f32::Shape<W>::NW;
  auto kern = f32::f32_forward_kernel<W, K1Q, OT, ACT>;
  const long long tiles = (p.n + 15) / 16;
  long long g = resident_slots(kern, NW * 64, st);
  const long long cap = (tiles + NW - 1) / NW;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(kern, dim3((unsigned)g), dim3(NW * 64), 0, st, p);
  return hipGetLastError();
}

// per-mode instantiations (dmip_f32_{cde,post,cdiffe}.hip)
hipError_t launch_f32_sampler_cde(const F32SamplerParams& p, int width, int xdim, int n_y, hipStream_t st, bool* ok);
hipError_t launch_f32_sampler_post(const F32SamplerParams& p, int width, int xdim, int n_y, hipStream_t st, bool* ok);
hipError_t launch_f32_sampler_cdiffe(const F32SamplerParams& p, int width, int xdim, int ydim, int n_y, hipStream_t st,
                                     bool* ok);

}  // namespace dmip
