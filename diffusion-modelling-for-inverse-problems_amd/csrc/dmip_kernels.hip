// dmip kernels for gfx950 (MI355X, CDNA4): the fused persistent reverse-SDE sampler, the score
// MLP forward, and the small prep/debug kernels behind the C-ABI in include/dmip.h.
//
// Data flow of the sampler (one wave = 32 posterior chains, 8 waves = one workgroup):
//   * The chain state (x, RNG) lives in VGPRs for all num_steps; HBM is written once at the end.
//   * Hidden activations never leave the registers: a layer's 32x32 f32 accumulator tile (column =
//     chain on the lane, rows = hidden units in the 16 registers) is activated, packed to bf16 and
//     used directly as the B operand of the next layer's v_mfma_f32_32x32x16_bf16. The weight
//     (A) fragments are pre-permuted on the host to the matching k order.
//   * Weights: layer 1 (with the y-conditioning folded in), the output layer and the biases are
//     LDS-resident; the W x W hidden layers are LDS-resident when they fit and otherwise streamed
//     from L2 through an R-slot LDS ring by LDS-DMA (global_load_lds_dwordx4), one row tile
//     (32 rows x W) per slot, with counted vmcnt waits and raw s_barriers.
//   * Layer 1 runs on MFMA with split-bf16 operands (x, tau and the weights as hi+lo pairs), so
//     the chain state enters the net at ~fp32 accuracy.
// Reference: models/diffusion.py:27-46 (loop), sdes.py:77-87 (drift/diffusion), nets.py:17-35 (MLP).
#include "dmip_device.h"
#include "dmip_internal.h"

#include <cstdlib>

namespace dmip {

// LDS layout of one workgroup: NNET networks (net 0 = the CDE / CDiffE / likelihood net, net 1 =
// the prior net of the Posterior estimator) share one weight ring. AOR: the output layers stream
// through the ring too (one more chunk per network after its hidden chunks; the host appends the
// output image to each network's hidden image) -- the two-network sampler at width 512, whose
// resident output layers (2 x 32 KiB) would not leave room for the ring. L1R: layer 1 streams through
// the ring ahead of the hidden chunks, TPC row tiles (K1S KiB each) per chunk -- CDiffE at width 512,
// whose 27-input split layer 1 is 96 KiB.
template <int W, int NL, int K1S, int NNET, int R, bool RES, bool AOR = false, bool L1R = false>
struct Lay {
  static constexpr int T = W / 32;            // 32-row tiles per layer
  static constexpr int KS = W / 16;           // 16-deep k-steps over a hidden layer
  static constexpr int CHUNK = KS * 1024;     // one row tile of a W x W layer, bf16 fragments
  static constexpr int NC = (NL - 1) * T;     // hidden chunks per network evaluation
  static constexpr int TPC = L1R ? KS / K1S : 1;        // layer-1 row tiles per ring chunk (L1R)
  static constexpr int L1C = L1R ? (T + TPC - 1) / TPC : 0;  // layer-1 chunks per network evaluation
  static constexpr int NCP = L1C + NC + (AOR ? 1 : 0);  // ring chunks per network evaluation
  static constexpr int NCT = NCP * NNET;      // ring chunks per step (all networks)
  static constexpr int A1_BYTES = T * K1S * 1024;
  static constexpr int AO_BYTES = KS * 1024;
  static constexpr int BH_BYTES = (NL - 1) * T * 2 * 16 * 4;
  static constexpr int BO_BYTES = 2 * 16 * 4;  // output bias, summed over the networks
  static constexpr int A1_OFF = 0;
  static constexpr int AO_OFF = A1_OFF + (L1R ? 0 : NNET * A1_BYTES);
  static constexpr int BH_OFF = AO_OFF + (AOR ? 0 : NNET * AO_BYTES);
  static constexpr int BO_OFF = BH_OFF + NNET * BH_BYTES;
  static constexpr int W_OFF = BO_OFF + BO_BYTES;
  static constexpr int SLOTS = RES ? NCT : R;
  static constexpr int TOTAL = W_OFF + SLOTS * CHUNK;
};

// ---------------------------------------------------------------------- shared LDS staging
template <int NW>
__device__ __forceinline__ void stage_blocks(char* lds, const char* g, int n_blocks, int w, int lane) {
  for (int p = w; p < n_blocks; p += NW) glds16(g + p * 1024, lds + p * 1024, lane);
}

__device__ __forceinline__ void stage_floats(float* lds, const float* g, int n, int tid, int nthreads) {
  for (int i = tid; i < n; i += nthreads) lds[i] = g[i];
}

// acc += sum_s A[s] * H[s] over one 32-row tile: A fragments streamed from LDS (1 KiB apart)
// with PF reads kept in flight, so the MFMA chain does not wait on each fragment's LDS latency.
// The reads and their counted waits are explicit: left to itself the compiler (at ~234 VGPRs)
// schedules each read right before its MFMA behind an lgkmcnt(0), which exposes the full LDS
// latency on every MFMA. A wait names the fragment it guards ("+v"), so the MFMA that uses the
// fragment cannot be scheduled above it. Younger LDS operations the compiler adds in between only
// make a counted wait stricter (LDS returns in order).
typedef __attribute__((address_space(3))) const char* lds_cptr;

template <int OFF>
__device__ __forceinline__ bf16x8 lds_read_b128(lds_cptr p) {
  bf16x8 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(p), "i"(OFF));
  return r;
}

template <int N>
__device__ __forceinline__ void lds_wait(bf16x8& guarded) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(guarded) : "i"(N));
}

template <int KS, int PF, bool F16, int S = 0>
__device__ __forceinline__ void mfma_chain(lds_cptr a_lane, const bf16x8 (&H)[KS], f32x16& acc, bf16x8 (&a)[PF + 1]) {
  if constexpr (S < KS) {
    if constexpr (S + PF < KS) a[(S + PF) % (PF + 1)] = lds_read_b128<(S + PF) * 1024>(a_lane);
    constexpr int younger = (KS - 1 - S) < PF ? (KS - 1 - S) : PF;  // reads issued after fragment S
    lds_wait<younger>(a[S % (PF + 1)]);
    if constexpr (F16) acc = mfma32h(a[S % (PF + 1)], H[S], acc);
    else acc = mfma32(a[S % (PF + 1)], H[S], acc);
    mfma_chain<KS, PF, F16, S + 1>(a_lane, H, acc, a);
  }
}

// F16: fp16 operands (the engine's hidden and output layers), else bf16
template <int KS, bool F16, int PF = 3>
__device__ __forceinline__ void mfma_row_tile(const char* a_lane_g, const bf16x8 (&H)[KS], f32x16& acc) {
  const lds_cptr a_lane = (lds_cptr)a_lane_g;
  bf16x8 a[PF + 1];
  if constexpr (PF >= 1) a[0] = lds_read_b128<0>(a_lane);
  if constexpr (PF >= 2 && KS > 1) a[1] = lds_read_b128<1024>(a_lane);
  if constexpr (PF >= 3 && KS > 2) a[2] = lds_read_b128<2048>(a_lane);
  static_assert(PF >= 1 && PF <= 3, "prefetch depth");
  mfma_chain<KS, PF, F16>(a_lane, H, acc, a);
}

// ------------------------------------------------------------------- network evaluation engine
// Evaluates NNET networks on one 32-chain tile per wave and sums their output layers into one
// accumulator tile (rows = output dims; the host packers define the row maps).
// Operand types: layer 1 is a bf16 MFMA over split-bf16 inputs (~fp32 chain state). The W x W hidden
// layers and the output layer are fp16 MFMAs (v_mfma_f32_32x32x16_f16, the bf16 rate) over fp16
// weights and fp16 activations in (-1, 1): 3 more mantissa bits than bf16 for the same issue, and
// layer 1's double tanh runs in packed fp16 (act_t_twice_pk_f16, two units per instruction).
// Measured against the all-bf16 engine on one box (profiles/README.md, r2 A/B): 1.5 % faster, and
// the 512-chain smoke trajectory 7x closer to the exact oracle (3.5e-4 vs 2.4e-3).
// Schedule: a layer's last tile is activated inside the next layer's first tile block (beside its
// MFMAs over the other k-steps), and a ring tile's bias is read before the ring barrier, whose
// compiler-visible lgkmcnt(0) covers it, so the first MFMA waits only for its own fragment.
// DIAG (timing ablations only, never on the product path): bit 0 = no ring barrier/DMA,
// bit 1 = hidden activations replaced by a cast, bit 2 = layer-1 activation replaced by a cast.
template <int W, int NL, int K1S, int NNET, int NW, int R, bool RES, bool CONSERVATIVE, int DIAG = 0,
          bool AOR = false, bool L1R = false>
struct Engine {
  using L = Lay<W, NL, K1S, NNET, R, RES, AOR, L1R>;
  static constexpr int T = L::T;
  static constexpr int KS = L::KS;
  static constexpr int PPW = RES ? 1 : KS / NW;

  char* lds;
  const char* hidden[2];
  long long gc;  // global chunk counter (ring mode)
  int w, lane;

  // Every network evaluation streams exactly NCT chunks, so when NCT % R == 0 the k-th chunk of an
  // evaluation always sits in slot k % R: with k a compile-time constant after unrolling, every ring
  // address is a constant offset (no per-chunk 64-bit counter arithmetic: that was ~30 scalar
  // instructions per chunk, issued by all waves at once right after the barrier).
  static constexpr bool STATIC_RING = (L::NCT % R) == 0;

  // issue chunk c (in [0, NCT)) of the evaluation into ring slot `slot`
  __device__ __forceinline__ void ring_issue_at(int c, int slot) {
    // opaque wave-uniform base, re-materialised at every issue: otherwise the compiler hoists every
    // chunk's 64-bit source address out of the step loop and holds them all in registers (2 VGPRs
    // per chunk with a per-lane address, 2 SGPRs -- spilled to VGPR lanes -- with a constant one)
    const char* base = c < L::NCP ? hidden[0] : hidden[1];
    asm volatile("" : "+s"(base));
    char* dst = lds + L::W_OFF + slot * L::CHUNK;
#pragma unroll
    for (int q = 0; q < PPW; ++q) {
      const int piece = w * PPW + q;
      glds16(base + (size_t)(c % L::NCP) * L::CHUNK + piece * 1024, dst + piece * 1024, lane);
    }
  }

  __device__ __forceinline__ void ring_issue(long long g) {
    // chunk index and network select stay scalar (the counter is wave-uniform; the segment loop of
    // the balanced sampler hides that from the divergence analysis)
    ring_issue_at(__builtin_amdgcn_readfirstlane((int)(g % L::NCT)), __builtin_amdgcn_readfirstlane((int)(g % R)));
  }

  // k: index of the chunk within the current network evaluation (a constant after unrolling)
  __device__ __forceinline__ const char* chunk_sync(int k) {
    if constexpr (DIAG & 1) {
      asm volatile("" ::: "memory");
      return lds + L::W_OFF + (int)((gc++) % R) * L::CHUNK;
    } else {
      if constexpr (CONSERVATIVE) wait_vmcnt<0>();
      else wait_vmcnt<(R - 2) * PPW>();
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) the compiler sees: covers the bias reads
      lds_barrier();
      if constexpr (STATIC_RING) {
        ring_issue_at((k + R - 1) % L::NCT, (k + R - 1) % R);
        return lds + L::W_OFF + (k % R) * L::CHUNK;
      } else {
        ring_issue(gc + R - 1);
        const char* slot = lds + L::W_OFF + (int)(gc % R) * L::CHUNK;
        ++gc;
        return slot;
      }
    }
  }

  __device__ __forceinline__ f32x16 bias_tile(int off) const {
    const float* b = (const float*)(lds + off) + (lane >> 5) * 16;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = b[r];
    return acc;
  }

  // the last tile of a layer, activated inside the next layer's first tile block; TW: layer 1's
  // double tanh (t-form, packed fp16) or a hidden layer's r-form
  template <bool TW>
  __device__ __forceinline__ void act_carry(const f32x16& carry, bf16x8 (&H)[KS]) {
    act_pack<TW, (DIAG & (TW ? 4 : 2)) != 0>(carry, H[2 * (T - 1)], H[2 * (T - 1) + 1]);
  }

  // layer 1 of net NI from the B1 operand (split-bf16 inputs), double tanh (nets.py:21-26); returns
  // the last tile's pre-activation
  template <int NI>
  __device__ __forceinline__ f32x16 layer1(const bf16x8 (&B1)[K1S], bf16x8 (&H)[KS]) {
    f32x16 pend;
    const char* a1c = nullptr;  // L1R: the ring slot holding this row tile's layer-1 chunk
#pragma unroll
    for (int rt = 0; rt < T; ++rt) {
      asm volatile("" ::: "memory");
      f32x16 acc = {};
      if constexpr (L1R) {
        if (rt % L::TPC == 0) a1c = chunk_sync(NI * L::NCP + rt / L::TPC);
      }
#pragma unroll
      for (int s = 0; s < K1S; ++s) {
        const char* src = L1R ? a1c + ((rt % L::TPC) * K1S + s) * 1024
                              : lds + L::A1_OFF + NI * L::A1_BYTES + (rt * K1S + s) * 1024;
        const bf16x8 a = *(const bf16x8*)(src + lane * 16);
        acc = mfma32(a, B1[s], acc);
      }
      if (rt > 0) act_pack<true, (DIAG & 4) != 0>(pend, H[2 * (rt - 1)], H[2 * (rt - 1) + 1]);
      pend = acc;
    }
    return pend;
  }

  // one W x W layer (fp16 MFMAs); the activation of tile rt-1 is issued in tile rt's block so it
  // overlaps the MFMAs (the compiler interleaves them; explicit orders measured slower,
  // profiles/README.md). Returns the last tile's pre-activation.
  template <int NI, int LI, bool TW>
  __device__ __forceinline__ f32x16 hidden_layer(bf16x8 (&Hin)[KS], const f32x16& carry, bf16x8 (&Hout)[KS]) {
    f32x16 pend;
#pragma unroll
    for (int rt = 0; rt < T; ++rt) {
      const int boff = L::BH_OFF + NI * L::BH_BYTES + ((LI * T + rt) * 2) * 64;
      f32x16 acc;
      const char* wb;
      if constexpr (RES) {
        // keep the resident weights in LDS: without this the compiler hoists every fragment
        // read out of the step loop into (spilled) registers
        asm volatile("" ::: "memory");
        wb = lds + L::W_OFF + ((NI * (NL - 1) + LI) * T + rt) * L::CHUNK;
        acc = bias_tile(boff);
      } else {
        acc = bias_tile(boff);
        wb = chunk_sync(NI * L::NCP + L::L1C + LI * T + rt);
      }
      if (rt == 0) act_carry<TW>(carry, Hin);
      mfma_row_tile<KS, true>(wb + lane * 16, Hin, acc);
      if (rt > 0) act_pack<false, (DIAG & 2) != 0>(pend, Hout[2 * (rt - 1)], Hout[2 * (rt - 1) + 1]);
      pend = acc;
    }
    return pend;
  }

  // hidden layers LI.. of net NI, then its output layer accumulated into `out`
  template <int NI, int LI, bool TW>
  __device__ __forceinline__ void hidden_stack(bf16x8 (&Ha)[KS], bf16x8 (&Hb)[KS], const f32x16& carry,
                                               f32x16& out) {
    if constexpr (LI == NL - 1) {
      asm volatile("" ::: "memory");
      if constexpr (AOR) {
        const char* wb = chunk_sync(NI * L::NCP + L::L1C + L::NC);
        act_carry<TW>(carry, Ha);
        mfma_row_tile<KS, true>(wb + lane * 16, Ha, out);
      } else {
        act_carry<TW>(carry, Ha);
        mfma_row_tile<KS, true>(lds + L::AO_OFF + NI * L::AO_BYTES + lane * 16, Ha, out);
      }
    } else {
      const f32x16 c2 = hidden_layer<NI, LI, TW>(Ha, carry, Hb);
      hidden_stack<NI, LI + 1, false>(Hb, Ha, c2, out);
    }
  }

  template <int NI>
  __device__ __forceinline__ void eval_net(const bf16x8 (&B1)[K1S], f32x16& out) {
    bf16x8 Ha[KS], Hb[KS];
    const f32x16 c1 = layer1<NI>(B1, Ha);
    hidden_stack<NI, 0, true>(Ha, Hb, c1, out);
  }

  // sum over the networks of their outputs (+ the summed output bias)
  __device__ __forceinline__ f32x16 eval(const bf16x8 (&B1)[K1S]) {
    asm volatile("" ::: "memory");
    f32x16 out = bias_tile(L::BO_OFF);
    eval_net<0>(B1, out);
    if constexpr (NNET > 1) {
      // only accumulator registers 0-3 carry output rows in the sampler's row map (rows 0-3, duplicated
      // into lanes 32-63); carry just those through the second network
      float keep[4] = {out[0], out[1], out[2], out[3]};
      __builtin_amdgcn_sched_barrier(0);
      f32x16 out2 = {};
      eval_net<1>(B1, out2);
#pragma unroll
      for (int r = 0; r < 4; ++r) out2[r] += keep[r];
      return out2;
    }
    return out;
  }

  // resident parts (and the whole hidden stack in resident mode); then start the ring.
  // The output bias is the sum of the networks' output biases.
  __device__ __forceinline__ void prologue(const char* const (&a1)[2], const char* const (&ao)[2],
                                           const float* const (&bh)[2], const float* const (&bo)[2]) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int ni = 0; ni < NNET; ++ni) {
      if constexpr (!L1R) stage_blocks<NW>(lds + L::A1_OFF + ni * L::A1_BYTES, a1[ni], T * K1S, w, lane);
      if constexpr (!AOR) stage_blocks<NW>(lds + L::AO_OFF + ni * L::AO_BYTES, ao[ni], KS, w, lane);
      if constexpr (RES) stage_blocks<NW>(lds + L::W_OFF + ni * L::NC * L::CHUNK, hidden[ni], L::NC * KS, w, lane);
      stage_floats((float*)(lds + L::BH_OFF + ni * L::BH_BYTES), bh[ni], L::BH_BYTES / 4, tid, NW * 64);
    }
    for (int i = tid; i < L::BO_BYTES / 4; i += NW * 64)
      ((float*)(lds + L::BO_OFF))[i] = NNET > 1 ? bo[0][i] + bo[1][i] : bo[0][i];
    wait_vmcnt<0>();
    __syncthreads();
    if constexpr (!RES) {
      for (int q = 0; q < R - 1; ++q) ring_issue(q);
    }
  }

  __device__ __forceinline__ void epilogue() {
    wait_vmcnt<0>();  // no LDS-DMA may still be landing when the workgroup retires
  }
};

// B1 operand of layer 1: u = [hi(v) | lo(v) | hi(v) | 1 | 1 | 0...] over NV varying inputs;
// lane half h supplies u[16 s + 8 h + j].
template <int NV, int K1S>
__device__ __forceinline__ void build_b1(const float (&v)[NV], int h, bf16x8 (&B1)[K1S]) {
  __bf16 vh[NV], vl[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    vh[k] = (__bf16)v[k];
    vl[k] = (__bf16)(v[k] - (float)vh[k]);
  }
#pragma unroll
  for (int s = 0; s < K1S; ++s) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      // both candidate slot values (h = 0 and h = 1) are compile-time; select by lane half
      auto slot = [&](int k) -> __bf16 {
        if (k < NV) return vh[k];
        if (k < 2 * NV) return vl[k - NV];
        if (k < 3 * NV) return vh[k - 2 * NV];
        if (k < 3 * NV + 2) return (__bf16)1.0f;
        return (__bf16)0.0f;
      };
      B1[s][j] = h ? slot(16 * s + 8 + j) : slot(16 * s + j);
    }
  }
}

// rewrite the x slots (inputs 0..D-1) of a build_b1 operand after x changed
template <int NV, int D, int K1S>
__device__ __forceinline__ void patch_b1_x(const float (&x)[D], int h, bf16x8 (&B1)[K1S]) {
#pragma unroll
  for (int k = 0; k < D; ++k) {
    const __bf16 hi = (__bf16)x[k];
    const __bf16 lo = (__bf16)(x[k] - (float)hi);
    const int slots[3] = {k, NV + k, 2 * NV + k};
    const __bf16 vals[3] = {hi, lo, hi};
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int sl = slots[q];
      if (h == ((sl >> 3) & 1)) B1[sl >> 4][sl & 7] = vals[q];
    }
  }
}

// ------------------------------------------------------------------------- sampler kernel
__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

constexpr int MODE_CDE = SAMPLER_CDE, MODE_POSTERIOR = SAMPLER_POSTERIOR, MODE_CDIFFE = SAMPLER_CDIFFE;

constexpr int k1s_of(int slots) { return (slots + 15) / 16; }

// The fused reverse-SDE sampler (all num_steps in one launch).
//   MODE_CDE:       a = net(x, y, T-t)                          (models/diffusion.py:27-46)
//   MODE_POSTERIOR: a = g (lik(x, y, T-t) + prior(x, T-t))      (nets.py:155-157 via the same loop)
//   MODE_CDIFFE:    y_t ~ q(y_t | y) at T-t, a = net(x, y_t, T-t)[:xdim]   (repaired
//                   models/diffusion.py:158-180; the y part of the joint update is discarded)
// then mu = g a + 0.5 beta x, x <- x + delta mu + sqrt(delta) g xi.
//
// Work distribution (persistent, preemptive): the G = grid.x workgroups of a y -- at most as many as
// the GPU holds at once -- share its 32-chain tiles through the balanced WaveSchedule of
// dmip_device.h (McNaughton's wrap-around rule, hand-over of split tiles through global memory):
// every wave of every CU stays busy to the end, and a chain's arithmetic does not depend on which
// wave runs it (bit-identical to an unsplit run).
// STAMP: diagnostic build only (dmip_em_sample_stamps) -- per-wave cycle sums of the step phases
// [layer 1 + B1, hidden layers, output layer + RNG + EM update], written to p.stamps.
template <int MODE, int W, int NL, int D, int M, int NW, int R, bool RES>
struct SamplerLds {
  static constexpr int NNET = MODE == MODE_POSTERIOR ? 2 : 1;
  static constexpr int NV = MODE == MODE_CDIFFE ? D + M + 1 : D + 1;  // inputs that vary per chain
  static constexpr int K1S = k1s_of(3 * NV + 2);
  static constexpr bool AOR = NNET > 1 && W >= 512;  // output layers through the ring (Lay)
  static constexpr bool L1R = MODE == MODE_CDIFFE && W >= 512;  // layer 1 through the ring (Lay)
  using L = Lay<W, NL, K1S, NNET, R, RES, AOR, L1R>;
  static constexpr int TOTAL = L::TOTAL;
};

template <int MODE, int W, int NL, int D, int M, int NW, int R, bool RES, bool NOISE, bool STAMP = false,
          int DIAG = 0>
__global__ void __launch_bounds__(NW * 64, (NW * 64 + 255) / 256)
em_sampler_kernel(SamplerParams p) {
  using SL = SamplerLds<MODE, W, NL, D, M, NW, R, RES>;
  constexpr int NNET = SL::NNET;
  constexpr int NV = SL::NV;
  constexpr int K1S = SL::K1S;
  using L = typename SL::L;
  static_assert(SL::TOTAL <= 160 * 1024, "LDS budget");
  static_assert(RES || (L::KS % NW == 0), "ring pieces per wave");
  static_assert(D <= 4, "sampler output rows are duplicated into both lane halves (D <= 4)");
  static_assert(!(NOISE && MODE != MODE_CDE), "noise injection: CDE only");
  __shared__ __attribute__((aligned(16))) char lds[SL::TOTAL];

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = lane >> 5;
  const int yi = blockIdx.y;

  Engine<W, NL, K1S, NNET, NW, R, RES, NOISE, DIAG, SL::AOR, SL::L1R> eng{lds, {p.hidden, p.hidden2}, 0, w, lane};
  {
    const size_t a1_stride = (size_t)L::T * K1S * 1024;
    const char* const a1[2] = {p.a1 + (p.a1_per_y ? yi * a1_stride : 0), p.a1_2};
    const char* const ao[2] = {p.ao, p.ao2};
    const float* const bh[2] = {p.bias_hidden, p.bias_hidden2};
    const float* const bo[2] = {p.bias_out, p.bias_out2};
    eng.prologue(a1, ao, bh, bo);
  }
  // CDiffE: this workgroup's observation, read from LDS every step (wave-uniform broadcast)
  __shared__ float yobs[M > 0 ? M : 1];
  if constexpr (MODE == MODE_CDIFFE) {
    stage_floats(yobs, p.y_obs + (size_t)yi * M, M, threadIdx.x, NW * 64);
    __syncthreads();
  }
  // ---- this wave's schedule (wave-uniform)
  const int S = p.num_steps;
  const long long tiles_y = (p.n_chains + 31) / 32;
  const long long n_waves = (long long)gridDim.x * NW;  // waves sharing this y
  const long long gw = (long long)blockIdx.x * NW + w;  // this wave among them
  constexpr int XW = sampler_xfer_words(D);
  const WaveSchedule sched(tiles_y, S, n_waves, gw);
  const int n_seg = sched.n_seg;

  unsigned long long ph[3] = {0, 0, 0};
  unsigned long long clk0 = 0, rt0 = 0;
  if constexpr (STAMP) {
    clk0 = stamp();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }
  const size_t noise_step = (size_t)gridDim.y * p.n_chains * D;

  for (int sgi = 0; sgi < n_seg; ++sgi) {
  const Seg sg = sched.segment(sgi);
  const long long c_local = (long long)(sg.job >= 0 ? sg.job : 0) * 32 + (lane & 31);
  const bool valid = sg.job >= 0 && c_local < p.n_chains;
  const long long c_rd = valid ? c_local : 0;
  float x[D];
  Rng rng;
  bool lost = false;  // the hand-over never arrived: the tile's output is poisoned and reported
  if (sg.kind == 2) {  // resume the tile the previous wave of the grid handed over
    const size_t slot = (size_t)yi * n_waves + gw - 1;
    // bounded: never hang the GPU (the flag is normally set C - S steps early)
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
    float n[D];
    if constexpr (NOISE) {
      const float* src = p.noise + (((size_t)yi * p.n_chains + c_rd) * D);
#pragma unroll
      for (int k = 0; k < D; ++k) n[k] = src[k];
    } else {
      rng_normals<D>(rng, n);
    }
#pragma unroll
    for (int k = 0; k < D; ++k) x[k] = __fadd_rn(__fmul_rn(n[k], p.stdv), p.mean);
  }

  SnapCursor snap(p.snap_every, sg.s0);
  for (int i = sg.s0; i < sg.s1; ++i) {
    unsigned long long t0 = 0, t1 = 0, t2 = 0;
    if constexpr (STAMP) t0 = stamp();
    const StepCoef cf = step_coef(sg.kind == 3 ? 0 : i, S, p.T, p.bmin, p.bdiff);
    float v[NV];
#pragma unroll
    for (int k = 0; k < D; ++k) v[k] = x[k];
    if constexpr (MODE == MODE_CDIFFE) {
      // y_t = eps * std(T-t) + mean_weight(T-t) * y  (sdes.py:37-44, on the observation part of z_0)
      const float mw = vp_mean_weight(cf.tau, p.bmin, p.bdiff);
      const float sd = vp_std(cf.tau, p.bmin, p.bdiff);
      float eps[M];
      rng_normals<M>(rng, eps);
#pragma unroll
      for (int k = 0; k < M; ++k) v[D + k] = __fadd_rn(__fmul_rn(eps[k], sd), __fmul_rn(mw, yobs[k]));
      asm volatile("" ::: "memory");  // keep the observation in LDS, not in registers across the step
    }
    v[NV - 1] = cf.tau;
    bf16x8 B1[K1S];
    build_b1<NV, K1S>(v, h, B1);
    if constexpr (MODE != MODE_CDE) __builtin_amdgcn_sched_barrier(0);
    if constexpr (MODE == MODE_CDIFFE) {
      // Langevin corrector steps at this time, before the predictor (Song et al. 2021 PC sampling):
      // s = a/g, eps = 2 alpha (snr |z| / |s|)^2 with the norms at their expected values for the VP
      // perturbation kernel (|z| ~ sqrt(d), |s| ~ sqrt(d) / std(T - t)), i.e. eps = 2 alpha snr^2
      // var(T - t) -- one step size per time step, as score_sde's batch-averaged norms give, instead of a
      // per-chain ratio that explodes where a chain's |s| is small (measured: profiles/r3_e2e_cdiffe_pc.json);
      // x <- x + eps s + sqrt(2 eps) z, alpha = exp(-beta delta) (the discrete VP alpha 1 - beta delta of
      // score_sde, kept positive for coarse step counts). y_t is held fixed; only x's slots of the
      // layer-1 operand change.
      for (int c = 0; c < p.n_corr; ++c) {
        const f32x16 oc = eng.eval(B1);
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
        for (int k = 0; k < D; ++k) x[k] = x[k] + es * sc[k] + ns * z[k];
        patch_b1_x<NV, D, K1S>(x, h, B1);
      }
    }
    if constexpr (STAMP) t1 = stamp();
    f32x16 out = eng.eval(B1);
    if constexpr (STAMP) t2 = stamp();
    float xi[D];
    if constexpr (NOISE) {
      const float* src = p.noise + noise_step * (sg.kind == 3 ? 1 : i + 1) + (((size_t)yi * p.n_chains + c_rd) * D);
#pragma unroll
      for (int k = 0; k < D; ++k) xi[k] = src[k];
    } else {
      rng_normals<D>(rng, xi);
    }
#pragma unroll
    for (int k = 0; k < D; ++k) {
      // PosteriorScore returns g * (prior + likelihood) (nets.py:155-157)
      const float a = MODE == MODE_POSTERIOR ? __fmul_rn(cf.g, out[k]) : out[k];
      x[k] = em_update(x[k], a, xi[k], cf, p.delta, p.sqrt_delta);
    }
    snap.at_step<D>(i, p.snap_every, p.snap_out, gridDim.y, yi, p.n_chains, c_local, sg.kind != 3 && valid && h == 0, x);
    if constexpr (STAMP) {
      const unsigned long long t3 = stamp();
      ph[0] += t1 - t0;
      ph[1] += t2 - t1;
      ph[2] += t3 - t2;
    }
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
  } else if (sg.kind != 3 && valid && h == 0) {
    float* dst = p.x_out + ((size_t)yi * p.n_chains + c_local) * D;
#pragma unroll
    for (int k = 0; k < D; ++k) dst[k] = x[k];
  }
  }  // segments
  eng.epilogue();
  if constexpr (STAMP) {
    const unsigned long long clk1 = stamp();
    const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
      unsigned long long* o = p.stamps + ((size_t)(blockIdx.y * gridDim.x + blockIdx.x) * NW + w) * 5;
      o[0] = ph[0];
      o[1] = ph[1];
      o[2] = ph[2];
      o[3] = clk1 - clk0;  // shader clock ticks over the step loop
      o[4] = rt1 - rt0;    // 100 MHz constant clock over the same span
    }
  }
}

// ---------------------------------------------------------------------- MLP forward kernel
// out[n] = MLP(cat[x, y, t]) for arbitrary rows (model.sde.a(x, y, t), nets.py:32-35); every
// input column varies per row, so layer 1 takes the whole row as split-bf16 slots.
template <int W, int NL, int IN, int NW, int R, bool RES, bool SPLIT = true>
__global__ void __launch_bounds__(NW * 64, (NW * 64 + 255) / 256)
mlp_forward_kernel(ForwardParams p) {
  // SPLIT: layer-1 slots [hi(v) | lo(v) | hi(v) | 1 | 1] (~fp32); otherwise [v | 1 | 1] (bf16 inputs,
  // used where the split image does not fit the LDS budget: width 512 with wide inputs)
  constexpr int K1S = SPLIT ? (3 * IN + 2 + 15) / 16 : (IN + 2 + 15) / 16;
  using L = Lay<W, NL, K1S, 1, R, RES>;
  static_assert(L::TOTAL <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) char lds[L::TOTAL];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = lane >> 5;
  Engine<W, NL, K1S, 1, NW, R, RES, true> net{lds, {p.hidden, p.hidden}, 0, w, lane};
  {
    const char* const a1[2] = {p.a1, p.a1};
    const char* const ao[2] = {p.ao, p.ao};
    const float* const bh[2] = {p.bias_hidden, p.bias_hidden};
    const float* const bo[2] = {p.bias_out, p.bias_out};
    net.prologue(a1, ao, bh, bo);
  }

  const long long n_tiles = (p.n + 31) / 32;
  const long long rounds = (n_tiles + (long long)gridDim.x * NW - 1) / ((long long)gridDim.x * NW);
  for (long long rd = 0; rd < rounds; ++rd) {
    const long long tile = (rd * gridDim.x + blockIdx.x) * NW + w;
    const long long row = tile * 32 + (lane & 31);
    const bool valid = row < p.n;
    float v[IN];
    const long long rr = valid ? row : 0;
#pragma unroll
    for (int k = 0; k < IN; ++k) {
      float val;
      if (k < p.xdim) val = p.x[rr * p.xdim + k];
      else if (k < p.xdim + p.ydim) val = p.y[(p.y_stride ? rr * p.y_stride : 0) + (k - p.xdim)];
      else val = p.t[p.t_stride ? rr : 0];
      v[k] = val;
    }
    __bf16 vh[IN], vl[IN];
#pragma unroll
    for (int k = 0; k < IN; ++k) {
      vh[k] = (__bf16)v[k];
      vl[k] = (__bf16)(v[k] - (float)vh[k]);
    }
    bf16x8 B1[K1S];
#pragma unroll
    for (int s = 0; s < K1S; ++s) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        auto slot = [&](int k) -> __bf16 {
          if constexpr (SPLIT) {
            if (k < IN) return vh[k];
            if (k < 2 * IN) return vl[k - IN];
            if (k < 3 * IN) return vh[k - 2 * IN];
            if (k < 3 * IN + 2) return (__bf16)1.0f;
          } else {
            if (k < IN) return vh[k];
            if (k < IN + 2) return (__bf16)1.0f;
          }
          return (__bf16)0.0f;
        };
        B1[s][j] = h ? slot(16 * s + 8 + j) : slot(16 * s + j);
      }
    }
    const f32x16 out = net.eval(B1);
    if (valid) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int orow = (r & 3) + 8 * (r >> 2) + 4 * h;
        if (orow < p.out_dim) p.out[row * p.out_dim + orow] = out[r];
      }
    }
  }
  net.epilogue();
}

// ------------------------------------------------------------------ per-y layer-1 prep kernel
// A1 fragment blocks for the sampler: row j of the augmented layer-1 matrix is
//   [hi(cW_v) | hi(cW_v) | lo(cW_v) | hi(c_j) | lo(c_j) | 0...]   (v = x columns, then t)
// with c = 2 log2(e) and c_j = c (b1_j + W1_{j,y} . y) -- the y-conditioning is hoisted out of
// the step loop into this per-y bias.
__global__ void a1_prep_kernel(A1PrepParams p) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int yi = blockIdx.y;
  if (j >= p.width) return;
  const float* wrow = p.w1 + (size_t)j * p.in_dim;
  double cj = p.b1[j];
  for (int m = 0; m < p.ydim; ++m) cj += (double)wrow[p.y_col0 + m] * (double)p.y[(size_t)yi * p.ydim + m];
  cj *= (double)kTanhScale;
  const int nv = p.xdim + 1;
  const int kpad = p.k1s * 16;
  __bf16* blk = (__bf16*)(p.a1 + (size_t)yi * (p.width / 32) * p.k1s * 1024);
  const int rt = j / 32, i = j % 32;
  for (int k = 0; k < kpad; ++k) {
    float val = 0.0f;
    int vk = -1, part = 0;
    if (k < nv) { vk = k; part = 0; }
    else if (k < 2 * nv) { vk = k - nv; part = 0; }
    else if (k < 3 * nv) { vk = k - 2 * nv; part = 1; }
    if (vk >= 0) {
      const int col = vk < p.xdim ? vk : p.t_col;
      const float cw = (float)((double)kTanhScale * (double)wrow[col]);
      const __bf16 hi = (__bf16)cw;
      val = part == 0 ? (float)hi : (float)(__bf16)(cw - (float)hi);
    } else if (k == 3 * nv) {
      val = (float)(__bf16)(float)cj;
    } else if (k == 3 * nv + 1) {
      const float cf = (float)cj;
      val = (float)(__bf16)(cf - (float)(__bf16)cf);
    }
    const int s = k / 16, hh = (k % 16) / 8, jj = k % 8;
    const int ln = i + 32 * hh;
    blk[((size_t)(rt * p.k1s + s) * 64 + ln) * 8 + jj] = (__bf16)val;
  }
}

// --------------------------------------------------------------------------- debug kernels
__global__ void rng_words_kernel(unsigned long long seed, long long chain_offset, unsigned long long stream,
                                 long long n, int n_words, unsigned int* out) {
  const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  Rng r = rng_init(seed, (uint64_t)(chain_offset + c), stream);
  for (int k = 0; k < n_words; ++k) out[c * n_words + k] = rng_next(r);
}

__global__ void rng_normals_kernel(unsigned long long seed, long long chain_offset, unsigned long long stream,
                                   long long n, int n_pairs, float* out) {
  const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  Rng r = rng_init(seed, (uint64_t)(chain_offset + c), stream);
  for (int k = 0; k < n_pairs; ++k) {
    float a, b;
    rng_normal_pair(r, a, b);
    out[(c * n_pairs + k) * 2] = a;
    out[(c * n_pairs + k) * 2 + 1] = b;
  }
}

__global__ void schedule_kernel(int S, float T, float bmin, float bdiff, float* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > S) return;
  const float ts = __fmul_rn(linspace_at(i, S), T);
  const StepCoef c = step_coef(i, S, T, bmin, bdiff);
  out[i * 4 + 0] = ts;
  out[i * 4 + 1] = c.tau;
  out[i * 4 + 2] = c.beta;
  out[i * 4 + 3] = c.g;
}

// ------------------------------------------------------------------------------ dispatch
// workgroups per y: enough to fill every CU slot once (the kernel balances the work inside a
// workgroup), never more than one per NW tiles
template <typename Kern>
static unsigned sampler_wgs_per_y(Kern kern, int nthreads, long long n_chains, int n_y, hipStream_t st) {
  // the hand-over schedule needs every workgroup of the grid resident at once, so the slot count is
  // that of the stream's device (cached per device and kernel instantiation)
  const int slots = resident_slots(kern, nthreads, st);
  const long long nw = nthreads / 64;
  const long long tiles = (n_chains + 31) / 32;
  long long g = slots / (n_y > 0 ? n_y : 1);
  const long long cap = (tiles + nw - 1) / nw;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (unsigned)g;
}

// the hand-over buffers of a launch: per y and grid wave, the state words and a flag (zeroed)
static hipError_t with_xfer(SamplerParams& p, const dim3& grid, int nw, int d, hipStream_t st, char** buf) {
  return alloc_handover((size_t)grid.x * grid.y * nw, d, st, buf, &p.xfer, &p.xflag);
}

hipError_t alloc_handover(size_t slots, int d, hipStream_t st, char** buf, float** xfer, unsigned** xflag) {
  const size_t state_bytes = slots * sampler_xfer_words(d) * sizeof(float);
  hipError_t e = hipMallocAsync((void**)buf, state_bytes + slots * sizeof(unsigned), st);
  if (e != hipSuccess) return e;
  *xfer = (float*)*buf;
  *xflag = (unsigned*)(*buf + state_bytes);
  // only the flags are zeroed: a consumer reads a slot's state only after its flag is set, and writes NaN
  // (not the slot's contents) for a tile whose hand-over never arrived. (Zeroing the state too was ~5 MB of
  // memset traffic per headline launch.)
  return hipMemsetAsync(*xflag, 0, slots * sizeof(unsigned), st);
}

template <int MODE, int W, int NL, int D, int M, int NW, int R, bool RES>
static hipError_t launch_sampler_t(const SamplerParams& p_in, int n_y, hipStream_t st) {
  const dim3 grid(sampler_wgs_per_y(em_sampler_kernel<MODE, W, NL, D, M, NW, R, RES, false>, NW * 64, p_in.n_chains, n_y, st),
                  (unsigned)n_y);
  SamplerParams p = p_in;
  char* buf = nullptr;
  hipError_t e = with_xfer(p, grid, NW, D, st, &buf);
  if (e != hipSuccess) return e;
  if constexpr (MODE == MODE_CDE) {
    if (p.stamps)
      hipLaunchKernelGGL((em_sampler_kernel<MODE, W, NL, D, M, NW, R, RES, false, true>), grid, dim3(NW * 64), 0, st, p);
    else if (p.noise)
      hipLaunchKernelGGL((em_sampler_kernel<MODE, W, NL, D, M, NW, R, RES, true>), grid, dim3(NW * 64), 0, st, p);
    else
      hipLaunchKernelGGL((em_sampler_kernel<MODE, W, NL, D, M, NW, R, RES, false>), grid, dim3(NW * 64), 0, st, p);
  } else {
    hipLaunchKernelGGL((em_sampler_kernel<MODE, W, NL, D, M, NW, R, RES, false>), grid, dim3(NW * 64), 0, st, p);
  }
  e = hipGetLastError();
  (void)hipFreeAsync(buf, st);
  return e;
}

template <int W, int NL, int IN, int NW, int R, bool RES, bool SPLIT = true>
static hipError_t launch_forward_t(const ForwardParams& p, hipStream_t st) {
  const long long tiles = (p.n + 31) / 32;
  long long wgs = (tiles + NW - 1) / NW;
  if (wgs > 2048) wgs = 2048;
  if (wgs < 1) wgs = 1;
  hipLaunchKernelGGL((mlp_forward_kernel<W, NL, IN, NW, R, RES, SPLIT>), dim3((unsigned)wgs), dim3(NW * 64), 0, st, p);
  return hipGetLastError();
}

// Compiled shapes: widths 64 / 128 (hidden layers LDS-resident), 256 (4-slot ring) and 512 (4-wave
// workgroups, 3 x 32 KiB ring slots; Posterior with its output layers and CDiffE with its layer 1 in
// the ring); 2 or 3 hidden layers; xdim 2 or 3. The CDE and
// Posterior kernels take any ydim (y is folded into the per-y layer-1 bias, M = 0); CDiffE feeds y_t
// through layer 1 and is compiled for the two problems' (xdim, ydim) = (2, 2) and (3, 23).
#define DMIP_W_CASES(X, MODE, NL, D, M) \
  X(MODE, 64, NL, D, M, 8, 0, true)     \
  X(MODE, 128, NL, D, M, 8, 0, true)    \
  X(MODE, 256, NL, D, M, 8, 4, false)
#define DMIP_W512_CASE(X, MODE, NL, D, M) X(MODE, 512, NL, D, M, 4, 3, false)
#define DMIP_SHAPES(X, MODE, W512, M2, M3)                              \
  DMIP_W_CASES(X, MODE, 3, 2, M2) DMIP_W_CASES(X, MODE, 3, 3, M3)      \
  DMIP_W_CASES(X, MODE, 2, 2, M2) DMIP_W_CASES(X, MODE, 2, 3, M3)      \
  W512(X, MODE, 3, 2, M2) W512(X, MODE, 3, 3, M3) W512(X, MODE, 2, 2, M2) W512(X, MODE, 2, 3, M3)
#define DMIP_ALL_SHAPES(X)                                \
  DMIP_SHAPES(X, MODE_CDE, DMIP_W512_CASE, 0, 0)          \
  DMIP_SHAPES(X, MODE_POSTERIOR, DMIP_W512_CASE, 0, 0)    \
  DMIP_SHAPES(X, MODE_CDIFFE, DMIP_W512_CASE, 2, 23)

// Development knob (not part of the ABI): DMIP_SAMPLER_VARIANT=10x runs the timing ablations
// (DIAG = x) of the width-256 CDE sampler; see profiles/README.md.
static int sampler_variant() {
  const char* e = getenv("DMIP_SAMPLER_VARIANT");
  return e ? atoi(e) : 0;
}

hipError_t launch_sampler(const SamplerParams& p_in, int mode, int width, int n_hidden, int xdim, int ydim, int n_y,
                          hipStream_t st, bool* supported) {
  *supported = true;
  const int var = sampler_variant();
  if (mode == MODE_CDE && width == 256 && n_hidden == 3 && xdim == 3 &&
      var >= 101 && var <= 107) {
    const dim3 grid(sampler_wgs_per_y(em_sampler_kernel<MODE_CDE, 256, 3, 3, 0, 8, 4, false, false>, 512,
                                      p_in.n_chains, n_y, st),
                    (unsigned)n_y);
    SamplerParams p = p_in;
    char* buf = nullptr;
    hipError_t e = with_xfer(p, grid, 8, 3, st, &buf);
    if (e != hipSuccess) return e;
    switch (var) {
#define DG(d) \
  case 100 + d: hipLaunchKernelGGL((em_sampler_kernel<MODE_CDE, 256, 3, 3, 0, 8, 4, false, false, false, d>), grid, dim3(512), 0, st, p); break;
      DG(1) DG(2) DG(3) DG(4) DG(5) DG(6) DG(7)
#undef DG
      default: break;
    }
    e = hipGetLastError();
    (void)hipFreeAsync(buf, st);
    return e;
  }
  const SamplerParams& p = p_in;
#define X(MODEv, Wv, NLv, Dv, Mv, NWv, Rv, RESv)                                                  \
  if (mode == MODEv && width == Wv && n_hidden == NLv && xdim == Dv && (Mv == 0 || ydim == Mv)) \
    return launch_sampler_t<MODEv, Wv, NLv, Dv, Mv, NWv, Rv, RESv>(p, n_y, st);
  DMIP_ALL_SHAPES(X)
#undef X
  *supported = false;
  return hipSuccess;
}

bool sampler_shape_supported(int mode, int width, int n_hidden, int xdim, int ydim) {
#define X(MODEv, Wv, NLv, Dv, Mv, NWv, Rv, RESv) \
  if (mode == MODEv && width == Wv && n_hidden == NLv && xdim == Dv && (Mv == 0 || ydim == Mv)) return true;
  DMIP_ALL_SHAPES(X)
#undef X
  return false;
}

constexpr bool forward_split_c(int width, int in_dim) { return width < 512 || 3 * in_dim + 2 <= 32; }
bool forward_split(int width, int in_dim) { return forward_split_c(width, in_dim); }

hipError_t launch_forward(const ForwardParams& p, int width, int n_hidden, int in_dim, hipStream_t st,
                          bool* supported) {
  *supported = true;
  if (width == 512) {
    // 32 KiB ring slots: two slots, and layer 1 split only while its image stays at 32 KiB
#define X5(NLv, INv)              \
    if (n_hidden == NLv && in_dim == INv) \
      return launch_forward_t<512, NLv, INv, 4, 2, false, forward_split_c(512, INv)>(p, st);
    X5(3, 5) X5(3, 27) X5(3, 3) X5(3, 4)
#undef X5
    *supported = false;
    return hipSuccess;
  }
#define X(Wv, NWv, Rv, RESv, NLv, INv) \
  if (width == Wv && n_hidden == NLv && in_dim == INv) return launch_forward_t<Wv, NLv, INv, NWv, Rv, RESv>(p, st);
#define XW(NLv, INv) X(64, 8, 0, true, NLv, INv) X(128, 8, 0, true, NLv, INv) X(256, 8, 4, false, NLv, INv)
  // CDE / likelihood nets x(2) y(2) t and x(3) y(23) t; prior MLP2 nets x t; CDiffE: same input widths
  XW(3, 5) XW(3, 27) XW(3, 3) XW(3, 4) XW(2, 5) XW(2, 27) XW(2, 3) XW(2, 4)
#undef XW
#undef X
  *supported = false;
  return hipSuccess;
}

hipError_t launch_a1_prep(const A1PrepParams& p, int n_y, hipStream_t st) {
  dim3 grid((unsigned)((p.width + 127) / 128), (unsigned)n_y);
  hipLaunchKernelGGL(a1_prep_kernel, grid, dim3(128), 0, st, p);
  return hipGetLastError();
}

hipError_t launch_rng_words(unsigned long long seed, long long off, unsigned long long stream, long long n,
                            int n_words, unsigned int* out, hipStream_t st) {
  hipLaunchKernelGGL(rng_words_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, seed, off, stream, n,
                     n_words, out);
  return hipGetLastError();
}

hipError_t launch_rng_normals(unsigned long long seed, long long off, unsigned long long stream, long long n,
                              int n_pairs, float* out, hipStream_t st) {
  hipLaunchKernelGGL(rng_normals_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, seed, off, stream, n,
                     n_pairs, out);
  return hipGetLastError();
}

hipError_t launch_schedule(int S, float T, float bmin, float bdiff, float* out, hipStream_t st) {
  hipLaunchKernelGGL(schedule_kernel, dim3((unsigned)((S + 256) / 256)), dim3(256), 0, st, S, T, bmin, bdiff, out);
  return hipGetLastError();
}

}  // namespace dmip
