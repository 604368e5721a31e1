// fp32-accurate CDE sampler, k-major multi-tile engine: DMIP_PREC_F32X3 at the headline shape (scatterometry
// and linear CDE, hidden_layers [256]*3, BASELINE configs[1]).
//
// Same arithmetic as dmip_x3.h (every product W_hi h_hi + W_hi h_lo + W_lo h_hi on v_mfma_f32_16x16x32_f16,
// fp32 accumulation, r-form tanh by exp2 + rcp); a different work decomposition, set by what bounds the
// one-tile-per-wave engine (profiles/r3_x3_pmc.txt): with 128 chains per CU each step streams the two
// 256 KiB hidden layers from L2 into LDS (4 bytes per weight: hi and lo), so the LDS-DMA issue, the
// per-chunk barriers and the layer-1 VALU phase -- which the two lock-stepped waves of a SIMD reach
// together -- cost more than the matrix work leaves room for. Here:
//   * one wave per SIMD holds NT chain tiles (16 chains each: 48 chains at NT = 3, 384 registers of
//     activations), so every streamed weight byte feeds NT x as many MFMAs;
//   * the W x W layers stream k-major: chunk q of a layer is k-step q (32 input units) of all 16 output
//     tiles, hi and lo fragments (32 KiB). A layer's input is consumed one k-step per chunk, so the
//     previous layer's activation (and layer 1's double tanh) is spread over the 8 chunks beside their
//     MFMAs instead of sitting in a VALU-only phase; all 16 output tiles accumulate in registers;
//   * 16 chunks per step on a 4-slot ring: chunk k of a step is always in slot k % 4, so every ring
//     address, source offset and DMA destination is a compile-time constant; the DMA is
//     buffer_load_dwordx4 ... lds with the image offset in an SGPR (no per-lane address arithmetic);
//   * hidden layer 2 streams as two output halves (each k-major, two k-steps per chunk), so half 1 runs the
//     output layer over half 0's finished units beside its MFMAs (layer2); ring fragments are read one o-step
//     ahead, and the chains' RNG states wait in LDS through the step (the registers that layout needs);
//   * the output layer (3 rows) is LDS-resident as one fragment per k-step: rows 0..D-1 hold W_hi, rows
//     4..4+D-1 W_lo, so A . h_hi yields W_hi h_hi and W_lo h_hi in lane groups 0 and 1 and A . h_lo yields
//     W_hi h_lo in group 0 (8 KiB instead of a 16-row hi + lo chunk);
//   * the step's work that does not depend on the network leaves the matrix-idle phases (round 5): the EM
//     update's normals are drawn inside hidden layer 2's last chunk (free of output-layer work), lane group t
//     drawing chain tile t's (one Box-Muller pass for all NT tiles instead of NT), and parked in LDS beside the
//     RNG states; the step coefficients (tau, beta, g) come from a per-launch table (scalar loads) instead of
//     a division and an f64 square root per step; the output rows' partial sums meet by v_permlane16/32_swap
//     (no LDS round trip); the resident layer-1 image holds lane groups 0-1 only (groups 2-3 of the layer-1
//     B operand are zero k-slots, so those lanes read group 0-1's finite weights), which frees the LDS for
//     the normals.
// The hidden layers accumulate each output element in the order of dmip_x3.h (k-steps ascending; per
// k-step hi.h_lo, lo.h_hi, hi.h_hi): bit-identical hidden activations; the output layer's three partial
// sums are added at the end ((hi.h_hi + hi.h_lo) + lo.h_hi), within an ulp of the one-chain order.
// Chain state, RNG, schedule, EM update, snapshots and hand-over are the other engines' (dmip_device.h).
#pragma once
#include "dmip_x3.h"

namespace dmip {
namespace x3k {

using x3::f32x4;
using x3::mfma16;

constexpr int W = 256, ST = 16, KQ = 8, NH = 2;  // [256]*3: layer 1 + two W x W layers
constexpr int CHUNK = 32768;                     // k-step q of a W x W layer: 16 tiles x (hi, lo) x 1 KiB
constexpr int NCHUNK = NH * KQ;                  // ring chunks per step
constexpr int R = 4;                             // ring slots
#ifndef DMIP_X3K_PF
#define DMIP_X3K_PF 1
#endif
#ifndef DMIP_X3K_SYNC_O
#define DMIP_X3K_SYNC_O 8
#endif
constexpr int PF = DMIP_X3K_PF;                  // ring fragment pairs read ahead (o-steps)
constexpr int SYNC_O = DMIP_X3K_SYNC_O;          // the o-step of a chunk that holds the next chunk's barrier
static_assert(SYNC_O + PF < 16 && SYNC_O < 15, "the barrier precedes the next chunk's first reads, pieces follow it");
// waves per workgroup: one per SIMD for 2-3 chain tiles per wave (up to 512 registers), two per SIMD for
// one tile per wave (<= 256 registers: each wave's VALU chains issue between the other's MFMAs)
template <int NT>
struct KWaves {
  static constexpr int NWV = NT == 1 ? 8 : 4;
  static constexpr int PPW = CHUNK / 1024 / NWV;  // LDS-DMA pieces per wave per chunk
};
static_assert(NCHUNK % R == 0, "static ring: chunk k of every step in slot k % R");

struct KLay {
  // [16 tiles][32 lanes][8 fp16] (K1Q = 1): lanes 32-63 hold k-slots 16-31, zero in the B operand of every
  // x3k shape (3 (D + 1) <= 15 slots), so they read lanes 0-31's (finite) fragments instead
  static constexpr int L1 = 0, L1_BYTES = ST * 512;
  static constexpr int OUT = L1 + L1_BYTES, OUT_BYTES = KQ * 1024;  // [8 k-steps][64][8]
  static constexpr int BIAS = OUT + OUT_BYTES;            // floats: c(b1 + W1_y y) | hidden 1 | hidden 2 | out[16]
  static constexpr int BF = (NH + 1) * W + 16;
  static constexpr int BIAS_BYTES = (BF * 4 + 15) / 16 * 16;
  static constexpr int RING = BIAS + BIAS_BYTES;
  // the chains' RNG states, parked in LDS while the network is evaluated ([wave][tile][word][16 chains]): 12
  // registers fewer through the step
  static constexpr int RNGP = RING + R * CHUNK, RNGP_BYTES = 3072;
  // the EM update's normals of the step, drawn in hidden layer 2 ([wave][tile][k][16 chains] floats, k < 3)
  static constexpr int NRM = RNGP + RNGP_BYTES, NRM_BYTES = 2304;
  static constexpr int TOTAL = NRM + NRM_BYTES;
};
static_assert(KLay::TOTAL <= 160 * 1024, "LDS budget");

typedef __attribute__((address_space(3))) void lds_void;

// diagnostic phase stamps (DIAG & 2 only, never in a product kernel): the shader cycle counter, read in an
// asm statement so that no code moves across it
__device__ __forceinline__ uint64_t stamp() {
  uint64_t t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
  return t;
}

// activate k-step q's two input tiles (z0 = tile 2q, z1 = tile 2q + 1) into the (hi, lo) B operands:
// dword d of the operand carries units (2d, 2d + 1) of the lane's 8 k-slots (dmip_x3.h act_store)
template <bool L1>
__device__ __forceinline__ void act_kstep(const f32x4& z0, const f32x4& z1, u32x4& hh, u32x4& hl) {
  float r[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    r[k] = L1 ? x3::x3_act_r2(z0[k]) : x3::x3_act_r(z0[k]);
    r[4 + k] = L1 ? x3::x3_act_r2(z1[k]) : x3::x3_act_r(z1[k]);
  }
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    uint32_t h, l;
    x3::split_pair(r[2 * d], r[2 * d + 1], h, l);
    hh[d] = h;
    hl[d] = l;
  }
}

template <int D, int NT, bool NOISE, int DIAG>
struct KEngine {
  static constexpr int NWV = KWaves<NT>::NWV, PPW = KWaves<NT>::PPW;
  char* lds;
  const char* ring_lane;  // ring base + 16 lane
  const char* out_lane;   // resident output fragments + 16 lane
  __amdgpu_buffer_rsrc_t rs;
  unsigned voff;          // this wave's DMA pieces: w PPW KiB + 16 lane
  int w, g;
  uint32_t* rng_park;  // this wave's parked RNG states [tile][word][16 chains]
  float* nrm;          // this wave's normals of the step [tile][k][16 chains]
  mutable uint64_t ph_vm = 0, ph_bar = 0;  // DIAG & 2: cycles in the ring's vmcnt waits and barriers

  // piece Q of chunk C of the step image into slot S (LDS-DMA: 1 KiB per wave-instruction)
  // (round 6: the instruction's 12-bit offset carries Q's KiB within a group of four pieces -- the hardware adds it to
  // both the memory and the LDS address -- so four consecutive pieces share M0 and the scalar offset: two scalar moves
  // per four pieces instead of two per piece)
  template <int C, int S, int Q>
  __device__ __forceinline__ void issue_piece() const {
    constexpr int QH = Q >> 2, QL = Q & 3;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(lds + KLay::RING + S * CHUNK + (w * PPW + 4 * QH) * 1024),
                                             16, voff, C * CHUNK + QH * 4096, QL * 1024, 0);
  }
  template <int C, int S, int Q = 0>
  __device__ __forceinline__ void issue() const {
    if constexpr (Q < PPW) {
      issue_piece<C, S, Q>();
      issue<C, S, Q + 1>();
    }
  }

  // Ring protocol. Chunk K's barrier B(K) sits in the MIDDLE of chunk K - 1 (o-step 8), not at a chunk
  // boundary: before it each wave waits for its own pieces of chunk K (vmcnt), after it every wave's
  // pieces have landed and every wave has finished chunk K - 2, whose slot ((K + 2) % R) the rest of
  // chunk K - 1 refills with chunk K + 2, piece by piece beside its MFMAs. So the first fragments of
  // chunk K are read ahead at the end of chunk K - 1 (no LDS latency bubble at a chunk start), and the
  // barrier waits on nothing but the other waves (no lgkmcnt(0): every read of a refilled slot was consumed
  // by an MFMA whose operand wait has retired it).
  __device__ __forceinline__ void start(u32x4 (&fpre)[PF][2]) const {
    if constexpr (!(DIAG & 1)) {
      issue<0, 0>();
      issue<1, 1>();
      issue<2, 2>();
      wait_vmcnt<2 * PPW>();  // chunk 0 landed (this wave's pieces)
    }
    barrier();
    const x3::lds_cptr b0 = (x3::lds_cptr)ring_lane;
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      fpre[i][0] = x3::lds_rd<0>(b0 + i * 2048);
      fpre[i][1] = x3::lds_rd<1024>(b0 + i * 2048);
      x3::lds_wait2<0>(fpre[i][0], fpre[i][1]);
    }
  }

  __device__ __forceinline__ void barrier() const {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }

  // B(KN), in the middle of chunk KN - 1: this wave's pieces of chunk KN have landed (chunk KN + 1's, issued
  // in chunk KN - 2, may still be in flight), then the workgroup barrier
  template <int KN>
  __device__ __forceinline__ void sync_mid() const {
    if constexpr (DIAG & 1) return;
    uint64_t s0 = 0, s1 = 0;
    if constexpr (DIAG & 2) s0 = stamp();
    wait_vmcnt<PPW>();
    if constexpr (DIAG & 2) s1 = stamp(), ph_vm += s1 - s0;
    barrier();
    if constexpr (DIAG & 2) ph_bar += stamp() - s1;
  }

  __device__ __forceinline__ f32x4 bias4(int li, int o) const {
    return *(const f32x4*)((const float*)(lds + KLay::BIAS) + li * W + 16 * o + 4 * g);
  }

  // one W x W layer, k-major: In (f32 pre-activations of the previous layer, NT x 16 tiles) -> Out.
  // Hh/Hl hold k-step 0's operands on entry (activated by the caller); k-step q + 1's are activated
  // from In during chunk q, a slice per output tile beside that tile's MFMAs. fpre: the first PF
  // fragment pairs of the layer's first chunk on entry, of the next chunk on exit.
  template <int LI, bool IN_L1>
  __device__ __forceinline__ void layer(const f32x4 (&In)[NT][ST], f32x4 (&Out)[NT][ST], u32x4 (&Hh)[NT],
                                        u32x4 (&Hl)[NT], u32x4 (&fpre)[PF][2]) const {
#pragma unroll
    for (int o = 0; o < ST; ++o) {
      const f32x4 b = bias4(LI, o);
#pragma unroll
      for (int t = 0; t < NT; ++t) Out[t][o] = b;
    }
    chunk<LI, IN_L1, 0>(In, Out, Hh, Hl, fpre);
  }

  template <int LI, bool IN_L1, int Q>
  __device__ __forceinline__ void chunk(const f32x4 (&In)[NT][ST], f32x4 (&Out)[NT][ST], u32x4 (&Hh)[NT],
                                        u32x4 (&Hl)[NT], u32x4 (&fpre)[PF][2]) const {
    if constexpr (Q < KQ) {
      constexpr int K = (LI - 1) * KQ + Q;  // chunk index in the step
      const x3::lds_cptr base = (x3::lds_cptr)(ring_lane + (K % R) * CHUNK);
      const x3::lds_cptr nbase = (x3::lds_cptr)(ring_lane + ((K + 1) % R) * CHUNK);
      u32x4 Nh[NT], Nl[NT];
      u32x4 f[PF + 1][2];
#pragma unroll
      for (int i = 0; i < PF; ++i) f[i][0] = fpre[i][0], f[i][1] = fpre[i][1];
      ostep<LI, IN_L1, Q, 0>(base, nbase, In, Out, Hh, Hl, Nh, Nl, f, fpre);
      // the next chunk's first fragments (read at the last PF o-steps) are complete before they leave the
      // chunk: an asm load's registers must not be copied before its data lands
#pragma unroll
      for (int i = 0; i < PF; ++i) x3::lds_wait2<0>(fpre[i][0], fpre[i][1]);
      if constexpr (Q + 1 < KQ) {
#pragma unroll
        for (int t = 0; t < NT; ++t) Hh[t] = Nh[t], Hl[t] = Nl[t];
      }
      chunk<LI, IN_L1, Q + 1>(In, Out, Hh, Hl, fpre);
    }
  }

  // o-step O of chunk K = (LI, Q): tile O's 3 NT MFMAs (fragments read PF tiles ahead -- across the chunk
  // boundary at the last PF o-steps -- by explicit ds_read_b128 with counted lgkmcnt waits; left to itself the
  // compiler hoists all 32 reads to the chunk's top, 128 more registers), beside one slice of the work the
  // chunk carries: the activation of k-step Q + 1's operand pair (t, d) = (O / 4, O % 4) for O < 4 NT;
  // B(K + 1) at O = SYNC_O; LDS-DMA pieces of chunk K + 3 after it. (The asm reads and waits are scheduling
  // boundaries: what is placed in an o-step stays beside its MFMAs.)
  template <int LI, bool IN_L1, int Q, int O>
  __device__ __forceinline__ void ostep(x3::lds_cptr base, x3::lds_cptr nbase, const f32x4 (&In)[NT][ST],
                                        f32x4 (&Out)[NT][ST], const u32x4 (&Hh)[NT], const u32x4 (&Hl)[NT],
                                        u32x4 (&Nh)[NT], u32x4 (&Nl)[NT], u32x4 (&f)[PF + 1][2],
                                        u32x4 (&fpre)[PF][2]) const {
    if constexpr (O < ST) {
      constexpr int K = (LI - 1) * KQ + Q;
      ring_pre<O>(base, nbase, f, fpre);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        Out[t][O] = mfma16(f[O % (PF + 1)][0], Hl[t], Out[t][O]);
        Out[t][O] = mfma16(f[O % (PF + 1)][1], Hh[t], Out[t][O]);
        Out[t][O] = mfma16(f[O % (PF + 1)][0], Hh[t], Out[t][O]);
      }
      if constexpr (Q + 1 < KQ && act_pair_at(O) >= 0) {
        constexpr int P = act_pair_at(O), t = P / 4, d = P % 4;
        const f32x4& z = In[t][2 * Q + 2 + d / 2];
        const int e = 2 * (d % 2);
        const float r0 = IN_L1 ? x3::x3_act_r2(z[e]) : x3::x3_act_r(z[e]);
        const float r1 = IN_L1 ? x3::x3_act_r2(z[e + 1]) : x3::x3_act_r(z[e + 1]);
        uint32_t h, l;
        x3::split_pair(r0, r1, h, l);
        Nh[t][d] = h;
        Nl[t][d] = l;
      }
      ring_post<K, O>();
      ostep<LI, IN_L1, Q, O + 1>(base, nbase, In, Out, Hh, Hl, Nh, Nl, f, fpre);
    }
  }

  // the ring's part of o-step O: the fragment pair PF o-steps ahead (across the chunk boundary at the last PF o-steps:
  // the next chunk's, whose barrier has passed at O = SYNC_O), then the wait for this o-step's pair
  template <int O>
  __device__ __forceinline__ void ring_pre(x3::lds_cptr base, x3::lds_cptr nbase, u32x4 (&f)[PF + 1][2],
                                           u32x4 (&fpre)[PF][2]) const {
    if constexpr (O + PF < ST) {
      f[(O + PF) % (PF + 1)][0] = x3::lds_rd<(O + PF) * 2048>(base);
      f[(O + PF) % (PF + 1)][1] = x3::lds_rd<(O + PF) * 2048 + 1024>(base);
    } else {
      fpre[O + PF - ST][0] = x3::lds_rd<(O + PF - ST) * 2048>(nbase);
      fpre[O + PF - ST][1] = x3::lds_rd<(O + PF - ST) * 2048 + 1024>(nbase);
    }
    // PF younger fragment pairs are in flight (an output-fragment read between them only makes it stricter)
    x3::lds_wait2<2 * PF>(f[O % (PF + 1)][0], f[O % (PF + 1)][1]);
  }
  // hidden layer 1: the o-step that activates operand pair P (< 4 NT) of the next k-step -- pair P at o-step P, or
  // (DMIP_X3K_ACT_SPREAD) the 4 NT pairs spread evenly over the 16 o-steps
  static constexpr int act_ostep(int P) {
#ifdef DMIP_X3K_ACT_SPREAD
    return (P * ST) / (4 * NT);
#else
    return P;
#endif
  }
  static constexpr int act_pair_at(int O) {
    for (int P = 0; P < 4 * NT; ++P)
      if (act_ostep(P) == O) return P;
    return -1;
  }
  // B(K + 1) at O = SYNC_O; the PPW LDS-DMA pieces of chunk K + 3 spread over o-steps SYNC_O + 1 .. 15 (SYNC_O = 8:
  // two at O = 9, then one per o-step)
  static constexpr int piece_ostep(int q) { return SYNC_O + 1 + (q * (15 - SYNC_O)) / PPW; }
  template <int K, int O, int Q = 0>
  __device__ __forceinline__ void ring_pieces() const {
    if constexpr (Q < PPW) {
      if constexpr (piece_ostep(Q) == O) issue_piece<(K + R - 1) % NCHUNK, (K + R - 1) % R, Q>();
      ring_pieces<K, O, Q + 1>();
    }
  }
  template <int K, int O>
  __device__ __forceinline__ void ring_post() const {
    if constexpr (O == SYNC_O) sync_mid<(K + 1) % NCHUNK>();
    if constexpr (!(DIAG & 1) && O > SYNC_O) ring_pieces<K, O>();
  }

  // ---- hidden layer 2 in two output halves (ring chunks 8..11: output tiles 0..7; 12..15: tiles 8..15), each
  // k-major with two k-steps per chunk: o-step O of chunk (H, Q2) is tile 8 H + O % 8 at k-step 2 Q2 + O / 8.
  // Half 0 activates the layer's input just in time (k-step k + 1 beside k-step k's eight o-steps) and keeps
  // every k-step's operands; half 1 reuses them and runs the output layer's first four k-steps (units 0..127,
  // half 0's finished tiles) beside its MFMAs, a pair of units per o-step. Each output element still
  // accumulates its k-steps in ascending order, and the output layer its k-steps too: bit-identical to the
  // one-pass layer. What stays outside the ring is the output layer's last four k-steps.
  __device__ __forceinline__ void layer2(const f32x4 (&In)[NT][ST], f32x4 (&Out)[NT][ST], const u32x4 (&Hh)[NT],
                                         const u32x4 (&Hl)[NT], u32x4 (&fpre)[PF][2], f32x4 (&oH)[NT],
                                         f32x4 (&oL)[NT]) const {
    u32x4 Ah[KQ][NT], Al[KQ][NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) Ah[0][t] = Hh[t], Al[0][t] = Hl[t];
#pragma unroll
    for (int o = 0; o < ST / 2; ++o) {
      const f32x4 b = bias4(2, o);
#pragma unroll
      for (int t = 0; t < NT; ++t) Out[t][o] = b;
    }
    u32x4 fo, eh, el;
    chunk2<0, 0>(In, Out, Ah, Al, fpre, oH, oL, fo, eh, el);
#pragma unroll
    for (int o = ST / 2; o < ST; ++o) {
      const f32x4 b = bias4(2, o);
#pragma unroll
      for (int t = 0; t < NT; ++t) Out[t][o] = b;
    }
    chunk2<1, 0>(In, Out, Ah, Al, fpre, oH, oL, fo, eh, el);
  }

  template <int H, int Q2>
  __device__ __forceinline__ void chunk2(const f32x4 (&In)[NT][ST], f32x4 (&Out)[NT][ST], u32x4 (&Ah)[KQ][NT],
                                         u32x4 (&Al)[KQ][NT], u32x4 (&fpre)[PF][2], f32x4 (&oH)[NT],
                                         f32x4 (&oL)[NT], u32x4& fo, u32x4& eh, u32x4& el) const {
    if constexpr (Q2 < KQ / 2) {
      constexpr int K = KQ + (KQ / 2) * H + Q2;
      const x3::lds_cptr base = (x3::lds_cptr)(ring_lane + (K % R) * CHUNK);
      const x3::lds_cptr nbase = (x3::lds_cptr)(ring_lane + ((K + 1) % R) * CHUNK);
      u32x4 f[PF + 1][2];
#pragma unroll
      for (int i = 0; i < PF; ++i) f[i][0] = fpre[i][0], f[i][1] = fpre[i][1];
      ostep2<H, Q2, 0>(base, nbase, In, Out, Ah, Al, f, fpre, oH, oL, fo, eh, el);
#pragma unroll
      for (int i = 0; i < PF; ++i) x3::lds_wait2<0>(fpre[i][0], fpre[i][1]);
      chunk2<H, Q2 + 1>(In, Out, Ah, Al, fpre, oH, oL, fo, eh, el);
    }
  }

  template <int H, int Q2, int O>
  __device__ __forceinline__ void ostep2(x3::lds_cptr base, x3::lds_cptr nbase, const f32x4 (&In)[NT][ST],
                                         f32x4 (&Out)[NT][ST], u32x4 (&Ah)[KQ][NT], u32x4 (&Al)[KQ][NT],
                                         u32x4 (&f)[PF + 1][2], u32x4 (&fpre)[PF][2], f32x4 (&oH)[NT], f32x4 (&oL)[NT],
                                         u32x4& fo, u32x4& eh, u32x4& el) const {
    if constexpr (O < ST) {
      constexpr int K = KQ + (KQ / 2) * H + Q2;
      constexpr int o = (ST / 2) * H + O % 8, k = 2 * Q2 + O / 8;
      ring_pre<O>(base, nbase, f, fpre);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        Out[t][o] = mfma16(f[O % (PF + 1)][0], Al[k][t], Out[t][o]);
        Out[t][o] = mfma16(f[O % (PF + 1)][1], Ah[k][t], Out[t][o]);
        Out[t][o] = mfma16(f[O % (PF + 1)][0], Ah[k][t], Out[t][o]);
      }
      if constexpr (H == 0 && k + 1 < KQ) {  // pairs O % 8 and 8 + O % 8 of k-step k + 1
        act_pair<k + 1, O % 8>(In, Ah, Al);
        act_pair<k + 1, 8 + O % 8>(In, Ah, Al);
      }
      if constexpr (H == 1 && Q2 == KQ / 2 - 1 && !NOISE) rng_slice<O>(rs_);
      if constexpr (H == 1) {  // output-layer pair G = 16 Q2 + O: unit (q, t) = (G / 4 / NT, G / 4 % NT), pair G % 4
        constexpr int G = 16 * Q2 + O, u = G / 4, d = G % 4, q = u / NT, t = u % NT;
        if constexpr (q < KQ / 2) {
          // the unit's output fragment, read at its first pair (after this o-step's ring reads) and waited
          // for at its last: the three later o-steps' ring reads (two each) are younger
          if constexpr (d == 0) fo = x3::lds_rd<q * 1024>((x3::lds_cptr)out_lane);
          const f32x4& z = Out[t][2 * q + d / 2];
          constexpr int e = 2 * (d % 2);
          uint32_t h, l;
          x3::split_pair(x3::x3_act_r(z[e]), x3::x3_act_r(z[e + 1]), h, l);
          eh[d] = h;
          el[d] = l;
          if constexpr (d == 3) {
            x3::lds_wait1<6>(fo);
            oH[t] = mfma16(fo, eh, oH[t]);
            oL[t] = mfma16(fo, el, oL[t]);
          }
        }
      }
      ring_post<K, O>();
      ostep2<H, Q2, O + 1>(base, nbase, In, Out, Ah, Al, f, fpre, oH, oL, fo, eh, el);
    }
  }

  // ---- the EM update's normals, drawn in hidden layer 2's last chunk (chunk (1, KQ/2 - 1) holds no output-layer
  // work for any NT): lane group t < NT draws chain tile t's D normals from its parked RNG state (the draws
  // rng_normals<D> makes, in the same order), parks the state again and leaves the normals in LDS for the EM
  // update, which every lane group reads. One Box-Muller pass serves all NT tiles.
  struct RngSlice {
    Rng r;
    uint32_t a, b;
    float u2, rad;
    float n[4];
  };
  mutable RngSlice rs_;
  // rng_normal_pair (dmip_device.h) cut into one dependent stage per o-step -- the same operations in the same
  // order, so the same bits -- so that each stage sits beside its o-step's MFMAs: O = 0 unpark, then per pair
  // P (base 1 + 4 P): the two xoshiro words, the uniforms and log2, the square root, cos / sin; O = 9 park
  template <int O>
  __device__ __forceinline__ void rng_slice(RngSlice& st) const {
    static_assert(D <= 4, "two normal pairs");
    const int tg = g < NT ? g : NT - 1;  // lane groups beyond the tiles repeat the last tile's draw, unstored
    const int j = threadIdx.x & 15;
    if constexpr (O == 0) {
      const uint32_t* d = rng_park + tg * 64;
      st.r = Rng{d[j], d[16 + j], d[32 + j], d[48 + j]};
    }
    constexpr int P = (O - 1) / 4, E = (O - 1) % 4;
    if constexpr (O >= 1 && P < (D + 1) / 2) {
      if constexpr (E == 0) {
        st.a = rng_next(st.r);
        st.b = rng_next(st.r);
      } else if constexpr (E == 1) {
        const float u1 = 1.0f - (float)(st.a >> 8) * 0x1p-24f;
        st.u2 = (float)(st.b >> 8) * 0x1p-24f;
        st.rad = -1.3862943611198906f * __log2f(u1);
      } else if constexpr (E == 2) {
        st.rad = __fsqrt_rn(st.rad);  // sqrt(-2 ln u1)
      } else {
        st.n[2 * P] = st.rad * __builtin_amdgcn_cosf(st.u2);
        st.n[2 * P + 1] = st.rad * __builtin_amdgcn_sinf(st.u2);
      }
    }
    if constexpr (O == 9) {
      if (g < NT) {
        uint32_t* d = rng_park + g * 64;
        d[j] = st.r.s0, d[16 + j] = st.r.s1, d[32 + j] = st.r.s2, d[48 + j] = st.r.s3;
        float* o = nrm + g * (D * 16);
#pragma unroll
        for (int k = 0; k < D; ++k) o[k * 16 + j] = st.n[k];
      }
    }
  }

  // activate operand pair P = (t, d) of k-step k (hidden layer 2's input) into Ah[k][t][d], Al[k][t][d]
  template <int k, int P>
  __device__ __forceinline__ void act_pair(const f32x4 (&In)[NT][ST], u32x4 (&Ah)[KQ][NT],
                                           u32x4 (&Al)[KQ][NT]) const {
    if constexpr (P < 4 * NT) {
      constexpr int t = P / 4, d = P % 4, e = 2 * (d % 2);
      const f32x4& z = In[t][2 * k + d / 2];
      uint32_t h, l;
      x3::split_pair(x3::x3_act_r(z[e]), x3::x3_act_r(z[e + 1]), h, l);
      Ah[k][t][d] = h;
      Al[k][t][d] = l;
    }
  }
};

// Layer 1's B operand of every chain tile, branch-free: input n takes k-slots 3n, 3n + 1, 3n + 2 as
// [v_hi, v_lo, v_hi] (x3::l1_operand's layout and bits: split_pair rounds as its casts do); lane group 0 holds
// k-slots 0-7, group 1 slots 8-15, groups 2-3 zero (3 (D + 1) <= 12 slots). x3::l1_operand selected the 16-bit
// slots per lane group through exec-mask branches; here whole dwords are masked in.
template <int D, int NT>
__device__ __forceinline__ void l1_operands(const float (&x)[NT][D], float tau, int g, u32x4 (&b)[NT]) {
  static_assert(D == 2 || D == 3, "x3k shapes");
  const uint32_t m0 = g == 0 ? 0xFFFFFFFFu : 0u, m1 = g == 1 ? 0xFFFFFFFFu : 0u;
  // (lo half of a, lo half of b) and (hi half of a, hi half of b)
  auto lo2 = [](uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x05040100u); };
  auto hi2 = [](uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x07060302u); };
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    uint32_t H01, L01, H23, L23;
    x3::split_pair(x[t][0], x[t][1], H01, L01);
    if constexpr (D == 3) x3::split_pair(x[t][2], tau, H23, L23);
    else x3::split_pair(tau, 0.0f, H23, L23);
    // slots of group 0: (hi0 lo0) (hi0 hi1) (lo1 hi1) (hi2 lo2); group 1: (hi2 hi3) (lo3 hi3) 0 0  [D = 3, "2" = x2,
    // "3" = tau]; D = 2: group 0 (hi0 lo0) (hi0 hi1) (lo1 hi1) (hiT loT), group 1 (hiT 0) 0 0 0
    const uint32_t g0[4] = {lo2(H01, L01), H01, hi2(L01, H01), lo2(H23, L23)};
    uint32_t g1[4];
    if constexpr (D == 3) g1[0] = H23, g1[1] = hi2(L23, H23), g1[2] = 0u, g1[3] = 0u;
    else g1[0] = H23, g1[1] = 0u, g1[2] = 0u, g1[3] = 0u;
#pragma unroll
    for (int d = 0; d < 4; ++d) b[t][d] = (g0[d] & m0) | (g1[d] & m1);
  }
}

// layer 1's tile O: its A fragment (lanes 32-63 read lanes 0-31's, KLay::L1) and bias row (per-y c (b1 + W1_y y))
template <int O>
__device__ __forceinline__ void l1_read(x3::lds_cptr la, x3::lds_cptr lb, u32x4& a, u32x4& b) {
  a = x3::lds_rd<O * 512>(la);
  b = x3::lds_rd<O * 64>(lb);
}

// tile O of layer 1 for every chain tile (fragments of tiles O, O + 1 in flight on entry; O + 2's issued here)
template <int O, int NT, int ST>
__device__ __forceinline__ void l1_tile(x3::lds_cptr la, x3::lds_cptr lb, u32x4 (&fa)[3], u32x4 (&fb)[3],
                                        const u32x4 (&b1)[NT], f32x4 (&P)[NT][ST]) {
  if constexpr (O < ST) {
    if constexpr (O + 2 < ST) l1_read<O + 2>(la, lb, fa[(O + 2) % 3], fb[(O + 2) % 3]);
    // the pairs of tiles O + 1 and O + 2 are younger than O's
    x3::lds_wait2<(O + 2 < ST) ? 4 : ((O + 1 < ST) ? 2 : 0)>(fa[O % 3], fb[O % 3]);
    const f32x4 c = __builtin_bit_cast(f32x4, fb[O % 3]);
#pragma unroll
    for (int t = 0; t < NT; ++t) P[t][O] = mfma16(fa[O % 3], b1[t], c);
    l1_tile<O + 1>(la, lb, fa, fb, b1, P);
  }
}

// ---------------------------------------------------------------------------- sampler kernel
// The reverse-SDE loop (models/diffusion.py:27-46) for the CDE, a = net(x, y, tau) with y folded into the
// per-y layer-1 bias; mu = g a + 0.5 beta x, x <- x + delta mu + sqrt(delta) g xi (dmip_device.h
// em_update). Work: the balanced WaveSchedule over jobs of NT 16-chain tiles.
template <int D, int NT, bool NOISE, int DIAG = 0>
__global__ void __launch_bounds__(KWaves<NT>::NWV * 64, KWaves<NT>::NWV / 4) x3k_sampler_kernel(X3SamplerParams p) {
  constexpr int NWV = KWaves<NT>::NWV, PPW = KWaves<NT>::PPW;
  using L = KLay;
  static_assert(D <= 4, "output rows of a chain sit in lane group 0 (D <= 4)");
  __shared__ __attribute__((aligned(16))) char lds[L::TOTAL];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, j = lane & 15;
  const int yi = blockIdx.y;

  KEngine<D, NT, NOISE, DIAG> eng;
  eng.lds = lds;
  eng.ring_lane = lds + L::RING + lane * 16;
  eng.out_lane = lds + L::OUT + lane * 16;
  eng.rs = __builtin_amdgcn_make_buffer_rsrc((void*)p.net[0].kstream, 0, NCHUNK * CHUNK, 0x00020000);
  eng.voff = (unsigned)(w * PPW * 1024 + lane * 16);
  eng.w = w;
  eng.g = g;
  eng.rng_park = (uint32_t*)(lds + L::RNGP) + w * NT * 64;
  eng.nrm = (float*)(lds + L::NRM) + w * NT * D * 16;
  {
    const uint4* s1 = (const uint4*)p.net[0].l1;  // [16 tiles][64 lanes] -> lanes 0-31 of each tile
    uint4* d1 = (uint4*)(lds + L::L1);
    for (int e = threadIdx.x; e < L::L1_BYTES / 16; e += NWV * 64) d1[e] = s1[(e >> 5) * 64 + (e & 31)];
    const uint4* so = (const uint4*)p.net[0].kout;
    uint4* dout = (uint4*)(lds + L::OUT);
    for (int e = threadIdx.x; e < L::OUT_BYTES / 16; e += NWV * 64) dout[e] = so[e];
    float* bl = (float*)(lds + L::BIAS);
    for (int i = threadIdx.x; i < L::BF; i += NWV * 64) bl[i] = i < W ? p.bias_y[(size_t)yi * W + i] : p.net[0].bias[i];
    __syncthreads();
  }
  u32x4 fpre[PF][2];  // the first fragment pairs of the next ring chunk (read ahead across phases)
  eng.start(fpre);
  const char* l1_lane = lds + L::L1 + (lane & 31) * 16;  // lanes 32-63: zero k-slots of B (KLay::L1)
  const char* out_lane = lds + L::OUT + lane * 16;

  const int S = p.num_steps;
  constexpr int JC = 16 * NT;  // chains per job
  const long long jobs_y = (p.n_chains + JC - 1) / JC;
  const long long n_waves = (long long)gridDim.x * NWV;
  const long long gw = (long long)blockIdx.x * NWV + w;
  constexpr int XT = sampler_xfer_words(D);  // hand-over words per tile
  const WaveSchedule sched(jobs_y, S, n_waves, gw);
  const size_t noise_step = (size_t)gridDim.y * p.n_chains * D;

  uint64_t ph[6] = {0, 0, 0, 0, 0, 0};  // DIAG & 2: cycles per phase (L1, H1, H2, output, EM, barrier waits)
  // a chain state out of the split's range (x3::report_range), checked on each segment's final state: an
  // input beyond fp16's range splits into inf / NaN halves, whose NaN the network carries to every later
  // step (a per-step check held registers in the step loop and pushed a chain's RNG word to scratch)
  bool oor = false;
  for (int sgi = 0; sgi < sched.n_seg; ++sgi) {
    const Seg sg = sched.segment(sgi);
    long long c_loc[NT];
    bool valid[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      c_loc[t] = (long long)(sg.job >= 0 ? sg.job : 0) * JC + 16 * t + j;
      valid[t] = sg.job >= 0 && c_loc[t] < p.n_chains;
    }
    float x[NT][D];
    // wave-private LDS slots of the tiles' RNG states: lane group 0 writes at a segment's start, lane group t
    // draws tile t's normals in hidden layer 2 (KEngine::rng_slice), every lane reads its chain's words
    uint32_t* rng_park = eng.rng_park;
    static_assert(KWaves<NT>::NWV * NT * 256 <= KLay::RNGP_BYTES, "RNG parking space");
    static_assert(KWaves<NT>::NWV * NT * 3 * 64 <= KLay::NRM_BYTES, "normals space");
    auto park = [&](int t, const Rng& r) {
      if (g == 0) {
        uint32_t* d = rng_park + t * 64;
        d[j] = r.s0, d[16 + j] = r.s1, d[32 + j] = r.s2, d[48 + j] = r.s3;
      }
    };
    auto unpark = [&](int t) {
      const uint32_t* d = rng_park + t * 64;
      return Rng{d[j], d[16 + j], d[32 + j], d[48 + j]};
    };
    if (sg.kind == 2) {  // resume the job the previous wave of the grid handed over
      const size_t slot = (size_t)yi * n_waves + gw - 1;
      const bool lost = handover_wait(p.xflag + slot, p.spin_limit, p.err, kErrHandover, lane);
      // compact slot: one copy per chain (lane group 0 stored it), [tile][word][16 chains]
      const float* src = p.xfer + slot * (size_t)(NT * XT);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const float* st = src + t * (D + 4) * 16;
#pragma unroll
        for (int k = 0; k < D; ++k) x[t][k] = lost ? __builtin_nanf("") : st[k * 16 + j];
        park(t, Rng{__float_as_uint(st[(D + 0) * 16 + j]), __float_as_uint(st[(D + 1) * 16 + j]),
                    __float_as_uint(st[(D + 2) * 16 + j]), __float_as_uint(st[(D + 3) * 16 + j])});
      }
    } else {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        Rng rng = rng_init(p.seed, (uint64_t)(p.chain_offset + c_loc[t]), (uint64_t)yi);
        float n0[D];
        if constexpr (NOISE) {
          const float* src = p.noise + ((size_t)yi * p.n_chains + (valid[t] ? c_loc[t] : 0)) * D;
#pragma unroll
          for (int k = 0; k < D; ++k) n0[k] = src[k];
        } else {
          rng_normals<D>(rng, n0);
        }
        park(t, rng);
#pragma unroll
        for (int k = 0; k < D; ++k) x[t][k] = __fadd_rn(__fmul_rn(n0[k], p.stdv), p.mean);
      }
    }

    int snap_next = p.snap_every > 0 ? (sg.s0 / p.snap_every + 1) * p.snap_every : -1;
    for (int i0 = sg.s0; i0 < sg.s1; ++i0) {
      const int i = sg.kind == 3 ? 0 : i0;  // idle steps: a dummy job at step 0, discarded
      const float4 c4 = ((const float4*)p.coef)[i];  // step_coef(i, ...) of this launch (x3k_coef_kernel)
      const StepCoef cf{c4.x, c4.y, c4.z};
      uint64_t t0 = 0;
      if constexpr (DIAG & 2) t0 = stamp();

      // ---- layer 1 (resident image, one MFMA per tile and chain tile), pre-activations in P
      f32x4 P[NT][ST];
      {
        u32x4 b1[NT];
        l1_operands(x, cf.tau, g, b1);
        // the A fragments and the per-y bias rows (the MFMAs' C input) by explicit reads two tiles ahead with
        // counted waits: left to itself the compiler waited lgkmcnt(0) before every tile's MFMAs and routed the
        // bias through AGPRs (then copied P back out of them, each copy behind the MFMA's full latency)
        const x3::lds_cptr la = (x3::lds_cptr)l1_lane;
        const x3::lds_cptr lb = (x3::lds_cptr)(lds + L::BIAS + 16 * g);
        u32x4 fa[3], fb[3];
        l1_read<0>(la, lb, fa[0], fb[0]);
        l1_read<1>(la, lb, fa[1], fb[1]);
        l1_tile<0>(la, lb, fa, fb, b1, P);
      }
      u32x4 Hh[NT], Hl[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) act_kstep<true>(P[t][0], P[t][1], Hh[t], Hl[t]);
      // ---- hidden layers 1 and 2 (ring chunks 0..7, 8..15)
      f32x4 Q[NT][ST];
      uint64_t t1 = 0;
      if constexpr (DIAG & 2) t1 = stamp(), ph[0] += t1 - t0;
      eng.template layer<1, true>(P, Q, Hh, Hl, fpre);
      uint64_t t2 = 0;
      if constexpr (DIAG & 2) t2 = stamp(), ph[1] += t2 - t1;
#pragma unroll
      for (int t = 0; t < NT; ++t) act_kstep<false>(Q[t][0], Q[t][1], Hh[t], Hl[t]);
      // ---- hidden layer 2 (ring chunks 8..15, two output halves) with the output layer's first half
      // (resident output fragments: rows 0..D-1 W_hi, 4..4+D-1 W_lo)
      f32x4 P2[NT][ST];
      f32x4 oH[NT], oL[NT];
      {
        const f32x4 bo = g == 0 ? eng.bias4(NH + 1, 0) : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int t = 0; t < NT; ++t) oH[t] = bo, oL[t] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      }
      eng.layer2(Q, P2, Hh, Hl, fpre, oH, oL);
      uint64_t t3 = 0;
      if constexpr (DIAG & 2) t3 = stamp(), ph[2] += t3 - t2;
      // ---- the output layer's second half (units 128..255)
      {
#pragma unroll
        for (int q = KQ / 2; q < KQ; ++q) {
          const u32x4 fo = *(const u32x4*)(out_lane + q * 1024);
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            u32x4 eh, el;
            act_kstep<false>(P2[t][2 * q], P2[t][2 * q + 1], eh, el);
            oH[t] = mfma16(fo, eh, oH[t]);
            oL[t] = mfma16(fo, el, oL[t]);
          }
        }
      }
      uint64_t t4 = 0;
      if constexpr (DIAG & 2) t4 = stamp(), ph[3] += t4 - t3;
      // ---- a(x) on every lane of chain j, the EM update
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        float a[D];
#pragma unroll
        for (int k = 0; k < D; ++k) {
          // lane group 0 holds W_hi h_hi (oH) and W_hi h_lo (oL) of row k, group 1 W_lo h_hi (oH): permlane16_swap
          // brings groups 0 and 1 together in both (groups 2-3 likewise, zero rows), permlane32_swap copies
          // lanes 0-31's sum to lanes 32-63 -- the order (hi.h_hi + hi.h_lo) + lo.h_hi of the earlier shuffles
          const auto sh = __builtin_amdgcn_permlane16_swap(__float_as_uint(oH[t][k]), __float_as_uint(oH[t][k]),
                                                           false, false);
          const auto sl = __builtin_amdgcn_permlane16_swap(__float_as_uint(oL[t][k]), __float_as_uint(oL[t][k]),
                                                           false, false);
          const float v = (__uint_as_float(sh[0]) + __uint_as_float(sl[0])) + __uint_as_float(sh[1]);
          a[k] = __uint_as_float(__builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                                  false)[0]);
        }
        float xi[D];
        if constexpr (NOISE) {
          const float* src = p.noise + noise_step * (i + 1) + ((size_t)yi * p.n_chains + (valid[t] ? c_loc[t] : 0)) * D;
#pragma unroll
          for (int k = 0; k < D; ++k) xi[k] = src[k];
        } else {  // drawn in hidden layer 2 (KEngine::rng_slice)
#pragma unroll
          for (int k = 0; k < D; ++k) xi[k] = eng.nrm[(t * D + k) * 16 + j];
        }
#pragma unroll
        for (int k = 0; k < D; ++k) x[t][k] = em_update(x[t][k], a[k], xi[k], cf, p.delta, p.sqrt_delta);
      }
      if constexpr (DIAG & 2) {
        ph[4] += stamp() - t4;
        continue;  // snap_out holds the stamps
      }
      if (i0 + 1 == snap_next) {
        snap_next += p.snap_every;
        if (sg.kind != 3 && g == 0) {
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            if (!valid[t]) continue;
            float* dst = p.snap_out +
                         (((size_t)((i0 + 1) / p.snap_every - 1) * gridDim.y + yi) * p.n_chains + c_loc[t]) * D;
#pragma unroll
            for (int k = 0; k < D; ++k) dst[k] = x[t][k];
          }
        }
      }
    }
    // only chains whose results are returned: an idle segment's dummy tile and padded lanes may diverge freely
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int k = 0; k < D; ++k) oor |= sg.kind != 3 && valid[t] && !(__builtin_fabsf(x[t][k]) <= 65504.0f);  // NaN included
    if (sg.kind == 1) {  // hand the job over to the next wave of the grid
      const size_t slot = (size_t)yi * n_waves + gw;
      float* dst = p.xfer + slot * (size_t)(NT * XT);
      if (g == 0) {  // the four lane groups hold identical copies of a chain's state: store one
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          float* st = dst + t * (D + 4) * 16;
#pragma unroll
          for (int k = 0; k < D; ++k) st[k * 16 + j] = x[t][k];
          const Rng rng = unpark(t);
          st[(D + 0) * 16 + j] = __uint_as_float(rng.s0);
          st[(D + 1) * 16 + j] = __uint_as_float(rng.s1);
          st[(D + 2) * 16 + j] = __uint_as_float(rng.s2);
          st[(D + 3) * 16 + j] = __uint_as_float(rng.s3);
        }
      }
      handover_publish(p.xflag + slot, lane, p.debug_flags);
    } else if (sg.kind != 3 && g == 0) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if (!valid[t]) continue;
        float* dst = p.x_out + ((size_t)yi * p.n_chains + c_loc[t]) * D;
#pragma unroll
        for (int k = 0; k < D; ++k) dst[k] = x[t][k];
      }
    }
  }
  wait_vmcnt<0>();  // the prefetched chunks of a step that never ran land before the workgroup exits
  x3::report_range(oor, p.err, lane);
  if constexpr (DIAG & 2) {
    if (lane == 0) {
      uint64_t* dst = (uint64_t*)p.snap_out + ((size_t)yi * n_waves + gw) * 8;
#pragma unroll
      for (int k = 0; k < 5; ++k) dst[k] = ph[k];
      dst[5] = (uint64_t)sched.C;
      dst[6] = eng.ph_vm;
      dst[7] = eng.ph_bar;
    }
  }
}

}  // namespace x3k

// the launch's step coefficients: coef[i] = step_coef(i) (the kernel loads them instead of recomputing a division
// and an f64 square root at every step; the same device function, so the same bits)
template <int DUMMY = 0>
__global__ void x3k_coef_kernel(float4* coef, int S, float T, float bmin, float bdiff) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < S) {
    const StepCoef c = step_coef(i, S, T, bmin, bdiff);
    coef[i] = make_float4(c.tau, c.beta, c.g, 0.0f);
  }
}

template <int D, int NT, bool NOISE, int DIAG = 0>
inline hipError_t launch_x3k_sampler_t(const X3SamplerParams& p, int n_y, hipStream_t st) {
  constexpr int NWV = x3k::KWaves<NT>::NWV;
  auto kern = x3k::x3k_sampler_kernel<D, NT, NOISE, DIAG>;
  const long long jobs = (p.n_chains + 16 * NT - 1) / (16 * NT);
  long long g = resident_slots(kern, NWV * 64, st) / (n_y > 0 ? n_y : 1);
  const long long cap = (jobs + NWV - 1) / NWV;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  X3SamplerParams q = p;
  char* buf = nullptr;
  // hand-over slots of NT tiles: (NT (D + 4) - 4 + 4) 64 words each
  hipError_t e = alloc_handover((size_t)g * n_y * NWV, NT * (D + 4) - 4, st, &buf, &q.xfer, &q.xflag);
  if (e != hipSuccess) return e;
  const int S = p.num_steps > 0 ? p.num_steps : 1;
  float4* coef = nullptr;
  if ((e = hipMallocAsync((void**)&coef, (size_t)S * sizeof(float4), st)) != hipSuccess) {
    (void)hipFreeAsync(buf, st);
    return e;
  }
  hipLaunchKernelGGL(x3k_coef_kernel<0>, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, st, coef, S, p.T, p.bmin,
                     p.bdiff);
  q.coef = (const float*)coef;
  hipLaunchKernelGGL(kern, dim3((unsigned)g, (unsigned)n_y), dim3(NWV * 64), 0, st, q);
  e = hipGetLastError();
  (void)hipFreeAsync(coef, st);
  (void)hipFreeAsync(buf, st);
  return e;
}

}  // namespace dmip
