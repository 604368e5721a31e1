// fp32-accurate score networks at the fp16 matrix rate: the DMIP_PREC_F32X3 reverse-SDE samplers.
//
// The reference computes its score network in fp32 (nets.py:32-35, models/diffusion.py:38-42). Every
// product here is formed as a three-term fp16 split on v_mfma_f32_16x16x32_f16 (fp32 accumulation):
//     W h  ~  W_hi h_hi + W_hi h_lo + W_lo h_hi,   v_hi = fp16(v), v_lo = fp16(v - v_hi)
// The dropped W_lo h_lo is <= 2^-24 |W h|, and the lo parts are held to ~2^-24 absolute (fp16 subnormals
// are honoured by the f16 MFMAs on gfx950): measured on the device, the split product's error is
// 2^-23.2 of sum |w h| against 2^-23.0 for an f32 fmaf chain (profiles/r3_mfma_f16_check.txt,
// scripts/ubench/mfma_f16_check.hip). Three fp16 MFMAs cost 3/16 of one f32 MFMA of the same work:
// this engine runs the reference's fp32 arithmetic at ~5x the exact-f32 engine's (dmip_f32.h) rate.
//
// Layout (one wave = 16 chains, v_mfma_f32_16x16x32_f16):
//   * a layer's output tile is 16 units x 16 chains: lane (g = l >> 4, j = l & 15) holds units
//     16 o + 4 g + r (r = 0..3) of chain j. Two consecutive tiles 2q, 2q + 1 are the B operand of
//     k-step q of the next layer with no lane movement: lane (g, j) supplies k-slots 8 g + m, which
//     the host maps to unit kperm16(q, g, m) = 32 q + 16 (m >> 2) + 4 g + (m & 3) of the weight image.
//   * activations stay in registers as (hi, lo) fp16 pairs: W/32 B fragments each (W = 256: 64 VGPRs
//     for a layer's input, 64 for its output), so a 512-thread workgroup keeps 2 waves per SIMD.
//   * weight images (dmip_capi.cpp pack_x3_net): output tile o, k-step q, part p (hi / lo), lane
//     l = i + 16 g holds A[16 o + i][kperm16(q, g, 0..7)] -- one ds_read_b128 per lane per fragment;
//     a tile is W/16 KiB (both parts). The W x W layers and the output layer stream from L2 through
//     an R-slot LDS ring by LDS-DMA (the protocol of dmip_f32.h), CHUNK = CT tiles (<= 32 KiB);
//     layer 1 and the biases are LDS-resident.
//   * layer 1 (x, tau -- or every input for CDiffE -- plus its bias in the accumulator init): input n
//     takes k-slots 3n, 3n+1, 3n+2 with B = [v_hi, v_lo, v_hi] against A = [W_hi, W_hi, W_lo].
//   * activations in r-form, r = 1 / (1 + 2^zs) = (1 - tanh z) / 2 (zs = 2 log2(e) z, the scale folded
//     into the weights); "1 - 2r" is folded into the next layer's weights (-2 W) and bias (b + sum W).
//     Layer 1's double tanh (nets.py:21-26) is r1 = act_r(zs), r2 = act_r(c (1 - 2 r1)) -- exp2 + rcp
//     at ~1 ulp each, no polynomial (the 16-bit engine's degree-4 fit is 1.7e-5 off).
// The chain state, schedule, RNG, EM update, snapshots, hand-over and predictor-corrector are those of
// the other two engines (dmip_device.h): all three precisions draw identical noise chain by chain.
#pragma once
#include "dmip_device.h"
#include "dmip_internal.h"

namespace dmip {
namespace x3 {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma16(const u32x4& a, const u32x4& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                0);
}

template <int W>
struct Shape {
  static constexpr int ST = W / 16;                        // 16-row output tiles per layer
  static constexpr int KQ = W / 32;                        // 32-deep k-steps over a W-wide input
  static constexpr int TILE = KQ * 2048;                   // one output tile: hi + lo fragments per k-step
  static constexpr int CT0 = 32768 / TILE;
  static constexpr int CT = CT0 < 1 ? 1 : (CT0 > ST ? ST : CT0);  // tiles per ring chunk
  static constexpr int CHUNK = CT * TILE;
  static constexpr int NCH = ST / CT;                      // chunks per W x W layer
  static constexpr int NW = W == 512 ? 4 : 8;              // W = 512: one wave per SIMD (2 x 128 VGPR activations)
  static constexpr int PPW = CHUNK / 1024 / NW;            // LDS-DMA pieces per wave per chunk
  static_assert(ST % CT == 0 && PPW >= 1 && CHUNK % (1024 * NW) == 0, "ring geometry");
};

constexpr int kLdsBudget = 160 * 1024;
// A/B knob (scripts/build_variant.sh): the round-5 per-piece scalar offsets and LDS addresses
#ifndef DMIP_X3_NO_IMM
#define DMIP_X3_NO_IMM 0
#endif
constexpr bool X3_NO_IMM = DMIP_X3_NO_IMM;
constexpr int kMaxHidden = 3;
constexpr int k1q_of(int nv) { return (3 * nv + 31) / 32; }
constexpr int align16(int v) { return (v + 15) / 16 * 16; }

// LDS: layer-1 images, biases (per network: layer 1 | hidden layers | output rows 0..15), the
// observation (CDiffE), the ring. L1R: layer 1 is not resident but streams through the ring ahead of the
// hidden chunks (CDiffE at width 512: its 27-input split image is 96 KiB).
// L1H: a one-k-step layer 1 over at most 5 inputs (15 k-slots) leaves lane groups 2-3 of its B operand zero, so its
// resident image holds lanes 0-31 of each tile (512 B) and lanes 32-63 read those finite weights (dmip_x3k.h KLay):
// half the LDS, which gives the Posterior at W = 512 (two layer-1 images) a third ring slot
template <int W, int NNET, int K1Q, int M, bool L1R = false, bool L1H = false>
struct XLay {
  using S = Shape<W>;
  static constexpr int L1_BYTES = L1R ? 0 : (L1H ? S::ST * 512 : S::ST * K1Q * 1024);
  static constexpr int BF = kMaxHidden * W + 16;  // bias floats per network
  static constexpr int L1 = 0;
  static constexpr int BIAS = L1 + NNET * L1_BYTES;
  static constexpr int BIAS_BYTES = align16(BF * 4);
  static constexpr int YOBS = BIAS + NNET * BIAS_BYTES;
  static constexpr int RING = align16(YOBS + (M > 0 ? M : 1) * 4);
  static constexpr int R0 = (kLdsBudget - RING) / S::CHUNK;
  static constexpr int R = R0 > 4 ? 4 : R0;
  static constexpr int TOTAL = RING + R * S::CHUNK;
  static_assert(R >= 2, "LDS budget: fewer than two ring slots");
};

// split a pair of f32 values into an (hi, lo) pair of packed fp16 dwords: v = hi + lo to ~2^-22 |v|.
// lo = fp16(v - hi) in one instruction per half: v_fma_mix{lo,hi}_f16 takes hi as an fp16 operand,
// forms v - hi exactly and rounds once (3 instructions per pair instead of cvt, 2 cvt back, 2 sub, cvt;
// bit-identical, scripts/ubench/fma_mix_check.hip)
__device__ __forceinline__ void split_pair(float a, float b, uint32_t& hi, uint32_t& lo) {
  hi = cvt_pk_f16(a, b);
  asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(lo) : "v"(hi), "v"(a));
  asm("v_fma_mixhi_f16 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(lo) : "v"(hi), "v"(b));
}

// A-fragment reads of the MFMA chains: explicit ds_read_b128 kept PF k-steps ahead with counted
// lgkmcnt waits (left to itself the compiler reads each fragment right before its MFMA behind an
// lgkmcnt(0)). A wait names the fragments it guards ("+v"), so their MFMAs cannot move above it;
// LDS returns in order, so younger LDS operations only make a counted wait stricter.
typedef __attribute__((address_space(3))) const char* lds_cptr;

template <int OFF>
__device__ __forceinline__ u32x4 lds_rd(lds_cptr p) {
  u32x4 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(p), "i"(OFF));
  return r;
}

template <int N>
__device__ __forceinline__ void lds_wait2(u32x4& a, u32x4& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "i"(N));
}

template <int N>
__device__ __forceinline__ void lds_wait1(u32x4& a) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(a) : "i"(N));
}

// compiler-visible lgkmcnt(0): the compiler's own LDS reads (biases) are known complete after it
__device__ __forceinline__ void lgkm_drain() { __builtin_amdgcn_s_waitcnt(0xC07F); }

constexpr int cmin(int a, int b) { return a < b ? a : b; }

// acc[u / KQ] += W_hi h_hi + W_hi h_lo + W_lo h_hi over the NU = n_tiles KQ k-steps of a chunk: k-step u
// has its hi / lo fragments at (2u, 2u + 1) KiB from `base` (per-lane address); PF k-steps prefetched
template <int KQ, int NU, int PF, int U = 0>
__device__ __forceinline__ void split_chain(lds_cptr base, const u32x4 (&Hh)[KQ], const u32x4 (&Hl)[KQ],
                                            f32x4 (&acc)[(NU + KQ - 1) / KQ], u32x4 (&fa)[PF + 1][2]) {
  if constexpr (U < NU) {
    if constexpr (U + PF < NU) {
      fa[(U + PF) % (PF + 1)][0] = lds_rd<(2 * (U + PF)) * 1024>(base);
      fa[(U + PF) % (PF + 1)][1] = lds_rd<(2 * (U + PF) + 1) * 1024>(base);
    }
    lds_wait2<2 * cmin(NU - 1 - U, PF)>(fa[U % (PF + 1)][0], fa[U % (PF + 1)][1]);
    constexpr int t = U / KQ, q = U % KQ;
    acc[t] = mfma16(fa[U % (PF + 1)][0], Hl[q], acc[t]);
    acc[t] = mfma16(fa[U % (PF + 1)][1], Hh[q], acc[t]);
    acc[t] = mfma16(fa[U % (PF + 1)][0], Hh[q], acc[t]);
    split_chain<KQ, NU, PF, U + 1>(base, Hh, Hl, acc, fa);
  }
}

// split_chain with a hook run beside k-step U's MFMAs (hook.template at<U>(): the ring's LDS-DMA pieces, spread)
template <int KQ, int NU, int PF, typename Hook, int U = 0>
__device__ __forceinline__ void split_chain_h(lds_cptr base, const u32x4 (&Hh)[KQ], const u32x4 (&Hl)[KQ],
                                              f32x4 (&acc)[(NU + KQ - 1) / KQ], u32x4 (&fa)[PF + 1][2],
                                              const Hook& hook) {
  if constexpr (U < NU) {
    if constexpr (U + PF < NU) {
      fa[(U + PF) % (PF + 1)][0] = lds_rd<(2 * (U + PF)) * 1024>(base);
      fa[(U + PF) % (PF + 1)][1] = lds_rd<(2 * (U + PF) + 1) * 1024>(base);
    }
    lds_wait2<2 * cmin(NU - 1 - U, PF)>(fa[U % (PF + 1)][0], fa[U % (PF + 1)][1]);
    constexpr int t = U / KQ, q = U % KQ;
    acc[t] = mfma16(fa[U % (PF + 1)][0], Hl[q], acc[t]);
    acc[t] = mfma16(fa[U % (PF + 1)][1], Hh[q], acc[t]);
    acc[t] = mfma16(fa[U % (PF + 1)][0], Hh[q], acc[t]);
    hook.template at<U, NU>();
    split_chain_h<KQ, NU, PF, Hook, U + 1>(base, Hh, Hl, acc, fa, hook);
  }
}

template <int KQ, int NU, int PF, typename Hook>
__device__ __forceinline__ void split_product_h(lds_cptr base, const u32x4 (&Hh)[KQ], const u32x4 (&Hl)[KQ],
                                                f32x4 (&acc)[(NU + KQ - 1) / KQ], const Hook& hook) {
  u32x4 fa[PF + 1][2];
#pragma unroll
  for (int u = 0; u < cmin(PF, NU); ++u) {
    if (u == 0) fa[0][0] = lds_rd<0>(base), fa[0][1] = lds_rd<1024>(base);
    if (u == 1) fa[1][0] = lds_rd<2048>(base), fa[1][1] = lds_rd<3072>(base);
    if (u == 2) fa[2][0] = lds_rd<4096>(base), fa[2][1] = lds_rd<5120>(base);
  }
  split_chain_h<KQ, NU, PF, Hook>(base, Hh, Hl, acc, fa, hook);
}

template <int KQ, int NU, int PF>
__device__ __forceinline__ void split_product(lds_cptr base, const u32x4 (&Hh)[KQ], const u32x4 (&Hl)[KQ],
                                              f32x4 (&acc)[(NU + KQ - 1) / KQ]) {
  u32x4 fa[PF + 1][2];
#pragma unroll
  for (int u = 0; u < cmin(PF, NU); ++u) {
    // (unrolled: u is a constant) the first PF k-steps' fragments
    if (u == 0) fa[0][0] = lds_rd<0>(base), fa[0][1] = lds_rd<1024>(base);
    if (u == 1) fa[1][0] = lds_rd<2048>(base), fa[1][1] = lds_rd<3072>(base);
    if (u == 2) fa[2][0] = lds_rd<4096>(base), fa[2][1] = lds_rd<5120>(base);
  }
  static_assert(PF >= 1 && PF <= 3, "prefetch depth");
  split_chain<KQ, NU, PF>(base, Hh, Hl, acc, fa);
}

// layer 1: one fragment per k-step (the split lives in the k-slots), NU = n_tiles K1Q k-steps in tile order
// STR: bytes between consecutive fragments (1024; 512 for a half-size image holding lanes 0-31 only, XLay L1H)
template <int K1Q, int NU, int PF, int F = 0, int STR = 1024>
__device__ __forceinline__ void l1_chain(lds_cptr base, const u32x4 (&b1)[K1Q], f32x4 (&acc)[NU / K1Q],
                                         u32x4 (&fa)[PF + 1]) {
  if constexpr (F < NU) {
    if constexpr (F + PF < NU) fa[(F + PF) % (PF + 1)] = lds_rd<(F + PF) * STR>(base);
    lds_wait1<cmin(NU - 1 - F, PF)>(fa[F % (PF + 1)]);
    acc[F / K1Q] = mfma16(fa[F % (PF + 1)], b1[F % K1Q], acc[F / K1Q]);
    l1_chain<K1Q, NU, PF, F + 1, STR>(base, b1, acc, fa);
  }
}

// r-form activation r = 1 / (1 + 2^zs) (v_exp_f32 + v_rcp_f32, ~1 ulp each)
__device__ __forceinline__ float x3_act_r(float zs) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(zs));
}

// layer 1's tanh(tanh(z)) in r-form: r1 = (1 - tanh z)/2, then r2 = (1 - tanh(tanh z))/2 with
// tanh z = 1 - 2 r1 (both tanh arguments pre-scaled by c = 2 log2(e))
__device__ __forceinline__ float x3_act_r2(float zs) {
  const float r1 = x3_act_r(zs);
  return x3_act_r(__builtin_fmaf(-2.0f * kTanhScale, r1, kTanhScale));
}

// The network engine: NNET networks of nl layers (runtime, 1..3) of width W share one weight ring;
// each evaluation streams (nl - 1) NCH hidden chunks then one output chunk, in the host image's order.
// DIAG (timing ablations only, never on the product path; DMIP_X3_DIAG): bit 0 = no ring (no DMA, no
// barrier: stale weights), bit 1 = hidden activations replaced by the split alone, bit 2 = the same for
// layer 1's double tanh, bit 3 = no ring barrier (DMA and vmcnt waits kept), bit 4 = no LDS-DMA pieces (barrier kept),
// bit 5 = no vmcnt wait for the ring (pieces and barrier kept: the weights may be read before they land)
template <int W, int NNET, int K1Q, int R, int RING_OFF, int DIAG = 0, bool L1R = false, bool L1H = false>
struct XEngine {
  using S = Shape<W>;
  static constexpr int ST = S::ST, KQ = S::KQ, CT = S::CT, NCH = S::NCH, NW = S::NW, PPW = S::PPW;
  static constexpr int CHUNK = S::CHUNK, TILE = S::TILE;

  char* lds;
  const char* img[2];
  int l1_off[2];
  int bias_off[2];
  int nl;       // hidden layers (layer 1 + nl - 1 W x W layers)
  int ncn;      // chunks per network evaluation
  int c_issue;  // next chunk to issue, in [0, NNET ncn)
  int s_issue;  // its ring slot
  int s_read;   // ring slot of the next chunk to consume
  int w, lane, g;

  // chunks of layer 1 in the stream (L1R): k-step q of every output tile, ST KiB
  static constexpr int NL1C = L1R ? K1Q : 0;
  // resident weights: at W = 64 one network's whole stream (at most kMaxHidden 16 KiB chunks: the W x W layers and
  // the output tile) fits the ring, so it is loaded once per launch and every chunk_sync is a plain slot address --
  // no barrier, no LDS-DMA, no vmcnt wait per chunk (the linear problem's networks, BASELINE configs[0])
  static constexpr bool RES = W == 64 && NNET == 1 && !L1R && R >= kMaxHidden && (DIAG & 1) == 0;
  static_assert(!L1R || ST * 1024 == CHUNK, "a streamed layer-1 chunk is one k-step of all output tiles");

  __device__ __forceinline__ void init(int n_hidden) {
    nl = n_hidden;
    ncn = NL1C + (nl - 1) * NCH + 1;
    c_issue = s_issue = s_read = 0;
    voff = (unsigned)(w * PPW * 1024 + lane * 16);
  }

  // the refill of the next chunk to issue: its source and ring slot (then the stream position advances); its PPW
  // pieces per wave go out at once (ring_issue) or spread beside the consuming chunk's MFMAs (SpreadPieces)
  // (buffer LDS-DMA, as dmip_x3k.h's: the network image's buffer resource, the chunk's byte offset as the scalar
  // offset, the wave's and lane's part as the per-lane offset -- no per-piece 64-bit address arithmetic)
  __amdgpu_buffer_rsrc_t dma_rsrc;
  unsigned voff;  // w PPW KiB + 16 lane
  int dma_soff;
  char* dma_dst;
  __device__ __forceinline__ void ring_target() {
    const int c = __builtin_amdgcn_readfirstlane(c_issue);
    const int n = __builtin_amdgcn_readfirstlane(ncn);
    // (round 6 tried setting a one-network engine's resource once, in init, and only the offset per chunk: with the
    // immediate-offset pieces below it gave wrong chains at W = 512 with 1 and 3 hidden layers, right ones with 2, and
    // either change alone was right; not understood, not kept -- scripts/x3_w512_debug.py)
    dma_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)(c < n ? img[0] : img[1]), 0, n * CHUNK, 0x00020000);
    dma_soff = __builtin_amdgcn_readfirstlane((c < n ? c : c - n) * CHUNK);
    dma_dst = lds + RING_OFF + __builtin_amdgcn_readfirstlane(s_issue) * CHUNK;
    c_issue = c_issue + 1 == NNET * ncn ? 0 : c_issue + 1;
    s_issue = s_issue + 1 == R ? 0 : s_issue + 1;
  }
  // (round 6: the instruction's 12-bit offset carries Q's KiB within a group of four pieces -- the hardware adds it to
  // both the memory and the LDS address -- so four consecutive pieces share M0 and the scalar offset)
  // (CDiffE at W = 512, L1R, keeps the per-piece form: with the shared offsets its streamed layer 1 spilled 12 B)
  static constexpr bool IMM = !X3_NO_IMM && !L1R;
  template <int Q>
  __device__ __forceinline__ void ring_piece() const {
    if constexpr ((DIAG & 16) != 0) return;
    constexpr int QH = IMM ? Q >> 2 : Q, QL = IMM ? Q & 3 : 0;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(dma_rsrc, (lds_void*)(dma_dst + (w * PPW + (IMM ? 4 : 1) * QH) * 1024), 16,
                                             voff, dma_soff + QH * (IMM ? 4096 : 1024), QL * 1024, 0);
  }
  template <int Q = 0>
  __device__ __forceinline__ void ring_pieces() const {
    if constexpr (Q < PPW) {
      ring_piece<Q>();
      ring_pieces<Q + 1>();
    }
  }
  __device__ __forceinline__ void ring_issue() {
    ring_target();
    ring_pieces();
  }
  // the hook of split_product_h: piece Q of the pending refill beside k-step U = (Q NU) / PPW of the chunk
  struct SpreadPieces {
    const XEngine* e;
    template <int U, int NU, int Q = 0>
    __device__ __forceinline__ void at() const {
      if constexpr (Q < PPW) {
        if constexpr ((Q * NU) / PPW == U) e->template ring_piece<Q>();
        at<U, NU, Q + 1>();
      }
    }
  };
  // Round 5: a hidden or output chunk's refill pieces are spread over its k-steps (one per NU / PPW MFMA groups)
  // instead of a burst of PPW LDS-DMA instructions at the chunk start, which held the wave's issue for ~100-185
  // cycles a piece (MI355X_MICROARCH.md) before the first MFMA. DMIP_X3_BURST_DMA (A/B builds) keeps the burst.
#ifdef DMIP_X3_BURST_DMA
  static constexpr bool SPREAD = false;
#else
  // (with R = 2 slots -- the Posterior's two layer-1 images at W = 512 -- a refill is consumed by the very next
  // chunk, and pieces issued late in a chunk would land after it starts: those rings keep the burst)
  static constexpr bool SPREAD = !RES && (DIAG & 1) == 0 && R >= 3;
#endif

  // the next chunk of the stream, landed (own pieces counted, the others' by the barrier); the slot
  // read one chunk ago is refilled R - 1 chunks ahead
  __device__ __forceinline__ const char* chunk_sync() {
    if constexpr (RES) {
      const char* slot = lds + RING_OFF + s_read * CHUNK;
      s_read = s_read + 1 == ncn ? 0 : s_read + 1;
      return slot;
    }
    if constexpr (DIAG & 1) {
      asm volatile("" ::: "memory");
      const char* slot = lds + RING_OFF + s_read * CHUNK;
      s_read = s_read + 1 == R ? 0 : s_read + 1;
      return slot;
    }
    if constexpr ((DIAG & 32) == 0) wait_vmcnt<(R - 2) * PPW>();
    if constexpr ((DIAG & 8) == 0) lds_barrier();
    ring_issue();
    const char* slot = lds + RING_OFF + s_read * CHUNK;
    s_read = s_read + 1 == R ? 0 : s_read + 1;
    return slot;
  }
  // chunk_sync for a chunk whose MFMAs issue the refill's pieces themselves (split_product_h + SpreadPieces): the
  // same waits and barrier, the refill's target set but nothing issued yet. The pieces of a refill are all issued
  // within the chunk that set it, so the vmcnt accounting of chunk_sync holds.
  __device__ __forceinline__ const char* chunk_sync_deferred() {
    if constexpr ((DIAG & 32) == 0) wait_vmcnt<(R - 2) * PPW>();
    if constexpr ((DIAG & 8) == 0) lds_barrier();
    ring_target();
    const char* slot = lds + RING_OFF + s_read * CHUNK;
    s_read = s_read + 1 == R ? 0 : s_read + 1;
    return slot;
  }

  __device__ __forceinline__ void stage(char* dst, const char* src, int bytes) {
    for (int blk = w; blk < bytes / 1024; blk += NW) glds16(src + blk * 1024, dst + blk * 1024, lane);
  }

  __device__ __forceinline__ void start() {
    if constexpr (RES) {  // the whole stream into slots 0 .. ncn - 1, landed and visible before the first step
      for (int q = 0; q < ncn; ++q) ring_issue();
      wait_vmcnt<0>();
      __syncthreads();
      return;
    }
    wait_vmcnt<0>();
    __syncthreads();
    for (int q = 0; q < R - 1; ++q) ring_issue();
  }

  __device__ __forceinline__ void finish() { wait_vmcnt<0>(); }

  // accumulator init of tile `tile` of layer li (0 = layer 1; nl = the output layer)
  __device__ __forceinline__ f32x4 bias4(int ni, int li, int tile) const {
    return *(const f32x4*)((const float*)(lds + bias_off[ni]) + li * W + 16 * tile + 4 * g);
  }

  // activate tile o (compile-time after unrolling) into the (hi, lo) B operands of the next layer
  template <bool L1>
  __device__ __forceinline__ void act_store(const f32x4& z, int o, u32x4 (&Oh)[KQ], u32x4 (&Ol)[KQ]) const {
    float r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if constexpr (L1 ? (DIAG & 4) != 0 : (DIAG & 2) != 0) r[k] = z[k];
      else r[k] = L1 ? x3_act_r2(z[k]) : x3_act_r(z[k]);
    }
    uint32_t h0, l0, h1, l1;
    split_pair(r[0], r[1], h0, l0);
    split_pair(r[2], r[3], h1, l1);
    const int q = o >> 1, d = (o & 1) * 2;
    Oh[q][d] = h0, Oh[q][d + 1] = h1;
    Ol[q][d] = l0, Ol[q][d + 1] = l1;
  }

  // layer 1 from the resident image and the B operand b1 (all ST tiles' pre-activations in one prefetched
  // MFMA chain), then the double tanh of every tile
  __device__ __forceinline__ void layer1(int ni, const u32x4 (&b1)[K1Q], u32x4 (&Oh)[KQ], u32x4 (&Ol)[KQ]) {
    asm volatile("" ::: "memory");
    f32x4 acc[ST];
#pragma unroll
    for (int o = 0; o < ST; ++o) acc[o] = bias4(ni, 0, o);
    lgkm_drain();
    constexpr int STR = L1H ? 512 : 1024;
    const lds_cptr base = (lds_cptr)(lds + l1_off[ni] + (L1H ? (lane & 31) : lane) * 16);
    constexpr int NU = ST * K1Q;
    u32x4 fa[4];
    fa[0] = lds_rd<0>(base);
    if constexpr (NU > 1) fa[1] = lds_rd<STR>(base);
    if constexpr (NU > 2) fa[2] = lds_rd<2 * STR>(base);
    l1_chain<K1Q, NU, 3, 0, STR>(base, b1, acc, fa);
#pragma unroll
    for (int o = 0; o < ST; ++o) act_store<true>(acc[o], o, Oh, Ol);
  }

  // layer 1 streamed through the ring (L1R): chunk q holds k-step q of all ST output tiles ([o][64][8]); all
  // ST accumulators stay in registers over the K1Q chunks, then the double tanh of every tile
  __device__ __forceinline__ void layer1_ring(int ni, const u32x4 (&b1)[K1Q], u32x4 (&Oh)[KQ], u32x4 (&Ol)[KQ]) {
    f32x4 acc[ST];
#pragma unroll
    for (int o = 0; o < ST; ++o) acc[o] = bias4(ni, 0, o);
    lgkm_drain();
#pragma unroll
    for (int q = 0; q < K1Q; ++q) {
      const char* ch = chunk_sync();
      const lds_cptr base = (lds_cptr)(ch + lane * 16);
      u32x4 fa[4];
      fa[0] = lds_rd<0>(base);
      fa[1] = lds_rd<1024>(base);
      fa[2] = lds_rd<2048>(base);
      const u32x4 bq[1] = {b1[q]};
      if (q + 1 < K1Q) l1_chain<1, ST, 3>(base, bq, acc, fa);
      else l1_chain_act<0>(base, bq[0], acc, fa, Oh, Ol);  // each tile activated once complete
    }
  }
  // the last layer-1 chunk: tile F's MFMA, then the double tanh of tile F - 2 (its MFMA retired), so the
  // accumulators free progressively instead of all ST staying live beside the activated operands
  template <int F>
  __device__ __forceinline__ void l1_chain_act(lds_cptr base, const u32x4& b, f32x4 (&acc)[ST], u32x4 (&fa)[4],
                                               u32x4 (&Oh)[KQ], u32x4 (&Ol)[KQ]) const {
    if constexpr (F < ST + 2) {
      if constexpr (F < ST) {
        if constexpr (F + 3 < ST) fa[(F + 3) % 4] = lds_rd<(F + 3) * 1024>(base);
        lds_wait1<cmin(ST - 1 - F, 3)>(fa[F % 4]);
        acc[F] = mfma16(fa[F % 4], b, acc[F]);
      }
      if constexpr (F >= 2) act_store<true>(acc[F - 2], F - 2, Oh, Ol);
      l1_chain_act<F + 1>(base, b, acc, fa, Oh, Ol);
    }
  }

  __device__ __forceinline__ void hidden(int ni, int li, const u32x4 (&Hh)[KQ], const u32x4 (&Hl)[KQ],
                                         u32x4 (&Oh)[KQ], u32x4 (&Ol)[KQ]) {
    f32x4 pend[CT];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      f32x4 acc[CT];
#pragma unroll
      for (int t = 0; t < CT; ++t) acc[t] = bias4(ni, li, c * CT + t);
      lgkm_drain();
      if constexpr (SPREAD) {
        const char* ch = chunk_sync_deferred();
        split_product_h<KQ, CT * KQ, 2>((lds_cptr)(ch + lane * 16), Hh, Hl, acc, SpreadPieces{this});
      } else {
        const char* ch = chunk_sync();
        split_product<KQ, CT * KQ, 2>((lds_cptr)(ch + lane * 16), Hh, Hl, acc);
      }
      // the previous chunk's tiles are activated beside this chunk's MFMAs
      if (c > 0) {
#pragma unroll
        for (int t = 0; t < CT; ++t) act_store<false>(pend[t], (c - 1) * CT + t, Oh, Ol);
      }
#pragma unroll
      for (int t = 0; t < CT; ++t) pend[t] = acc[t];
    }
#pragma unroll
    for (int t = 0; t < CT; ++t) act_store<false>(pend[t], (NCH - 1) * CT + t, Oh, Ol);
  }

  // output rows 0..15 (tile 0 of the output chunk)
  __device__ __forceinline__ f32x4 output(int ni, const u32x4 (&Hh)[KQ], const u32x4 (&Hl)[KQ]) {
    f32x4 acc[1] = {bias4(ni, nl, 0)};
    lgkm_drain();
    if constexpr (SPREAD) {
      const char* ch = chunk_sync_deferred();
      split_product_h<KQ, KQ, 2>((lds_cptr)(ch + lane * 16), Hh, Hl, acc, SpreadPieces{this});
    } else {
      const char* ch = chunk_sync();
      split_product<KQ, KQ, 2>((lds_cptr)(ch + lane * 16), Hh, Hl, acc);
    }
    return acc[0];
  }

  // one network: layer 1, the nl - 1 hidden layers (ping-pong), the output tile
  __device__ __forceinline__ f32x4 eval(int ni, const u32x4 (&b1)[K1Q]) {
    u32x4 Ah[KQ], Al[KQ], Bh[KQ], Bl[KQ];
    if constexpr (L1R) layer1_ring(ni, b1, Ah, Al);
    else layer1(ni, b1, Ah, Al);
    for (int li = 1; li < nl; li += 2) {
      hidden(ni, li, Ah, Al, Bh, Bl);
      if (li + 1 < nl) hidden(ni, li + 1, Bh, Bl, Ah, Al);
    }
    if (((nl - 1) & 1) != 0) return output(ni, Bh, Bl);
    return output(ni, Ah, Al);
  }
};

// layer-1 B operand: input n at k-slots 3n (hi), 3n+1 (lo), 3n+2 (hi); lane group g supplies slots
// 32 q + 8 g + m of its chain
template <int NV, int K1Q>
__device__ __forceinline__ void l1_operand(const float (&v)[NV], int g, u32x4 (&b)[K1Q]) {
  _Float16 vh[NV], vl[NV];
#pragma unroll
  for (int n = 0; n < NV; ++n) {
    vh[n] = (_Float16)v[n];
    vl[n] = (_Float16)(v[n] - (float)vh[n]);
  }
  auto slot = [&](int s) -> _Float16 {
    const int n = s / 3, p = s % 3;
    if (n >= NV) return (_Float16)0.0f;
    return p == 1 ? vl[n] : vh[n];
  };
#pragma unroll
  for (int q = 0; q < K1Q; ++q) {
    f16x8 e;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const _Float16 c0 = slot(32 * q + m), c1 = slot(32 * q + 8 + m), c2 = slot(32 * q + 16 + m),
                     c3 = slot(32 * q + 24 + m);
      e[m] = g == 0 ? c0 : (g == 1 ? c1 : (g == 2 ? c2 : c3));
    }
    b[q] = __builtin_bit_cast(u32x4, e);
  }
}

// Range of the split: every layer-1 input v is carried as fp16 hi + lo, exact to ~2^-22 |v| for |v| <= 65504
// (fp16's largest finite value; below 2^-14 hi is subnormal and the pair holds ~2^-24 absolute). A chain whose
// input leaves it (a diverging trajectory) is flagged and reported through the device status word.
template <int NV>
__device__ __forceinline__ bool out_of_range(const float (&v)[NV]) {
  bool o = false;
#pragma unroll
  for (int n = 0; n < NV; ++n) o |= __builtin_fabsf(v[n]) > 65504.0f;  // (false for NaN: a lost hand-over)
  return o;
}
// (compare-and-swap from 0: a hand-over timeout already recorded -- its NaN state would also read as out of
// range -- keeps its own code)
__device__ __forceinline__ void report_range(bool oor, unsigned* err, int lane) {
  if (__builtin_amdgcn_ballot_w64(oor) != 0 && lane == 0) {
    unsigned expected = 0u;
    __hip_atomic_compare_exchange_strong(err, &expected, kErrRange, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---------------------------------------------------------------------------- sampler kernel
// The reverse-SDE loop (models/diffusion.py:27-46) with fp32-accurate networks:
//   MODE_CDE        a = net(x, y, tau), y folded into the per-y layer-1 bias (f64 prep)
//   MODE_POSTERIOR  a = g (lik(x, y, tau) + prior(x, tau))            (nets.py:155-157)
//   MODE_CDIFFE     y_t = eps std(tau) + mean_weight(tau) y, a = net(x, y_t, tau)[:D]   (+ Langevin
//                   corrector steps before each predictor step)
// then mu = g a + 0.5 beta x, x <- x + delta mu + sqrt(delta) g xi (dmip_device.h em_update). Work
// distribution: the balanced WaveSchedule over 16-chain tiles (as dmip_f32.h).
template <int MODE, int W, int D, int M, int DIAG = 0>
struct SamplerCfg {
  static constexpr int NNET = MODE == SAMPLER_POSTERIOR ? 2 : 1;
  static constexpr int NV = MODE == SAMPLER_CDIFFE ? D + M + 1 : D + 1;  // layer-1 inputs (y folded for CDE)
  static constexpr int K1Q = k1q_of(NV);
  // CDiffE's split layer 1 over all inputs streams through the ring when it would not fit resident
  static constexpr bool L1R = MODE == SAMPLER_CDIFFE && Shape<W>::ST * K1Q * 1024 > 48 * 1024;
  static constexpr bool L1H = !L1R && K1Q == 1 && 3 * NV <= 16;
  using L = XLay<W, NNET, K1Q, M, L1R, L1H>;
  using E = XEngine<W, NNET, K1Q, L::R, L::RING, DIAG, L1R, L1H>;
};

template <int MODE, int W, int D, int M, bool NOISE, int DIAG = 0>
__global__ void __launch_bounds__(Shape<W>::NW * 64, Shape<W>::NW / 4) x3_sampler_kernel(X3SamplerParams p) {
  using C = SamplerCfg<MODE, W, D, M, DIAG>;
  using L = typename C::L;
  using E = typename C::E;
  constexpr int NW = Shape<W>::NW, ST = Shape<W>::ST, K1Q = C::K1Q;
  static_assert(L::TOTAL <= kLdsBudget, "LDS budget");
  static_assert(D <= 4, "output rows of a chain sit in lane group 0 (D <= 4)");
  __shared__ __attribute__((aligned(16))) char lds[L::TOTAL];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, j = lane & 15;
  const int yi = blockIdx.y;

  E eng{lds, {p.net[0].stream, p.net[1].stream}, {L::L1, L::L1 + L::L1_BYTES}, {L::BIAS, L::BIAS + L::BIAS_BYTES}};
  eng.w = w, eng.lane = lane, eng.g = g;
  eng.init(p.n_hidden);
  {
    const int bf = p.n_hidden * W + 16;
    for (int ni = 0; ni < C::NNET; ++ni) {
      if constexpr (C::L1H) {  // lanes 0-31 of each tile's 1 KiB ([tile][64 lanes][16 B] -> [tile][32][16 B])
        const uint4* s1 = (const uint4*)p.net[ni].l1;
        uint4* d1 = (uint4*)(lds + L::L1 + ni * L::L1_BYTES);
        for (int e = threadIdx.x; e < L::L1_BYTES / 16; e += NW * 64) d1[e] = s1[(e >> 5) * 64 + (e & 31)];
      } else {
        eng.stage(lds + L::L1 + ni * L::L1_BYTES, p.net[ni].l1, L::L1_BYTES);
      }
      float* bl = (float*)(lds + L::BIAS + ni * L::BIAS_BYTES);
      // CDE / likelihood: layer 1's bias is the per-y c (b1 + W1_y y) (x3_bias_prep_kernel)
      const bool per_y = ni == 0 && MODE != SAMPLER_CDIFFE;
      for (int i = threadIdx.x; i < bf; i += NW * 64)
        bl[i] = (per_y && i < W) ? p.bias_y[(size_t)yi * W + i] : p.net[ni].bias[i];
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
  (void)ST;
  bool oor = false;  // a layer-1 input out of the split's range (report_range)

  for (int sgi = 0; sgi < sched.n_seg; ++sgi) {
    const Seg sg = sched.segment(sgi);
    const long long c_local = (long long)(sg.job >= 0 ? sg.job : 0) * 16 + j;
    const bool valid = sg.job >= 0 && c_local < p.n_chains;
    const long long c_rd = valid ? c_local : 0;
    const bool live = sg.kind != 3 && valid;  // a chain whose result is kept (idle segments and padded lanes are not)
    // the chain index again where it is needed after the step loop or per snapshot, from the wave-uniform job and the
    // lane id (v_mbcnt), so that no per-lane index stays live across the loop (at W = 512 it was spilled to scratch)
    auto chain_now = [&]() __attribute__((always_inline)) {
      const int jl = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) & 15;
      return (long long)(sg.job >= 0 ? sg.job : 0) * 16 + jl;
    };
    Rng rng;
    float x[D];
    if (sg.kind == 2) {  // resume the tile the previous wave of the grid handed over
      const size_t slot = (size_t)yi * n_waves + gw - 1;
      const bool lost = handover_wait(p.xflag + slot, p.spin_limit, p.err, kErrHandover, lane);
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
      float v[C::NV];
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
      v[C::NV - 1] = cf.tau;

      // a(x) at this step's time (and y_t): output rows 0..D-1 of every chain, on all its lanes. Always
      // inlined: an outlined call would put the activation arrays on the scratch stack.
      auto score = [&](const float (&vin)[C::NV], float (&a)[D]) __attribute__((always_inline)) {
        u32x4 b1[K1Q];
        l1_operand<C::NV, K1Q>(vin, g, b1);
        oor |= live && out_of_range(vin);  // only chains whose results are returned
        f32x4 out = eng.eval(0, b1);
        if constexpr (C::NNET > 1) out = out + eng.eval(1, b1);  // likelihood + prior, then g * (...)
#pragma unroll
        for (int k = 0; k < D; ++k) a[k] = __shfl(out[k], j, 64);
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
      {
        const long long cn = chain_now();
        snap.at_step<D>(i0, p.snap_every, p.snap_out, gridDim.y, yi, p.n_chains, cn,
                        sg.kind != 3 && sg.job >= 0 && cn < p.n_chains && g == 0, x);
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
    } else if (const long long cn = chain_now(); sg.kind != 3 && sg.job >= 0 && cn < p.n_chains && g == 0) {
      float* dst = p.x_out + ((size_t)yi * p.n_chains + cn) * D;
#pragma unroll
      for (int k = 0; k < D; ++k) dst[k] = x[k];
    }
  }
  eng.finish();
  report_range(oor, p.err, lane);
}

}  // namespace x3

// ----------------------------------------------------------------- launch helpers (per TU)
template <int MODE, int W, int D, int M, bool NOISE, int DIAG = 0>
inline hipError_t launch_x3_sampler_t(const X3SamplerParams& p, int n_y, hipStream_t st) {
  constexpr int NW = x3::Shape<W>::NW;
  auto kern = x3::x3_sampler_kernel<MODE, W, D, M, NOISE, DIAG>;
  const long long tiles = (p.n_chains + 15) / 16;
  long long g = resident_slots(kern, NW * 64, st) / (n_y > 0 ? n_y : 1);
  const long long cap = (tiles + NW - 1) / NW;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  // the balanced schedule's hand-over needs every workgroup of the grid resident at once: g is
  // capped by the stream device's occupancy above
  X3SamplerParams q = p;
  char* buf = nullptr;
  hipError_t e = alloc_handover((size_t)g * n_y * NW, D, st, &buf, &q.xfer, &q.xflag);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)g, (unsigned)n_y), dim3(NW * 64), 0, st, q);
  e = hipGetLastError();
  (void)hipFreeAsync(buf, st);
  return e;
}

template <int MODE, int W, int D, int M>
inline hipError_t launch_x3_sampler_n(const X3SamplerParams& p, int n_y, hipStream_t st) {
  if constexpr (MODE == SAMPLER_CDE) {
    if (p.noise) return launch_x3_sampler_t<MODE, W, D, M, true>(p, n_y, st);
  }
  return launch_x3_sampler_t<MODE, W, D, M, false>(p, n_y, st);
}

// per-mode instantiations (dmip_x3_{cde,post,cdiffe}.hip)
hipError_t launch_x3_sampler_cde(const X3SamplerParams& p, int width, int xdim, int n_y, hipStream_t st, bool* ok);
hipError_t launch_x3_sampler_post(const X3SamplerParams& p, int width, int xdim, int n_y, hipStream_t st, bool* ok);
hipError_t launch_x3_sampler_cdiffe(const X3SamplerParams& p, int width, int xdim, int ydim, int n_y, hipStream_t st,
                                    bool* ok);

}  // namespace dmip
