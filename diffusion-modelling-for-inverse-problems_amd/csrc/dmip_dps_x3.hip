// Diffusion posterior sampling (BASELINE config 4; dmip_surrogate.hip dps_kernel documents the method) at the
// reference's fp32 accuracy on the fp16 matrix rate: every product as the three-term split of dmip_x3.h
// (W_hi h_hi + W_hi h_lo + W_lo h_hi on v_mfma_f32_16x16x32_f16, fp32 accumulation).
//
// Per step and chain (tau = T - t_i):
//   s = prior(x, tau)                                   MLP2 [256]^3, double tanh on layer 1 (nets.py:37-57)
//   x0 = (x + var s) / mean_weight                      Tweedie
//   f = F(x0); v = dL/df                                the scatterometry surrogate (utils_scatterometry.py:8-25)
//   gx = J_F^T v                                        its reverse pass (ReLU masks)
//   G = (gx + var J_s^T gx) / mean_weight               the prior's vector-Jacobian product (reverse pass)
//   x <- EM(x, g s) - lambda G
// The exact-f32 kernel forms J_s by forward tangents (four prior passes); here one reverse pass through the prior
// replaces the three tangent passes: the forward keeps the hidden tanh layers' derivatives (4 r (1 - r) in r-form)
// in registers, 128 per lane; layer 1's (16 r1 (1 - r1) r2 (1 - r2) of its double tanh) is recomputed in the
// reverse pass from its pre-activation, one MFMA per tile on the resident image.
//
// Layout (one wave = 16 chains, four waves per workgroup, one per SIMD): a layer's output tile is 16 units x 16
// chains (lane (g, j): units 16 o + 4 g + r of chain j), which is the next layer's B operand with no lane movement
// (dmip_x3.h). Every 256-wide layer streams from L2 through a 4-slot LDS ring in 32 KiB chunks of two output tiles
// (hi + lo fragments of all eight k-steps); the per-step chunk stream is the prior's forward (hidden 2, 3, output),
// the surrogate's forward (hidden 2, 3, output), its reverse pass (W4^T, W3^T, W2^T, W1^T) and the prior's reverse
// pass (W4^T, W3^T, W2^T, W1's x columns): 70 chunks. Both networks' layer 1 and all biases are LDS-resident.
// The reverse passes carry a per-chain power-of-two scale (exact) so the split operands stay inside fp16's range;
// a surrogate activation or an input beyond it is reported (kErrRange, dmip_device_status), as the fp32x3 samplers
// do, and the Python default resamples in exact f32.
#include "dmip_x3.h"

#include <cstdlib>
#include <utility>

namespace dmip {
namespace dx3 {

using x3::f32x4;
using x3::lds_cptr;
using x3::mfma16;

constexpr int W = 256, ST = 16, KQ = 8, CT = 2, TILE = KQ * 2048, CHUNK = CT * TILE, NCH = ST / CT;
constexpr int NW = 4, R = 4, PPW = CHUNK / 1024 / NW;
// fragment pairs read ahead in a chunk's MFMA chain, in units (3 MFMAs each); DMIP_DPS_FPF = 2 for A/B builds
#ifdef DMIP_DPS_FPF
constexpr int FPF = DMIP_DPS_FPF;
#else
constexpr int FPF = 1;
#endif
static_assert(FPF == 1 || FPF == 2, "read-ahead depth");
// timing ablations of A/B builds only (never the product library; the range report is off in them):
// DMIP_DPS_DIAG bit 0 = no LDS-DMA pieces (stale weights), bit 1 = no ring barriers, bit 2 = no ring vmcnt waits
#ifdef DMIP_DPS_DIAG
constexpr int DDIAG = DMIP_DPS_DIAG;
#else
constexpr int DDIAG = 0;
#endif
__device__ __forceinline__ void ring_barrier() {
  if constexpr ((DDIAG & 2) == 0) lds_barrier();
}
template <int N>
__device__ __forceinline__ void ring_vmcnt() {
  if constexpr ((DDIAG & 4) == 0) wait_vmcnt<N>();
}
static_assert(CHUNK == 32768 && PPW == 8, "ring geometry");
// the per-step chunk stream: prior image chunks [0, 17) = P2 (8) | P3 (8) | Pout (1), then the surrogate's 35,
// then prior chunks [17, 35) = P4^T (1) | P3^T (8) | P2^T (8) | P1^T (1)
constexpr int NPF = 17, NS = 35, NPB = 18, NSTREAM = NPF + NS + NPB;

// LDS
constexpr int RING = 0;
constexpr int PL1 = RING + R * CHUNK;        // prior layer 1: [16 tiles][32 lanes][16 B] (lanes 32-63 read 0-31)
constexpr int SL1 = PL1 + ST * 512;          // surrogate layer 1, same layout
constexpr int PB = SL1 + ST * 512;           // prior: c b1 | init2 | init3 [256] | out init [16]
constexpr int SB = PB + (3 * W + 16) * 4;    // surrogate: b1 | b2 | b3 [256] | b4 [32]
constexpr int YO = SB + (3 * W + 32) * 4;    // the workgroup's y [32]
constexpr int TOTAL = YO + 32 * 4;
static_assert(TOTAL <= 160 * 1024, "LDS budget");

typedef __attribute__((address_space(3))) void lds_void;

struct Eng {
  char* lds;
  // the per-step chunk stream in stream order (DPS: launch_dps_x3 copies the prior's 17 forward chunks, the
  // surrogate's 35 and the prior's 18 reverse chunks into one image; MH: the surrogate's image, whose first 17 chunks
  // are its forward pass): chunk c of a step is image chunk c
  const char* img;
  int c_issue, s_issue, s_read;
  int w, lane, g;
  int nstream = NSTREAM;

  // the next refill: its source chunk and ring slot (the stream position advances); its PPW pieces per wave go out at
  // once (ring_issue) or beside the consuming chunk's MFMAs (Spread, split_product_h). The pieces are buffer LDS-DMA
  // (dmip_x3k.h's form): the image's buffer resource, the chunk's byte offset as the scalar offset, the wave's and
  // lane's part as the per-lane offset -- no per-piece 64-bit address arithmetic (a VALU and two SALU a piece with
  // global_load_lds). Round 6: one image in stream order, one buffer resource, the chunk's offset c * 32 KiB (round 5
  // selected between two images' resources and offsets per chunk: 8 more SGPRs in a kernel at the 106-SGPR limit,
  // whose spills cost ~850 v_readlane / v_writelane per step)
  __amdgpu_buffer_rsrc_t dma_rsrc;
  unsigned voff;  // w PPW KiB + 16 lane
  int dma_soff;
  char* dma_dst;
  __device__ __forceinline__ void init_dma() {
    dma_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)img, 0, nstream * CHUNK, 0x00020000);
    voff = (unsigned)(w * PPW * 1024 + lane * 16);
  }
  __device__ __forceinline__ void ring_target() {
    const int c = __builtin_amdgcn_readfirstlane(c_issue);
    dma_soff = c * CHUNK;
    dma_dst = lds + RING + __builtin_amdgcn_readfirstlane(s_issue) * CHUNK;
    c_issue = c + 1 == nstream ? 0 : c + 1;
    s_issue = s_issue + 1 == R ? 0 : s_issue + 1;
  }
  // (round 6: Q's KiB within a group of four pieces in the instruction's offset, which the hardware adds to both the
  // memory and the LDS address: four pieces share M0 and the scalar offset)
  template <int Q>
  __device__ __forceinline__ void ring_piece() const {
    if constexpr ((DDIAG & 1) != 0) return;
    constexpr int QH = Q >> 2, QL = Q & 3;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(dma_rsrc, (lds_void*)(dma_dst + (w * PPW + 4 * QH) * 1024), 16, voff,
                                             dma_soff + QH * 4096, QL * 1024, 0);
  }
  __device__ __forceinline__ void ring_issue() {
    ring_target();
    ring_piece<0>(), ring_piece<1>(), ring_piece<2>(), ring_piece<3>();
    ring_piece<4>(), ring_piece<5>(), ring_piece<6>(), ring_piece<7>();
  }
  // the hook of x3::split_product_h: piece Q of the pending refill beside k-step unit (Q NU) / PPW (round 5: a burst
  // of PPW LDS-DMA instructions at the chunk start held the wave's issue ~100-185 cycles a piece)
  struct Spread {
    const Eng* e;
    template <int U, int NU, int Q = 0>
    __device__ __forceinline__ void at() const {
      if constexpr (Q < PPW) {
        if constexpr ((Q * NU) / PPW == U) e->template ring_piece<Q>();
        at<U, NU, Q + 1>();
      }
    }
  };

  // the next chunk of the stream, landed (own pieces counted, the others' by the barrier); the slot read one
  // chunk ago is refilled R - 1 chunks ahead -- its pieces issued here (chunk_sync) or by the chunk's MFMAs
  // (chunk_sync_deferred + Spread: every piece of a refill within the chunk that set it, so the vmcnt count holds)
  __device__ __forceinline__ lds_cptr chunk_sync() {
    ring_vmcnt<(R - 2) * PPW>();
    ring_barrier();
    ring_issue();
    const char* slot = lds + RING + s_read * CHUNK;
    s_read = s_read + 1 == R ? 0 : s_read + 1;
    return (lds_cptr)(slot + lane * 16);
  }
  __device__ __forceinline__ lds_cptr chunk_sync_deferred() {
    ring_vmcnt<(R - 2) * PPW>();
    ring_barrier();
    ring_target();
    const char* slot = lds + RING + s_read * CHUNK;
    s_read = s_read + 1 == R ? 0 : s_read + 1;
    return (lds_cptr)(slot + lane * 16);
  }

  __device__ __forceinline__ f32x4 bias4(int off_bytes, int tile) const {
    return *(const f32x4*)(lds + off_bytes + (16 * tile + 4 * g) * 4);
  }

  // MID (round 5; dmip_x3k.h's ring protocol): chunk c + 1's barrier B(c + 1) in the MIDDLE of chunk c (after unit
  // NU / 2), then the refill of chunk c - 1's slot spread over the rest of chunk c, and chunk c + 1's first fragment
  // pair read ahead at the last unit (nxt). At one wave per SIMD a wave reaching the barrier early waits while its
  // MFMAs are still in the pipe, and no chunk starts with an LDS-latency bubble. R = 4: a refill issued in chunk c
  // lands by B(c + 2)'s wait, one and a half chunks later.
  u32x4 nxt0, nxt1;  // the next chunk's unit 0 fragment pair
  u32x4 nxa0, nxa1;  // and its unit 1 pair (FPF = 2)
  __device__ __forceinline__ void start_mid() {
    for (int q = 0; q < R - 1; ++q) ring_issue();
    ring_vmcnt<(R - 2) * PPW>();
    ring_barrier();
    const lds_cptr b0 = (lds_cptr)(lds + RING + lane * 16);
    nxt0 = x3::lds_rd<0>(b0);
    nxt1 = x3::lds_rd<1024>(b0);
    if constexpr (FPF == 2) {
      nxa0 = x3::lds_rd<2048>(b0);
      nxa1 = x3::lds_rd<3072>(b0);
    }
    wait_next();
  }
  __device__ __forceinline__ void wait_next() {
    if constexpr (FPF == 2) x3::lds_wait2<0>(nxa0, nxa1);
    x3::lds_wait2<0>(nxt0, nxt1);
  }
  // the current chunk's lane base, the ring advanced: the next chunk's lane base in nb
  __device__ __forceinline__ lds_cptr take(lds_cptr& nb) {
    const lds_cptr b = (lds_cptr)(lds + RING + s_read * CHUNK + lane * 16);
    s_read = s_read + 1 == R ? 0 : s_read + 1;
    nb = (lds_cptr)(lds + RING + s_read * CHUNK + lane * 16);
    return b;
  }
};
static_assert(R == 4, "MID's vmcnt accounting: one younger refill in flight at B(c + 1)");
template <int NU, int U, int Q = 0>
__device__ __forceinline__ void mid_pieces(const Eng& e);

// units U0 .. U1 - 1 of a chunk of NU k-step units (unit u: hi / lo fragments at 2u, 2u + 1 KiB), accumulator of unit
// U = acc[(U - U0) / KQ_], B operand (Hh, Hl)[U % KQ_]; fragment pairs are read FPF units ahead, fa[U % (FPF + 1)]
// holds unit U's pair on entry (units 0 .. FPF - 1: nxt, nxa)
template <int KQ_, int NU, int U0, int U1, int NA, int U = U0>
__device__ __forceinline__ void mid_units(Eng& e, lds_cptr base, lds_cptr nbase, const u32x4 (&Hh)[KQ_],
                                          const u32x4 (&Hl)[KQ_], f32x4 (&acc)[NA], u32x4 (&fa)[FPF + 1][2]) {
  if constexpr (U < U1) {
    constexpr int MIDU = NU / 2;
    static_assert(MIDU < NU - FPF, "the barrier precedes the read-ahead");
    constexpr int A = U + FPF, S = U % (FPF + 1);
    if constexpr (A < NU) {
      fa[A % (FPF + 1)][0] = x3::lds_rd<(2 * A) * 1024>(base);
      fa[A % (FPF + 1)][1] = x3::lds_rd<(2 * A + 1) * 1024>(base);
    } else if constexpr (A == NU) {  // after B(c + 1): the next chunk has landed for every wave
      e.nxt0 = x3::lds_rd<0>(nbase);
      e.nxt1 = x3::lds_rd<1024>(nbase);
    } else {
      e.nxa0 = x3::lds_rd<2048>(nbase);
      e.nxa1 = x3::lds_rd<3072>(nbase);
    }
    x3::lds_wait2<2 * FPF>(fa[S][0], fa[S][1]);
    constexpr int t = (U - U0) / KQ_, q = U % KQ_;
    acc[t] = mfma16(fa[S][0], Hl[q], acc[t]);
    acc[t] = mfma16(fa[S][1], Hh[q], acc[t]);
    acc[t] = mfma16(fa[S][0], Hh[q], acc[t]);
    if constexpr (U == MIDU) {  // own pieces of chunk c + 1 landed (chunk c + 2's younger), then everyone's
      ring_vmcnt<PPW>();
      ring_barrier();
      e.ring_target();  // chunk c - 1's slot: every wave has passed its last read
    }
    if constexpr (U > MIDU) mid_pieces<NU, U>(e);
    mid_units<KQ_, NU, U0, U1, NA, U + 1>(e, base, nbase, Hh, Hl, acc, fa);
  }
}
template <int NU, int U, int Q>
__device__ __forceinline__ void mid_pieces(const Eng& e) {
  if constexpr (Q < PPW) {
    constexpr int MIDU = NU / 2;
    if constexpr (MIDU + 1 + (Q * (NU - 1 - MIDU)) / PPW == U) e.template ring_piece<Q>();
    mid_pieces<NU, U, Q + 1>(e);
  }
}
// a whole chunk of NU units
template <int KQ_, int NU, int NA>
__device__ __forceinline__ void mid_chunk(Eng& e, const u32x4 (&Hh)[KQ_], const u32x4 (&Hl)[KQ_], f32x4 (&acc)[NA]) {
  lds_cptr nb;
  const lds_cptr b = e.take(nb);
  u32x4 fa[FPF + 1][2];
  fa[0][0] = e.nxt0, fa[0][1] = e.nxt1;
  if constexpr (FPF == 2) fa[1][0] = e.nxa0, fa[1][1] = e.nxa1;
  mid_units<KQ_, NU, 0, NU, NA>(e, b, nb, Hh, Hl, acc, fa);
  e.wait_next();  // an asm load's registers must not leave the chunk before its data lands
}

// (hi, lo) B operand of k-step q from two accumulator-form tiles' f32 values v[2 q], v[2 q + 1] (dmip_x3.h
// act_store's dword order)
__device__ __forceinline__ void store_pair(const float (&a)[4], int o, u32x4 (&Oh)[KQ], u32x4 (&Ol)[KQ]) {
  uint32_t h0, l0, h1, l1;
  x3::split_pair(a[0], a[1], h0, l0);
  x3::split_pair(a[2], a[3], h1, l1);
  const int q = o >> 1, d = (o & 1) * 2;
  Oh[q][d] = h0, Oh[q][d + 1] = h1;
  Ol[q][d] = l0, Ol[q][d + 1] = l1;
}

__device__ __forceinline__ bool beyond_fp16(float v) { return !(__builtin_fabsf(v) <= 65504.0f); }
// the running max |v| of the values a chain splits, checked once at the end (range_bad): a value beyond fp16's range
// is finite and > 65504 or inf when it first appears -- what follows from it may be NaN, but the max has seen the
// first one. Kept as float bits in a signed int: for non-negative floats the integer order is the float order, and
// v_max3_i32 needs none of the NaN-quieting v_max a float max inserts before each operand; |v| is v's bits with the
// sign cleared (a NaN then sorts above inf). Pinned by an empty asm: otherwise the compiler re-associates a whole
// pass's max chain into one tree at its end and keeps every tracked value alive until then (DPS: 176 B of scratch and
// 55 more AGPRs; the multi-tile MH engine: hundreds of spilled registers)
__device__ __forceinline__ void track4(int& mx, const float (&v)[4]) {  // any sign
  constexpr int M = 0x7fffffff;
  mx = max(max(mx, __float_as_int(v[0]) & M), __float_as_int(v[1]) & M);
  mx = max(max(mx, __float_as_int(v[2]) & M), __float_as_int(v[3]) & M);
  asm("" : "+v"(mx));
}
__device__ __forceinline__ void track4_pos(int& mx, const float (&v)[4]) {  // v >= +0 (relu outputs)
  mx = max(max(mx, __float_as_int(v[0])), __float_as_int(v[1]));
  mx = max(max(mx, __float_as_int(v[2])), __float_as_int(v[3]));
  asm("" : "+v"(mx));
}
__device__ __forceinline__ bool range_bad(int mx) { return !(__int_as_float(mx) <= 65504.0f); }
// relu on the bits (v_max_i32 with 0; the float select costs a NaN-quieting v_max more): z > 0 passes, every other
// value (-0 and the negative NaNs included) becomes +0
__device__ __forceinline__ float relu_bits(float z) { return __int_as_float(max(__float_as_int(z), 0)); }
// relu and its mask bit, packed per lane in a VGPR word. Left to itself the compiler keeps each bit of the word as the
// compare's 64-lane SGPR pair; at the kernel's 106-SGPR limit the 64 masks of a surrogate layer then spill to VGPR lanes
// (≈830 v_writelane / v_readlane per step). Round 6: the empty asm after each update pins the word in a VGPR, so
// the bits are built by VALU (no lane spills, no scratch; same box 843 -> 835 ms, profiles/r6_vmask/). (The bit as
// min(relu bits, 1), DMIP_DPS_BITS_MASK, also removed the lane spills but spilled 172 B of VGPRs and lost 1.8 %.)
__device__ __forceinline__ void relu_mask(float z, float& h, uint32_t& m, int bit) {
#ifdef DMIP_DPS_BITS_MASK
  const int hb = max(__float_as_int(z), 0);
  h = __int_as_float(hb);
  m |= min((uint32_t)hb, 1u) << bit;
#else
  const bool pos = z > 0.0f;
  h = pos ? z : 0.0f;
  m |= (pos ? 1u : 0u) << bit;
  asm volatile("" : "+v"(m));
#endif
}

// The per-tile epilogues of a 256 -> 256 layer (tile o of the layer's output, f32 pre-activations z):
//   PriorFwd:  r = 1 / (1 + 2^z) (z pre-scaled by 2 log2 e; the next layer is folded for r), D = 4 r (1 - r)
//   SurFwd:    h = relu(z), mask bit, range flag
//   Back:      g = z * D (prior, tanh') or z * mask (surrogate, relu') -- the reverse pass's next B operand
struct EpiPriorFwd {
  float (*D)[4];
  __device__ __forceinline__ void operator()(const f32x4& z, int o, u32x4 (&Oh)[KQ], u32x4 (&Ol)[KQ]) const {
    float r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      r[k] = x3::x3_act_r(z[k]);
      D[o][k] = 4.0f * r[k] * (1.0f - r[k]);
    }
    store_pair(r, o, Oh, Ol);
  }
};
struct EpiSurFwd {
  uint32_t* m;  // [2]: bit 4 (o & 7) + k of word o >> 3
  int* mx;
  __device__ __forceinline__ void operator()(const f32x4& z, int o, u32x4 (&Oh)[KQ], u32x4 (&Ol)[KQ]) const {
    float h[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) relu_mask(z[k], h[k], m[o >> 3], (o & 7) * 4 + k);
    track4_pos(*mx, h);
    store_pair(h, o, Oh, Ol);
  }
};
struct EpiBackD {
  const float (*D)[4];
  int* mx;
  __device__ __forceinline__ void operator()(const f32x4& z, int o, u32x4 (&Oh)[KQ], u32x4 (&Ol)[KQ]) const {
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = z[k] * D[o][k];
    track4(*mx, v);
    store_pair(v, o, Oh, Ol);
  }
};
// the reverse pass into layer 1: g = z * dh1/dz1 with layer 1's double-tanh derivative recomputed per tile from its
// pre-activation (one MFMA on the resident image; 64 registers fewer than keeping it from the forward)
struct EpiBackL1 {
  const char* lds;
  int lane, g;
  u32x4 b1;
  int* mx;
  __device__ __forceinline__ void operator()(const f32x4& z, int o, u32x4 (&Oh)[KQ], u32x4 (&Ol)[KQ]) const {
    const u32x4 a = *(const u32x4*)(lds + PL1 + o * 512 + (lane & 31) * 16);
    const f32x4 c = *(const f32x4*)(lds + PB + (16 * o + 4 * g) * 4);
    const f32x4 z1 = mfma16(a, b1, c);
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float r1 = x3::x3_act_r(z1[k]);
      const float r2 = x3::x3_act_r(__builtin_fmaf(-2.0f * kTanhScale, r1, kTanhScale));
      v[k] = z[k] * (16.0f * r1 * (1.0f - r1) * r2 * (1.0f - r2));
    }
    track4(*mx, v);
    store_pair(v, o, Oh, Ol);
  }
};
struct EpiBackMask {
  const uint32_t* m;
  int* mx;
  __device__ __forceinline__ void operator()(const f32x4& z, int o, u32x4 (&Oh)[KQ], u32x4 (&Ol)[KQ]) const {
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // z AND the bit sign-extended to 32 (v_bfe_i32 + v_and: +0 where relu was off)
      const int keep = __builtin_amdgcn_sbfe((int)m[o >> 3], (o & 7) * 4 + k, 1);
      v[k] = __int_as_float(__float_as_int(z[k]) & keep);
    }
    track4(*mx, v);
    store_pair(v, o, Oh, Ol);
  }
};

// a streamed 256 -> 256 layer: NCH chunks of CT tiles; accumulators start at the bias (bias_off >= 0) or zero; each
// chunk's tiles go to the epilogue while the next chunk's MFMAs run
template <typename Epi>
__device__ __forceinline__ void layer256(Eng& e, const u32x4 (&Hh)[KQ], const u32x4 (&Hl)[KQ], int bias_off,
                                         const Epi& epi, u32x4 (&Oh)[KQ], u32x4 (&Ol)[KQ]) {
  f32x4 pend[CT];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    f32x4 acc[CT];
#pragma unroll
    for (int t = 0; t < CT; ++t) acc[t] = bias_off >= 0 ? e.bias4(bias_off, c * CT + t) : f32x4{0.f, 0.f, 0.f, 0.f};
    mid_chunk<KQ, CT * KQ>(e, Hh, Hl, acc);
    if (c > 0) {
#pragma unroll
      for (int t = 0; t < CT; ++t) epi(pend[t], (c - 1) * CT + t, Oh, Ol);
    }
#pragma unroll
    for (int t = 0; t < CT; ++t) pend[t] = acc[t];
  }
#pragma unroll
  for (int t = 0; t < CT; ++t) epi(pend[t], (NCH - 1) * CT + t, Oh, Ol);
}

// one chunk of NTL tiles over all KQ k-steps of a 256-wide input (output layers, the layer-1 transposes)
template <int NTL>
__device__ __forceinline__ void small256(Eng& e, const u32x4 (&Hh)[KQ], const u32x4 (&Hl)[KQ], int bias_off,
                                         f32x4 (&acc)[NTL]) {
#pragma unroll
  for (int t = 0; t < NTL; ++t) acc[t] = bias_off >= 0 ? e.bias4(bias_off, t) : f32x4{0.f, 0.f, 0.f, 0.f};
  mid_chunk<KQ, NTL * KQ>(e, Hh, Hl, acc);
}

// the transposed output layers (16 tiles, one k-step: the output rows): B = the split of the reverse pass's input
// vector; in two halves of 8 tiles, the first half's epilogue beside the second half's MFMAs (32 accumulator
// registers live instead of 64)
template <typename Epi>
__device__ __forceinline__ void wide1(Eng& e, const u32x4& Bh, const u32x4& Bl, const Epi& epi, u32x4 (&Oh)[KQ],
                                      u32x4 (&Ol)[KQ]) {
  const u32x4 bh[1] = {Bh}, bl[1] = {Bl};
  f32x4 a0[ST / 2], a1[ST / 2];
#pragma unroll
  for (int t = 0; t < ST / 2; ++t) a0[t] = a1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  {  // one chunk of ST units (one k-step per tile), in two halves of accumulators
    lds_cptr nb;
    const lds_cptr b = e.take(nb);
    u32x4 fa[FPF + 1][2];
    fa[0][0] = e.nxt0, fa[0][1] = e.nxt1;
    if constexpr (FPF == 2) fa[1][0] = e.nxa0, fa[1][1] = e.nxa1;
    mid_units<1, ST, 0, ST / 2, ST / 2>(e, b, nb, bh, bl, a0, fa);
    mid_units<1, ST, ST / 2, ST, ST / 2>(e, b, nb, bh, bl, a1, fa);
    e.wait_next();
  }
#pragma unroll
  for (int t = 0; t < ST / 2; ++t) epi(a0[t], t, Oh, Ol);
#pragma unroll
  for (int t = 0; t < ST / 2; ++t) epi(a1[t], ST / 2 + t, Oh, Ol);
}

template <int O, typename Act>
__device__ __forceinline__ void l1_step(lds_cptr la, lds_cptr lb, u32x4 (&fa)[3], u32x4 (&fb)[3], const u32x4& b,
                                        const Act& act) {
  if constexpr (O < ST) {
    if constexpr (O + 2 < ST) fa[(O + 2) % 3] = x3::lds_rd<(O + 2) * 512>(la), fb[(O + 2) % 3] = x3::lds_rd<(O + 2) * 64>(lb);
    x3::lds_wait2<(O + 2 < ST) ? 4 : ((O + 1 < ST) ? 2 : 0)>(fa[O % 3], fb[O % 3]);
    act(mfma16(fa[O % 3], b, __builtin_bit_cast(f32x4, fb[O % 3])), O);
    l1_step<O + 1>(la, lb, fa, fb, b, act);
  }
}

// a resident layer 1 ([16 tiles][32 lanes] image, one MFMA per tile) from the B operand b, then each tile to `act`
template <typename Act>
__device__ __forceinline__ void layer1(const Eng& e, int l1_off, int bias_off, const u32x4& b, const Act& act) {
  const lds_cptr la = (lds_cptr)(e.lds + l1_off + (e.lane & 31) * 16);
  const lds_cptr lb = (lds_cptr)(e.lds + bias_off + 16 * e.g);
  u32x4 fa[3], fb[3];
  fa[0] = x3::lds_rd<0>(la), fb[0] = x3::lds_rd<0>(lb);
  fa[1] = x3::lds_rd<512>(la), fb[1] = x3::lds_rd<64>(lb);
  l1_step<0>(la, lb, fa, fb, b, act);
}
// layer-1 B operand over NV <= 5 inputs: input n in k-slots 3n, 3n + 1, 3n + 2 as [hi, lo, hi] (x3::l1_operand's
// layout), lane group 0 slots 0-7, group 1 slots 8-15, groups 2-3 zero
template <int NV>
__device__ __forceinline__ u32x4 l1_b(const float (&v)[NV], int g) {
  u32x4 b[1];
  x3::l1_operand<NV, 1>(v, g, b);
  return b[0];
}

// a per-chain vector of up to 4 components (all lanes of the chain hold it) as the B operand of a one-k-step
// transposed layer: rows 0..3 of the k-step are lane group 0's m = 0..3 (kperm16(0, 0, m) = m)
__device__ __forceinline__ void vec_b(const float (&v)[4], int g, u32x4& bh, u32x4& bl) {
  uint32_t h0, l0, h1, l1;
  x3::split_pair(v[0], v[1], h0, l0);
  x3::split_pair(v[2], v[3], h1, l1);
  const bool z = g != 0;
  bh = u32x4{z ? 0u : h0, z ? 0u : h1, 0u, 0u};
  bl = u32x4{z ? 0u : l0, z ? 0u : l1, 0u, 0u};
}

// rows 0..3 of an accumulator tile live in lane group 0 (registers 0..3): every lane of chain j gets them
__device__ __forceinline__ float bcast_g0(float v) {
  const auto s1 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(__builtin_amdgcn_permlane32_swap(s1[0], s1[0], false, false)[0]);
}

// 2^e with e = the exponent of max |v| (exact scaling: the reverse passes are linear per chain)
__device__ __forceinline__ float pow2_of(float m) {
  if (!(m > 0.0f) || !(m < 3.0e38f)) return 1.0f;
  int e;
  (void)frexpf(m, &e);
  return ldexpf(1.0f, e);
}

__global__ void __launch_bounds__(NW * 64, 1) dps_x3_kernel(DpsX3Params p) {
  __shared__ __attribute__((aligned(16))) char lds[TOTAL];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, j = lane & 15;
  const int yi = blockIdx.y;
  const long long c_local = (long long)blockIdx.x * (NW * 16) + w * 16 + j;
  const bool valid = c_local < p.n_chains;
  Eng e{lds, p.img, 0, 0, 0, w, lane, g};
  e.init_dma();
  {
    // resident parts: the two layer-1 images (lanes 0-31 of each tile), the biases, y
    const uint4* s1 = (const uint4*)p.pl1;
    const uint4* s2 = (const uint4*)p.sl1;
    uint4* d1 = (uint4*)(lds + PL1);
    uint4* d2 = (uint4*)(lds + SL1);
    for (int i = threadIdx.x; i < ST * 32; i += NW * 64) {
      d1[i] = s1[(i >> 5) * 64 + (i & 31)];
      d2[i] = s2[(i >> 5) * 64 + (i & 31)];
    }
    float* pb = (float*)(lds + PB);
    for (int i = threadIdx.x; i < 3 * W + 16; i += NW * 64) pb[i] = p.pbias[i];
    float* sb = (float*)(lds + SB);
    for (int i = threadIdx.x; i < 3 * W + 32; i += NW * 64) sb[i] = p.sbias[i];
    float* yo = (float*)(lds + YO);
    for (int i = threadIdx.x; i < 32; i += NW * 64) yo[i] = i < kSurYdim ? p.y[(size_t)yi * kSurYdim + i] : 0.0f;
    __syncthreads();
    e.start_mid();
  }
  const float* ylds = (const float*)(lds + YO);

  Rng rng = rng_init(p.seed, (uint64_t)(p.chain_offset + c_local), (uint64_t)yi);
  float x[3];
  {
    float n0[3];
    rng_normals<3>(rng, n0);
#pragma unroll
    for (int d = 0; d < 3; ++d) x[d] = __fadd_rn(__fmul_rn(n0[d], p.stdv), p.mean);
  }
  bool oor = false;
  int vmax = 0;  // track4's running max of the split values (float bits)
  const int S = p.num_steps;
  for (int i = 0; i < S; ++i) {
    const float4 c4 = ((const float4*)p.coef)[2 * i];      // tau, beta, g (dmip_device.h step_coef)
    const float4 c5 = ((const float4*)p.coef)[2 * i + 1];  // mean_weight, var (vp_mean_weight, vp_std^2)
    const StepCoef cf{c4.x, c4.y, c4.z};
    const float mw = c5.x, var = c5.y;
    for (int d = 0; d < 3; ++d) oor |= beyond_fp16(x[d]);

    // ---- prior forward: layer 1 (double tanh), hidden 2, hidden 3 (derivatives kept), output rows 0..2
    float D2[ST][4], D3[ST][4];
    u32x4 Ah[KQ], Al[KQ], Bh[KQ], Bl[KQ];
    const float vin[4] = {x[0], x[1], x[2], cf.tau};
    const u32x4 b1p = l1_b<4>(vin, g);
    layer1(e, PL1, PB, b1p, [&](const f32x4& z, int o) {
      float r2[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) r2[k] = x3::x3_act_r2(z[k]);
      store_pair(r2, o, Ah, Al);
    });
    layer256(e, Ah, Al, PB + W * 4, EpiPriorFwd{D2}, Bh, Bl);
    layer256(e, Bh, Bl, PB + 2 * W * 4, EpiPriorFwd{D3}, Ah, Al);
    float sc[3];
    {
      f32x4 acc[1];
      small256<1>(e, Ah, Al, PB + 3 * W * 4, acc);
#pragma unroll
      for (int d = 0; d < 3; ++d) sc[d] = bcast_g0(acc[0][d]);
    }

    // ---- Tweedie estimate, surrogate forward (masks kept)
    float x0h[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      x0h[d] = (x[d] + var * sc[d]) / mw;
      oor |= beyond_fp16(x0h[d]);
    }
    uint32_t m1[2] = {0u, 0u}, m2[2] = {0u, 0u}, m3[2] = {0u, 0u};
    layer1(e, SL1, SB, l1_b<3>(x0h, g), [&](const f32x4& z, int o) {
      float h[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) relu_mask(z[k], h[k], m1[o >> 3], (o & 7) * 4 + k);
      track4_pos(vmax, h);
      store_pair(h, o, Ah, Al);
    });
    layer256(e, Ah, Al, SB + W * 4, EpiSurFwd{m2, &vmax}, Bh, Bl);
    layer256(e, Bh, Bl, SB + 2 * W * 4, EpiSurFwd{m3, &vmax}, Ah, Al);
    f32x4 f[2];
    small256<2>(e, Ah, Al, SB + 3 * W * 4, f);

    // ---- the guidance's output-space vector v = dL/df and its step size (dps_kernel's two modes)
    f32x4 v[2];
    float scale;
    if (p.mode == 0) {  // NLL: the likelihood terms of get_log_posterior (no boundary prior)
      const float a2 = p.a * p.a;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * t + 4 * g + r;
          float vk = 0.0f;
          if (row < kSurYdim) {
            const float fk = f[t][r];
            const float af = p.a * fk;
            const float pref = af * af + p.b2;
            const float res = ylds[row] - fk;
            const float q = res * res / pref;
            vk = (a2 * fk * (1.0f - q) - res) / pref;
          }
          v[t][r] = vk;
        }
      scale = p.zeta * p.delta * cf.beta;  // zeta delta g^2
    } else {  // NORM: v = d||r||^2/df = -2 r, step zeta / ||r||
      float rr = 0.0f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * t + 4 * g + r;
          const float res = row < kSurYdim ? ylds[row] - f[t][r] : 0.0f;
          rr += res * res;
          v[t][r] = -2.0f * res;
        }
      rr += __shfl_xor(rr, 16, 64);
      rr += __shfl_xor(rr, 32, 64);
      scale = p.zeta * __frsqrt_rn(fmaxf(rr, 1e-30f));
    }

    // ---- surrogate reverse pass gx = J_F^T v, scaled per chain by a power of two (exact)
    float gx[3];
    {
      float mx = 0.0f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, __builtin_fabsf(v[t][r]));
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float s2 = pow2_of(mx), is2 = 1.0f / s2;
      float vs[2][4];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) vs[t][r] = v[t][r] * is2;
      // B of the one-k-step W4^T: rows 0..31 = output rows (tiles 0, 1 in m = 0..3, 4..7)
      uint32_t h0, l0, h1, l1, h2, l2, h3, l3;
      x3::split_pair(vs[0][0], vs[0][1], h0, l0);
      x3::split_pair(vs[0][2], vs[0][3], h1, l1);
      x3::split_pair(vs[1][0], vs[1][1], h2, l2);
      x3::split_pair(vs[1][2], vs[1][3], h3, l3);
      wide1(e, u32x4{h0, h1, h2, h3}, u32x4{l0, l1, l2, l3}, EpiBackMask{m3, &vmax}, Ah, Al);
      layer256(e, Ah, Al, -1, EpiBackMask{m2, &vmax}, Bh, Bl);
      layer256(e, Bh, Bl, -1, EpiBackMask{m1, &vmax}, Ah, Al);
      f32x4 acc[1];
      small256<1>(e, Ah, Al, -1, acc);
#pragma unroll
      for (int d = 0; d < 3; ++d) gx[d] = bcast_g0(acc[0][d]) * s2;
    }

    // ---- prior reverse pass: J_s^T gx, same scaling
    float jt[3];
    {
      const float mx = fmaxf(fmaxf(__builtin_fabsf(gx[0]), __builtin_fabsf(gx[1])), __builtin_fabsf(gx[2]));
      const float s2 = pow2_of(mx), is2 = 1.0f / s2;
      const float u[4] = {gx[0] * is2, gx[1] * is2, gx[2] * is2, 0.0f};
      u32x4 bh, bl;
      vec_b(u, g, bh, bl);
      wide1(e, bh, bl, EpiBackD{D3, &vmax}, Ah, Al);
      layer256(e, Ah, Al, -1, EpiBackD{D2, &vmax}, Bh, Bl);
      layer256(e, Bh, Bl, -1, EpiBackL1{lds, lane, g, b1p, &vmax}, Ah, Al);
      f32x4 acc[1];
      small256<1>(e, Ah, Al, -1, acc);
#pragma unroll
      for (int d = 0; d < 3; ++d) jt[d] = bcast_g0(acc[0][d]) * s2;
    }

    // ---- EM predictor with the guidance step (dps_kernel's update)
    float xi[3];
    rng_normals<3>(rng, xi);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float gt = (gx[k] + var * jt[k]) / mw;
      const float xe = em_update(x[k], __fmul_rn(cf.g, sc[k]), xi[k], cf, p.delta, p.sqrt_delta);
      x[k] = xe - scale * gt;
    }
  }
  wait_vmcnt<0>();  // the prefetched chunks of a step that never ran land before the workgroup exits
  if constexpr (DDIAG == 0) x3::report_range((oor || range_bad(vmax)) && valid, p.err, lane);
  if (valid && g == 0) {
    float* dst = p.x_out + ((size_t)yi * p.n_chains + c_local) * 3;
#pragma unroll
    for (int d = 0; d < 3; ++d) dst[d] = x[d];
  }
}

// ---------------------------------------------------------------------------- fp32x3 Metropolis-Hastings
// The fused random-walk MH of dmip_surrogate.hip mh_kernel (generate_scatterometry_ground_truth.py:26-28, 59-62 with
// anneal_to_energy, models/SNF.py:250-275) with the surrogate's three streamed layers as three-term fp16 splits: the
// forward half of the DPS kernel's surrogate pass (layer 1 resident, S2 | S3 | Sout streamed, 17 chunks per step,
// the mid-chunk ring protocol). Same RNG consumption per chain (x0 ~ U[-1, 1]^3 unless given, then per step 3
// proposal normals and one acceptance uniform), same energy function and acceptance test; four waves of 16 chains.

// get_log_posterior's energy of one chain (dmip_surrogate.hip energy, the same operations): 0.5 sum log pref +
// 0.5 sum (y - f)^2 / pref + lam sum of the box violations, pref = (a f)^2 + b^2
__device__ __forceinline__ float mh_energy(const f32x4 (&f)[2], const float* y, const float (&x)[3], float a,
                                           float b2, float lam, int g) {
  float slog = 0.0f, ssq = 0.0f;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * t + 4 * g + r;
      if (row < kSurYdim) {
        const float fk = f[t][r];
        const float af = a * fk;
        const float pref = af * af + b2;
        const float res = y[row] - fk;
        slog += logf(pref);
        ssq += res * res / pref;
      }
    }
  slog += __shfl_xor(slog, 16, 64);
  slog += __shfl_xor(slog, 32, 64);
  ssq += __shfl_xor(ssq, 16, 64);
  ssq += __shfl_xor(ssq, 32, 64);
  float bd = 0.0f;
#pragma unroll
  for (int d = 0; d < 3; ++d) bd += fmaxf(x[d] - 1.0f, 0.0f) + fmaxf(-1.0f - x[d], 0.0f);
  return 0.5f * slog + 0.5f * ssq + lam * bd;
}

// the surrogate's forward pass at x (every lane of the chain holds x): output rows f (tiles 0, 1), range flag
__device__ __forceinline__ void sur_forward(Eng& e, const float (&x)[3], int g, int& vmax, f32x4 (&f)[2]) {
  u32x4 Ah[KQ], Al[KQ], Bh[KQ], Bl[KQ];
  uint32_t m2[2] = {0u, 0u}, m3[2] = {0u, 0u};
  layer1(e, SL1, SB, l1_b<3>(x, g), [&](const f32x4& z, int o) {
    float h[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) h[k] = relu_bits(z[k]);
    track4_pos(vmax, h);
    store_pair(h, o, Ah, Al);
  });
  layer256(e, Ah, Al, SB + W * 4, EpiSurFwd{m2, &vmax}, Bh, Bl);
  layer256(e, Bh, Bl, SB + 2 * W * 4, EpiSurFwd{m3, &vmax}, Ah, Al);
  small256<2>(e, Ah, Al, SB + 3 * W * 4, f);
}

// ---- the multi-tile forward engine of the MH kernel (MT tiles of 16 chains per wave; DPS keeps one tile because the
// prior's forward derivatives must live until its reverse pass). The hidden layers run k-major, as dmip_x3k.h's
// sampler does: chunk q of a layer is k-step q for all 16 output tiles, gathered by the LDS-DMA pieces straight from
// the DPS image's m-major chunks (a 1 KiB piece is one (tile, k-step, hi|lo) fragment, so the gather costs only the
// piece addresses). Every A fragment pair then feeds 3 MT MFMAs, a tile's 16 accumulators (64 registers) are the
// only per-tile state beside its input operands, and the input's k-step q dies after chunk q -- so MT tiles fit
// where the m-major order (input and output operands live together, 128 registers a tile) does not. The chunk's
// LDS reads and its share of the refill (the guide's 60-185 issue cycles per 1 KiB piece) are spread over MT times
// the matrix work. Same ring and mid-chunk barrier protocol as mid_units; the output layer's chunk stays m-major.
// compile-time loops over the tiles (the index is a constant in every body)
template <typename F, int... I>
__device__ __forceinline__ void sfor_impl(const F& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(const F& f) {
  sfor_impl(f, std::make_integer_sequence<int, N>{});
}
struct EngK {
  char* lds;
  const char* img;  // the surrogate's DPS image: S2 | S3 (8 m-major chunks each) | Sout | ...
  int c_issue, s_issue, s_read;
  int w, lane, g;
  static constexpr int NSTR = 2 * NCH + 1;  // 16 k-major hidden chunks + the output chunk per step
  // (global_load_lds here, not Eng's buffer form: with it the three-tile variant spills 184 B instead of 20 and runs
  // 5 % slower, profiles/r5_dma_buffer/)
  const char* dma_src;
  char* dma_dst;
  int dma_a, dma_b;  // piece Q's source: dma_src + (Q / 4) dma_a + ((Q / 2) % 2) dma_b + (Q % 2) KiB
  __device__ __forceinline__ void ring_target() {
    const int c = __builtin_amdgcn_readfirstlane(c_issue);
    // hidden chunk c (layer c / 8, k-step q = c % 8): wave w's pieces 8 w + Q are the fragments (tile 4 w + Q / 2,
    // k-step q, Q % 2) at m-major chunk 2 w + Q / 4, unit 8 ((Q / 2) % 2) + q; the output chunk is contiguous
    const bool hid = c < 2 * NCH;
    const char* src = hid ? img + (size_t)(c >> 3) * NCH * CHUNK + (c & 7) * 2048 + w * 2 * CHUNK
                          : img + (size_t)2 * NCH * CHUNK + w * PPW * 1024;
    dma_a = __builtin_amdgcn_readfirstlane(hid ? CHUNK : 4096);
    dma_b = __builtin_amdgcn_readfirstlane(hid ? CHUNK / 2 : 2048);
    const uint64_t addr = (uint64_t)src;
    const char* base = (const char*)(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(addr >> 32)) << 32) |
                                     (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)addr));
    asm volatile("" : "+s"(base));
    dma_src = base;
    dma_dst = lds + RING + __builtin_amdgcn_readfirstlane(s_issue) * CHUNK + w * PPW * 1024;
    c_issue = c + 1 == NSTR ? 0 : c + 1;
    s_issue = s_issue + 1 == R ? 0 : s_issue + 1;
  }
  template <int Q>
  __device__ __forceinline__ void ring_piece() const {
    glds16(dma_src + (Q / 4) * dma_a + ((Q / 2) % 2) * dma_b + (Q % 2) * 1024, dma_dst + Q * 1024, lane);
  }
  __device__ __forceinline__ void ring_issue() {
    ring_target();
    ring_piece<0>(), ring_piece<1>(), ring_piece<2>(), ring_piece<3>();
    ring_piece<4>(), ring_piece<5>(), ring_piece<6>(), ring_piece<7>();
  }
  __device__ __forceinline__ f32x4 bias4(int off_bytes, int tile) const {
    return *(const f32x4*)(lds + off_bytes + (16 * tile + 4 * g) * 4);
  }
  u32x4 nxt0, nxt1;  // the next chunk's unit 0 fragment pair
  u32x4 nxa0, nxa1;  // and its unit 1 pair (FPF = 2)
  __device__ __forceinline__ void start_mid() {
    for (int q = 0; q < R - 1; ++q) ring_issue();
    wait_vmcnt<(R - 2) * PPW>();
    lds_barrier();
    const lds_cptr b0 = (lds_cptr)(lds + RING + lane * 16);
    nxt0 = x3::lds_rd<0>(b0);
    nxt1 = x3::lds_rd<1024>(b0);
    if constexpr (FPF == 2) {
      nxa0 = x3::lds_rd<2048>(b0);
      nxa1 = x3::lds_rd<3072>(b0);
    }
    wait_next();
  }
  __device__ __forceinline__ void wait_next() {
    if constexpr (FPF == 2) x3::lds_wait2<0>(nxa0, nxa1);
    x3::lds_wait2<0>(nxt0, nxt1);
  }
  __device__ __forceinline__ lds_cptr take(lds_cptr& nb) {
    const lds_cptr b = (lds_cptr)(lds + RING + s_read * CHUNK + lane * 16);
    s_read = s_read + 1 == R ? 0 : s_read + 1;
    nb = (lds_cptr)(lds + RING + s_read * CHUNK + lane * 16);
    return b;
  }
};
static_assert(PPW == 8, "EngK::ring_issue");
template <int NU, int U, int Q = 0>
__device__ __forceinline__ void mid_pieces_k(const EngK& e) {
  if constexpr (Q < PPW) {
    constexpr int MIDU = NU / 2;
    if constexpr (MIDU + 1 + (Q * (NU - 1 - MIDU)) / PPW == U) e.template ring_piece<Q>();
    mid_pieces_k<NU, U, Q + 1>(e);
  }
}
// k-step q's B operand pair of tile m from the previous layer's pre-activations In[m][2q], In[m][2q + 1] (store_pair's
// dword order): relu, the running max (track4_pos's, over the pre-activations: a negative one sorts below the +0 its
// relu gives), the split
template <int MT, typename M>
__device__ __forceinline__ void act_pair(const f32x4 (&In)[MT][ST], int q, M m, int (&vmax)[MT], u32x4& nh,
                                         u32x4& nl) {
  float a[4], b[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) a[k] = relu_bits(In[m][2 * q][k]), b[k] = relu_bits(In[m][2 * q + 1][k]);
  int v = vmax[m];
  v = max(max(v, __float_as_int(In[m][2 * q][0])), __float_as_int(In[m][2 * q][1]));
  v = max(max(v, __float_as_int(In[m][2 * q][2])), __float_as_int(In[m][2 * q][3]));
  v = max(max(v, __float_as_int(In[m][2 * q + 1][0])), __float_as_int(In[m][2 * q + 1][1]));
  v = max(max(v, __float_as_int(In[m][2 * q + 1][2])), __float_as_int(In[m][2 * q + 1][3]));
  asm("" : "+v"(v));  // pinned (track4)
  vmax[m] = v;
  uint32_t h0, l0, h1, l1, h2, l2, h3, l3;
  x3::split_pair(a[0], a[1], h0, l0);
  x3::split_pair(a[2], a[3], h1, l1);
  x3::split_pair(b[0], b[1], h2, l2);
  x3::split_pair(b[2], b[3], h3, l3);
  nh = u32x4{h0, h1, h2, h3};
  nl = u32x4{l0, l1, l2, l3};
}
// one 16-unit chunk for MT tiles. OUT = false: k-major hidden chunk QK (unit U = output tile U, LDS fragment pair U);
// OUT = true: the output layer's m-major chunk walked k-step by k-step (unit U = tile U % 2 at k-step U / 2, LDS pair
// 8 (U % 2) + U / 2). (Hh, Hl): the current k-step's operands; the next k-step's are formed from In beside the MFMAs
// into (Nh, Nl) -- hidden: tile m's at unit m, taken over after the chunk; output: all at the k-step's second unit.
template <int MT, bool OUT, int QK, int NA, int U = 0>
__device__ __forceinline__ void units_k(EngK& e, lds_cptr base, lds_cptr nbase, const f32x4 (&In)[MT][ST],
                                        f32x4 (&Out)[MT][NA], u32x4 (&Hh)[MT], u32x4 (&Hl)[MT], u32x4 (&Nh)[MT],
                                        u32x4 (&Nl)[MT], u32x4 (&fa)[2][2], int (&vmax)[MT]) {
  constexpr int NU = 16;
  if constexpr (U < NU) {
    constexpr int MIDU = NU / 2;
    constexpr int PAIR = OUT ? 8 * ((U + 1) % 2) + (U + 1) / 2 : U + 1;  // the next unit's fragment pair
    if constexpr (U + 1 < NU) {
      fa[(U + 1) % 2][0] = x3::lds_rd<(2 * PAIR) * 1024>(base);
      fa[(U + 1) % 2][1] = x3::lds_rd<(2 * PAIR + 1) * 1024>(base);
    } else {
      e.nxt0 = x3::lds_rd<0>(nbase);
      e.nxt1 = x3::lds_rd<1024>(nbase);
    }
    x3::lds_wait2<2>(fa[U % 2][0], fa[U % 2][1]);
    constexpr int t = OUT ? U % 2 : U;
    sfor<MT>([&](auto m) {
      Out[m][t] = mfma16(fa[U % 2][0], Hl[m], Out[m][t]);
      Out[m][t] = mfma16(fa[U % 2][1], Hh[m], Out[m][t]);
      Out[m][t] = mfma16(fa[U % 2][0], Hh[m], Out[m][t]);
    });
    if constexpr (OUT) {
      if constexpr (U % 2 == 1 && U / 2 + 1 < KQ) {
        sfor<MT>([&](auto m) { act_pair(In, U / 2 + 1, m, vmax, Nh[m], Nl[m]); });
        sfor<MT>([&](auto m) { Hh[m] = Nh[m], Hl[m] = Nl[m]; });
      }
    } else if constexpr (QK + 1 < KQ && U < MT) {
      act_pair(In, QK + 1, std::integral_constant<int, U>{}, vmax, Nh[U], Nl[U]);
    }
    if constexpr (U == MIDU) {
      wait_vmcnt<PPW>();
      lds_barrier();
      e.ring_target();
    }
    if constexpr (U > MIDU) mid_pieces_k<NU, U>(e);
    units_k<MT, OUT, QK, NA, U + 1>(e, base, nbase, In, Out, Hh, Hl, Nh, Nl, fa, vmax);
  }
}
template <int MT, bool OUT, int QK, int NA>
__device__ __forceinline__ void chunk_k(EngK& e, const f32x4 (&In)[MT][ST], f32x4 (&Out)[MT][NA], u32x4 (&Hh)[MT],
                                        u32x4 (&Hl)[MT], int (&vmax)[MT]) {
  lds_cptr nb;
  const lds_cptr b = e.take(nb);
  u32x4 fa[2][2], Nh[MT], Nl[MT];
  fa[0][0] = e.nxt0, fa[0][1] = e.nxt1;
  units_k<MT, OUT, QK, NA>(e, b, nb, In, Out, Hh, Hl, Nh, Nl, fa, vmax);
  x3::lds_wait2<0>(e.nxt0, e.nxt1);
  if constexpr (!OUT && QK + 1 < KQ) sfor<MT>([&](auto m) { Hh[m] = Nh[m], Hl[m] = Nl[m]; });
}
// a 256 -> 256 hidden layer, k-major: In (the previous layer's pre-activations) -> Out (bias first)
template <int MT, int QK = 0>
__device__ __forceinline__ void hidden_k(EngK& e, const f32x4 (&In)[MT][ST], f32x4 (&Out)[MT][ST], u32x4 (&Hh)[MT],
                                         u32x4 (&Hl)[MT], int (&vmax)[MT]) {
  if constexpr (QK < KQ) {
    chunk_k<MT, false, QK, ST>(e, In, Out, Hh, Hl, vmax);
    hidden_k<MT, QK + 1>(e, In, Out, Hh, Hl, vmax);
  }
}

template <int MT, int O, typename Act>
__device__ __forceinline__ void l1_step_mt(lds_cptr la, lds_cptr lb, u32x4 (&fa)[3], u32x4 (&fb)[3],
                                           const u32x4 (&b)[MT], const Act& act) {
  if constexpr (O < ST) {
    if constexpr (O + 2 < ST) fa[(O + 2) % 3] = x3::lds_rd<(O + 2) * 512>(la), fb[(O + 2) % 3] = x3::lds_rd<(O + 2) * 64>(lb);
    x3::lds_wait2<(O + 2 < ST) ? 4 : ((O + 1 < ST) ? 2 : 0)>(fa[O % 3], fb[O % 3]);
    sfor<MT>([&](auto m) {
      act(mfma16(fa[O % 3], b[m], __builtin_bit_cast(f32x4, fb[O % 3])), std::integral_constant<int, O>{}, m);
    });
    l1_step_mt<MT, O + 1>(la, lb, fa, fb, b, act);
  }
}

// the surrogate's forward pass for MT tiles (tile m's chains hold x[m]): output rows f[m] (tiles 0, 1). The same
// products, in the same order per output, as mh_x3_kernel's one-tile m-major pass: the results are bit-identical.
template <int MT>
__device__ __forceinline__ void sur_forward_mt(EngK& e, const float (&x)[MT][3], int g, int (&vmax)[MT],
                                               f32x4 (&f)[MT][2]) {
  f32x4 P[MT][ST], Q[MT][ST];
  {  // layer 1, resident: one MFMA per tile and chain tile, pre-activations into P
    u32x4 b[MT];
    sfor<MT>([&](auto m) { b[m] = l1_b<3>(x[m], g); });
    const lds_cptr la = (lds_cptr)(e.lds + SL1 + (e.lane & 31) * 16);
    const lds_cptr lb = (lds_cptr)(e.lds + SB + 16 * e.g);
    u32x4 fa[3], fb[3];
    fa[0] = x3::lds_rd<0>(la), fb[0] = x3::lds_rd<0>(lb);
    fa[1] = x3::lds_rd<512>(la), fb[1] = x3::lds_rd<64>(lb);
    l1_step_mt<MT, 0>(la, lb, fa, fb, b, [&](const f32x4& z, auto o, auto m) { P[m][o] = z; });
  }
  u32x4 Hh[MT], Hl[MT];
  sfor<MT>([&](auto m) { act_pair(P, 0, m, vmax, Hh[m], Hl[m]); });
  sfor<ST>([&](auto t) {
    const f32x4 b = e.bias4(SB + W * 4, t);
    sfor<MT>([&](auto m) { Q[m][t] = b; });
  });
  hidden_k<MT>(e, P, Q, Hh, Hl, vmax);
  sfor<MT>([&](auto m) { act_pair(Q, 0, m, vmax, Hh[m], Hl[m]); });
  sfor<ST>([&](auto t) {
    const f32x4 b = e.bias4(SB + 2 * W * 4, t);
    sfor<MT>([&](auto m) { P[m][t] = b; });
  });
  hidden_k<MT>(e, Q, P, Hh, Hl, vmax);
  sfor<MT>([&](auto m) { act_pair(P, 0, m, vmax, Hh[m], Hl[m]); });
  sfor<2>([&](auto t) {
    const f32x4 b = e.bias4(SB + 3 * W * 4, t);
    sfor<MT>([&](auto m) { f[m][t] = b; });
  });
  chunk_k<MT, true, 0, 2>(e, P, f, Hh, Hl, vmax);
}

__global__ void __launch_bounds__(NW * 64, 1) mh_x3_kernel(MhX3Params p) {
  __shared__ __attribute__((aligned(16))) char lds[TOTAL];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, j = lane & 15;
  const int yi = blockIdx.y;
  const long long c_local = (long long)blockIdx.x * (NW * 16) + w * 16 + j;
  const bool valid = c_local < p.n_chains;
  const long long cc = valid ? c_local : 0;
  Eng e{lds, p.simg, 0, 0, 0, w, lane, g};
  e.nstream = kDpsX3SurFwdChunks;
  e.init_dma();
  {
    const uint4* s2 = (const uint4*)p.sl1;
    uint4* d2 = (uint4*)(lds + SL1);
    for (int i = threadIdx.x; i < ST * 32; i += NW * 64) d2[i] = s2[(i >> 5) * 64 + (i & 31)];
    float* sb = (float*)(lds + SB);
    for (int i = threadIdx.x; i < 3 * W + 32; i += NW * 64) sb[i] = p.sbias[i];
    float* yo = (float*)(lds + YO);
    for (int i = threadIdx.x; i < 32; i += NW * 64) yo[i] = i < kSurYdim ? p.y[(size_t)yi * kSurYdim + i] : 0.0f;
    __syncthreads();
    e.start_mid();
  }
  const float* ylds = (const float*)(lds + YO);
  Rng rng = rng_init(p.seed, (uint64_t)(p.chain_offset + c_local), (uint64_t)yi);
  float x[3];
  if (p.x_init) {
#pragma unroll
    for (int d = 0; d < 3; ++d) x[d] = p.x_init[((size_t)yi * p.n_chains + cc) * 3 + d];
  } else {  // torch.rand(n, 3) * 2 - 1 (generate_scatterometry_ground_truth.py:27)
#pragma unroll
    for (int d = 0; d < 3; ++d) x[d] = (float)(rng_next(rng) >> 8) * 0x1p-24f * 2.0f - 1.0f;
  }
  bool oor = false;
  int vmax = 0;  // track4's running max of the split values (float bits)
  for (int d = 0; d < 3; ++d) oor |= beyond_fp16(x[d]);
  f32x4 f[2];
  sur_forward(e, x, g, vmax, f);
  const float e0 = mh_energy(f, ylds, x, p.a, p.b2, p.lam, g);
  float e_cur = e0;
  for (int s = 0; s < p.num_steps; ++s) {
    float xi[3];
    rng_normals<3>(rng, xi);
    const float u = (float)(rng_next(rng) >> 8) * 0x1p-24f;
    float xp[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      xp[d] = x[d] + p.noise_std * xi[d];
      oor |= beyond_fp16(xp[d]);
    }
    sur_forward(e, xp, g, vmax, f);
    const float e_prop = mh_energy(f, ylds, xp, p.a, p.b2, p.lam, g);
    const bool acc = u < expf(-e_prop + e_cur);
#pragma unroll
    for (int d = 0; d < 3; ++d) x[d] = acc ? xp[d] : x[d];
    e_cur = acc ? e_prop : e_cur;
  }
  wait_vmcnt<0>();  // the prefetched chunks of a step that never ran land before the workgroup exits
  x3::report_range((oor || range_bad(vmax)) && valid, p.err, lane);
  if (valid && g == 0) {
    float* dst = p.x_out + ((size_t)yi * p.n_chains + c_local) * 3;
#pragma unroll
    for (int d = 0; d < 3; ++d) dst[d] = x[d];
    if (p.e_out) p.e_out[(size_t)yi * p.n_chains + c_local] = e_cur - e0;
  }
}

// mh_x3_kernel on the k-major multi-tile engine: 16 MT chains per wave, tile m's chain j at 64 MT block + 16 (MT w + m)
// + j; per chain the same RNG stream, proposals, energy and acceptance test as mh_x3_kernel
template <int MT>
__global__ void __launch_bounds__(NW * 64, 1) mh_x3_mt_kernel(MhX3Params p) {
  __shared__ __attribute__((aligned(16))) char lds[TOTAL];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, j = lane & 15;
  const int yi = blockIdx.y;
  long long c_local[MT];
  bool valid[MT];
  sfor<MT>([&](auto m) {
    c_local[m] = (long long)blockIdx.x * (NW * 16 * MT) + (MT * w + m) * 16 + j;
    valid[m] = c_local[m] < p.n_chains;
  });
  EngK e{lds, p.simg, 0, 0, 0, w, lane, g};
  {
    const uint4* s2 = (const uint4*)p.sl1;
    uint4* d2 = (uint4*)(lds + SL1);
    for (int i = threadIdx.x; i < ST * 32; i += NW * 64) d2[i] = s2[(i >> 5) * 64 + (i & 31)];
    float* sb = (float*)(lds + SB);
    for (int i = threadIdx.x; i < 3 * W + 32; i += NW * 64) sb[i] = p.sbias[i];
    float* yo = (float*)(lds + YO);
    for (int i = threadIdx.x; i < 32; i += NW * 64) yo[i] = i < kSurYdim ? p.y[(size_t)yi * kSurYdim + i] : 0.0f;
    __syncthreads();
    e.start_mid();
  }
  const float* ylds = (const float*)(lds + YO);
  Rng rng[MT];
  float x[MT][3];
  bool oor = false;
  sfor<MT>([&](auto m) {
    rng[m] = rng_init(p.seed, (uint64_t)(p.chain_offset + c_local[m]), (uint64_t)yi);
    const long long cc = valid[m] ? c_local[m] : 0;
    if (p.x_init) {
#pragma unroll
      for (int d = 0; d < 3; ++d) x[m][d] = p.x_init[((size_t)yi * p.n_chains + cc) * 3 + d];
    } else {  // torch.rand(n, 3) * 2 - 1 (generate_scatterometry_ground_truth.py:27)
#pragma unroll
      for (int d = 0; d < 3; ++d) x[m][d] = (float)(rng_next(rng[m]) >> 8) * 0x1p-24f * 2.0f - 1.0f;
    }
#pragma unroll
    for (int d = 0; d < 3; ++d) oor |= valid[m] && beyond_fp16(x[m][d]);
  });
  int vmax[MT];  // act_pair's running max (float bits)
  sfor<MT>([&](auto m) { vmax[m] = 0; });
  f32x4 f[MT][2];
  sur_forward_mt<MT>(e, x, g, vmax, f);
  float e0[MT], e_cur[MT];
  sfor<MT>([&](auto m) { e_cur[m] = e0[m] = mh_energy(f[m], ylds, x[m], p.a, p.b2, p.lam, g); });
  for (int s = 0; s < p.num_steps; ++s) {
    float xp[MT][3], u[MT];
    sfor<MT>([&](auto m) {
      float xi[3];
      rng_normals<3>(rng[m], xi);
      u[m] = (float)(rng_next(rng[m]) >> 8) * 0x1p-24f;
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        xp[m][d] = x[m][d] + p.noise_std * xi[d];
        oor |= valid[m] && beyond_fp16(xp[m][d]);
      }
    });
    sur_forward_mt<MT>(e, xp, g, vmax, f);
    sfor<MT>([&](auto m) {
      const float e_prop = mh_energy(f[m], ylds, xp[m], p.a, p.b2, p.lam, g);
      const bool acc = u[m] < expf(-e_prop + e_cur[m]);
#pragma unroll
      for (int d = 0; d < 3; ++d) x[m][d] = acc ? xp[m][d] : x[m][d];
      e_cur[m] = acc ? e_prop : e_cur[m];
    });
  }
  wait_vmcnt<0>();  // the prefetched chunks of a step that never ran land before the workgroup exits
  sfor<MT>([&](auto m) { oor |= valid[m] && range_bad(vmax[m]); });
  x3::report_range(oor, p.err, lane);
  sfor<MT>([&](auto m) {
    if (valid[m] && g == 0) {
      float* dst = p.x_out + ((size_t)yi * p.n_chains + c_local[m]) * 3;
#pragma unroll
      for (int d = 0; d < 3; ++d) dst[d] = x[m][d];
      if (p.e_out) p.e_out[(size_t)yi * p.n_chains + c_local[m]] = e_cur[m] - e0[m];
    }
  });
}

// the per-step coefficients: (tau, beta, g, 0), (mean_weight, var, 0, 0) -- the device functions every sampler uses
__global__ void dps_x3_coef_kernel(float4* coef, int S, float T, float bmin, float bdiff) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < S) {
    const StepCoef c = step_coef(i, S, T, bmin, bdiff);
    const float sd = vp_std(c.tau, bmin, bdiff);
    coef[2 * i] = make_float4(c.tau, c.beta, c.g, 0.0f);
    coef[2 * i + 1] = make_float4(vp_mean_weight(c.tau, bmin, bdiff), sd * sd, 0.0f, 0.0f);
  }
}

}  // namespace dx3

hipError_t launch_mh_x3(const MhX3Params& p, int n_y, hipStream_t st) {
  // DMIP_MH_MT (A/B knob): 1 = the one-tile m-major kernel, 2 or 3 tiles k-major -- all three bit-identical. Unset:
  // 2 or 3 by the workgroup rounds each leaves on the CUs (one workgroup per CU). Same box (profiles/r5_mh_mt/,
  // r5_mh_rows/): a 3-tile workgroup takes 1.45x a 2-tile one (100 rows x 30k: 359 vs 371 ms), so 3 tiles win once
  // their rounds are full -- 10 rows x 30k x 1000: MT = 2 204 ms (10 rounds) against 229 ms (7 rounds of 192-chain
  // workgroups); 1000 rows: MT = 3
  static const int forced = [] {
    const char* v = getenv("DMIP_MH_MT");
    const int n = v ? atoi(v) : 0;
    return n >= 1 && n <= 3 ? n : 0;
  }();
  int mt = forced;
  if (!mt) {
    int n_cu = 256;
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, stream_device(st));
    if (n_cu < 1) n_cu = 256;
    auto rounds = [&](int t) {
      const long long wg = (p.n_chains + dx3::NW * 16 * t - 1) / (dx3::NW * 16 * t) * n_y;
      return (double)((wg + n_cu - 1) / n_cu);
    };
    mt = rounds(3) * 1.45 < rounds(2) ? 3 : 2;
  }
  const long long per_wg = dx3::NW * 16 * mt;
  const dim3 grid((unsigned)((p.n_chains + per_wg - 1) / per_wg), (unsigned)n_y), block(dx3::NW * 64);
  if (mt == 1)
    hipLaunchKernelGGL(dx3::mh_x3_kernel, grid, block, 0, st, p);
  else if (mt == 2)
    hipLaunchKernelGGL(dx3::mh_x3_mt_kernel<2>, grid, block, 0, st, p);
  else
    hipLaunchKernelGGL(dx3::mh_x3_mt_kernel<3>, grid, block, 0, st, p);
  return hipGetLastError();
}

hipError_t launch_dps_x3(const DpsX3Params& p, int n_y, hipStream_t st) {
  const long long per_wg = dx3::NW * 16;
  const int S = p.num_steps > 0 ? p.num_steps : 1;
  // one launch-scoped allocation: the stream-ordered image (the kernel's one buffer resource), then the step table
  constexpr size_t kImg = (size_t)dx3::NSTREAM * dx3::CHUNK;
  char* buf = nullptr;
  hipError_t e = hipMallocAsync((void**)&buf, kImg + (size_t)2 * S * sizeof(float4), st);
  if (e != hipSuccess) return e;
  float4* coef = (float4*)(buf + kImg);
  constexpr size_t C = dx3::CHUNK;
  if ((e = hipMemcpyAsync(buf, p.pimg, dx3::NPF * C, hipMemcpyDeviceToDevice, st)) != hipSuccess ||
      (e = hipMemcpyAsync(buf + dx3::NPF * C, p.simg, dx3::NS * C, hipMemcpyDeviceToDevice, st)) != hipSuccess ||
      (e = hipMemcpyAsync(buf + (dx3::NPF + dx3::NS) * C, p.pimg + dx3::NPF * C, dx3::NPB * C, hipMemcpyDeviceToDevice,
                          st)) != hipSuccess) {
    (void)hipFreeAsync(buf, st);
    return e;
  }
  hipLaunchKernelGGL(dx3::dps_x3_coef_kernel, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, st, coef, S, p.T, p.bmin,
                     p.bdiff);
  DpsX3Params q = p;
  q.img = buf;
  q.coef = (const float*)coef;
  const dim3 grid((unsigned)((p.n_chains + per_wg - 1) / per_wg), (unsigned)n_y), block(dx3::NW * 64);
  hipLaunchKernelGGL(dx3::dps_x3_kernel, grid, block, 0, st, q);
  e = hipGetLastError();
  (void)hipFreeAsync(buf, st);
  return e;
}

}  // namespace dmip
