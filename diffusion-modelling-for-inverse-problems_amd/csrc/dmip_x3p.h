// fp32-accurate CDE sampler on 32x32 tiles with two chain tiles per wave in ping-pong: DMIP_PREC_F32X3 at the
// headline shape (scatterometry and linear CDE, hidden_layers [256]*3, BASELINE configs[1]).
//
// Same arithmetic as dmip_x3.h / dmip_x3k.h for layer 1 and the two W x W layers (every product
// W_hi h_hi + W_hi h_lo + W_lo h_hi, fp32 accumulation, r-form tanh by exp2 + rcp), the output layer in
// exact f32 on the vector ALUs. What bounds the 16x16 k-major engine (dmip_x3k.h) is vector issue beside
// its MFMAs -- a v_mfma_f32_16x16x32_f16 holds the SIMD's issue for 8 of its 16 cycles -- and the VALU-only
// phases every chain tile of a wave reaches at the same moment (output-layer activation, EM, layer 1:
// ~20 % of a step with the matrix pipe idle; profiles/r3_x3k_stamps). Here:
//   * v_mfma_f32_32x32x16_f16 (holds issue for 8 of 32 cycles: twice the room for the activations);
//   * one wave per SIMD holds TWO 32-chain tiles A and B (64 chains per wave, as many per streamed weight
//     byte as the 16x16 engine's 48 and more), kept in 256 + ~130 registers by never storing a whole
//     layer's pre-activations twice:
//       - layer 1 is fused into hidden layer 1, which streams k-major: chunk q = layer-1 output tile q
//         (32 units = hidden layer 1's k-steps 2q, 2q+1) for all 8 output tiles; layer-1 tile q of a
//         chain tile is one MFMA + its double tanh, computed just before the chunk that consumes it;
//       - hidden layer 2 streams output-major: chunk c = its output tile c over all 16 k-steps, so each
//         output tile is complete one chunk at a time and its activation feeds the output layer (f32
//         FMAs) at once -- hidden layer 2's pre-activations are never stored;
//   * ping-pong: every 32 KiB chunk is consumed first by tile A's MFMAs (8 units of 6 MFMAs), then by
//     tile B's. The vector work of one tile (its layer-1 tiles, hidden-layer-1 activation, output layer,
//     EM update, RNG) is placed beside the OTHER tile's MFMAs, so no phase of a step leaves the matrix
//     pipe idle while the vector ALUs catch up;
//   * the weight ring is dmip_x3k.h's: 16 chunks per step on 4 static slots (chunk k in slot k % 4), the
//     barrier in the middle of a chunk, LDS-DMA pieces spread over the units after it; every LDS read of
//     the hot loop is an explicit ds_read_b128 one unit ahead with a counted lgkmcnt wait.
// Registers (one wave, 512; the compiler selects the AGPR form for every builtin MFMA of a kernel this size):
// the layer state -- hidden layer 1's accumulators Q, converted in place into hidden layer 2's (hi, lo) operands
// X -- fills the 256 AGPRs in hidden layer 1; in hidden layer 2, 224 registers of X (written by v_accvgpr_write)
// and the two tiles' accumulators. Both layers' accumulators start from a bias MFMA (bias hi/mid/lo fragment
// against a ones column) instead of a copy into AGPRs. Layer 1's MFMA is inline asm in the VGPR form (its
// accumulator would not fit beside Q), its wait states padded inside the string (cdna_hip_programming.md §5.7
// item 2: 2 states after a VALU write before the MFMA reads it, 18 after its 16-pass write before a VALU reads).
// Chain state, RNG, schedule, EM update, snapshots and hand-over follow the other engines (dmip_device.h):
// the same noise chain by chain.
#pragma once
#include "dmip_x3.h"

namespace dmip {
namespace x3p {

using x3::f32x4;
using x3::lds_cptr;

__device__ __forceinline__ f32x16 mma(const u32x4& a, const u32x4& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                0);
}

constexpr int W = 256, OT = 8, KS = 16;  // [256]*3: 8 32-unit tiles, 16 k-steps of 16
constexpr int NCH = 16;                  // ring chunks per step: hidden layer 1 (k-major) then 2 (output-major)
constexpr int CHUNK = 32768;             // 16 fragment pairs (hi, lo) x 1 KiB
constexpr int R = 4;                     // ring slots
constexpr int NWV = 4;                   // one wave per SIMD
constexpr int PPW = CHUNK / 1024 / NWV;  // LDS-DMA pieces per wave per chunk
constexpr int JC = 64;                   // chains per wave (two 32-chain tiles)
static_assert(NCH % R == 0 && PPW == 8, "static ring; units 5..12 of a chunk issue its 8 pieces");

struct PLay {
  // [8 layer-1 tiles][64 lanes][8 fp16], then hidden layers 1 and 2's biases as an A fragment per output tile
  // (k-slots 0..2 of lane half 0: their hi, mid and lo parts; against a ones column they initialise the AGPR
  // accumulators)
  static constexpr int L1 = 0, L1_BYTES = 3 * OT * 1024;
  static constexpr int OW = L1 + L1_BYTES, OW_BYTES = OT * 2 * 256;  // f32 [c][lane half][row < 4][4 groups][4]
  static constexpr int BIAS = OW + OW_BYTES;                      // floats: layer 1's per-y bias
  static constexpr int BIAS_BYTES = W * 4;
  static constexpr int RING = BIAS + BIAS_BYTES;
  static constexpr int TOTAL = RING + R * CHUNK;
};
static_assert(PLay::RING % 16 == 0 && PLay::TOTAL <= 160 * 1024, "LDS budget");
constexpr int OW_IMAGE_FLOATS = OT * 2 * 64 + 16;  // host image: the f32 output rows, then the output init[16]

// ---------------------------------------------------------------------------------- the schedule
// A step is 16 chunks x 16 units; unit U of chunk K: half h = U / 8 (0: tile A's MFMAs, 1: tile B's), pu =
// U % 8 (fragment pairs 2 pu, 2 pu + 1 of the chunk). The vector work ("filler") placed in each unit:
//   L1 MFMA:  (K <= 6, pu 7) the MFMA tile's layer-1 tile K + 1, whose activation pairs run in the next half;
//             (15, B pu 5) tile A's layer-1 tile 0 of the next step; (0, A pu 5) tile B's of this step
//   L1 pairs: activation pair pu of the other tile's layer-1 tile: (K, A) for tile B's tile K (K >= 1),
//             (K, B) for tile A's tile K + 1 (K <= 6); after the tails: (15, B) / (0, A) pu 6 and 7, four each
//   Q act:    hidden layer 1's output tile o activated into hidden layer 2's (hi, lo) operands once it is
//             complete and before hidden layer 2 needs it (table qact)
//   H2 out:   hidden layer 2's output tile c of a chain tile (complete after its half of chunk 8 + c) through
//             the output layer: four parts of 4 units, in the other half's pu 0..3 (tile B's c = 7 in (0, A))
//   xi:       the EM step's normals, drawn in slack: tile A in (12, B) pu 6, tile B in (12, A) pu 6
//   tail:     output rows reduced over the lane halves, EM update, layer-1 operand: tile A in (15, B) pu 4,
//             tile B (the previous step's) in (0, A) pu 4
constexpr int l1m_tile(int K, int U) {  // L1 MFMA in unit (K, U): chain tile, or -1
  if (K <= 6 && U % 8 == 7) return U / 8;
  if (K == 15 && U == 13) return 0;
  if (K == 0 && U == 5) return 1;
  return -1;
}
constexpr int l1m_q(int K, int U) { return (K == 15 || (K == 0 && U == 5)) ? 0 : K + 1; }
// L1 activation pairs in unit (K, U): first pair, count (0: none); the tile is the other half's
constexpr int l1p_first(int K, int U) {
  if ((K == 15 && U >= 14) || (K == 0 && U >= 6 && U < 8)) return 4 * (U % 8 - 6);
  return U % 8;
}
constexpr int l1p_count(int K, int U) {
  if ((K == 15 && U >= 14) || (K == 0 && U >= 6 && U < 8)) return 4;
  if (K == 15 || (K == 0 && U < 8)) return 0;
  if (U < 8) return (K >= 1 && K <= 7) ? 1 : 0;  // tile B's layer-1 tile K
  return K <= 6 ? 1 : 0;                         // tile A's layer-1 tile K + 1
}
constexpr int l1p_tile(int K, int U) { return (K == 15) ? 0 : (U < 8 ? 1 : 0); }
// hidden-layer-1 output tile activation in unit (K, U): chain tile * 8 + o, or -1. Tile A's tile o is complete
// after unit (7, o), tile B's after (7, 8 + o); A's are needed from (8, o), B's from (8, 8 + o). The region
// carries more vector work than its MFMAs cover (the one burst of a step): spread so that no unit after it idles.
constexpr int qact(int K, int U) {
  if (K == 7 && U >= 1 && U <= 5) return U - 1;        // A 0..4
  if (K == 7 && U >= 8 && U <= 10) return U - 3;       // A 5..7
  if (K == 7 && U >= 11) return 8 + (U - 11);          // B 0..4
  if (K == 8 && U <= 1) return 8 + 5 + U;              // B 5, 6
  if (K == 8 && U == 12) return 8 + 7;                 // B 7
  return -1;
}
// hidden layer 2 output part in unit (K, U): chain tile * 64 + c * 4 + part, or -1
constexpr int h2o(int K, int U) {
  if (K >= 8 && U >= 8 && U < 12) return 0 * 64 + (K - 8) * 4 + (U - 8);
  if (K >= 9 && U < 4) return 1 * 64 + (K - 9) * 4 + U;
  if (K == 0 && U < 4) return 1 * 64 + 7 * 4 + U;
  return -1;
}

typedef __attribute__((address_space(3))) void lds_void;

// Diagnostic phase stamps (scripts/x3p_stamps.py): only a library built with -DDMIP_X3P_DIAG (make diag,
// never the product build) carries them; its sampler writes per-wave cycle counts (one per ring chunk, the
// barrier waits, the step count) into the snapshot buffer instead of snapshots.
#ifdef DMIP_X3P_DIAG
constexpr bool kDiag = true;
#else
constexpr bool kDiag = false;
#endif
__device__ __forceinline__ uint64_t stamp() {
  uint64_t t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
  return t;
}

// values read by explicit ds_read_b128 in one unit for the next
struct Pre {
  u32x4 f[4];    // fragment pairs 2 pu (hi, lo), 2 pu + 1 (hi, lo)
  u32x4 hb;      // the accumulator init's bias fragment (hidden layer 1: chunk 0; hidden layer 2: a half's first unit)
  u32x4 l1f;     // layer-1 fragment of an L1 MFMA
  f32x16 l1b;    // its per-y bias
  f32x4 ow[4];   // output rows (4 units) of an H2 out part
};

template <int OFF>
__device__ __forceinline__ u32x4 rd(lds_cptr p) {
  return x3::lds_rd<OFF>(p);
}
// a VGPR dword into an AGPR (hidden layer 2's operands)
__device__ __forceinline__ uint32_t to_agpr(uint32_t v) {
  uint32_t a;
  asm("v_accvgpr_write_b32 %0, %1" : "=a"(a) : "v"(v));
  return a;
}
// VGPR-form MFMAs. Layer 1: P = A . b + c, the operand b just written by the vector ALUs (2 states before), P read
// by them in the next unit (18 states after).
__device__ __forceinline__ f32x16 mma_l1(const u32x4& a, const u32x4& b, const f32x16& c) {
  f32x16 d;
  asm volatile(
      "s_nop 1\n\t"
      "v_mfma_f32_32x32x16_f16 %0, %1, %2, %3\n\t"
      "s_nop 7\n\ts_nop 7\n\ts_nop 1"
      : "=&v"(d)
      : "v"(a), "v"(b), "v"(c));
  return d;
}

template <int OFF>
__device__ __forceinline__ f32x4 rdf(lds_cptr p) {
  return __builtin_bit_cast(f32x4, x3::lds_rd<OFF>(p));
}
template <int N>
__device__ __forceinline__ void wait_frags(Pre& c) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(c.f[0]), "+v"(c.f[1]), "+v"(c.f[2]), "+v"(c.f[3]) : "i"(N));
}
template <typename T>
__device__ __forceinline__ void touch(T& v) {
  asm volatile("" : "+v"(v));
}
template <typename T>
__device__ __forceinline__ void touch_a(T& v) {
  asm volatile("" : "+a"(v));
}

// the unit's vector work interleaved with its N MFMAs: each MFMA followed by up to 5 vector instructions (one wave
// per SIMD hides about 5 single-issue instructions per 32x32x16 gap, MI355X_MICROARCH.md constants table)
template <int N>
__device__ __forceinline__ void interleave() {
  if constexpr (N > 0) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
    interleave<N - 1>();
  }
}

// layer-1 operand dword d of k-half e from a pair of activated values
__device__ __forceinline__ void act2_l1(float z0, float z1, uint32_t& h, uint32_t& l) {
  x3::split_pair(x3::x3_act_r2(z0), x3::x3_act_r2(z1), h, l);
}
__device__ __forceinline__ void act2(float z0, float z1, uint32_t& h, uint32_t& l) {
  x3::split_pair(x3::x3_act_r(z0), x3::x3_act_r(z1), h, l);
}

template <int D, bool NOISE>
struct PWave {
  // LDS lane bases: ring slots 0-1 and 2-3, layer-1 image, biases, output rows
  lds_cptr rb0, rb2, l1b, bb, owb;
  char* lds;
  __amdgpu_buffer_rsrc_t rs;
  unsigned voff;
  int w, h;
  // chain state (both lane halves hold a chain's copy)
  float x[2][D];
  Rng rng[2];
  float xi[2][D];
  u32x4 b1[2];           // layer-1 B operand (x, tau) per chain tile
  u32x4 ones;            // fp16 1.0 in k-slots 0..2 of every chain (lane half 0): the bias hi, mid, lo
  u32x4 Hh[2][2], Hl[2][2];  // hidden-layer-1 B operands of the current chunk (k-steps 2q, 2q + 1)
  f32x16 P[2];           // layer-1 tile being activated
  f32x16 Q[2][OT];       // hidden layer 1 accumulators
  u32x4 Xh[2][KS], Xl[2][KS];  // hidden layer 2 B operands (activated hidden layer 1)
  f32x16 acc[2];         // hidden layer 2 output tile
  float aP[2][D];        // output rows, partial over this lane half's units
  float oinit[D];
  // step coefficients: tile A completes step `cur` in chunk 15, tile B completes step `prev` in chunk 0
  StepCoef cf_cur, cf_prev;
  float tau_next;
  float delta, sqrt_delta;
  bool first;  // first step of a segment: tile B has no previous step to complete
  bool oor = false;  // a layer-1 input out of the split's range (x3::report_range)
  bool live[2] = {false, false};  // the segment's tiles hold returned chains (not idle, not padded lanes)
  uint64_t ph[17], t_last;  // kDiag: cycles per ring chunk, barrier waits

  // ------------------------------------------------------------------ ring (dmip_x3k.h protocol)
  template <int C, int S, int Qp>
  __device__ __forceinline__ void issue_piece() const {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(lds + PLay::RING + S * CHUNK + (w * PPW + Qp) * 1024), 16,
                                             voff, C * CHUNK + Qp * 1024, 0, 0);
  }
  template <int C, int S, int Qp = 0>
  __device__ __forceinline__ void issue() const {
    if constexpr (Qp < PPW) {
      issue_piece<C, S, Qp>();
      issue<C, S, Qp + 1>();
    }
  }
  __device__ __forceinline__ void barrier() const {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  // chunks 0..2 in flight, chunk 0 landed for every wave
  __device__ __forceinline__ void ring_start() const {
    issue<0, 0>();
    issue<1, 1>();
    issue<2, 2>();
    wait_vmcnt<2 * PPW>();
    barrier();
  }
  // B(K) in the middle of chunk K - 1: this wave's pieces of chunk K have landed, then the workgroup barrier
  __device__ __forceinline__ void sync_mid() {
    wait_vmcnt<PPW>();
    uint64_t t0 = 0;
    if constexpr (kDiag) t0 = stamp();
    barrier();
    if constexpr (kDiag) ph[16] += stamp() - t0;
  }

  // ------------------------------------------------------------------ reads for a unit
  // unit 32 O + 8 q + 4 h + k of layer LI (0: layer 1 per y, 2: hidden layer 2)
  template <int LI, int O>
  __device__ __forceinline__ f32x16 rd_bias16() const {
    const f32x4 a = rdf<(LI * W + 32 * O + 0) * 4>(bb);
    const f32x4 b = rdf<(LI * W + 32 * O + 8) * 4>(bb);
    const f32x4 c = rdf<(LI * W + 32 * O + 16) * 4>(bb);
    const f32x4 d = rdf<(LI * W + 32 * O + 24) * 4>(bb);
    return f32x16{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3], c[0], c[1], c[2], c[3], d[0], d[1], d[2], d[3]};
  }
  // every value unit (K, U) uses, read by the unit before it; returns the number of reads
  template <int K, int U>
  __device__ __forceinline__ int reads(Pre& n) const {
    constexpr int s = K % R, p0 = 2 * (U % 8);
    constexpr int off = (s & 1) * CHUNK + p0 * 2048;
    const lds_cptr rb = s < 2 ? rb0 : rb2;
    n.f[0] = rd<off>(rb);
    n.f[1] = rd<off + 1024>(rb);
    n.f[2] = rd<off + 2048>(rb);
    n.f[3] = rd<off + 3072>(rb);
    int cnt = 4;
    if constexpr (K == 0) {
      n.hb = rd<(OT + U % 8) * 1024>(l1b);
      cnt += 1;
    }
    if constexpr (K >= 8 && U % 8 == 0) {
      n.hb = rd<(2 * OT + K - 8) * 1024>(l1b);
      cnt += 1;
    }
    if constexpr (l1m_tile(K, U) >= 0) {
      constexpr int q = l1m_q(K, U);
      n.l1f = rd<q * 1024>(l1b);
      n.l1b = rd_bias16<0, q>();
      cnt += 5;
    }
    if constexpr (h2o(K, U) >= 0) {
      constexpr int c = (h2o(K, U) % 64) / 4, part = h2o(K, U) % 4;
#pragma unroll
      for (int k = 0; k < D; ++k) {
        // (unrolled: k is a constant)
        if (k == 0) n.ow[0] = rdf<c * 512 + 0 * 64 + part * 16>(owb);
        if (k == 1) n.ow[1] = rdf<c * 512 + 1 * 64 + part * 16>(owb);
        if (k == 2) n.ow[2] = rdf<c * 512 + 2 * 64 + part * 16>(owb);
        if (k == 3) n.ow[3] = rdf<c * 512 + 3 * 64 + part * 16>(owb);
      }
      cnt += D;
    }
    return cnt;
  }
  template <int K, int U>
  static constexpr int n_reads() {
    return 4 + (K == 0 ? 1 : 0) + (K >= 8 && U % 8 == 0 ? 1 : 0) + (l1m_tile(K, U) >= 0 ? 5 : 0) +
           (h2o(K, U) >= 0 ? D : 0);
  }
  template <int K, int U>
  __device__ __forceinline__ void wait_cur(Pre& c) const {
    constexpr int KN = U == 15 ? (K + 1) % NCH : K, UN = (U + 1) % 16;
    wait_frags<n_reads<KN, UN>()>(c);
    if constexpr (K == 0 || (K >= 8 && U % 8 == 0)) touch(c.hb);
    if constexpr (l1m_tile(K, U) >= 0) touch(c.l1f), touch(c.l1b);
    if constexpr (h2o(K, U) >= 0) {
#pragma unroll
      for (int k = 0; k < D; ++k) touch(c.ow[k]);
    }
  }

  // ------------------------------------------------------------------ vector work
  template <int T>
  __device__ __forceinline__ void l1_pair(int d) {
    const int e = d >> 2, dd = d & 3;
    uint32_t hh, ll;
    act2_l1(P[T][8 * e + 2 * dd], P[T][8 * e + 2 * dd + 1], hh, ll);
    Hh[T][e][dd] = hh;
    Hl[T][e][dd] = ll;
    touch(Hh[T][e]), touch(Hl[T][e]);  // done in this unit, not sunk towards its use
  }
  template <int T, int O>
  __device__ __forceinline__ void q_act() {
    float r[16];  // the tile's 16 activations stage by stage (see h2_out)
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = __builtin_amdgcn_exp2f(Q[T][O][i]);
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = 1.0f + r[i];
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = __builtin_amdgcn_rcpf(r[i]);
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int dd = 0; dd < 4; ++dd) {
        uint32_t hh, ll;
        x3::split_pair(r[8 * e + 2 * dd], r[8 * e + 2 * dd + 1], hh, ll);
        // 224 of the 256 operand registers in AGPRs, beside hidden layer 2's two accumulators; the last
        // two k-steps of tile B (32 registers) in VGPRs
        if constexpr (T == 1 && O == OT - 1) {
          Xh[T][2 * O + e][dd] = hh;
          Xl[T][2 * O + e][dd] = ll;
        } else {
          Xh[T][2 * O + e][dd] = to_agpr(hh);
          Xl[T][2 * O + e][dd] = to_agpr(ll);
        }
      }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      if constexpr (T == 1 && O == OT - 1) touch(Xh[T][2 * O + e]), touch(Xl[T][2 * O + e]);
      else touch_a(Xh[T][2 * O + e]), touch_a(Xl[T][2 * O + e]);
    }
  }
  // activate registers 4 part .. 4 part + 3 of hidden layer 2's output tile and add their output-row terms
  template <int T, int PART>
  __device__ __forceinline__ void h2_out(const f32x4 (&ow)[4]) {
    // the four r-form activations stage by stage (exp2, add, rcp), so no instruction waits on the one before it
    // (a transcendental's result read by the next instruction costs a wait state)
    float r[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) r[m] = __builtin_amdgcn_exp2f(acc[T][4 * PART + m]);
#pragma unroll
    for (int m = 0; m < 4; ++m) r[m] = 1.0f + r[m];
#pragma unroll
    for (int m = 0; m < 4; ++m) r[m] = __builtin_amdgcn_rcpf(r[m]);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
#pragma unroll
      for (int k = 0; k < D; ++k) aP[T][k] = __builtin_fmaf(ow[k][m], r[m], aP[T][k]);
    }
#pragma unroll
    for (int k = 0; k < D; ++k) touch(aP[T][k]);
  }
  template <int T>
  __device__ __forceinline__ void draw_xi(const float* noise, size_t nidx) {
    if constexpr (NOISE) {
#pragma unroll
      for (int k = 0; k < D; ++k) xi[T][k] = noise[nidx + k];
    } else {
      rng_normals<D>(rng[T], xi[T]);
    }
#pragma unroll
    for (int k = 0; k < D; ++k) touch(xi[T][k]);
  }
  // output rows over both lane halves, the EM update of the step with coefficients cf, the next layer-1
  // operand at tau_n; KEEP = false discards the update (tile B before its first step)
  template <int T>
  __device__ __forceinline__ void tail(const StepCoef& cf, float tau_n, bool keep) {
    float v[D + 1];
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(aP[T][k]), __float_as_uint(aP[T][k]), false,
                                                       false);
      const float a = oinit[k] + (__uint_as_float(sw[0]) + __uint_as_float(sw[1]));  // (half 0 + half 1)
      const float xn = em_update(x[T][k], a, xi[T][k], cf, delta, sqrt_delta);
      x[T][k] = keep ? xn : x[T][k];
      aP[T][k] = 0.0f;
      v[k] = x[T][k];
    }
    v[D] = tau_n;
    u32x4 b[1];
    x3::l1_operand<D + 1, 1>(v, h, b);
    oor |= live[T] && x3::out_of_range(v);
    b1[T] = b[0];
    touch(b1[T]);
#pragma unroll
    for (int k = 0; k < D; ++k) touch(x[T][k]);
  }

  // ------------------------------------------------------------------ one unit
  template <int K, int U>
  __device__ __forceinline__ void unit(Pre& cur, const float* noise, size_t nidxA, size_t nidxB) {
    constexpr int hf = U / 8, pu = U % 8;
    constexpr int KN = U == 15 ? (K + 1) % NCH : K, UN = (U + 1) % 16;
    static_assert(n_reads<KN, UN>() <= 15, "lgkmcnt counts to 15");
    // a unit is its own scheduling region: its vector work is interleaved with ITS MFMAs
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (kDiag && U == 0) {
      const uint64_t t = stamp();
      ph[(K + NCH - 1) % NCH] += t - t_last;
      t_last = t;
    }
    Pre nxt;
    (void)reads<KN, UN>(nxt);
    wait_cur<K, U>(cur);
    // ---- MFMAs of chain tile hf
    if constexpr (K < 8) {
      f32x16 c = Q[hf][pu];
      if constexpr (K == 0) c = mma(cur.hb, ones, f32x16{});  // bias hi + lo, exact in f32
      c = mma(cur.f[0], Hl[hf][0], c);
      c = mma(cur.f[1], Hh[hf][0], c);
      c = mma(cur.f[0], Hh[hf][0], c);
      c = mma(cur.f[2], Hl[hf][1], c);
      c = mma(cur.f[3], Hh[hf][1], c);
      c = mma(cur.f[2], Hh[hf][1], c);
      Q[hf][pu] = c;
    } else {
      f32x16 a = acc[hf];
      if constexpr (pu == 0) a = mma(cur.hb, ones, f32x16{});  // bias hi + mid + lo
      a = mma(cur.f[0], Xl[hf][2 * pu], a);
      a = mma(cur.f[1], Xh[hf][2 * pu], a);
      a = mma(cur.f[0], Xh[hf][2 * pu], a);
      a = mma(cur.f[2], Xl[hf][2 * pu + 1], a);
      a = mma(cur.f[3], Xh[hf][2 * pu + 1], a);
      a = mma(cur.f[2], Xh[hf][2 * pu + 1], a);
      acc[hf] = a;
    }
    // ---- vector work
    if constexpr (h2o(K, U) >= 0) {
      constexpr int T = h2o(K, U) / 64, part = h2o(K, U) % 4;
      h2_out<T, part>(cur.ow);
    }
    if constexpr (qact(K, U) >= 0) q_act<qact(K, U) / 8, qact(K, U) % 8>();
    if constexpr (K == 12 && U == 14) draw_xi<0>(noise, nidxA);
    if constexpr (K == 12 && U == 6) draw_xi<1>(noise, nidxB);
    if constexpr (K == 15 && U == 12) tail<0>(cf_cur, tau_next, true);
    if constexpr (K == 0 && U == 4) tail<1>(cf_prev, cf_cur.tau, !first);
    if constexpr (l1m_tile(K, U) >= 0) P[l1m_tile(K, U)] = mma_l1(cur.l1f, b1[l1m_tile(K, U)], cur.l1b);
    if constexpr (l1p_count(K, U) > 0) {
      constexpr int T = l1p_tile(K, U);
#pragma unroll
      for (int i = 0; i < l1p_count(K, U); ++i) l1_pair<T>(l1p_first(K, U) + i);
    }
    interleave<((K == 0 || (K >= 8 && pu == 0)) ? 7 : 6)>();
    // ---- ring
    if constexpr (U == 4) sync_mid();
    if constexpr (U >= 5 && U < 5 + PPW) issue_piece<(K + R - 1) % NCH, (K + R - 1) % R, U - 5>();
    cur = nxt;
  }

  template <int K, int U>
  __device__ __forceinline__ void run(Pre& cur, const float* noise, size_t nidxA, size_t nidxB) {
    if constexpr (K < NCH) {
      unit<K, U>(cur, noise, nidxA, nidxB);
      if constexpr (U + 1 < 16) run<K, U + 1>(cur, noise, nidxA, nidxB);
      else run<K + 1, 0>(cur, noise, nidxA, nidxB);
    }
  }

  // prologue of a segment: tile A's layer-1 tile 0 (the steady state computes it in chunk 15 of the step before)
  __device__ __forceinline__ void prologue_a(float tau) {
    float v[D + 1];
#pragma unroll
    for (int k = 0; k < D; ++k) v[k] = x[0][k];
    v[D] = tau;
    u32x4 b[1];
    x3::l1_operand<D + 1, 1>(v, h, b);
    oor |= live[0] && x3::out_of_range(v);
    b1[0] = b[0];
    typedef __attribute__((address_space(3))) const u32x4* lds_u4;
    typedef __attribute__((address_space(3))) const float* lds_f;
    const u32x4 f = *(lds_u4)l1b;
    const lds_f bp = (lds_f)bb;
    f32x16 bias;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int k = 0; k < 4; ++k) bias[4 * q + k] = bp[8 * q + k];
    P[0] = mma_l1(f, b1[0], bias);
#pragma unroll
    for (int d = 0; d < 8; ++d) l1_pair<0>(d);
  }
  // epilogue of a segment: tile B's last step (hidden layer 2 tile 7 through the output layer, the EM update)
  __device__ __forceinline__ void epilogue_b(const StepCoef& cf) {
    typedef __attribute__((address_space(3))) const f32x4* lds_f4;
    const lds_f4 o = (lds_f4)owb;
#pragma unroll
    for (int part = 0; part < 4; ++part) {
      f32x4 ow[4];
#pragma unroll
      for (int k = 0; k < D; ++k) ow[k] = o[7 * 32 + k * 4 + part];
      if (part == 0) h2_out<1, 0>(ow);
      if (part == 1) h2_out<1, 1>(ow);
      if (part == 2) h2_out<1, 2>(ow);
      if (part == 3) h2_out<1, 3>(ow);
    }
    tail<1>(cf, 0.0f, true);
  }
};

// ---------------------------------------------------------------------------- sampler kernel
// The reverse-SDE loop (models/diffusion.py:27-46) for the CDE, a = net(x, y, tau) with y folded into the
// per-y layer-1 bias; mu = g a + 0.5 beta x, x <- x + delta mu + sqrt(delta) g xi (dmip_device.h em_update).
// Work: the balanced WaveSchedule over jobs of 64 chains (two tiles). Tile B runs half a chunk behind tile A,
// so it completes step i in chunk 0 of the loop iteration of step i + 1 (or in the segment's epilogue).
template <int D, bool NOISE>
__global__ void __launch_bounds__(NWV * 64, 1) x3p_sampler_kernel(X3SamplerParams p) {
  using L = PLay;
  static_assert(D >= 1 && D <= 4, "output rows: at most 4");
  __shared__ __attribute__((aligned(16))) char lds[L::TOTAL];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = lane >> 5, j = lane & 31;
  const int yi = blockIdx.y;

  PWave<D, NOISE> e;
  e.lds = lds;
  e.w = w;
  e.h = h;
  e.rs = __builtin_amdgcn_make_buffer_rsrc((void*)p.net[0].pstream, 0, NCH * CHUNK, 0x00020000);
  e.voff = (unsigned)(w * PPW * 1024 + lane * 16);
  e.rb0 = (lds_cptr)(lds + L::RING + lane * 16);
  e.rb2 = (lds_cptr)(lds + L::RING + 2 * CHUNK + lane * 16);
  e.l1b = (lds_cptr)(lds + L::L1 + lane * 16);
  e.bb = (lds_cptr)(lds + L::BIAS + 16 * h);
  e.owb = (lds_cptr)(lds + L::OW + 256 * h);
  e.ones = h == 0 ? u32x4{0x3C003C00u, 0x00003C00u, 0u, 0u} : u32x4{0u, 0u, 0u, 0u};  // k-slots 0..2
  e.delta = p.delta;
  e.sqrt_delta = p.sqrt_delta;
  {
    const uint4* s1 = (const uint4*)p.net[0].pl1;
    uint4* d1 = (uint4*)(lds + L::L1);
    for (int i = threadIdx.x; i < L::L1_BYTES / 16; i += NWV * 64) d1[i] = s1[i];
    const uint4* so = (const uint4*)p.net[0].pow;
    uint4* dow = (uint4*)(lds + L::OW);
    for (int i = threadIdx.x; i < L::OW_BYTES / 16; i += NWV * 64) dow[i] = so[i];
    float* bl = (float*)(lds + L::BIAS);
    for (int i = threadIdx.x; i < W; i += NWV * 64) bl[i] = p.bias_y[(size_t)yi * W + i];
    __syncthreads();
  }
  {
    const float* oi = (const float*)p.net[0].pow + OT * 2 * 64;
#pragma unroll
    for (int k = 0; k < D; ++k) e.oinit[k] = oi[k];
  }
  e.acc[1] = f32x16{};
  if constexpr (kDiag) {
#pragma unroll
    for (int k = 0; k < 17; ++k) e.ph[k] = 0;
  }
  e.ring_start();
  if constexpr (kDiag) e.t_last = stamp();
  Pre cur;
  (void)e.template reads<0, 0>(cur);  // unit (0, 0)'s values; its wait covers them

  const int S = p.num_steps;
  const long long jobs_y = (p.n_chains + JC - 1) / JC;
  const long long n_waves = (long long)gridDim.x * NWV;
  const long long gw = (long long)blockIdx.x * NWV + w;
  constexpr int XT = sampler_xfer_words(D);  // hand-over words per wave: 2 tiles x (D + 4) x 32 lanes
  const WaveSchedule sched(jobs_y, S, n_waves, gw);
  const size_t noise_step = (size_t)gridDim.y * p.n_chains * D;

  for (int sgi = 0; sgi < sched.n_seg; ++sgi) {
    const Seg sg = sched.segment(sgi);
    long long c_loc[2];
    bool valid[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      c_loc[t] = (long long)(sg.job >= 0 ? sg.job : 0) * JC + 32 * t + j;
      valid[t] = sg.job >= 0 && c_loc[t] < p.n_chains;
      e.live[t] = sg.kind != 3 && valid[t];
    }
    if (sg.kind == 2) {  // resume the job the previous wave of the grid handed over
      const size_t slot = (size_t)yi * n_waves + gw - 1;
      const bool lost = handover_wait(p.xflag + slot, p.spin_limit, p.err, kErrHandover, lane);
      const float* src = p.xfer + slot * (size_t)XT;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const float* st = src + t * (D + 4) * 32;
#pragma unroll
        for (int k = 0; k < D; ++k) e.x[t][k] = lost ? __builtin_nanf("") : st[k * 32 + j];
        e.rng[t].s0 = __float_as_uint(st[(D + 0) * 32 + j]);
        e.rng[t].s1 = __float_as_uint(st[(D + 1) * 32 + j]);
        e.rng[t].s2 = __float_as_uint(st[(D + 2) * 32 + j]);
        e.rng[t].s3 = __float_as_uint(st[(D + 3) * 32 + j]);
      }
    } else {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        e.rng[t] = rng_init(p.seed, (uint64_t)(p.chain_offset + c_loc[t]), (uint64_t)yi);
        float n0[D];
        if constexpr (NOISE) {
          const float* src = p.noise + ((size_t)yi * p.n_chains + (valid[t] ? c_loc[t] : 0)) * D;
#pragma unroll
          for (int k = 0; k < D; ++k) n0[k] = src[k];
        } else {
          rng_normals<D>(e.rng[t], n0);
        }
#pragma unroll
        for (int k = 0; k < D; ++k) e.x[t][k] = __fadd_rn(__fmul_rn(n0[k], p.stdv), p.mean);
      }
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int k = 0; k < D; ++k) e.aP[t][k] = 0.0f;
    const int i_first = sg.kind == 3 ? 0 : sg.s0;
    e.cf_prev = step_coef(i_first, S, p.T, p.bmin, p.bdiff);
    e.prologue_a(e.cf_prev.tau);
    e.first = true;

    for (int i0 = sg.s0; i0 < sg.s1; ++i0) {
      const int i = sg.kind == 3 ? 0 : i0;  // idle steps: a dummy job at step 0, discarded
      e.cf_cur = step_coef(i, S, p.T, p.bmin, p.bdiff);
      e.tau_next = step_coef(sg.kind == 3 ? 0 : (i + 1 < S ? i + 1 : i), S, p.T, p.bmin, p.bdiff).tau;
      size_t nA = 0, nB = 0;
      if constexpr (NOISE) {
        nA = noise_step * (i + 1) + ((size_t)yi * p.n_chains + (valid[0] ? c_loc[0] : 0)) * D;
        nB = noise_step * (i + 1) + ((size_t)yi * p.n_chains + (valid[1] ? c_loc[1] : 0)) * D;
      }
      e.template run<0, 0>(cur, p.noise, nA, nB);
      e.cf_prev = e.cf_cur;
      e.first = false;
      // snapshots: tile A after step i0, tile B after step i0 - 1 (completed in chunk 0 of this step)
      if (!kDiag && p.snap_every > 0 && sg.kind != 3 && h == 0) {
        if ((i0 + 1) % p.snap_every == 0 && valid[0]) {
          float* dst = p.snap_out + (((size_t)((i0 + 1) / p.snap_every - 1) * gridDim.y + yi) * p.n_chains + c_loc[0]) * D;
#pragma unroll
          for (int k = 0; k < D; ++k) dst[k] = e.x[0][k];
        }
        if (i0 > sg.s0 && i0 % p.snap_every == 0 && valid[1]) {
          float* dst = p.snap_out + (((size_t)(i0 / p.snap_every - 1) * gridDim.y + yi) * p.n_chains + c_loc[1]) * D;
#pragma unroll
          for (int k = 0; k < D; ++k) dst[k] = e.x[1][k];
        }
      }
    }
    e.epilogue_b(e.cf_prev);
    {  // tile B's snapshot of the segment's last step
      const int last = sg.s1 - 1;
      if (!kDiag && p.snap_every > 0 && (last + 1) % p.snap_every == 0 && sg.kind != 3 && h == 0 && valid[1]) {
        float* dst = p.snap_out + (((size_t)((last + 1) / p.snap_every - 1) * gridDim.y + yi) * p.n_chains + c_loc[1]) * D;
#pragma unroll
        for (int k = 0; k < D; ++k) dst[k] = e.x[1][k];
      }
    }
    if (sg.kind == 1) {  // hand the job over to the next wave of the grid
      const size_t slot = (size_t)yi * n_waves + gw;
      float* dst = p.xfer + slot * (size_t)XT;
      if (h == 0) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          float* st = dst + t * (D + 4) * 32;
#pragma unroll
          for (int k = 0; k < D; ++k) st[k * 32 + j] = e.x[t][k];
          st[(D + 0) * 32 + j] = __uint_as_float(e.rng[t].s0);
          st[(D + 1) * 32 + j] = __uint_as_float(e.rng[t].s1);
          st[(D + 2) * 32 + j] = __uint_as_float(e.rng[t].s2);
          st[(D + 3) * 32 + j] = __uint_as_float(e.rng[t].s3);
        }
      }
      handover_publish(p.xflag + slot, lane, p.debug_flags);
    } else if (sg.kind != 3 && h == 0) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (!valid[t]) continue;
        float* dst = p.x_out + ((size_t)yi * p.n_chains + c_loc[t]) * D;
#pragma unroll
        for (int k = 0; k < D; ++k) dst[k] = e.x[t][k];
      }
    }
  }
  wait_vmcnt<0>();  // the prefetched chunks of a step that never ran land before the workgroup exits
  x3::report_range(e.oor, p.err, lane);
  if constexpr (kDiag) {
    if (lane == 0 && p.snap_out) {
      uint64_t* dst = (uint64_t*)p.snap_out + ((size_t)yi * n_waves + gw) * 18;
#pragma unroll
      for (int k = 0; k < 17; ++k) dst[k] = e.ph[k];
      dst[17] = (uint64_t)sched.C;
    }
  }
}

}  // namespace x3p

template <int D, bool NOISE>
inline hipError_t launch_x3p_sampler_t(const X3SamplerParams& p, int n_y, hipStream_t st) {
  using namespace x3p;
  auto kern = x3p_sampler_kernel<D, NOISE>;
  const long long jobs = (p.n_chains + JC - 1) / JC;
  long long g = resident_slots(kern, NWV * 64, st) / (n_y > 0 ? n_y : 1);
  const long long cap = (jobs + NWV - 1) / NWV;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  X3SamplerParams q = p;
  char* buf = nullptr;
  hipError_t e = alloc_handover((size_t)g * n_y * NWV, D, st, &buf, &q.xfer, &q.xflag);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)g, (unsigned)n_y), dim3(NWV * 64), 0, st, q);
  e = hipGetLastError();
  (void)hipFreeAsync(buf, st);
  return e;
}

}  // namespace dmip
