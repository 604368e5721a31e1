// Fused score-matching training step: loss value and parameter gradients of the CDE training losses
// (losses.py:42-242 as called by CDE.train_epoch, models/diffusion.py:74-89) for one batch: by default
// a forward half and a reverse half (two kernels, see PH below), or the one-kernel build
// (DMIP_TRAIN_SPLIT=0), plus a deterministic reduction.
//
// Formulation (restated and pinned in oracle/dmip_oracle.py:loss_grad):
//  * forward pass with forward-mode jets through the MLP (nets.py:17-35, double tanh on layer 1):
//    primal P at (x_t, y, t); tangent V along d/dt of (x_t(t), y, t) (the total derivative of
//    batch_gradient, losses.py:20-26); tangents E0, E1 along x_t (the divergence, losses.py:14-18) and
//    second-order E00, E01, E11 (grad_x of div s, losses.py:88-89); IC primal C at (x, y, 0);
//  * per-sample DSM / ScoreFPE / cScoreFPE / IC terms and their adjoints;
//  * reverse pass through the P, V and C streams (grad_x is detached in the reference, so the
//    E-streams need no reverse), recomputing the forward activations layer by layer instead of
//    storing them; weight gradients as sample-contracted MFMA products through an LDS transpose.
//
// Precision: the primal-type streams (P, V, C) are split-bf16 products (W_hi h_hi + W_hi h_lo +
// W_lo h_hi, ~fp32): near a trained optimum the loss adjoints are small residuals (s std + eps, the
// FPE and IC residuals) and plain bf16 weights perturb the gradient by up to ~10 % (measured in a
// numpy bf16 simulation of the trained fixture); the jet streams E* (detached grad_x) and the reverse
// products stay plain bf16 (<0.5 % on the same fixture).
//
// Layout: 16 samples per tile and wave; every stream is a 64 x 16 (units x samples) matrix held as
// four 16x16 accumulator tiles (v_mfma_f32_16x16x32_bf16: unit = 16R + 4(lane>>4) + reg, sample =
// lane & 15), which repack into the next layer's B operand with no lane movement (k-permuted weight
// fragments, as in the sampler). Weight-gradient products contract over samples and use
// v_mfma_f32_32x32x16_bf16 (K = the tile's 16 samples). The reverse half's workgroup accumulates one
// gradient partial in LDS with its waves taking turns (below); the one-kernel build accumulates per-wave
// rows of `partials` (global, 4-wave build) or LDS regions (2-wave build). loss_grad_reduce_kernel sums
// the rows in a fixed order: the gradients are bit-reproducible.
#include <algorithm>
#include <cstdlib>

#include "dmip_device.h"
#include "dmip_internal.h"
#include "dmip_stepdev.h"

namespace dmip {
namespace train {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

constexpr int W = kTrainWidth;  // hidden width
constexpr int D = kTrainXdim;   // xdim
constexpr int M = kTrainYdim;   // ydim
constexpr int IN = D + M + 1;   // cat[x, y, t] (nets.py:33)
constexpr int OUT = D;          // CDE drift
#ifndef DMIP_TRAIN_NWV
#define DMIP_TRAIN_NWV 4
#endif
// waves per workgroup: 4 = one wave on each SIMD of the CU, with the per-wave gradient partial in
// global memory (its own row of `partials`, L2/MALL-resident); 2 = the partial in LDS, which limits
// the workgroup to 2 waves (2 of 4 SIMDs) by its 158 KiB of LDS
constexpr int NWV = DMIP_TRAIN_NWV;
constexpr bool GACC_GLOBAL = NWV > 2;
constexpr int NS = 16;          // samples per tile
// row stride (bf16 elements) of the per-wave transposed scratch [unit][sample]: 16 samples padded
// to 24 (48 bytes), so put_t's four lane groups (rows 4 apart) land on disjoint banks (row offsets
// 0 / 48 / 32 / 16 banks) and tread's 16-byte rows stay aligned and conflict-free (12-bank steps);
// unpadded (32 bytes) groups 0/2 and 1/3 collided: ~75 % of LDS-active cycles were bank conflicts
constexpr int RS = 24;
constexpr int NSTREAM = 8;      // P, V, C, E0, E1, E00, E01, E11
static_assert(W == 64 && D == 2, "compiled for the linear problem's width-64 CDE");
static_assert(3 * IN + 2 <= 32, "layer-1 split operand fits one k-step");

// PH: 0 = the fused kernel (forward jets, loss terms and reverse pass in one wave, one wave per SIMD);
// 1 = the forward half (jets + per-sample loss terms and adjoints into p.adj; two waves per SIMD);
// 2 = the reverse half (adjoints from p.adj, recompute + weight gradients; its layer loop unrolled, one wave per
// SIMD -- an 8-wave two-per-SIMD build spilled and measured slower). Round 5: each wave OWNS fixed
// 32 x 32 blocks of the workgroup's weight gradient and keeps them in registers for the whole launch -- block
// (T, U) = (w >> 1, w & 1) of every W x W layer, and the output layer's block U = w - 2 (waves 2-3) or layer 1's
// block T = w (waves 0-1). At each layer the waves write their tile's transposed adjoints and activations (double-
// buffered scratch), one workgroup barrier, then every wave contracts ITS blocks over the samples of all four waves'
// tiles (wave order 0..3, stream order within: a fixed summation order, deterministic). Round 3's turns (one LDS
// partial, four barrier-separated turns of read-add-write per layer: 16 barriers and 256 LDS read-modify-writes per
// tile) become one barrier per layer and no adds; the biases and loss sums meet once, at the end, in wave order.
// (~160 global atomics per tile in the fused kernel: its L2 atomic rate alone, ~50 ns per 256-byte wave-instruction
// per CU, was ~130 us of the 0.3 ms)
template <int NL, int PH = 0>
struct TL {
  static constexpr int NW = PH == 0 ? NWV : 4;               // waves per workgroup
  static constexpr bool OWN = PH >= 2;                       // each wave owns fixed gradient blocks in registers
  static constexpr int NBUF = OWN ? 2 : 1;                   // transposed scratch sets per wave (layer-parity buffered)
  static constexpr bool GG = PH == 0 ? GACC_GLOBAL : false;  // gradient partial rows in global memory
  static constexpr int RSV = PH >= 2 ? 16 : RS;              // scratch row stride (reverse half: unpadded, to fit)
  static constexpr int p_w(int l) { return l == 0 ? 0 : W * IN + W + (l - 1) * (W * W + W); }
  static constexpr int p_b(int l) { return l == NL ? p_w(NL) + OUT * W : p_w(l) + (l == 0 ? W * IN : W * W); }
  static constexpr int NPARAM = p_w(NL) + OUT * W + OUT;
  static constexpr int PART = NPARAM + 4;                // per-wave partial: grads + 3 loss sums (+pad)
  // LDS (bytes)
  static constexpr int WF = 0;                           // forward fragments, hidden W x W layers (bf16 hi)
  static constexpr int WFL = WF + (NL - 1) * 8192;       // their bf16 residuals (lo), for the split products
  static constexpr int WT = WFL + (NL - 1) * 8192;       // transposed fragments (reverse pass)
  static constexpr int A1 = WT + (NL - 1) * 8192;        // layer-1 split fragments
  static constexpr int AOT = A1 + 4096;                  // output layer transposed
  static constexpr int BIAS = AOT + 4096;                // fp32 [NL + 1][64]: b_l of hidden l, b_out at NL
  static constexpr int AO = BIAS + (NL + 1) * W * 4;     // output layer, rows duplicated per lane group (forward)
  static constexpr int AOL = AO + 2048;                  // its lo residuals (forward)
  static constexpr int COL = AOL + 2048;                 // fp32 [D][64]: layer-1 weight columns of x (forward)
  static constexpr int WAVE = COL + D * W * 4;
  static constexpr int IMG = PH >= 2 ? AO : WAVE;        // image bytes this kernel copies (reverse: no forward-only parts)
  static constexpr int GACC = 0;                         // per wave: fp32 gradient partial (param order, LDS mode)
  static constexpr int SCR = (GG || OWN) ? 0 : ((PART * 4 + 15) / 16) * 16;  // per wave: 6 transposed [64][16] bf16
  static constexpr int SET = 6 * W * RSV * 2;            // one transposed scratch set (bytes)
  static constexpr int WAVE_BYTES = PH == 1 ? 0 : SCR + NBUF * SET;
  static constexpr int TOTAL = IMG + NW * WAVE_BYTES;
  static_assert(TOTAL <= 160 * 1024, "LDS budget");
  // OWN: the flush's bias / loss partial reuses the scratch (after the last tile)
  static_assert(!OWN || PART * 4 <= NW * WAVE_BYTES, "flush partial fits the scratch");
};

__device__ __forceinline__ int kp(int s, int g, int j) { return 32 * s + 16 * (j >> 2) + 4 * g + (j & 3); }

__device__ __forceinline__ __bf16 bf_hi(float v) { return (__bf16)v; }
__device__ __forceinline__ __bf16 bf_lo(float v) { return (__bf16)(v - (float)(__bf16)v); }

// tanh as 1 - 2/(1 + e^2z): exp2 + rcp. Near 0 the form cancels to ~2^-23 ABSOLUTE error (not relative);
// every consumer here is a split-bf16 product (~2^-17 relative of the products' scale) or a 1 - h^2
// derivative, so the small-|z| polynomial branch it once had (a compare, a select and 5 more VALU per
// call, ~500 calls per tile) bought nothing measurable (tests/test_gpu_parity.py gates, round 3)
__device__ __forceinline__ float tanh_f(float z) {
  const float e = __builtin_amdgcn_exp2f(2.8853900817779268f * z);
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + e);
}

__device__ __forceinline__ float sgn(float v) { return (float)((v > 0.0f) - (v < 0.0f)); }

// B operand of layer 1 for one stream: slots [hi(u) | lo(u) | hi(u) | one | one | 0...]; lane group g
// supplies slots 8g..8g+7 of its sample
__device__ __forceinline__ bf16x8 b1_operand(const float (&u)[IN], float one, int g) {
  __bf16 sl[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    if (k < IN) sl[k] = bf_hi(u[k]);
    else if (k < 2 * IN) sl[k] = bf_lo(u[k - IN]);
    else if (k < 3 * IN) sl[k] = bf_hi(u[k - 2 * IN]);
    else if (k < 3 * IN + 2) sl[k] = (__bf16)one;
    else sl[k] = (__bf16)0.0f;
  }
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = g == 0 ? sl[j] : (g == 1 ? sl[8 + j] : (g == 2 ? sl[16 + j] : sl[24 + j]));
  return r;
}

__device__ __forceinline__ const bf16x8& frag(const char* base, int idx, int lane) {
  return *(const bf16x8*)(base + (idx * 64 + lane) * 16);
}

// element (unit row, sample col) of a transposed scratch block: row stride RSV. The unpadded layout (RSV = 16,
// 32-byte rows, the reverse half) is swizzled for both of its access patterns (MI355X_MICROARCH.md §LDS):
//  * put_t's ds_write_b16 (lane groups of 32, bank = dword mod 32): lanes 0-31 write rows r and r + 4 of an
//    8-row group, so those must sit in different 8-bank quarters of the 128-byte bank row: within each 8-row
//    group row r takes 32-byte block pi(r) = 2 (r & 3) + (r >> 2) (rows 0-3 even blocks, rows 4-7 odd);
//  * tread's ds_read_b128 (lane groups of 16, bank = dword mod 64): a group reads rows {0-3, 12-15, 20-27} (or
//    {4-11, 16-19, 28-31}) of a 32-row block, same 16-byte half; with pi two of those rows share a block mod
//    8, one in an even and one in an odd 8-row group, so the two 16-byte halves of rows 8..15 mod 16 swap.
// Every group then touches distinct banks (round 3's swizzle alone left put_t's rows r, r + 4 colliding:
// SQ_LDS_BANK_CONFLICT 2.49M per dispatch, 45 % of LDS-active cycles, profiles/r4_pmc_config5_reverse.json)
template <int RSV>
__device__ __forceinline__ int sidx(int row, int col) {
  if constexpr (RSV == 16) {
    const int blk = (row & ~7) | ((row & 3) << 1) | ((row >> 2) & 1);
    return blk * 16 + (((col >> 3) ^ ((row >> 3) & 1)) << 3) + (col & 7);
  }
  return row * RSV + col;
}

// write one acc-form stream (64 units x 16 samples) transposed: scr[unit][sample] bf16
template <int RSV>
__device__ __forceinline__ void put_t(__bf16* scr, const f32x4 (&z)[4], int g, int c16) {
#pragma unroll
  for (int R = 0; R < 4; ++R)
#pragma unroll
    for (int r = 0; r < 4; ++r) scr[sidx<RSV>(16 * R + 4 * g + r, c16)] = (__bf16)z[R][r];
}

__device__ __forceinline__ void pack_b(const f32x4 (&z)[4], bf16x8 (&b)[2]) {
#pragma unroll
  for (int R = 0; R < 4; ++R)
#pragma unroll
    for (int r = 0; r < 4; ++r) b[R >> 1][4 * (R & 1) + r] = (__bf16)z[R][r];
}

// split-bf16 B operand of an acc-form stream: hi = bf16(v), lo = bf16(v - hi)
__device__ __forceinline__ void pack_b2(const f32x4 (&z)[4], bf16x8 (&b)[2], bf16x8 (&bl)[2]) {
#pragma unroll
  for (int R = 0; R < 4; ++R)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      b[R >> 1][4 * (R & 1) + r] = bf_hi(z[R][r]);
      bl[R >> 1][4 * (R & 1) + r] = bf_lo(z[R][r]);
    }
}

// one 16-row tile of W (two k-steps) times a stream: plain bf16, or split (~fp32)
__device__ __forceinline__ f32x4 mm(const bf16x8& a0, const bf16x8& a1, const bf16x8 (&h)[2], f32x4 acc) {
  acc = mfma16(a0, h[0], acc);
  return mfma16(a1, h[1], acc);
}
__device__ __forceinline__ f32x4 mm3(const bf16x8& a0, const bf16x8& a1, const bf16x8& l0, const bf16x8& l1,
                                     const bf16x8 (&h)[2], const bf16x8 (&hl)[2], f32x4 acc) {
  acc = mfma16(l0, h[0], acc);
  acc = mfma16(l1, h[1], acc);
  acc = mfma16(a0, hl[0], acc);
  acc = mfma16(a1, hl[1], acc);
  acc = mfma16(a0, h[0], acc);
  return mfma16(a1, h[1], acc);
}

// the 32x32x16 operand of a sample-contracted product: lane (i, hh) reads row (row0 + i), samples 8hh..8hh+7
template <int RSV>
__device__ __forceinline__ bf16x8 tread(const __bf16* scr, int row, bool ok, int hh) {
  // branch-free: every row < 64 is inside the scratch block; rows that are not operands read as zero
  const u32x4 v = *(const u32x4*)(scr + sidx<RSV>(row, 8 * hh));
  const u32x4 z = {0u, 0u, 0u, 0u};
  return __builtin_bit_cast(bf16x8, ok ? v : z);
}

// Records (the record reverse half, PH = 3; p.rec): the forward half keeps, per tile and hidden layer li (z_li = the
// layer's pre-activation: layer 1 at li = 0), what the reverse pass needs of that layer instead of recomputing the
// forward: the activations of the P, V and C streams (h_P, h_V = d1 z_V, h_C: the operands of the next layer's weight-
// gradient contraction, which rounds them to bf16 anyway, so bf16 records are bit-identical to recomputed ones) and the
// three coefficients of the activation's reverse, zbar_P = d1 hbar_P + (d2 z_V) hbar_V, zbar_V = d1 hbar_V,
// zbar_C = d1_C hbar_C (d1, d1_C in (0, 1]: fp16; d2 z_V: bf16). Layout: for each (tile, li, row-tile pair Rp,
// quantity q) lane l's 8 values (R = 2 Rp + (0, 1), r) -- unit 16 R + 4 (l >> 4) + r of sample l & 15 -- as one
// 16-byte piece, piece (Rp, q) being 64 lanes x 16 B contiguous: the reverse half reads it with one coalesced dwordx4
// per lane (36 loads per tile, so a tile's loads fit the 6-bit vmcnt counter beside the inputs'); the forward half
// writes each R's 8-byte half as soon as its values exist, holding nothing across R. Value (R, r) is half r & 1 of
// dword 2 (R & 1) + (r >> 1). 12 KiB per (tile, layer): 36 KiB per 16-sample tile at NL = 3, 151 MB at batch 65,536.
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)a) | ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)b) << 16);
}
__device__ __forceinline__ uint32_t pk_f16(float a, float b) {
  return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)a) | ((uint32_t)__builtin_bit_cast(uint16_t, (_Float16)b) << 16);
}

template <int NL>
__device__ __forceinline__ u32x4* rec_at(uint32_t* rec, long long tile, int li, int Rp, int q, int lane) {
  return (u32x4*)rec + ((((size_t)tile * NL + li) * 2 + Rp) * kTrainRecQ + q) * 64 + lane;
}
// row tile R's 8-byte half of its piece
template <int NL>
__device__ __forceinline__ u32x2* rec_half(uint32_t* rec, long long tile, int li, int R, int q, int lane) {
  return (u32x2*)rec_at<NL>(rec, tile, li, R >> 1, q, lane) + (R & 1);
}

// value (R, r) of a quantity's two pieces
template <bool F16>
__device__ __forceinline__ float rec_val(const u32x4 (&d)[2], int R, int r) {
  const uint32_t wd = d[R >> 1][2 * (R & 1) + (r >> 1)];
  const uint16_t h = (r & 1) ? (uint16_t)(wd >> 16) : (uint16_t)(wd & 0xffffu);
  if constexpr (F16) return (float)__builtin_bit_cast(_Float16, h);
  return __builtin_bit_cast(float, (uint32_t)h << 16);
}

// the forward half's record writes: row tile R's coefficients (q 3..5) as soon as they exist, and the activations
// (q 0..2) straight from the packed bf16 B operand of the next layer once its R pair is complete -- the bf16 hi part,
// the same RNE rounding -- so the writes hold no extra registers across R
// The forward half's record writes go through a per-tile buffer resource (the tile is wave-uniform): the piece's
// offset is a compile-time scalar offset and the lane's 16 bytes (+ 8 for an odd row tile) the per-lane offset, so no
// 64-bit address is formed or kept per store (with global stores the records spilled 128 B of the forward half's
// 256-register budget)
template <int NL>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rec_rsrc(uint32_t* rec, long long tile) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)((char*)rec + (size_t)tile * NL * kTrainRecTileBytes), 0,
                                           NL * kTrainRecTileBytes, 0x00020000);
}
constexpr int rec_off(int li, int Rp, int q) { return ((li * 2 + Rp) * kTrainRecQ + q) * 1024; }
// cache policy of the record stores (A/B knob DMIP_TRAIN_REC_AUX; 0 = default)
#ifndef DMIP_TRAIN_REC_AUX
#define DMIP_TRAIN_REC_AUX 0
#endif
constexpr int kRecAux = DMIP_TRAIN_REC_AUX;

// row tile R's coefficients (q 3..5): each R's 8-byte half at once (holds nothing across R; storing each value pair
// as soon as it exists, or full 16-byte pieces at odd R, measured more spills)
template <int NL>
__device__ __forceinline__ void rec_put_coef(__amdgpu_buffer_rsrc_t rr, int li, int R, int lane, const float (&d1)[4],
                                             const float (&b)[4], const float (&d1c)[4]) {
  const int vo = lane * 16 + (R & 1) * 8;
  __builtin_amdgcn_raw_buffer_store_b64(u32x2{pk_f16(d1[0], d1[1]), pk_f16(d1[2], d1[3])}, rr, vo,
                                        rec_off(li, R >> 1, 3), kRecAux);
  __builtin_amdgcn_raw_buffer_store_b64(u32x2{pk_bf16(b[0], b[1]), pk_bf16(b[2], b[3])}, rr, vo,
                                        rec_off(li, R >> 1, 4), kRecAux);
  __builtin_amdgcn_raw_buffer_store_b64(u32x2{pk_f16(d1c[0], d1c[1]), pk_f16(d1c[2], d1c[3])}, rr, vo,
                                        rec_off(li, R >> 1, 5), kRecAux);
}
template <int NL>
__device__ __forceinline__ void rec_put_h(__amdgpu_buffer_rsrc_t rr, int li, int Rp, int lane, const bf16x8 (&h)[3][2]) {
#pragma unroll
  for (int q = 0; q < 3; ++q)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, h[q][Rp]), rr, lane * 16, rec_off(li, Rp, q), kRecAux);
}

// The shared part of the LDS image (weight fragments, biases, layer-1 columns), packed ONCE per
// launch into a global buffer by train_pack_kernel; every workgroup then copies it into LDS with
// coalesced 16-byte loads (instead of each workgroup converting the fp32 weights with strided reads).
template <int NL>
__device__ __forceinline__ void pack_weights(const TrainParams& p, char* base, int tid, int nth) {
  using L = TL<NL>;
  {
    __bf16* wf = (__bf16*)(base + L::WF);
    __bf16* wfl = (__bf16*)(base + L::WFL);
    __bf16* wt = (__bf16*)(base + L::WT);
    for (int e = tid; e < (NL - 1) * 4096; e += nth) {
      const int l = e / 4096, r0 = e % 4096;
      const int R = r0 / 1024, s = (r0 / 512) & 1, ln = (r0 / 8) & 63, j = r0 & 7;
      const int row = 16 * R + (ln & 15), k = kp(s, ln >> 4, j);
      const float* Wl = p.w[l + 1];
      wf[e] = bf_hi(Wl[row * W + k]);
      wfl[e] = bf_lo(Wl[row * W + k]);
      wt[e] = (__bf16)Wl[k * W + row];
    }
    __bf16* a1 = (__bf16*)(base + L::A1);
    for (int e = tid; e < 2048; e += nth) {
      const int R = e / 512, ln = (e / 8) & 63, j = e & 7;
      const int row = 16 * R + (ln & 15), k = 8 * (ln >> 4) + j;
      const float* W0 = p.w[0] + row * IN;
      __bf16 o = (__bf16)0.0f;
      if (k < IN) o = bf_hi(W0[k]);
      else if (k < 2 * IN) o = bf_hi(W0[k - IN]);
      else if (k < 3 * IN) o = bf_lo(W0[k - 2 * IN]);
      else if (k == 3 * IN) o = bf_hi(p.b[0][row]);
      else if (k == 3 * IN + 1) o = bf_lo(p.b[0][row]);
      a1[e] = o;
    }
    __bf16* ao = (__bf16*)(base + L::AO);
    __bf16* aol = (__bf16*)(base + L::AOL);
    for (int e = tid; e < 1024; e += nth) {
      const int s = e / 512, ln = (e / 8) & 63, j = e & 7;
      const int o = (ln & 15) & 3;
      const float v = o < OUT ? p.w[NL][o * W + kp(s, ln >> 4, j)] : 0.0f;
      ao[e] = bf_hi(v);
      aol[e] = bf_lo(v);
    }
    __bf16* aot = (__bf16*)(base + L::AOT);
    for (int e = tid; e < 2048; e += nth) {
      const int R = e / 512, ln = (e / 8) & 63, j = e & 7;
      const int unit = 16 * R + (ln & 15), k = 8 * (ln >> 4) + j;
      aot[e] = k < OUT ? (__bf16)p.w[NL][k * W + unit] : (__bf16)0.0f;
    }
    float* bias = (float*)(base + L::BIAS);
    for (int e = tid; e < (NL + 1) * W; e += nth) {
      const int l = e / W, u = e % W;
      float v = 0.0f;
      if (l >= 1 && l < NL) v = p.b[l][u];
      else if (l == NL && u < OUT) v = p.b[NL][u];
      bias[e] = v;
    }
    float* col = (float*)(base + L::COL);
    for (int e = tid; e < D * W; e += nth) col[e] = p.w[0][(e % W) * IN + e / W];
  }
}

template <int NL>
__global__ void __launch_bounds__(256) train_pack_kernel(TrainParams p) {
  pack_weights<NL>(p, p.packed, blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x);
}

// add into the wave's gradient partial: in global memory a no-return float atomic (the wave does not
// wait for a load of its own row before every update: those read-modify-write round trips sat on the
// tile's dependency chain); the row is the wave's own, and its updates to one address are issued in
// program order, so the sums keep a fixed order. In LDS a plain add.
// OWN: a workgroup barrier after this wave's LDS operations have completed (the reverse half's layer barrier, and
// the flush's wave-ordered turns)
__device__ __forceinline__ void turn_barrier() {
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
#ifndef DMIP_TRAIN_TIMING_NO_TURN_BARRIER  // timing ablation only (scripts/gpu_c5_ablate.sh): wrong gradients
  __builtin_amdgcn_s_barrier();
#endif
}

// inclusive scan over each 16-lane row by DPP row shifts: lane 15 of a row holds the sum of the row's 16 lanes, always
// summed in the same order (deterministic)
__device__ __forceinline__ float row_sum16(float v) {
#define DMIP_ROW_SHR(n) \
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x110 + (n), 0xf, 0xf, true))
  DMIP_ROW_SHR(1);
  DMIP_ROW_SHR(2);
  DMIP_ROW_SHR(4);
  DMIP_ROW_SHR(8);
#undef DMIP_ROW_SHR
  return v;
}

// timing ablation only (scripts/gpu_r6_c5abl.sh; wrong gradients): the reverse half's weight-gradient contraction
// MFMAs left out (their scratch reads stay)
#ifdef DMIP_TRAIN_TIMING_NO_CONTRACT
#define DMIP_TRAIN_CONTRACT(stmt) asm volatile("" ::"v"(A), "v"(Bm))
#else
#define DMIP_TRAIN_CONTRACT(stmt) stmt
#endif

template <bool GG>
__device__ __forceinline__ void gadd(float* a, float v) {
  if constexpr (GG) (void)__hip_atomic_fetch_add(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *a += v;
}

template <int NL, int PH = 0>
__global__ void __launch_bounds__((TL<NL, PH>::NW * 64), (PH == 1 ? 2 : 1)) loss_grad_kernel(TrainParams p) {
  using L = TL<NL, PH>;
  constexpr int NWV = L::NW;
  constexpr bool GACC_GLOBAL = L::GG;
  constexpr int RS = L::RSV;
  __shared__ __attribute__((aligned(16))) char lds[L::TOTAL];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c16 = lane & 15, g = lane >> 4;
  const int i32 = lane & 31, hh = lane >> 5;

  // ---- the shared LDS image (packed once per launch by train_pack_kernel): 16-byte copies
  {
    static_assert(L::IMG % 16 == 0, "LDS image is a whole number of 16-byte pieces");
    const uint4* src = (const uint4*)p.packed;
    uint4* dst = (uint4*)lds;
    if constexpr (PH == 3) {  // the record reverse reads the transposed images only (W^T for hbar, the output's)
      static_assert(L::A1 - L::WT == L::AOT - L::WT - 4096 && L::WT % 16 == 0 && L::AOT % 16 == 0, "image layout");
#pragma unroll 4
      for (int e = tid; e < (L::A1 - L::WT) / 16; e += NWV * 64) dst[L::WT / 16 + e] = src[L::WT / 16 + e];
      for (int e = tid; e < 4096 / 16; e += NWV * 64) dst[L::AOT / 16 + e] = src[L::AOT / 16 + e];
    } else {
#pragma unroll 4
      for (int e = tid; e < L::IMG / 16; e += NWV * 64) dst[e] = src[e];
    }
    if constexpr (PH == 1 || L::OWN) {
    } else if constexpr (!GACC_GLOBAL) {
      float* gacc = (float*)(lds + L::WAVE + w * L::WAVE_BYTES + L::GACC);
      for (int e = lane; e < L::PART; e += 64) gacc[e] = 0.0f;
    } else {
      float* gacc = p.partials + ((size_t)blockIdx.x * NWV + w) * L::PART;
      for (int e = lane; e < L::PART; e += 64) gacc[e] = 0.0f;
      __threadfence();  // the zeroes are in L2 before the first atomic of this wave lands
    }
  }
  __syncthreads();

  const char* wfr = lds + L::WF;
  const char* wtr = lds + L::WT;
  const char* a1r = lds + L::A1;
  const char* aor = lds + L::AO;
  const char* aotr = lds + L::AOT;
  const float* bias = (const float*)(lds + L::BIAS);
  const float* col = (const float*)(lds + L::COL);
  char* wave_base = lds + L::IMG + w * L::WAVE_BYTES;
  // OWN: the flush's bias / loss partial (in the scratch, after the last tile)
  float* gacc = L::OWN ? (float*)(lds + L::IMG)
                       : (GACC_GLOBAL ? p.partials + ((size_t)blockIdx.x * NWV + w) * L::PART : (float*)(wave_base + L::GACC));
  __bf16* scr = (__bf16*)(wave_base + L::SCR);
  int sbuf = 0;  // OWN: this layer's scratch set (alternates with every layer processed)
  auto S_ = [&](int k) { return scr + (sbuf * 6 + k) * W * RS; };
  // OWN: scratch k of wave v's current set
  auto SV = [&](int v, int k) {
    return (const __bf16*)(lds + L::IMG + v * L::WAVE_BYTES + L::SCR) + (sbuf * 6 + k) * W * RS;
  };
  // OWN: this wave's gradient blocks, accumulated over every tile of the workgroup
  f32x16 gW[NL > 1 ? NL - 1 : 1];  // block (w >> 1, w & 1) of W x W layer l at gW[l - 1]
  f32x16 gX;                       // waves 0-1: layer 1's block T = w; waves 2-3: the output layer's block U = w - 2
#pragma unroll
  for (int l = 0; l < (NL > 1 ? NL - 1 : 1); ++l) gW[l] = f32x16{};
  gX = f32x16{};

  f32x4 bbar[NL > 1 ? NL - 1 : 1][4];  // per-lane bias-gradient partials of the hidden W x W layers
#pragma unroll
  for (int l = 0; l < NL - 1; ++l)
#pragma unroll
    for (int R = 0; R < 4; ++R) bbar[l][R] = f32x4{};
  float bobar[OUT] = {};
  float lsum[3] = {0.0f, 0.0f, 0.0f};  // DSM, IC, PDE row sums (lane group 0 only)

  const long long n_tiles = (p.n + NS - 1) / NS;
  // OWN: every wave of the workgroup runs the same rounds (a wave past the end runs an all-invalid tile),
  // so the layer barriers match
  // REC: the records of the wave's tile, all hidden layers. They are loaded one tile ahead: layer li's registers are
  // refilled with the NEXT tile's layer li as soon as this tile's pass B has used them (its coefficients, at step li),
  // so a tile's records are in flight during the previous tile's later layers. The first tile's are loaded here. A
  // wave past the end reads the last tile's (finite) records: its adjoints are zero, so they add nothing.
  constexpr bool REC = PH == 3;
  u32x4 rc[REC ? NL : 1][kTrainRecQ][2];
  const long long tile_step = (long long)gridDim.x * NWV;
  auto rec_load = [&](long long tl, int li) {
    const long long tt = tl < n_tiles ? tl : n_tiles - 1;
#pragma unroll
    for (int q = 0; q < kTrainRecQ; ++q)
#pragma unroll
      for (int Rp = 0; Rp < 2; ++Rp) rc[li][q][Rp] = *rec_at<NL>(p.rec, tt, li, Rp, q, lane);
  };
  // REC: the per-sample inputs and the forward half's adjoint record are loaded one tile ahead as well, and issued at
  // the start of the previous tile, i.e. before that tile's record refills: waiting for them (vmcnt counts in issue
  // order) then never waits for the younger record loads too
  struct In {
    float x[D], y[M], eps[D], t;
    float4 a0, a1, a2;
  };
  auto in_load = [&](long long tl) {
    In v;
    const long long sj = tl * NS + c16;
    const long long sc = sj < p.n ? sj : p.n - 1;  // a sample past the end loads sample n - 1 (masked by `valid`)
    static_assert(D == 2 && M == 2, "the inputs load as float2");
    const float2 xv = *(const float2*)(p.x + sc * D), ev = *(const float2*)(p.eps + sc * D);
    const float2 yv = *(const float2*)(p.y + sc * M);
    v.x[0] = xv.x, v.x[1] = xv.y, v.eps[0] = ev.x, v.eps[1] = ev.y, v.y[0] = yv.x, v.y[1] = yv.y;
    v.t = p.t[sc];
    const float4* ar = (const float4*)(p.adj + sc * kTrainAdj);
    v.a0 = ar[0], v.a1 = ar[1], v.a2 = ar[2];
    return v;
  };
  In in_next{};
  if constexpr (REC) {
    in_next = in_load((long long)blockIdx.x * NWV + w);
#pragma unroll
    for (int li = NL - 1; li >= 0; --li) rec_load((long long)blockIdx.x * NWV + w, li);
    // the first tile's loads land before the loop: otherwise the compiler's wait counts at the loop head, merged
    // over the prologue path (where it may have issued the records before the inputs) and the back edge, drain the
    // previous tile's record refills in every iteration
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  }
  for (long long tile0 = (long long)blockIdx.x * NWV + (L::OWN ? 0 : w); tile0 < n_tiles;
       tile0 += (long long)gridDim.x * NWV) {
    const long long tile = tile0 + (L::OWN ? w : 0);
    const long long si = tile * NS + c16;
    const bool valid = si < p.n;
    // ---------------------------------------------------------------- per-sample inputs
    float x[D], y[M], eps[D], t;
    In in_cur{};
    if constexpr (REC) {
      in_cur = in_next;
      in_next = in_load(tile + tile_step);
#pragma unroll
      for (int k = 0; k < D; ++k) x[k] = valid ? in_cur.x[k] : 0.0f, eps[k] = valid ? in_cur.eps[k] : 0.0f;
#pragma unroll
      for (int k = 0; k < M; ++k) y[k] = valid ? in_cur.y[k] : 0.0f;
      t = valid ? in_cur.t : 0.5f;
    } else if (valid) {
#pragma unroll
      for (int k = 0; k < D; ++k) x[k] = p.x[si * D + k], eps[k] = p.eps[si * D + k];
#pragma unroll
      for (int k = 0; k < M; ++k) y[k] = p.y[si * M + k];
      t = p.t[si];
    } else {
#pragma unroll
      for (int k = 0; k < D; ++k) x[k] = 0.0f, eps[k] = 0.0f;
#pragma unroll
      for (int k = 0; k < M; ++k) y[k] = 0.0f;
      t = 0.5f;
    }
    // VP-SDE terms at t (sdes.py:21-44) and their t-derivatives
    const float ex = __expf(-0.5f * t * t * p.bdiff - t * p.bmin);
    const float alpha = __expf(-0.25f * t * t * p.bdiff - 0.5f * t * p.bmin);
    const float std_ = sqrtf(1.0f - ex);
    const float beta = p.bmin + p.bdiff * t;
    const float gg = sqrtf(beta);
    const float dalpha = alpha * (-0.5f * t * p.bdiff - 0.5f * p.bmin);
    const float dstd = ex * (t * p.bdiff + p.bmin) / (2.0f * std_);
    const float dg = p.bdiff / (2.0f * gg);
    // the per-sample terms divide by g(t) about 20 times: one correctly rounded reciprocal, then products (each a
    // full-precision fp32 division expands to ~10 VALU; the products differ by at most an ulp, far inside the
    // kernel's gates, tests/test_gpu_parity.py)
    const float igg = 1.0f / gg;
    float xt[D], xd[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
      xt[k] = eps[k] * std_ + alpha * x[k];
      xd[k] = dalpha * x[k] + dstd * eps[k];
    }
    float uP[IN], uV[IN], uC[IN];
#pragma unroll
    for (int k = 0; k < D; ++k) uP[k] = xt[k], uV[k] = xd[k], uC[k] = x[k];
#pragma unroll
    for (int k = 0; k < M; ++k) uP[D + k] = y[k], uV[D + k] = 0.0f, uC[D + k] = y[k];
    uP[IN - 1] = t, uV[IN - 1] = 1.0f, uC[IN - 1] = 0.0f;
    const bf16x8 BP = b1_operand(uP, 1.0f, g), BV = b1_operand(uV, 0.0f, g), BC = b1_operand(uC, 1.0f, g);

    float abP[OUT], abV[OUT], abC[OUT];
    if constexpr (PH >= 2) {  // the forward half's adjoints and loss terms of this sample
      const float4* rec = (const float4*)(p.adj + (valid ? si : 0) * kTrainAdj);
      const float4 r0 = REC ? in_cur.a0 : rec[0], r1 = REC ? in_cur.a1 : rec[1], r2 = REC ? in_cur.a2 : rec[2];
      const bool ok = valid;
      abP[0] = ok ? r0.x : 0.0f, abP[1] = ok ? r0.y : 0.0f, abV[0] = ok ? r0.z : 0.0f, abV[1] = ok ? r0.w : 0.0f;
      abC[0] = ok ? r1.x : 0.0f, abC[1] = ok ? r1.y : 0.0f;
      if (valid && g == 0) {
        lsum[0] += r1.z;
        lsum[1] += r1.w;
        lsum[2] += r2.x;
      }
    } else {
    // ======================================================== pass F: forward with jets
    float aS[NSTREAM][OUT];
    {
      // the record reverse half's input (PH 1 with p.rec; a uniform branch per layer)
#ifdef DMIP_TRAIN_TIMING_NO_REC_STORE
      const bool recw = false;  // timing ablation only (A/B builds): the forward half writes no records
#else
      const bool recw = PH == 1 && p.rec != nullptr;
#endif
      const __amdgpu_buffer_rsrc_t rr = rec_rsrc<NL>(recw ? p.rec : (uint32_t*)p.adj, tile);
      bf16x8 H[NSTREAM][2], HL[3][2];  // HL: lo residuals of the split streams P, V, C
#pragma unroll
      for (int R = 0; R < 4; ++R) {
        const bf16x8 a = frag(a1r, R, lane);
        const f32x4 zP = mfma16(a, BP, f32x4{}), zV = mfma16(a, BV, f32x4{}), zC = mfma16(a, BC, f32x4{});
        float cd1[4], cb[4], cd1c[4];  // records: the reverse's coefficients
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int u = 16 * R + 4 * g + r;
          const float pz = tanh_f(zP[r]), h = tanh_f(pz);
          const float q = 1.0f - pz * pz, k1 = 1.0f - h * h;
          const float d1 = k1 * q, d2 = -2.0f * q * (h * d1 + pz * k1);
          const float w0 = col[u], w1 = col[W + u];
          const float pc = tanh_f(zC[r]), hc = tanh_f(pc);
          const float v[NSTREAM] = {h, d1 * zV[r], hc, d1 * w0, d1 * w1,
                                    d2 * w0 * w0, d2 * w0 * w1, d2 * w1 * w1};
#pragma unroll
          for (int S = 0; S < NSTREAM; ++S) H[S][R >> 1][4 * (R & 1) + r] = bf_hi(v[S]);
#pragma unroll
          for (int S = 0; S < 3; ++S) HL[S][R >> 1][4 * (R & 1) + r] = bf_lo(v[S]);
          // the reverse's layer-1 coefficients (pass B, li == 0): d1, d2 z_V, d1_C of the double tanh
          cd1[r] = d1, cb[r] = d2 * zV[r], cd1c[r] = (1.0f - hc * hc) * (1.0f - pc * pc);
        }
        if (recw) {
          rec_put_coef<NL>(rr, 0, R, lane, cd1, cb, cd1c);
          if (R & 1) rec_put_h<NL>(rr, 0, R >> 1, lane, *(const bf16x8(*)[3][2])H);
        }
      }
#pragma unroll
      for (int l = 1; l < NL; ++l) {
        bf16x8 Hn[NSTREAM][2], HLn[3][2];
        const char* wl = wfr + (l - 1) * 8192;
        const char* wll = lds + L::WFL + (l - 1) * 8192;
#pragma unroll
        for (int R = 0; R < 4; ++R) {
          const bf16x8 a0 = frag(wl, 2 * R, lane), a1 = frag(wl, 2 * R + 1, lane);
          const bf16x8 l0 = frag(wll, 2 * R, lane), l1 = frag(wll, 2 * R + 1, lane);
          f32x4 bt;
#pragma unroll
          for (int r = 0; r < 4; ++r) bt[r] = bias[l * W + 16 * R + 4 * g + r];
          f32x4 Z[NSTREAM];
#pragma unroll
          for (int S = 0; S < NSTREAM; ++S) {
            Z[S] = (S == 0 || S == 2) ? bt : f32x4{};
            if (S < 3) Z[S] = mm3(a0, a1, l0, l1, H[S], HL[S], Z[S]);
            else Z[S] = mm(a0, a1, H[S], Z[S]);
          }
          float cd1[4], cb[4], cd1c[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float h = tanh_f(Z[0][r]);
            const float d1 = 1.0f - h * h, d2 = -2.0f * h * d1;
            const float hc = tanh_f(Z[2][r]);
            const float v[NSTREAM] = {h,
                                      d1 * Z[1][r],
                                      hc,
                                      d1 * Z[3][r],
                                      d1 * Z[4][r],
                                      d1 * Z[5][r] + d2 * Z[3][r] * Z[3][r],
                                      d1 * Z[6][r] + d2 * Z[3][r] * Z[4][r],
                                      d1 * Z[7][r] + d2 * Z[4][r] * Z[4][r]};
#pragma unroll
            for (int S = 0; S < NSTREAM; ++S) Hn[S][R >> 1][4 * (R & 1) + r] = bf_hi(v[S]);
#pragma unroll
            for (int S = 0; S < 3; ++S) HLn[S][R >> 1][4 * (R & 1) + r] = bf_lo(v[S]);
            cd1[r] = d1, cb[r] = d2 * Z[1][r], cd1c[r] = 1.0f - hc * hc;
          }
          if (recw) {
            rec_put_coef<NL>(rr, l, R, lane, cd1, cb, cd1c);
            if (R & 1) rec_put_h<NL>(rr, l, R >> 1, lane, *(const bf16x8(*)[3][2])Hn);
          }
        }
#pragma unroll
        for (int S = 0; S < NSTREAM; ++S) H[S][0] = Hn[S][0], H[S][1] = Hn[S][1];
#pragma unroll
        for (int S = 0; S < 3; ++S) HL[S][0] = HLn[S][0], HL[S][1] = HLn[S][1];
      }
      const bf16x8 o0 = frag(aor, 0, lane), o1 = frag(aor, 1, lane);
      const bf16x8 ol0 = frag(lds + L::AOL, 0, lane), ol1 = frag(lds + L::AOL, 1, lane);
      f32x4 bo{};
#pragma unroll
      for (int r = 0; r < OUT; ++r) bo[r] = bias[NL * W + r];
#pragma unroll
      for (int S = 0; S < NSTREAM; ++S) {
        f32x4 acc = (S == 0 || S == 2) ? bo : f32x4{};
        if (S < 3) acc = mm3(o0, o1, ol0, ol1, H[S], HL[S], acc);
        else acc = mm(o0, o1, H[S], acc);
#pragma unroll
        for (int k = 0; k < OUT; ++k) aS[S][k] = acc[k];
      }
    }

    // ======================================================== per-sample loss terms and adjoints
    {
      float s[OUT], dLds[OUT];
#pragma unroll
      for (int k = 0; k < OUT; ++k) s[k] = aS[0][k] * igg, dLds[k] = 0.0f, abV[k] = 0.0f, abC[k] = 0.0f;
      float dsm = 0.0f;
#pragma unroll
      for (int k = 0; k < OUT; ++k) {
        const float rr = s[k] * std_ + eps[k];
        dsm += 0.5f * rr * rr;
        if (p.has_dsm) dLds[k] += rr * std_ * p.inv_n;
      }
      float pde = 0.0f;
      if (p.pde != 0) {
        float dsdt[OUT], u[OUT], dds[OUT];
#pragma unroll
        for (int k = 0; k < OUT; ++k) dsdt[k] = aS[1][k] * igg - aS[0][k] * dg * (igg * igg);
        if (p.pde == 1) {  // ScoreFPELoss (losses.py:78-98)
          float J[OUT][D];
#pragma unroll
          for (int i = 0; i < OUT; ++i)
#pragma unroll
            for (int a = 0; a < D; ++a) J[i][a] = aS[3 + a][i] * igg;
          // second-order streams: 5 = (0,0), 6 = (0,1), 7 = (1,1)
#pragma unroll
          for (int j = 0; j < D; ++j) {
            float gx = s[j];
#pragma unroll
            for (int i = 0; i < OUT; ++i) {
              const int lo = i < j ? i : j, hi = i < j ? j : i;
              const int sidx = lo == 0 ? (hi == 0 ? 5 : 6) : 7;
              gx += aS[sidx][i] * igg + (2.0f * s[i] + xt[i]) * J[i][j];
            }
            u[j] = dsdt[j] - 0.5f * beta * gx;
          }
          float rows = 0.0f;
#pragma unroll
          for (int k = 0; k < OUT; ++k) {
            rows += p.pde_l1 ? fabsf(u[k]) : u[k] * u[k];
            dds[k] = p.pde_l1 ? sgn(u[k]) / OUT : 2.0f * u[k] / OUT;
          }
          pde = p.lam * rows / OUT;
        } else {  // ConditionalScoreFPELoss (losses.py:100-124)
          const float s3 = std_ * std_ * std_;
          float rows = 0.0f;
#pragma unroll
          for (int k = 0; k < OUT; ++k) {
            u[k] = s3 * dsdt[k] - 0.5f * eps[k] * beta * alpha * alpha;
            rows += p.pde_l1 ? fabsf(u[k]) : u[k] * u[k];
            dds[k] = (p.pde_l1 ? sgn(u[k]) : 2.0f * u[k]) * s3;
          }
          pde = p.lam * rows;
        }
#pragma unroll
        for (int k = 0; k < OUT; ++k) {
          const float c = p.lam * dds[k] * p.inv_n;
          abV[k] = c * igg;
          dLds[k] += c * (-dg * igg);
        }
      }
      float ic = 0.0f;
      if (p.has_ic) {  // initial condition (losses.py:213-219) with the linear problem's score
        const float g0 = sqrtf(p.bmin);
        float res[M];
#pragma unroll
        for (int i = 0; i < M; ++i) res[i] = y[i] - (p.icA[i * D + 0] * x[0] + p.icA[i * D + 1] * x[1] + p.icb[i]);
        float rs[M];
#pragma unroll
        for (int jj = 0; jj < M; ++jj) rs[jj] = res[0] * p.icS[jj * M + 0] + res[1] * p.icS[jj * M + 1];
        float rows = 0.0f;
#pragma unroll
        for (int k = 0; k < D; ++k) {
          const float target = -x[k] + rs[0] * p.icA[0 * D + k] + rs[1] * p.icA[1 * D + k];
          const float dl = aS[2][k] / g0 - target;
          rows += p.ic_l1 ? fabsf(dl) : dl * dl;
          const float dd = p.lam2 * (p.ic_l1 ? sgn(dl) : 2.0f * dl) / D;
          abC[k] = dd * p.inv_n / g0;
        }
        ic = p.lam2 * rows / D;
      }
#pragma unroll
      for (int k = 0; k < OUT; ++k) abP[k] = dLds[k] * igg;
      if (!valid) {
#pragma unroll
        for (int k = 0; k < OUT; ++k) abP[k] = abV[k] = abC[k] = 0.0f;
      } else if (g == 0) {
        lsum[0] += dsm;
        lsum[1] += ic;
        lsum[2] += pde;
        if constexpr (PH == 1) {
          float4* rec = (float4*)(p.adj + si * kTrainAdj);
          rec[0] = make_float4(abP[0], abP[1], abV[0], abV[1]);
          rec[1] = make_float4(abC[0], abC[1], dsm, ic);
          rec[2] = make_float4(pde, 0.0f, 0.0f, 0.0f);
        }
      }
    }
    }  // PH != 2
    if constexpr (PH == 1) continue;

    // ======================================================== pass B: reverse with recomputation
    f32x4 hbar[3][4];  // adjoint of the current layer's output, streams P, V, C (acc form)
    // the reverse half is specialised per layer (every branch on li and the bias-partial index constant);
    // the fused kernel keeps the loop (its code size)
    constexpr int kLiUnroll = PH >= 2 ? NL + 1 : 1;
#pragma unroll kLiUnroll
    for (int li = NL; li >= 0; --li) {
      if constexpr (L::OWN) sbuf ^= 1;
      // ---- recompute P, V, C forward: h_{li-1} (B form + transposed into scratch 3..5) and z_li
      bf16x8 H[3][2], HL[3][2];
      f32x4 Z[3][4];
      if constexpr (REC) {  // h_{li-1} from the records instead: the recompute's put_t, bit for bit, 16-bit stores
        if (li >= 1) {
#pragma unroll
          for (int S = 0; S < 3; ++S) {
            __bf16* sc = S_(3 + S);
#pragma unroll
            for (int R = 0; R < 4; ++R)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const uint32_t wd = rc[li >= 1 ? li - 1 : 0][S][R >> 1][2 * (R & 1) + (r >> 1)];
                sc[sidx<RS>(16 * R + 4 * g + r, c16)] = __builtin_bit_cast(__bf16, (uint16_t)((r & 1) ? wd >> 16 : wd));
              }
          }
        }
      } else {
#pragma unroll
        for (int R = 0; R < 4; ++R) {
          const bf16x8 a = frag(a1r, R, lane);
          Z[0][R] = mfma16(a, BP, f32x4{});
          Z[1][R] = mfma16(a, BV, f32x4{});
          Z[2][R] = mfma16(a, BC, f32x4{});
        }
#pragma unroll
        for (int l = 1; l <= NL; ++l) {
          if (l > li) break;
          // activation of layer l-1 -> H
          f32x4 Hf[3][4];
#pragma unroll
          for (int R = 0; R < 4; ++R)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float h, d1, hc;
              if (l == 1) {
                const float pz = tanh_f(Z[0][R][r]);
                h = tanh_f(pz);
                d1 = (1.0f - h * h) * (1.0f - pz * pz);
                hc = tanh_f(tanh_f(Z[2][R][r]));
              } else {
                h = tanh_f(Z[0][R][r]);
                d1 = 1.0f - h * h;
                hc = tanh_f(Z[2][R][r]);
              }
              Hf[0][R][r] = h;
              Hf[1][R][r] = d1 * Z[1][R][r];
              Hf[2][R][r] = hc;
            }
#pragma unroll
          for (int S = 0; S < 3; ++S) pack_b2(Hf[S], H[S], HL[S]);
          if (l == li) {
#pragma unroll
            for (int S = 0; S < 3; ++S) put_t<RS>(S_(3 + S), Hf[S], g, c16);
          }
          if (l == NL) break;  // li == NL: the output layer's pre-activation is not needed
          const char* wl = wfr + (l - 1) * 8192;
          const char* wll = lds + L::WFL + (l - 1) * 8192;
#pragma unroll
          for (int R = 0; R < 4; ++R) {
            const bf16x8 a0 = frag(wl, 2 * R, lane), a1 = frag(wl, 2 * R + 1, lane);
            const bf16x8 l0 = frag(wll, 2 * R, lane), l1 = frag(wll, 2 * R + 1, lane);
            f32x4 bt;
#pragma unroll
            for (int r = 0; r < 4; ++r) bt[r] = bias[l * W + 16 * R + 4 * g + r];
#pragma unroll
            for (int S = 0; S < 3; ++S) Z[S][R] = mm3(a0, a1, l0, l1, H[S], HL[S], S == 1 ? f32x4{} : bt);
          }
        }
      }

      if (li == NL) {
        // ---- output layer: zbar = abar (per sample); W_NL-bar += abar h^T; b-bar; h-bar = W^T abar
        const float* ab[3] = {abP, abV, abC};
        if (g == 0) {
#pragma unroll
          for (int S = 0; S < 3; ++S)
#pragma unroll
            for (int o = 0; o < OUT; ++o) S_(S)[sidx<RS>(o, c16)] = (__bf16)ab[S][o];
#pragma unroll
          for (int o = 0; o < OUT; ++o) bobar[o] += abP[o] + abC[o];
        }
        if constexpr (L::OWN) {
          turn_barrier();  // every wave's scratch of this layer has landed
          if (w >= 2) {    // the output layer's block U = w - 2, over the four waves' tiles
            const int U = w - 2;
#pragma unroll
            for (int v = 0; v < 4; ++v)
#pragma unroll
              for (int S = 0; S < 3; ++S) {
                const bf16x8 A = tread<RS>(SV(v, S), i32, i32 < OUT, hh);
                const bf16x8 Bm = tread<RS>(SV(v, 3 + S), 32 * U + i32, true, hh);
                DMIP_TRAIN_CONTRACT(gX = mfma32(A, Bm, gX));
              }
          }
        } else {
          __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's scratch writes landed
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int U = 0; U < 2; ++U) {
            f32x16 acc{};
#pragma unroll
            for (int S = 0; S < 3; ++S) {
              const bf16x8 A = tread<RS>(S_(S), i32, i32 < OUT, hh);
              const bf16x8 Bm = tread<RS>(S_(3 + S), 32 * U + i32, true, hh);
              acc = mfma32(A, Bm, acc);
            }
            if (hh == 0) {
#pragma unroll
              for (int o = 0; o < OUT; ++o) gadd<GACC_GLOBAL>(&gacc[L::p_w(NL) + o * W + 32 * U + i32], acc[o]);
            }
          }
        }
#pragma unroll
        for (int S = 0; S < 3; ++S) {
          bf16x8 Bm{};
#pragma unroll
          for (int j = 0; j < OUT; ++j) Bm[j] = g == 0 ? (__bf16)ab[S][j] : (__bf16)0.0f;
#pragma unroll
          for (int R = 0; R < 4; ++R) hbar[S][R] = mfma16(frag(aotr, R, lane), Bm, f32x4{});
        }
        __builtin_amdgcn_wave_barrier();
        continue;
      }

      // ---- tanh layer li (li == 0: the double tanh of layer 1): zbar from hbar
      f32x4 zb[3][4];
      if constexpr (REC) {  // the coefficients from the records
        const int lr = li < NL ? li : 0;
#pragma unroll
        for (int R = 0; R < 4; ++R)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float d1 = rec_val<true>(rc[lr][3], R, r), b = rec_val<false>(rc[lr][4], R, r);
            const float d1c = rec_val<true>(rc[lr][5], R, r);
            zb[0][R][r] = d1 * hbar[0][R][r] + b * hbar[1][R][r];
            zb[1][R][r] = d1 * hbar[1][R][r];
            zb[2][R][r] = d1c * hbar[2][R][r];
          }
        rec_load(tile + tile_step, lr);  // this tile is done with layer lr's records: the next tile's
      } else {
#pragma unroll
      for (int R = 0; R < 4; ++R)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float d1, d2, d1c;
          if (li == 0) {
            const float pz = tanh_f(Z[0][R][r]), h = tanh_f(pz);
            const float q = 1.0f - pz * pz, k1 = 1.0f - h * h;
            d1 = k1 * q;
            d2 = -2.0f * q * (h * d1 + pz * k1);
            const float pc = tanh_f(Z[2][R][r]), hc = tanh_f(pc);
            d1c = (1.0f - hc * hc) * (1.0f - pc * pc);
          } else {
            const float h = tanh_f(Z[0][R][r]);
            d1 = 1.0f - h * h;
            d2 = -2.0f * h * d1;
            const float hc = tanh_f(Z[2][R][r]);
            d1c = 1.0f - hc * hc;
          }
          zb[0][R][r] = d1 * hbar[0][R][r] + d2 * Z[1][R][r] * hbar[1][R][r];
          zb[1][R][r] = d1 * hbar[1][R][r];
          zb[2][R][r] = d1c * hbar[2][R][r];
        }
      }
#pragma unroll
      for (int S = 0; S < 3; ++S) put_t<RS>(S_(S), zb[S], g, c16);
      if (li == 0) {
        // layer-1 inputs transposed: rows 0..IN-1 = u, row IN = the bias column (1 for P and C)
        if (g == 0) {
          const float* us[3] = {uP, uV, uC};
#pragma unroll
          for (int S = 0; S < 3; ++S) {
#pragma unroll
            for (int k = 0; k < IN; ++k) S_(3 + S)[sidx<RS>(k, c16)] = (__bf16)us[S][k];
            S_(3 + S)[sidx<RS>(IN, c16)] = (__bf16)(S == 1 ? 0.0f : 1.0f);
          }
        }
      } else if (li >= 1) {
#pragma unroll
        for (int R = 0; R < 4; ++R) bbar[(li - 1) > 0 ? li - 1 : 0][R] += zb[0][R] + zb[2][R];
      }
      if constexpr (L::OWN) {
        turn_barrier();  // every wave's scratch of this layer has landed
        if (li == 0) {
          if (w < 2) {  // layer 1's block T = w (weight columns i32 < IN, the bias at i32 == IN)
#pragma unroll
            for (int v = 0; v < 4; ++v)
#pragma unroll
              for (int S = 0; S < 3; ++S) {
                const bf16x8 A = tread<RS>(SV(v, S), 32 * w + i32, true, hh);
                const bf16x8 Bm = tread<RS>(SV(v, 3 + S), i32, i32 <= IN, hh);
                DMIP_TRAIN_CONTRACT(gX = mfma32(A, Bm, gX));
              }
          }
        } else {  // W x W layer li: block (T, U) = (w >> 1, w & 1)
          const int T = w >> 1, U = w & 1;
#pragma unroll
          for (int v = 0; v < 4; ++v)
#pragma unroll
            for (int S = 0; S < 3; ++S) {
              const bf16x8 A = tread<RS>(SV(v, S), 32 * T + i32, true, hh);
              const bf16x8 Bm = tread<RS>(SV(v, 3 + S), 32 * U + i32, true, hh);
              DMIP_TRAIN_CONTRACT(gW[(li - 1) > 0 ? li - 1 : 0] = mfma32(A, Bm, gW[(li - 1) > 0 ? li - 1 : 0]));
            }
        }
      } else {
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
      }
      if (li == 0) {
        if constexpr (!L::OWN) {
#pragma unroll
          for (int T = 0; T < 2; ++T) {
            f32x16 acc{};
#pragma unroll
            for (int S = 0; S < 3; ++S) {
              const bf16x8 A = tread<RS>(S_(S), 32 * T + i32, true, hh);
              const bf16x8 Bm = tread<RS>(S_(3 + S), i32, i32 <= IN, hh);
              acc = mfma32(A, Bm, acc);
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int row = 32 * T + (r & 3) + 8 * (r >> 2) + 4 * hh;
              if (i32 < IN) gadd<GACC_GLOBAL>(&gacc[L::p_w(0) + row * IN + i32], acc[r]);
              else if (i32 == IN) gadd<GACC_GLOBAL>(&gacc[L::p_b(0) + row], acc[r]);
            }
          }
        }
      } else {
        const int pw = L::p_w(li);
#pragma unroll
        for (int T = 0; T < 2 && !L::OWN; ++T)
#pragma unroll
          for (int U = 0; U < 2; ++U) {
            f32x16 acc{};
#pragma unroll
            for (int S = 0; S < 3; ++S) {
              const bf16x8 A = tread<RS>(S_(S), 32 * T + i32, true, hh);
              const bf16x8 Bm = tread<RS>(S_(3 + S), 32 * U + i32, true, hh);
              acc = mfma32(A, Bm, acc);
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int row = 32 * T + (r & 3) + 8 * (r >> 2) + 4 * hh;
              gadd<GACC_GLOBAL>(&gacc[pw + row * W + 32 * U + i32], acc[r]);
            }
          }
        // h-bar of layer li-1 = W_li^T zbar
        const char* wl = wtr + (li - 1) * 8192;
#pragma unroll
        for (int S = 0; S < 3; ++S) {
          bf16x8 zbB[2];
          pack_b(zb[S], zbB);
#pragma unroll
          for (int R = 0; R < 4; ++R) {
            f32x4 acc = mfma16(frag(wl, 2 * R, lane), zbB[0], f32x4{});
            hbar[S][R] = mfma16(frag(wl, 2 * R + 1, lane), zbB[1], acc);
          }
        }
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
    }
  }

  if constexpr (PH == 1) return;  // the forward half: its adjoints and loss terms are in p.adj
  // ---- flush: bias partials (reduce the 16 sample lanes of each lane group) and loss sums; OWN: the weight
  // blocks straight from registers to the workgroup's row; each wave reduces its bias / loss partials over its 16
  // sample lanes by DPP row shifts (no LDS, all waves at once), the four waves' results meet in LDS in wave order
  // (one barrier; deterministic), then that partial goes to the row. (Round 5 reduced by lane shuffles, one wave at a
  // time: ~128 dependent LDS permutes per wave, serialised over the four waves -- a fixed cost of every launch.)
  if constexpr (L::OWN) {
    float* row = p.partials + (size_t)blockIdx.x * L::PART;
    {
      const int T = w >> 1, U = w & 1;
#pragma unroll
      for (int l = 1; l < NL; ++l)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          row[L::p_w(l) + (32 * T + (r & 3) + 8 * (r >> 2) + 4 * hh) * W + 32 * U + i32] = gW[l - 1][r];
    }
    if (w < 2) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rr = 32 * w + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (i32 < IN) row[L::p_w(0) + rr * IN + i32] = gX[r];
        else if (i32 == IN) row[L::p_b(0) + rr] = gX[r];
      }
    } else if (hh == 0) {  // output rows o < OUT sit in registers o of lane half 0
#pragma unroll
      for (int o = 0; o < OUT; ++o) row[L::p_w(NL) + o * W + 32 * (w - 2) + i32] = gX[o];
    }
    constexpr int NB = (NL - 1) * W + OUT + 3;  // hidden biases, output bias, loss sums
    float* bp = gacc;                            // [NWV][NB] in the (now free) scratch
    turn_barrier();  // the last tile's scratch reads are done
#pragma unroll
    for (int l = 0; l < NL - 1; ++l)
#pragma unroll
      for (int R = 0; R < 4; ++R)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = row_sum16(bbar[l][R][r]);
          if (c16 == 15) bp[w * NB + l * W + 16 * R + 4 * g + r] = v;
        }
    // the output bias and the loss sums live in lane group 0 only: row 0's sum is the wave's
#pragma unroll
    for (int o = 0; o < OUT; ++o) {
      const float v = row_sum16(g == 0 ? bobar[o] : 0.0f);
      if (lane == 15) bp[w * NB + (NL - 1) * W + o] = v;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float v = row_sum16(g == 0 ? lsum[k] : 0.0f);
      if (lane == 15) bp[w * NB + (NL - 1) * W + OUT + k] = v;
    }
    turn_barrier();
    for (int e = tid; e < NB; e += NWV * 64) {
      float v = bp[e];
#pragma unroll
      for (int v_ = 1; v_ < NWV; ++v_) v += bp[v_ * NB + e];
      const int idx = e < (NL - 1) * W ? L::p_b(e / W + 1) + e % W
                                       : (e < (NL - 1) * W + OUT ? L::p_b(NL) + e - (NL - 1) * W
                                                                 : L::NPARAM + e - (NL - 1) * W - OUT);
      row[idx] = v;
    }
    return;
  }
  for (int turn = 0; turn < (L::OWN ? NWV : 1); ++turn) {
    if constexpr (L::OWN) {
      turn_barrier();
      if (w != turn) continue;
    }
#pragma unroll
  for (int l = 0; l < NL - 1; ++l)
#pragma unroll
    for (int R = 0; R < 4; ++R)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = bbar[l][R][r];
#pragma unroll
        for (int m = 1; m < 16; m <<= 1) v += __shfl_xor(v, m, 64);
        if (c16 == 0) gadd<GACC_GLOBAL>(&gacc[L::p_b(l + 1) + 16 * R + 4 * g + r], v);
      }
#pragma unroll
  for (int o = 0; o < OUT; ++o) {
    float v = g == 0 ? bobar[o] : 0.0f;
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) v += __shfl_xor(v, m, 64);
    if (lane == 0) gadd<GACC_GLOBAL>(&gacc[L::p_b(NL) + o], v);
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    float v = lsum[k];
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) v += __shfl_xor(v, m, 64);
    if (lane == 0) {
      if constexpr (L::OWN) gacc[L::NPARAM + k] += v;
      else gacc[L::NPARAM + k] = v;
    }
  }
  }  // turns
  if constexpr (L::OWN) {
    turn_barrier();
    float* row = p.partials + (size_t)blockIdx.x * L::PART;
    // the hidden and output biases and the loss sums (the weight blocks and layer 1's bias are in the row already)
    for (int e = tid; e < L::PART; e += NWV * 64) {
      bool mine = e >= L::NPARAM || (e >= L::p_b(NL) && e < L::p_b(NL) + OUT);
#pragma unroll
      for (int l = 1; l < NL; ++l) mine |= e >= L::p_b(l) && e < L::p_b(l) + W;
      if (mine) row[e] = gacc[e];
    }
    return;
  }
  if constexpr (GACC_GLOBAL) {
    // fold the workgroup's NWV rows into its first row, in wave order (deterministic), so the
    // reduction reads one row per workgroup
    __threadfence();
    __syncthreads();
    float* rows = p.partials + (size_t)blockIdx.x * NWV * L::PART;
    // the rows were updated by L2 atomics: read them at agent scope (past this CU's L1)
    auto rd = [](float* a) { return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    for (int e = tid; e < L::PART; e += NWV * 64) {
      float v = rd(rows + e);
#pragma unroll
      for (int ww = 1; ww < NWV; ++ww) v += rd(rows + (size_t)ww * L::PART + e);
      rows[e] = v;
    }
    return;
  }
  // one partial per workgroup: wave 0's region + wave 1's region, in that order (deterministic)
  __syncthreads();
  float* part = p.partials + (size_t)blockIdx.x * L::PART;
  const float* g0 = (const float*)(lds + L::IMG + L::GACC);
  for (int e = tid; e < L::PART; e += NWV * 64) {
    float v = g0[e];
#pragma unroll
    for (int ww = 1; ww < NWV; ++ww) v += ((const float*)(lds + L::IMG + ww * L::WAVE_BYTES + L::GACC))[e];
    part[e] = v;
  }
}

// grads[k] = sum over the per-workgroup partials in a fixed order (deterministic); slots nparam..+2
// are the DSM / IC / PDE row sums -> loss_out = {loss, PDE, IC, DSM} means. 64 slots per block, the
// partials split over kRedGroups thread groups (rows g, g + 16, ...), combined in LDS in group order (f64).
// total_flags (bit 0 DSM, 1 IC, 2 PDE, bit 3 = set): the block holding the three loss slots also writes
// loss_out[0] (their sum, as loss_total_kernel), saving that launch.
// ADAM (the captured bf16 step's last launch, TrainFuse): then torch's Adam on each parameter its thread has just
// summed (the same float the separate adam_kernel would read back from .grad), and in the last workgroup to finish
// (a counter of finished workgroups) the step counters' advance. Every workgroup reads the step counter before it
// counts itself finished, so the advance follows all of this step's reads.
constexpr int kRedGroups = 16;  // 1024 threads: 16 rows in flight per slot (4 groups left the reduction latency-bound)
template <bool ADAM>
__global__ void __launch_bounds__(64 * kRedGroups) loss_grad_reduce_kernel(const float* partials, int n_parts,
                                                                          int stride, int nparam, float* grads,
                                                                          float* loss_out, float inv_n, int total_flags,
                                                                          AdamParams ap, StepCounters* ctr) {
  __shared__ double red[kRedGroups][64];
  __shared__ float lm[3];
  __shared__ stepdev::AdamScalars sc;  // ADAM: the step's scalars once per workgroup (double pow)
  const int pi = threadIdx.x & 63, pg = threadIdx.x >> 6;
  const int k = blockIdx.x * 64 + pi;
  if (ADAM && threadIdx.x == 64) sc = stepdev::adam_scalars(ap);
  double s = 0.0;
  if (k < nparam + 3) {
#pragma unroll 4
    for (int i = pg; i < n_parts; i += kRedGroups) s += (double)partials[(size_t)i * stride + k];
  }
  red[pg][pi] = s;
  __syncthreads();
  if (pg == 0 && k < nparam + 3) {
    s = red[0][pi];
#pragma unroll
    for (int q = 1; q < kRedGroups; ++q) s += red[q][pi];
    if (k < nparam) {
      const float gk = (float)s;
      grads[k] = gk;
      if constexpr (ADAM) stepdev::adam_one(ap, sc, k, gk);
    } else {
      const float mean = (float)(s * inv_n);
      const int c = k - nparam;  // 0 DSM, 1 IC, 2 PDE
      loss_out[3 - c] = mean;
      lm[c] = mean;
    }
  }
  if ((total_flags & 8) && blockIdx.x == (unsigned)(nparam / 64)) {
    __syncthreads();
    if (threadIdx.x == 0)
      loss_out[0] = ((total_flags & 1) ? lm[0] : 0.0f) + ((total_flags & 2) ? lm[1] : 0.0f) + ((total_flags & 4) ? lm[2] : 0.0f);
  }
  if constexpr (ADAM) {
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence();
      if (atomicAdd(&ctr->done, 1u) == gridDim.x - 1) {  // the last workgroup: every read of the counters is done
        ctr->done = 0u;
        ctr->draw += 1;
        ctr->step += 1;
      }
    }
  }
}

__global__ void loss_total_kernel(float* loss_out, int has_dsm, int has_ic, int has_pde) {
  loss_out[0] = (has_dsm ? loss_out[3] : 0.0f) + (has_ic ? loss_out[2] : 0.0f) + (has_pde ? loss_out[1] : 0.0f);
}

// The captured bf16 step's first launch (TrainFuse): workgroups [0, n_pack) pack the weight image
// (train_pack_kernel's work), the rest draw t and eps (and stage the batch) as train_draws_kernel
template <int NL>
__global__ void __launch_bounds__(256) plan_prologue_kernel(TrainDrawsParams dp, TrainParams tp, int n_pack) {
  if ((int)blockIdx.x < n_pack) {
    pack_weights<NL>(tp, tp.packed, blockIdx.x * blockDim.x + threadIdx.x, n_pack * blockDim.x);
    return;
  }
  stepdev::draw_one(dp, (long long)(blockIdx.x - n_pack) * blockDim.x + threadIdx.x);
}


}  // namespace train

constexpr int kPackBlocks = 32;  // train_pack_kernel's grid (and the pack part of plan_prologue_kernel's)

// the forward / reverse split (two kernels at two waves per SIMD) or the fused one-wave-per-SIMD kernel;
// DMIP_TRAIN_SPLIT=0 selects the fused kernel (A/B knob, read once per process)
bool train_split() {
  static const bool v = [] {
    const char* e = getenv("DMIP_TRAIN_SPLIT");
    return e ? atoi(e) != 0 : true;
  }();
  return v;
}

// the record reverse half (loss_grad_kernel<NL, 3>) or the recomputing one (<NL, 2>); DMIP_TRAIN_REC=0 selects the
// latter (A/B knob, read once per process)
bool train_rec() {
  static const bool v = [] {
    const char* e = getenv("DMIP_TRAIN_REC");
    return e ? atoi(e) != 0 : true;
  }();
  return v;
}

// the records follow the adjoint rows in the adj allocation (train_adj_bytes)
static size_t rec_offset(long long batch) { return ((size_t)batch * kTrainAdj * sizeof(float) + 255) / 256 * 256; }
static uint32_t* rec_ptr(float* adj, long long batch) {
  return adj && train_rec() ? (uint32_t*)((char*)adj + rec_offset(batch)) : nullptr;
}

// the reverse half's kernel
template <int NL>
static void launch_reverse(const TrainParams& q, int n_wg, hipStream_t st) {
  using namespace train;
  if (q.rec)
    hipLaunchKernelGGL((loss_grad_kernel<NL, 3>), dim3(n_wg), dim3(TL<NL, 3>::NW * 64), 0, st, q);
  else
    hipLaunchKernelGGL((loss_grad_kernel<NL, 2>), dim3(n_wg), dim3(TL<NL, 2>::NW * 64), 0, st, q);
}

int train_nparam(int n_hidden) {
  return n_hidden == 3 ? train::TL<3>::NPARAM : (n_hidden == 2 ? train::TL<2>::NPARAM : -1);
}

hipError_t launch_loss_grad(const TrainParams& p, int n_hidden, float* grads, float* loss_out, float* partials,
                            int n_wg, hipStream_t st) {
  using namespace train;
  const int part = n_hidden == 3 ? TL<3>::PART : TL<2>::PART;
  const int nparam = train_nparam(n_hidden);
  TrainParams q = p;
  q.partials = partials;
  q.rec = rec_ptr(p.adj, p.n);
  if (n_hidden == 3)
    hipLaunchKernelGGL(train_pack_kernel<3>, dim3(kPackBlocks), dim3(256), 0, st, q);
  else
    hipLaunchKernelGGL(train_pack_kernel<2>, dim3(kPackBlocks), dim3(256), 0, st, q);
  hipError_t e0 = hipGetLastError();
  if (e0 != hipSuccess) return e0;
  if (train_split()) {
    // forward half: 4-wave workgroups, two per CU (two waves per SIMD); reverse half: the caller's n_wg
    if (!q.adj) return hipErrorInvalidValue;
    const long long tiles = (p.n + NS - 1) / NS;
    const long long g1 = std::min<long long>(2LL * n_wg, (tiles + 3) / 4);
    if (n_hidden == 3) {
      hipLaunchKernelGGL((loss_grad_kernel<3, 1>), dim3((unsigned)g1), dim3(TL<3, 1>::NW * 64), 0, st, q);
      launch_reverse<3>(q, n_wg, st);
    } else {
      hipLaunchKernelGGL((loss_grad_kernel<2, 1>), dim3((unsigned)g1), dim3(TL<2, 1>::NW * 64), 0, st, q);
      launch_reverse<2>(q, n_wg, st);
    }
  } else if (n_hidden == 3) {
    hipLaunchKernelGGL(loss_grad_kernel<3>, dim3(n_wg), dim3(NWV * 64), 0, st, q);
  } else {
    hipLaunchKernelGGL(loss_grad_kernel<2>, dim3(n_wg), dim3(NWV * 64), 0, st, q);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // the loss total rides on the reduction when the three loss slots share one 64-slot block
  const bool fused_total = nparam / 64 == (nparam + 2) / 64;
  const int flags = fused_total ? 8 | (p.has_dsm ? 1 : 0) | (p.has_ic ? 2 : 0) | (p.pde != 0 ? 4 : 0) : 0;
  hipLaunchKernelGGL(loss_grad_reduce_kernel<false>, dim3((nparam + 3 + 63) / 64), dim3(64 * kRedGroups), 0, st,
                     partials, n_wg, part * train_partials_per_wg(), nparam, grads, loss_out, p.inv_n, flags,
                     AdamParams{}, (StepCounters*)nullptr);
  e = hipGetLastError();
  if (e != hipSuccess || fused_total) return e;
  hipLaunchKernelGGL(loss_total_kernel, dim3(1), dim3(1), 0, st, loss_out, p.has_dsm, p.has_ic, p.pde != 0);
  return hipGetLastError();
}

const void* train_plan_prologue_func(int n_hidden) {
  return n_hidden == 3 ? (const void*)train::plan_prologue_kernel<3> : (const void*)train::plan_prologue_kernel<2>;
}

hipError_t launch_loss_grad_fused(const TrainParams& p, int n_hidden, float* grads, float* loss_out, float* partials,
                                  int n_wg, const TrainFuse& f, hipStream_t st) {
  using namespace train;
  if (!train_split() || !p.adj || (n_hidden != 2 && n_hidden != 3)) return hipErrorInvalidValue;
  const int part = n_hidden == 3 ? TL<3>::PART : TL<2>::PART;
  const int nparam = train_nparam(n_hidden);
  if (f.adam.off[f.adam.n] != nparam) return hipErrorInvalidValue;  // Adam's flat order is the gradient's
  TrainParams q = p;
  q.partials = partials;
  q.rec = rec_ptr(p.adj, p.n);
  const unsigned draw_blocks = (unsigned)((f.draws.batch + 255) / 256);
  const dim3 pg(kPackBlocks + draw_blocks), pb(256);
  if (n_hidden == 3)
    hipLaunchKernelGGL(plan_prologue_kernel<3>, pg, pb, 0, st, f.draws, q, kPackBlocks);
  else
    hipLaunchKernelGGL(plan_prologue_kernel<2>, pg, pb, 0, st, f.draws, q, kPackBlocks);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const long long tiles = (p.n + NS - 1) / NS;
  const long long g1 = std::min<long long>(2LL * n_wg, (tiles + 3) / 4);
  if (n_hidden == 3) {
    hipLaunchKernelGGL((loss_grad_kernel<3, 1>), dim3((unsigned)g1), dim3(TL<3, 1>::NW * 64), 0, st, q);
    launch_reverse<3>(q, n_wg, st);
  } else {
    hipLaunchKernelGGL((loss_grad_kernel<2, 1>), dim3((unsigned)g1), dim3(TL<2, 1>::NW * 64), 0, st, q);
    launch_reverse<2>(q, n_wg, st);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const bool fused_total = nparam / 64 == (nparam + 2) / 64;
  const int flags = fused_total ? 8 | (p.has_dsm ? 1 : 0) | (p.has_ic ? 2 : 0) | (p.pde != 0 ? 4 : 0) : 0;
  hipLaunchKernelGGL(loss_grad_reduce_kernel<true>, dim3((nparam + 3 + 63) / 64), dim3(64 * kRedGroups), 0, st,
                     partials, n_wg, part * train_partials_per_wg(), nparam, grads, loss_out, p.inv_n, flags, f.adam,
                     f.ctr);
  if ((e = hipGetLastError()) != hipSuccess || fused_total) return e;
  hipLaunchKernelGGL(loss_total_kernel, dim3(1), dim3(1), 0, st, loss_out, p.has_dsm, p.has_ic, p.pde != 0);
  return hipGetLastError();
}

int train_partial_stride(int n_hidden) { return n_hidden == 3 ? train::TL<3>::PART : train::TL<2>::PART; }
int train_packed_bytes(int n_hidden) { return n_hidden == 3 ? train::TL<3>::WAVE : train::TL<2>::WAVE; }
int train_partials_per_wg() { return train_split() ? 1 : (train::GACC_GLOBAL ? train::NWV : 1); }
int train_waves_per_wg() { return train_split() ? train::TL<3, 2>::NW : train::NWV; }
size_t train_adj_bytes(long long batch) {
  if (!train_split()) return 0;
  if (!train_rec()) return (size_t)batch * kTrainAdj * sizeof(float);
  // the adjoint rows, then the records: 16-sample tiles x at most 3 hidden layers
  return rec_offset(batch) + (size_t)((batch + 15) / 16) * 3 * kTrainRecTileBytes;
}

}  // namespace dmip
