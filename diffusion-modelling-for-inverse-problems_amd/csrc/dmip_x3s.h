// The latency engine of the fp32x3 CDE sampler at width 64 (round 6; BASELINE configs[0], the linear problem's
// [64]^3 networks at 1000 chains x 200 steps).
//
// The one-tile engine (dmip_x3.h) gives a 16-chain tile to one wave, which computes all four 16-unit output tiles of
// every layer itself. At 1000 chains that is 63 waves on a 1024-SIMD chip, and a step is one wave's dependent chain:
// layer 1, two hidden layers and the output layer, each with all four tiles' MFMAs and activations in sequence
// (~2.9 us per step, half of it stalls). Here a tile belongs to a WORKGROUP of four waves: wave w computes output tile
// w of each 64-wide layer (its KQ = 2 k-steps, three split products each, then the activation of its 16 units), the
// four waves swap their activated (hi, lo) fragments through LDS (one ds_write_b128, one barrier, four ds_read_b128 per
// layer), and every wave computes the output tile, the EM update and the RNG of the same 16 chains redundantly, so the
// chain state needs no exchange. Each wave keeps its own tile's weight fragments and biases in registers for the whole
// launch: the step loop reads no weights.
//
// Every value is formed exactly as in the one-tile engine (the same fragments, MFMA order, activations, splits,
// EM update and RNG), so the two engines' samples are bit-identical (tests/test_gpu_x3.py); no hand-over or balanced
// schedule is needed, since a launch has at most kMaxTiles tiles, one per workgroup. (Computing all four layer-1
// tiles in every wave instead of exchanging them was measured slower: 0.375 vs 0.340 ms per config-1 call; so was
// drawing the step's noise before the network instead of after it: 0.260-0.269 vs 0.252-0.254 ms per launch,
// scripts/bench_x3s_kernel.py.)
#pragma once
#include <cstdlib>

#include "dmip_x3.h"

namespace dmip {
namespace x3s {

using x3::f32x4;
using x3::mfma16;

constexpr int W = 64, KQ = x3::Shape<W>::KQ, NWS = x3::Shape<W>::ST;  // 2 k-steps; 4 waves = 4 output tiles
constexpr int CHUNK = x3::Shape<W>::CHUNK;                             // one 64-wide layer's 4 tiles (16 KiB)
static_assert(KQ == 2 && NWS == 4 && x3::Shape<W>::NCH == 1, "one stream chunk per 64-wide layer");
// launches up to this many tiles (all ys) take this engine: one workgroup per tile, <= 4 waves per SIMD (at 4,096
// tiles, 65,536 chains x 200 steps, it took 1.82-1.86 ms against the one-tile engine's 1.49-1.53: DMIP_X3S_MAX_TILES
// A/B build, scripts/archive/gpu_r6_x3s_tiles.sh)
#ifndef DMIP_X3S_MAX_TILES
#define DMIP_X3S_MAX_TILES 1024
#endif
constexpr long long kMaxTiles = DMIP_X3S_MAX_TILES;

__device__ __forceinline__ u32x4 ld16(const char* p) { return *(const u32x4*)p; }
__device__ __forceinline__ f32x4 ld4(const float* p) { return *(const f32x4*)p; }

// activation of this wave's tile into its (hi, lo) dwords: units 4 g + r (r = 0, 1 -> h0 / l0; 2, 3 -> h1 / l1), as
// dmip_x3.h act_store
template <bool L1>
__device__ __forceinline__ void act_split(const f32x4& z, uint32_t& h0, uint32_t& h1, uint32_t& l0, uint32_t& l1) {
  float r[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) r[k] = L1 ? x3::x3_act_r2(z[k]) : x3::x3_act_r(z[k]);
  x3::split_pair(r[0], r[1], h0, l0);
  x3::split_pair(r[2], r[3], h1, l1);
}

// the next layer's B operands from the four waves' tiles: k-step q takes tiles 2q, 2q + 1 (dmip_x3.h layout: dwords
// d, d + 1 of Oh[q] from tile 2q + d / 2). Double-buffered by parity: a wave can reach the next write of a buffer only
// after the barrier of the layer in between, which every wave reaches after its reads of that buffer.
__device__ __forceinline__ void exchange(u32x4 (*xb)[NWS][64], int& par, int w, int lane, uint32_t h0, uint32_t h1,
                                         uint32_t l0, uint32_t l1, u32x4 (&Hh)[KQ], u32x4 (&Hl)[KQ]) {
  xb[par][w][lane] = u32x4{h0, h1, l0, l1};
  __syncthreads();
  const u32x4 t0 = xb[par][0][lane], t1 = xb[par][1][lane], t2 = xb[par][2][lane], t3 = xb[par][3][lane];
  Hh[0] = u32x4{t0.x, t0.y, t1.x, t1.y};
  Hl[0] = u32x4{t0.z, t0.w, t1.z, t1.w};
  Hh[1] = u32x4{t2.x, t2.y, t3.x, t3.y};
  Hl[1] = u32x4{t2.z, t2.w, t3.z, t3.w};
  par ^= 1;
}

// one tile over a 64-wide input: k-step q as W_hi h_lo + W_lo h_hi + W_hi h_hi (dmip_x3.h split_chain order)
__device__ __forceinline__ f32x4 tile64(const u32x4 (&f)[KQ][2], const u32x4 (&Hh)[KQ], const u32x4 (&Hl)[KQ],
                                        f32x4 acc) {
#pragma unroll
  for (int q = 0; q < KQ; ++q) {
    acc = mfma16(f[q][0], Hl[q], acc);
    acc = mfma16(f[q][1], Hh[q], acc);
    acc = mfma16(f[q][0], Hh[q], acc);
  }
  return acc;
}

template <int D, bool NOISE>
__global__ void __launch_bounds__(NWS * 64) x3s_sampler_kernel(X3SamplerParams p) {
  constexpr int NV = D + 1;  // x and tau (y is folded into the per-y layer-1 bias)
  static_assert(D <= 4, "output rows of a chain sit in lane group 0");
  static_assert(x3::k1q_of(NV) == 1 && 3 * NV <= 16, "one-k-step layer 1 over lanes 0-31 (dmip_x3.h XLay L1H)");
  __shared__ u32x4 xb[2][NWS][64];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, j = lane & 15;
  const int yi = blockIdx.y;
  const int nl = p.n_hidden;  // 1..3 (checked by the host)

  // this wave's tile w of every layer, in registers: the layer-1 fragment (lanes 32-63 read lanes 0-31's weights, as
  // the one-tile engine's half image does), the W x W layers' (hi, lo) fragments of chunk li - 1 and the output tile's
  // of chunk nl - 1; the biases (layer 1: the per-y c)
  const u32x4 f1 = ld16(p.net[0].l1 + ((size_t)w * 64 + (lane & 31)) * 16);
  u32x4 fh[2][KQ][2], fo[KQ][2];
  f32x4 bh[2];
#pragma unroll
  for (int li = 1; li < 3; ++li) {
    const bool on = li < nl;
#pragma unroll
    for (int q = 0; q < KQ; ++q)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        fh[li - 1][q][s] = on ? ld16(p.net[0].stream + (size_t)(li - 1) * CHUNK + (2 * (w * KQ + q) + s) * 1024 + lane * 16)
                              : u32x4{0u, 0u, 0u, 0u};
    bh[li - 1] = on ? ld4(p.net[0].bias + li * W + 16 * w + 4 * g) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int q = 0; q < KQ; ++q)
#pragma unroll
    for (int s = 0; s < 2; ++s) fo[q][s] = ld16(p.net[0].stream + (size_t)(nl - 1) * CHUNK + (2 * q + s) * 1024 + lane * 16);
  f32x4 b1;
  if (p.bias_y) {
    b1 = ld4(p.bias_y + (size_t)yi * W + 16 * w + 4 * g);
  } else {  // c (b1 + W1_y y) of this lane's 4 units, in f64 as x3_bias_prep_kernel (dmip_x3.hip) forms it
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int u = 16 * w + 4 * g + r;
      const float* wrow = p.l1w + (size_t)u * p.l1_in;
      double c = p.l1b[u];
      for (int m = 0; m < p.ydim; ++m) c += (double)wrow[D + m] * (double)p.y_obs[(size_t)yi * p.ydim + m];
      b1[r] = (float)((double)kTanhScale * c);
    }
  }
  const f32x4 bo = ld4(p.net[0].bias + nl * W + 4 * g);

  const int S = p.num_steps;
  const long long tiles_y = (p.n_chains + 15) / 16;
  const size_t noise_step = (size_t)gridDim.y * p.n_chains * D;
  bool oor = false;  // a layer-1 input out of the split's range (x3::report_range)
  int par = 0;
  for (long long t = blockIdx.x; t < tiles_y; t += gridDim.x) {  // workgroup-uniform: the barriers stay matched
    const long long c_local = t * 16 + j;
    const bool valid = c_local < p.n_chains;
    const long long c_rd = valid ? c_local : 0;
    Rng rng = rng_init(p.seed, (uint64_t)(p.chain_offset + c_local), (uint64_t)yi);
    float x[D];
    {
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
    SnapCursor snap(p.snap_every, 0);
    for (int i = 0; i < S; ++i) {
      const StepCoef cf = step_coef(i, S, p.T, p.bmin, p.bdiff);
      float v[NV];
#pragma unroll
      for (int k = 0; k < D; ++k) v[k] = x[k];
      v[NV - 1] = cf.tau;
      u32x4 bv[1];
      x3::l1_operand<NV, 1>(v, g, bv);
      oor |= valid && x3::out_of_range(v);

      u32x4 Hh[KQ], Hl[KQ];
      uint32_t h0, h1, l0, l1;
      act_split<true>(mfma16(f1, bv[0], b1), h0, h1, l0, l1);
      exchange(xb, par, w, lane, h0, h1, l0, l1, Hh, Hl);
#pragma unroll
      for (int li = 1; li < 3; ++li) {
        if (li < nl) {
          act_split<false>(tile64(fh[li - 1], Hh, Hl, bh[li - 1]), h0, h1, l0, l1);
          exchange(xb, par, w, lane, h0, h1, l0, l1, Hh, Hl);
        }
      }
      const f32x4 out = tile64(fo, Hh, Hl, bo);
      float a[D];
#pragma unroll
      for (int k = 0; k < D; ++k) a[k] = __shfl(out[k], j, 64);

      float xi[D];
      if constexpr (NOISE) {
        const float* src = p.noise + noise_step * (i + 1) + ((size_t)yi * p.n_chains + c_rd) * D;
#pragma unroll
        for (int k = 0; k < D; ++k) xi[k] = src[k];
      } else {
        rng_normals<D>(rng, xi);
      }
#pragma unroll
      for (int k = 0; k < D; ++k) x[k] = em_update(x[k], a[k], xi[k], cf, p.delta, p.sqrt_delta);
      snap.at_step<D>(i, p.snap_every, p.snap_out, gridDim.y, yi, p.n_chains, c_local, valid && g == 0 && w == 0, x);
    }
    if (valid && g == 0 && w == 0) {
      float* dst = p.x_out + ((size_t)yi * p.n_chains + c_local) * D;
#pragma unroll
      for (int k = 0; k < D; ++k) dst[k] = x[k];
    }
  }
  if (w == 0) x3::report_range(oor, p.err, lane);
}

}  // namespace x3s

// small CDE launches at width 64 (all ys' tiles <= x3s::kMaxTiles) take the latency engine; DMIP_X3_SPLIT=0 keeps
// the one-tile engine (A/B and the bit-identity test)
inline bool x3s_eligible(const X3SamplerParams& p, int n_y) {
  const char* e = getenv("DMIP_X3_SPLIT");
  if (e && e[0] == '0') return false;
  const long long tiles = (p.n_chains + 15) / 16;
  return p.n_hidden >= 1 && p.n_hidden <= 3 && tiles >= 1 && tiles * (n_y > 0 ? n_y : 1) <= x3s::kMaxTiles;
}
// (launch_x3_sampler_cde takes the latency engine exactly when this holds, x3s_sampler_eligible below)

template <int D>
inline hipError_t launch_x3s_sampler(const X3SamplerParams& p, int n_y, hipStream_t st) {
  const long long tiles = (p.n_chains + 15) / 16;
  const dim3 grid((unsigned)tiles, (unsigned)(n_y > 0 ? n_y : 1)), block(x3s::NWS * 64);
  if (p.noise) hipLaunchKernelGGL((x3s::x3s_sampler_kernel<D, true>), grid, block, 0, st, p);
  else hipLaunchKernelGGL((x3s::x3s_sampler_kernel<D, false>), grid, block, 0, st, p);
  return hipGetLastError();
}

}  // namespace dmip
