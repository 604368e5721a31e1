// fp32-accurate CDE sampler on 32x32 tiles: DMIP_PREC_F32X3 at the headline shape (scatterometry and linear
// CDE, hidden_layers [256]*3, BASELINE configs[1]), the default engine there.
//
// Same arithmetic as dmip_x3.h / dmip_x3k.h (every product W_hi h_hi + W_hi h_lo + W_lo h_hi, fp32
// accumulation, r-form tanh by exp2 + rcp) and the k-major ring of dmip_x3k.h, on v_mfma_f32_32x32x16_f16
// instead of 16x16x32. What bounds the 16x16 engine is vector issue: each 16x16x32 MFMA holds the SIMD's
// vector issue for 8 of its 16 cycles (MI355X_MICROARCH.md, constants table), which leaves ~19k issue
// cycles per wave-step for ~25k of activation work (exp2, add, rcp and the hi/lo split per unit, AGPR
// reads). A 32x32x16 MFMA holds issue for 8 of its 32 cycles: the same flops leave twice the room.
//   * one wave per SIMD holds one 32-chain tile; a layer's output is 8 tiles of 32 units x 32 chains:
//     lane (h = l >> 5, i = l & 31) holds units 32 o + 8 (r >> 2) + 4 h + (r & 3) (r = 0..15) of chain i,
//     which is directly the B operand of k-steps 2 o (r = 0..7) and 2 o + 1 (r = 8..15) of the next layer
//     (host k-permutation kperm32, the 16-bit engine's);
//   * W x W layers stream k-major: chunk q = the previous layer's output tile q = k-steps 2q, 2q + 1 of all
//     8 output tiles, hi and lo (32 KiB); o-step O = (tile O / 2, k-step half O % 2) is 3 MFMAs (96 cycles)
//     beside an activation pair of the next chunk's operands (even O) or a DMA piece (O = 5..12);
//   * 16 chunks per step on a static 4-slot ring with the mid-chunk barrier of dmip_x3k.h;
//   * layer 1 (x, tau in 3 k-slots each, one k-step) and the output layer (one fragment per k-step: rows
//     0..D-1 W_hi, rows 4..4+D-1 W_lo, which land in lane halves 0 and 1) are LDS-resident.
// Chain state, RNG, schedule, EM update, snapshots and hand-over are the other engines' (dmip_device.h).
#pragma once
#include "dmip_x3.h"

namespace dmip {
namespace x3w {

using x3::f32x4;

__device__ __forceinline__ f32x16 mfma32w(const u32x4& a, const u32x4& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                0);
}

constexpr int W = 256, OT = 8, KQ = 8, NH = 2;  // [256]*3: 8 32-unit tiles; chunk q = input tile q
constexpr int CHUNK = 32768;                    // 16 o-steps x (hi, lo) x 1 KiB
constexpr int NCHUNK = NH * KQ;                 // ring chunks per step
constexpr int R = 4;                            // ring slots
constexpr int NWV = 4;                          // one wave per SIMD
constexpr int PPW = CHUNK / 1024 / NWV;         // LDS-DMA pieces per wave per chunk
constexpr int JC = 32;                          // chains per wave
static_assert(NCHUNK % R == 0, "static ring: chunk k of every step in slot k % R");

struct WLay {
  static constexpr int L1 = 0, L1_BYTES = OT * 1024;       // [8 tiles][64 lanes][8 fp16]
  static constexpr int OUT = L1 + L1_BYTES, OUT_BYTES = 2 * KQ * 1024;  // [16 k-steps][64][8]
  static constexpr int BIAS = OUT + OUT_BYTES;             // floats: c(b1 + W1_y y) | hidden 1 | hidden 2 | out[16]
  static constexpr int BF = (NH + 1) * W + 16;
  static constexpr int BIAS_BYTES = (BF * 4 + 15) / 16 * 16;
  static constexpr int RING = BIAS + BIAS_BYTES;
  static constexpr int TOTAL = RING + R * CHUNK;
};
static_assert(WLay::TOTAL <= 160 * 1024, "LDS budget");

typedef __attribute__((address_space(3))) void lds_void;

// activate an output tile's half e (accumulator registers 8e .. 8e + 7) into the (hi, lo) B operands of
// k-step 2 o + e: dword d carries units (2d, 2d + 1) of the half
template <bool L1>
__device__ __forceinline__ void act_half(const f32x16& z, int e, u32x4& hh, u32x4& hl) {
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const float r0 = L1 ? x3::x3_act_r2(z[8 * e + 2 * d]) : x3::x3_act_r(z[8 * e + 2 * d]);
    const float r1 = L1 ? x3::x3_act_r2(z[8 * e + 2 * d + 1]) : x3::x3_act_r(z[8 * e + 2 * d + 1]);
    uint32_t h, l;
    x3::split_pair(r0, r1, h, l);
    hh[d] = h;
    hl[d] = l;
  }
}

struct WEngine {
  char* lds;
  const char* ring_lane;  // ring base + 16 lane
  __amdgpu_buffer_rsrc_t rs;
  unsigned voff;          // this wave's DMA pieces: w PPW KiB + 16 lane
  int w, h;

  template <int C, int S, int Q>
  __device__ __forceinline__ void issue_piece() const {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(lds + WLay::RING + S * CHUNK + (w * PPW + Q) * 1024), 16,
                                             voff, C * CHUNK + Q * 1024, 0, 0);
  }
  template <int C, int S, int Q = 0>
  __device__ __forceinline__ void issue() const {
    if constexpr (Q < PPW) {
      issue_piece<C, S, Q>();
      issue<C, S, Q + 1>();
    }
  }

  __device__ __forceinline__ void barrier() const {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }

  // ring protocol of dmip_x3k.h: B(K) in the middle of chunk K - 1; chunk K + 2 refills slot (K + 2) % R
  // piece by piece in the rest of chunk K - 1; the first fragments of a chunk are read ahead
  __device__ __forceinline__ void start(u32x4 (&fpre)[2][2]) const {
    issue<0, 0>();
    issue<1, 1>();
    issue<2, 2>();
    wait_vmcnt<2 * PPW>();
    barrier();
    const x3::lds_cptr b0 = (x3::lds_cptr)ring_lane;
    fpre[0][0] = x3::lds_rd<0>(b0);
    fpre[0][1] = x3::lds_rd<1024>(b0);
    fpre[1][0] = x3::lds_rd<2048>(b0);
    fpre[1][1] = x3::lds_rd<3072>(b0);
    x3::lds_wait2<0>(fpre[1][0], fpre[1][1]);
    x3::lds_wait2<0>(fpre[0][0], fpre[0][1]);
  }

  template <int KN>
  __device__ __forceinline__ void sync_mid() const {
    wait_vmcnt<PPW>();
    barrier();
  }

  // accumulator init of output tile o of layer li: unit 32 o + 8 (r >> 2) + 4 h + (r & 3)
  __device__ __forceinline__ f32x16 bias16(int li, int o) const {
    const float* b = (const float*)(lds + WLay::BIAS) + li * W + 32 * o + 4 * h;
    f32x16 v;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 t = *(const f32x4*)(b + 8 * q);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[4 * q + k] = t[k];
    }
    return v;
  }

  // one W x W layer, k-major: In (f32 pre-activations of the previous layer, 8 tiles) -> Out. Hh/Hl hold
  // input tile 0's operands (k-steps 0, 1) on entry; tile q + 1's are activated during chunk q.
  template <int LI, bool IN_L1>
  __device__ __forceinline__ void layer(const f32x16 (&In)[OT], f32x16 (&Out)[OT], u32x4 (&Hh)[2], u32x4 (&Hl)[2],
                                        u32x4 (&fpre)[2][2]) const {
#pragma unroll
    for (int o = 0; o < OT; ++o) Out[o] = bias16(LI, o);
    chunk<LI, IN_L1, 0>(In, Out, Hh, Hl, fpre);
  }

  template <int LI, bool IN_L1, int Q>
  __device__ __forceinline__ void chunk(const f32x16 (&In)[OT], f32x16 (&Out)[OT], u32x4 (&Hh)[2], u32x4 (&Hl)[2],
                                        u32x4 (&fpre)[2][2]) const {
    if constexpr (Q < KQ) {
      constexpr int K = (LI - 1) * KQ + Q;
      const x3::lds_cptr base = (x3::lds_cptr)(ring_lane + (K % R) * CHUNK);
      const x3::lds_cptr nbase = (x3::lds_cptr)(ring_lane + ((K + 1) % R) * CHUNK);
      u32x4 Nh[2], Nl[2];
      u32x4 f[3][2];
      f[0][0] = fpre[0][0], f[0][1] = fpre[0][1];
      f[1][0] = fpre[1][0], f[1][1] = fpre[1][1];
      ostep<LI, IN_L1, Q, 0>(base, nbase, In, Out, Hh, Hl, Nh, Nl, f, fpre);
      x3::lds_wait2<0>(fpre[0][0], fpre[0][1]);
      x3::lds_wait2<0>(fpre[1][0], fpre[1][1]);
      if constexpr (Q + 1 < KQ) {
        Hh[0] = Nh[0], Hh[1] = Nh[1], Hl[0] = Nl[0], Hl[1] = Nl[1];
      }
      chunk<LI, IN_L1, Q + 1>(In, Out, Hh, Hl, fpre);
    }
  }

  // o-step O of chunk K = (LI, Q): output tile O / 2, k-step half O % 2 -- 3 MFMAs (96 cycles; fragments
  // read two o-steps ahead, across the chunk boundary at O = 14, 15) beside at most two slices of the
  // chunk's other work, spread so that no o-step's vector issue exceeds the 3 x 24 cycles its MFMAs leave:
  // the activation of the next input tile's pair O / 2 at even O; B(K + 1) at O = 4 (chunk K + 1's pieces
  // were issued a chunk and a half earlier); DMA piece O - 5 of chunk K + 3 at O = 5..12
  template <int LI, bool IN_L1, int Q, int O>
  __device__ __forceinline__ void ostep(x3::lds_cptr base, x3::lds_cptr nbase, const f32x16 (&In)[OT],
                                        f32x16 (&Out)[OT], const u32x4 (&Hh)[2], const u32x4 (&Hl)[2],
                                        u32x4 (&Nh)[2], u32x4 (&Nl)[2], u32x4 (&f)[3][2],
                                        u32x4 (&fpre)[2][2]) const {
    if constexpr (O < 16) {
      constexpr int K = (LI - 1) * KQ + Q;
      constexpr int o = O >> 1, e = O & 1;
      if constexpr (O + 2 < 16) {
        f[(O + 2) % 3][0] = x3::lds_rd<(O + 2) * 2048>(base);
        f[(O + 2) % 3][1] = x3::lds_rd<(O + 2) * 2048 + 1024>(base);
      } else {
        fpre[O + 2 - 16][0] = x3::lds_rd<(O + 2 - 16) * 2048>(nbase);
        fpre[O + 2 - 16][1] = x3::lds_rd<(O + 2 - 16) * 2048 + 1024>(nbase);
      }
      x3::lds_wait2<4>(f[O % 3][0], f[O % 3][1]);
      Out[o] = mfma32w(f[O % 3][0], Hl[e], Out[o]);
      Out[o] = mfma32w(f[O % 3][1], Hh[e], Out[o]);
      Out[o] = mfma32w(f[O % 3][0], Hh[e], Out[o]);
      if constexpr (Q + 1 < KQ && O % 2 == 0) {
        constexpr int ne = O >> 3, d = (O >> 1) & 3;
        const f32x16& z = In[Q + 1];
        const float r0 = IN_L1 ? x3::x3_act_r2(z[8 * ne + 2 * d]) : x3::x3_act_r(z[8 * ne + 2 * d]);
        const float r1 = IN_L1 ? x3::x3_act_r2(z[8 * ne + 2 * d + 1]) : x3::x3_act_r(z[8 * ne + 2 * d + 1]);
        uint32_t hv, lv;
        x3::split_pair(r0, r1, hv, lv);
        Nh[ne][d] = hv;
        Nl[ne][d] = lv;
      }
      if constexpr (O == 4) sync_mid<(K + 1) % NCHUNK>();
      if constexpr (O >= 5 && O < 5 + PPW) issue_piece<(K + R - 1) % NCHUNK, (K + R - 1) % R, O - 5>();
      ostep<LI, IN_L1, Q, O + 1>(base, nbase, In, Out, Hh, Hl, Nh, Nl, f, fpre);
    }
  }
};
static_assert(PPW == 8, "o-steps 5..12 issue the 8 DMA pieces of a chunk");

// ---------------------------------------------------------------------------- sampler kernel
// The reverse-SDE loop (models/diffusion.py:27-46) for the CDE, a = net(x, y, tau) with y folded into the
// per-y layer-1 bias; mu = g a + 0.5 beta x, x <- x + delta mu + sqrt(delta) g xi (dmip_device.h
// em_update). Work: the balanced WaveSchedule over jobs of 32 chains.
template <int D, bool NOISE>
__global__ void __launch_bounds__(NWV * 64, 1) x3w_sampler_kernel(X3SamplerParams p) {
  using L = WLay;
  static_assert(D <= 4, "output rows of a chain sit in lane half 0 (D <= 4)");
  __shared__ __attribute__((aligned(16))) char lds[L::TOTAL];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = lane >> 5, i = lane & 31;
  const int yi = blockIdx.y;
  constexpr int NV = D + 1;  // layer-1 inputs: x, tau (y folded into the bias)

  WEngine eng;
  eng.lds = lds;
  eng.ring_lane = lds + L::RING + lane * 16;
  eng.rs = __builtin_amdgcn_make_buffer_rsrc((void*)p.net[0].wstream, 0, NCHUNK * CHUNK, 0x00020000);
  eng.voff = (unsigned)(w * PPW * 1024 + lane * 16);
  eng.w = w;
  eng.h = h;
  {
    const uint4* s1 = (const uint4*)p.net[0].wl1;
    uint4* d1 = (uint4*)(lds + L::L1);
    for (int e = threadIdx.x; e < L::L1_BYTES / 16; e += NWV * 64) d1[e] = s1[e];
    const uint4* so = (const uint4*)p.net[0].wout;
    uint4* dout = (uint4*)(lds + L::OUT);
    for (int e = threadIdx.x; e < L::OUT_BYTES / 16; e += NWV * 64) dout[e] = so[e];
    float* bl = (float*)(lds + L::BIAS);
    for (int k = threadIdx.x; k < L::BF; k += NWV * 64) bl[k] = k < W ? p.bias_y[(size_t)yi * W + k] : p.net[0].bias[k];
    __syncthreads();
  }
  u32x4 fpre[2][2];
  eng.start(fpre);
  const char* l1_lane = lds + L::L1 + lane * 16;
  const char* out_lane = lds + L::OUT + lane * 16;

  const int S = p.num_steps;
  const long long jobs_y = (p.n_chains + JC - 1) / JC;
  const long long n_waves = (long long)gridDim.x * NWV;
  const long long gw = (long long)blockIdx.x * NWV + w;
  constexpr int XT = sampler_xfer_words(D);
  const WaveSchedule sched(jobs_y, S, n_waves, gw);
  const size_t noise_step = (size_t)gridDim.y * p.n_chains * D;

  for (int sgi = 0; sgi < sched.n_seg; ++sgi) {
    const Seg sg = sched.segment(sgi);
    const long long c_loc = (long long)(sg.job >= 0 ? sg.job : 0) * JC + i;
    const bool valid = sg.job >= 0 && c_loc < p.n_chains;
    Rng rng;
    float x[D];
    if (sg.kind == 2) {  // resume the job the previous wave of the grid handed over
      const size_t slot = (size_t)yi * n_waves + gw - 1;
      const bool lost = handover_wait(p.xflag + slot, p.spin_limit, p.err, kErrHandover, lane);
      const float* st = p.xfer + slot * (size_t)XT;
#pragma unroll
      for (int k = 0; k < D; ++k) x[k] = lost ? __builtin_nanf("") : st[k * 64 + lane];
      rng.s0 = __float_as_uint(st[(D + 0) * 64 + lane]);
      rng.s1 = __float_as_uint(st[(D + 1) * 64 + lane]);
      rng.s2 = __float_as_uint(st[(D + 2) * 64 + lane]);
      rng.s3 = __float_as_uint(st[(D + 3) * 64 + lane]);
    } else {
      rng = rng_init(p.seed, (uint64_t)(p.chain_offset + c_loc), (uint64_t)yi);
      float n0[D];
      if constexpr (NOISE) {
        const float* src = p.noise + ((size_t)yi * p.n_chains + (valid ? c_loc : 0)) * D;
#pragma unroll
        for (int k = 0; k < D; ++k) n0[k] = src[k];
      } else {
        rng_normals<D>(rng, n0);
      }
#pragma unroll
      for (int k = 0; k < D; ++k) x[k] = __fadd_rn(__fmul_rn(n0[k], p.stdv), p.mean);
    }

    int snap_next = p.snap_every > 0 ? (sg.s0 / p.snap_every + 1) * p.snap_every : -1;
    for (int i0 = sg.s0; i0 < sg.s1; ++i0) {
      const int si = sg.kind == 3 ? 0 : i0;  // idle steps: a dummy job at step 0, discarded
      const StepCoef cf = step_coef(si, S, p.T, p.bmin, p.bdiff);

      // ---- layer 1 (resident image: one MFMA per output tile), pre-activations in P
      f32x16 P[OT];
      {
        float v[NV];
#pragma unroll
        for (int k = 0; k < D; ++k) v[k] = x[k];
        v[NV - 1] = cf.tau;
        u32x4 b1[1];
        x3::l1_operand<NV, 1>(v, h, b1);
#pragma unroll
        for (int o = 0; o < OT; ++o) {
          const u32x4 a = *(const u32x4*)(l1_lane + o * 1024);
          P[o] = mfma32w(a, b1[0], eng.bias16(0, o));
        }
      }
      u32x4 Hh[2], Hl[2];
      act_half<true>(P[0], 0, Hh[0], Hl[0]);
      act_half<true>(P[0], 1, Hh[1], Hl[1]);
      // ---- hidden layers 1 and 2 (ring chunks 0..7, 8..15)
      f32x16 Q[OT];
      eng.template layer<1, true>(P, Q, Hh, Hl, fpre);
      act_half<false>(Q[0], 0, Hh[0], Hl[0]);
      act_half<false>(Q[0], 1, Hh[1], Hl[1]);
      f32x16 P2[OT];
      eng.template layer<2, false>(Q, P2, Hh, Hl, fpre);
      // ---- output layer (resident): rows 0..D-1 W_hi (lane half 0), rows 4..4+D-1 W_lo (lane half 1)
      f32x16 oH, oL;
      {
        const f32x16 bo = eng.bias16(NH + 1, 0);
#pragma unroll
        for (int r = 0; r < 16; ++r) oH[r] = h == 0 && r < 4 ? bo[r] : 0.0f, oL[r] = 0.0f;
#pragma unroll
        for (int s = 0; s < 2 * KQ; ++s) {
          const u32x4 fo = *(const u32x4*)(out_lane + s * 1024);
          u32x4 eh, el;
          act_half<false>(P2[s >> 1], s & 1, eh, el);
          oH = mfma32w(fo, eh, oH);
          oL = mfma32w(fo, el, oL);
        }
      }
      // ---- a(x) on every lane of chain i, the EM update
      float a[D];
#pragma unroll
      for (int k = 0; k < D; ++k) {
        const float lo_w = __shfl(oH[k], i + 32, 64);  // W_lo h_hi of row k (lane half 1)
        const float v = (oH[k] + oL[k]) + lo_w;
        a[k] = __shfl(v, i, 64);
      }
      float xi[D];
      if constexpr (NOISE) {
        const float* src = p.noise + noise_step * (si + 1) + ((size_t)yi * p.n_chains + (valid ? c_loc : 0)) * D;
#pragma unroll
        for (int k = 0; k < D; ++k) xi[k] = src[k];
      } else {
        rng_normals<D>(rng, xi);
      }
#pragma unroll
      for (int k = 0; k < D; ++k) x[k] = em_update(x[k], a[k], xi[k], cf, p.delta, p.sqrt_delta);
      if (i0 + 1 == snap_next) {
        snap_next += p.snap_every;
        if (sg.kind != 3 && h == 0 && valid) {
          float* dst = p.snap_out + (((size_t)((i0 + 1) / p.snap_every - 1) * gridDim.y + yi) * p.n_chains + c_loc) * D;
#pragma unroll
          for (int k = 0; k < D; ++k) dst[k] = x[k];
        }
      }
    }
    if (sg.kind == 1) {  // hand the job over to the next wave of the grid
      const size_t slot = (size_t)yi * n_waves + gw;
      float* st = p.xfer + slot * (size_t)XT;
#pragma unroll
      for (int k = 0; k < D; ++k) st[k * 64 + lane] = x[k];
      st[(D + 0) * 64 + lane] = __uint_as_float(rng.s0);
      st[(D + 1) * 64 + lane] = __uint_as_float(rng.s1);
      st[(D + 2) * 64 + lane] = __uint_as_float(rng.s2);
      st[(D + 3) * 64 + lane] = __uint_as_float(rng.s3);
      handover_publish(p.xflag + slot, lane, p.debug_flags);
    } else if (sg.kind != 3 && h == 0 && valid) {
      float* dst = p.x_out + ((size_t)yi * p.n_chains + c_loc) * D;
#pragma unroll
      for (int k = 0; k < D; ++k) dst[k] = x[k];
    }
  }
  wait_vmcnt<0>();  // the prefetched chunks of a step that never ran land before the workgroup exits
}

}  // namespace x3w

template <int D, bool NOISE>
inline hipError_t launch_x3w_sampler_t(const X3SamplerParams& p, int n_y, hipStream_t st) {
  using namespace x3w;
  auto kern = x3w_sampler_kernel<D, NOISE>;
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
