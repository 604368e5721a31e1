// Device-side building blocks shared by the dmip kernels (gfx950 / CDNA4 only).
//
//  * MFMA fragment types for v_mfma_f32_32x32x16_bf16 (wave64, 32x32 f32 accumulator tile).
//  * The per-chain counter-keyed RNG (splitmix64-seeded xoshiro128** + Box-Muller), restated
//    bit-for-bit on the integer side by oracle/dmip_oracle.py (rng_init/rng_next/rng_normals).
//  * The reverse-time schedule and VP-SDE coefficients with the reference's fp32 rounding
//    (models/diffusion.py:31-42, sdes.py:21-35,77-87): every multiply/add is an explicit
//    round-to-nearest intrinsic so the compiler cannot contract them into FMAs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dmip {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// 2*log2(e): pre-activations are produced pre-scaled by this so tanh needs no extra multiply.
constexpr float kTanhScale = 2.8853900817779268f;

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// the same 32x32x16 tile on fp16 operands; the 16-bit fragments live in bf16x8 registers either way
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x16 mfma32h(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                0);
}

// ------------------------------------------------------------------------------------ RNG
struct Rng {
  uint32_t s0, s1, s2, s3;
};

__device__ __forceinline__ uint64_t splitmix_next(uint64_t& st) {
  st += 0x9E3779B97F4A7C15ull;
  uint64_t z = st;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Keyed by the GLOBAL chain index: identical draws however chains are split over
// workgroups / GPUs.
__device__ __forceinline__ Rng rng_init(uint64_t seed, uint64_t chain, uint64_t stream) {
  uint64_t sm = seed + chain * 0xD1B54A32D192ED03ull + stream * 0x8CB92BA72F3D8DD7ull;
  uint64_t z0 = splitmix_next(sm);
  uint64_t z1 = splitmix_next(sm);
  Rng r;
  r.s0 = (uint32_t)z0;
  r.s1 = (uint32_t)(z0 >> 32);
  r.s2 = (uint32_t)z1;
  r.s3 = (uint32_t)(z1 >> 32);
  if ((r.s0 | r.s1 | r.s2 | r.s3) == 0u) r.s0 = 1u;
  return r;
}

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }

__device__ __forceinline__ uint32_t rng_next(Rng& r) {
  const uint32_t result = rotl32(r.s1 * 5u, 7) * 9u;
  const uint32_t t = r.s1 << 9;
  r.s2 ^= r.s0;
  r.s3 ^= r.s1;
  r.s1 ^= r.s2;
  r.s0 ^= r.s3;
  r.s2 ^= t;
  r.s3 = rotl32(r.s3, 11);
  return result;
}

// Box-Muller on 24-bit uniforms: u1 in (0,1] for the log, u2 in [0,1) in revolutions
// (v_sin_f32 / v_cos_f32 take their argument in units of 2*pi).
__device__ __forceinline__ void rng_normal_pair(Rng& r, float& n0, float& n1) {
  const uint32_t a = rng_next(r);
  const uint32_t b = rng_next(r);
  const float u1 = 1.0f - (float)(a >> 8) * 0x1p-24f;
  const float u2 = (float)(b >> 8) * 0x1p-24f;
  const float rad = __fsqrt_rn(-1.3862943611198906f * __log2f(u1));  // sqrt(-2 ln u1)
  n0 = rad * __builtin_amdgcn_cosf(u2);
  n1 = rad * __builtin_amdgcn_sinf(u2);
}

template <int D>
__device__ __forceinline__ void rng_normals(Rng& r, float (&n)[D]) {
#pragma unroll
  for (int p = 0; p < (D + 1) / 2; ++p) {
    float a, b;
    rng_normal_pair(r, a, b);
    n[2 * p] = a;
    if (2 * p + 1 < D) n[2 * p + 1] = b;
  }
}

// ------------------------------------------------------------------------------ schedule
// NOTE: HIP's __fmul_rn/__fadd_rn are plain operators; libdmip is compiled with
// -ffp-contract=off so they are not fused into FMAs (which would change the last bit of
// beta / the EM update vs the reference). Intended FMAs are written as explicit builtins.
// torch.linspace(0,1,S+1)[i] in fp32 (ATen CPU kernel: first half i*step, second half
// 1-(S-i)*step with a single rounding) -- models/diffusion.py:34.
__device__ __forceinline__ float linspace_at(int i, int S) {
  const float step = __fdiv_rn(1.0f, (float)S);
  if (i < (S + 1) / 2) return __fmul_rn((float)i, step);
  return __fmaf_rn(-(float)(S - i), step, 1.0f);
}

struct StepCoef {
  float tau;   // T - t_i, the time the net and coefficients see (sdes.py:78)
  float beta;  // beta(T - t_i)                                    (sdes.py:21-22)
  float g;     // sqrt(beta) (pow 0.5)                             (sdes.py:33-35)
};

__device__ __forceinline__ StepCoef step_coef(int i, int S, float T, float bmin, float bdiff) {
  StepCoef c;
  const float ts = __fmul_rn(linspace_at(i, S), T);
  c.tau = __fsub_rn(T, ts);
  c.beta = __fadd_rn(bmin, __fmul_rn(bdiff, c.tau));
  // correctly rounded sqrt: the f64 square root is correctly rounded and rounding it to f32 is
  // innocuous (53 >= 2*24 + 2); hipcc's f32 __fsqrt_rn is not correctly rounded on gfx950
  c.g = (float)__dsqrt_rn((double)c.beta);
  return c;
}

// mean_weight(t) = exp(-0.25 t^2 (bmax-bmin) - 0.5 t bmin) and var(t) = 1 - exp(-0.5 t^2 (bmax-bmin)
// - t bmin) in the reference's evaluation order (sdes.py:24-28); exp within 1 ulp.
__device__ __forceinline__ float vp_mean_weight(float t, float bmin, float bdiff) {
  const float a = __fmul_rn(__fmul_rn(-0.25f, __fmul_rn(t, t)), bdiff);
  return expf(__fsub_rn(a, __fmul_rn(__fmul_rn(0.5f, t), bmin)));
}
__device__ __forceinline__ float vp_std(float t, float bmin, float bdiff) {
  const float a = __fmul_rn(__fmul_rn(-0.5f, __fmul_rn(t, t)), bdiff);
  const float var = __fsub_rn(1.0f, expf(__fsub_rn(a, __fmul_rn(t, bmin))));
  return (float)__dsqrt_rn((double)var);  // var ** 0.5, correctly rounded
}

// x <- fl(x + fl(delta*mu)) + fl(fl(sqrt(delta)*g)*xi),  mu = fl(g*a) - fl(fl(-0.5*beta)*x)
// (models/diffusion.py:40-42 with sdes.py:77-79,86-87 at lambda = 0).
__device__ __forceinline__ float em_update(float x, float a, float xi, const StepCoef& c,
                                           float delta, float sqrt_delta) {
  const float mu = __fsub_rn(__fmul_rn(c.g, a), __fmul_rn(__fmul_rn(-0.5f, c.beta), x));
  const float drift = __fadd_rn(x, __fmul_rn(delta, mu));
  return __fadd_rn(drift, __fmul_rn(__fmul_rn(sqrt_delta, c.g), xi));
}

// Trajectory snapshots: x of a chain after every `every`-th step (0-based step i, i + 1 a multiple
// of every) into snap [S / every][n_y][n_chains][D] -- the only HBM writes of a chain before its final
// state. The cursor holds the next snapshot step of the segment [s0, s1), so a step pays one scalar
// compare (-1: snapshots off).
struct SnapCursor {
  int next;
  __device__ __forceinline__ SnapCursor(int every, int s0) : next(every > 0 ? (s0 / every + 1) * every : -1) {}
  template <int D>
  __device__ __forceinline__ void at_step(int i, int every, float* snap, int n_y, int yi, long long n_chains,
                                          long long c, bool write, const float (&x)[D]) {
    if (i + 1 != next) return;
    next += every;
    if (!write) return;
    float* dst = snap + (((size_t)((i + 1) / every - 1) * n_y + yi) * n_chains + c) * D;
#pragma unroll
    for (int k = 0; k < D; ++k) dst[k] = x[k];
  }
};

// ---------------------------------------------------------------------------- activation
// Hidden layers propagate r = 1/(1+exp(2z)) instead of tanh(z) = 1 - 2r; the "1 - 2r" is folded
// into the next layer on the host (weights -2W, bias b + sum_k W). The pre-activation arrives
// already multiplied by 2*log2(e), so one layer's activation is exp2 + add + rcp.
__device__ __forceinline__ float act_r(float zs) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(zs));
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// two f32 -> one dword of two bf16 (v_cvt_pk_bf16_f32, round to nearest even; a in the low half).
// Converting explicit pairs keeps the packed conversion without letting the SLP vectoriser also
// fuse the neighbouring scalar FMAs into v_pk_fma_f32 (a measured anti-lever beside MFMAs).
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t cvt_pk_bf16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, bf16x2));
}
__device__ __forceinline__ uint32_t cvt_pk_f16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, f16x2));
}

// tanh(tanh(z)) of the reference's first layer (nets.py:21-26 double Tanh) for a PAIR of units,
// returned in t-form (the value itself; the host packs the next layer for a t-form input) as an fp16
// pair. With e = exp(-2|z|) in (0, 1], tanh|z| = (1 - e)/(1 + e) and tanh(tanh|z|) = (1 - e) q(e),
// q a degree-4 fit (max abs error 1.7e-5, exact 0 at z = 0). e is computed in f32, the Horner
// steps in packed fp16 (v_pk_fma_f16: two units per instruction), the signs of z moved in with one
// v_perm + v_bfi: 24 issue cycles per unit against 34 for the same polynomial in scalar f32
// (profiles/README.md, r2 variants). fp16 evaluation error <= ~5e-4 absolute, at the size of the
// 16-bit rounding of the result itself.
__device__ __forceinline__ uint32_t act_t_twice_pk_f16(float za, float zb) {
  const f32x2 e32 = {__builtin_amdgcn_exp2f(-__builtin_fabsf(za)), __builtin_amdgcn_exp2f(-__builtin_fabsf(zb))};
  const f16x2 e = __builtin_convertvector(e32, f16x2);
  auto c = [](float v) { return f16x2{(_Float16)v, (_Float16)v}; };
  f16x2 q = __builtin_elementwise_fma(e, c(-0.17045435309410095f), c(0.5245547890663147f));
  q = __builtin_elementwise_fma(q, e, c(-0.5390751957893372f));
  q = __builtin_elementwise_fma(q, e, c(-0.07747964560985565f));
  q = __builtin_elementwise_fma(q, e, c(0.761600136756897f));
  const f16x2 r = __builtin_elementwise_fma(-e, q, q);
  const uint32_t sg = __builtin_amdgcn_perm(__float_as_uint(zb), __float_as_uint(za), 0x07000300u);
  return (sg & 0x80008000u) | (__builtin_bit_cast(uint32_t, r) & 0x7FFF7FFFu);
}

// activate one 32x32 accumulator tile into the next layer's fp16 B fragments (lo: registers 0-7,
// hi: registers 8-15). TWICE: layer 1's double tanh (t-form), else the r-form of a hidden layer.
// CAST_ONLY: timing ablation (the pre-activation itself).
template <bool TWICE, bool CAST_ONLY = false>
__device__ __forceinline__ void act_pack(const f32x16& acc, bf16x8& lo, bf16x8& hi) {
  u32x4 l, h;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if constexpr (CAST_ONLY) {
      l[i] = cvt_pk_f16(acc[2 * i], acc[2 * i + 1]);
      h[i] = cvt_pk_f16(acc[8 + 2 * i], acc[8 + 2 * i + 1]);
    } else if constexpr (TWICE) {
      l[i] = act_t_twice_pk_f16(acc[2 * i], acc[2 * i + 1]);
      h[i] = act_t_twice_pk_f16(acc[8 + 2 * i], acc[8 + 2 * i + 1]);
    } else {
      l[i] = cvt_pk_f16(act_r(acc[2 * i]), act_r(acc[2 * i + 1]));
      h[i] = cvt_pk_f16(act_r(acc[8 + 2 * i]), act_r(acc[8 + 2 * i + 1]));
    }
  }
  lo = __builtin_bit_cast(bf16x8, l);
  hi = __builtin_bit_cast(bf16x8, h);
}

// ------------------------------------------------------------- balanced persistent schedule
// The persistent samplers' work distribution (dmip_kernels.hip em_sampler_kernel, dmip_f32.h
// f32_sampler_kernel): the tiles_y * S wave-steps of one y are cut into one equal segment of
// C = ceil(tiles_y S / n_waves) steps per wave of the grid (McNaughton's wrap-around rule), so every
// wave stays busy to the end whatever the chain count. A tile cut by a segment boundary runs its
// first part at the START of the earlier wave's segment and its second part at the END of the next
// wave's (order-safe since C >= S); its state goes through global memory with a release/acquire
// flag. All waves of a workgroup run exactly C steps (an idle segment computes on a dummy tile), so
// the weight ring's barriers stay paired. A chain's arithmetic does not depend on which wave runs it.
// Segment kinds: 0 whole tile, 1 first part handed over, 2 second part taken over, 3 idle.
struct Seg {
  int job, s0, s1, kind;
};

struct WaveSchedule {
  long long C, used;
  int S, a_job, a_len, b_job, b_from, f_first, n_full, n_seg;

  __device__ __forceinline__ WaveSchedule(long long tiles_y, int S_, long long n_waves, long long gw) {
    S = S_;
    C = S;
    a_job = -1, a_len = 0, b_job = -1, b_from = 0, f_first = 0, n_full = 0;
    if (tiles_y <= n_waves) {
      if (gw < tiles_y) f_first = (int)gw, n_full = 1;
    } else {
      C = (tiles_y * S + n_waves - 1) / n_waves;  // > S
      const long long lo = gw * C;
      const long long hi = lo + C < tiles_y * S ? lo + C : tiles_y * S;
      if (lo < hi) {
        const int j_lo = (int)(lo / S), r_lo = (int)(lo % S);
        const int j_hi = (int)(hi / S), r_hi = (int)(hi % S);
        if (r_lo > 0) b_job = j_lo, b_from = r_lo;
        if (r_hi > 0) a_job = j_hi, a_len = r_hi;
        f_first = r_lo > 0 ? j_lo + 1 : j_lo;
        n_full = j_hi - f_first > 0 ? j_hi - f_first : 0;
      }
    }
    used = (long long)a_len + (long long)n_full * S + (b_job >= 0 ? S - b_from : 0);
    n_seg = __builtin_amdgcn_readfirstlane((a_job >= 0) + n_full + (b_job >= 0) + (C > used));
  }

  // order: A, whole tiles, idle, B -- B must END at step C (the last wave's segment is short)
  __device__ __forceinline__ Seg segment_raw(int k) const {
    if (a_job >= 0) {
      if (k == 0) return Seg{a_job, 0, a_len, 1};
      --k;
    }
    if (k < n_full) return Seg{f_first + k, 0, S, 0};
    k -= n_full;
    if (C > used) {
      if (k == 0) return Seg{-1, 0, (int)(C - used), 3};
      --k;
    }
    return Seg{b_job, b_from, S, 2};
  }

  // wave-uniform by construction; said so, or a ring counter would be treated as divergent
  __device__ __forceinline__ Seg segment(int k) const {
    const Seg s = segment_raw(k);
    return Seg{__builtin_amdgcn_readfirstlane(s.job), __builtin_amdgcn_readfirstlane(s.s0),
               __builtin_amdgcn_readfirstlane(s.s1), __builtin_amdgcn_readfirstlane(s.kind)};
  }
};

// consumer side of a hand-over: wait (bounded) for the producer's flag. Giving up is an error the
// host sees through dmip_device_status (kErrHandover), never silently wrong chains: returns true
// when the state never arrived (the caller then poisons the tile's output).
__device__ __forceinline__ bool handover_wait(const unsigned* flag, unsigned spin_limit, unsigned* err, unsigned code,
                                              int lane) {
  bool lost = false;
  for (unsigned spins = 0; __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == 0u;) {
    if (++spins > spin_limit) {
      lost = true;
      break;
    }
    __builtin_amdgcn_s_sleep(8);
  }
  if (lost && lane == 0) __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return lost;
}

// producer side: every lane's state stores are visible device-wide before the flag
__device__ __forceinline__ void handover_publish(unsigned* flag, int lane, int debug_flags) {
  __threadfence();
  if (lane == 0 && !(debug_flags & 1)) __hip_atomic_store(flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------------ sync primitives
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  // vmcnt = N (bits 3:0 and 15:14), expcnt = 7 and lgkmcnt = 15 (no wait on those)
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

__device__ __forceinline__ void lds_barrier() {
  // all of this wave's LDS reads have returned, then a raw workgroup barrier. The asm memory
  // clobbers keep the compiler from moving LDS accesses across it and the sched_barriers keep
  // register-only instructions (MFMAs) on their side too -- otherwise the last MFMAs of a tile
  // slide past the barrier and the next activation stalls on them. No vmcnt(0) is implied, so
  // LDS-DMA weight prefetches stay in flight across the barrier.
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

typedef __attribute__((address_space(3))) void lds_void;

// one 1 KiB wave-instruction of LDS-DMA: lane l copies 16 B from g + 16 l to lds + 16 l.
__device__ __forceinline__ void glds16(const char* g_wave_base, char* lds_wave_base, int lane) {
  __builtin_amdgcn_global_load_lds((const void*)(g_wave_base + lane * 16),
                                   (lds_void*)lds_wave_base, 16, 0, 0);
}

}  // namespace dmip
