// Internal (non-exported) launch interface between the C-ABI layer (dmip_capi.cpp) and the
// kernels (dmip_kernels.hip). Plain structs of device pointers; no torch types anywhere.
#pragma once
#include <hip/hip_runtime.h>


namespace dmip {

constexpr int kMaxDevices = 64;

// the device a stream belongs to (the current device for the null stream)
inline int stream_device(hipStream_t st) {
  int dev = 0;
  hipDevice_t d = 0;
  if (st != nullptr && hipStreamGetDevice(st, &d) == hipSuccess) return (int)d;
  (void)hipGetDevice(&dev);
  return dev;
}

// number of workgroups of kernel `fn` the stream's device holds at once (CUs x occupancy), cached per
// (kernel address, block size, device). Keyed by the kernel's ADDRESS: every sampler instantiation
// has the same function type, and a type-keyed cache once handed one kernel's slot count to all of
// them -- a grid larger than the resident set breaks the balanced schedule's co-residency.
int resident_slots_impl(const void* fn, int nthreads, hipStream_t st);

template <typename Kern>
int resident_slots(Kern kern, int nthreads, hipStream_t st) {
  return resident_slots_impl(reinterpret_cast<const void*>(kern), nthreads, st);
}

// Sampler modes (dmip_kernels.hip em_sampler_kernel)
enum { SAMPLER_CDE = 0, SAMPLER_POSTERIOR = 1, SAMPLER_CDIFFE = 2 };

struct SamplerParams {
  // network 0: the CDE / CDiffE network, or the Posterior estimator's likelihood network
  const char* hidden;         // (NL-1)*(W/32) row-tile chunks of (W/16) KiB bf16 fragments
  const char* a1;             // layer-1 blocks [W/32][K1S] KiB, per y ([n_y][...]) when a1_per_y
  const char* ao;             // output layer blocks [W/16] KiB (rows duplicated into both lane halves)
  const float* bias_hidden;   // [NL-1][W/32][2][16] accumulator init per lane half
  const float* bias_out;      // [2][16]
  int a1_per_y;
  // network 1 (Posterior only): the prior network (x, t); its layer 1 is shared by all y
  const char* hidden2;
  const char* a1_2;
  const char* ao2;
  const float* bias_hidden2;
  const float* bias_out2;
  const float* y_obs;         // CDiffE: observations [n_y][ydim] (re-diffused every step)
  int n_corr;                 // CDiffE: Langevin corrector steps per time step (0 = plain EM)
  float snr;                  // CDiffE: corrector signal-to-noise ratio
  const float* noise;         // injected normals [S+1][n_y][n_chains][D] (slot 0 -> x0) or null
  float* x_out;               // [n_y][n_chains][D]
  float* snap_out;            // trajectory snapshots [S / snap_every][n_y][n_chains][D] or null
  int snap_every;             // write x after every snap_every-th step (0: final output only)
  long long n_chains;         // chains per y
  long long chain_offset;     // global index of chain 0 (keys the RNG)
  int num_steps;
  float T, bmin, bdiff, delta, sqrt_delta, mean, stdv;
  unsigned long long seed;
  unsigned long long* stamps; // diagnostic build only: [n_wg * NW][3] phase cycle sums, else null
  // hand-over of split tiles between waves (set by launch_sampler): per y and wave of the grid, the
  // chain state [D + 4][64] words and a ready flag (zeroed before the launch)
  float* xfer;
  unsigned int* xflag;
  // device status word (dmip_device_status): set to kErrHandover when a consumer wave gives up
  // waiting for a hand-over flag; the tile's chains are then written as NaN
  unsigned int* err;
  unsigned int spin_limit;    // s_sleep(8) rounds before a consumer gives up (default 2^22, ~1 s)
  int debug_flags;            // test hook only: bit 0 = producers never publish (forces the timeout)
};

// device status codes written by kernels into the per-device status word
constexpr unsigned kErrHandover = 1u;
// a fp32x3 sampler's layer-1 input (chain state x, tau, CDiffE's y_t) left the fp16 range of its hi/lo split
// (|v| > 65504): those chains are not fp32-accurate (dmip_device_status reports it; the Python estimators
// resample with the exact-f32 engine)
constexpr unsigned kErrRange = 2u;

// hand-over state of a split tile, per grid wave: x[D] + the xoshiro128** state, one word per lane
constexpr int sampler_xfer_words(int D) { return (D + 4) * 64; }
// zeroed hand-over buffers for `slots` grid waves (freed by the caller with hipFreeAsync(*buf))
hipError_t alloc_handover(size_t slots, int d, hipStream_t st, char** buf, float** xfer, unsigned** xflag);

struct ForwardParams {
  const char* hidden;
  const char* a1;             // [W/32][K1S] KiB, all inputs varying
  const char* ao;             // [W/16] KiB, natural output rows
  const float* bias_hidden;
  const float* bias_out;
  const float* x;             // [n][xdim]
  const float* y;             // [n][ydim] (y_stride = ydim) or one row (y_stride = 0)
  const float* t;             // [n] (t_stride = 1) or one value (t_stride = 0)
  float* out;                 // [n][out_dim]
  long long n;
  long long y_stride;
  int t_stride;
  int xdim, ydim, out_dim;
};

struct A1PrepParams {
  const float* w1;   // [width][in_dim] fp32 (nn.Linear layout)
  const float* b1;   // [width]
  const float* y;    // [n_y][ydim]
  char* a1;          // out: [n_y][width/32][k1s] KiB
  int width, in_dim, xdim, ydim, y_col0, t_col, k1s;
};

// Fused training step (dmip_train.hip): the linear problem's width-64 CDE (x 2, y 2).
constexpr int kTrainWidth = 64, kTrainXdim = 2, kTrainYdim = 2;

struct TrainParams {
  const float* w[4];          // device fp32 weights, nn.Linear layout [out][in], layers 0..n_hidden
  const float* b[4];
  const float* x;             // [n][xdim] clean samples
  const float* y;             // [n][ydim]
  const float* t;             // [n] diffusion times (sample_t)
  const float* eps;           // [n][xdim] forward-diffusion noise (base_sde.sample's randn)
  long long n;
  float inv_n, bmin, bdiff;
  int has_dsm, has_ic, pde, pde_l1, ic_l1;  // pde: 0 none, 1 ScoreFPE, 2 cScoreFPE
  float lam, lam2;
  float icA[4], icb[2], icS[4];  // linear-problem IC target: -x + ((y - (A x + b)) S^T) A
  float* partials;            // [n_waves][partial stride]
  char* packed;               // the shared LDS image of the weight fragments (written by the pack kernel)
  float* adj;                 // split build: [n][kTrainAdj] per-sample loss adjoints + loss terms (forward -> reverse)
  // split build, record reverse (train_rec()): per tile and hidden layer li, the forward's activations of the P, V, C
  // streams (bf16) and the reverse's activation-derivative coefficients (dmip_train.hip, "records"); null: the
  // reverse half recomputes the forward instead
  uint32_t* rec;
};
constexpr int kTrainAdj = 12;  // abP[2] abV[2] abC[2] dsm ic pde, padded to 48 bytes
constexpr int kTrainRecQ = 6;  // record quantities per unit: h_P, h_V, h_C (bf16), d1 (fp16), d2 z_V (bf16), d1_C (fp16)
constexpr int kTrainRecTileBytes = kTrainRecQ * 64 * 16 * 2;  // one (tile, layer): 16 units x 16 samples per lane group

bool train_split();
int train_nparam(int n_hidden);
int train_partial_stride(int n_hidden);
int train_waves_per_wg();
int train_partials_per_wg();
int train_packed_bytes(int n_hidden);
size_t train_adj_bytes(long long batch);  // 0 unless the forward / reverse split kernels run (incl. the records)
bool train_rec();  // the record reverse half (DMIP_TRAIN_REC, default on) instead of the recomputing one
hipError_t launch_loss_grad(const TrainParams& p, int n_hidden, float* grads, float* loss_out, float* partials,
                            int n_wg, hipStream_t st);

// Scatterometry surrogate (dmip_surrogate.hip): 3 -> 256 -> 256 -> 256 -> 23 ReLU, exact f32 MFMA.
constexpr int kSurW = 256, kSurXdim = 3, kSurYdim = 23;

struct SurrogateParams {
  // packed f32 weight images (dmip_capi.cpp pack_surrogate)
  const float* l1;     // [16 tiles][64 lanes]: W1 | b1 as k = 0..3
  const char* w2;      // [16 tiles][16 q][64][4] forward 256 x 256 images
  const char* w3;
  const char* w4;      // [2 tiles][16 q][64][4] output layer, rows >= 23 zero
  const char* w3t;     // transposed images for the reverse pass
  const char* w2t;
  const char* w4t;     // [16 tiles][2 q][64][4]
  const char* w1t;     // [16 q][64][4] (rows >= 3 zero)
  const float* bias;   // b1 | b2 | b3 [256] | b4 [32]
  // evaluation
  const float* x;      // [n][3]
  const float* y;      // [n][23] (y_stride = 23) or one row (0)
  long long y_stride;
  long long n;
  float* f_out;        // [n][23]
  float* e_out;        // [n]  (MH: [n_y][n_chains] E(x_S) - E(x_0), optional)
  float* g_out;        // [n][3]
  float a, b2, lam;    // noise model a, b^2 and the boundary weight lambda
  // Metropolis-Hastings
  long long n_chains, chain_offset;
  int num_steps;
  float noise_std;
  unsigned long long seed;
  const float* x_init; // [n_y][n_chains][3] or null (uniform on [-1, 1]^3 from the RNG)
  const float* noise;  // injected proposals [S][n_y][n_chains][3] or null
  const float* unif;   // injected uniforms  [S][n_y][n_chains]
  float* x_out;        // [n_y][n_chains][3]
};

// DPS sampler (config 4): the prior score network MLP2 (x, t) -> x in exact f32 with forward-mode
// Jacobian, the surrogate residual gradient, the EM predictor (dmip_surrogate.hip dps_kernel).
constexpr int kDpsPriorW = 256;

struct DpsParams {
  SurrogateParams s;   // surrogate images (forward + reverse) and y_obs in s.y ([n_y][23])
  const float* pl1;    // prior layer 1 [16 tiles][2 k-steps][64]: (W1 x-cols | t-col), (b1, 0, 0, 0)
  const char* pw2;     // prior 256 x 256 images [16][16][64][4]
  const char* pw3;
  const char* pw4;     // prior output [1 tile][16][64][4] (rows >= 3 zero)
  const float* pbias;  // b2 | b3 [256] | b4 [16]
  float T, bmin, bdiff, delta, sqrt_delta, mean, stdv, zeta;
  int mode;            // 0: NLL guidance (zeta grad log p(y|x0) in the score), 1: Chung residual-norm step
};

hipError_t launch_dps(const DpsParams& p, int n_y, hipStream_t st);

// DPS at fp32 accuracy on the fp16 matrix rate (dmip_dps_x3.hip): x3-split images of the prior (MLP2 [256]^3, x 3)
// and of the surrogate, packed by dmip_capi.cpp (pack_dps_x3_prior / pack_dps_x3_surrogate)
constexpr int kDpsX3Chunk = 32768;
constexpr int kDpsX3PriorChunks = 35;  // P2 (8) | P3 (8) | Pout (1) | P4^T (1) | P3^T (8) | P2^T (8) | P1^T (1)
constexpr int kDpsX3SurChunks = 35;    // S2 (8) | S3 (8) | Sout (1) | S4^T (1) | S3^T (8) | S2^T (8) | S1^T (1)
struct DpsX3Params {
  const char* pimg;     // the prior's chunks [35][32 KiB]
  const char* simg;     // the surrogate's chunks [35][32 KiB]
  const char* pl1;      // prior layer 1 over (x, t), split, scaled by 2 log2 e: [16 tiles][64][8] fp16
  const char* sl1;      // surrogate layer 1 over x, split: [16][64][8] fp16
  const float* pbias;   // prior: c b1 | folded init2 | folded init3 [256] | folded output init [16]
  const float* sbias;   // surrogate: b1 | b2 | b3 [256] | b4 [32]
  const float* y;       // [n_y][23]
  long long n_chains, chain_offset;
  int num_steps;
  float T, bmin, bdiff, delta, sqrt_delta, mean, stdv, zeta;
  int mode;             // 0: NLL guidance, 1: residual-norm step (DpsParams)
  float a, b2;          // the noise model (NLL mode)
  unsigned long long seed;
  float* x_out;         // [n_y][n_chains][3]
  unsigned int* err;    // device status word (kErrRange)
  const float* coef;    // per-step (tau, beta, g, 0), (mean_weight, var, 0, 0): filled by launch_dps_x3
  const char* img;      // the per-step chunk stream in stream order [70][32 KiB]: filled by launch_dps_x3
};
hipError_t launch_dps_x3(const DpsX3Params& p, int n_y, hipStream_t st);

// fp32x3 random-walk MH (dmip_dps_x3.hip mh_x3_kernel): the surrogate's forward chunks S2 | S3 | Sout of the DPS image
constexpr int kDpsX3SurFwdChunks = 17;
struct MhX3Params {
  const char* simg;     // the surrogate's fp32x3 chunks (DpsX3Params::simg; the first 17 used)
  const char* sl1;      // its layer 1 over x, split: [16][64][8] fp16
  const float* sbias;   // b1 | b2 | b3 [256] | b4 [32]
  const float* y;       // [n_y][23]
  long long n_chains, chain_offset;
  int num_steps;
  float noise_std, a, b2, lam;
  unsigned long long seed;
  const float* x_init;  // [n_y][n_chains][3] or null (x0 ~ U[-1, 1]^3 from the chain RNG)
  float* x_out;         // [n_y][n_chains][3]
  float* e_out;         // [n_y][n_chains] E(x_S) - E(x_0), or null
  unsigned int* err;    // device status word (kErrRange)
};
hipError_t launch_mh_x3(const MhX3Params& p, int n_y, hipStream_t st);

hipError_t launch_surrogate_eval(const SurrogateParams& p, int mode, int n_wg, hipStream_t st);
int surrogate_rows_per_wg();
hipError_t launch_mh(const SurrogateParams& p, int n_y, hipStream_t st);

// Exact-f32 networks (dmip_f32.hip, DMIP_PREC_F32): images packed by dmip_capi.cpp pack_f32_net.
struct F32Net {
  const float* l1;     // [W/16 tiles][K1Q][64]: layer 1 over every input column, then the bias column
  const char* stream;  // [(L-1) W/16 hidden tiles + OT output tiles][W/16 q][64][4] floats
  const float* bias;   // [(L-1)][W] hidden biases, then [16 OT] output bias (rows >= out_dim zero)
};

struct F32SamplerParams {
  F32Net net[2];              // net 0: CDE / CDiffE / likelihood; net 1: the Posterior prior
  const float* l1y;           // CDE / likelihood: per-y layer-1 images [n_y][W/16][K1Q][64] (y folded in)
  int n_hidden;
  const float* y_obs;         // CDiffE observations [n_y][ydim]
  int n_corr;
  float snr;
  const float* noise;         // CDE: injected normals [S+1][n_y][n_chains][D] or null
  float* x_out;               // [n_y][n_chains][D]
  float* snap_out;            // trajectory snapshots [S / snap_every][n_y][n_chains][D] or null
  int snap_every;             // 0: none
  long long n_chains, chain_offset;
  int num_steps;
  float T, bmin, bdiff, delta, sqrt_delta, mean, stdv;
  unsigned long long seed;
  // balanced schedule (as SamplerParams): hand-over state and flags per y and grid wave, the device
  // status word, the consumer's spin bound and the test hook (bit 0: producers never publish)
  float* xfer;
  unsigned int* xflag;
  unsigned int* err;
  unsigned int spin_limit;
  int debug_flags;
  int act;                    // 0 tanh, 1 SiLU (dmip_act: the activation chain; SiLU for SAMPLER_CDE only)
};

struct F32ForwardParams {
  F32Net net;
  int n_hidden;
  const float* x;
  const float* y;
  const float* t;
  float* out;
  long long n, y_stride;
  int t_stride, xdim, ydim, out_dim;
  int k1q;                    // layer-1 k-steps of the image: ceil((in_dim + 1) / 4)
  int act;                    // 0 tanh, 1 SiLU (dmip_act)
};

struct F32L1PrepParams {
  const float* w1;  // [width][in_dim] (nn.Linear layout)
  const float* b1;
  const float* y;   // [n_y][ydim]
  float* l1y;       // out: [n_y][width/16][k1q][64]
  int width, in_dim, xdim, ydim, k1q;
};

hipError_t launch_f32_sampler(const F32SamplerParams& p, int mode, int width, int n_hidden, int xdim, int ydim,
                              int n_y, hipStream_t st, bool* supported);
bool f32_sampler_supported(int mode, int width, int n_hidden, int xdim, int ydim);
hipError_t launch_f32_forward(const F32ForwardParams& p, int width, int ot, hipStream_t st, bool* supported);
hipError_t launch_f32_l1_prep(const F32L1PrepParams& p, int n_y, hipStream_t st);

// fp32-accurate split-fp16 networks (dmip_x3.h, DMIP_PREC_F32X3): images packed by dmip_capi.cpp pack_x3_net.
struct X3Net {
  const char* l1;      // [W/16 tiles][K1Q][64 lanes][8 fp16]: layer-1 image (x, t columns -- or every column, CDiffE)
  const char* stream;  // [(L-1) NCH hidden chunks + 1 output chunk][CHUNK bytes] (dmip_x3.h Shape)
  const float* bias;   // [L W + 16]: c b1 | folded hidden biases | folded output bias (rows 0..15)
  // the k-major engine (dmip_x3k.h; width 256, 3 hidden layers): W x W layers as [layer][k-step][16 tiles]
  // [hi, lo][64][8] and the output layer as [k-step][64][8] with rows 0..D-1 = W_hi, 4..4+D-1 = W_lo
  const char* kstream = nullptr;
  const char* kout = nullptr;
  // the paired-tile 32x32 engine (dmip_x3p.h; width 256, 3 hidden layers): 16 chunks of 32 KiB (hidden
  // layer 1 k-major [q][o][e][hi, lo][64][8], hidden layer 2 output-major [c][s][hi, lo][64][8]), layer 1
  // as [8 tiles][64][8], the output layer in f32 [c][lane half][row][4][4] + its init[16]
  const char* pstream = nullptr;
  const char* pl1 = nullptr;
  const float* pow = nullptr;
};

struct X3SamplerParams {
  X3Net net[2];               // net 0: CDE / CDiffE / likelihood; net 1: the Posterior prior
  const float* bias_y;        // CDE / likelihood: per-y layer-1 bias c (b1 + W1_y y) [n_y][W]
  int n_hidden;
  const float* y_obs;         // CDiffE observations [n_y][ydim]
  int n_corr;
  float snr;
  const float* noise;         // CDE: injected normals [S+1][n_y][n_chains][D] or null
  float* x_out;               // [n_y][n_chains][D]
  float* snap_out;            // trajectory snapshots or null
  int snap_every;
  long long n_chains, chain_offset;
  int num_steps;
  float T, bmin, bdiff, delta, sqrt_delta, mean, stdv;
  unsigned long long seed;
  float* xfer;                // balanced schedule hand-over (as SamplerParams)
  unsigned int* xflag;
  unsigned int* err;
  unsigned int spin_limit;
  int debug_flags;
  const float* coef;          // x3k: per-step (tau, beta, g, 0) [num_steps][4] of step_coef (its launch fills it)
  // the width-64 latency engine (dmip_x3s.h) with bias_y null: layer 1's per-y bias from W1 [W][l1_in], b1 and y_obs
  // [n_y][ydim] in the kernel, as x3_bias_prep_kernel forms it (no prep launch, no allocation)
  const float* l1w;
  const float* l1b;
  int l1_in, ydim;
};
// the latency engine takes this launch (CDE, width 64, xdim 2 or 3, 1-3 hidden layers, <= 1,024 tiles over all ys;
// DMIP_X3_SPLIT=0 opts out): launch_x3_sampler_cde's own test, exposed so the caller can skip the bias prep
bool x3s_sampler_eligible(int mode, int width, int n_hidden, int xdim, long long n_chains, int n_y);

struct X3BiasPrepParams {
  const float* w1;  // [width][in_dim] (nn.Linear layout)
  const float* b1;
  const float* y;   // [n_y][ydim]
  float* bias_y;    // out: [n_y][width] = c (b1 + W1_y y), f64 accumulation
  int width, in_dim, xdim, ydim;
};

hipError_t launch_x3_sampler(const X3SamplerParams& p, int mode, int width, int n_hidden, int xdim, int ydim, int n_y,
                             hipStream_t st, bool* supported);
bool x3_sampler_supported(int mode, int width, int n_hidden, int xdim, int ydim);
// the k-major multi-tile engine (dmip_x3k.h): CDE, width 256, 3 hidden layers, xdim 2 or 3
bool x3k_sampler_supported(int mode, int width, int n_hidden, int xdim);
hipError_t launch_x3k_sampler(const X3SamplerParams& p, int xdim, int n_y, hipStream_t st, bool* ok);
// the paired-tile 32x32 engine (dmip_x3p.h; A/B library only, opt-in DMIP_X3P=1): CDE, width 256, 3 hidden
// layers, xdim 2 or 3
bool x3p_sampler_supported(int mode, int width, int n_hidden, int xdim);
hipError_t launch_x3p_sampler(const X3SamplerParams& p, int xdim, int n_y, hipStream_t st, bool* ok);
hipError_t launch_x3_bias_prep(const X3BiasPrepParams& p, int n_y, hipStream_t st);
// geometry of the x3 images (dmip_x3.h Shape) for the host packer
int x3_chunk_bytes(int width);
int x3_tiles_per_chunk(int width);

// ---- exact-f32 training engine (dmip_gemm.hip): MFMA GEMM with fused epilogues
enum {
  GEMM_EPI_NONE = 0,      // C = acc
  GEMM_EPI_BIAS = 1,      // C = acc + bias[n]
  GEMM_EPI_BIAS_TANH = 2, // C = tanh(acc + bias[n]), aux_out = 1 - C^2
  GEMM_EPI_BIAS_TANH2 = 3,// C = tanh(tanh(acc + bias[n])), aux_out = its derivative
  GEMM_EPI_MUL_AUX = 4,   // C = acc * aux_in
  GEMM_EPI_WGRAD = 5      // columns < n-1 -> C ([dW]), column n-1 -> bias_out[m] ([db])
};

struct GemmParams {
  const float* a;
  const float* b;
  float* c;
  long long m, n, k;
  long long lda, ldb, ldc;
  int epi;
  const float* bias;
  const float* aux_in;    // MUL_AUX: [m][ldaux]
  float* aux_out;         // TANH epilogues: [m][ldaux]
  long long ldaux;
  float* bias_out;        // WGRAD: [m]
  float* part;            // split-K partials [splits][m][n]
};

struct PosteriorParams {
  long long batch;
  int xdim, ydim;
  float bmin, bdiff, lam;
  const float* x;         // [B][xdim]
  const float* y;         // [B][ydim]
  const float* t;         // [B]
  const float* eps;       // [B][xdim]
  float* alpha;           // [B]
  float* stdv;            // [B]
  float* x_t;             // [B][xdim]
  float* prior_in;        // [B][xdim + 2]: x_t, t, 1
  float* lik_in;          // [B][xdim + ydim + 2]: x_t, y, t, 1
  const float* s_prior;   // [B][xdim]
  const float* s_lik;     // [B][xdim]
  float* x0;              // [B][xdim]
  const float* u;         // [B][xdim]: J_F^T v (surrogate reverse pass)
  const float* jtu;       // [B][xdim + 1]: the prior's input gradient for the adjoint u
  float* target;          // [B][xdim]
  float* adj_prior;       // [B][xdim]
  float* adj_lik;         // [B][xdim]
  float* rows;            // [B][2]: per-row prior DSM and likelihood terms
  float* loss_out;        // [3]: loss, PriorLoss, LikelihoodLoss
};

// ---- exact-f32 score-matching losses at any width (dmip_jets.hip): stacked jet streams
constexpr int kJetsMaxLayers = 9;
// DSMLoss needs only the primal stream: any state dimension up to this (CDiffE trains on z = (x, y))
constexpr int kJetsMaxDsmDim = 64;

struct JetsParams {
  long long batch;
  int xdim, ydim, out_dim;
  float bmin, bdiff, lam, lam2;
  int has_dsm, pde, pde_l1, ic_l1;      // pde: 0 none, 1 ScoreFPE, 2 conditional ScoreFPE
  float icA[4], icb[2], icS[4];         // linear-problem IC target (used when ic_target is null)
  const float* x;                       // [B][xdim]
  const float* y;                       // [B][ydim]
  const float* t;                       // [B]
  const float* eps;                     // [B][xdim]
  const float* ic_target;               // [B][xdim] or null
  // stream blocks (B rows each): P = 0, then V, C, the first-order E_a and the second-order pairs
  int n_streams, n_bwd, blk_v, blk_c, blk_e, n_e, n_pair;
  float* scal;                          // [B][8]: alpha, std, beta, g, g'
  float* x_t;                           // [B][xdim]
  float* h[kJetsMaxLayers];             // layer inputs [n_streams B][in_l + 1]
  float* aux[kJetsMaxLayers];           // hidden layer l: [3][B][width_l] (d1, d2 z_V, d1 of C)
  float* z;                             // [n_streams B][max width] pre-activations
  float* a_out;                         // [n_streams B][out_dim]
  float* zbar;                          // [n_bwd][B][out_dim] output adjoints
  float* zbar_a;                        // [n_bwd B][max width] hidden adjoints (ping-pong)
  float* zbar_b;
  float* hbar;                          // [n_bwd B][max width]
  float* rows;                          // [B][3]: DSM, PDE, IC per row
  float* loss_out;                      // [4]: loss, PDE-Loss, Initial Condition, DSM
  float* part;                          // split-K partials
  int splits;
};

hipError_t launch_jets_loss_grad(const JetsParams& p, int n_hidden, const int* widths, const float* const* W,
                                 const float* const* b, float* grads, hipStream_t st);

hipError_t launch_gemm_f32(const GemmParams& p, bool ta, bool tb, int splits, hipStream_t st);
// split count of a weight-gradient GEMM [m x n] over k sample rows: ~4 workgroups per CU, >= 128 rows
// per split, at most cap
int gemm_wgrad_splits(long long m, long long n, long long k, int cap);

// ---- device-side rest of a training step (dmip_step.hip)
struct TrainDrawsParams {
  long long batch;
  int xdim, debias;
  unsigned long long seed, stream_id;
  float t_add, T;
  float a, b, te, r_te, A_te, Z;  // sample_vp_truncated_q constants (sdes.py), host-computed in f64
  float* t;                       // [B]
  float* eps;                     // [B][xdim]
  // captured step graphs (dmip_train_plan): the step's draw stream is stream_id + *draw_ctr, read on
  // the device, so one graph replays every step (null: stream_id alone)
  const unsigned long long* draw_ctr;
  // captured step graphs: the batch is copied from the caller's x / y into the graph's staging buffers by
  // the draws launch itself (the step updates x_src / y_src in the graph's kernel node; null: no copy)
  const float* x_src;
  const float* y_src;
  float* x_dst;
  float* y_dst;
  int ydim;
};

constexpr int kAdamMaxTensors = 16;

struct AdamParams {
  int n;
  float* param[kAdamMaxTensors];
  const float* grad[kAdamMaxTensors];
  float* m[kAdamMaxTensors];
  float* v[kAdamMaxTensors];
  long long off[kAdamMaxTensors + 1];  // prefix sums of the tensors' sizes
  // torch's scalars, each rounded from Python double as torch passes them: lerp weight 1 - beta1,
  // beta2, addcmul value 1 - beta2, eps, lr / bias_correction1, sqrt(bias_correction2)
  float w1, beta2, w2, eps, step_size, bc2_sqrt;
  // captured step graphs: the step is *step_ctr + 1 (torch increments before the update) and the
  // bias corrections are formed on the device in double from lr / beta1 / beta2 (null: the host's)
  const long long* step_ctr;
  double lr_d, beta1_d, beta2_d;
};

// the per-step counters a captured training-step graph advances at its end
struct StepCounters {
  unsigned long long draw;  // draws' stream offset
  long long step;           // optimizer steps taken
  unsigned int done;        // fused reduction + Adam: workgroups finished this step (the last advances the counters)
  unsigned int pad;
};
hipError_t launch_counters_advance(StepCounters* c, hipStream_t st);

// The captured bf16 training step's fused launches (dmip_train_plan; dmip_train.hip): the weight image's pack runs
// in the draws launch (plan_prologue_kernel: pack workgroups + draw workgroups), and the gradient reduction applies
// torch's Adam to each parameter it has just summed and, in its last workgroup, advances the step counters -- four
// launches per step (prologue, forward half, reverse half, reduction) instead of seven plus two batch copies.
struct TrainFuse {
  TrainDrawsParams draws;
  AdamParams adam;
  StepCounters* ctr;
};
hipError_t launch_loss_grad_fused(const TrainParams& p, int n_hidden, float* grads, float* loss_out, float* partials,
                                  int n_wg, const TrainFuse& f, hipStream_t st);
const void* train_plan_prologue_func(int n_hidden);  // the kernel node a plan step updates (bf16)
const void* train_draws_func();                      // the same for the exact-f32 plan

hipError_t launch_train_draws(const TrainDrawsParams& p, hipStream_t st);
hipError_t launch_adam(const AdamParams& p, hipStream_t st);
hipError_t launch_ones_column(float* h, long long rows, int ld, hipStream_t st);
hipError_t launch_posterior_stage(const PosteriorParams& p, int stage, hipStream_t st);

hipError_t launch_histogram(const float* x, long long n, int d, int nbins, double lo, double hi, int n_hist,
                            unsigned int* counts, hipStream_t st);

hipError_t launch_sampler(const SamplerParams& p, int mode, int width, int n_hidden, int xdim, int ydim, int n_y,
                          hipStream_t st, bool* supported);
bool sampler_shape_supported(int mode, int width, int n_hidden, int xdim, int ydim);
bool forward_split(int width, int in_dim);
hipError_t launch_forward(const ForwardParams& p, int width, int n_hidden, int in_dim, hipStream_t st,
                          bool* supported);
hipError_t launch_a1_prep(const A1PrepParams& p, int n_y, hipStream_t st);
hipError_t launch_rng_words(unsigned long long seed, long long off, unsigned long long stream, long long n,
                            int n_words, unsigned int* out, hipStream_t st);
hipError_t launch_rng_normals(unsigned long long seed, long long off, unsigned long long stream, long long n,
                              int n_pairs, float* out, hipStream_t st);
hipError_t launch_schedule(int S, float T, float bmin, float bdiff, float* out, hipStream_t st);

}  // namespace dmip
