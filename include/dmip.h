/* dmip.h -- C ABI of libdmip.so, the MI355X (gfx950) conditional score-diffusion posterior
 * sampler. Plain pointers and sizes only; every device pointer is caller-owned HIP device memory
 * and every call is asynchronous on the given hipStream_t (passed as void*; NULL = default stream).
 *
 * The reference (maffos/Diffusion-Modelling-for-inverse-problems) has no FFI: its boundary is the
 * Python object API. Each entry point below states the reference interface it replaces; the
 * Python host package (diffusion-modelling-for-inverse-problems_amd/) binds these with ctypes
 *  behind the reference's own class and function names.
 *
 * Errors: every function returns a dmip_status; on failure dmip_last_error() (thread-local)
 * describes it. Handles are immutable after creation and may be shared between threads.
 */
#ifndef DMIP_H_
#define DMIP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DMIP_ABI_VERSION 9

typedef enum {
  DMIP_OK = 0,
  DMIP_ERR_INVALID = 1,     /* bad argument (maps to ValueError)                  */
  DMIP_ERR_UNSUPPORTED = 2, /* shape with no compiled kernel (maps to ValueError) */
  DMIP_ERR_HIP = 3,         /* HIP runtime failure (maps to RuntimeError)          */
  DMIP_ERR_ALLOC = 4        /* device allocation failure (maps to RuntimeError)    */
} dmip_status;

/* Column layout of the network input (nets.py:33 MLP: cat[x, y, t]; nets.py:54 MLP2: cat[x, t]). */
typedef enum { DMIP_INPUT_X_Y_T = 0, DMIP_INPUT_X_T = 1 } dmip_input_layout;

/* Activation chain (nets.py:17-30): Linear -> Tanh -> Tanh -> [Linear -> Tanh]*(L-1) -> Linear.
 * The first hidden layer applies tanh twice because MLP registers its activation module a second
 * time as `self.act` (nets.py:26). DMIP_ACT_TANH is the single-tanh chain (not compiled).
 * DMIP_ACT_SILU_TWICE_FIRST (ABI 8): the same chain for an MLP built with nn.SiLU() (nets.py:17's `activation`
 * argument; SiLU(z) = z sigmoid(z)), twice on layer 1 by the same registration. It is compiled for the exact-f32
 * network forward (dmip_mlp_forward at DMIP_PREC_F32 / F32X3) and the exact-f32 CDE sampler (dmip_em_sample at
 * DMIP_PREC_F32); every other entry point refuses a SiLU network with DMIP_ERR_UNSUPPORTED. */
typedef enum { DMIP_ACT_TANH_TWICE_FIRST = 0, DMIP_ACT_TANH = 1, DMIP_ACT_SILU_TWICE_FIRST = 2 } dmip_act;

/* Arithmetic of the network GEMMs; the chain state, the schedule and the SDE update are fp32 in both.
 *   DMIP_PREC_FP16  16-bit MFMA operands, fp32 accumulation: layer 1 is a bf16 MFMA over split hi+lo
 *                   bf16 inputs (~fp32), the hidden and output layers fp16 MFMAs over fp16 weights and
 *                   activations (3 more mantissa bits than bf16 at the same rate); tanh by exp2 + rcp,
 *                   layer 1's double tanh in packed fp16. The throughput mode.
 *                   DMIP_PREC_BF16 is the same value: for the samplers and the network forward a deprecated
 *                   name of DMIP_PREC_FP16; for the config-5 training kernel (dmip_loss_grad,
 *                   dmip_train_plan_desc) the name of what it computes (split-bf16 products).
 *   DMIP_PREC_F32   exact f32: every product and sum in f32 (v_mfma_f32_16x16x4_f32, an fmaf chain),
 *                   libm-accurate tanh -- the reference's own arithmetic (nets.py:32-35 in fp32).
 *                   The bit-level parity mode; ~1/10 of the fp16 throughput.
 *   DMIP_PREC_F32X3 fp32-accurate at the fp16 matrix rate: every product as the three-term fp16 split
 *                   W_hi h_hi + W_hi h_lo + W_lo h_hi on v_mfma_f32_16x16x32_f16 (fp32 accumulation; error
 *                   2^-23.2 of sum |w h| measured against 2^-23.0 for an f32 fmaf chain), tanh by exp2 + rcp
 *                   at ~1 ulp (no polynomial). The reference-precision throughput mode (samplers; the
 *                   network forward runs the exact-f32 kernel).
 *                   Range: the split holds a value to ~2^-22 relative for |v| <= 65504 (fp16's largest
 *                   finite value) and to ~2^-24 absolute below 2^-14 (fp16 subnormals). The scaled weights
 *                   (layer 1 x 2 log2(e), hidden layers x 4 log2(e), output rows x 2) must fit (the folded
 *                   biases stay f32): a network that does not is refused at sampling time (DMIP_ERR_UNSUPPORTED, "fp16
 *                   range"). The layer-1 inputs (chain state x, t; CDiffE's y_t) are checked in the kernel --
 *                   at every step, or (the headline CDE engine) on each segment's final state, where an input
 *                   that left the range shows as non-finite or > 65504: a chain that leaves the range is
 *                   reported by dmip_device_status ("fp16 range") -- those chains are not fp32-accurate. The
 *                   Python estimators resample with DMIP_PREC_F32 then.
 * All three draw the same RNG stream per chain, so the modes are comparable chain by chain. */
typedef enum {
  DMIP_PREC_FP16 = 0,
  DMIP_PREC_F32 = 1,
  DMIP_PREC_F32X3 = 2,
  DMIP_PREC_BF16 = DMIP_PREC_FP16 /* see above: the training kernel's split-bf16; the samplers' deprecated name */
} dmip_precision;

/* VariancePreservingSDE (sdes.py:9-19): beta(t) = beta_min + (beta_max - beta_min) t. */
typedef struct {
  double beta_min; /* python floats of the reference; rounded to fp32 exactly where torch rounds */
  double beta_max;
  double T;
} dmip_vpsde;

/* The three estimators' reverse samplers (models/diffusion.py:59-229). */
typedef enum { DMIP_SAMPLER_CDE = 0, DMIP_SAMPLER_POSTERIOR = 1, DMIP_SAMPLER_CDIFFE = 2 } dmip_sampler_mode;

typedef struct dmip_mlp dmip_mlp;

/* Create a score-network handle from fp32 host weights (nn.Linear layout W[out][in], b[out]).
 * Replaces: constructing nets.MLP / nets.MLP2 (nets.py:17-57) and moving it to the device
 * (models/diffusion.py:66-71, 187-199); weights in the reference state_dict order 0,3,5,7.
 *   in_dim       network input width (x + y + 1 for X_Y_T, x + 1 for X_T)
 *   out_dim      network output width (the `a` drift, xdim for CDE)
 *   n_hidden     number of hidden layers L (len(hidden_layers))
 *   widths       L hidden widths (all equal; 64, 128 or 256 compiled)
 *   weights[i]   layer i weight, i = 0..L (L+1 linear layers)
 *   biases[i]    layer i bias
 * The handle owns packed device copies (16-bit MFMA fragments in the kernels' layouts, and the exact-f32
 * images of the DMIP_PREC_F32 kernels). */
int dmip_mlp_create(int in_dim, int out_dim, int n_hidden, const int* widths, int act_mode, int input_layout,
                    int xdim, const float* const* weights, const float* const* biases, dmip_mlp** out);

int dmip_mlp_destroy(dmip_mlp* net);

/* out[n][out_dim] = net(cat[x, y, t]) for arbitrary rows.
 * Replaces: MLP.forward / MLP2.forward (nets.py:32-35, 52-57), i.e. model.sde.a(x, y, t) as used by
 * the evaluate() score-MSE (main_diffusion_scatterometry.py:65-67) and the losses.
 *   y_stride  0: one y row broadcast to all rows; ydim: per-row y      (ignored for X_T)
 *   t_stride  0: one t broadcast;                 1: per-row t */
int dmip_mlp_forward(const dmip_mlp* net, const float* x_dev, const float* y_dev, int64_t y_stride,
                     const float* t_dev, int t_stride, int64_t n, float* out_dev, int precision, void* stream);

/* Fused reverse-time Euler-Maruyama posterior sampler (one launch for all num_steps).
 * Replaces: BaseClassDiffusionModel.forward (models/diffusion.py:27-46) for CDE, i.e.
 * x0 = randn*std + mean; for i < S: x <- x + delta*mu(t_i, x, y) + sqrt(delta)*sigma*xi_i with
 * mu = g(T-t) a(x, y, T-t) + 0.5 beta(T-t) x and sigma = g(T-t) (sdes.py:77-87), ts = linspace(0,1,S+1)*T.
 *   y_dev       [n_y][ydim] conditioning observations; chains of y index k go to x_out[k]
 *   n_chains    chains per y;  chain_offset: global index of chain 0 (keys the RNG, so a shard of a
 *               larger run draws exactly the chains it would draw in the full run)
 *   seed        RNG seed; the chain-c stream of y index k is a function of (seed, chain_offset + c, k)
 *   noise_dev   NULL for the internal RNG, or injected standard normals [S+1][n_y][n_chains][xdim]
 *               (slot 0 -> x0) to replay a captured reference trajectory
 *   x_out_dev   [n_y][n_chains][xdim] fp32 */
int dmip_em_sample(const dmip_mlp* net, const dmip_vpsde* sde, const float* y_dev, int n_y, int ydim, int xdim,
                   int64_t n_chains, int64_t chain_offset, int num_steps, float mean, float stdv, uint64_t seed,
                   int precision, const float* noise_dev, float* x_out_dev, void* stream);

/* Fused sampler of the PosteriorDiffusionEstimator (models/diffusion.py:182-229): the same EM loop as
 * dmip_em_sample with a = PosteriorScore(x, y, T-t) = g(T-t) (prior(x, T-t) + likelihood(x, y, T-t))
 * (nets.py:143-157). Both networks are evaluated in the same kernel from one shared weight ring.
 *   prior       MLP2 handle (DMIP_INPUT_X_T, in_dim = xdim + 1, out_dim = xdim)
 *   likelihood  MLP handle (DMIP_INPUT_X_Y_T, in_dim = xdim + ydim + 1, out_dim = xdim)
 * Both must have the same hidden width and depth. Other arguments as dmip_em_sample (no injection). */
int dmip_em_sample_posterior(const dmip_mlp* prior, const dmip_mlp* likelihood, const dmip_vpsde* sde,
                             const float* y_dev, int n_y, int ydim, int xdim, int64_t n_chains, int64_t chain_offset,
                             int num_steps, float mean, float stdv, uint64_t seed, int precision, float* x_out_dev,
                             void* stream);

/* Fused sampler of CDiffE (models/diffusion.py:109-180; the reference's loop raises TypeError at
 * :174, so this implements the repaired semantics consistent with its training, :129-137): every
 * step re-diffuses the observation, y_t = eps std(T-t) + mean_weight(T-t) y (sdes.py:37-44), evaluates
 * the joint score a(x, y_t, T-t) (out_dim = xdim + ydim) and takes the EM step on the x part.
 *   net   MLP handle (DMIP_INPUT_X_Y_T, in_dim = xdim + ydim + 1, out_dim = xdim + ydim)
 *   corrector_steps, snr   predictor-corrector sampling (BASELINE config 3; no reference code): before
 *         each predictor step, corrector_steps Langevin steps at the same time and y_t (Song et al.
 *         2021): s = a/g on the x rows, eps = 2 alpha (snr |z| / |s|)^2 with the norms at their
 *         expected values for the VP perturbation kernel, i.e. eps = 2 alpha snr^2 var(T-t) (one step
 *         size per time step, as score_sde's batch-averaged norms; a per-chain ratio diverges),
 *         x <- x + eps s + sqrt(2 eps) z, alpha = exp(-beta(T-t) delta) (score_sde's discrete VP
 *         alpha 1 - beta delta to first order, positive at any step count). 0 = plain EM.
 *         snr is therefore NOT score_sde's measured-norm snr: score_sde measures |s| on the batch, so
 *         for a trained score whose norm differs from sqrt(d)/std(T-t) the same snr value takes a
 *         different step here than there (the step is a fixed function of t, shard-invariant).
 * Other arguments as dmip_em_sample (no injection). */
int dmip_em_sample_cdiffe(const dmip_mlp* net, const dmip_vpsde* sde, const float* y_dev, int n_y, int ydim, int xdim,
                          int64_t n_chains, int64_t chain_offset, int num_steps, float mean, float stdv, uint64_t seed,
                          int precision, int corrector_steps, float snr, float* x_out_dev, void* stream);

/* Trajectory snapshots (north_star: "coalesced HBM writes only at snapshot steps"). The sampler of
 * `mode` (DMIP_SAMPLER_CDE: net; _POSTERIOR: net = the likelihood, prior = the prior; _CDIFFE: net, with
 * corrector_steps / snr as dmip_em_sample_cdiffe) in one launch as above, which additionally writes
 * every chain's x after each snapshot_every-th EM step:
 *   snap_out_dev  [num_steps / snapshot_every][n_y][n_chains][xdim] fp32, slot k = x after step
 *                 (k + 1) * snapshot_every (the last slot equals x_out when snapshot_every divides num_steps)
 * The reference keeps only the final samples (models/diffusion.py:27-46); the snapshots are the states
 * its loop holds at those steps. Between snapshots chain state stays in registers. */
int dmip_em_sample_snapshots(int mode, const dmip_mlp* net, const dmip_mlp* prior, const dmip_vpsde* sde,
                             const float* y_dev, int n_y, int ydim, int xdim, int64_t n_chains, int64_t chain_offset,
                             int num_steps, float mean, float stdv, uint64_t seed, int precision, int corrector_steps,
                             float snr, int snapshot_every, float* snap_out_dev, float* x_out_dev, void* stream);

/* ---- training: fused loss value + parameter gradients ----------------------------------------- */
typedef enum { DMIP_LOSS_DSM = 0, DMIP_LOSS_DSM_PDE = 1, DMIP_LOSS_PINN = 2, DMIP_LOSS_PINN2 = 3 } dmip_loss_kind;
typedef enum { DMIP_PDE_NONE = 0, DMIP_PDE_FPE = 1, DMIP_PDE_CFPE = 2 } dmip_pde_kind;
typedef enum { DMIP_METRIC_L1 = 0, DMIP_METRIC_L2 = 1 } dmip_metric;

/* Loss configuration, mirroring the reference loss objects (losses.py:126-290):
 *   kind        DSMLoss (.mean() as CDE.train_epoch takes it), DSM_PDELoss, PINNLoss, PINNLoss2
 *   pde         ScoreFPELoss (exact divergence) or ConditionalScoreFPELoss; NONE for DSM
 *   pde_metric / ic_metric   L1 / L2;  lam, lam2 the PDE / initial-condition weights
 *   ic_A, ic_b, ic_Sinv      initial-condition target of PINNLoss(2): the linear problem's analytic
 *               posterior score -x + ((y - (A x + b)) Sinv^T) A (linear_problem.py:61-65), row-major 2x2 */
typedef struct {
  int kind, pde, pde_metric, ic_metric;
  float lam, lam2;
  float ic_A[4], ic_b[2], ic_Sinv[4];
} dmip_loss_cfg;

/* One training step's loss and gradients for the CDE score network, fused (forward jets, per-sample
 * loss terms, hand-written reverse pass, deterministic batch reduction).
 * Replaces: the loss_fn(...) call + loss.backward() inside CDE.train_epoch (models/diffusion.py:80-89)
 * for DSMLoss / DSM_PDELoss / PINNLoss / PINNLoss2 (losses.py:42-290), with the forward diffusion
 * x_t = eps std(t) + mean_weight(t) x done in the kernel (sdes.py:37-49).
 *   weights_dev / biases_dev   device fp32 parameters of the n_hidden + 1 linear layers (the torch
 *               parameters themselves, nn.Linear layout); read, not modified
 *   x_dev [batch][xdim], y_dev [batch][ydim], t_dev [batch] (sample_t), eps_dev [batch][xdim]
 *   grad_out_dev  [n_params] fp32, written (not accumulated) in the reference parameter order
 *               (0.weight, 0.bias, 3.weight, 3.bias, ...)
 *   loss_out_dev  [4] fp32: the loss, and the PDE / initial-condition / DSM component means
 * Compiled for the linear problem's network: in_dim 5, out_dim 2, xdim 2, widths 64, n_hidden 2 or 3. */
int dmip_loss_grad(int in_dim, int out_dim, int n_hidden, const int* widths, int xdim,
                   const float* const* weights_dev, const float* const* biases_dev, const dmip_vpsde* sde,
                   const dmip_loss_cfg* cfg, const float* x_dev, const float* y_dev, const float* t_dev,
                   const float* eps_dev, int64_t batch, float* grad_out_dev, float* loss_out_dev, void* stream);

/* The same losses, gradients and outputs in exact f32 at any network shape (hidden widths up to 4096,
 * 1-8 hidden layers, xdim <= 4; the reference configs' [512]*3 included): forward-mode jets as
 * stacked streams through MFMA GEMMs with fused epilogues (dmip_jets.hip), reverse pass through the
 * primal, time-tangent and initial-condition streams, deterministic split-K reductions.
 *   ic_target_dev  [batch][xdim] initial-condition target score_posterior(x, y) (PINNLoss's
 *                  initial_condition, e.g. the scatterometry -energy_grad, main_diffusion_scatterometry.py:
 *                  142-145), or NULL for the linear problem's analytic target from cfg (xdim = ydim = 2) */
int dmip_loss_grad_f32(int in_dim, int out_dim, int n_hidden, const int* widths, int xdim,
                       const float* const* weights_dev, const float* const* biases_dev, const dmip_vpsde* sde,
                       const dmip_loss_cfg* cfg, const float* x_dev, const float* y_dev, const float* t_dev,
                       const float* eps_dev, const float* ic_target_dev, int64_t batch, float* grad_out_dev,
                       float* loss_out_dev, void* stream);

/* The rest of a training step on the device (dmip_step.hip), so a whole step is a few launches:
 * dmip_train_draws  the batch's diffusion times t (BaseClassDiffusionModel.sample_t, models/diffusion.py:
 *                   48-58: debias = the truncated beta/var inverse-CDF sampler (sdes.py sample_vp_truncated_q
 *                   restated), else uniform; + t_add with the t > T correction) and the forward-diffusion
 *                   noise eps [batch][xdim] (sdes.py:37-49), from the chain-keyed generator
 *                   (seed, sample index, stream_id)
 * dmip_adam_step    torch.optim.Adam's update (amsgrad off, no weight decay; step = the step count after
 *                   the increment) on the optimizer's own exp_avg / exp_avg_sq tensors, all parameter
 *                   tensors (<= 16) in one launch */
int dmip_train_draws(uint64_t seed, uint64_t stream_id, int64_t batch, int xdim, int debias, const dmip_vpsde* sde,
                     double t_epsilon, float t_add, float* t_out_dev, float* eps_out_dev, void* stream);
int dmip_adam_step(int n_tensors, float* const* params, const float* const* grads, float* const* exp_avg,
                   float* const* exp_avg_sq, const int64_t* numel, double lr, double beta1, double beta2, double eps,
                   int64_t step, void* stream);

/* One whole CDE training step as a captured hipGraph (HIP graphs in place of a tracing compiler): the
 * step's launches -- dmip_train_draws, the loss + gradients (dmip_loss_grad_f32's sequence, or the bf16
 * kernel), dmip_adam_step -- recorded once for a fixed batch size with persistent scratch, and replayed
 * per batch by one hipGraphLaunch after copying the batch into the plan's staging buffers. The per-step
 * scalars live in a device counter pair the graph advances at its end: the draws' stream id is
 * first_draw + (steps replayed), Adam's step is step0 + (steps replayed) + 1, with its bias corrections
 * formed on the device in double. Replaces, per batch, the body of CDE.train_epoch's loop
 * (models/diffusion.py:76-102: sample_t, base_sde.sample, loss_fn, backward, optimizer.step).
 *   grads        consecutive views of one flat fp32 buffer in the reference parameter order (the
 *                loss writes it); params / exp_avg / exp_avg_sq / numel as dmip_adam_step
 *   cfg          as dmip_loss_grad_f32, with the built-in (linear-problem) initial condition only
 *   t_dev [batch], eps_dev [batch][xdim], loss_dev [4] (loss, PDE, IC, DSM): caller-owned device buffers
 *                the replays write (the latest step's draws and loss) */
typedef struct dmip_train_plan dmip_train_plan;
typedef struct {
  int in_dim, out_dim, n_hidden;
  const int* widths;
  int xdim;
  const float* const* weights_dev;
  const float* const* biases_dev;
  dmip_vpsde sde;
  dmip_loss_cfg cfg;
  int precision;                       /* DMIP_PREC_F32 (any width) or DMIP_PREC_BF16 (config-5 kernel) */
  int64_t batch;
  uint64_t seed, first_draw;           /* draws: (seed, sample, first_draw + step) */
  int debias;
  double t_epsilon;
  float t_add;
  int n_tensors;
  float* const* params;
  float* const* grads;
  float* const* exp_avg;
  float* const* exp_avg_sq;
  const int64_t* numel;
  double lr, beta1, beta2, eps;
  int64_t step0;                       /* optimizer steps already taken */
  float* t_dev;
  float* eps_dev;
  float* loss_dev;
} dmip_train_plan_desc;
int dmip_train_plan_create(const dmip_train_plan_desc* desc, dmip_train_plan** out);
int dmip_train_plan_step(dmip_train_plan* plan, const float* x_dev, const float* y_dev, void* stream);
/* set the counters (draws = the stream offset past first_draw, steps = optimizer steps taken), e.g. after
 * steps taken outside the plan; synchronises the stream */
int dmip_train_plan_set_counters(dmip_train_plan* plan, uint64_t draws_done, int64_t steps_done, void* stream);
int dmip_train_plan_destroy(dmip_train_plan* plan);

/* Non-zero when dmip_loss_grad has a kernel for this network shape. */
int dmip_loss_grad_supported(int in_dim, int out_dim, int n_hidden, const int* widths, int xdim);

/* ---- evaluation ------------------------------------------------------------------------------ */
/* counts[h][b0][b1]...[b_{d-1}] += number of points of x[h] in that bin, binned exactly like
 * numpy.histogramdd(x[h], bins=(nbins,)*d, range=[(lo, hi)]*d) (float64 edges, right edge closed,
 * outside points dropped). Replaces: the np.histogramdd calls of the evaluate drivers
 * (main_diffusion_scatterometry.py:71-74).
 *   x_dev      [n_hist][n][d] fp32;  d in 1..3
 *   counts_dev [n_hist][nbins^d] 32-bit counters, accumulated (zero it first); uint32 in the kernel --
 *              an int32 buffer (what the Python layer allocates) holds the same bits for counts < 2^31 */
int dmip_histogram(const float* x_dev, int64_t n, int d, int nbins, double lo, double hi, int n_hist,
                   uint32_t* counts_dev, void* stream);

/* ---- scatterometry forward model --------------------------------------- */
typedef struct dmip_surrogate dmip_surrogate;

/* Noise model and prior of the scatterometry problem (utils_scatterometry.py:18-21): y = f(x) +
 * b eps1 + a f(x) eps2, boundary-penalty prior with weight lambd_bd. */
typedef struct {
  float a, b, lambd_bd;
} dmip_scat_noise;

/* Create a handle for the frozen scatterometry surrogate nn.Sequential(Linear(3,256), ReLU,
 * Linear(256,256), ReLU, Linear(256,256), ReLU, Linear(256,23)) from fp32 host weights (state_dict
 * keys 0, 2, 4, 6; nn.Linear layout). Replaces: load_forward_model (utils_scatterometry.py:8-25).
 * Compiled for exactly that shape (in 3, widths [256]*3, out 23); arithmetic is exact f32 (f32
 * MFMA, fmaf-chain accumulation). */
int dmip_surrogate_create(int in_dim, int out_dim, int n_hidden, const int* widths, const float* const* weights,
                          const float* const* biases, dmip_surrogate** out);
int dmip_surrogate_destroy(dmip_surrogate* s);

/* f_out[n][23] = forward_model(x[n][3]) (the surrogate's forward, e.g. datasets.py:11-13). */
int dmip_surrogate_forward(const dmip_surrogate* s, const float* x_dev, int64_t n, float* f_out_dev, void* stream);

/* e_out[n] = get_log_posterior(x, forward_model, a, b, y, lambd_bd) (utils_scatterometry.py:30-38,
 * the NEGATIVE log posterior up to a constant) and, if grad_out_dev is not NULL, grad_out[n][3] =
 * d e / d x as energy_grad computes it by autograd (models/SNF.py:234-237; the posterior score is
 * its negative, main_diffusion_scatterometry.py:65-66).
 *   y_dev [n][23] (y_stride = 23) or one observation broadcast to all rows (y_stride = 0) */
int dmip_log_posterior(const dmip_surrogate* s, const dmip_scat_noise* noise, const float* x_dev, const float* y_dev,
                       int64_t y_stride, int64_t n, float* e_out_dev, float* grad_out_dev, void* stream);

/* Random-walk Metropolis-Hastings ground-truth sampler, fused (all steps in one launch, chain state
 * in registers). Replaces: anneal_to_energy(x0, energy, METR_STEPS, noise_std) (models/SNF.py:250-275)
 * with energy = get_log_posterior(., y) as generate_scatterometry_ground_truth.py:26-28,59-62 drives it:
 * x_prop = x + noise_std xi, accept iff u < exp(E(x) - E(x_prop)).
 *   y_dev       [n_y][23]; chains of y index k go to x_out[k]
 *   x_init_dev  [n_y][n_chains][3] start points, or NULL for x0 ~ U[-1, 1]^3 from the chain RNG
 *               (torch.rand(n, 3) * 2 - 1, generate_scatterometry_ground_truth.py:27)
 *   noise_dev / unif_dev   NULL, or injected proposal normals [S][n_y][n_chains][3] and acceptance
 *               uniforms [S][n_y][n_chains] (replaying captured draws; both or neither)
 *   x_out_dev   [n_y][n_chains][3];  e_out_dev (optional) [n_y][n_chains] = E(x_S) - E(x_0)
 * The RNG stream of chain c of y index k is a function of (seed, chain_offset + c, k). */
int dmip_mh_sample(const dmip_surrogate* s, const dmip_scat_noise* noise, const float* y_dev, int n_y,
                   int64_t n_chains, int64_t chain_offset, int num_steps, float noise_std, uint64_t seed,
                   const float* x_init_dev, const float* noise_dev, const float* unif_dev, float* x_out_dev,
                   float* e_out_dev, void* stream);

/* dmip_mh_sample with a precision (ABI 9): DMIP_PREC_F32 = dmip_mh_sample; DMIP_PREC_F32X3 = the same chains with
 * the surrogate's products as the three-term fp16 split of the fp32x3 samplers (the forward half of
 * dmip_dps_sample_ex's surrogate pass) -- the same RNG stream, proposals, energy and acceptance test per chain.
 * fp32x3 takes no injected draws (DMIP_ERR_UNSUPPORTED); a weight beyond fp16's range is refused
 * (DMIP_ERR_UNSUPPORTED, "fp16 range"); a proposal or hidden activation beyond it is reported by
 * dmip_device_status ("fp16 range"), and the Python caller then resamples with DMIP_PREC_F32. */
int dmip_mh_sample_ex(const dmip_surrogate* s, const dmip_scat_noise* noise, const float* y_dev, int n_y,
                      int64_t n_chains, int64_t chain_offset, int num_steps, float noise_std, uint64_t seed,
                      const float* x_init_dev, const float* noise_dev, const float* unif_dev, int precision,
                      float* x_out_dev, float* e_out_dev, void* stream);

/* Diffusion posterior sampling (DPS, Chung et al. 2023) on the reference's Euler-Maruyama predictor:
 * BASELINE config 4. The reference has no sampling-time guidance (its "Posterior"
 * estimator learns the likelihood score with PosteriorLoss, losses.py:293-386); this is the build's
 * definition, computing on the fly the quantity PosteriorLoss.likelihood_target trains towards. Per step,
 * tau = T - t_i:
 *   s, J = prior(x, tau) and ds/dx        (prior = the PosteriorDiffusionEstimator's MLP2 prior score net)
 *   x0_hat = (x + var(tau) s) / mean_weight(tau)                          (Tweedie, losses.py:380)
 *   G = dL(x0_hat(x))/dx = (I + var J^T) (dL/dx0_hat) / mean_weight
 *   x <- x + delta (g^2 s + beta x / 2) + sqrt(delta) g xi  -  lambda G
 *   mode DMIP_DPS_NLL:  L = the likelihood part of get_log_posterior (noise model `noise`; no boundary
 *                       prior), lambda = zeta delta g^2: the EM step of the score s + zeta grad log p(y|x0_hat)
 *   mode DMIP_DPS_NORM: L = ||y - F(x0_hat)||^2, lambda = zeta / ||y - F(x0_hat)|| (Chung et al. Alg. 1)
 * with F the scatterometry surrogate. One fused launch for all steps, exact f32 arithmetic.
 *   prior   MLP handle (DMIP_INPUT_X_T, xdim 3, hidden layers [256]*3)
 *   fwd     surrogate handle;  noise: required for DMIP_DPS_NLL;  y_dev [n_y][23];  x_out_dev [n_y][n_chains][3]
 * RNG, sharding and the other arguments as dmip_em_sample (no injection). */
typedef enum { DMIP_DPS_NLL = 0, DMIP_DPS_NORM = 1 } dmip_dps_mode;
int dmip_dps_sample(const dmip_mlp* prior, const dmip_surrogate* fwd, const dmip_scat_noise* noise,
                    const dmip_vpsde* sde, const float* y_dev, int n_y, int64_t n_chains, int64_t chain_offset,
                    int num_steps, float mean, float stdv, uint64_t seed, int mode, float zeta, float* x_out_dev,
                    void* stream);

/* dmip_dps_sample with a precision (ABI 7): DMIP_PREC_F32 = dmip_dps_sample (exact f32 MFMA, J by three forward
 * tangents); DMIP_PREC_F32X3 = the same method at the reference's fp32 accuracy on the fp16 matrix rate (every
 * product as the three-term fp16 split of the fp32x3 samplers; J^T by one reverse pass through the prior). fp32x3
 * range: a weight beyond fp16's range is refused (DMIP_ERR_UNSUPPORTED, "fp16 range"); a chain whose input,
 * surrogate activation or reverse-pass value leaves it is reported by dmip_device_status ("fp16 range"), and the
 * Python estimators then resample with DMIP_PREC_F32. Same RNG stream per chain as dmip_dps_sample. */
int dmip_dps_sample_ex(const dmip_mlp* prior, const dmip_surrogate* fwd, const dmip_scat_noise* noise,
                       const dmip_vpsde* sde, const float* y_dev, int n_y, int64_t n_chains, int64_t chain_offset,
                       int num_steps, float mean, float stdv, uint64_t seed, int mode, float zeta, int precision,
                       float* x_out_dev, void* stream);

/* ---- PosteriorLoss training step ------------------------------------------ */
/* Loss value, components and the parameter gradients of PosteriorLoss(forward_model, a, b, lam)(sde, x,
 * y, t) + loss.backward() (losses.py:293-386) as PosteriorDiffusionEstimator.train_epoch drives it
 * (models/diffusion.py:204-229), with the forward diffusion x_t = eps std(t) + mean_weight(t) x in the
 * step (sdes.py:37-49; eps caller-drawn, the reference's randn_like). Exact f32 throughout: the two
 * networks' forward and reverse passes as MFMA GEMMs with fused tanh / derivative epilogues, the
 * likelihood target (I + std^2 J_s^T) J_F^T (v2 + a^2 (v3 - v1)) -- the reference's three VJPs and three
 * vector-Hessian products, which it takes without create_graph (constants for the gradients), combined
 * by linearity -- through the fused surrogate reverse pass, deterministic split-K reductions.
 *   xdim, ydim          3, 23 (the scatterometry surrogate)
 *   n_hidden, widths    hidden layers of both networks (any widths, equal for the two networks)
 *   prior_w/b, lik_w/b  device fp32 parameters (nn.Linear layout, n_hidden + 1 layers) of the
 *                       MLP2 prior (x, t) and the MLP likelihood (x, y, t) networks
 *   fwd, noise, lam     the surrogate handle, its noise model (a, b), the likelihood-loss weight
 *   x, y, t, eps        [batch][3], [batch][23], [batch], [batch][3]
 *   grad_prior / grad_lik   [n_params] each, written in the reference parameter order
 *   loss_out            [3]: loss, PriorLoss, LikelihoodLoss (the reference's returned dict)
 *   target_out          optional [batch][3]: the likelihood target (NULL: not returned) */
int dmip_posterior_loss_grad(int xdim, int ydim, int n_hidden, const int* widths, const float* const* prior_w,
                             const float* const* prior_b, const float* const* lik_w, const float* const* lik_b,
                             const dmip_surrogate* fwd, const dmip_scat_noise* noise, float lam, const dmip_vpsde* sde,
                             const float* x_dev, const float* y_dev, const float* t_dev, const float* eps_dev,
                             int64_t batch, float* grad_prior_dev, float* grad_lik_dev, float* loss_out_dev,
                             float* target_out_dev, void* stream);

/* Test hooks for the parity suite (integer RNG stream, normals, schedule). */
int dmip_rng_words(uint64_t seed, int64_t chain_offset, uint64_t stream_id, int64_t n_chains, int n_words,
                   uint32_t* out_dev, void* stream);
int dmip_rng_normals(uint64_t seed, int64_t chain_offset, uint64_t stream_id, int64_t n_chains, int n_pairs,
                     float* out_dev, void* stream);
/* out[(S+1)][4] = (ts_i, T - ts_i, beta(T - ts_i), sqrt(beta)) exactly as the sampler computes them
 * (models/diffusion.py:34, sdes.py:21-35). */
int dmip_schedule(int num_steps, const dmip_vpsde* sde, float* out_dev, void* stream);

/* ---- DIAGNOSTIC entry point: not part of the drop-in boundary (no reference interface; the package only declares
 * its ctypes signature; scripts/stamps.py calls it). Exported by libdmip.so so the phase stamps need no second library.
 * Diagnostic build of the sampler (same math, internal RNG, chain_offset 0) that also writes per-wave
 * cycle sums of the three step phases [layer 1, hidden layers, output layer + EM update], then the
 * s_memtime and s_memrealtime (100 MHz) spans of the whole step loop, to
 * stamps_dev[(workgroup * waves_per_workgroup + wave) * 5 + k]. Never used on the product path; its
 * run time is not representative (the stamps serialise the phases). */
int dmip_em_sample_stamps(const dmip_mlp* net, const dmip_vpsde* sde, const float* y_dev, int n_y, int ydim,
                          int xdim, int64_t n_chains, int num_steps, uint64_t seed, float* x_out_dev,
                          uint64_t* stamps_dev, void* stream);

const char* dmip_last_error(void);
int dmip_abi_version(void);

/* Synchronise `stream` and report asynchronous kernel failures of its device since the last call:
 * DMIP_OK, or DMIP_ERR_HIP with dmip_last_error() naming the failure (the status is then cleared).
 * Today the only such failure is the balanced sampler's hand-over timeout (a consumer wave gave up
 * waiting for the wave that ran the first part of its tile; those chains are written as NaN).
 * The Python layer calls it after every host-facing sampling call (model(y, ...)). */
int dmip_device_status(void* stream);
/* Non-zero when this build has a kernel for the given sampler (dmip_sampler_mode) and shape in bf16
 * (dmip_sampler_supported) or exact f32 (dmip_sampler_supported_f32: widths 64/128/256/512, 1-3
 * hidden layers, xdim 2 or 3; CDiffE for (xdim, ydim) = (2, 2) and (3, 23)). */
int dmip_sampler_supported(int mode, int width, int n_hidden, int xdim, int ydim);
int dmip_sampler_supported_f32(int mode, int width, int n_hidden, int xdim, int ydim);
/* The same question for any dmip_precision (DMIP_PREC_F32X3: widths 64/128/256/512, 1-3 hidden layers,
 * xdim 2 or 3; CDiffE for (xdim, ydim) = (2, 2), and (3, 23) up to width 256). */
int dmip_sampler_supported_precision(int precision, int mode, int width, int n_hidden, int xdim, int ydim);

#ifdef __cplusplus
}
#endif

#endif /* DMIP_H_ */
