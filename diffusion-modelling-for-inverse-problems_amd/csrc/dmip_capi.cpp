// libdmip.so C-ABI (include/dmip.h): handle management, host-side weight packing into the
// kernels' MFMA fragment layouts, argument validation, stream-ordered launches.
//
// Packing conventions (shared with dmip_kernels.hip):
//   * One 1 KiB fragment block = 64 lanes x 8 bf16, the A operand of one
//     v_mfma_f32_32x32x16_bf16: lane l = i + 32h holds A[row i][k = 8h + j], j = 0..7.
//   * Hidden layer k-order: the B operand is the previous layer's accumulator registers, so
//     element j of lane half h in k-step s is hidden unit kperm(s, h, j) (see below).
//   * r-form activations: kernels carry r = 1/(1+exp(2z)) = (1 - tanh z)/2 after a single tanh,
//     so the next layer uses weights -2W and bias b + sum_k W; after layer 1's double tanh they
//     carry the value itself (t-form: weights W, bias b). Pre-activations of tanh layers are
//     scaled by c = 2 log2(e) (exp2 instead of exp).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/dmip.h"
#include "dmip_internal.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(DMIP_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

constexpr double kC = 2.8853900817779268;  // 2 log2(e)

uint16_t f2bf(float f) {  // round to nearest even (inputs are finite)
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

float bf2f(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

// fp16 images of the hidden and output layers (the engine's v_mfma_f32_32x32x16_f16 operands):
// round to nearest even, subnormals kept, |v| <= 65504 (trained and random-init weights are far inside)
uint16_t f2h(float f) {
  const _Float16 h = (_Float16)f;
  uint16_t u;
  std::memcpy(&u, &h, 2);
  return u;
}

float h2f(uint16_t u) {
  _Float16 h;
  std::memcpy(&h, &u, 2);
  return (float)h;
}

// f32 A-fragment images for v_mfma_f32_16x16x4_f32 (dmip_surrogate.hip): k-step (q, r) of output
// tile o, lane l = i + 16 g, holds M[16 o + i][16 q + 4 g + r]; stored [o][q][lane][r] (one float4
// per lane per q). M(row, col) returns 0 outside the matrix.
template <typename F>
std::vector<char> pack_f32_tiles(int n_tiles, int n_q, F M) {
  std::vector<float> v((size_t)n_tiles * n_q * 64 * 4);
  for (int o = 0; o < n_tiles; ++o)
    for (int q = 0; q < n_q; ++q)
      for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 4; ++r)
          v[(((size_t)o * n_q + q) * 64 + l) * 4 + r] = M(16 * o + (l & 15), 16 * q + 4 * (l >> 4) + r);
  std::vector<char> b(v.size() * 4);
  std::memcpy(b.data(), v.data(), b.size());
  return b;
}

inline int kperm(int s, int h, int j) { return 32 * (s >> 1) + 16 * (s & 1) + 8 * (j >> 2) + 4 * h + (j & 3); }
inline int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }
inline int k1s_for(int n_slots) { return (n_slots + 15) / 16; }

// One device status word per device (kernels report asynchronous failures into it; read and
// cleared by dmip_device_status). Allocated on first use, never freed (4 bytes per device).
std::mutex g_status_mu;
unsigned* g_status[dmip::kMaxDevices] = {};

unsigned* status_word(int dev) {
  if (dev < 0 || dev >= dmip::kMaxDevices) return nullptr;
  std::lock_guard<std::mutex> lk(g_status_mu);
  if (!g_status[dev]) {
    int cur = dev;
    (void)hipGetDevice(&cur);
    if (cur != dev) (void)hipSetDevice(dev);
    unsigned* w = nullptr;
    if (hipMalloc((void**)&w, sizeof(unsigned)) == hipSuccess && hipMemset(w, 0, sizeof(unsigned)) == hipSuccess)
      g_status[dev] = w;
    if (cur != dev) (void)hipSetDevice(cur);
  }
  return g_status[dev];
}

// a pinned host mirror of the status word: dmip_device_status copies the word into it on the stream and synchronises
// once (round 6; before, a stream synchronise and then a blocking 4-byte hipMemcpy: two round trips per read)
unsigned* g_status_host[dmip::kMaxDevices] = {};
unsigned* status_host(int dev) {
  if (dev < 0 || dev >= dmip::kMaxDevices) return nullptr;
  std::lock_guard<std::mutex> lk(g_status_mu);
  if (!g_status_host[dev]) {
    unsigned* h = nullptr;
    if (hipHostMalloc((void**)&h, sizeof(unsigned), hipHostMallocDefault) == hipSuccess) g_status_host[dev] = h;
  }
  return g_status_host[dev];
}

// test hook (not ABI): DMIP_DEBUG_NO_HANDOVER=1 makes the balanced sampler's producers never publish
// their hand-over, with a short spin bound, so the consumer's timeout path runs
int debug_no_handover() {
  const char* e = getenv("DMIP_DEBUG_NO_HANDOVER");
  return e && e[0] == '1' ? 1 : 0;
}

template <typename T>
int upload(T** dst, const std::vector<T>& src) {
  *dst = nullptr;
  if (src.empty()) return DMIP_OK;
  hipError_t e = hipMalloc((void**)dst, src.size() * sizeof(T));
  if (e != hipSuccess) return fail(DMIP_ERR_ALLOC, std::string("hipMalloc: ") + hipGetErrorString(e));
  e = hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_fail(e, "hipMemcpy");
  return DMIP_OK;
}

}  // namespace

namespace dmip {

int resident_slots_impl(const void* fn, int nthreads, hipStream_t st) {
  static std::mutex mu;
  static std::map<std::tuple<const void*, int, int>, int> cache;
  const int dev = stream_device(st);
  const auto key = std::make_tuple(fn, nthreads, dev);
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  int n_cu = 256, per_cu = 1, cur = dev;
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipGetDevice(&cur);
  if (cur != dev) (void)hipSetDevice(dev);  // the occupancy query is for the current device
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, nthreads, 0) != hipSuccess || per_cu < 1) per_cu = 1;
  if (cur != dev) (void)hipSetDevice(cur);
  const int slots = (n_cu > 0 ? n_cu : 256) * per_cu;
  std::lock_guard<std::mutex> lk(mu);
  cache[key] = slots;
  return slots;
}

}  // namespace dmip

struct dmip_mlp {
  int in_dim = 0, out_dim = 0, n_hidden = 0, width = 0, act_mode = 0, layout = 0, xdim = 0;
  int k1s_full = 0;
  char* hidden = nullptr;         // [(L-1)][W/32][W/16] KiB
  char* ao_samp = nullptr;        // [W/16] KiB, output rows duplicated into lanes 32-63
  char* ao_full = nullptr;        // [W/16] KiB, natural output rows
  float* bias_hidden = nullptr;   // [(L-1)][W/32][2][16]
  float* bias_out_samp = nullptr; // [2][16]
  float* bias_out_full = nullptr; // [2][16]
  char* a1_full = nullptr;        // [W/32][k1s_full] KiB (every input column varying)
  char* ring_l1 = nullptr;        // width 512: [layer-1 chunks (split image) | hidden | output] (CDiffE sampler)
  float* w1 = nullptr;            // layer-1 fp32 [W][in_dim] (per-y prep of the sampler's A1)
  float* b1 = nullptr;
  // exact-f32 images of a DPS prior (MLP2 (x, t), x 3, widths [256]*3): dmip_dps_sample
  float* dps_l1 = nullptr;        // [16 tiles][2 k-steps][64]
  char* dps_w2 = nullptr;         // [16][16][64][4]
  char* dps_w3 = nullptr;
  char* dps_w4 = nullptr;         // [1][16][64][4], rows >= 3 zero
  float* dps_bias = nullptr;      // b2 | b3 | b4[16]
  // fp32x3 images of a DPS prior (dmip_dps_x3.hip): the chunk stream, layer 1, the biases; none when a weight is
  // beyond fp16's range (dps_x3_range: that magnitude)
  char* dps_x3_img = nullptr;     // [kDpsX3PriorChunks][32 KiB]
  char* dps_x3_l1 = nullptr;      // [16 tiles][64][8] fp16, scaled by 2 log2 e
  float* dps_x3_bias = nullptr;   // c b1 | init2 | init3 [256] | out init [16]
  double dps_x3_range = 0.0;
  // exact-f32 images (DMIP_PREC_F32, dmip_f32.h): every input column + bias as layer 1
  float* f32_l1 = nullptr;        // [W/16][k1q][64]
  char* f32_stream = nullptr;     // [(L-1) W/16 + f32_ot chunks][W/16][64][4]
  float* f32_bias = nullptr;      // [(L-1)][W] | [16 f32_ot]
  int f32_k1q = 0, f32_ot = 0;
  // fp32-accurate split-fp16 images (DMIP_PREC_F32X3, dmip_x3.h); none when a scaled weight or folded bias
  // is outside fp16's range (x3_range: that magnitude, reported by em_sample_x3)
  double x3_range = 0.0;
  char* x3_l1 = nullptr;          // [W/16][K1Q][64][8] fp16 over (x, t)
  char* x3_l1_full = nullptr;     // the same over every input column (X_Y_T networks: CDiffE)
  char* x3_stream = nullptr;      // hidden chunks | output chunk
  char* x3_stream_l1r = nullptr;  // CDiffE at width 512: layer-1 chunks ([K1Q][W/16 tiles][64][8]) | x3_stream
  float* x3_bias = nullptr;       // [L W + 16]
  // the k-major engine's images (dmip_x3k.h; width 256, 3 hidden layers, xdim <= 4)
  char* x3k_stream = nullptr;     // [2 layers][8 k-steps][16 tiles][hi, lo][64][8] fp16
  char* x3k_out = nullptr;        // [8 k-steps][64][8]: rows 0..xdim-1 W_hi, rows 4..4+xdim-1 W_lo
  // the paired-tile 32x32 engine's images (dmip_x3p.h; same shapes)
  char* x3p_stream = nullptr;     // [16 chunks][32 KiB]
  char* x3p_l1 = nullptr;         // [8 layer-1 tiles][64][8] | [2 hidden layers][8 bias tiles][64][8] fp16
  float* x3p_ow = nullptr;        // f32 output rows [8][2][4][4][4] | init[16]
  ~dmip_mlp() {
    for (void* p : {(void*)ring_l1, (void*)hidden, (void*)ao_samp, (void*)ao_full, (void*)bias_hidden, (void*)bias_out_samp,
                    (void*)bias_out_full, (void*)a1_full, (void*)w1, (void*)b1, (void*)dps_l1, (void*)dps_w2,
                    (void*)dps_w3, (void*)dps_w4, (void*)dps_bias, (void*)f32_l1, (void*)f32_stream,
                    (void*)f32_bias, (void*)x3_l1, (void*)x3_l1_full, (void*)x3_stream, (void*)x3_stream_l1r,
                    (void*)x3_bias,
                    (void*)x3k_stream, (void*)x3k_out, (void*)x3p_stream, (void*)x3p_l1, (void*)x3p_ow,
                    (void*)dps_x3_img, (void*)dps_x3_l1, (void*)dps_x3_bias})
      if (p) (void)hipFree(p);
  }
};

namespace {

// exact-f32 images of a network (dmip_f32.h FEngine): layer 1 over every input column then the bias
// column; the W x W layers and the output layer as 16-row chunks in stream order; the biases.
int pack_f32_net(dmip_mlp* net, const float* const* weights, const float* const* biases) {
  const int W = net->width, L = net->n_hidden, IN = net->in_dim, OUT = net->out_dim, ST = W / 16;
  const int K1Q = (IN + 1 + 3) / 4, OT = (OUT + 15) / 16;
  net->f32_k1q = K1Q;
  net->f32_ot = OT;
  std::vector<float> l1((size_t)ST * K1Q * 64);
  for (int o = 0; o < ST; ++o)
    for (int s = 0; s < K1Q; ++s)
      for (int l = 0; l < 64; ++l) {
        const int u = 16 * o + (l & 15), c = 4 * s + (l >> 4);
        l1[((size_t)o * K1Q + s) * 64 + l] = c < IN ? weights[0][(size_t)u * IN + c] : (c == IN ? biases[0][u] : 0.0f);
      }
  std::vector<char> stream;
  for (int li = 1; li < L; ++li) {
    const float* Wl = weights[li];
    std::vector<char> img = pack_f32_tiles(ST, ST, [Wl, W](int r, int c) { return Wl[(size_t)r * W + c]; });
    stream.insert(stream.end(), img.begin(), img.end());
  }
  const float* Wo = weights[L];
  std::vector<char> oimg =
      pack_f32_tiles(OT, ST, [Wo, W, OUT](int r, int c) { return r < OUT ? Wo[(size_t)r * W + c] : 0.0f; });
  stream.insert(stream.end(), oimg.begin(), oimg.end());
  std::vector<float> bias((size_t)(L - 1) * W + 16 * OT, 0.0f);
  for (int li = 1; li < L; ++li)
    for (int k = 0; k < W; ++k) bias[(size_t)(li - 1) * W + k] = biases[li][k];
  for (int k = 0; k < OUT; ++k) bias[(size_t)(L - 1) * W + k] = biases[L][k];
  int rc = DMIP_OK;
  if ((rc = upload(&net->f32_l1, l1)) || (rc = upload(&net->f32_stream, stream)) || (rc = upload(&net->f32_bias, bias)))
    return rc;
  return DMIP_OK;
}

dmip::F32Net f32_net(const dmip_mlp* n) { return dmip::F32Net{n->f32_l1, n->f32_stream, n->f32_bias}; }

// the activation chain's code in the exact-f32 kernels (dmip_f32.h act_f32): 0 tanh, 1 SiLU. Only the exact-f32
// forward and the exact-f32 CDE sampler compile the SiLU chain; every other kernel computes tanh.
int f32_act(const dmip_mlp* n) { return n->act_mode == DMIP_ACT_SILU_TWICE_FIRST ? 1 : 0; }

int act_refused(const char* what) {
  return fail(DMIP_ERR_UNSUPPORTED, std::string(what) +
                                        ": the SiLU chain is compiled for the exact-f32 forward and the exact-f32 "
                                        "CDE sampler only (DMIP_PREC_F32)");
}

// ---- fp32-accurate split-fp16 images (DMIP_PREC_F32X3, dmip_x3.h). A 16x16x32 f16 fragment block:
// lane l = i + 16 g holds A[row i][k-slot 8 g + m], m = 0..7. Hidden-layer k-slots follow the previous
// layer's accumulator tiles: slot (q, g, m) is unit kperm16(q, g, m).
inline int kperm16(int q, int g, int m) { return 32 * q + 16 * (m >> 2) + 4 * g + (m & 3); }
inline int x3_k1q(int nv) { return (3 * nv + 31) / 32; }

// v = hi + lo in fp16 (hi = fp16(v), lo = fp16(v - hi))
void split_h(double v, uint16_t& hi, uint16_t& lo) {
  hi = f2h((float)v);
  lo = f2h((float)(v - (double)h2f(hi)));
}

#ifdef DMIP_WITH_X3P
// 32x32x16 fragments (dmip_x3p.h): lane l = i + 32 h holds A[row i][k-slot 8 h + j]; k-step s of a hidden layer
// covers the previous layer's accumulator registers 8 (s & 1) .. + 7 of its output tile s >> 1
inline int kperm32(int s, int h, int j) { return 32 * (s >> 1) + 16 * (s & 1) + 8 * (j >> 2) + 4 * h + (j & 3); }

// the paired-tile engine's images of a [256]*3 CDE (dmip_x3p.h): the same hi / lo split and folded scales as
// pack_x3_layer / pack_x3_l1 in the 32x32x16 fragment layout; hidden layer 1's bias (`init1`, already folded)
// and hidden layer 2's (`init1`, `init2`: the folded inits of pack_x3_layer) as three-part fp16 A fragments per
// output tile; the output layer in f32 (r-form fold: A = -2 W, init = b + sum_k W, in double)
int pack_x3p(dmip_mlp* net, const float* const* weights, const float* const* biases, const float* init1,
             const float* init2) {
  const int W = net->width, IN = net->in_dim, D = net->xdim, OT = W / 32, KS = W / 16;
  std::vector<uint16_t> l1((size_t)3 * OT * 512, 0);
  std::vector<int> cols;
  for (int k = 0; k < D; ++k) cols.push_back(k);
  cols.push_back(IN - 1);
  const int NV = (int)cols.size();
  for (int o = 0; o < OT; ++o)
    for (int l = 0; l < 64; ++l) {
      const int i = l & 31, h = l >> 5;
      for (int j = 0; j < 8; ++j) {
        const int sl = 8 * h + j, n = sl / 3, pt = sl % 3;
        if (n >= NV) continue;
        uint16_t hi, lo;
        split_h(kC * (double)weights[0][(size_t)(32 * o + i) * IN + cols[n]], hi, lo);
        l1[((size_t)o * 64 + l) * 8 + j] = pt < 2 ? hi : lo;
      }
      for (int li = 1; li <= 2 && h == 0; ++li) {  // bias = hi + mid + lo in k-slots 0..2 (against ones)
        const double v = (double)(li == 1 ? init1 : init2)[32 * o + i];
        const uint16_t a = f2h((float)v);
        const double r1 = v - (double)h2f(a);
        const uint16_t b = f2h((float)r1);
        const uint16_t c = f2h((float)(r1 - (double)h2f(b)));
        uint16_t* dst = &l1[((size_t)(li * OT + o) * 64 + l) * 8];
        dst[0] = a, dst[1] = b, dst[2] = c;
      }
    }
  std::vector<char> stream;
  std::vector<uint16_t> hi((size_t)W * W), lo((size_t)W * W), img((size_t)OT * KS * 1024);
  for (int li = 1; li <= 2; ++li) {
    for (int r = 0; r < W; ++r)
      for (int k = 0; k < W; ++k)
        split_h(-2.0 * kC * (double)weights[li][(size_t)r * W + k], hi[(size_t)r * W + k], lo[(size_t)r * W + k]);
    size_t at = 0;
    // hidden layer 1 k-major: chunk q, output tile o, k-step half e; hidden layer 2 output-major: chunk c, k-step s
    for (int a = 0; a < OT; ++a)
      for (int b = 0; b < KS; ++b)
        for (int pt = 0; pt < 2; ++pt)
          for (int l = 0; l < 64; ++l)
            for (int j = 0; j < 8; ++j) {
              const int row = li == 1 ? 32 * (b >> 1) + (l & 31) : 32 * a + (l & 31);
              const int s = li == 1 ? 2 * a + (b & 1) : b;
              const size_t src = (size_t)row * W + kperm32(s, l >> 5, j);
              img[at++] = pt == 0 ? hi[src] : lo[src];
            }
    const char* p = (const char*)img.data();
    stream.insert(stream.end(), p, p + img.size() * 2);
  }
  std::vector<float> ow((size_t)OT * 2 * 64 + 16, 0.0f);
  for (int c = 0; c < OT; ++c)
    for (int h = 0; h < 2; ++h)
      for (int k = 0; k < D && k < 4; ++k)
        for (int part = 0; part < 4; ++part)
          for (int m = 0; m < 4; ++m)
            ow[(((size_t)c * 2 + h) * 4 + k) * 16 + part * 4 + m] =
                (float)(-2.0 * (double)weights[3][(size_t)k * W + 32 * c + 8 * part + 4 * h + m]);
  for (int k = 0; k < D && k < 4; ++k) {
    double acc = (double)biases[3][k];
    for (int u = 0; u < W; ++u) acc += (double)weights[3][(size_t)k * W + u];
    ow[(size_t)OT * 2 * 64 + k] = (float)acc;
  }
  std::vector<char> l1b(l1.size() * 2);
  std::memcpy(l1b.data(), l1.data(), l1b.size());
  int rc = DMIP_OK;
  if ((rc = upload(&net->x3p_stream, stream)) || (rc = upload(&net->x3p_l1, l1b)) || (rc = upload(&net->x3p_ow, ow)))
    return rc;
  return DMIP_OK;
}

#endif  // DMIP_WITH_X3P

// [n_tiles][KQ][hi, lo][64][8] fp16 split of A[r][c] = get(r, c): lane i + 16 g of tile o holds A[16 o + i][kperm16(q,
// g, m)], m = 0..7 -- pack_x3_layer's layout without its r-form fold (the DPS engine's plain and transposed layers).
// *maxabs: the largest |A| (the split needs it inside fp16's range)
template <typename Get>
std::vector<uint16_t> pack_x3_plain(int n_tiles, int KQ, Get get, double* maxabs) {
  std::vector<uint16_t> img((size_t)n_tiles * KQ * 2 * 512, 0);
  for (int o = 0; o < n_tiles; ++o)
    for (int q = 0; q < KQ; ++q)
      for (int l = 0; l < 64; ++l)
        for (int m = 0; m < 8; ++m) {
          const double v = (double)get(16 * o + (l & 15), kperm16(q, l >> 4, m));
          *maxabs = std::max(*maxabs, std::fabs(v));
          uint16_t hi, lo;
          split_h(v, hi, lo);
          img[((((size_t)o * KQ + q) * 2 + 0) * 64 + l) * 8 + m] = hi;
          img[((((size_t)o * KQ + q) * 2 + 1) * 64 + l) * 8 + m] = lo;
        }
  return img;
}

// append an image to a chunk stream, zero-padded to whole 32 KiB chunks
void append_chunks(std::vector<char>& out, const std::vector<uint16_t>& img) {
  const size_t bytes = img.size() * 2, padded = (bytes + dmip::kDpsX3Chunk - 1) / dmip::kDpsX3Chunk * dmip::kDpsX3Chunk;
  const size_t at = out.size();
  out.resize(at + padded, 0);
  std::memcpy(out.data() + at, img.data(), bytes);
}

// layer-1 image over the input columns `cols` (scaled by c): input n at k-slots 3n, 3n+1, 3n+2 with
// A = [W_hi, W_hi, W_lo] (the kernel's B = [v_hi, v_lo, v_hi])
std::vector<uint16_t> pack_x3_l1(const float* W1, int W, int in_dim, const std::vector<int>& cols, double scale = kC) {
  const int NV = (int)cols.size(), K1Q = x3_k1q(NV), ST = W / 16;
  std::vector<uint16_t> img((size_t)ST * K1Q * 512, 0);
  for (int o = 0; o < ST; ++o)
    for (int q = 0; q < K1Q; ++q)
      for (int l = 0; l < 64; ++l)
        for (int m = 0; m < 8; ++m) {
          const int i = l & 15, g = l >> 4, s = 32 * q + 8 * g + m, n = s / 3, p = s % 3;
          if (n >= NV) continue;
          uint16_t hi, lo;
          split_h(scale * (double)W1[(size_t)(16 * o + i) * in_dim + cols[n]], hi, lo);
          img[(((size_t)o * K1Q + q) * 64 + l) * 8 + m] = p < 2 ? hi : lo;
        }
  return img;
}

// [n_tiles][KQ][2][64][8] image of an r-form-input layer: A = scale * (-2 W), init = scale b - 0.5 sum_k A
// (with A = hi + lo as the kernel applies it); rows >= n_rows zero
void pack_x3_layer(const float* Wl, const float* bl, int n_rows, int W, int n_tiles, double scale,
                   std::vector<uint16_t>& img, float* init) {
  const int KQ = W / 32;
  img.assign((size_t)n_tiles * KQ * 2 * 512, 0);
  std::vector<uint16_t> hi((size_t)n_rows * W), lo((size_t)n_rows * W);
  for (int r = 0; r < n_rows; ++r) {
    double acc = 0.0;
    for (int k = 0; k < W; ++k) {
      split_h(-2.0 * scale * (double)Wl[(size_t)r * W + k], hi[(size_t)r * W + k], lo[(size_t)r * W + k]);
      acc += (double)h2f(hi[(size_t)r * W + k]) + (double)h2f(lo[(size_t)r * W + k]);
    }
    init[r] = (float)(scale * (double)bl[r] - 0.5 * acc);
  }
  for (int o = 0; o < n_tiles; ++o)
    for (int q = 0; q < KQ; ++q)
      for (int p = 0; p < 2; ++p)
        for (int l = 0; l < 64; ++l)
          for (int m = 0; m < 8; ++m) {
            const int row = 16 * o + (l & 15);
            if (row >= n_rows) continue;
            const size_t src = (size_t)row * W + kperm16(q, l >> 4, m);
            img[((((size_t)o * KQ + q) * 2 + p) * 64 + l) * 8 + m] = p == 0 ? hi[src] : lo[src];
          }
}

// the fp32x3 DPS engine's prior images (dmip_dps_x3.hip): layer 1 over (x, t) scaled by 2 log2 e; the forward chunks
// P2 | P3 (pack_x3_layer: r-form folds) | Pout (folded, scale 1); the reverse chunks P4^T (one k-step: the 3 output
// rows) | P3^T | P2^T (plain transposes) | P1^T (W1's x columns); biases c b1 | init2 | init3 | out init
int pack_dps_x3_prior(dmip_mlp* net, const float* const* weights, const float* const* biases) {
  const int W = 256;
  const float *W1 = weights[0], *W2 = weights[1], *W3 = weights[2], *W4 = weights[3];
  double mx = 0.0;
  std::vector<float> bias((size_t)3 * W + 16, 0.0f);
  for (int u = 0; u < W; ++u) bias[u] = (float)(kC * (double)biases[0][u]);
  std::vector<char> chunks;
  std::vector<uint16_t> img;
  pack_x3_layer(W2, biases[1], W, W, 16, kC, img, bias.data() + W);
  for (uint16_t h : img) mx = std::max(mx, std::fabs((double)h2f(h)));
  append_chunks(chunks, img);
  pack_x3_layer(W3, biases[2], W, W, 16, kC, img, bias.data() + 2 * W);
  for (uint16_t h : img) mx = std::max(mx, std::fabs((double)h2f(h)));
  append_chunks(chunks, img);
  pack_x3_layer(W4, biases[3], 3, W, 1, 1.0, img, bias.data() + 3 * W);
  for (uint16_t h : img) mx = std::max(mx, std::fabs((double)h2f(h)));
  append_chunks(chunks, img);
  append_chunks(chunks, pack_x3_plain(16, 1, [&](int r, int c) { return c < 3 ? W4[(size_t)c * W + r] : 0.0f; }, &mx));
  append_chunks(chunks, pack_x3_plain(16, 8, [&](int r, int c) { return W3[(size_t)c * W + r]; }, &mx));
  append_chunks(chunks, pack_x3_plain(16, 8, [&](int r, int c) { return W2[(size_t)c * W + r]; }, &mx));
  append_chunks(chunks, pack_x3_plain(1, 8, [&](int r, int c) { return r < 3 ? W1[(size_t)c * 4 + r] : 0.0f; }, &mx));
  for (size_t i = 0; i < (size_t)W * 4; ++i) mx = std::max(mx, kC * std::fabs((double)W1[i]));
  if (!(mx <= 65504.0) || chunks.size() != (size_t)dmip::kDpsX3PriorChunks * dmip::kDpsX3Chunk) {
    net->dps_x3_range = std::isfinite(mx) ? mx : 1e300;
    return DMIP_OK;  // no fp32x3 DPS for this prior (fp16 range)
  }
  const std::vector<uint16_t> l1 = pack_x3_l1(W1, W, 4, {0, 1, 2, 3});
  std::vector<char> l1b(l1.size() * 2);
  std::memcpy(l1b.data(), l1.data(), l1b.size());
  int rc = DMIP_OK;
  if ((rc = upload(&net->dps_x3_img, chunks)) || (rc = upload(&net->dps_x3_l1, l1b)) ||
      (rc = upload(&net->dps_x3_bias, bias)))
    return rc;
  return DMIP_OK;
}

// largest magnitude the fp32x3 images would hold in fp16: layer 1 scaled by 2 log2(e), the hidden layers by
// -2 * 2 log2(e), the output rows by -2 (r-form folds). The folded hidden biases stay f32 (x3_bias) in the
// product engines, so they do not limit them (only the A/B paired engine stores them in fp16: x3p_bias_range)
double x3_max_scaled(const dmip_mlp* net, const float* const* weights) {
  const int W = net->width, L = net->n_hidden, IN = net->in_dim, OUT = net->out_dim;
  double m = 0.0;
  for (size_t i = 0; i < (size_t)W * IN; ++i) m = std::max(m, kC * std::fabs((double)weights[0][i]));
  for (int li = 1; li < L; ++li)
    for (size_t i = 0; i < (size_t)W * W; ++i) m = std::max(m, 2.0 * kC * std::fabs((double)weights[li][i]));
  for (size_t i = 0; i < (size_t)std::min(OUT, 16) * W; ++i) m = std::max(m, 2.0 * std::fabs((double)weights[L][i]));
  return m;
}

#ifdef DMIP_WITH_X3P
// the paired engine's fp16 folded hidden biases kC (b + sum_k W) (pack_x3p): their largest magnitude
double x3p_bias_range(const dmip_mlp* net, const float* const* weights, const float* const* biases) {
  const int W = net->width, L = net->n_hidden;
  double m = 0.0;
  for (int li = 1; li < L; ++li)
    for (int r = 0; r < W; ++r) {
      double acc = (double)biases[li][r];
      for (int k = 0; k < W; ++k) acc += (double)weights[li][(size_t)r * W + k];
      m = std::max(m, kC * std::fabs(acc));
    }
  return m;
}
#endif

int pack_x3_net(dmip_mlp* net, const float* const* weights, const float* const* biases) {
  const int W = net->width, L = net->n_hidden, IN = net->in_dim, OUT = net->out_dim, ST = W / 16;
  const int chunk = dmip::x3_chunk_bytes(W);
  if (chunk == 0) return DMIP_OK;  // no x3 kernels at this width
  const double mx = x3_max_scaled(net, weights);
  if (!(mx <= 65504.0)) {  // beyond fp16 (or not finite): no split images; fp32x3 requests are refused
    net->x3_range = std::isfinite(mx) ? mx : 1e300;
    return DMIP_OK;
  }
  std::vector<int> xt;
  for (int k = 0; k < net->xdim; ++k) xt.push_back(k);
  xt.push_back(IN - 1);
  std::vector<int> full;
  for (int k = 0; k < IN; ++k) full.push_back(k);
  const std::vector<uint16_t> l1 = pack_x3_l1(weights[0], W, IN, xt);
  std::vector<uint16_t> l1f;
  if (net->layout == DMIP_INPUT_X_Y_T) l1f = pack_x3_l1(weights[0], W, IN, full);
  std::vector<float> bias((size_t)L * W + 16, 0.0f);
  for (int u = 0; u < W; ++u) bias[u] = (float)(kC * (double)biases[0][u]);
  std::vector<char> stream;
  std::vector<uint16_t> img;
  // k-major engine (dmip_x3k.h): the same hi / lo fragments, a layer's chunk q = k-step q of all its
  // tiles ([o][q][p] -> [q][o][p])
  const bool kmajor = W == 256 && L == 3 && net->xdim >= 1 && net->xdim <= 4;
  const int KQ = W / 32;
  std::vector<char> kstream;
  for (int li = 1; li < L; ++li) {
    pack_x3_layer(weights[li], biases[li], W, W, ST, kC, img, bias.data() + (size_t)li * W);
    const char* b = (const char*)img.data();
    stream.insert(stream.end(), b, b + img.size() * 2);
    if (kmajor && li == 1)
      for (int q = 0; q < KQ; ++q)
        for (int o = 0; o < ST; ++o) {
          const char* f = b + (((size_t)o * KQ + q) * 2) * 1024;
          kstream.insert(kstream.end(), f, f + 2048);
        }
    if (kmajor && li == 2)  // two output halves, each k-major: chunk (h, q2) = k-steps 2 q2, 2 q2 + 1 of tiles 8h..8h+7
      for (int h = 0; h < 2; ++h)
        for (int q2 = 0; q2 < KQ / 2; ++q2)
          for (int kk = 0; kk < 2; ++kk)
            for (int o = 8 * h; o < 8 * h + 8; ++o) {
              const char* f = b + (((size_t)o * KQ + 2 * q2 + kk) * 2) * 1024;
              kstream.insert(kstream.end(), f, f + 2048);
            }
  }
  const int orows = OUT < 16 ? OUT : 16;  // the samplers read output rows 0..15 (the x rows)
  pack_x3_layer(weights[L], biases[L], orows, W, 1, 1.0, img, bias.data() + (size_t)L * W);
  std::vector<uint16_t> kout;
  if (kmajor) {  // one fragment per k-step: rows 0..D-1 the hi parts, rows 4..4+D-1 the lo parts
    const int D = net->xdim;
    kout.assign((size_t)KQ * 512, 0);
    for (int q = 0; q < KQ; ++q)
      for (int l = 0; l < 64; ++l) {
        const int i = l & 15, gg = l >> 4;
        int row = -1, part = 0;
        if (i < D) row = i, part = 0;
        else if (i >= 4 && i < 4 + D) row = i - 4, part = 1;
        if (row < 0) continue;
        for (int m = 0; m < 8; ++m)
          kout[((size_t)q * 64 + l) * 8 + m] = img[(((size_t)q * 2 + part) * 64 + row + 16 * gg) * 8 + m];
      }
  }
  std::vector<char> ochunk((size_t)chunk, 0);
  std::memcpy(ochunk.data(), img.data(), img.size() * 2);
  stream.insert(stream.end(), ochunk.begin(), ochunk.end());
  std::vector<char> l1b(l1.size() * 2), l1fb(l1f.size() * 2);
  std::memcpy(l1b.data(), l1.data(), l1b.size());
  if (!l1f.empty()) std::memcpy(l1fb.data(), l1f.data(), l1fb.size());
  int rc = DMIP_OK;
  if ((rc = upload(&net->x3_l1, l1b)) || (rc = upload(&net->x3_l1_full, l1fb)) || (rc = upload(&net->x3_stream, stream)) ||
      (rc = upload(&net->x3_bias, bias)))
    return rc;
  const int k1q_full = x3_k1q(IN);
  if (!l1f.empty() && ST * 1024 == chunk && ST * k1q_full * 1024 > 48 * 1024) {
    // the sampler streams this layer 1 through the ring (dmip_x3.h L1R): chunk q = k-step q of every tile
    std::vector<char> s1((size_t)k1q_full * chunk);
    for (int q = 0; q < k1q_full; ++q)
      for (int o = 0; o < ST; ++o)
        std::memcpy(s1.data() + ((size_t)q * ST + o) * 1024, l1fb.data() + ((size_t)o * k1q_full + q) * 1024, 1024);
    s1.insert(s1.end(), stream.begin(), stream.end());
    if ((rc = upload(&net->x3_stream_l1r, s1))) return rc;
  }
  if (kmajor) {
    std::vector<char> koutb(kout.size() * 2);
    std::memcpy(koutb.data(), kout.data(), koutb.size());
    if ((rc = upload(&net->x3k_stream, kstream)) || (rc = upload(&net->x3k_out, koutb))) return rc;
#ifdef DMIP_WITH_X3P
    if (net->xdim <= 4 && x3p_bias_range(net, weights, biases) <= 65504.0 &&
        (rc = pack_x3p(net, weights, biases, bias.data() + W, bias.data() + 2 * W)))
      return rc;
#endif
  }
  return DMIP_OK;
}

}  // namespace

extern "C" {

const char* dmip_last_error(void) { return g_err.c_str(); }

int dmip_device_status(void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int dev = dmip::stream_device(st);
  unsigned* w = status_word(dev);
  if (!w) return fail(DMIP_ERR_ALLOC, "device status word");
  unsigned* h = status_host(dev);
  hipError_t e = hipSuccess;
  unsigned v = 0;
  if (h) {  // the word's copy ordered after the stream's work, then one synchronise
    if ((e = hipMemcpyAsync(h, w, sizeof(unsigned), hipMemcpyDeviceToHost, st)) != hipSuccess)
      return hip_fail(e, "hipMemcpyAsync");
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    v = *(volatile unsigned*)h;
  } else {
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    if ((e = hipMemcpy(&v, w, sizeof(unsigned), hipMemcpyDeviceToHost)) != hipSuccess) return hip_fail(e, "hipMemcpy");
  }
  if (v == 0) return DMIP_OK;
  (void)hipMemset(w, 0, sizeof(unsigned));
  if (v == dmip::kErrHandover)
    return fail(DMIP_ERR_HIP, "sampler: a split tile's hand-over never arrived (workgroups of the balanced schedule "
                              "were not co-resident); the affected chains were written as NaN");
  if (v == dmip::kErrRange)
    return fail(DMIP_ERR_HIP, "fp32x3 sampler: a chain's layer-1 input left the fp16 range of the split arithmetic "
                              "(|x| > 65504); those chains are not fp32-accurate (use DMIP_PREC_F32)");
  return fail(DMIP_ERR_HIP, "device status " + std::to_string(v));
}

int dmip_abi_version(void) { return DMIP_ABI_VERSION; }

#ifdef DMIP_WITH_X3P
// not ABI: present only in the A/B library (make diag), which also holds the paired-tile engine (DMIP_X3P=1)
int dmip_x3p_available(void) { return 1; }
#endif

int dmip_sampler_supported(int mode, int width, int n_hidden, int xdim, int ydim) {
  return dmip::sampler_shape_supported(mode, width, n_hidden, xdim, ydim) ? 1 : 0;
}

int dmip_sampler_supported_f32(int mode, int width, int n_hidden, int xdim, int ydim) {
  return dmip::f32_sampler_supported(mode, width, n_hidden, xdim, ydim) ? 1 : 0;
}

int dmip_sampler_supported_precision(int precision, int mode, int width, int n_hidden, int xdim, int ydim) {
  switch (precision) {
    case DMIP_PREC_FP16: return dmip::sampler_shape_supported(mode, width, n_hidden, xdim, ydim) ? 1 : 0;
    case DMIP_PREC_F32: return dmip::f32_sampler_supported(mode, width, n_hidden, xdim, ydim) ? 1 : 0;
    case DMIP_PREC_F32X3: return dmip::x3_sampler_supported(mode, width, n_hidden, xdim, ydim) ? 1 : 0;
    default: return 0;
  }
}

int dmip_mlp_create(int in_dim, int out_dim, int n_hidden, const int* widths, int act_mode, int input_layout,
                    int xdim, const float* const* weights, const float* const* biases, dmip_mlp** out) {
  if (!out || !widths || !weights || !biases) return fail(DMIP_ERR_INVALID, "null argument");
  *out = nullptr;
  if (n_hidden < 1) return fail(DMIP_ERR_INVALID, "n_hidden must be >= 1");
  const int W = widths[0];
  for (int i = 1; i < n_hidden; ++i)
    if (widths[i] != W) return fail(DMIP_ERR_UNSUPPORTED, "hidden widths must all be equal");
  if (W % 32 != 0 || W < 32) return fail(DMIP_ERR_UNSUPPORTED, "hidden width must be a multiple of 32");
  if (out_dim < 1 || out_dim > 32) return fail(DMIP_ERR_UNSUPPORTED, "out_dim must be in [1, 32]");
  if (act_mode != DMIP_ACT_TANH_TWICE_FIRST && act_mode != DMIP_ACT_SILU_TWICE_FIRST)
    return fail(DMIP_ERR_UNSUPPORTED, "compiled activation chains: DMIP_ACT_TANH_TWICE_FIRST, DMIP_ACT_SILU_TWICE_FIRST");
  if (input_layout != DMIP_INPUT_X_Y_T && input_layout != DMIP_INPUT_X_T)
    return fail(DMIP_ERR_INVALID, "unknown input layout");
  if (xdim < 1 || xdim + 1 > in_dim) return fail(DMIP_ERR_INVALID, "xdim inconsistent with in_dim");
  if (input_layout == DMIP_INPUT_X_T && in_dim != xdim + 1)
    return fail(DMIP_ERR_INVALID, "X_T layout needs in_dim == xdim + 1");
  for (int i = 0; i <= n_hidden; ++i)
    if (!weights[i] || !biases[i]) return fail(DMIP_ERR_INVALID, "null layer pointer");

  dmip_mlp* net = new (std::nothrow) dmip_mlp;
  if (!net) return fail(DMIP_ERR_ALLOC, "host allocation");
  net->in_dim = in_dim;
  net->out_dim = out_dim;
  net->n_hidden = n_hidden;
  net->width = W;
  net->act_mode = act_mode;
  net->layout = input_layout;
  net->xdim = xdim;
  const int T = W / 32, KS = W / 16, L = n_hidden;

  // ---- hidden W x W layers (fp16 images). Input in r-form (after a single tanh): A = fp16(-2c W),
  // init = c b - 0.5 sum_k A. Input in t-form (the first W x W layer: layer 1's double tanh is
  // emitted as the value itself, dmip_device.h act_t_twice_pk_f16): A = fp16(c W), init = c b.
  std::vector<uint16_t> hid((size_t)(L - 1) * T * KS * 512);
  std::vector<float> bh((size_t)(L - 1) * T * 32);
  for (int li = 0; li < L - 1; ++li) {
    const float* Wl = weights[li + 1];
    const float* bl = biases[li + 1];
    const bool t_form = li == 0;
    std::vector<uint16_t> A((size_t)W * W);
    std::vector<float> init(W);
    for (int r = 0; r < W; ++r) {
      double acc = 0.0;
      for (int k = 0; k < W; ++k) {
        const float v = (float)((t_form ? 1.0 : -2.0) * kC * (double)Wl[(size_t)r * W + k]);
        const uint16_t a = f2h(v);
        A[(size_t)r * W + k] = a;
        acc += (double)h2f(a);
      }
      init[r] = (float)(kC * (double)bl[r] - (t_form ? 0.0 : 0.5 * acc));
    }
    for (int rt = 0; rt < T; ++rt)
      for (int s = 0; s < KS; ++s)
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 8; ++j) {
            const int i = l & 31, h = l >> 5;
            hid[(((size_t)(li * T + rt) * KS + s) * 64 + l) * 8 + j] = A[(size_t)(rt * 32 + i) * W + kperm(s, h, j)];
          }
    for (int rt = 0; rt < T; ++rt)
      for (int h = 0; h < 2; ++h)
        for (int r = 0; r < 16; ++r) bh[((size_t)(li * T + rt) * 2 + h) * 16 + r] = init[rt * 32 + acc_row(r, h)];
  }

  // ---- output layer (fp16 image): A = fp16(-2 W), init = b - 0.5 sum_k A (no tanh scale: raw
  // drift a); t-form input (L == 1: directly after layer 1's double tanh): A = fp16(W), init = b
  const float* Wo = weights[L];
  const float* bo = biases[L];
  const bool out_t_form = L == 1;
  std::vector<uint16_t> Ao((size_t)out_dim * W);
  std::vector<float> init_o(out_dim);
  for (int d = 0; d < out_dim; ++d) {
    double acc = 0.0;
    for (int k = 0; k < W; ++k) {
      const float v = (float)((out_t_form ? 1.0 : -2.0) * (double)Wo[(size_t)d * W + k]);
      const uint16_t a = f2h(v);
      Ao[(size_t)d * W + k] = a;
      acc += (double)h2f(a);
    }
    init_o[d] = (float)((double)bo[d] - (out_t_form ? 0.0 : 0.5 * acc));
  }
  std::vector<uint16_t> ao_s((size_t)KS * 512, 0), ao_f((size_t)KS * 512, 0);
  std::vector<float> bo_s(32, 0.0f), bo_f(32, 0.0f);
  for (int s = 0; s < KS; ++s)
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 8; ++j) {
        const int i = l & 31, h = l >> 5;
        const int ds = i < 4 ? i : (i < 8 ? i - 4 : -1);  // sampler: rows 0-3 duplicated at 4-7
        if (ds >= 0 && ds < out_dim) ao_s[((size_t)s * 64 + l) * 8 + j] = Ao[(size_t)ds * W + kperm(s, h, j)];
        if (i < out_dim) ao_f[((size_t)s * 64 + l) * 8 + j] = Ao[(size_t)i * W + kperm(s, h, j)];
      }
  for (int h = 0; h < 2; ++h)
    for (int r = 0; r < 16; ++r) {
      const int row = acc_row(r, h);
      const int ds = row < 4 ? row : (row < 8 ? row - 4 : -1);
      if (ds >= 0 && ds < out_dim) bo_s[h * 16 + r] = init_o[ds];
      if (row < out_dim) bo_f[h * 16 + r] = init_o[row];
    }

  // ---- layer 1, forward variant: every column varying, split bf16 [hi | hi | lo | b_hi | b_lo]
  const float* W1 = weights[0];
  const float* b1 = biases[0];
  const int IN = in_dim;
  const bool split = dmip::forward_split(W, IN);
  net->k1s_full = split ? k1s_for(3 * IN + 2) : k1s_for(IN + 2);
  auto pack_a1 = [&](bool split, int K1S) {
  std::vector<uint16_t> a1f((size_t)T * K1S * 512, 0);
  for (int jr = 0; jr < W; ++jr) {
    const int rt = jr / 32, i = jr % 32;
    for (int k = 0; k < K1S * 16; ++k) {
      float val = 0.0f;
      auto hilo = [&](double v, bool lo) {
        const float f = (float)v;
        const uint16_t hi = f2bf(f);
        return lo ? bf2f(f2bf(f - bf2f(hi))) : bf2f(hi);
      };
      if (split) {
        if (k < IN) val = hilo(kC * W1[(size_t)jr * IN + k], false);
        else if (k < 2 * IN) val = hilo(kC * W1[(size_t)jr * IN + k - IN], false);
        else if (k < 3 * IN) val = hilo(kC * W1[(size_t)jr * IN + k - 2 * IN], true);
        else if (k == 3 * IN) val = hilo(kC * b1[jr], false);
        else if (k == 3 * IN + 1) val = hilo(kC * b1[jr], true);
      } else {  // [v | 1 | 1] x [W | b_hi | b_lo]
        if (k < IN) val = hilo(kC * W1[(size_t)jr * IN + k], false);
        else if (k == IN) val = hilo(kC * b1[jr], false);
        else if (k == IN + 1) val = hilo(kC * b1[jr], true);
      }
      const int s = k / 16, hh = (k % 16) / 8, jj = k % 8;
      a1f[(((size_t)(rt * K1S + s)) * 64 + i + 32 * hh) * 8 + jj] = f2bf(val);
    }
  }
  return a1f;
  };
  const std::vector<uint16_t> a1f = pack_a1(split, net->k1s_full);

  int rc = DMIP_OK;
  if (input_layout == DMIP_INPUT_X_T && xdim == 3 && in_dim == 4 && out_dim == 3 && L == 3 && W == dmip::kDpsPriorW) {
    // exact-f32 images for the DPS sampler's prior (dmip_surrogate.hip dps_kernel)
    const float *P1 = weights[0], *P2 = weights[1], *P3 = weights[2], *P4 = weights[3];
    std::vector<float> l1((size_t)16 * 2 * 64), pb((size_t)2 * W + 16, 0.0f);
    for (int o = 0; o < 16; ++o)
      for (int l = 0; l < 64; ++l) {
        const int row = 16 * o + (l & 15), g = l >> 4;
        l1[((size_t)o * 2 + 0) * 64 + l] = P1[(size_t)row * 4 + g];
        l1[((size_t)o * 2 + 1) * 64 + l] = g == 0 ? biases[0][row] : 0.0f;
      }
    for (int k = 0; k < W; ++k) pb[k] = biases[1][k], pb[W + k] = biases[2][k];
    for (int k = 0; k < 3; ++k) pb[2 * W + k] = biases[3][k];
    const auto sqm = [W](const float* Wm) { return [Wm, W](int r, int c) { return Wm[(size_t)r * W + c]; }; };
    if ((rc = upload(&net->dps_l1, l1)) || (rc = upload(&net->dps_bias, pb)) ||
        (rc = upload(&net->dps_w2, pack_f32_tiles(16, 16, sqm(P2)))) ||
        (rc = upload(&net->dps_w3, pack_f32_tiles(16, 16, sqm(P3)))) ||
        (rc = upload(&net->dps_w4, pack_f32_tiles(1, 16, [&](int r, int c) { return r < 3 ? P4[(size_t)r * W + c] : 0.0f; }))) ||
        (rc = pack_dps_x3_prior(net, weights, biases))) {
      delete net;
      return rc;
    }
  }
  std::vector<char> hid_b(hid.size() * 2), ao_sb(ao_s.size() * 2), ao_fb(ao_f.size() * 2), a1f_b(a1f.size() * 2);
  std::memcpy(hid_b.data(), hid.data(), hid_b.size());
  std::memcpy(ao_sb.data(), ao_s.data(), ao_sb.size());
  std::memcpy(ao_fb.data(), ao_f.data(), ao_fb.size());
  std::memcpy(a1f_b.data(), a1f.data(), a1f_b.size());
  // the output image also follows the hidden chunks in one buffer: the two-network sampler at width 512
  // streams it through the weight ring as the network's last chunk (dmip_kernels.hip Lay<AOR>)
  hid_b.insert(hid_b.end(), ao_sb.begin(), ao_sb.end());
  // the CDiffE sampler at width 512 streams its split layer 1 (3 in + 2 slots, 6 KiB per row tile at
  // in_dim 27) through the ring as well: [ceil(T / TPC) layer-1 chunks of TPC row tiles | hidden | output]
  // (dmip_kernels.hip Lay<L1R>)
  std::vector<char> ring_b;
  if (W == 512 && input_layout == DMIP_INPUT_X_Y_T) {
    const int k1s = k1s_for(3 * IN + 2), chunk = (W / 16) * 1024, tpc = chunk / (k1s * 1024);
    if (tpc >= 1) {
      const std::vector<uint16_t> a1s = pack_a1(true, k1s);
      const int l1c = (T + tpc - 1) / tpc;
      ring_b.assign((size_t)l1c * chunk, 0);
      for (int rt = 0; rt < T; ++rt)
        std::memcpy(ring_b.data() + (size_t)(rt / tpc) * chunk + (size_t)(rt % tpc) * k1s * 1024,
                    (const char*)a1s.data() + (size_t)rt * k1s * 1024, (size_t)k1s * 1024);
      ring_b.insert(ring_b.end(), hid_b.begin(), hid_b.end());
    }
  }
  std::vector<float> w1v(W1, W1 + (size_t)W * IN), b1v(b1, b1 + W);
  if (!ring_b.empty() && (rc = upload(&net->ring_l1, ring_b))) {
    delete net;
    return rc;
  }
  if ((rc = upload(&net->hidden, hid_b)) || (rc = upload(&net->ao_samp, ao_sb)) || (rc = upload(&net->ao_full, ao_fb)) ||
      (rc = upload(&net->bias_hidden, bh)) || (rc = upload(&net->bias_out_samp, bo_s)) ||
      (rc = upload(&net->bias_out_full, bo_f)) || (rc = upload(&net->a1_full, a1f_b)) ||
      (rc = upload(&net->w1, w1v)) || (rc = upload(&net->b1, b1v)) || (rc = pack_f32_net(net, weights, biases)) ||
      (rc = pack_x3_net(net, weights, biases))) {
    delete net;
    return rc;
  }
  *out = net;
  return DMIP_OK;
}

int dmip_mlp_destroy(dmip_mlp* net) {
  delete net;
  return DMIP_OK;
}

int dmip_mlp_forward(const dmip_mlp* net, const float* x_dev, const float* y_dev, int64_t y_stride,
                     const float* t_dev, int t_stride, int64_t n, float* out_dev, int precision, void* stream) {
  if (!net || !x_dev || !t_dev || !out_dev) return fail(DMIP_ERR_INVALID, "null argument");
  if (precision != DMIP_PREC_FP16 && precision != DMIP_PREC_F32 && precision != DMIP_PREC_F32X3)
    return fail(DMIP_ERR_INVALID, "unknown precision");
  if (n < 0) return fail(DMIP_ERR_INVALID, "n < 0");
  if (n == 0) return DMIP_OK;
  const int ydim = net->layout == DMIP_INPUT_X_Y_T ? net->in_dim - net->xdim - 1 : 0;
  if (ydim > 0 && !y_dev) return fail(DMIP_ERR_INVALID, "y required for an X_Y_T network");
  if (ydim > 0 && y_stride != 0 && y_stride != ydim) return fail(DMIP_ERR_INVALID, "y_stride must be 0 or ydim");
  if (t_stride != 0 && t_stride != 1) return fail(DMIP_ERR_INVALID, "t_stride must be 0 or 1");
  if (precision == DMIP_PREC_F32 || precision == DMIP_PREC_F32X3) {  // F32X3: the exact-f32 forward (fp32 either way)
    dmip::F32ForwardParams q{};
    q.net = f32_net(net);
    q.n_hidden = net->n_hidden;
    q.x = x_dev;
    q.y = y_dev;
    q.t = t_dev;
    q.out = out_dev;
    q.n = n;
    q.y_stride = y_stride;
    q.t_stride = t_stride;
    q.xdim = net->xdim;
    q.ydim = ydim;
    q.out_dim = net->out_dim;
    q.k1q = net->f32_k1q;
    q.act = f32_act(net);
    bool ok = false;
    hipError_t e = dmip::launch_f32_forward(q, net->width, net->f32_ot, (hipStream_t)stream, &ok);
    if (!ok)
      return fail(DMIP_ERR_UNSUPPORTED, "no compiled f32 forward kernel for width " + std::to_string(net->width) +
                                            ", layers " + std::to_string(net->n_hidden) + ", in_dim " +
                                            std::to_string(net->in_dim) + ", out_dim " + std::to_string(net->out_dim));
    if (e != hipSuccess) return hip_fail(e, "mlp_forward (f32) launch");
    return DMIP_OK;
  }
  if (f32_act(net)) return act_refused("mlp_forward at DMIP_PREC_FP16");
  dmip::ForwardParams p{};
  p.hidden = net->hidden;
  p.a1 = net->a1_full;
  p.ao = net->ao_full;
  p.bias_hidden = net->bias_hidden;
  p.bias_out = net->bias_out_full;
  p.x = x_dev;
  p.y = y_dev;
  p.t = t_dev;
  p.out = out_dev;
  p.n = n;
  p.y_stride = y_stride;
  p.t_stride = t_stride;
  p.xdim = net->xdim;
  p.ydim = ydim;
  p.out_dim = net->out_dim;
  bool ok = false;
  hipError_t e = dmip::launch_forward(p, net->width, net->n_hidden, net->in_dim, (hipStream_t)stream, &ok);
  if (!ok) return fail(DMIP_ERR_UNSUPPORTED, "no compiled forward kernel for width " + std::to_string(net->width) +
                                                 ", layers " + std::to_string(net->n_hidden) + ", in_dim " +
                                                 std::to_string(net->in_dim));
  if (e != hipSuccess) return hip_fail(e, "mlp_forward launch");
  return DMIP_OK;
}

struct SampleArgs {
  const dmip_vpsde* sde;
  const float* y_dev;
  int n_y, ydim, xdim;
  int64_t n_chains, chain_offset;
  int num_steps;
  float mean, stdv;
  uint64_t seed;
  int precision;
  const float* noise_dev;
  float* x_out_dev;
  void* stream;
  uint64_t* stamps;
  int n_corr = 0;
  float snr = 0.16f;
  int snap_every = 0;
  float* snap_out_dev = nullptr;
};

static void fill_schedule(const SampleArgs& a, float& T, float& bmin, float& bdiff, float& delta, float& sqrt_delta) {
  T = (float)a.sde->T;
  bmin = (float)a.sde->beta_min;
  bdiff = (float)(a.sde->beta_max - a.sde->beta_min);
  delta = (float)(a.sde->T / (double)a.num_steps);
  sqrt_delta = (float)std::sqrt(a.sde->T / (double)a.num_steps);
}

// exact-f32 samplers (dmip_f32.h): same loop, RNG and sharding as the bf16 kernels; arguments
// already validated by em_sample_impl
static int em_sample_f32(int mode, const dmip_mlp* net0, const dmip_mlp* net1, const SampleArgs& a) {
  const int xdim = a.xdim, ydim = a.ydim;
  if (!dmip::f32_sampler_supported(mode, net0->width, net0->n_hidden, xdim, ydim))
    return fail(DMIP_ERR_UNSUPPORTED, "no compiled f32 sampler (mode " + std::to_string(mode) + ") for width " +
                                          std::to_string(net0->width) + ", layers " + std::to_string(net0->n_hidden) +
                                          ", xdim " + std::to_string(xdim) + ", ydim " + std::to_string(ydim));
  hipStream_t st = (hipStream_t)a.stream;
  dmip::F32SamplerParams p{};
  p.net[0] = f32_net(net0);
  if (net1) p.net[1] = f32_net(net1);
  p.n_hidden = net0->n_hidden;
  float* l1y = nullptr;
  if (mode != DMIP_SAMPLER_CDIFFE) {
    // y is constant per y index: layer 1 over (x, t) with W1_y y + b1 folded into the bias column
    const int k1q = (xdim + 2 + 3) / 4;
    hipError_t e = hipMallocAsync((void**)&l1y, (size_t)a.n_y * (net0->width / 16) * k1q * 64 * sizeof(float), st);
    if (e != hipSuccess) return fail(DMIP_ERR_ALLOC, std::string("hipMallocAsync: ") + hipGetErrorString(e));
    dmip::F32L1PrepParams lp{net0->w1, net0->b1, a.y_dev, l1y, net0->width, net0->in_dim, xdim, ydim, k1q};
    if ((e = dmip::launch_f32_l1_prep(lp, a.n_y, st)) != hipSuccess) {
      (void)hipFreeAsync(l1y, st);
      return hip_fail(e, "f32 layer-1 prep launch");
    }
    p.l1y = l1y;
  }
  p.y_obs = a.y_dev;
  p.n_corr = a.n_corr;
  p.snr = a.snr;
  p.noise = a.noise_dev;
  p.x_out = a.x_out_dev;
  p.snap_out = a.snap_out_dev;
  p.snap_every = a.snap_every;
  p.n_chains = a.n_chains;
  p.chain_offset = a.chain_offset;
  p.num_steps = a.num_steps;
  fill_schedule(a, p.T, p.bmin, p.bdiff, p.delta, p.sqrt_delta);
  p.mean = a.mean;
  p.stdv = a.stdv;
  p.seed = a.seed;
  p.err = status_word(dmip::stream_device(st));
  if (!p.err) {
    if (l1y) (void)hipFreeAsync(l1y, st);
    return fail(DMIP_ERR_ALLOC, "device status word");
  }
  p.debug_flags = debug_no_handover();
  p.spin_limit = p.debug_flags ? (1u << 10) : (1u << 22);
  p.act = f32_act(net0);
  bool ok = false;
  hipError_t e = dmip::launch_f32_sampler(p, mode, net0->width, net0->n_hidden, xdim, ydim, a.n_y, st, &ok);
  if (l1y) (void)hipFreeAsync(l1y, st);
  if (!ok) return fail(DMIP_ERR_UNSUPPORTED, "no compiled f32 sampler");
  if (e != hipSuccess) return hip_fail(e, "f32 sampler launch");
  return DMIP_OK;
}

// DMIP_X3K=0 selects the one-tile-per-wave fp32x3 engine (dmip_x3.h) at the k-major engine's shape too
// (A/B and parity of the two engines; not part of the ABI)
static bool x3k_enabled() {
  const char* e = getenv("DMIP_X3K");
  return !(e && e[0] == '0');
}
#ifdef DMIP_WITH_X3P
// A/B library only (make diag): DMIP_X3P=1 selects the paired-tile 32x32 engine (dmip_x3p.h) instead of the
// 16x16 k-major one (dmip_x3k.h) at its shape. It measured slower (profiles/r4_ab_x3p_vs_x3k.json), so the
// product library libdmip.so does not contain it.
static bool x3p_enabled() {
  const char* e = getenv("DMIP_X3P");
  return e && e[0] == '1';
}
#endif

// fp32-accurate split-fp16 samplers (dmip_x3.h): same loop, RNG and sharding as the other engines;
// arguments already validated by em_sample_impl
static int em_sample_x3(int mode, const dmip_mlp* net0, const dmip_mlp* net1, const SampleArgs& a) {
  const int xdim = a.xdim, ydim = a.ydim;
  for (const dmip_mlp* n : {net0, net1})
    if (n && n->x3_range > 0.0)
      return fail(DMIP_ERR_UNSUPPORTED, "fp32x3: a weight is outside the fp16 range of the split engine (largest "
                                        "scaled |w| " + std::to_string(n->x3_range) + " > 65504); use DMIP_PREC_F32");
  if (!dmip::x3_sampler_supported(mode, net0->width, net0->n_hidden, xdim, ydim) || !net0->x3_stream ||
      (mode == DMIP_SAMPLER_CDIFFE && !net0->x3_l1_full) || (net1 && !net1->x3_stream))
    return fail(DMIP_ERR_UNSUPPORTED, "no compiled f32x3 sampler (mode " + std::to_string(mode) + ") for width " +
                                          std::to_string(net0->width) + ", layers " + std::to_string(net0->n_hidden) +
                                          ", xdim " + std::to_string(xdim) + ", ydim " + std::to_string(ydim));
  hipStream_t st = (hipStream_t)a.stream;
  dmip::X3SamplerParams p{};
  p.net[0] = dmip::X3Net{mode == DMIP_SAMPLER_CDIFFE ? net0->x3_l1_full : net0->x3_l1, net0->x3_stream, net0->x3_bias};
  if (mode == DMIP_SAMPLER_CDIFFE && net0->x3_stream_l1r) p.net[0].stream = net0->x3_stream_l1r;  // L1R layout
  if (net1) p.net[1] = dmip::X3Net{net1->x3_l1, net1->x3_stream, net1->x3_bias};
  p.n_hidden = net0->n_hidden;
  float* bias_y = nullptr;
  if (dmip::x3s_sampler_eligible(mode, net0->width, net0->n_hidden, xdim, a.n_chains, a.n_y)) {
    // the width-64 latency engine forms the per-y bias itself (round 6: one launch and one allocation fewer)
    p.l1w = net0->w1;
    p.l1b = net0->b1;
    p.l1_in = net0->in_dim;
    p.ydim = ydim;
  } else if (mode != DMIP_SAMPLER_CDIFFE) {
    // y is constant per y index: c (b1 + W1_y y) becomes layer 1's per-y bias (f64 prep)
    hipError_t e = hipMallocAsync((void**)&bias_y, (size_t)a.n_y * net0->width * sizeof(float), st);
    if (e != hipSuccess) return fail(DMIP_ERR_ALLOC, std::string("hipMallocAsync: ") + hipGetErrorString(e));
    dmip::X3BiasPrepParams bp{net0->w1, net0->b1, a.y_dev, bias_y, net0->width, net0->in_dim, xdim, ydim};
    if ((e = dmip::launch_x3_bias_prep(bp, a.n_y, st)) != hipSuccess) {
      (void)hipFreeAsync(bias_y, st);
      return hip_fail(e, "x3 bias prep launch");
    }
  }
  p.bias_y = bias_y;
  p.y_obs = a.y_dev;
  p.n_corr = a.n_corr;
  p.snr = a.snr;
  p.noise = a.noise_dev;
  p.x_out = a.x_out_dev;
  p.snap_out = a.snap_out_dev;
  p.snap_every = a.snap_every;
  p.n_chains = a.n_chains;
  p.chain_offset = a.chain_offset;
  p.num_steps = a.num_steps;
  fill_schedule(a, p.T, p.bmin, p.bdiff, p.delta, p.sqrt_delta);
  p.mean = a.mean;
  p.stdv = a.stdv;
  p.seed = a.seed;
  p.err = status_word(dmip::stream_device(st));
  if (!p.err) {
    if (bias_y) (void)hipFreeAsync(bias_y, st);
    return fail(DMIP_ERR_ALLOC, "device status word");
  }
  p.debug_flags = debug_no_handover();
  p.spin_limit = p.debug_flags ? (1u << 10) : (1u << 22);
  bool ok = false;
  hipError_t e;
#ifdef DMIP_WITH_X3P
  if (mode == DMIP_SAMPLER_CDE && net0->x3p_stream && dmip::x3p_sampler_supported(mode, net0->width, net0->n_hidden, xdim) &&
      x3k_enabled() && x3p_enabled()) {
    // the paired-tile 32x32 engine at its shape (dmip_x3p.h; A/B library only)
    p.net[0].pstream = net0->x3p_stream;
    p.net[0].pl1 = net0->x3p_l1;
    p.net[0].pow = net0->x3p_ow;
    e = dmip::launch_x3p_sampler(p, xdim, a.n_y, st, &ok);
  } else
#endif
  if (mode == DMIP_SAMPLER_CDE && net0->x3k_stream &&
             dmip::x3k_sampler_supported(mode, net0->width, net0->n_hidden, xdim) && x3k_enabled()) {
    // the k-major multi-tile engine at its shape (dmip_x3k.h)
    p.net[0].kstream = net0->x3k_stream;
    p.net[0].kout = net0->x3k_out;
    e = dmip::launch_x3k_sampler(p, xdim, a.n_y, st, &ok);
  } else {
    e = dmip::launch_x3_sampler(p, mode, net0->width, net0->n_hidden, xdim, ydim, a.n_y, st, &ok);
  }
  if (bias_y) (void)hipFreeAsync(bias_y, st);
  if (!ok) return fail(DMIP_ERR_UNSUPPORTED, "no compiled f32x3 sampler");
  if (e != hipSuccess) return hip_fail(e, "f32x3 sampler launch");
  return DMIP_OK;
}

// net0: the CDE / CDiffE network or the Posterior likelihood; net1: the Posterior prior (else null)
static int em_sample_impl(int mode, const dmip_mlp* net0, const dmip_mlp* net1, const SampleArgs& a) {
  const int xdim = a.xdim, ydim = a.ydim;
  if (!net0 || !a.sde || !a.y_dev || !a.x_out_dev || (mode == DMIP_SAMPLER_POSTERIOR && !net1))
    return fail(DMIP_ERR_INVALID, "null argument");
  if (a.precision != DMIP_PREC_FP16 && a.precision != DMIP_PREC_F32 && a.precision != DMIP_PREC_F32X3)
    return fail(DMIP_ERR_INVALID, "unknown precision");
  if (a.noise_dev && mode != DMIP_SAMPLER_CDE) return fail(DMIP_ERR_INVALID, "noise injection: CDE sampler only");
  if (net0->layout != DMIP_INPUT_X_Y_T) return fail(DMIP_ERR_INVALID, "sampler needs an x,y,t network");
  const int out_expected = mode == DMIP_SAMPLER_CDIFFE ? xdim + ydim : xdim;
  if (xdim != net0->xdim || net0->out_dim != out_expected)
    return fail(DMIP_ERR_INVALID, "xdim does not match the network");
  if (ydim != net0->in_dim - xdim - 1) return fail(DMIP_ERR_INVALID, "ydim does not match the network");
  if (mode == DMIP_SAMPLER_POSTERIOR) {
    if (net1->layout != DMIP_INPUT_X_T || net1->xdim != xdim || net1->out_dim != xdim)
      return fail(DMIP_ERR_INVALID, "prior must be an x,t network with out_dim == xdim");
    if (net1->width != net0->width || net1->n_hidden != net0->n_hidden)
      return fail(DMIP_ERR_UNSUPPORTED, "prior and likelihood networks must have the same hidden layers");
  }
  if (a.n_y < 1 || a.n_y > 65535) return fail(DMIP_ERR_INVALID, "n_y must be in [1, 65535]");
  if (a.n_chains < 0 || a.chain_offset < 0) return fail(DMIP_ERR_INVALID, "negative chain count/offset");
  if (a.num_steps < 1) return fail(DMIP_ERR_INVALID, "num_steps must be >= 1");
  if (!(a.sde->T > 0.0)) return fail(DMIP_ERR_INVALID, "T must be > 0");
  if (f32_act(net0) || (net1 && f32_act(net1))) {
    if (a.precision != DMIP_PREC_F32 || mode != DMIP_SAMPLER_CDE) return act_refused("em_sample");
  }
  if (a.n_chains == 0) return DMIP_OK;
  if (a.precision == DMIP_PREC_F32) return em_sample_f32(mode, net0, net1, a);
  if (a.precision == DMIP_PREC_F32X3) return em_sample_x3(mode, net0, net1, a);
  if (!dmip::sampler_shape_supported(mode, net0->width, net0->n_hidden, xdim, ydim))
    return fail(DMIP_ERR_UNSUPPORTED, "no compiled sampler (mode " + std::to_string(mode) + ") for width " +
                                          std::to_string(net0->width) + ", layers " + std::to_string(net0->n_hidden) +
                                          ", xdim " + std::to_string(xdim) + ", ydim " + std::to_string(ydim));
  hipStream_t st = (hipStream_t)a.stream;
  dmip::SamplerParams p{};
  char* a1 = nullptr;
  p.hidden = net0->hidden;
  if (mode == DMIP_SAMPLER_CDIFFE) {
    // y_t varies per chain: layer 1 takes every input column (the forward kernel's image); at width 512
    // the split layer-1 image streams through the ring ahead of the hidden chunks
    p.a1 = net0->a1_full;
    p.a1_per_y = 0;
    if (net0->width == 512) {
      if (!net0->ring_l1) return fail(DMIP_ERR_UNSUPPORTED, "no ring image for this network");
      p.hidden = net0->ring_l1;
    }
  } else {
    // y is constant per y index: fold W1_y y + b1 into a per-y layer-1 bias
    const int T = net0->width / 32;
    const int k1s = k1s_for(3 * (xdim + 1) + 2);
    hipError_t e = hipMallocAsync((void**)&a1, (size_t)a.n_y * T * k1s * 1024, st);
    if (e != hipSuccess) return fail(DMIP_ERR_ALLOC, std::string("hipMallocAsync: ") + hipGetErrorString(e));
    dmip::A1PrepParams ap{};
    ap.w1 = net0->w1;
    ap.b1 = net0->b1;
    ap.y = a.y_dev;
    ap.a1 = a1;
    ap.width = net0->width;
    ap.in_dim = net0->in_dim;
    ap.xdim = xdim;
    ap.ydim = ydim;
    ap.y_col0 = xdim;
    ap.t_col = net0->in_dim - 1;
    ap.k1s = k1s;
    e = dmip::launch_a1_prep(ap, a.n_y, st);
    if (e != hipSuccess) {
      (void)hipFreeAsync(a1, st);
      return hip_fail(e, "a1_prep launch");
    }
    p.a1 = a1;
    p.a1_per_y = 1;
  }
  p.ao = net0->ao_samp;
  p.bias_hidden = net0->bias_hidden;
  p.bias_out = net0->bias_out_samp;
  if (mode == DMIP_SAMPLER_POSTERIOR) {
    // the prior's (x, t) layer-1 image is the sampler's B1 slot layout over (x, tau)
    p.hidden2 = net1->hidden;
    p.a1_2 = net1->a1_full;
    p.ao2 = net1->ao_samp;
    p.bias_hidden2 = net1->bias_hidden;
    p.bias_out2 = net1->bias_out_samp;
  }
  p.y_obs = a.y_dev;
  p.n_corr = a.n_corr;
  p.snr = a.snr;
  p.noise = a.noise_dev;
  p.x_out = a.x_out_dev;
  p.snap_out = a.snap_out_dev;
  p.snap_every = a.snap_every;
  p.n_chains = a.n_chains;
  p.chain_offset = a.chain_offset;
  p.num_steps = a.num_steps;
  p.T = (float)a.sde->T;
  p.bmin = (float)a.sde->beta_min;
  p.bdiff = (float)(a.sde->beta_max - a.sde->beta_min);
  p.delta = (float)(a.sde->T / (double)a.num_steps);
  p.sqrt_delta = (float)std::sqrt(a.sde->T / (double)a.num_steps);
  p.mean = a.mean;
  p.stdv = a.stdv;
  p.seed = a.seed;
  p.stamps = (unsigned long long*)a.stamps;
  p.err = status_word(dmip::stream_device(st));
  if (!p.err) {
    if (a1) (void)hipFreeAsync(a1, st);
    return fail(DMIP_ERR_ALLOC, "device status word");
  }
  p.debug_flags = debug_no_handover();
  p.spin_limit = p.debug_flags ? (1u << 10) : (1u << 22);
  bool ok = false;
  hipError_t e = dmip::launch_sampler(p, mode, net0->width, net0->n_hidden, xdim, ydim, a.n_y, st, &ok);
  if (a1) (void)hipFreeAsync(a1, st);
  if (!ok) return fail(DMIP_ERR_UNSUPPORTED, "no compiled sampler");
  if (e != hipSuccess) return hip_fail(e, "em_sampler launch");
  return DMIP_OK;
}

int dmip_em_sample(const dmip_mlp* net, const dmip_vpsde* sde, const float* y_dev, int n_y, int ydim, int xdim,
                   int64_t n_chains, int64_t chain_offset, int num_steps, float mean, float stdv, uint64_t seed,
                   int precision, const float* noise_dev, float* x_out_dev, void* stream) {
  const SampleArgs a{sde,  y_dev, n_y,       ydim,      xdim,      n_chains, chain_offset, num_steps,
                     mean, stdv,  seed,      precision, noise_dev, x_out_dev, stream,      nullptr};
  return em_sample_impl(DMIP_SAMPLER_CDE, net, nullptr, a);
}

int dmip_em_sample_posterior(const dmip_mlp* prior, const dmip_mlp* likelihood, const dmip_vpsde* sde,
                             const float* y_dev, int n_y, int ydim, int xdim, int64_t n_chains, int64_t chain_offset,
                             int num_steps, float mean, float stdv, uint64_t seed, int precision, float* x_out_dev,
                             void* stream) {
  if (!prior) return fail(DMIP_ERR_INVALID, "null argument");
  const SampleArgs a{sde,  y_dev, n_y,       ydim,      xdim,    n_chains, chain_offset, num_steps,
                     mean, stdv,  seed,      precision, nullptr, x_out_dev, stream,      nullptr};
  return em_sample_impl(DMIP_SAMPLER_POSTERIOR, likelihood, prior, a);
}

int dmip_em_sample_cdiffe(const dmip_mlp* net, const dmip_vpsde* sde, const float* y_dev, int n_y, int ydim, int xdim,
                          int64_t n_chains, int64_t chain_offset, int num_steps, float mean, float stdv, uint64_t seed,
                          int precision, int corrector_steps, float snr, float* x_out_dev, void* stream) {
  if (corrector_steps < 0) return fail(DMIP_ERR_INVALID, "corrector_steps must be >= 0");
  if (corrector_steps > 0 && !(snr > 0.0f)) return fail(DMIP_ERR_INVALID, "snr must be > 0");
  SampleArgs a{sde,  y_dev, n_y,       ydim,      xdim,    n_chains, chain_offset, num_steps,
               mean, stdv,  seed,      precision, nullptr, x_out_dev, stream,      nullptr};
  a.n_corr = corrector_steps;
  a.snr = snr;
  return em_sample_impl(DMIP_SAMPLER_CDIFFE, net, nullptr, a);
}

int dmip_em_sample_snapshots(int mode, const dmip_mlp* net, const dmip_mlp* prior, const dmip_vpsde* sde,
                             const float* y_dev, int n_y, int ydim, int xdim, int64_t n_chains, int64_t chain_offset,
                             int num_steps, float mean, float stdv, uint64_t seed, int precision, int corrector_steps,
                             float snr, int snapshot_every, float* snap_out_dev, float* x_out_dev, void* stream) {
  if (mode != DMIP_SAMPLER_CDE && mode != DMIP_SAMPLER_POSTERIOR && mode != DMIP_SAMPLER_CDIFFE)
    return fail(DMIP_ERR_INVALID, "unknown sampler mode");
  if (snapshot_every < 1 || snapshot_every > num_steps)
    return fail(DMIP_ERR_INVALID, "snapshot_every must be in [1, num_steps]");
  if (!snap_out_dev) return fail(DMIP_ERR_INVALID, "null snapshot buffer");
  if (mode == DMIP_SAMPLER_POSTERIOR && !prior) return fail(DMIP_ERR_INVALID, "null argument");
  if (mode != DMIP_SAMPLER_CDIFFE && corrector_steps != 0)
    return fail(DMIP_ERR_INVALID, "corrector steps: CDiffE sampler only");
  if (corrector_steps < 0) return fail(DMIP_ERR_INVALID, "corrector_steps must be >= 0");
  if (corrector_steps > 0 && !(snr > 0.0f)) return fail(DMIP_ERR_INVALID, "snr must be > 0");
  SampleArgs a{sde,  y_dev, n_y,       ydim,      xdim,    n_chains, chain_offset, num_steps,
               mean, stdv,  seed,      precision, nullptr, x_out_dev, stream,      nullptr};
  a.n_corr = corrector_steps;
  a.snr = snr;
  a.snap_every = snapshot_every;
  a.snap_out_dev = snap_out_dev;
  return em_sample_impl(mode, net, mode == DMIP_SAMPLER_POSTERIOR ? prior : nullptr, a);
}

int dmip_em_sample_stamps(const dmip_mlp* net, const dmip_vpsde* sde, const float* y_dev, int n_y, int ydim,
                          int xdim, int64_t n_chains, int num_steps, uint64_t seed, float* x_out_dev,
                          uint64_t* stamps_dev, void* stream) {
  if (!stamps_dev) return fail(DMIP_ERR_INVALID, "null stamps buffer");
  const SampleArgs a{sde,  y_dev, n_y,  ydim,           xdim,    n_chains,  0,      num_steps,
                     0.0f, 1.0f,  seed, DMIP_PREC_FP16, nullptr, x_out_dev, stream, stamps_dev};
  return em_sample_impl(DMIP_SAMPLER_CDE, net, nullptr, a);
}

static bool train_shape_ok(int in_dim, int out_dim, int n_hidden, const int* widths, int xdim) {
  if (!widths || (n_hidden != 2 && n_hidden != 3)) return false;
  for (int i = 0; i < n_hidden; ++i)
    if (widths[i] != dmip::kTrainWidth) return false;
  return xdim == dmip::kTrainXdim && out_dim == dmip::kTrainXdim &&
         in_dim == dmip::kTrainXdim + dmip::kTrainYdim + 1;
}

int dmip_loss_grad_supported(int in_dim, int out_dim, int n_hidden, const int* widths, int xdim) {
  return train_shape_ok(in_dim, out_dim, n_hidden, widths, xdim) ? 1 : 0;
}

}  // extern "C"

// Scratch of a loss + gradient launch sequence: null = stream-ordered allocation per call (the C-ABI
// entry points); query = report the bytes only (no launch); else the caller's persistent buffer (the
// captured training-step graph, dmip_train_plan).
struct Workspace {
  char* ptr = nullptr;
  size_t bytes = 0;
  bool query = false;
};

static int loss_grad_bf16_impl(int in_dim, int out_dim, int n_hidden, const int* widths, int xdim,
                               const float* const* weights_dev, const float* const* biases_dev, const dmip_vpsde* sde,
                               const dmip_loss_cfg* cfg, const float* x_dev, const float* y_dev, const float* t_dev,
                               const float* eps_dev, int64_t batch, float* grad_out_dev, float* loss_out_dev,
                               void* stream, Workspace* ws, const dmip::TrainFuse* fuse = nullptr) {
  if (!weights_dev || !biases_dev || !sde || !cfg || !x_dev || !y_dev || !t_dev || !eps_dev || !grad_out_dev ||
      !loss_out_dev)
    return fail(DMIP_ERR_INVALID, "null argument");
  if (!train_shape_ok(in_dim, out_dim, n_hidden, widths, xdim))
    return fail(DMIP_ERR_UNSUPPORTED, "no compiled training kernel for this network (compiled: in 5, out 2, xdim 2, "
                                      "widths 64, 2 or 3 hidden layers)");
  for (int i = 0; i <= n_hidden; ++i)
    if (!weights_dev[i] || !biases_dev[i]) return fail(DMIP_ERR_INVALID, "null layer pointer");
  if (batch < 1) return fail(DMIP_ERR_INVALID, "batch must be >= 1");
  if (cfg->kind < DMIP_LOSS_DSM || cfg->kind > DMIP_LOSS_PINN2) return fail(DMIP_ERR_INVALID, "unknown loss kind");
  const bool needs_pde = cfg->kind != DMIP_LOSS_DSM;
  if (needs_pde && cfg->pde != DMIP_PDE_FPE && cfg->pde != DMIP_PDE_CFPE)
    return fail(DMIP_ERR_INVALID, "pde must be DMIP_PDE_FPE or DMIP_PDE_CFPE for this loss");
  for (int m : {cfg->pde_metric, cfg->ic_metric})
    if (m != DMIP_METRIC_L1 && m != DMIP_METRIC_L2) return fail(DMIP_ERR_INVALID, "metric must be L1 or L2");
  if (!(sde->beta_min > 0.0)) return fail(DMIP_ERR_INVALID, "beta_min must be > 0");
  hipStream_t st = (hipStream_t)stream;
  dmip::TrainParams p{};
  for (int i = 0; i <= n_hidden; ++i) p.w[i] = weights_dev[i], p.b[i] = biases_dev[i];
  p.x = x_dev;
  p.y = y_dev;
  p.t = t_dev;
  p.eps = eps_dev;
  p.n = batch;
  p.inv_n = (float)(1.0 / (double)batch);
  p.bmin = (float)sde->beta_min;
  p.bdiff = (float)(sde->beta_max - sde->beta_min);
  p.has_dsm = cfg->kind == DMIP_LOSS_DSM || cfg->kind == DMIP_LOSS_DSM_PDE || cfg->kind == DMIP_LOSS_PINN;
  p.has_ic = cfg->kind == DMIP_LOSS_PINN || cfg->kind == DMIP_LOSS_PINN2;
  p.pde = needs_pde ? cfg->pde : 0;
  p.pde_l1 = cfg->pde_metric == DMIP_METRIC_L1;
  p.ic_l1 = cfg->ic_metric == DMIP_METRIC_L1;
  p.lam = cfg->lam;
  p.lam2 = cfg->lam2;
  for (int i = 0; i < 4; ++i) p.icA[i] = cfg->ic_A[i], p.icS[i] = cfg->ic_Sinv[i];
  p.icb[0] = cfg->ic_b[0];
  p.icb[1] = cfg->ic_b[1];
  // one workgroup per CU (LDS-bound; one wave per SIMD), 16-sample tiles strided over the waves
  int n_cu = 256;
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dmip::stream_device(st));
  if (n_cu < 1) n_cu = 256;
  const int64_t tiles = (batch + 15) / 16;
  const int64_t per_wg = dmip::train_waves_per_wg();
  int n_wg = (int)std::min<int64_t>((int64_t)n_cu, (tiles + per_wg - 1) / per_wg);
  if (n_wg < 1) n_wg = 1;
  const size_t part_bytes =
      (size_t)n_wg * dmip::train_partials_per_wg() * dmip::train_partial_stride(n_hidden) * sizeof(float);
  // one scratch allocation: the partial rows, then the packed LDS image of the weights
  const size_t part_pad = (part_bytes + 255) / 256 * 256;
  const size_t packed_pad = ((size_t)dmip::train_packed_bytes(n_hidden) + 255) / 256 * 256;
  const size_t need = part_pad + packed_pad + dmip::train_adj_bytes(batch);
  if (ws && ws->query) {
    ws->bytes = need;
    return DMIP_OK;
  }
  float* partials = nullptr;
  hipError_t e = hipSuccess;
  if (ws) {
    if (ws->bytes < need) return fail(DMIP_ERR_INVALID, "workspace too small");
    partials = (float*)ws->ptr;
  } else if ((e = hipMallocAsync((void**)&partials, need, st)) != hipSuccess) {
    return fail(DMIP_ERR_ALLOC, std::string("hipMallocAsync: ") + hipGetErrorString(e));
  }
  p.packed = (char*)partials + part_pad;
  p.adj = dmip::train_adj_bytes(batch) ? (float*)((char*)partials + part_pad + packed_pad) : nullptr;
  e = fuse ? dmip::launch_loss_grad_fused(p, n_hidden, grad_out_dev, loss_out_dev, partials, n_wg, *fuse, st)
           : dmip::launch_loss_grad(p, n_hidden, grad_out_dev, loss_out_dev, partials, n_wg, st);
  if (!ws) (void)hipFreeAsync(partials, st);
  if (e != hipSuccess) return hip_fail(e, "loss_grad launch");
  return DMIP_OK;
}

static int loss_grad_f32_impl(int in_dim, int out_dim, int n_hidden, const int* widths, int xdim,
                              const float* const* weights_dev, const float* const* biases_dev, const dmip_vpsde* sde,
                              const dmip_loss_cfg* cfg, const float* x_dev, const float* y_dev, const float* t_dev,
                              const float* eps_dev, const float* ic_target_dev, int64_t batch, float* grad_out_dev,
                              float* loss_out_dev, void* stream, Workspace* ws) {
  if (!widths || !weights_dev || !biases_dev || !sde || !cfg || !x_dev || !y_dev || !t_dev || !eps_dev ||
      !grad_out_dev || !loss_out_dev)
    return fail(DMIP_ERR_INVALID, "null argument");
  if (n_hidden < 1 || n_hidden > dmip::kJetsMaxLayers - 1) return fail(DMIP_ERR_UNSUPPORTED, "n_hidden must be in [1, 8]");
  if (out_dim != xdim) return fail(DMIP_ERR_UNSUPPORTED, "f32 training: score networks with out_dim == xdim");
  if (xdim < 1 || xdim > (cfg->kind == DMIP_LOSS_DSM ? dmip::kJetsMaxDsmDim : 4))
    return fail(DMIP_ERR_UNSUPPORTED, "f32 training: xdim in [1, 4] (DSMLoss: [1, 64])");
  const int ydim = in_dim - xdim - 1;
  if (ydim < 0) return fail(DMIP_ERR_INVALID, "in_dim must be xdim + ydim + 1");
  for (int i = 0; i < n_hidden; ++i)
    if (widths[i] < 1 || widths[i] > 4096) return fail(DMIP_ERR_INVALID, "hidden widths must be in [1, 4096]");
  for (int i = 0; i <= n_hidden; ++i)
    if (!weights_dev[i] || !biases_dev[i]) return fail(DMIP_ERR_INVALID, "null layer pointer");
  if (batch < 1) return fail(DMIP_ERR_INVALID, "batch must be >= 1");
  if (cfg->kind < DMIP_LOSS_DSM || cfg->kind > DMIP_LOSS_PINN2) return fail(DMIP_ERR_INVALID, "unknown loss kind");
  const bool has_pde = cfg->kind != DMIP_LOSS_DSM;
  const bool has_ic = cfg->kind == DMIP_LOSS_PINN || cfg->kind == DMIP_LOSS_PINN2;
  if (has_pde && cfg->pde != DMIP_PDE_FPE && cfg->pde != DMIP_PDE_CFPE)
    return fail(DMIP_ERR_INVALID, "pde must be DMIP_PDE_FPE or DMIP_PDE_CFPE for this loss");
  if (has_ic && !ic_target_dev && (xdim != 2 || ydim != 2))
    return fail(DMIP_ERR_INVALID, "initial-condition target required (the built-in one is the linear problem's, 2-D)");
  if (!(sde->beta_min > 0.0)) return fail(DMIP_ERR_INVALID, "beta_min must be > 0");
  hipStream_t st = (hipStream_t)stream;
  const int64_t B = batch;
  dmip::JetsParams p{};
  p.batch = B;
  p.xdim = xdim;
  p.ydim = ydim;
  p.out_dim = out_dim;
  p.bmin = (float)sde->beta_min;
  p.bdiff = (float)(sde->beta_max - sde->beta_min);
  p.lam = cfg->lam;
  p.lam2 = cfg->lam2;
  p.has_dsm = cfg->kind != DMIP_LOSS_PINN2;
  p.pde = has_pde ? cfg->pde : 0;
  p.pde_l1 = cfg->pde_metric == DMIP_METRIC_L1;
  p.ic_l1 = cfg->ic_metric == DMIP_METRIC_L1;
  for (int i = 0; i < 4; ++i) p.icA[i] = cfg->ic_A[i], p.icS[i] = cfg->ic_Sinv[i];
  p.icb[0] = cfg->ic_b[0];
  p.icb[1] = cfg->ic_b[1];
  p.x = x_dev;
  p.y = y_dev;
  p.t = t_dev;
  p.eps = eps_dev;
  p.ic_target = ic_target_dev;
  const bool fpe = has_pde && cfg->pde == DMIP_PDE_FPE;
  p.blk_v = has_pde ? 1 : -1;
  p.blk_c = has_ic ? (has_pde ? 2 : 1) : -1;
  p.n_bwd = 1 + (has_pde ? 1 : 0) + (has_ic ? 1 : 0);
  p.blk_e = p.n_bwd;
  p.n_e = fpe ? xdim : 0;
  p.n_pair = fpe ? xdim * (xdim + 1) / 2 : 0;
  p.n_streams = p.n_bwd + p.n_e + p.n_pair;
  int wmax = in_dim + 1;
  for (int i = 0; i < n_hidden; ++i) wmax = std::max(wmax, widths[i] + 1);
  p.splits = 64;  // the cap: each weight-gradient GEMM picks its own split count (dmip_jets.hip wgrad_splits)
  const int64_t nS = p.n_streams, nb = p.n_bwd;
  std::vector<std::pair<float**, size_t>> plan;
  for (int l = 0; l <= n_hidden; ++l) plan.emplace_back(&p.h[l], (size_t)nS * B * ((l == 0 ? in_dim : widths[l - 1]) + 1));
  for (int l = 0; l < n_hidden; ++l) plan.emplace_back(&p.aux[l], (size_t)3 * B * widths[l]);
  plan.emplace_back(&p.scal, (size_t)B * 8);
  plan.emplace_back(&p.x_t, (size_t)B * xdim);
  plan.emplace_back(&p.z, (size_t)nS * B * wmax);
  plan.emplace_back(&p.a_out, (size_t)nS * B * out_dim);
  plan.emplace_back(&p.zbar, (size_t)nb * B * out_dim);
  plan.emplace_back(&p.zbar_a, (size_t)nb * B * wmax);
  plan.emplace_back(&p.zbar_b, (size_t)nb * B * wmax);
  plan.emplace_back(&p.hbar, (size_t)nb * B * wmax);
  plan.emplace_back(&p.rows, (size_t)B * 3);
  plan.emplace_back(&p.part, (size_t)p.splits * wmax * wmax);
  size_t total = 0;
  for (auto& q : plan) total += (q.second * sizeof(float) + 255) / 256 * 256;
  if (ws && ws->query) {
    ws->bytes = total;
    return DMIP_OK;
  }
  char* scratch = nullptr;
  hipError_t e = hipSuccess;
  if (ws) {
    if (ws->bytes < total) return fail(DMIP_ERR_INVALID, "workspace too small");
    scratch = ws->ptr;
  } else if ((e = hipMallocAsync((void**)&scratch, total, st)) != hipSuccess) {
    return fail(DMIP_ERR_ALLOC, std::string("hipMallocAsync: ") + hipGetErrorString(e));
  }
  size_t o = 0;
  for (auto& q : plan) {
    *q.first = (float*)(scratch + o);
    o += (q.second * sizeof(float) + 255) / 256 * 256;
  }
  p.loss_out = loss_out_dev;
  e = dmip::launch_jets_loss_grad(p, n_hidden, widths, weights_dev, biases_dev, grad_out_dev, st);
  if (!ws) (void)hipFreeAsync(scratch, st);
  if (e != hipSuccess) return hip_fail(e, "loss_grad_f32 launch");
  return DMIP_OK;
}

extern "C" {

int dmip_loss_grad(int in_dim, int out_dim, int n_hidden, const int* widths, int xdim,
                   const float* const* weights_dev, const float* const* biases_dev, const dmip_vpsde* sde,
                   const dmip_loss_cfg* cfg, const float* x_dev, const float* y_dev, const float* t_dev,
                   const float* eps_dev, int64_t batch, float* grad_out_dev, float* loss_out_dev, void* stream) {
  return loss_grad_bf16_impl(in_dim, out_dim, n_hidden, widths, xdim, weights_dev, biases_dev, sde, cfg, x_dev,
                             y_dev, t_dev, eps_dev, batch, grad_out_dev, loss_out_dev, stream, nullptr);
}

int dmip_loss_grad_f32(int in_dim, int out_dim, int n_hidden, const int* widths, int xdim,
                       const float* const* weights_dev, const float* const* biases_dev, const dmip_vpsde* sde,
                       const dmip_loss_cfg* cfg, const float* x_dev, const float* y_dev, const float* t_dev,
                       const float* eps_dev, const float* ic_target_dev, int64_t batch, float* grad_out_dev,
                       float* loss_out_dev, void* stream) {
  return loss_grad_f32_impl(in_dim, out_dim, n_hidden, widths, xdim, weights_dev, biases_dev, sde, cfg, x_dev, y_dev,
                            t_dev, eps_dev, ic_target_dev, batch, grad_out_dev, loss_out_dev, stream, nullptr);
}

}  // extern "C"

static int draws_params(uint64_t seed, uint64_t stream_id, int64_t batch, int xdim, int debias, const dmip_vpsde* sde,
                        double t_epsilon, float t_add, float* t_out_dev, float* eps_out_dev, dmip::TrainDrawsParams& p) {
  if (!sde || !t_out_dev || !eps_out_dev) return fail(DMIP_ERR_INVALID, "null argument");
  if (batch < 0 || xdim < 1 || xdim > 4) return fail(DMIP_ERR_INVALID, "batch >= 0 and xdim in [1, 4]");
  if (!(sde->T > 0.0) || !(sde->beta_min > 0.0)) return fail(DMIP_ERR_INVALID, "bad SDE parameters");
  p = dmip::TrainDrawsParams{};
  p.batch = batch;
  p.xdim = xdim;
  p.debias = debias ? 1 : 0;
  p.seed = seed;
  p.stream_id = stream_id;
  p.t_add = t_add;
  p.T = (float)sde->T;
  const double a = sde->beta_max - sde->beta_min, b = sde->beta_min, te = t_epsilon;
  const double B_te = 0.5 * a * te * te + b * te;
  const double r_te = (b + a * te) / (1.0 - std::exp(-B_te));
  const double A_te = std::log(std::expm1(B_te));
  const double B_T = 0.5 * a * sde->T * sde->T + b * sde->T;
  p.a = (float)a;
  p.b = (float)b;
  p.te = (float)te;
  p.r_te = (float)r_te;
  p.A_te = (float)A_te;
  p.Z = (float)(te * r_te + std::log(std::expm1(B_T)) - A_te);
  p.t = t_out_dev;
  p.eps = eps_out_dev;
  return DMIP_OK;
}

static int adam_params(int n_tensors, float* const* params, const float* const* grads, float* const* exp_avg,
                       float* const* exp_avg_sq, const int64_t* numel, double lr, double beta1, double beta2,
                       double eps, int64_t step, dmip::AdamParams& p) {
  if (!params || !grads || !exp_avg || !exp_avg_sq || !numel) return fail(DMIP_ERR_INVALID, "null argument");
  if (n_tensors < 1 || n_tensors > dmip::kAdamMaxTensors)
    return fail(DMIP_ERR_UNSUPPORTED, "n_tensors must be in [1, 16]");
  if (step < 1) return fail(DMIP_ERR_INVALID, "step must be >= 1 (torch increments before the update)");
  p = dmip::AdamParams{};
  p.n = n_tensors;
  p.off[0] = 0;
  for (int k = 0; k < n_tensors; ++k) {
    if (!params[k] || !grads[k] || !exp_avg[k] || !exp_avg_sq[k] || numel[k] < 0)
      return fail(DMIP_ERR_INVALID, "null tensor or negative size");
    p.param[k] = params[k];
    p.grad[k] = grads[k];
    p.m[k] = exp_avg[k];
    p.v[k] = exp_avg_sq[k];
    p.off[k + 1] = p.off[k] + numel[k];
  }
  // torch.optim.Adam's scalars, in Python double like torch computes them
  const double bc1 = 1.0 - std::pow(beta1, (double)step), bc2 = 1.0 - std::pow(beta2, (double)step);
  p.step_size = (float)(lr / bc1);
  p.bc2_sqrt = (float)std::sqrt(bc2);
  p.w1 = (float)(1.0 - beta1);
  p.beta2 = (float)beta2;
  p.w2 = (float)(1.0 - beta2);
  p.eps = (float)eps;
  p.lr_d = lr;
  p.beta1_d = beta1;
  p.beta2_d = beta2;
  return DMIP_OK;
}

// ----------------------------------------------------------------- captured training-step graph
struct dmip_train_plan {
  hipGraphExec_t exec = nullptr;
  hipGraph_t graph = nullptr;
  int64_t batch = 0;
  int xdim = 0, ydim = 0;
  float *x = nullptr, *y = nullptr;          // staging: the batch is copied in at each replay
  float *t = nullptr, *eps = nullptr, *loss = nullptr;  // caller-owned
  char* ws = nullptr;
  dmip::StepCounters* ctr = nullptr;
  int device = 0;
  // the draws launch stages the batch itself: each step points that kernel node's x_src / y_src at the caller's
  // batch (hipGraphExecKernelNodeSetParams) instead of two copy nodes; `stage_node` null: copies (fallback)
  hipGraphNode_t stage_node = nullptr;
  hipKernelNodeParams stage_kp{};
  int stage_nargs = 0;
  alignas(16) char stage_args[3][1024];      // the node's argument values (TrainDrawsParams first)
  void* stage_argv[3] = {};
};

// makes `dev` the current device for the guard's scope (and restores the caller's)
struct DeviceGuard {
  int prev = -1, dev = -1;
  explicit DeviceGuard(int d) : dev(d) {
    if (hipGetDevice(&prev) == hipSuccess && prev != dev && dev >= 0) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0 && prev != dev && dev >= 0) (void)hipSetDevice(prev);
  }
};

// the device that owns a device pointer (the current device if the runtime cannot tell)
static int pointer_device(const void* p) {
  hipPointerAttribute_t a{};
  int cur = 0;
  (void)hipGetDevice(&cur);
  if (!p) return cur;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // clear only the error this query left (a non-device pointer)
    return cur;
  }
  return a.device >= 0 ? a.device : cur;
}

static void plan_free(dmip_train_plan* pl) {
  if (!pl) return;
  if (pl->exec) (void)hipGraphExecDestroy(pl->exec);
  if (pl->graph) (void)hipGraphDestroy(pl->graph);
  for (void* q : {(void*)pl->x, (void*)pl->y, (void*)pl->ws, (void*)pl->ctr})
    if (q) (void)hipFree(q);
  delete pl;
}

extern "C" {

int dmip_train_draws(uint64_t seed, uint64_t stream_id, int64_t batch, int xdim, int debias, const dmip_vpsde* sde,
                     double t_epsilon, float t_add, float* t_out_dev, float* eps_out_dev, void* stream) {
  dmip::TrainDrawsParams p{};
  const int rc = draws_params(seed, stream_id, batch, xdim, debias, sde, t_epsilon, t_add, t_out_dev, eps_out_dev, p);
  if (rc != DMIP_OK || batch == 0) return rc;
  hipError_t e = dmip::launch_train_draws(p, (hipStream_t)stream);
  return e == hipSuccess ? DMIP_OK : hip_fail(e, "train_draws launch");
}

int dmip_adam_step(int n_tensors, float* const* params, const float* const* grads, float* const* exp_avg,
                   float* const* exp_avg_sq, const int64_t* numel, double lr, double beta1, double beta2, double eps,
                   int64_t step, void* stream) {
  dmip::AdamParams p{};
  const int rc = adam_params(n_tensors, params, grads, exp_avg, exp_avg_sq, numel, lr, beta1, beta2, eps, step, p);
  if (rc != DMIP_OK) return rc;
  hipError_t e = dmip::launch_adam(p, (hipStream_t)stream);
  return e == hipSuccess ? DMIP_OK : hip_fail(e, "adam launch");
}

int dmip_train_plan_create(const dmip_train_plan_desc* d, dmip_train_plan** out) {
  if (!d || !out || !d->widths || !d->weights_dev || !d->biases_dev || !d->t_dev || !d->eps_dev || !d->loss_dev)
    return fail(DMIP_ERR_INVALID, "null argument");
  *out = nullptr;
  if (d->batch < 1) return fail(DMIP_ERR_INVALID, "batch must be >= 1");
  if (d->precision != DMIP_PREC_BF16 && d->precision != DMIP_PREC_F32) return fail(DMIP_ERR_INVALID, "unknown precision");
  const int ydim = d->in_dim - d->xdim - 1;
  if (d->xdim < 1 || d->xdim > 4 || ydim < 0) return fail(DMIP_ERR_INVALID, "xdim in [1, 4] and in_dim = xdim + ydim + 1");
  const bool has_ic = d->cfg.kind == DMIP_LOSS_PINN || d->cfg.kind == DMIP_LOSS_PINN2;
  if (has_ic && (d->xdim != 2 || ydim != 2))
    return fail(DMIP_ERR_UNSUPPORTED, "captured steps take the built-in (linear-problem) initial condition only");
  const bool bf16 = d->precision == DMIP_PREC_BF16;
  if (bf16 && !train_shape_ok(d->in_dim, d->out_dim, d->n_hidden, d->widths, d->xdim))
    return fail(DMIP_ERR_UNSUPPORTED, "no compiled bf16 training kernel for this network");
  dmip::AdamParams ap{};
  int rc = adam_params(d->n_tensors, d->params, d->grads, d->exp_avg, d->exp_avg_sq, d->numel, d->lr, d->beta1,
                       d->beta2, d->eps, 1, ap);
  if (rc != DMIP_OK) return rc;
  for (int k = 1; k < d->n_tensors; ++k)
    if (d->grads[k] != d->grads[0] + ap.off[k])
      return fail(DMIP_ERR_INVALID, "grads must be consecutive views of one flat buffer (reference parameter order)");
  // everything the plan allocates, and its capture stream, live on the parameters' device, whatever the
  // caller's current device is (the weights, optimizer state and the replay stream are that device's)
  const DeviceGuard guard(pointer_device(d->weights_dev[0]));
  auto* pl = new dmip_train_plan();
  pl->batch = d->batch;
  pl->xdim = d->xdim;
  pl->ydim = ydim;
  pl->t = d->t_dev;
  pl->eps = d->eps_dev;
  pl->loss = d->loss_dev;
  pl->device = guard.dev;
  const int64_t B = d->batch;
  auto alloc = [&](void** q, size_t bytes) { return hipMalloc(q, bytes < 4 ? 4 : bytes); };
  hipError_t e = hipSuccess;
  if ((e = alloc((void**)&pl->x, (size_t)B * d->xdim * 4)) != hipSuccess ||
      (e = alloc((void**)&pl->y, (size_t)B * ydim * 4)) != hipSuccess ||
      (e = alloc((void**)&pl->ctr, sizeof(dmip::StepCounters))) != hipSuccess) {
    plan_free(pl);
    return fail(DMIP_ERR_ALLOC, std::string("hipMalloc: ") + hipGetErrorString(e));
  }
  dmip::StepCounters c0{0ull, (long long)d->step0};
  if ((e = hipMemcpy(pl->ctr, &c0, sizeof(c0), hipMemcpyHostToDevice)) != hipSuccess) {
    plan_free(pl);
    return hip_fail(e, "counter init");
  }
  // workspace of the loss sequence, sized by a query pass
  Workspace ws;
  ws.query = true;
  const dmip::TrainFuse* fuse = nullptr;  // bf16: the fused prologue / reduction + Adam launches (set below)
  auto loss_seq = [&](hipStream_t st, Workspace* w) {
    return bf16 ? loss_grad_bf16_impl(d->in_dim, d->out_dim, d->n_hidden, d->widths, d->xdim, d->weights_dev,
                                      d->biases_dev, &d->sde, &d->cfg, pl->x, pl->y, pl->t, pl->eps, B,
                                      d->grads[0], pl->loss, st, w, fuse)
                : loss_grad_f32_impl(d->in_dim, d->out_dim, d->n_hidden, d->widths, d->xdim, d->weights_dev,
                                     d->biases_dev, &d->sde, &d->cfg, pl->x, pl->y, pl->t, pl->eps, nullptr, B,
                                     d->grads[0], pl->loss, st, w);
  };
  if ((rc = loss_seq(nullptr, &ws)) != DMIP_OK) {
    plan_free(pl);
    return rc;
  }
  if ((e = alloc((void**)&pl->ws, ws.bytes)) != hipSuccess) {
    plan_free(pl);
    return fail(DMIP_ERR_ALLOC, std::string("hipMalloc: ") + hipGetErrorString(e));
  }
  ws.ptr = pl->ws;
  ws.query = false;
  dmip::TrainDrawsParams dp{};
  if ((rc = draws_params(d->seed, d->first_draw, B, d->xdim, d->debias, &d->sde, d->t_epsilon, d->t_add, pl->t,
                         pl->eps, dp)) != DMIP_OK) {
    plan_free(pl);
    return rc;
  }
  dp.draw_ctr = &pl->ctr->draw;
  ap.step_ctr = &pl->ctr->step;
  // the draws launch stages the batch (x_src / y_src set per step in its kernel node)
  dp.x_src = pl->x, dp.y_src = pl->y, dp.x_dst = pl->x, dp.y_dst = pl->y, dp.ydim = ydim;
  // bf16 (the config-5 kernel): four launches -- the pack in the draws launch, Adam and the counters in the
  // gradient reduction (dmip::TrainFuse); exact f32: draws -> loss + gradients -> Adam -> advance the counters
  const dmip::TrainFuse fz{dp, ap, pl->ctr};
  if (bf16 && dmip::train_split()) fuse = &fz;
  hipStream_t cs = nullptr;
  if ((e = hipStreamCreateWithFlags(&cs, hipStreamNonBlocking)) != hipSuccess) {
    plan_free(pl);
    return hip_fail(e, "capture stream");
  }
  hipGraph_t g = nullptr;
  e = hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed);
  if (e == hipSuccess) {
    hipError_t le = hipSuccess;
    int lrc = DMIP_OK;
    if (fuse) {
      lrc = loss_seq(cs, &ws);
    } else {
      le = dmip::launch_train_draws(dp, cs);
      lrc = le == hipSuccess ? loss_seq(cs, &ws) : DMIP_ERR_HIP;
      if (lrc == DMIP_OK && (le = dmip::launch_adam(ap, cs)) == hipSuccess) le = dmip::launch_counters_advance(pl->ctr, cs);
    }
    e = hipStreamEndCapture(cs, &g);
    if (e == hipSuccess && (le != hipSuccess || lrc != DMIP_OK)) e = le != hipSuccess ? le : hipErrorUnknown;
  }
  if (e == hipSuccess) e = hipGraphInstantiate(&pl->exec, g, nullptr, nullptr, 0);
  (void)hipStreamDestroy(cs);
  if (e != hipSuccess) {
    if (g) (void)hipGraphDestroy(g);
    plan_free(pl);
    return hip_fail(e, "training-step graph capture");
  }
  pl->graph = g;
  // the staging kernel node: its arguments are kept here and re-pointed at each step's batch
  const void* stage_fn = fuse ? dmip::train_plan_prologue_func(d->n_hidden) : dmip::train_draws_func();
  size_t nn = 0;
  if (hipGraphGetNodes(g, nullptr, &nn) == hipSuccess && nn > 0) {
    std::vector<hipGraphNode_t> nodes(nn);
    if (hipGraphGetNodes(g, nodes.data(), &nn) == hipSuccess)
      for (size_t i = 0; i < nn && !pl->stage_node; ++i) {
        hipGraphNodeType ty;
        hipKernelNodeParams kp{};
        if (hipGraphNodeGetType(nodes[i], &ty) != hipSuccess || ty != hipGraphNodeTypeKernel) continue;
        if (hipGraphKernelNodeGetParams(nodes[i], &kp) != hipSuccess || kp.func != stage_fn || !kp.kernelParams) continue;
        // prologue (TrainDrawsParams, TrainParams, int) or draws (TrainDrawsParams)
        const size_t sizes[3] = {sizeof(dmip::TrainDrawsParams), sizeof(dmip::TrainParams), sizeof(int)};
        const int nargs = fuse ? 3 : 1;
        for (int a = 0; a < nargs; ++a) {
          std::memcpy(pl->stage_args[a], kp.kernelParams[a], sizes[a]);
          pl->stage_argv[a] = pl->stage_args[a];
        }
        pl->stage_kp = kp;
        pl->stage_kp.kernelParams = pl->stage_argv;
        pl->stage_kp.extra = nullptr;
        pl->stage_nargs = nargs;
        pl->stage_node = nodes[i];
      }
  }
  (void)hipGetLastError();
  *out = pl;
  return DMIP_OK;
}

int dmip_train_plan_step(dmip_train_plan* pl, const float* x_dev, const float* y_dev, void* stream) {
  if (!pl || !x_dev || (pl->ydim > 0 && !y_dev)) return fail(DMIP_ERR_INVALID, "null argument");
  hipStream_t st = (hipStream_t)stream;
  const DeviceGuard guard(pl->device);
  hipError_t e = hipSuccess;
  if (pl->stage_node) {  // the draws launch copies the batch in: point its node at this step's x / y
    auto* dp = (dmip::TrainDrawsParams*)pl->stage_args[0];
    dp->x_src = x_dev;
    dp->y_src = pl->ydim > 0 ? y_dev : pl->y;
    e = hipGraphExecKernelNodeSetParams(pl->exec, pl->stage_node, &pl->stage_kp);
  } else {
    e = hipMemcpyAsync(pl->x, x_dev, (size_t)pl->batch * pl->xdim * 4, hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess && pl->ydim > 0)
      e = hipMemcpyAsync(pl->y, y_dev, (size_t)pl->batch * pl->ydim * 4, hipMemcpyDeviceToDevice, st);
  }
  if (e == hipSuccess) e = hipGraphLaunch(pl->exec, st);
  return e == hipSuccess ? DMIP_OK : hip_fail(e, "training-step graph launch");
}

int dmip_train_plan_set_counters(dmip_train_plan* pl, uint64_t draws_done, int64_t steps_done, void* stream) {
  if (!pl) return fail(DMIP_ERR_INVALID, "null argument");
  if (steps_done < 0) return fail(DMIP_ERR_INVALID, "steps_done must be >= 0");
  // stream-ordered after earlier replays; the source is copied before this call returns
  const dmip::StepCounters c{(unsigned long long)draws_done, (long long)steps_done};
  hipError_t e = hipMemcpyAsync(pl->ctr, &c, sizeof(c), hipMemcpyHostToDevice, (hipStream_t)stream);
  if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
  return e == hipSuccess ? DMIP_OK : hip_fail(e, "counter update");
}

int dmip_train_plan_destroy(dmip_train_plan* pl) {
  if (!pl) return DMIP_OK;
  const DeviceGuard guard(pl->device);
  (void)hipDeviceSynchronize();  // no replay may still be running on the plan's device
  plan_free(pl);
  return DMIP_OK;
}

int dmip_histogram(const float* x_dev, int64_t n, int d, int nbins, double lo, double hi, int n_hist,
                   uint32_t* counts_dev, void* stream) {
  if (!x_dev || !counts_dev) return fail(DMIP_ERR_INVALID, "null argument");
  if (d < 1 || d > 3 || nbins < 1 || nbins > 4096 || n < 0 || n_hist < 1 || n_hist > 65535 || !(hi > lo))
    return fail(DMIP_ERR_INVALID, "bad histogram shape or range");
  if (n == 0) return DMIP_OK;
  hipError_t e = dmip::launch_histogram(x_dev, n, d, nbins, lo, hi, n_hist, (unsigned int*)counts_dev,
                                        (hipStream_t)stream);
  return e == hipSuccess ? DMIP_OK : hip_fail(e, "histogram launch");
}

}  // extern "C"

// ------------------------------------------------------------------- scatterometry surrogate
struct dmip_surrogate {
  float* l1 = nullptr;
  float* bias = nullptr;
  char* img[7] = {};  // w2, w3, w4, w3t, w2t, w4t, w1t
  // fp32x3 images (dmip_dps_x3.hip): chunks S2 | S3 | Sout | S4^T | S3^T | S2^T | S1^T, layer 1, biases; none when
  // a weight is beyond fp16's range (x3_range)
  char* x3_img = nullptr;
  char* x3_l1 = nullptr;
  float* x3_bias = nullptr;  // b1 | b2 | b3 [256] | b4 [32]
  double x3_range = 0.0;
  ~dmip_surrogate() {
    if (l1) (void)hipFree(l1);
    if (bias) (void)hipFree(bias);
    for (char* p : img)
      if (p) (void)hipFree(p);
    for (void* p : {(void*)x3_img, (void*)x3_l1, (void*)x3_bias})
      if (p) (void)hipFree(p);
  }
};

namespace {

int surrogate_check(const dmip_surrogate* s, int64_t n) {
  if (!s) return fail(DMIP_ERR_INVALID, "null surrogate handle");
  if (n < 0) return fail(DMIP_ERR_INVALID, "n < 0");
  return DMIP_OK;
}

int surrogate_n_wg(int64_t rows, hipStream_t st) {
  int n_cu = 256;
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dmip::stream_device(st));
  if (n_cu < 1) n_cu = 256;
  const int64_t per = dmip::surrogate_rows_per_wg();
  return (int)std::max<int64_t>(1, std::min<int64_t>(n_cu, (rows + per - 1) / per));
}

void surrogate_params(const dmip_surrogate* s, dmip::SurrogateParams& p) {
  p.l1 = s->l1;
  p.bias = s->bias;
  p.w2 = s->img[0];
  p.w3 = s->img[1];
  p.w4 = s->img[2];
  p.w3t = s->img[3];
  p.w2t = s->img[4];
  p.w4t = s->img[5];
  p.w1t = s->img[6];
}

int noise_check(const dmip_scat_noise* nz, dmip::SurrogateParams& p) {
  if (!nz) return fail(DMIP_ERR_INVALID, "null noise model");
  if (!(nz->b > 0.0f) || !(nz->a >= 0.0f) || !(nz->lambd_bd >= 0.0f))
    return fail(DMIP_ERR_INVALID, "noise model needs b > 0, a >= 0, lambd_bd >= 0");
  p.a = nz->a;
  p.b2 = (float)((double)nz->b * (double)nz->b);  // python b**2, rounded once to f32 (torch scalar add)
  p.lam = nz->lambd_bd;
  return DMIP_OK;
}

}  // namespace

extern "C" {

int dmip_surrogate_create(int in_dim, int out_dim, int n_hidden, const int* widths, const float* const* weights,
                          const float* const* biases, dmip_surrogate** out) {
  using dmip::kSurW;
  if (!out || !widths || !weights || !biases) return fail(DMIP_ERR_INVALID, "null argument");
  *out = nullptr;
  if (in_dim != dmip::kSurXdim || out_dim != dmip::kSurYdim || n_hidden != 3)
    return fail(DMIP_ERR_UNSUPPORTED, "surrogate compiled for in 3, out 23, 3 hidden layers");
  for (int i = 0; i < 3; ++i)
    if (widths[i] != kSurW) return fail(DMIP_ERR_UNSUPPORTED, "surrogate compiled for hidden widths [256]*3");
  for (int i = 0; i < 4; ++i)
    if (!weights[i] || !biases[i]) return fail(DMIP_ERR_INVALID, "null layer pointer");
  const float *W1 = weights[0], *W2 = weights[1], *W3 = weights[2], *W4 = weights[3];
  const int XD = dmip::kSurXdim, YD = dmip::kSurYdim;
  auto sq = [](const float* Wm) {
    return [Wm](int r, int c) { return Wm[(size_t)r * kSurW + c]; };
  };
  auto tr = [](const float* Wm) {
    return [Wm](int r, int c) { return Wm[(size_t)c * kSurW + r]; };
  };
  std::vector<char> imgs[7] = {
      pack_f32_tiles(16, 16, sq(W2)),
      pack_f32_tiles(16, 16, sq(W3)),
      pack_f32_tiles(2, 16, [&](int r, int c) { return r < YD ? W4[(size_t)r * kSurW + c] : 0.0f; }),
      pack_f32_tiles(16, 16, tr(W3)),
      pack_f32_tiles(16, 16, tr(W2)),
      pack_f32_tiles(16, 2, [&](int r, int c) { return c < YD ? W4[(size_t)c * kSurW + r] : 0.0f; }),
      pack_f32_tiles(1, 16, [&](int r, int c) { return r < XD ? W1[(size_t)c * XD + r] : 0.0f; }),
  };
  std::vector<float> l1((size_t)16 * 64), bias((size_t)3 * kSurW + 32, 0.0f);
  for (int o = 0; o < 16; ++o)
    for (int l = 0; l < 64; ++l) {
      const int row = 16 * o + (l & 15), g = l >> 4;
      l1[(size_t)o * 64 + l] = g < XD ? W1[(size_t)row * XD + g] : biases[0][row];
    }
  for (int li = 0; li < 3; ++li)
    for (int k = 0; k < kSurW; ++k) bias[(size_t)li * kSurW + k] = biases[li][k];
  for (int k = 0; k < YD; ++k) bias[(size_t)3 * kSurW + k] = biases[3][k];

  dmip_surrogate* s = new (std::nothrow) dmip_surrogate;
  if (!s) return fail(DMIP_ERR_ALLOC, "host allocation");
  int rc = DMIP_OK;
  if ((rc = upload(&s->l1, l1)) || (rc = upload(&s->bias, bias))) {
    delete s;
    return rc;
  }
  for (int i = 0; i < 7; ++i)
    if ((rc = upload(&s->img[i], imgs[i]))) {
      delete s;
      return rc;
    }
  {  // the fp32x3 DPS engine's images (plain splits; the surrogate is ReLU, no folds)
    double mx = 0.0;
    std::vector<char> chunks;
    append_chunks(chunks, pack_x3_plain(16, 8, [&](int r, int c) { return W2[(size_t)r * kSurW + c]; }, &mx));
    append_chunks(chunks, pack_x3_plain(16, 8, [&](int r, int c) { return W3[(size_t)r * kSurW + c]; }, &mx));
    append_chunks(chunks, pack_x3_plain(2, 8, [&](int r, int c) { return r < YD ? W4[(size_t)r * kSurW + c] : 0.0f; }, &mx));
    append_chunks(chunks, pack_x3_plain(16, 1, [&](int r, int c) { return c < YD ? W4[(size_t)c * kSurW + r] : 0.0f; }, &mx));
    append_chunks(chunks, pack_x3_plain(16, 8, [&](int r, int c) { return W3[(size_t)c * kSurW + r]; }, &mx));
    append_chunks(chunks, pack_x3_plain(16, 8, [&](int r, int c) { return W2[(size_t)c * kSurW + r]; }, &mx));
    append_chunks(chunks, pack_x3_plain(1, 8, [&](int r, int c) { return r < XD ? W1[(size_t)c * XD + r] : 0.0f; }, &mx));
    for (size_t i = 0; i < (size_t)kSurW * XD; ++i) mx = std::max(mx, std::fabs((double)W1[i]));
    if (!(mx <= 65504.0) || chunks.size() != (size_t)dmip::kDpsX3SurChunks * dmip::kDpsX3Chunk) {
      s->x3_range = std::isfinite(mx) ? mx : 1e300;
    } else {
      const std::vector<uint16_t> l1x = pack_x3_l1(W1, kSurW, XD, {0, 1, 2}, 1.0);
      std::vector<char> l1b(l1x.size() * 2);
      std::memcpy(l1b.data(), l1x.data(), l1b.size());
      if ((rc = upload(&s->x3_img, chunks)) || (rc = upload(&s->x3_l1, l1b)) || (rc = upload(&s->x3_bias, bias))) {
        delete s;
        return rc;
      }
    }
  }
  *out = s;
  return DMIP_OK;
}

int dmip_surrogate_destroy(dmip_surrogate* s) {
  delete s;
  return DMIP_OK;
}

int dmip_surrogate_forward(const dmip_surrogate* s, const float* x_dev, int64_t n, float* f_out_dev, void* stream) {
  if (int rc = surrogate_check(s, n)) return rc;
  if (n == 0) return DMIP_OK;
  if (!x_dev || !f_out_dev) return fail(DMIP_ERR_INVALID, "null argument");
  dmip::SurrogateParams p{};
  surrogate_params(s, p);
  p.x = x_dev;
  p.n = n;
  p.f_out = f_out_dev;
  hipError_t e = dmip::launch_surrogate_eval(p, 0, surrogate_n_wg(n, (hipStream_t)stream), (hipStream_t)stream);
  return e == hipSuccess ? DMIP_OK : hip_fail(e, "surrogate_forward launch");
}

int dmip_log_posterior(const dmip_surrogate* s, const dmip_scat_noise* noise, const float* x_dev, const float* y_dev,
                       int64_t y_stride, int64_t n, float* e_out_dev, float* grad_out_dev, void* stream) {
  if (int rc = surrogate_check(s, n)) return rc;
  dmip::SurrogateParams p{};
  if (int rc = noise_check(noise, p)) return rc;
  if (y_stride != 0 && y_stride != dmip::kSurYdim) return fail(DMIP_ERR_INVALID, "y_stride must be 0 or 23");
  if (n == 0) return DMIP_OK;
  if (!x_dev || !y_dev || !e_out_dev) return fail(DMIP_ERR_INVALID, "null argument");
  surrogate_params(s, p);
  p.x = x_dev;
  p.y = y_dev;
  p.y_stride = y_stride;
  p.n = n;
  p.e_out = e_out_dev;
  p.g_out = grad_out_dev;
  hipError_t e = dmip::launch_surrogate_eval(p, grad_out_dev ? 2 : 1, surrogate_n_wg(n, (hipStream_t)stream), (hipStream_t)stream);
  return e == hipSuccess ? DMIP_OK : hip_fail(e, "log_posterior launch");
}

int dmip_mh_sample(const dmip_surrogate* s, const dmip_scat_noise* noise, const float* y_dev, int n_y,
                   int64_t n_chains, int64_t chain_offset, int num_steps, float noise_std, uint64_t seed,
                   const float* x_init_dev, const float* noise_dev, const float* unif_dev, float* x_out_dev,
                   float* e_out_dev, void* stream) {
  if (int rc = surrogate_check(s, n_chains)) return rc;
  dmip::SurrogateParams p{};
  if (int rc = noise_check(noise, p)) return rc;
  if (!y_dev || !x_out_dev) return fail(DMIP_ERR_INVALID, "null argument");
  if (n_y < 1 || n_y > 65535) return fail(DMIP_ERR_INVALID, "n_y must be in [1, 65535]");
  if (chain_offset < 0) return fail(DMIP_ERR_INVALID, "negative chain offset");
  if (num_steps < 0) return fail(DMIP_ERR_INVALID, "num_steps must be >= 0");
  if (!(noise_std >= 0.0f)) return fail(DMIP_ERR_INVALID, "noise_std must be >= 0");
  if ((noise_dev == nullptr) != (unif_dev == nullptr))
    return fail(DMIP_ERR_INVALID, "inject both the proposal normals and the uniforms, or neither");
  if (n_chains == 0) return DMIP_OK;
  surrogate_params(s, p);
  p.y = y_dev;
  p.n_chains = n_chains;
  p.chain_offset = chain_offset;
  p.num_steps = num_steps;
  p.noise_std = noise_std;
  p.seed = seed;
  p.x_init = x_init_dev;
  p.noise = noise_dev;
  p.unif = unif_dev;
  p.x_out = x_out_dev;
  p.e_out = e_out_dev;
  hipError_t e = dmip::launch_mh(p, n_y, (hipStream_t)stream);
  return e == hipSuccess ? DMIP_OK : hip_fail(e, "mh_sample launch");
}

int dmip_mh_sample_ex(const dmip_surrogate* s, const dmip_scat_noise* noise, const float* y_dev, int n_y,
                      int64_t n_chains, int64_t chain_offset, int num_steps, float noise_std, uint64_t seed,
                      const float* x_init_dev, const float* noise_dev, const float* unif_dev, int precision,
                      float* x_out_dev, float* e_out_dev, void* stream) {
  if (precision == DMIP_PREC_F32)
    return dmip_mh_sample(s, noise, y_dev, n_y, n_chains, chain_offset, num_steps, noise_std, seed, x_init_dev,
                          noise_dev, unif_dev, x_out_dev, e_out_dev, stream);
  if (precision != DMIP_PREC_F32X3) return fail(DMIP_ERR_INVALID, "MH precision: DMIP_PREC_F32 or DMIP_PREC_F32X3");
  if (int rc = surrogate_check(s, n_chains)) return rc;
  dmip::SurrogateParams sp{};
  if (int rc = noise_check(noise, sp)) return rc;
  if (!y_dev || !x_out_dev) return fail(DMIP_ERR_INVALID, "null argument");
  if (n_y < 1 || n_y > 65535) return fail(DMIP_ERR_INVALID, "n_y must be in [1, 65535]");
  if (chain_offset < 0) return fail(DMIP_ERR_INVALID, "negative chain offset");
  if (num_steps < 0) return fail(DMIP_ERR_INVALID, "num_steps must be >= 0");
  if (!(noise_std >= 0.0f)) return fail(DMIP_ERR_INVALID, "noise_std must be >= 0");
  if (noise_dev || unif_dev) return fail(DMIP_ERR_UNSUPPORTED, "fp32x3 MH: injected draws need DMIP_PREC_F32");
  if (!s->x3_img)
    return fail(DMIP_ERR_UNSUPPORTED, "fp32x3 MH: a weight is outside the fp16 range of the split engine (largest |w| " +
                                          std::to_string(s->x3_range) + " > 65504); use DMIP_PREC_F32");
  if (n_chains == 0) return DMIP_OK;
  hipStream_t st = (hipStream_t)stream;
  dmip::MhX3Params p{};
  p.simg = s->x3_img;
  p.sl1 = s->x3_l1;
  p.sbias = s->x3_bias;
  p.y = y_dev;
  p.n_chains = n_chains;
  p.chain_offset = chain_offset;
  p.num_steps = num_steps;
  p.noise_std = noise_std;
  p.a = sp.a;
  p.b2 = sp.b2;
  p.lam = sp.lam;
  p.seed = seed;
  p.x_init = x_init_dev;
  p.x_out = x_out_dev;
  p.e_out = e_out_dev;
  p.err = status_word(dmip::stream_device(st));
  if (!p.err) return fail(DMIP_ERR_ALLOC, "device status word");
  hipError_t e = dmip::launch_mh_x3(p, n_y, st);
  return e == hipSuccess ? DMIP_OK : hip_fail(e, "mh_sample (fp32x3) launch");
}

int dmip_dps_sample(const dmip_mlp* prior, const dmip_surrogate* fwd, const dmip_scat_noise* noise,
                    const dmip_vpsde* sde, const float* y_dev, int n_y, int64_t n_chains, int64_t chain_offset,
                    int num_steps, float mean, float stdv, uint64_t seed, int mode, float zeta, float* x_out_dev,
                    void* stream) {
  if (!prior || !fwd || !sde || !y_dev || !x_out_dev) return fail(DMIP_ERR_INVALID, "null argument");
  if (mode != DMIP_DPS_NLL && mode != DMIP_DPS_NORM) return fail(DMIP_ERR_INVALID, "unknown DPS guidance mode");
  if (f32_act(prior)) return act_refused("dps_sample");
  dmip::DpsParams p{};
  if (mode == DMIP_DPS_NLL) {
    if (int rc = noise_check(noise, p.s)) return rc;
  }
  if (!prior->dps_l1)
    return fail(DMIP_ERR_UNSUPPORTED, "DPS prior must be an x,t network (MLP2) with xdim 3 and hidden layers [256]*3");
  if (n_y < 1 || n_y > 65535) return fail(DMIP_ERR_INVALID, "n_y must be in [1, 65535]");
  if (n_chains < 0 || chain_offset < 0) return fail(DMIP_ERR_INVALID, "negative chain count/offset");
  if (num_steps < 1) return fail(DMIP_ERR_INVALID, "num_steps must be >= 1");
  if (!(sde->T > 0.0)) return fail(DMIP_ERR_INVALID, "T must be > 0");
  if (!(zeta >= 0.0f)) return fail(DMIP_ERR_INVALID, "zeta must be >= 0");
  if (n_chains == 0) return DMIP_OK;
  surrogate_params(fwd, p.s);
  p.mode = mode;
  p.s.y = y_dev;
  p.s.n_chains = n_chains;
  p.s.chain_offset = chain_offset;
  p.s.num_steps = num_steps;
  p.s.seed = seed;
  p.s.x_out = x_out_dev;
  p.pl1 = prior->dps_l1;
  p.pw2 = prior->dps_w2;
  p.pw3 = prior->dps_w3;
  p.pw4 = prior->dps_w4;
  p.pbias = prior->dps_bias;
  p.T = (float)sde->T;
  p.bmin = (float)sde->beta_min;
  p.bdiff = (float)(sde->beta_max - sde->beta_min);
  p.delta = (float)(sde->T / (double)num_steps);
  p.sqrt_delta = (float)std::sqrt(sde->T / (double)num_steps);
  p.mean = mean;
  p.stdv = stdv;
  p.zeta = zeta;
  hipError_t e = dmip::launch_dps(p, n_y, (hipStream_t)stream);
  return e == hipSuccess ? DMIP_OK : hip_fail(e, "dps_sample launch");
}

int dmip_dps_sample_ex(const dmip_mlp* prior, const dmip_surrogate* fwd, const dmip_scat_noise* noise,
                       const dmip_vpsde* sde, const float* y_dev, int n_y, int64_t n_chains, int64_t chain_offset,
                       int num_steps, float mean, float stdv, uint64_t seed, int mode, float zeta, int precision,
                       float* x_out_dev, void* stream) {
  if (precision == DMIP_PREC_F32)
    return dmip_dps_sample(prior, fwd, noise, sde, y_dev, n_y, n_chains, chain_offset, num_steps, mean, stdv, seed,
                           mode, zeta, x_out_dev, stream);
  if (precision != DMIP_PREC_F32X3) return fail(DMIP_ERR_INVALID, "DPS precision: DMIP_PREC_F32 or DMIP_PREC_F32X3");
  if (!prior || !fwd || !sde || !y_dev || !x_out_dev) return fail(DMIP_ERR_INVALID, "null argument");
  if (f32_act(prior)) return act_refused("dps_sample_ex");
  if (mode != DMIP_DPS_NLL && mode != DMIP_DPS_NORM) return fail(DMIP_ERR_INVALID, "unknown DPS guidance mode");
  dmip::DpsX3Params p{};
  if (mode == DMIP_DPS_NLL) {
    dmip::SurrogateParams sp{};
    if (int rc = noise_check(noise, sp)) return rc;
    p.a = sp.a;
    p.b2 = sp.b2;
  }
  if (!prior->dps_l1)
    return fail(DMIP_ERR_UNSUPPORTED, "DPS prior must be an x,t network (MLP2) with xdim 3 and hidden layers [256]*3");
  if (!prior->dps_x3_img || !fwd->x3_img)
    return fail(DMIP_ERR_UNSUPPORTED, "fp32x3 DPS: a weight is outside the fp16 range of the split engine (largest |w| " +
                                          std::to_string(std::max(prior->dps_x3_range, fwd->x3_range)) +
                                          " > 65504); use DMIP_PREC_F32");
  if (n_y < 1 || n_y > 65535) return fail(DMIP_ERR_INVALID, "n_y must be in [1, 65535]");
  if (n_chains < 0 || chain_offset < 0) return fail(DMIP_ERR_INVALID, "negative chain count/offset");
  if (num_steps < 1) return fail(DMIP_ERR_INVALID, "num_steps must be >= 1");
  if (!(sde->T > 0.0)) return fail(DMIP_ERR_INVALID, "T must be > 0");
  if (!(zeta >= 0.0f)) return fail(DMIP_ERR_INVALID, "zeta must be >= 0");
  if (n_chains == 0) return DMIP_OK;
  hipStream_t st = (hipStream_t)stream;
  p.pimg = prior->dps_x3_img;
  p.simg = fwd->x3_img;
  p.pl1 = prior->dps_x3_l1;
  p.sl1 = fwd->x3_l1;
  p.pbias = prior->dps_x3_bias;
  p.sbias = fwd->x3_bias;
  p.y = y_dev;
  p.n_chains = n_chains;
  p.chain_offset = chain_offset;
  p.num_steps = num_steps;
  p.T = (float)sde->T;
  p.bmin = (float)sde->beta_min;
  p.bdiff = (float)(sde->beta_max - sde->beta_min);
  p.delta = (float)(sde->T / (double)num_steps);
  p.sqrt_delta = (float)std::sqrt(sde->T / (double)num_steps);
  p.mean = mean;
  p.stdv = stdv;
  p.zeta = zeta;
  p.mode = mode;
  p.seed = seed;
  p.x_out = x_out_dev;
  p.err = status_word(dmip::stream_device(st));
  if (!p.err) return fail(DMIP_ERR_ALLOC, "device status word");
  hipError_t e = dmip::launch_dps_x3(p, n_y, st);
  return e == hipSuccess ? DMIP_OK : hip_fail(e, "dps_sample (fp32x3) launch");
}

}  // extern "C"

// ---- A18: PosteriorLoss value + parameter gradients (GEMM-composed exact-f32 step, dmip_gemm.hip)
namespace {

struct MlpDims {
  int L;                      // hidden layers; linear layers 0..L
  std::vector<int> in, out;   // per linear layer
};

// one network's forward over the batch: layer inputs [B][in+1] (ones column last), hidden outputs
// with their activation derivatives, output [B][out]
struct MlpTape {
  std::vector<float*> h;      // h[l]: input matrix of layer l, [B][in_l + 1]; h[0] is the caller's
  std::vector<float*> d;      // d[l]: act'(z_l) of hidden layer l, [B][out_l]
  float* out = nullptr;       // [B][out_L]
};

hipError_t mlp_forward_f32(const MlpDims& dm, const float* const* W, const float* const* b, MlpTape& tp, int64_t B,
                           hipStream_t st) {
  for (int l = 0; l <= dm.L; ++l) {
    dmip::GemmParams g{};
    g.a = tp.h[l];
    g.lda = dm.in[l] + 1;
    g.b = W[l];
    g.ldb = dm.in[l];
    g.m = B;
    g.n = dm.out[l];
    g.k = dm.in[l];
    g.bias = b[l];
    if (l < dm.L) {
      g.c = tp.h[l + 1];
      g.ldc = dm.out[l] + 1;
      g.epi = l == 0 ? dmip::GEMM_EPI_BIAS_TANH2 : dmip::GEMM_EPI_BIAS_TANH;
      g.aux_out = tp.d[l];
      g.ldaux = dm.out[l];
    } else {
      g.c = tp.out;
      g.ldc = dm.out[l];
      g.epi = dmip::GEMM_EPI_BIAS;
    }
    hipError_t e = dmip::launch_gemm_f32(g, false, true, 1, st);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// reverse pass from the output adjoint `adj` [B][out_L]: with grads != null, [dW_l | db_l] into the
// flat reference-order gradient buffer; with in_grad != null, d/d(input) [B][in_0] (no parameter grads)
hipError_t mlp_backward_f32(const MlpDims& dm, const float* const* W, const MlpTape& tp, const float* adj, int64_t B,
                            float* delta_a, float* delta_b, float* grads, float* in_grad, float* part, int splits,
                            hipStream_t st) {
  std::vector<size_t> off(dm.L + 2, 0);
  for (int l = 0; l <= dm.L; ++l) off[l + 1] = off[l] + (size_t)dm.out[l] * dm.in[l] + dm.out[l];
  const float* dl = adj;  // adjoint of layer l's output, [B][out_l]
  float* bufs[2] = {delta_a, delta_b};
  for (int l = dm.L; l >= 0; --l) {
    hipError_t e;
    if (grads) {
      dmip::GemmParams g{};
      g.a = dl;
      g.lda = dm.out[l];
      g.b = tp.h[l];
      g.ldb = dm.in[l] + 1;
      g.m = dm.out[l];
      g.n = dm.in[l] + 1;
      g.k = B;
      g.c = grads + off[l];
      g.ldc = dm.in[l];
      g.epi = dmip::GEMM_EPI_WGRAD;
      g.bias_out = grads + off[l] + (size_t)dm.out[l] * dm.in[l];
      g.part = part;
      if ((e = dmip::launch_gemm_f32(g, true, false, dmip::gemm_wgrad_splits(g.m, g.n, g.k, splits), st)) != hipSuccess)
        return e;
    }
    if (l == 0 && !in_grad) break;
    dmip::GemmParams g{};
    g.a = dl;
    g.lda = dm.out[l];
    g.b = W[l];
    g.ldb = dm.in[l];
    g.m = B;
    g.n = dm.in[l];
    g.k = dm.out[l];
    if (l > 0) {
      float* nxt = bufs[l & 1];
      g.c = nxt;
      g.ldc = dm.in[l];
      g.epi = dmip::GEMM_EPI_MUL_AUX;
      g.aux_in = tp.d[l - 1];
      g.ldaux = dm.in[l];
      if ((e = dmip::launch_gemm_f32(g, false, false, 1, st)) != hipSuccess) return e;
      dl = nxt;
    } else {
      g.c = in_grad;
      g.ldc = dm.in[0];
      g.epi = dmip::GEMM_EPI_NONE;
      if ((e = dmip::launch_gemm_f32(g, false, false, 1, st)) != hipSuccess) return e;
    }
  }
  return hipSuccess;
}

}  // namespace

extern "C" {

int dmip_posterior_loss_grad(int xdim, int ydim, int n_hidden, const int* widths, const float* const* prior_w,
                             const float* const* prior_b, const float* const* lik_w, const float* const* lik_b,
                             const dmip_surrogate* fwd, const dmip_scat_noise* noise, float lam, const dmip_vpsde* sde,
                             const float* x_dev, const float* y_dev, const float* t_dev, const float* eps_dev,
                             int64_t batch, float* grad_prior_dev, float* grad_lik_dev, float* loss_out_dev,
                             float* target_out_dev, void* stream) {
  if (!widths || !prior_w || !prior_b || !lik_w || !lik_b || !fwd || !noise || !sde || !x_dev || !y_dev || !t_dev ||
      !eps_dev || !grad_prior_dev || !grad_lik_dev || !loss_out_dev)
    return fail(DMIP_ERR_INVALID, "null argument");
  if (xdim != dmip::kSurXdim || ydim != dmip::kSurYdim)
    return fail(DMIP_ERR_UNSUPPORTED, "PosteriorLoss: the scatterometry surrogate's shapes (xdim 3, ydim 23)");
  if (n_hidden < 1 || n_hidden > 8) return fail(DMIP_ERR_UNSUPPORTED, "n_hidden must be in [1, 8]");
  for (int i = 0; i < n_hidden; ++i)
    if (widths[i] < 1 || widths[i] > 4096) return fail(DMIP_ERR_INVALID, "hidden widths must be in [1, 4096]");
  for (int i = 0; i <= n_hidden; ++i)
    if (!prior_w[i] || !prior_b[i] || !lik_w[i] || !lik_b[i]) return fail(DMIP_ERR_INVALID, "null layer pointer");
  if (batch < 1) return fail(DMIP_ERR_INVALID, "batch must be >= 1");
  if (!(noise->b > 0.0f) || !(noise->a >= 0.0f)) return fail(DMIP_ERR_INVALID, "noise model needs b > 0, a >= 0");
  if (!(sde->beta_min > 0.0)) return fail(DMIP_ERR_INVALID, "beta_min must be > 0");
  hipStream_t st = (hipStream_t)stream;
  const int64_t B = batch;
  MlpDims dp, dl;  // prior MLP2 (x, t) and likelihood MLP (x, y, t)
  dp.L = dl.L = n_hidden;
  for (int l = 0; l <= n_hidden; ++l) {
    const int in_w = l == 0 ? 0 : widths[l - 1], out_w = l == n_hidden ? xdim : widths[l];
    dp.in.push_back(l == 0 ? xdim + 1 : in_w);
    dl.in.push_back(l == 0 ? xdim + ydim + 1 : in_w);
    dp.out.push_back(out_w);
    dl.out.push_back(out_w);
  }
  int wmax = xdim + ydim + 2;
  for (int i = 0; i < n_hidden; ++i) wmax = std::max(wmax, widths[i] + 1);
  const int splits = 64;  // the cap of every weight-gradient GEMM's own split count (gemm_wgrad_splits)
  // scratch (one allocation, carved in 256-byte aligned pieces)
  std::vector<std::pair<float**, size_t>> plan;
  auto need = [&](float** p, size_t n) { plan.emplace_back(p, n); };
  MlpTape tp, tl;
  tp.h.assign(n_hidden + 1, nullptr);
  tl.h.assign(n_hidden + 1, nullptr);
  tp.d.assign(n_hidden, nullptr);
  tl.d.assign(n_hidden, nullptr);
  for (int l = 0; l <= n_hidden; ++l) {
    need(&tp.h[l], (size_t)B * (dp.in[l] + 1));
    need(&tl.h[l], (size_t)B * (dl.in[l] + 1));
  }
  for (int l = 0; l < n_hidden; ++l) {
    need(&tp.d[l], (size_t)B * widths[l]);
    need(&tl.d[l], (size_t)B * widths[l]);
  }
  float *sp = nullptr, *sl = nullptr, *alpha = nullptr, *stdv = nullptr, *xt = nullptr, *x0 = nullptr, *u = nullptr,
        *jtu = nullptr, *tgt = nullptr, *ap = nullptr, *al = nullptr, *rows = nullptr, *da = nullptr, *db = nullptr,
        *part = nullptr;
  need(&sp, (size_t)B * xdim);
  need(&sl, (size_t)B * xdim);
  need(&alpha, B);
  need(&stdv, B);
  need(&xt, (size_t)B * xdim);
  need(&x0, (size_t)B * xdim);
  need(&u, (size_t)B * xdim);
  need(&jtu, (size_t)B * (xdim + 1));
  need(&tgt, (size_t)B * xdim);
  need(&ap, (size_t)B * xdim);
  need(&al, (size_t)B * xdim);
  need(&rows, (size_t)B * 2);
  need(&da, (size_t)B * wmax);
  need(&db, (size_t)B * wmax);
  need(&part, (size_t)splits * (size_t)wmax * (size_t)wmax);
  size_t total = 0;
  for (auto& q : plan) total += (q.second * sizeof(float) + 255) / 256 * 256;
  char* scratch = nullptr;
  hipError_t e = hipMallocAsync((void**)&scratch, total, st);
  if (e != hipSuccess) return fail(DMIP_ERR_ALLOC, std::string("hipMallocAsync: ") + hipGetErrorString(e));
  {
    size_t o = 0;
    for (auto& q : plan) {
      *q.first = (float*)(scratch + o);
      o += (q.second * sizeof(float) + 255) / 256 * 256;
    }
  }
  tp.out = sp;
  tl.out = sl;
  dmip::PosteriorParams pp{};
  pp.batch = B;
  pp.xdim = xdim;
  pp.ydim = ydim;
  pp.bmin = (float)sde->beta_min;
  pp.bdiff = (float)(sde->beta_max - sde->beta_min);
  pp.lam = lam;
  pp.x = x_dev;
  pp.y = y_dev;
  pp.t = t_dev;
  pp.eps = eps_dev;
  pp.alpha = alpha;
  pp.stdv = stdv;
  pp.x_t = xt;
  pp.prior_in = tp.h[0];
  pp.lik_in = tl.h[0];
  pp.s_prior = sp;
  pp.s_lik = sl;
  pp.x0 = x0;
  pp.u = u;
  pp.jtu = jtu;
  pp.target = target_out_dev ? target_out_dev : tgt;
  pp.adj_prior = ap;
  pp.adj_lik = al;
  pp.rows = rows;
  pp.loss_out = loss_out_dev;
  dmip::SurrogateParams sq{};
  surrogate_params(fwd, sq);
  sq.a = noise->a;
  sq.b2 = (float)((double)noise->b * (double)noise->b);
  sq.x = x0;
  sq.y = y_dev;
  sq.y_stride = ydim;
  sq.n = B;
  sq.g_out = u;
  auto run = [&]() -> hipError_t {
    hipError_t r;
    for (int l = 1; l <= n_hidden; ++l) {
      if ((r = dmip::launch_ones_column(tp.h[l], B, dp.in[l] + 1, st)) != hipSuccess) return r;
      if ((r = dmip::launch_ones_column(tl.h[l], B, dl.in[l] + 1, st)) != hipSuccess) return r;
    }
    if ((r = dmip::launch_posterior_stage(pp, 0, st)) != hipSuccess) return r;  // x_t, network inputs
    if ((r = mlp_forward_f32(dp, prior_w, prior_b, tp, B, st)) != hipSuccess) return r;
    if ((r = mlp_forward_f32(dl, lik_w, lik_b, tl, B, st)) != hipSuccess) return r;
    if ((r = dmip::launch_posterior_stage(pp, 1, st)) != hipSuccess) return r;  // Tweedie x0
    if ((r = dmip::launch_surrogate_eval(sq, 3, surrogate_n_wg(B, st), st)) != hipSuccess) return r;  // u = J_F^T v
    // J_s^T u: the prior's reverse pass to its input, no parameter gradients
    if ((r = mlp_backward_f32(dp, prior_w, tp, u, B, da, db, nullptr, jtu, part, splits, st)) != hipSuccess) return r;
    if ((r = dmip::launch_posterior_stage(pp, 2, st)) != hipSuccess) return r;  // target, adjoints, rows
    if ((r = mlp_backward_f32(dp, prior_w, tp, ap, B, da, db, grad_prior_dev, nullptr, part, splits, st)) != hipSuccess)
      return r;
    if ((r = mlp_backward_f32(dl, lik_w, tl, al, B, da, db, grad_lik_dev, nullptr, part, splits, st)) != hipSuccess)
      return r;
    return dmip::launch_posterior_stage(pp, 3, st);  // loss reduction
  };
  e = run();
  (void)hipFreeAsync(scratch, st);
  if (e != hipSuccess) return hip_fail(e, "posterior_loss_grad launch");
  return DMIP_OK;
}

}  // extern "C"

extern "C" {

int dmip_rng_words(uint64_t seed, int64_t chain_offset, uint64_t stream_id, int64_t n_chains, int n_words,
                   uint32_t* out_dev, void* stream) {
  if (!out_dev || n_chains < 0 || n_words < 0) return fail(DMIP_ERR_INVALID, "bad argument");
  if (n_chains == 0 || n_words == 0) return DMIP_OK;
  hipError_t e = dmip::launch_rng_words(seed, chain_offset, stream_id, n_chains, n_words, out_dev, (hipStream_t)stream);
  return e == hipSuccess ? DMIP_OK : hip_fail(e, "rng_words launch");
}

int dmip_rng_normals(uint64_t seed, int64_t chain_offset, uint64_t stream_id, int64_t n_chains, int n_pairs,
                     float* out_dev, void* stream) {
  if (!out_dev || n_chains < 0 || n_pairs < 0) return fail(DMIP_ERR_INVALID, "bad argument");
  if (n_chains == 0 || n_pairs == 0) return DMIP_OK;
  hipError_t e = dmip::launch_rng_normals(seed, chain_offset, stream_id, n_chains, n_pairs, out_dev, (hipStream_t)stream);
  return e == hipSuccess ? DMIP_OK : hip_fail(e, "rng_normals launch");
}

int dmip_schedule(int num_steps, const dmip_vpsde* sde, float* out_dev, void* stream) {
  if (!out_dev || !sde || num_steps < 1) return fail(DMIP_ERR_INVALID, "bad argument");
  hipError_t e = dmip::launch_schedule(num_steps, (float)sde->T, (float)sde->beta_min,
                                       (float)(sde->beta_max - sde->beta_min), out_dev, (hipStream_t)stream);
  return e == hipSuccess ? DMIP_OK : hip_fail(e, "schedule launch");
}

}  // extern "C"
