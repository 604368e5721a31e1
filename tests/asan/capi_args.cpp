// Host-side AddressSanitizer driver for libdmip's C-ABI (make asan; run by tests/test_asan.py).
// Exercises every entry point's argument validation with null / out-of-range / inconsistent
// arguments -- the paths that return before any device work -- plus the error-string plumbing, so
// ASan sees the validation code's reads of caller arrays (widths, weight tables) and the
// thread-local error buffer. Exits 0 when every call returned the documented status.
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>

#include "../../include/dmip.h"

static int failures = 0;

static void expect(int got, int want, const char* what) {
  if (got != want) {
    std::printf("FAIL %s: status %d, want %d (%s)\n", what, got, want, dmip_last_error());
    ++failures;
  }
}

int main() {
  expect(dmip_abi_version(), DMIP_ABI_VERSION, "abi version");
  const int w3[3] = {64, 64, 64}, wneq[3] = {64, 32, 64}, w1[1] = {96};
  const float* null4[4] = {nullptr, nullptr, nullptr, nullptr};
  dmip_mlp* net = nullptr;
  expect(dmip_mlp_create(5, 2, 3, w3, 0, 0, 2, null4, null4, &net), DMIP_ERR_INVALID, "create: null layers");
  expect(dmip_mlp_create(5, 2, 3, wneq, 0, 0, 2, null4, null4, &net), DMIP_ERR_UNSUPPORTED, "create: widths");
  expect(dmip_mlp_create(5, 2, 3, w3, 1, 0, 2, null4, null4, &net), DMIP_ERR_UNSUPPORTED, "create: act");
  expect(dmip_mlp_create(5, 40, 3, w3, 0, 0, 2, null4, null4, &net), DMIP_ERR_UNSUPPORTED, "create: out_dim");
  expect(dmip_mlp_create(5, 2, 0, w3, 0, 0, 2, null4, null4, &net), DMIP_ERR_INVALID, "create: n_hidden");
  expect(dmip_mlp_create(5, 2, 1, w1, 0, 7, 2, null4, null4, &net), DMIP_ERR_INVALID, "create: layout");
  expect(dmip_mlp_create(5, 2, 1, w1, 0, 1, 2, null4, null4, &net), DMIP_ERR_INVALID, "create: X_T in_dim");
  expect(dmip_mlp_create(5, 2, 3, nullptr, 0, 0, 2, null4, null4, &net), DMIP_ERR_INVALID, "create: null widths");
  if (net != nullptr) ++failures;
  dmip_vpsde sde{0.1, 20.0, 1.0};
  expect(dmip_mlp_forward(nullptr, nullptr, nullptr, 0, nullptr, 0, 4, nullptr, 0, nullptr), DMIP_ERR_INVALID,
         "forward: null");
  expect(dmip_em_sample(nullptr, &sde, nullptr, 1, 2, 2, 10, 0, 10, 0.f, 1.f, 1, 0, nullptr, nullptr, nullptr),
         DMIP_ERR_INVALID, "em_sample: null");
  expect(dmip_em_sample_posterior(nullptr, nullptr, &sde, nullptr, 1, 2, 2, 10, 0, 10, 0.f, 1.f, 1, 1, nullptr,
                                  nullptr),
         DMIP_ERR_INVALID, "posterior: null");
  expect(dmip_em_sample_cdiffe(nullptr, &sde, nullptr, 1, 2, 2, 10, 0, 10, 0.f, 1.f, 1, 0, -1, 0.16f, nullptr,
                               nullptr),
         DMIP_ERR_INVALID, "cdiffe: corrector steps");
  expect(dmip_em_sample_cdiffe(nullptr, &sde, nullptr, 1, 2, 2, 10, 0, 10, 0.f, 1.f, 1, 0, 1, 0.f, nullptr, nullptr),
         DMIP_ERR_INVALID, "cdiffe: snr");
  dmip_loss_cfg cfg{};
  expect(dmip_loss_grad(5, 2, 3, w3, 2, nullptr, nullptr, &sde, &cfg, nullptr, nullptr, nullptr, nullptr, 16, nullptr,
                        nullptr, nullptr),
         DMIP_ERR_INVALID, "loss_grad: null");
  expect(dmip_loss_grad_supported(5, 2, 3, w3, 2), 1, "loss_grad_supported");
  expect(dmip_loss_grad_supported(5, 2, 3, wneq, 2), 0, "loss_grad_supported widths");
  expect(dmip_histogram(nullptr, 10, 3, 75, -1.0, 1.0, 1, nullptr, nullptr), DMIP_ERR_INVALID, "histogram: null");
  dmip_surrogate* sur = nullptr;
  const int w256[3] = {256, 256, 256};
  expect(dmip_surrogate_create(3, 23, 3, w256, null4, null4, &sur), DMIP_ERR_INVALID, "surrogate: null layers");
  expect(dmip_surrogate_create(2, 23, 3, w256, null4, null4, &sur), DMIP_ERR_UNSUPPORTED, "surrogate: shape");
  dmip_scat_noise nz{0.2f, 0.01f, 1000.f};
  expect(dmip_log_posterior(nullptr, &nz, nullptr, nullptr, 0, 4, nullptr, nullptr, nullptr), DMIP_ERR_INVALID,
         "log_posterior: null");
  expect(dmip_mh_sample(nullptr, &nz, nullptr, 1, 10, 0, 5, 0.5f, 1, nullptr, nullptr, nullptr, nullptr, nullptr,
                        nullptr),
         DMIP_ERR_INVALID, "mh: null");
  expect(dmip_dps_sample(nullptr, nullptr, &nz, &sde, nullptr, 1, 10, 0, 5, 0.f, 1.f, 1, 0, 1.f, nullptr, nullptr),
         DMIP_ERR_INVALID, "dps: null");
  expect(dmip_rng_words(1, 0, 0, 10, 4, nullptr, nullptr), DMIP_ERR_INVALID, "rng_words: null");
  expect(dmip_schedule(0, &sde, nullptr, nullptr), DMIP_ERR_INVALID, "schedule: steps");
  expect(dmip_sampler_supported(0, 256, 3, 3, 23), 1, "supported bf16");
  expect(dmip_sampler_supported_f32(2, 512, 3, 3, 23), 1, "supported f32");
  expect(dmip_sampler_supported(2, 512, 3, 3, 23), 1, "supported bf16 CDiffE width 512");
  float dummy[4];
  expect(dmip_em_sample_snapshots(0, nullptr, nullptr, &sde, nullptr, 1, 2, 2, 10, 0, 10, 0.f, 1.f, 1, 0, 0, 0.16f,
                                  0, dummy, nullptr, nullptr),
         DMIP_ERR_INVALID, "snapshots: every");
  expect(dmip_em_sample_snapshots(0, nullptr, nullptr, &sde, nullptr, 1, 2, 2, 10, 0, 10, 0.f, 1.f, 1, 0, 0, 0.16f,
                                  2, nullptr, nullptr, nullptr),
         DMIP_ERR_INVALID, "snapshots: null buffer");
  dmip_train_plan* plan = nullptr;
  expect(dmip_train_plan_create(nullptr, &plan), DMIP_ERR_INVALID, "train_plan: null desc");
  dmip_train_plan_desc d{};
  expect(dmip_train_plan_create(&d, &plan), DMIP_ERR_INVALID, "train_plan: null pointers");
  expect(dmip_train_plan_step(nullptr, nullptr, nullptr, nullptr), DMIP_ERR_INVALID, "train_plan: null step");
  expect(dmip_train_plan_destroy(nullptr), DMIP_OK, "train_plan: destroy null");
  // the error buffer is thread-local: concurrent failures keep their own messages
  std::string a, b;
  std::thread t1([&] {
    dmip_schedule(0, &sde, nullptr, nullptr);
    a = dmip_last_error();
  });
  std::thread t2([&] {
    dmip_mlp_create(5, 2, 3, wneq, 0, 0, 2, null4, null4, &net);
    b = dmip_last_error();
  });
  t1.join();
  t2.join();
  if (a == b || a.empty() || b.empty()) {
    std::printf("FAIL thread-local errors: '%s' / '%s'\n", a.c_str(), b.c_str());
    ++failures;
  }
  std::printf("%s: %d failure(s)\n", failures ? "FAIL" : "ok", failures);
  return failures ? 1 : 0;
}
