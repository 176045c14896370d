// api_sanitize.cpp -- TEST INFRASTRUCTURE: the library's host code (csrc/api_*.cpp, built
// with -Xarch_host -fsanitize=address,undefined; device code unchanged) driven through the
// entry points that need no GPU: config / model / control-parameter defaults, the host
// ensemble fold, status strings, argument rejection, and fmskf_create failing cleanly without
// a device.  Built and run by tests/test_sanitizers.py (make -C roboken-fmskf-robot-controller_amd sanitize).
#include <cstdio>
#include <cstring>
#include <vector>
#include "fmskf.h"
int main() {
  fmskf_config cfg;
  for (uint32_t m = 0; m < 4; m++) {
    if (fmskf_config_init(&cfg, m, 1000) != FMSKF_OK) return 1;
    uint32_t n, mm, eb;
    if (fmskf_model_dims(m, &n, &mm, &eb) != FMSKF_OK) return 2;
  }
  if (fmskf_config_init(nullptr, 1, 1) != FMSKF_EINVAL) return 3;
  fmskf_ctrl_params p;
  if (fmskf_ctrl_params_init(&p) != FMSKF_OK) return 4;
  std::vector<double> recs(3 * 28, 0.0);
  for (int r = 0; r < 3; r++) { recs[r * 28] = 10.0 * (r + 1); for (int k = 1; k < 28; k++) recs[r * 28 + k] = 0.01 * k * (r + 1); }
  double mean[6], cov[21];
  if (fmskf_ensemble_combine(6, recs.data(), 3, mean, cov) != FMSKF_OK) return 5;
  (void)fmskf_ensemble_combine(6, recs.data(), 0, mean, cov);
  if (fmskf_ensemble_combine(6, nullptr, 3, mean, cov) == FMSKF_OK) return 6;
  for (int s = 0; s < 8; s++) (void)strlen(fmskf_strerror(s));
  fmskf_handle h = nullptr;
  int rc = fmskf_create(&cfg, &h);          // no GPU here: must fail cleanly
  std::printf("create rc=%d (%s) err=%s\n", rc, fmskf_strerror(rc), fmskf_last_error());
  if (rc == FMSKF_OK) fmskf_destroy(h);
  if (fmskf_tick(nullptr, nullptr) != FMSKF_EINVAL) return 7;
  // ABI 3: an ABI-2 caller, unknown flags, the reserved word and a COMP model mismatch are refused
  // before any device is touched
  fmskf_config c2;
  if (fmskf_config_init(&c2, FMSKF_MODEL_KF6, 100) != FMSKF_OK || c2.abi_version != 3u || c2.flags) return 8;
  c2.abi_version = 2u;
  if (fmskf_create(&c2, &h) != FMSKF_EINVAL) return 9;
  c2.abi_version = FMSKF_ABI_VERSION;
  c2.flags = 0x80u;
  if (fmskf_create(&c2, &h) != FMSKF_EINVAL) return 10;
  c2.flags = 0u;
  c2.reserved = 1u;
  if (fmskf_create(&c2, &h) != FMSKF_EINVAL) return 11;
  if (fmskf_config_init(&c2, FMSKF_MODEL_KF12D, 100) != FMSKF_OK) return 12;
  c2.flags = FMSKF_CFG_COMP_POS;
  if (fmskf_create(&c2, &h) != FMSKF_ENOTSUP) return 13;
  int w = 0, r = 0;
  if (fmskf_comm_info(nullptr, &w, &r) != FMSKF_EINVAL) return 14;
  if (fmskf_ensemble_end_count(nullptr, nullptr, nullptr, nullptr, nullptr) != FMSKF_EINVAL) return 15;
  if (fmskf_get_motor_status(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, FMSKF_MEM_HOST) !=
      FMSKF_EINVAL)
    return 16;
  uint32_t rows = 0;
  if (fmskf_get_state_lo(nullptr, nullptr, &rows, FMSKF_MEM_HOST) != FMSKF_EINVAL) return 17;
  // round 5: the fused CAN RX + ISR call refuses a null handle before anything else
  if (fmskf_isr_tick_can(nullptr, nullptr, nullptr, nullptr, nullptr, FMSKF_MEM_HOST) != FMSKF_EINVAL) return 18;
  float xms = 0.f;
  if (fmskf_ensemble_exchange_ms(nullptr, &xms) != FMSKF_EINVAL) return 19;
  (void)strlen(fmskf_rccl_library());
  std::printf("api sanitize ok\n");
  return 0;
}
