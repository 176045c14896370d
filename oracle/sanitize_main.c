/* sanitize_main.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Drives every entry point of the oracle restatement (fmskf_oracle.c) on small random and
 * adversarial inputs inside one executable built with -fsanitize=address,undefined
 * -fno-sanitize-recover=all (oracle/Makefile `sanitize`), so any out-of-bounds access,
 * use of uninitialised layout, misaligned access or integer UB in the checker itself ends
 * the run (run the CPU path under the sanitizers).  tests/test_oracle_sanitize.py
 * builds and runs it.  Inputs: garbage WT901 byte streams (random bytes, truncated and
 * corrupted frames), CAN frames with every angle / rpm / stamp extreme, KF / EKF / KF12D
 * ticks with NaN and huge inputs and validity masks, the control step with random power and
 * targets, the ensemble fold, the VehicleInfo fill. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fmskf_oracle.h"

static uint64_t rng_s = 0x464D534Bull;
static uint32_t rnd(void) {
  rng_s ^= rng_s << 13;
  rng_s ^= rng_s >> 7;
  rng_s ^= rng_s << 17;
  return (uint32_t)(rng_s >> 16);
}
static float rndf(float lo, float hi) { return lo + (hi - lo) * (float)(rnd() & 0xFFFFFF) / 16777216.0f; }

static void *xmalloc(size_t b) {
  void *p = malloc(b ? b : 1);
  if (!p) abort();
  memset(p, 0, b ? b : 1);
  return p;
}

static void wt901_frame(uint8_t *o, uint8_t type, int16_t w0, int16_t w1, int16_t w2, int16_t w3) {
  const int16_t w[4] = {w0, w1, w2, w3};
  o[0] = 0x55;
  o[1] = type;
  for (int k = 0; k < 4; k++) {
    o[2 + 2 * k] = (uint8_t)((uint16_t)w[k] & 0xFF);
    o[3 + 2 * k] = (uint8_t)((uint16_t)w[k] >> 8);
  }
  uint8_t s = 0;
  for (int k = 0; k < 10; k++) s = (uint8_t)(s + o[k]);
  o[10] = s;
}

static void check_wt901(void) {
  const size_t n = 37;
  const uint32_t stride = 96;
  orc_wt901 *s = xmalloc(n * sizeof(orc_wt901));
  uint8_t *bytes = xmalloc(n * stride);
  uint32_t *len = xmalloc(n * sizeof(uint32_t));
  for (size_t i = 0; i < n; i++) orc_wt901_reset(&s[i], (uint32_t)(rnd() % ORC_WT901_NREG));
  for (int poll = 0; poll < 60; poll++) {
    for (size_t i = 0; i < n; i++) {
      uint8_t *b = bytes + i * stride;
      uint32_t L = 0;
      const int kind = (int)(rnd() % 4);
      if (kind == 0) {  /* random bytes */
        L = rnd() % stride;
        for (uint32_t k = 0; k < L; k++) b[k] = (uint8_t)rnd();
      } else {          /* frames, some corrupted or truncated */
        const uint8_t types[] = {0x50, 0x51, 0x52, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5A, 0x5F};
        while (L + 11 <= stride && rnd() % 8) {
          wt901_frame(b + L, types[rnd() % 12], (int16_t)rnd(), (int16_t)rnd(), (int16_t)rnd(), (int16_t)rnd());
          if (kind == 2 && rnd() % 3 == 0) b[L + rnd() % 11] ^= (uint8_t)(1u << (rnd() % 8));
          L += 11;
        }
        if (kind == 3 && L > 3) L -= rnd() % 4;
      }
      len[i] = L;
    }
    orc_wt901_update_batch(n, s, bytes, stride, len, poll == 0);
  }
  for (size_t i = 0; i < n; i++) {  /* the byte-level entry points directly */
    for (int k = 0; k < 300; k++) orc_wt901_byte(&s[i], (uint8_t)rnd());
    (void)orc_wt901_is_com_comp(&s[i], bytes, 0);
    orc_wt901_update_data(&s[i]);
  }
  free(s);
  free(bytes);
  free(len);
}

static void check_can_rs(void) {
  const size_t n = 53;
  orc_m2006 *m = xmalloc(n * 4 * sizeof(orc_m2006));
  uint8_t *fr = xmalloc(n * 32);
  int16_t *st = xmalloc(n * 4 * sizeof(int16_t));
  uint8_t *present = xmalloc(n);
  for (size_t i = 0; i < n; i++)
    for (int w = 0; w < 4; w++) orc_m2006_reset(&m[i * 4 + w], w < 2 ? 1 : -1);
  float *pos = xmalloc(3 * n * 4), *vel = xmalloc(3 * n * 4), *yaw = xmalloc(n * 4);
  int64_t *prev = xmalloc(4 * n * 8), *sum = xmalloc(4 * n * 8);
  int16_t *rpm = xmalloc(n * 4 * 2);
  for (int t = 0; t < 200; t++) {
    for (size_t k = 0; k < n * 32; k++) fr[k] = (uint8_t)rnd();
    for (size_t k = 0; k < n * 4; k++) {
      const uint32_t r = rnd() % 5;  /* extremes: equal stamps, 0x7FFF wrap, INT16 limits */
      st[k] = r == 0 ? (int16_t)0 : r == 1 ? (int16_t)0x7FFF : r == 2 ? (int16_t)-32768 : (int16_t)rnd();
    }
    for (size_t i = 0; i < n; i++) present[i] = (uint8_t)rnd();
    orc_can_ingest_batch(n, m, fr, st, t % 3 ? present : NULL);
    for (size_t i = 0; i < n; i++) {
      yaw[i] = (t % 17 == 0) ? NAN : rndf(-180.f, 180.f);
      for (int w = 0; w < 4; w++) {
        sum[w * n + i] = m[i * 4 + w].angle_sum;
        rpm[i * 4 + w] = m[i * 4 + w].rpm;
      }
    }
    orc_rs_tick(n, pos, vel, prev, yaw, sum, rpm, t & 1, 1, 1);
  }
  free(m); free(fr); free(st); free(present); free(pos); free(vel); free(yaw); free(prev);
  free(sum); free(rpm);
}

static void check_kf(void) {
  const size_t n = 41;
  float *x6 = xmalloc(6 * n * 4), *P6 = xmalloc(21 * n * 4), *yaw = xmalloc(n * 4), *gz = xmalloc(n * 4);
  int16_t *rpm = xmalloc(n * 8);
  uint8_t *valid = xmalloc(n);
  float *z = xmalloc(6 * n * 4);
  orc_kf6_params p6;
  memset(&p6, 0, sizeof(p6));
  p6.dt = 1e-3f;
  p6.dt2 = p6.dt * p6.dt;
  for (int k = 0; k < 6; k++) p6.q[k * (k + 1) / 2 + k] = 1e-4f;
  for (int k = 0; k < 4; k++) p6.r[k * (k + 1) / 2 + k] = 1e-2f;
  for (size_t i = 0; i < n; i++)
    for (int k = 0; k < 6; k++) P6[(k * (k + 1) / 2 + k) * n + i] = 1.0f;
  for (int t = 0; t < 100; t++) {
    for (size_t i = 0; i < n; i++) {
      yaw[i] = (t == 50 && i == 3) ? NAN : rndf(-180.f, 180.f);
      gz[i] = (t == 60 && i == 4) ? 1e30f : rndf(-2000.f, 2000.f);
      for (int w = 0; w < 4; w++) rpm[i * 4 + w] = (int16_t)rnd();
      valid[i] = (uint8_t)(rnd() % 3 != 0);
    }
    orc_kf6_tick(n, x6, P6, yaw, gz, rpm, t & 1 ? valid : NULL, &p6, 1, 1, 1);
    p6.trig = t & 1;
  }
  orc_kf6_measure(n, yaw, gz, rpm, z, 0);

  float *x9 = xmalloc(10 * n * 4), *P9 = xmalloc(45 * n * 4); /* row 9: the heading low part */
  int16_t *raw = xmalloc(n * 16);
  orc_ekf9_params p9;
  memset(&p9, 0, sizeof(p9));
  p9.dt = 1e-3f;
  p9.dt2 = p9.dt * p9.dt;
  for (int k = 0; k < 9; k++) p9.q[k * (k + 1) / 2 + k] = 1e-4f;
  for (int k = 0; k < 6; k++) p9.r[k * (k + 1) / 2 + k] = 1e-2f;
  for (size_t i = 0; i < n; i++)
    for (int k = 0; k < 9; k++) P9[(k * (k + 1) / 2 + k) * n + i] = 1.0f;
  for (int t = 0; t < 60; t++) {
    for (size_t k = 0; k < n * 8; k++) raw[k] = (int16_t)rnd();
    for (size_t i = 0; i < n; i++) valid[i] = (uint8_t)(rnd() & 1);
    orc_ekf9_tick(n, x9, P9, raw, valid, &p9, 1, 1, 1);
  }
  orc_ekf9_measure(n, raw, z);

  double *x12 = xmalloc(12 * n * 8), *P12 = xmalloc(78 * n * 8), *z12 = xmalloc(8 * n * 8);
  orc_kf12d_params p12;
  memset(&p12, 0, sizeof(p12));
  p12.dt = 1e-3;
  p12.dt2 = 1e-6;
  for (int k = 0; k < 12; k++) p12.q[k * (k + 1) / 2 + k] = 1e-6;
  for (int k = 0; k < 8; k++) p12.r[k * (k + 1) / 2 + k] = 1e-3;
  p12.r[5 * 6 / 2 + 4] = 2e-4;  /* a correlated pair (4, 5) */
  double ci[36];
  if (!orc_kf12d_cinv(p12.r, ci)) abort();
  double bad[36];
  memset(bad, 0, sizeof(bad));
  if (orc_kf12d_cinv(bad, ci)) abort();  /* not positive definite */
  for (size_t i = 0; i < n; i++)
    for (int k = 0; k < 12; k++) P12[(k * (k + 1) / 2 + k) * n + i] = 1.0;
  for (int t = 0; t < 40; t++) {
    for (size_t k = 0; k < 8 * n; k++) z12[k] = (double)rndf(-3.f, 3.f);
    for (size_t i = 0; i < n; i++) valid[i] = (uint8_t)(rnd() % 4 != 0);
    orc_kf12d_tick(n, x12, P12, z12, valid, &p12, 1, 1, 1);
  }

  /* ensemble: partial over sub-ranges, combine, finalize (empty ranges included) */
  const size_t L6 = orc_ens_record_len(6), L12 = orc_ens_record_len(12);
  double *ra = xmalloc(L12 * 8), *rb = xmalloc(L12 * 8), *rc = xmalloc(L12 * 8);
  double mean[12], cov[78];
  orc_ens_partial_f32(n, 6, x6, 0, 0, ra);
  orc_ens_partial_f32(n, 6, x6, 0, n / 2, rb);
  orc_ens_combine(6, ra, rb, rc);
  orc_ens_partial_f32(n, 6, x6, n / 2, n, ra);
  orc_ens_combine(6, rc, ra, rb);
  orc_ens_finalize(6, rb, mean, cov);
  orc_ens_partial_f64(n, 12, x12, 3, n, ra);
  orc_ens_finalize(12, ra, mean, cov);
  (void)L6;
  free(ra); free(rb); free(rc);
  free(x6); free(P6); free(yaw); free(gz); free(rpm); free(valid); free(z);
  free(x9); free(P9); free(raw); free(x12); free(P12); free(z12);
}

static void check_ctrl(void) {
  const size_t n = 29;
  orc_ctrl *c = xmalloc(n * sizeof(orc_ctrl));
  int16_t *rpm = xmalloc(n * 8);
  const int8_t dir[4] = {1, 1, -1, -1};
  orc_ctrl_params p;
  orc_ctrl_params_make(&p, 100.f, 0.0075f, 0.02f, 0.01f, 0.004f, 0.5f, 10.f, 1.f, 1.0f / 1000.f, 3000);
  for (size_t i = 0; i < n; i++) orc_ctrl_reset(&c[i]);
  for (int t = 0; t < 400; t++) {
    for (size_t i = 0; i < n; i++) {
      if (rnd() % 50 == 0) c[i].power = (uint8_t)(rnd() & 1);
      if (rnd() % 40 == 0)
        for (int a = 0; a < 3; a++)
          orc_interp_set(&c[i].ax[a], rndf(-400.f, 400.f), rndf(1.f, 2000.f), rndf(10.f, 30000.f));
      for (int w = 0; w < 4; w++) rpm[i * 4 + w] = (int16_t)rnd();
    }
    orc_ctrl_step_batch(n, c, &p, rpm, dir);
  }
  uint8_t out[8];
  for (size_t i = 0; i < n; i++) orc_can_tx(c[i].curr, out);
  /* every float -> int conversion on the path has the M7's defined semantics, so the
   * extremes (past 2^31 turns, inf, NaN) go straight in: UBSan's float-cast-overflow and
   * signed-overflow checks must stay silent */
  const float ext[] = {NAN, INFINITY, -INFINITY, 3e9f, -3e9f, 0.0f, -0.0f, 1e-40f, 2147483520.f,
                       1.5e10f, -1.5e10f, 1e20f, -1e20f, 3.4e38f, -3.4e38f};
  for (size_t k = 0; k < sizeof(ext) / sizeof(ext[0]); k++) {
    (void)orc_f2i32_arm(ext[k]);
    (void)orc_f2u32_arm(ext[k]);
    (void)orc_curr_to_raw(ext[k], -1, 3000);
    (void)orc_normalize_rad_0to2pi(ext[k]);
    (void)orc_normalize_deg_0to360(ext[k]);
    (void)orc_sin(ext[k], 0);
    (void)orc_cos(ext[k], 0);
  }
  orc_vehicle_info vi;
  float data[16];
  uint8_t floor_[8] = {1, 0, 1, 0, 1, 0, 1, 0};
  for (int k = 0; k < 16; k++) data[k] = rndf(-1.f, 1.f);
  orc_vehicle_info_fill(&vi, 1.5f, -2.5f, 0.3f, 120.f, -80.f, 0.1f, data, 0, floor_, 12.f, 7u);
  orc_vehicle_info_fill(&vi, NAN, 1e12f, 0.f, -1e12f, 0.f, 0.f, data, 1, floor_, 0.f, 0u);
  free(c);
  free(rpm);
}

int main(void) {
  check_wt901();
  check_can_rs();
  check_kf();
  check_ctrl();
  float tab[513];
  orc_sin_table(tab);
  printf("sanitize ok\n");
  return 0;
}
