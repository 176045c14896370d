/*
 * cpu_port.c -- the CPU baseline of bench.py (TEST INFRASTRUCTURE ONLY: timed as
 * `cpu_baseline`, never part of the product; tests/test_cpu_port.py holds it bit-exact to the
 * oracle).
 *
 * The oracle's orc_kf6_tick / orc_rs_tick (fmskf_oracle.c) check one robot at a time through
 * a generic n-state update with run-time sparsity tables.  That is the right shape for a
 * checker and the wrong one for a baseline: this file is the same two ticks specialised the
 * way a tuned CPU build would be -- the KF6's H rows, F pattern and sizes fixed at compile
 * time, every small loop unrolled, and the robots of a block run in SIMD lanes (`omp simd`:
 * AVX-512 with -march=x86-64-v4, AVX2 with v3), OpenMP threads over blocks.  The operation
 * order is the oracle's (and therefore the GPU's): explicit fmaf where the oracle has one,
 * every other operation rounded on its own (-ffp-contract=off), so the results are bitwise
 * the oracle's.  TABLE512 trig only (the CMSIS table through gathers; libm sinf / cosf have
 * no bitwise-equal vector form).
 *
 * Reference arithmetic restated (through the oracle): VD_vehicle_controller.cpp:11-51 (RS
 * tick), util_mymath.hpp:16-25 (deg2rad, normalize_rad_0to2pi), CMSIS arm_sin_f32 /
 * arm_cos_f32 (A13), and the KF6 of SURVEY.md 8(a) A15 (no reference counterpart).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "fmskf_oracle.h"

#define PI_F 3.14159265358979f
static const float k_deg2rad = PI_F / 180.0f;
static const float k_rpm_to_radps = 2.0f * 3.1415926f / 60.0f;
static const float k_gear_ratio_inv = 1.0f / 36.0f;
static const float k_out_rad_per_raw = 2.0f * 3.1415926f / 8191.0f;
static const float k_wheel_r = 37.5f;
static const float k_wheel_l = 13.08148f;
static const float k_sqrtf2 = 1.41421356f;

static const float g_tab[513] = {
#include "../roboken-fmskf-robot-controller_amd/csrc/cmsis_sintab.inc"
};

#define BLK 1024 /* robots per OpenMP work item */

/* Cortex-M7 VCVT.S32.F32 / VCVT.U32.F32 (orc_f2i32_arm / orc_f2u32_arm): truncate, saturate,
 * NaN -> 0, as selects on a clamped conversion (no branches, so the robot loop vectorises) */
static inline int32_t f2i32_arm(float f) {
  const float c = f < -2147483648.0f ? -2147483648.0f : f > 2147483520.0f ? 2147483520.0f : f;
  int32_t t = (int32_t)(c == c ? c : 0.0f);
  t = f >= 2147483648.0f ? INT32_MAX : t;
  return f != f ? 0 : t;
}
/* only the low 16 bits of VCVT.U32.F32 are used (UXTH): an index into the table */
static inline int32_t f2u16_arm(float f) {
  const float c = f > 0.0f ? (f < 65536.0f ? f : 65536.0f) : 0.0f;  /* NaN, negatives -> 0 */
  int32_t t = (int32_t)c;                                           /* 65536.0f -> 65536 */
  t = f >= 4294967296.0f ? 0xFFFF : t;  /* saturated UINT32_MAX & 0xFFFF */
  return f >= 65536.0f && f < 4294967296.0f ? (int32_t)((uint32_t)(int64_t)f & 0xFFFFu) : t & 0xFFFF;
}

/* orc_table_lookup: CMSIS arm_sin_f32 on a phase in turns */
static inline float table_lookup(float in) {
  int32_t n = f2i32_arm(in);
  n = in < 0.0f ? (int32_t)((uint32_t)n - 1u) : n;
  in = in - (float)n;
  float findex = 512.0f * in;
  int32_t index = f2u16_arm(findex);
  const int wrap = index >= 512;
  index = index & -(int32_t)!wrap;  /* 0 past the end, as mask arithmetic (a select splits the load) */
  findex = wrap ? findex - 512.0f : findex;
  const float fract = findex - (float)index;
  const float a = g_tab[index];
  const float b = g_tab[index + 1];
  return (1.0f - fract) * a + fract * b;
}
static inline float tsin(float x) { return table_lookup(x * 0.159154943092f); }
static inline float tcos(float x) { return table_lookup(x * 0.159154943092f + 0.25f); }

static inline float wrap_pi(float a) {
  return a >= PI_F ? a - 2.0f * PI_F : a < -PI_F ? a + 2.0f * PI_F : a;
}
static inline float wrap_innov(float a) {
  return a > PI_F ? a - 2.0f * PI_F : a < -PI_F ? a + 2.0f * PI_F : a;
}

/* One robot's KF6 tick in registers: orc_kf6_meas1, then orc_kf_update_f32 (joint LDL^T,
 * m = 4, H rows 2, 5, 3, 4) and the predict (x += v dt, F = I + dt at (i, i + 3)), straight-line
 * (cpu_port_kf6.inc, written by gen_cpu_port.py), so the robot loop has no inner loops. */
static inline void kf6_robot(float *restrict xv, float *restrict Pv, size_t n, size_t i, float yaw, float gz,
                             const int16_t *rp, float dt, const float *R, const float *Q) {
  float x0 = xv[0 * n + i], x1 = xv[1 * n + i], x2 = xv[2 * n + i], x3 = xv[3 * n + i], x4 = xv[4 * n + i],
        x5 = xv[5 * n + i];
#define LD(k) float Ps##k = Pv[k * n + i];
  LD(0) LD(1) LD(2) LD(3) LD(4) LD(5) LD(6) LD(7) LD(8) LD(9) LD(10)
  LD(11) LD(12) LD(13) LD(14) LD(15) LD(16) LD(17) LD(18) LD(19) LD(20)
#undef LD
  /* measurement frontend (orc_kf6_meas1) */
  const float th = yaw * k_deg2rad;
  const float om = -(gz * k_deg2rad);
  const float m0 = (float)rp[0] * k_rpm_to_radps * k_gear_ratio_inv;
  const float m1 = (float)rp[1] * k_rpm_to_radps * k_gear_ratio_inv;
  const float m2 = (float)rp[2] * k_rpm_to_radps * k_gear_ratio_inv;
  const float m3 = (float)rp[3] * k_rpm_to_radps * k_gear_ratio_inv;
  const float v0 = (m0 + m1 + m2 + m3) * 0.25f * k_wheel_r;
  const float v1 = (-m0 + m1 - m2 + m3) * 0.25f * k_wheel_r;
  const float c = tcos(th), s = tsin(th);
  const float y0 = wrap_innov(th - x2);
  const float y1 = om - x5;
  const float y2 = (v0 * c - v1 * s) * 0.001f - x3;
  const float y3 = (v0 * s + v1 * c) * 0.001f - x4;
#include "cpu_port_kf6.inc"
  xv[0 * n + i] = x0; xv[1 * n + i] = x1; xv[2 * n + i] = x2;
  xv[3 * n + i] = x3; xv[4 * n + i] = x4; xv[5 * n + i] = x5;
#define ST(k) Pv[k * n + i] = Ps##k;
  ST(0) ST(1) ST(2) ST(3) ST(4) ST(5) ST(6) ST(7) ST(8) ST(9) ST(10)
  ST(11) ST(12) ST(13) ST(14) ST(15) ST(16) ST(17) ST(18) ST(19) ST(20)
#undef ST
}

int port_kf6_tick(size_t n, float *x, float *P, const float *yaw_deg, const float *gyro_z_dps,
                  const int16_t *rpm, const orc_kf6_params *prm, int nthreads) {
  if (prm->trig != ORC_TRIG_TABLE512) return -1;
  const float dt = prm->dt;
  float R[10], Q[21];
  memcpy(R, prm->r, sizeof(R));
  memcpy(Q, prm->q, sizeof(Q));
  const long long nb = (long long)((n + BLK - 1) / BLK);
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for num_threads(nthreads) schedule(static)
#endif
  for (long long b = 0; b < nb; b++) {
    const size_t i0 = (size_t)b * BLK, i1 = i0 + BLK < n ? i0 + BLK : n;
#pragma omp simd
    for (size_t i = i0; i < i1; i++)
      kf6_robot(x, P, n, i, yaw_deg[i], gyro_z_dps[i], rpm + 4 * i, dt, R, Q);
  }
  return 0;
}

/* orc_rs_tick (VD_task_main.cpp:366-372 + VEHICLE_CTRL::update, VD_vehicle_controller.cpp:
 * 11-51): correct, then the velocity and odometry predict, robots in SIMD lanes */
int port_rs_tick(size_t n, float *pos, float *vel, int64_t *prev, const float *yaw_deg,
                 const int64_t *sum, const int16_t *rpm, int trig, int nthreads) {
  if (trig != ORC_TRIG_TABLE512) return -1;
  const long long nb = (long long)((n + BLK - 1) / BLK);
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for num_threads(nthreads) schedule(static)
#endif
  for (long long b = 0; b < nb; b++) {
    const size_t i0 = (size_t)b * BLK, i1 = i0 + BLK < n ? i0 + BLK : n;
#pragma omp simd
    for (size_t i = i0; i < i1; i++) {
      const float th = yaw_deg[i] * k_deg2rad;  /* set_now_yaw_world(deg2rad(yaw)) */
      const float m0 = (float)rpm[i * 4 + 0] * k_rpm_to_radps * k_gear_ratio_inv;
      const float m1 = (float)rpm[i * 4 + 1] * k_rpm_to_radps * k_gear_ratio_inv;
      const float m2 = (float)rpm[i * 4 + 2] * k_rpm_to_radps * k_gear_ratio_inv;
      const float m3 = (float)rpm[i * 4 + 3] * k_rpm_to_radps * k_gear_ratio_inv;
      vel[i] = (m0 + m1 + m2 + m3) * 0.25f * k_wheel_r;
      vel[n + i] = (-m0 + m1 - m2 + m3) * 0.25f * k_wheel_r;
      vel[2 * n + i] = (-m0 - m1 + m2 + m3) * 0.25f / k_sqrtf2 / k_wheel_l * k_wheel_r;
      /* Mrad in double, narrowed to float (VD_vehicle_controller.cpp:38-39) */
#define MRAD(w)                                                                                   \
  const int64_t s##w = sum[w * n + i];                                                           \
  const float r##w = (float)((double)(s##w - prev[w * n + i]) * (double)k_out_rad_per_raw *      \
                             (double)k_gear_ratio_inv);                                          \
  prev[w * n + i] = s##w;
      MRAD(0) MRAD(1) MRAD(2) MRAD(3)
#undef MRAD
      const float loc[3] = {(r0 + r1 + r2 + r3) * 0.25f * k_wheel_r, (-r0 + r1 - r2 + r3) * 0.25f * k_wheel_r, 0.0f};
      /* normalize_rad_0to2pi (util_mymath.hpp:18-25) */
      float r = th;
      const int out = r < 0.0f || r >= 2.0f * PI_F;
      const int mod = f2i32_arm(r / (2.0f * PI_F));
      float rn = r - (mod * 2.0f * PI_F);
      rn = rn < 0.0f ? rn + 2.0f * PI_F : rn;
      r = out ? rn : r;
      const float c = tcos(r), s = tsin(r);
      pos[2 * n + i] = th;
      pos[i] = pos[i] + (loc[0] * c - loc[1] * s) * 0.001f;
      pos[n + i] = pos[n + i] + (loc[0] * s + loc[1] * c) * 0.001f;
    }
  }
  return 0;
}

int port_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
