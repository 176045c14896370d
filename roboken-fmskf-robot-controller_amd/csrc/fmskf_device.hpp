// fmskf_device.hpp -- device-side scalar math of the hot path (gfx950).
//
// Every routine restates a reference routine with the same IEEE operation order,
// and the whole library is compiled with -ffp-contract=off, so results are bit
// identical to the firmware's C++ semantics (FLT_EVAL_METHOD 0, no FMA
// contraction) -- the oracle (oracle/fmskf_oracle.c) checks exactly that.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fmskf {

// PI of CMSIS-DSP arm_math.h as used by util_mymath.hpp:13-14
#define FMSKF_PI_F 3.14159265358979f
#define FMSKF_PI_D 3.141592653589793

struct K {
  static constexpr float deg2rad = FMSKF_PI_F / 180.0f;                  // util_mymath.hpp:14
  static constexpr float two_pi = 2.0f * FMSKF_PI_F;
  static constexpr float rpm_to_radps = 2.0f * 3.1415926f / 60.0f;       // VD_motor_if_m2006.hpp:77
  static constexpr float gear_ratio_inv = 1.0f / 36.0f;                  // VD_motor_if_m2006.hpp:81
  static constexpr float out_rad_per_raw = 2.0f * 3.1415926f / 8191.0f;  // VD_motor_if_m2006.hpp:82
  static constexpr float wheel_r = 37.5f;                                // VD_vehicle_controller.hpp:82
  static constexpr float wheel_l = 13.08148f;                            // VD_vehicle_controller.hpp:85
  static constexpr float sqrtf2 = 1.41421356f;                           // VD_vehicle_controller.hpp:86
  static constexpr float g0 = 9.80665f;
  static constexpr int raw_per_rot = 8192;                               // VD_motor_if_m2006.hpp:76
};

// The 513-entry sine table over [0, 2pi] (CMSIS-DSP sinTable_f32 layout) is a
// per-handle device buffer filled at fmskf_create from (float)sin(2*pi*i/512);
// kernels receive it as a pointer (it stays L1/L2 resident: 2 KiB).

__device__ __forceinline__ float deg2rad(float d) { return d * K::deg2rad; }  // util_mymath.hpp:16

// The firmware's float -> integer casts are Cortex-M7 VCVT.S32.F32 / VCVT.U32.F32: truncate,
// saturate to the destination range, NaN -> 0.  gfx950's v_cvt_i32_f32 / v_cvt_u32_f32 do
// exactly that, so they are issued directly: a C++ cast of an out-of-range float is undefined,
// and these give the firmware's answer for every input (a heading past 2^31 turns, inf, NaN).
__device__ __forceinline__ int32_t cvt_i32_arm(float f) {
  int32_t r;
  asm("v_cvt_i32_f32 %0, %1" : "=v"(r) : "v"(f));
  return r;
}
__device__ __forceinline__ uint32_t cvt_u32_arm(float f) {
  uint32_t r;
  asm("v_cvt_u32_f32 %0, %1" : "=v"(r) : "v"(f));
  return r;
}

// util_mymath.hpp:18-25
__device__ __forceinline__ float normalize_rad_0to2pi(float d) {
  if (d < 0.0f || d >= 2.0f * FMSKF_PI_F) {
    int mod = cvt_i32_arm(d / (2.0f * FMSKF_PI_F));
    d -= (mod * 2.0f * FMSKF_PI_F);
    if (d < 0.0f) d = d + 2.0f * FMSKF_PI_F;
  }
  return d;
}

// util_mymath.hpp:27-34
__device__ __forceinline__ float normalize_deg_0to360(float d) {
  if (d < 0.0f || d >= 360.0f) {
    int mod = cvt_i32_arm(d / (360.0f));
    d -= (mod * 360.0f);
    if (d < 0.0f) d = d + 360.0f;
  }
  return d;
}

// CMSIS-DSP arm_sin_f32 / arm_cos_f32 published algorithm: scale to turns, floor,
// 512-entry table, linear interpolation.  The floor's decrement wraps (INT_MIN - 1 on the
// M7 is INT_MAX); the table index is VCVT.U32 then the low 16 bits (uint16_t), so it is
// always < 513 whatever `in` is.
__device__ __forceinline__ float table_lookup(float in, const float *__restrict__ tab) {
  int32_t n = cvt_i32_arm(in);
  if (in < 0.0f) n = (int32_t)((uint32_t)n - 1u);
  in = in - (float)n;
  float findex = 512.0f * in;
  uint32_t index = (uint16_t)cvt_u32_arm(findex);
  if (index >= 512u) {
    index = 0;
    findex -= 512.0f;
  }
  float fract = findex - (float)index;
  float a = tab[index];
  float b = tab[index + 1];
  return (1.0f - fract) * a + fract * b;
}

template <bool LIBM>
__device__ __forceinline__ float sin_p(float x, const float *tab) {
  if constexpr (LIBM) return sinf(x);
  else return table_lookup(x * 0.159154943092f, tab);
}
template <bool LIBM>
__device__ __forceinline__ float cos_p(float x, const float *tab) {
  if constexpr (LIBM) return cosf(x);
  else return table_lookup(x * 0.159154943092f + 0.25f, tab);
}

// VEHICLE_CTRL::update rpm -> motor-output rad/s, VD_vehicle_controller.cpp:21-24
__device__ __forceinline__ float rpm_to_mvel(int16_t rpm) {
  return (float)rpm * K::rpm_to_radps * K::gear_ratio_inv;
}

// VEHICLE_CTRL::conv_Mdir_to_Vdir, VD_vehicle_controller.cpp:126-130 (FL, BL, BR, FR)
__device__ __forceinline__ void mdir_to_vdir(float fl, float bl, float br, float fr, float &vx,
                                             float &vy, float &vth) {
  vx = (fl + bl + br + fr) * 0.25f * K::wheel_r;
  vy = (-fl + bl - br + fr) * 0.25f * K::wheel_r;
  vth = (-fl - bl + br + fr) * 0.25f / K::sqrtf2 / K::wheel_l * K::wheel_r;
}

// heading kept in [-pi, pi)
__device__ __forceinline__ float wrap_pi(float a) {
  if (a >= FMSKF_PI_F) a = a - 2.0f * FMSKF_PI_F;
  else if (a < -FMSKF_PI_F) a = a + 2.0f * FMSKF_PI_F;
  return a;
}
__device__ __forceinline__ float wrap_innov(float a) {
  if (a > FMSKF_PI_F) a = a - 2.0f * FMSKF_PI_F;
  else if (a < -FMSKF_PI_F) a = a + 2.0f * FMSKF_PI_F;
  return a;
}
// wrap_pi of a compensated angle hi + lo: hi -/+ fp32(2 pi) is exact (Sterbenz), the rest of
// 2 pi (2 pi - 6.28318548f = -1.7484555e-7) goes to lo
__device__ __forceinline__ void wrap_pi_c(float &hi, float &lo) {
  if (hi >= FMSKF_PI_F) {
    hi = hi - 2.0f * FMSKF_PI_F;
    lo = lo + 1.7484555e-7f;
  } else if (hi < -FMSKF_PI_F) {
    hi = hi + 2.0f * FMSKF_PI_F;
    lo = lo - 1.7484555e-7f;
  }
}
__device__ __forceinline__ double wrap_pi(double a) {
  if (a >= FMSKF_PI_D) a = a - 2.0 * FMSKF_PI_D;
  else if (a < -FMSKF_PI_D) a = a + 2.0 * FMSKF_PI_D;
  return a;
}
__device__ __forceinline__ double wrap_innov(double a) {
  if (a > FMSKF_PI_D) a = a - 2.0 * FMSKF_PI_D;
  else if (a < -FMSKF_PI_D) a = a + 2.0 * FMSKF_PI_D;
  return a;
}

// ---------------------------------------------------------------------------
// IMU_IF_WT901C::Data, formed where it is read.  updateData (imu_if_wt901c.cpp:91-129) is a
// pure function of 16 register words and q_init, so the WT901 kernel keeps the words of the
// last successful poll (the snapshot row, and the Yaw / GZ words the tick consumes: imu_yg),
// and the readers (fmskf_get_imu, VehicleInfo) form the page from them.  Snapshot row [N][16]
// int16: accel x y z (0-2), gyro x y (3-4), mag x y z (5-7), roll, pitch (8-9), q0-q3 (10-13),
// word 14 the flags below, word 15 zero.
// (the row's flags and width: fmskf_internal.hpp kSnapValid / kSnapLatched / kSnapWords)

// Data.angle[2] and Data.gyro[2] from the Yaw (low half) / GZ (high half) register words of
// DevState::imu_yg, with updateData's operations (imu_if_wt901c.cpp:91-129): the readers form the
// same floats the WT901 kernel stored before round 6.
__host__ __device__ __forceinline__ float imu_yaw_deg(uint32_t yg) {
  return (float)(int16_t)(yg & 0xFFFFu) / 32768.0f * 180.0f;
}
__host__ __device__ __forceinline__ float imu_gz_dps(uint32_t yg) {
  return -((float)(int16_t)(yg >> 16) / 32768.0f * 2000.0f);
}
// A tick's yaw / gyro z from the dword its lane loaded: the IMU state's word when the call left
// the plane NULL (`word`, wave-uniform: TickIn::imu_words), else the caller's float.  Both are
// [N] dwords, so a kernel loads the same way either way and selects the conversion -- with a mask,
// not `?:`: the compiler turned the uniform select into a branch around the conversion, whose
// s_waitcnt vmcnt(0) stalled the KF6 plane-input tick behind every load it had issued (37.7-38.6
// -> 42.3 us at 2^20)
__device__ __forceinline__ float tick_word_sel(bool word, uint32_t w, float conv) {
  const uint32_t m = 0u - (uint32_t)word;
  return __builtin_bit_cast(float, (__builtin_bit_cast(uint32_t, conv) & m) | (w & ~m));
}
__device__ __forceinline__ float tick_yaw(bool word, uint32_t w) { return tick_word_sel(word, w, imu_yaw_deg(w)); }
__device__ __forceinline__ float tick_gz(bool word, uint32_t w) { return tick_word_sel(word, w, imu_gz_dps(w)); }

// the snapshot row of robot i (DevState::imu_snap: 12 int16 words, AX AY AZ GX GY Roll Pitch
// Q0-Q3 and the flags) as six dwords (three 8-byte loads), and the page's 16 words in
// imu_data_page's order with the snapshot's magnetometer words
__device__ __forceinline__ void snap_row_load(const int16_t *snap, uint64_t i, uint32_t rw[6]) {
  const uint2 *p = reinterpret_cast<const uint2 *>(snap + 12 * i);
  const uint2 a = p[0], b = p[1], c = p[2];
  rw[0] = a.x;
  rw[1] = a.y;
  rw[2] = b.x;
  rw[3] = b.y;
  rw[4] = c.x;
  rw[5] = c.y;
}
__device__ __forceinline__ void snap_page_words(const uint32_t rw[6], int16_t hx, int16_t hy, int16_t hz,
                                                int16_t w[16]) {
  int16_t r[12];
#pragma unroll
  for (int k = 0; k < 6; k++) {
    r[2 * k] = (int16_t)(rw[k] & 0xFFFFu);
    r[2 * k + 1] = (int16_t)(rw[k] >> 16);
  }
#pragma unroll
  for (int k = 0; k < 5; k++) w[k] = r[k];
  w[5] = hx;
  w[6] = hy;
  w[7] = hz;
  w[8] = r[5];
  w[9] = r[6];
#pragma unroll
  for (int k = 0; k < 4; k++) w[10 + k] = r[7 + k];
  w[14] = r[11];
  w[15] = 0;
}

// the Data page of a snapshot row (same operations and order as updateData): yaw = angle[2]
// and gz = gyro[2] from the Yaw / GZ words; qi: q_init as it was when the poll ran
__device__ __forceinline__ void imu_data_page(const int16_t *w, float yaw, float gz, const float qi[4],
                                              float d[16]) {
  float acc[3], gyr[2], mag[3], ang[2], q[4];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    acc[k] = (float)w[k] / 32768.0f * 16.0f;
    mag[k] = (float)w[5 + k];
  }
#pragma unroll
  for (int k = 0; k < 2; k++) {
    gyr[k] = (float)w[3 + k] / 32768.0f * 2000.0f;
    ang[k] = (float)w[8 + k] / 32768.0f * 180.0f;
  }
#pragma unroll
  for (int k = 0; k < 4; k++) q[k] = (float)w[10 + k] / 32768.0f;
  d[0] = acc[0];
  d[1] = -acc[1];
  d[2] = -acc[2];
  d[3] = gyr[0];
  d[4] = -gyr[1];
  d[5] = gz;
  d[6] = mag[0];
  d[7] = -mag[1];
  d[8] = -mag[2];
  d[9] = normalize_deg_0to360(ang[0]) - 180.0f;
  d[10] = ang[1];
  d[11] = yaw;
  d[14] = -(qi[3] * q[0] + qi[2] * q[1] - qi[1] * q[2] - qi[0] * q[3]);
  d[13] = (-qi[2] * q[0] + qi[3] * q[1] + qi[0] * q[2] - qi[1] * q[3]);
  d[12] = -(qi[1] * q[0] - qi[0] * q[1] + qi[3] * q[2] - qi[2] * q[3]);
  d[15] = (qi[0] * q[0] + qi[1] * q[1] + qi[2] * q[2] + qi[3] * q[3]);
}

__host__ __device__ constexpr int pk(int i, int j) {
  return i >= j ? i * (i + 1) / 2 + j : j * (j + 1) / 2 + i;
}

// explicit fused multiply-add (one rounding: v_fma_f32 / v_fma_f64 == C99 fmaf / fma)
template <typename T> __device__ __forceinline__ T dfma(T a, T b, T c);
template <> __device__ __forceinline__ float dfma<float>(float a, float b, float c) {
  return __builtin_fmaf(a, b, c);
}
template <> __device__ __forceinline__ double dfma<double>(double a, double b, double c) {
  return __builtin_fma(a, b, c);
}

}  // namespace fmskf
