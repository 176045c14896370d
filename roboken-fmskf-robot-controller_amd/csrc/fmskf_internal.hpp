// fmskf_internal.hpp -- structures shared by the C-ABI layer (fmskf_api.cpp) and the
// kernel launchers (kernels_*.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fmskf {

constexpr int kBlock = 256;  // 4 waves of 64 lanes

// Device-resident state of one handle.  Every array is plane-major (SoA): element k of
// instance i lives at [k * N + i] unless the comment says [N][k].
struct DevState {
  uint64_t n = 0;
  // plane pitch (elements) of x and P: plane k of instance i at [k * pitch + i].  Never a
  // large power of two (see plane_pitch): power-of-two plane strides alias in the
  // memory-side cache / channel hash and cost ~20% of bandwidth at N = 2^20 (membench).
  uint64_t pitch = 0;
  uint32_t model = 0;
  // estimator state: x [nx][pitch], P [np][pitch] (element type float, or double for KF12D);
  // RS: x = (px, py, th, vx, vy, vth) floats
  void *x = nullptr;
  void *P = nullptr;
  int64_t *prev_sum = nullptr;  // RS: s64_rawAngleSumPrev [4][N]
  // WT901 / IMU_IF_WT901C
  int16_t *imu_reg = nullptr;     // sReg [0x90][N]
  uint32_t *imu_parser = nullptr; // parser window [3][N] (bytes 0..11, little-endian)
  uint8_t *imu_cnt = nullptr;     // parser byte count [N]
  uint8_t *imu_flags = nullptr;   // s_cDataUpdate [N]
  uint8_t *imu_err = nullptr;     // is_error [N]
  float *imu_qinit = nullptr;     // q_init [4][N]
  float *imu_data = nullptr;      // Data page [16][N]
  // MOTOR_IF_M2006 x 4 wheels
  int16_t *m_micro = nullptr;  // [N][4]
  int16_t *m_angle = nullptr;  // [N][4]
  int16_t *m_rpm = nullptr;    // [N][4]
  int16_t *m_curr = nullptr;   // [N][4]
  uint8_t *m_head = nullptr;   // [N][4]
  int64_t *m_sum = nullptr;    // [4][N]
  float *m_dlt = nullptr;      // [4][N]
  float *m_speed = nullptr;    // [4][N]
  float *m_iir_y = nullptr;    // [4][N]
  float *m_iir_x = nullptr;    // [4][N]
  unsigned long long *counters = nullptr;  // [8]
  float *sintab = nullptr;                 // [513]
};

// Per-tick input planes, already resolved to device pointers.  `stride` is the
// per-tick advance (in instances) for fmskf_tick_many.
struct TickIn {
  const float *yaw_deg;
  const float *gyro_z;
  const int16_t *rpm;        // [N][4]
  const int64_t *angle_sum;  // [4][N]
  const int16_t *raw;        // [N][8]
  const double *z;           // [8][N]
  const uint8_t *valid;      // [N] or null
  const float *sintab;       // 513-entry TABLE512 sine table (device)
  uint64_t stride;
  uint32_t n_ticks;
};

template <typename T, int NP, int MP>
struct KfParams {
  T dt;
  T q[NP];
  T r[MP];
};
using Kf6Params = KfParams<float, 21, 10>;
using Ekf9Params = KfParams<float, 45, 21>;
struct Kf12dParams {
  double dt;
  double q[78];
  double r[36];   // full packed 8x8 R (joint update)
  double r2[10];  // packed R of the arm-tip group (rows/cols 4..7), used by the sequential path
};
// true when R has no terms between the base group (0..3) and the tip group (4..7)
inline bool kf12d_sequential(const double *r36) {
  for (int i = 4; i < 8; i++)
    for (int j = 0; j < 4; j++)
      if (r36[i * (i + 1) / 2 + j] != 0.0) return false;
  return true;
}

// x / P plane pitch for N instances: N rounded up to 512, plus 256 -> an odd multiple of
// 1 KiB (fp32) between planes
inline uint64_t plane_pitch(uint64_t n) { return ((n + 511) / 512) * 512 + 256; }

struct Wt901Cfg {
  uint32_t read_reg_index;
};

// launchers (return hipError_t as int)
int launch_rs(const DevState &s, const TickIn &in, bool libm, bool correct, bool predict,
              hipStream_t st);
int launch_kf6(const DevState &s, const TickIn &in, const Kf6Params &p, bool libm, bool upd,
               bool pred, hipStream_t st);
int launch_ekf9(const DevState &s, const TickIn &in, const Ekf9Params &p, bool libm, bool upd,
                bool pred, hipStream_t st);
int launch_kf12d(const DevState &s, const TickIn &in, const Kf12dParams &p, bool upd, bool pred,
                 hipStream_t st);
int launch_wt901(const DevState &s, const uint8_t *bytes, uint32_t stride, const uint32_t *len,
                 int latch_qinit, uint32_t read_reg_index, hipStream_t st);
int launch_can(const DevState &s, const uint8_t *frames, const int16_t *stamps,
               const uint8_t *present, const int8_t dir[4], hipStream_t st);
int launch_trig(const float *x, float *sv, float *cv, uint64_t n, bool libm, const float *tab,
                hipStream_t st);
// ensemble: per-block partial records, then a single-block fold in block order
int launch_ensemble(const DevState &s, int nx, bool f64, double *blocks, double *out,
                    hipStream_t st);
int ensemble_nblocks(uint64_t n);
// readout helpers
int launch_fill64(void *p, uint64_t bits, uint64_t count, hipStream_t st);
// pose / body velocity readout as float planes: out [6][N] = x, y, th, vx_body_mmps, vy_body_mmps, w
int launch_readout(const DevState &s, float *out, hipStream_t st);

}  // namespace fmskf
