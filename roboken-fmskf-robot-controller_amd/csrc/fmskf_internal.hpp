// fmskf_internal.hpp -- structures shared by the C-ABI layer (api_*.cpp) and the
// kernel launchers (kernels_*.hip).  Not part of the public ABI.
#pragma once
#include <cstdlib>
#include <cmath>
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include "../../include/fmskf.h"

namespace fmskf {

constexpr int kBlock = 256;  // 4 waves of 64 lanes

// WT901 snapshot (fmskf_device.hpp imu_data_page): the page's 16 int16 words per robot, word 14
// the flags: a successful poll happened / that poll latched q_init.  Stored (round 6) as a
// 12-word row (DevState::imu_snap: AX AY AZ GX GY Roll Pitch Q0-Q3, the flags; kRowWords) plus the
// magnetometer, which a standard poll does not carry: the snapshot's HX-HZ are the sReg ones
// unless a poll after the last successful one wrote them (then DevState::imu_mag holds the
// snapshot's; kernels_ingest.hip F_MAGDET)
constexpr int kSnapWords = 16, kRowWords = 12;
enum : int { kSnapValid = 1, kSnapLatched = 2 };

// Device-resident state of one handle.  Every array is plane-major (SoA): element k of
// instance i lives at [k * N + i] unless the comment says [N][k].
struct DevState {
  uint64_t n = 0;
  // plane pitch (elements) of x and P: plane k of instance i at [k * pitch + i].  Never a
  // large power of two (see plane_pitch): power-of-two plane strides alias in the
  // memory-side cache / channel hash and cost ~20% of bandwidth at N = 2^20 (membench).
  uint64_t pitch = 0;
  // 0: x / P are planar [rows][pitch]; else the tile width W: tiled [ceil(N/W)][rows][W]
  // (EKF9, KF12D; tile_w)
  uint32_t tile = 0;
  uint32_t model = 0;
  // estimator state: x [nx][pitch], P [np][pitch] (element type float, or double for KF12D);
  // RS: x = (px, py, th, vx, vy, vth) floats
  void *x = nullptr;
  void *P = nullptr;
  int64_t *prev_sum = nullptr;  // RS: s64_rawAngleSumPrev, 64-robot tiles of wheel pairs (lane_rs.hpp rs_prev_at)
  float *thlo = nullptr;        // EKF9: the heading's low part [N] (compensated heading)
  // KF6 with FMSKF_CFG_COMP_POS: the low parts of px, py, P[0][0], P[1][0], P[1][1], tiled like
  // x and P ([N/2048][5][2048])
  float *xlo = nullptr;
  // WT901 / IMU_IF_WT901C
  int16_t *imu_reg = nullptr;     // sReg [0x90][N]
  uint32_t *imu_parser = nullptr; // parser window [3][N] (bytes 0..11, little-endian)
  uint8_t *imu_cnt = nullptr;     // parser byte count [N]
  uint8_t *imu_flags = nullptr;   // s_cDataUpdate [N]
  uint8_t *imu_err = nullptr;     // is_error [N]
  float *imu_qinit = nullptr;     // q_init [4][N]
  // IMU_IF::Data is not stored: the WT901 kernel keeps the register words updateData reads
  // (fmskf_device.hpp imu_data_page), and the readers form the page
  int16_t *imu_snap = nullptr;    // snapshot rows [N][12] of the last successful poll (kRowWords)
  int16_t *imu_mag = nullptr;     // [N][4] the snapshot's HX-HZ while sReg's moved on (F_MAGDET)
  // the Yaw (low half) and GZ (high half) register words of the last successful poll [N]: what
  // the tick reads as its yaw and gyro z (Data.angle[2], Data.gyro[2]: fmskf_device.hpp
  // imu_yaw_deg / imu_gz_dps, exact both ways).  Round 6: one dword plane instead of the two
  // float planes, and while F_ROWREGS is set (kernels_ingest.hip) also the live GZ / Yaw registers
  uint32_t *imu_yg = nullptr;
  float *imu_qprev = nullptr;     // [4][N] q_init before a poll that latched it (kSnapLatched)
  // MOTOR_IF_M2006 x 4 wheels
  int16_t *m_micro = nullptr;  // [N][4]
  int16_t *m_angle = nullptr;  // [N][4]
  int16_t *m_prev = nullptr;   // [N][4] the angle of the frame before (Status ring entry head - 1):
                               // flt_dltOutAngle_rad is formed from the two at readout
  int16_t *m_rpm = nullptr;    // [N][4]
  int16_t *m_curr = nullptr;   // [N][4]
  // s64_rawAngleSum of the four wheels, split (round 6): sum = hi * 2^32 + lo read as int32.  The
  // low words [N][4] (one 16-byte access per robot) change with every frame, the high words [N][4]
  // only when a frame's delta (|d| <= 4096) carries the low word out of the int32 range (the sum
  // crossing an odd multiple of 2^31: never for a wheel near its start).  The CAN RX moves 16 + 16 B
  // of sums per robot instead of 32 + 32; readers of the whole sum (the RS tick on the motor state,
  // the readouts) load both halves (lane_rs.hpp motor_sum_load).  m_sum_lo doubles as "the motor
  // state exists"; all-zero is the reset state.
  uint32_t *m_sum_lo = nullptr;
  int32_t *m_sum_hi = nullptr;
  float *m_iir_y = nullptr;    // [N][4] (one 16-byte access per robot in k_can4)
  int16_t *m_prev_micro = nullptr;  // [N][4] the stamp of the frame before (the IIR1's previous
                                    // sample x is formed from it: kernels_ingest.hip can_wheel)
  // Round 6: (m_micro, m_prev_micro) and (m_angle, m_prev) are two-slot histories.  A CAN RX writes
  // the new stamp and angle over the older slot and nothing else (16 B per robot instead of 32:
  // the newest pair becomes the previous one where it lies), and the host flips m_par: 0, the
  // newest are m_micro / m_angle (the checkpoint's order), 1, they are m_prev_micro / m_prev.
  // The launchers and readers take the slots through motor_slots().
  uint32_t m_par = 0;
  unsigned long long *counters = nullptr;  // [8]
  float *sintab = nullptr;                 // [513]
};

// the motor state's stamp / angle history slots in the current order (DevState::m_par): the newest
// frame's stamps and angles, and the ones before
struct MotorSlots {
  int16_t *micro, *angle, *prev_micro, *prev;
};
inline MotorSlots motor_slots(const DevState &s) {
  return s.m_par ? MotorSlots{s.m_prev_micro, s.m_prev, s.m_micro, s.m_angle}
                 : MotorSlots{s.m_micro, s.m_angle, s.m_prev_micro, s.m_prev};
}

// Per-tick input planes, already resolved to device pointers.  `stride` is the
// per-tick advance (in instances) for fmskf_tick_many.
struct TickIn {
  const float *yaw_deg;
  const float *gyro_z;
  const int16_t *rpm;        // [N][4]
  const int64_t *angle_sum;  // [4][sum_pitch]
  const int16_t *raw;        // [N][8]
  const double *z;           // [8][N]
  const uint8_t *valid;      // [N] or null
  const uint32_t *rec;       // KF6 [N] x 16-byte records {yaw, gz, rpm[4]} or null
  const float *sintab;       // 513-entry TABLE512 sine table (device)
  uint64_t stride;
  uint64_t sum_pitch;  // plane stride of angle_sum (the caller's)
  // the RS tick on the motor state's sums (angle_sum NULL): their [N][4] low / high halves
  const uint32_t *msum_lo;
  const int32_t *msum_hi;
  uint32_t n_ticks;
  // fmskf_tick_ensemble: the tick kernel also writes its blocks' ensemble records of the
  // post-tick state ([LEN][grid], ens_device.hpp) against the shift vector; null otherwise
  double *ens_blocks;
  const double *ens_shift;
  uint32_t ens_grid;  // the tick blocks (= block records); set by the launcher
  // fmskf_tick_ensemble_begin: the previous event's block records ([LEN][fold_nb]), folded by
  // LEN extra blocks at the front of this tick's grid into fold_out (ens_fold_front); null
  // otherwise
  uint32_t fold_nb;
  const double *fold_blocks;
  double *fold_out;
  // host side only (never read by a kernel): the event the fused ENS launch attaches to the
  // kernel's own completion signal (launch_signal), or null
  hipEvent_t ens_done;  // bit 0: yaw_deg points at the IMU state's Yaw words, bit 1: gyro_z at its GZ words (both
  // DevState::imu_yg, fmskf_device.hpp tick_yaw / tick_gz) -- a NULL plane of the call.  The host
  // resolves the pointer: selecting it in the kernel took the KF6 plane-input k_kf6t from 64 to 87
  // VGPRs (and a field inserted before the others, which moved their kernel-argument offsets, did
  // the same).
  uint32_t imu_words;
};

// k<<<g, kBlock, lds, st>>>(a); with `done`, the dispatch's own completion signal records the
// event (hipExtLaunchKernelGGL), so no marker packet follows the kernel on the stream
template <typename A>
inline void launch_signal(void (*k)(A), dim3 g, unsigned lds, hipStream_t st, hipEvent_t done, const A &a) {
  if (done) hipExtLaunchKernelGGL(k, g, dim3(kBlock), lds, st, nullptr, done, 0u, a);
  else k<<<g, kBlock, lds, st>>>(a);
}

template <typename T, int NP, int MP>
struct KfParams {
  T dt;
  T q[NP];
  T r[MP];
};
struct Kf6Params {
  float dt;
  float q[21];
  float r[10];
  // FMSKF_CFG_COMP_POS: the tiled low-part rows (px, py, P00, P10, P11); null = plain fp32
  float *lo;
};
constexpr uint32_t kKf6LoRows = 5;
struct Ekf9Params {
  float dt;
  float q[45];
  float r[21];
  float *thlo;  // [N] the compensated heading's low part (a hidden state row; th_add)
  // FMSKF_CFG_COMP_POS: the tiled low-part rows (px, py, P00, P10, P11); null = plain
  float *clo;
};
struct Kf12dParams {
  double dt;
  double q[78];
  double r[36];   // full packed 8x8 R (joint update)
  double r2[10];  // packed R of the arm-tip group (rows/cols 4..7), used by the sequential path
  double cinv[36];  // C^-1 of R = C C^T (packed lower), the decorrelated update's coefficients
  int decor;        // R positive definite: decorrelated scalar-sequential update
  // the default sparsity (kf12d_sparse): C^-1 nonzero only on its diagonal and at (3,2), Q only
  // inside the (pos, vel) pair blocks -> the kernel drops the other terms at compile time
  int sparse;
  const double *coef;  // device copy: cinv [36] then q [78] (read by scalar loads at their use)
};
// true when every C^-1 entry off the diagonal and (3,2), and every Q entry between different
// (pos, vel) pairs (pos k <-> vel k + 3; base k = 0..2, tip 6..8), is exactly zero
inline bool kf12d_sparse(const double *cinv36, const double *q78) {
  for (int a = 0; a < 8; a++)
    for (int b = 0; b < a; b++)
      if (!(a == 3 && b == 2) && cinv36[a * (a + 1) / 2 + b] != 0.0) return false;
  auto pair = [](int s) { return s < 6 ? s % 3 : 3 + (s - 6) % 3; };
  for (int i = 0; i < 12; i++)
    for (int j = 0; j <= i; j++)
      if (pair(i) != pair(j) && q78[i * (i + 1) / 2 + j] != 0.0) return false;
  return true;
}
// Cinv of R = C C^T, packed lower; false when R is not positive definite.  Same operations,
// in the same order, as the oracle's orc_kf12d_cinv (the canonical KF12D update uses it).
inline bool kf12d_cinv(const double *r, double *ci) {
  auto pk2 = [](int i, int j) { return i >= j ? i * (i + 1) / 2 + j : j * (j + 1) / 2 + i; };
  double c[8][8] = {}, v[8][8] = {};
  for (int j = 0; j < 8; j++) {
    double s = r[pk2(j, j)];
    for (int k = 0; k < j; k++) s = s - c[j][k] * c[j][k];
    if (!(s > 0.0) || !std::isfinite(s)) return false;
    c[j][j] = std::sqrt(s);
    for (int i = j + 1; i < 8; i++) {
      double t = r[pk2(i, j)];
      for (int k = 0; k < j; k++) t = t - c[i][k] * c[j][k];
      c[i][j] = t / c[j][j];
    }
  }
  for (int j = 0; j < 8; j++) {
    v[j][j] = 1.0 / c[j][j];
    for (int i = j + 1; i < 8; i++) {
      double t = 0.0;
      for (int k = j; k < i; k++) t = t + c[i][k] * v[k][j];
      v[i][j] = -t / c[i][i];
    }
  }
  for (int i = 0; i < 8; i++)
    for (int j = 0; j <= i; j++) ci[pk2(i, j)] = v[i][j];
  return true;
}
// true when R has no terms between the base group (0..3) and the tip group (4..7)
inline bool kf12d_sequential(const double *r36) {
  for (int i = 4; i < 8; i++)
    for (int j = 0; j < 4; j++)
      if (r36[i * (i + 1) / 2 + j] != 0.0) return false;
  return true;
}

// true when the EKF9 R (packed 6x6, as the kernels receive it) has no off-diagonal terms:
// the canonical EKF9 update is then the sequential scalar one (oracle orc_ekf9_tick)
inline bool ekf9_r_diagonal(const float *r21) {
  for (int i = 1; i < 6; i++)
    for (int j = 0; j < i; j++)
      if (r21[i * (i + 1) / 2 + j] != 0.0f) return false;
  return true;
}

// Vehicle control state, allocated on first use of the control entry
// points.  Planes at the state pitch:
//   ax  [3 axes][12][pitch]: VelInterpConstJerk page (vel_tgt, acl_max, jerk_p, jerk_m, dt1,
//                            dt2, dt3, vel_ini, acl_ini, dt) + vel_now, acl_now
//   pid [4 wheels][6][pitch]: FF_PI_D (now_val == prev_val, Integ, LPF now_Y, LPF prev_X,
//                            now_tgt, now_ctrl)
//   vel_tgt [3][pitch]       : now_vhcl_vel_tgt_mmps
// Round 6: the step's outputs nothing reads back -- vel_tgt, now_tgt, now_ctrl, 44 B per robot --
// are formed from the state it leaves when a reader asks (ctrl_lane.hpp ctrl_derive, host flag
// fmskf_ctx::ctrl_derived_stale), except for robots whose power was off (vel_tgt is the
// interpolators' last output, which their reset erased: the step stores it).
//   curr [N][4] int16        : MOTOR_IF_M2006::s16_rawCurr_tgt (one 8-byte access per robot)
//   power [N] u8             : isPowerOn
struct CtrlDev {
  uint64_t n = 0, pitch = 0;
  float *ax = nullptr;
  float *pid = nullptr;
  float *vel_tgt = nullptr;
  // [N][4] the rpm the last step ran on (0 after a power-off reset): FF_PI_D's now_val is
  // rpm_to_mvel(rpm) * GEAR_RATIO, so the step keeps the 8-byte record instead of the four float
  // now_val planes (round 6; the pid planes' now_val row is no longer used)
  int16_t *rpm_prev = nullptr;
  int16_t *curr = nullptr;
  uint8_t *power = nullptr;
};
constexpr int kAxF = 12, kPidF = 6;
// FF_PI_D / interpolator / current-limit parameters as the device uses them
struct CtrlPrm {
  float freq, dt, ff_gain, p_gain, i_gain, d_gain, i_limit, ff_limit, a1, b0, b1, ts;
  int32_t curr_limit;
  int32_t dir[4];
  // 1: the step also stores vel_tgt, now_tgt and now_ctrl (inside a graph capture: the replay's
  // readers cannot be brought up to date by the host); 0: they are formed on demand (ctrl_derive)
  uint32_t store_derived;
};

// x / P plane pitch for N instances: N rounded up to 512, plus 256 -> an odd multiple of
// 1 KiB (fp32) between planes
inline uint64_t plane_pitch(uint64_t n) { return ((n + 511) / 512) * 512 + 256; }

// Tiled state layout ("AoSoA"): instance i's row k at ((i / W) * rows + k) * W + i % W, W the
// tile width.  Block b (kBlock instances, a "chunk") owns columns (b % (W / kBlock)) * kBlock...
// of tile b / (W / kBlock): its rows are kBlock-element runs W elements apart, its base is
// wave-uniform.  Consecutive blocks land on different XCDs, so a wide tile has the XCDs
// reading and writing the same DRAM rows at the same time.  tools/membench.hip `tiles` (the
// non-temporal EKF9 pattern at 2^22 with the tick's 864-FMA compute phase, 64 KiB cap):
// W = 256 309-313 us, 512 290-291, 1024 282-284, 2048 279-281, 4096 282-284; KF12D's 90 fp64
// rows at 2^20 with 1280 fp64 FMAs: 256 269-270, 1024 268-269, 2048 263-265, 4096 259-260.
// (Against planar planes the 256-wide tile already measured 374.6 -> 353.6 us for EKF9.)  The
// KF6 state (FMSKF_KF6_TILED) and the control state's interpolator / FF_PI_D arrays
// (FMSKF_CTRL_TILED) use the fp32 width too; the RS state stays planar.  The allocation
// (rows x pitch, pitch >= N rounded up to W) always covers ceil(N / W) tiles.
template <typename T>
constexpr uint32_t tile_w() { return sizeof(T) == 8 ? 4096u : 2048u; }  // fp64 (KF12D) / fp32
inline uint32_t tile_w_elem(uint32_t elem) { return elem == 8 ? 4096u : 2048u; }

// Cache policy of the per-tick state stream.  When the state is several times the 256 MiB
// Infinity Cache, every state byte is read once and written once per tick from HBM; loading
// and storing it non-temporal (gfx950 `nt`, buffer aux bit 1) measured 15% faster on the
// tiled pattern at 2^22 EKF9 robots (tools/membench.hip: 352 -> 299 us), while it is slower
// when the state fits the Infinity Cache.  FMSKF_STATE_NT=0|1 forces it off or on.
constexpr int kStateNT = 2;
// Cache policy of the state STORES.  Every state line is written once per tick and not read
// again in the launch, so a store need not keep it in the XCD's L2: `sc1` (buffer aux bit 4)
// writes it to the memory side and drops it from L2 (MI355X_MICROARCH.md, store flavours).
// While the state lives in the Infinity Cache that measured 4% faster on the KF6 pattern at
// 2^20 (tools/membench.hip pol: 39.25 -> 37.6 us); past it the stores follow the loads (nt).
#ifndef FMSKF_ST_CACHED
#define FMSKF_ST_CACHED 16
#endif
#ifndef FMSKF_ST_STREAM
#define FMSKF_ST_STREAM 2
#endif
// the store policy that goes with a load policy CP (0: cache-resident state, kStateNT: streamed)
constexpr int st_pol(int cp) { return cp == kStateNT ? FMSKF_ST_STREAM : FMSKF_ST_CACHED; }
inline bool state_nt(uint64_t state_bytes) {
  static const int force = [] {
    const char *e = getenv("FMSKF_STATE_NT");
    return e ? atoi(e) : -1;
  }();
  if (force >= 0) return force != 0;
  return state_bytes > (256ull << 20);
}

// bytes per robot of the handle's estimator state (x, P and the hidden low-part rows): the part
// of the working set the ingest kernels' cache policies have to leave room for
inline uint64_t est_state_bytes(const DevState &s) {
  switch (s.model) {
    case FMSKF_MODEL_RS: return 56;
    case FMSKF_MODEL_KF6: return s.xlo ? 128 : 108;
    case FMSKF_MODEL_EKF9: return s.xlo ? 240 : 220;
    default: return 90 * 8;  // KF12D
  }
}

// Occupancy cap for the kernels that stream their state from HBM: dynamic LDS per block limits
// the resident blocks per CU (160 KiB / bytes), so fewer tile / plane streams compete for the
// HBM channels.  The environment variable (read once per call site) overrides the byte count.
#define FMSKF_LDS_CAP(NAME, HBM, DFLT)                              \
  ([&]() -> unsigned {                                              \
    static const int v_ = [] {                                      \
      const char *e_ = getenv(NAME);                                \
      return e_ ? atoi(e_) : -1;                                    \
    }();                                                            \
    return v_ >= 0 ? (unsigned)v_ : ((HBM) ? (unsigned)(DFLT) : 0u); \
  }())

#ifndef FMSKF_TILED
#define FMSKF_TILED 1
#endif
// the KF6 state tiled like EKF9's (2048 robots per tile row) instead of planar planes at the
// padded pitch; 0 builds the planar layout (A/B)
#ifndef FMSKF_KF6_TILED
#define FMSKF_KF6_TILED 1
#endif
// the control state's interpolator and FF_PI_D arrays tiled the same way (ctrl_lane.hpp
// Planes); 0 builds them planar at the state pitch (A/B)
#ifndef FMSKF_CTRL_TILED
#define FMSKF_CTRL_TILED 1
#endif
__host__ __device__ inline uint64_t st_at(uint32_t tile, uint64_t pitch, uint32_t rows, uint32_t k,
                                          uint64_t i) {
  return tile ? ((i / tile) * rows + k) * tile + i % tile : k * pitch + i;
}

struct Wt901Cfg {
  uint32_t read_reg_index;
};

// launchers (return hipError_t as int)
int launch_rs(const DevState &s, const TickIn &in, bool libm, bool correct, bool predict,
              hipStream_t st);
// in.ens_blocks set (upd and pred only): *ens_nb receives the grid, i.e. the record count
int launch_kf6(const DevState &s, const TickIn &in, const Kf6Params &p, bool libm, bool upd,
               bool pred, hipStream_t st, int *ens_nb = nullptr);
int launch_ekf9(const DevState &s, const TickIn &in, const Ekf9Params &p, bool libm, bool upd,
                bool pred, hipStream_t st, int *ens_nb = nullptr);
int launch_kf12d(const DevState &s, const TickIn &in, const Kf12dParams &p, bool upd, bool pred,
                 hipStream_t st, int *ens_nb = nullptr);
int launch_wt901(const DevState &s, const uint8_t *bytes, uint32_t stride, const uint32_t *len,
                 int latch_qinit, uint32_t read_reg_index, hipStream_t st);
int launch_can(const DevState &s, const uint8_t *frames, const int16_t *stamps,
               const uint8_t *present, const int8_t dir[4], hipStream_t st);
int launch_trig(const float *x, float *sv, float *cv, uint64_t n, bool libm, const float *tab,
                hipStream_t st);
// ensemble (kernels_misc.hip): per-block partial records of x, then the fold (one block per
// record element); launch_ens_fold folds records a tick kernel wrote (nb = its grid);
// launch_ens_shift sets the shift vector to robot 0's state
int launch_ensemble(const DevState &s, int nx, bool f64, double *blocks, const double *shift,
                    double *out, hipStream_t st);
int launch_ens_fold(int nx, const double *blocks, int nb, const double *shift, double *out,
                    hipStream_t st);
// the stand-alone partial alone (no fold): *nb receives the block-record count
int launch_ens_partial(const DevState &s, int nx, bool f64, double *blocks, const double *shift,
                       hipStream_t st, int *nb);
int launch_ens_shift(const DevState &s, int nx, bool f64, double *shift, hipStream_t st);
int ensemble_nblocks(uint64_t n);
// vehicle control step, TX frames, VehicleInfo export (kernels_ctrl.hip)
int launch_ctrl_set_target(const CtrlDev &c, const float *vel, const float *acl, const float *jrk,
                           const uint8_t *mask, hipStream_t st);
int launch_ctrl_derive(const CtrlDev &c, const CtrlPrm &p, hipStream_t st);
int launch_ctrl_step(const CtrlDev &c, const CtrlPrm &p, const int16_t *rpm, uint32_t rstride,
                     hipStream_t st);
int launch_can_tx(const CtrlDev &c, uint8_t *frames, hipStream_t st);
// the firmware ISR for the 6-state KF in one kernel (tick + control step + TX frame);
// hipErrorNotSupported where the three-kernel path applies instead (streamed state, huge N)
int launch_isr_kf6(const DevState &s, const TickIn &in, const Kf6Params &kp, bool libm, const CtrlDev &c,
                   const CtrlPrm &p, uint8_t *frames, hipStream_t st);
// the same with the tick's CAN RX fused in front (every wheel present; hipErrorNotSupported
// where that form does not apply)
int launch_isr_kf6_can(const DevState &s, const TickIn &in, const Kf6Params &kp, bool libm, const CtrlDev &c,
                       const CtrlPrm &p, uint8_t *frames, const uint8_t *can_frames, const int16_t *can_stamps,
                       const int8_t dir[4], hipStream_t st);
// fmskf_isr_tick for EKF9 in one kernel (hipErrorNotSupported where it does not apply); rpm:
// the control step's [N][4] rpm (the caller's plane or the motor state)
int launch_isr_ekf9(const DevState &s, const TickIn &in, const Ekf9Params &prm, bool libm, const CtrlDev &c,
                    const CtrlPrm &p, const int16_t *rpm, uint8_t *frames, hipStream_t st);
int launch_isr_ekf9_can(const DevState &s, const TickIn &in, const Ekf9Params &prm, bool libm, const CtrlDev &c,
                        const CtrlPrm &p, uint8_t *frames, const uint8_t *can_frames, const int16_t *can_stamps,
                        const int8_t dir[4], hipStream_t st);
// RS previous sums: the tick's tiled layout (lane_rs.hpp rs_prev_at) -> [4][pitch] planes
int launch_prev_out(const int64_t *prev, int64_t *dst, uint64_t n, uint64_t pitch, hipStream_t st);
// the motor state's split sums as int64: into the RS previous-sum tiles (to_prev), or [4][pitch]
// planes
int launch_motor_sums(const uint32_t *lo, const int32_t *hi, int64_t *dst, uint64_t n, uint64_t pitch, bool to_prev,
                      hipStream_t st);
// the WT901 register file made whole: the row-resident registers written back from the
// snapshot rows of the robots whose standard poll kept them there (kernels_ingest.hip F_ROWREGS)
int launch_wt901_regs_sync(const DevState &s, hipStream_t st);
int launch_isr_rs_can(const DevState &s, const TickIn &in, bool libm, const CtrlDev &c, const CtrlPrm &p,
                      uint8_t *frames, const uint8_t *can_frames, const int16_t *can_stamps, const int8_t dir[4],
                      bool prev_in_sums, hipStream_t st);
// the firmware ISR, reference semantics: RS tick + control step + TX frame in one kernel
int launch_isr_rs(const DevState &s, const TickIn &in, bool libm, const CtrlDev &c,
                  const CtrlPrm &p, uint8_t *frames, hipStream_t st);
// IMU_IF::Data [16][N] formed from the snapshot (fmskf_get_imu)
int launch_imu_data(const DevState &s, float *out, hipStream_t st);
int launch_vehicle_info(const DevState &s, const float *readout, void *out, const uint8_t *floor,
                        const float *cam_pitch, const uint32_t *fault, hipStream_t st);
// readout helpers
int launch_fill64(void *p, uint64_t bits, uint64_t count, hipStream_t st);
// tiled state arrays (kernels_misc.hip): fill row k with bits[k] (elem 4 or 8 bytes); convert
// between the tiled array (rows x N) and dense [rows][N] planes
int launch_tiled_fill(void *base, uint32_t rows, uint64_t n, const uint64_t *bits, uint32_t elem,
                      hipStream_t st);
int launch_untile(const void *tiled, void *dense, uint32_t rows, uint64_t n, uint32_t elem,
                  hipStream_t st);
int launch_tile(const void *dense, void *tiled, uint32_t rows, uint64_t n, uint32_t elem,
                hipStream_t st);
// pose / body velocity readout as float planes: out [6][N] = x, y, th, vx_body_mmps, vy_body_mmps, w
int launch_readout(const DevState &s, float *out, hipStream_t st);
// Status::flt_dltOutAngle_rad [N][4] from the last two raw angles (count = 4 N)
int launch_motor_dlt(const int16_t *angle, const int16_t *prev, float *out, uint64_t count, hipStream_t st);
// exchange the two motor history slots of every wheel (the caller flips DevState::m_par)
int launch_motor_swap(const DevState &s, hipStream_t st);

}  // namespace fmskf
