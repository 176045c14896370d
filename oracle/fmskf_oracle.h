/*
 * fmskf_oracle.h -- CPU restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libfmskf) links, loads or
 * calls this code.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, and only as the checker / the timed CPU baseline.
 *
 * Reference: Moryu-Io/Roboken-FMSKF-robot-controller (paths relative to the repo root).
 *
 * Parity status (see DESIGN.md "Oracle"):
 *   - WT901 byte parser + register file (A1, A2): PINNED against oracle/_ref,
 *     the reference's own lib/wt901c/wit_c_sdk.c compiled here, via the golden
 *     fixtures in tests/golden/wt901_*.npz.
 *   - IMU conversion (A3, A4), CAN unwrap (A8), odometry integrator (A9-A12):
 *     restated from the reference source; the reference files need Arduino /
 *     CMSIS-DSP / FreeRTOS headers absent from this image, so they are
 *     unbuildable here -> pinned only by known-answer tests derived from the
 *     reference constants (tests/test_oracle_known_answers.py).  Parity
 *     against the reference binary itself is UNPINNED for these rows.
 *   - CMSIS-DSP arm_sin_f32 / arm_cos_f32 (A13, third-party, absent): restated
 *     from the published CMSIS-DSP 5.x algorithm (512-entry table + linear
 *     interpolation).  UNPINNED against the device library.
 *   - KF / EKF math (A15): no reference counterpart (new math defined by the
 *     north star).  The fp32 restatement here is checked against an
 *     independent fp64 dense restatement (oracle/kf_ref.py).
 */
#ifndef FMSKF_ORACLE_H_
#define FMSKF_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_TRIG_TABLE512 = 0, ORC_TRIG_LIBM = 1 };

/* ---------------- scalar math (src/Utility/util_mymath.hpp) ---------------- */
float orc_deg2rad(float d);                 /* util_mymath.hpp:16 */
float orc_normalize_rad_0to2pi(float d);    /* util_mymath.hpp:18-25 */
float orc_normalize_deg_0to360(float d);    /* util_mymath.hpp:27-34 */
float orc_sin(float x, int trig);           /* util_mymath.hpp:44 -> arm_sin_f32 */
float orc_cos(float x, int trig);           /* util_mymath.hpp:45 -> arm_cos_f32 */
void  orc_eval_trig(const float *x, float *s, float *c, size_t n, int trig);
void  orc_sin_table(float out[513]);

/* ---------------- mecanum kinematics (VD_vehicle_controller.cpp) ---------- */
void orc_mdir_to_vdir(const float m[4], float v[3]);   /* :126-130 */
void orc_vdir_to_mdir(const float v[3], float m[4]);   /* :113-118 */

/* ---------------- WT901 byte parser + IMU conversion ---------------------- */
#define ORC_WT901_NREG 0x90
typedef struct {
  uint8_t  buf[256];          /* s_ucWitDataBuff (wit_c_sdk.c:11) */
  uint32_t cnt;               /* s_uiWitDataCnt  (wit_c_sdk.c:12) */
  uint32_t read_reg_index;    /* s_uiReadRegIndex (wit_c_sdk.c:12) */
  int16_t  reg[ORC_WT901_NREG];/* sReg (wit_c_sdk.c:13) */
  uint8_t  flags;             /* s_cDataUpdate (imu_if_wt901c.cpp:16) */
  uint8_t  is_error;          /* IMU_IF_WT901C::is_error */
  float    q_init[4];         /* IMU_IF_WT901C::q_init */
  float    data[16];          /* latest Data page: accel3 gyro3 mag3 angle3 qut4 */
  /* callback log (for pinning against the reference build) */
  uint32_t ncb;
  uint16_t cb_reg[64];
  uint16_t cb_num[64];
} orc_wt901;

void orc_wt901_reset(orc_wt901 *s, uint32_t read_reg_index);
void orc_wt901_byte(orc_wt901 *s, uint8_t b);                 /* WitSerialDataIn */
int  orc_wt901_is_com_comp(orc_wt901 *s, const uint8_t *bytes, uint32_t len); /* isComComp */
void orc_wt901_update_data(orc_wt901 *s);                     /* updateData */
/* IMU_IF_WT901C::update() on one poll's bytes; latch_qinit emulates init()'s
 * q_init latch (imu_if_wt901c.cpp:70-76) after a successful poll. */
void orc_wt901_update(orc_wt901 *s, const uint8_t *bytes, uint32_t len, int latch_qinit);
/* batched: bytes[i*stride ...], len[i] */
void orc_wt901_update_batch(size_t n, orc_wt901 *s, const uint8_t *bytes, uint32_t stride,
                            const uint32_t *len, int latch_qinit);

/* ---------------- M2006 / C610 CAN rx (VD_motor_if_m2006.cpp:32-72) ------- */
typedef struct {
  int16_t micro, angle, rpm, curr;  /* Status of status_buf[status_head] */
  float   dlt_out_angle_rad;
  float   speed_radps;
  uint8_t head;                     /* status_head */
  int8_t  dir;                      /* s8_motor_drive_dir */
  int64_t angle_sum;                /* s64_rawAngleSum */
  float   iir_prev_y, iir_prev_x;   /* UTIL::IIR1 state (util_iir.hpp:39-45) */
} orc_m2006;

void orc_m2006_reset(orc_m2006 *m, int dir);
void orc_m2006_rx(orc_m2006 *m, const uint8_t frame[8], int16_t micro);
/* frames [n][4][8], stamps [n][4], present [n] bit w = wheel w present (NULL: all) */
void orc_can_ingest_batch(size_t n, orc_m2006 *motors /*[n][4]*/, const uint8_t *frames,
                          const int16_t *stamps, const uint8_t *present);

/* ---------------- reference-semantics tick (RS) --------------------------- */
/* pos [3][n] (x m, y m, th rad), vel [3][n] (mm/s, mm/s, rad/s), prev [4][n],
 * yaw_deg [n], sum [4][n], rpm [n][4]. */
void orc_rs_tick(size_t n, float *pos, float *vel, int64_t *prev,
                 const float *yaw_deg, const int64_t *sum, const int16_t *rpm,
                 int trig, int do_correct, int do_predict);

/* ---------------- 6-state linear KF, fp32, same op order as the kernel ----- */
typedef struct {
  float dt, dt2;      /* dt2 = dt*dt computed in fp32 by the caller */
  float q[21];        /* process noise, packed lower triangle, row-major */
  float r[10];        /* measurement noise (theta, omega, vx, vy), packed */
  int   trig;
} orc_kf6_params;

/* x [6][n], P [21][n]; yaw_deg, gyro_z_dps [n]; rpm [n][4]; valid [n] or NULL */
void orc_kf6_tick(size_t n, float *x, float *P, const float *yaw_deg, const float *gyro_z_dps,
                  const int16_t *rpm, const uint8_t *valid, const orc_kf6_params *prm,
                  int do_update, int do_predict, int nthreads);
/* measurement frontend only: z [4][n] */
/* KF6 with FMSKF_CFG_COMP_POS: lo [5][n] = low parts of px, py, P00, P10, P11 */
void orc_kf6_tick_comp(size_t n, float *x, float *P, float *lo, const float *yaw_deg,
                       const float *gyro_z_dps, const int16_t *rpm, const uint8_t *valid,
                       const orc_kf6_params *prm, int do_update, int do_predict, int nthreads);
void orc_kf6_measure(size_t n, const float *yaw_deg, const float *gyro_z_dps,
                     const int16_t *rpm, float *z, int trig);

/* ---------------- 9-state EKF, fp32 --------------------------------------- */
typedef struct {
  float dt, dt2;
  float q[45];
  float r[21];        /* (theta, omega_gyro, ax, ay, vbx, vby) packed */
  int   trig;
} orc_ekf9_params;
/* x [10][n] (the 9 states, then the compensated heading's low part), P [45][n], raw [n][8]
 * int16 words (yaw, gz, ax, ay, rpm FL BL BR FR) */
void orc_ekf9_tick(size_t n, float *x, float *P, const int16_t *raw, const uint8_t *valid,
                   const orc_ekf9_params *prm, int do_update, int do_predict, int nthreads);
/* EKF9 with FMSKF_CFG_COMP_POS: clo [5][n] = low parts of px, py, P00, P10, P11 (NULL: plain) */
void orc_ekf9_tick_comp(size_t n, float *x, float *P, float *clo, const int16_t *raw, const uint8_t *valid,
                        const orc_ekf9_params *prm, int do_update, int do_predict, int nthreads);
void orc_ekf9_measure(size_t n, const int16_t *raw, float *z /*[6][n]*/);

/* ---------------- 12-state linear KF, fp64 -------------------------------- */
typedef struct {
  double dt, dt2;
  double q[78];
  double r[36];
} orc_kf12d_params;
/* Cinv of R = C C^T (packed lower); 0 when R is not positive definite */
int orc_kf12d_cinv(const double *r /*[36]*/, double *ci /*[36]*/);
/* x [12][n], P [78][n], z [8][n] */
void orc_kf12d_tick(size_t n, double *x, double *P, const double *z, const uint8_t *valid,
                    const orc_kf12d_params *prm, int do_update, int do_predict, int nthreads);

/* ---------------- ensemble statistics ------------------------------------ */
/* partial record = {count, mean[n], M2 packed[n(n+1)/2]} (Chan et al.) */
size_t orc_ens_record_len(int nx);
void orc_ens_partial_f32(size_t n, int nx, const float *x /*[nx][n]*/, size_t lo, size_t hi,
                         double *rec);
void orc_ens_partial_f64(size_t n, int nx, const double *x, size_t lo, size_t hi, double *rec);
void orc_ens_combine(int nx, const double *a, const double *b, double *out);
void orc_ens_finalize(int nx, const double *rec, double *mean, double *cov_packed);

/* ---------------- vehicle control step ---------- */
/* UTIL::VelInterpConstJerk (src/Utility/util_vel_interp.hpp:25-157): one active
 * StatusBuf page + the current velocity / acceleration.  The reference's two pages only
 * separate the ISR from the task on the MCU; set_target_params rewrites every field
 * of the inactive page and flips, so one page carries identical semantics. */
typedef struct {
  float vel_tgt, acl_max, jerk_p, jerk_m, dt1, dt2, dt3, vel_ini, acl_ini, dt;
  float vel_now, acl_now;
} orc_interp;
/* UTIL::FF_PI_D state (util_controller.hpp:28-37, 139-149, 170-186); prev_val == now_val
 * after every update, the IIR1's now_Y == prev_Y (util_iir.hpp:39-45) */
typedef struct {
  float val, integ, lpf_y, lpf_x, tgt, ctrl;
} orc_pid;
typedef struct {
  float freq, dt;                /* controller(_c_freq): freq_, dt_ = 1.0f / freq (:10) */
  float ff_gain, p_gain, i_gain, d_gain, i_limit, ff_limit;
  float a1, b0, b1;              /* velLpf_ coefficients (:99-101) */
  float ts;                      /* VelInterpConstJerk sample time */
  int16_t curr_limit_raw;        /* MOTOR_IF_M2006::s16_rawCurr_lim */
} orc_ctrl_params;

/* params from the construction arguments of VD_task_main.cpp:86-97,157-160 (freq 100 Hz,
 * FF 0.0075, P 0.02, I 0.01, D 0, I-limit 0.5, LPF 10 Hz, FF-limit 1, ts 1/1000 s) or any other */
void orc_ctrl_params_make(orc_ctrl_params *p, float c_freq, float ff, float pg, float ig, float dg,
                          float ilim, float lpf_freq, float ff_limit, float ts, int16_t clim);
void  orc_interp_reset(orc_interp *s);
void  orc_interp_set(orc_interp *s, float v_t, float a_m, float jrk);  /* set_target_params */
float orc_interp_update(orc_interp *s, float ts);                     /* update */
void  orc_pid_reset(orc_pid *c);
float orc_pid_update(orc_pid *c, const orc_ctrl_params *p, float nowval);  /* FF_PI_D::update */
/* MOTOR_IF_M2006::set_CurrA_tgt -> set_rawCurr_tgt -> sat_curr (VD_motor_if_m2006.hpp:36-37,59-60) */
int16_t orc_curr_to_raw(float amp, int dir, int16_t lim);
/* CAN_CTRL::tx_routine (VD_can_controller.hpp:43-55): 0x200 payload from 4 raw currents */
void orc_can_tx(const int16_t cur[4], uint8_t out[8]);

/* One robot's control state (VEHICLE_CTRL parts: 3 interpolators, 4 controllers, 4 motor
 * current targets, isPowerOn) and the per-tick step (VD_vehicle_controller.cpp:53-98). */
typedef struct {
  orc_interp ax[3];
  orc_pid    pid[4];
  int16_t    curr[4];
  float      vel_tgt[3];   /* now_vhcl_vel_tgt_mmps */
  uint8_t    power;        /* isPowerOn */
} orc_ctrl;
void orc_ctrl_reset(orc_ctrl *c);
void orc_ctrl_step(orc_ctrl *c, const orc_ctrl_params *p, const int16_t rpm[4], const int8_t dir[4]);
/* batched: ctrl [n], rpm [n][4] */
void orc_ctrl_step_batch(size_t n, orc_ctrl *c, const orc_ctrl_params *p, const int16_t *rpm,
                         const int8_t dir[4]);

/* ---------------- VehicleInfo export ---------------- */
/* RM_task_main.cpp:772-823 -> VehicleInfo.msg / VehiclePosition.msg / ImuInfo.msg /
 * FloorDetection.msg; natural C alignment, 84 bytes */
typedef struct {
  int32_t pos_x, pos_y;    /* (int32_t)(px*1000.0f) [mm] */
  float   pos_theta;       /* [rad] */
  int32_t vel_x, vel_y;    /* (int32_t)vx [mm/s] */
  float   vel_theta;       /* [rad/s] */
  uint8_t imu_fault;       /* 0xFF when is_error (all imu floats 0), else 0 */
  uint8_t pad_[3];
  float   imu_q[4];        /* qx qy qz qw = Data.qut[0..3] */
  float   imu_g[3];        /* Data.gyro */
  float   imu_a[3];        /* Data.accel */
  uint8_t floor[8];        /* right left forward back rightforward leftforward rightback leftback */
  float   cam_pitch;
  uint32_t fault;
} orc_vehicle_info;
/* ARM float -> int32 conversion (VCVT: round toward zero, saturating, NaN -> 0) */
int32_t orc_f2i32_arm(float f);
uint32_t orc_f2u32_arm(float f); /* VCVT.U32.F32: truncate, saturate, NaN -> 0 */
void orc_vehicle_info_fill(orc_vehicle_info *o, float px, float py, float pth, float vx, float vy,
                           float vth, const float imu_data[16], uint8_t is_error,
                           const uint8_t floor[8], float cam_pitch, uint32_t fault);

/* ---------------- timing helper for the CPU baseline --------------------- */
int orc_max_threads(void);

#ifdef __cplusplus
}
#endif
#endif
