/*
 * fmskf.h -- C ABI of the MI355X batched state-estimation engine (libfmskf.so).
 *
 * Drop-in for the IMU + mecanum-odometry fusion path of
 * Moryu-Io/Roboken-FMSKF-robot-controller, batched over N independent robots
 * ("instances").  Every per-tick entry point keeps the reference's per-tick call
 * shape (src/VehicleDrive/VD_task_main.cpp:366-372):
 *
 *     can_tx_routine_intr():  set_now_yaw_world(deg2rad(IMT::get_status_now_yaw()));   -> fmskf_correct
 *                             vhclCtrl.update();                                          -> fmskf_predict
 *                             (fused: fmskf_tick)
 *
 * Plain C: opaque handle, plain pointers and sizes, int status codes, no torch
 * types, no exceptions across the boundary.  All arrays are caller-owned; the
 * library never retains a caller pointer after a call returns.  Arrays are
 * "planes" (structure of arrays): plane k of an array with N instances starts
 * at element k*N.  `mem` says whether the caller's pointers are host
 * (FMSKF_MEM_HOST) or device (FMSKF_MEM_DEVICE, on the handle's device).
 *
 * Tick entry points are asynchronous on the handle's HIP stream
 * (fmskf_set_stream); fmskf_sync waits for them.  One handle per host thread;
 * distinct handles are independent.
 *
 * Reference interfaces replaced (file:line in the reference repository):
 *   IMT::IMU_IF / IMU_IF_WT901C          src/Imu/imu_if_base.hpp:8-32, imu_if_wt901c.hpp:8-42
 *   IMT::get_status_now_yaw / _imu       src/Imu/imu_task_main.cpp:86-104
 *   WIT SDK byte input                   lib/wt901c/wit_c_sdk.c:132-198
 *   VDT::MOTOR_IF_M2006::rx_callback     src/VehicleDrive/VD_motor_if_m2006.cpp:32-72
 *   VDT::VEHICLE_CTRL::set_now_yaw_world src/VehicleDrive/VD_vehicle_controller.hpp:57
 *   VDT::VEHICLE_CTRL::update (odometry) src/VehicleDrive/VD_vehicle_controller.cpp:6-51
 *   VEHICLE_CTRL::get_vehicle_*_latest   src/VehicleDrive/VD_vehicle_controller.hpp:59-60
 *   VDT::get_status_now_vehicle_pos_world/vel  src/VehicleDrive/VD_task_main.cpp:374-395
 *   VEHICLE_CTRL::update (control part)  src/VehicleDrive/VD_vehicle_controller.cpp:53-98
 *   VEHICLE_CTRL::set_target_vel/start/stop  VD_vehicle_controller.cpp:100-104, .hpp:54-55
 *   UTIL::VelInterpConstJerk / FF_PI_D   src/Utility/util_vel_interp.hpp:25-157,
 *                                        util_controller.hpp:92-186, util_iir.hpp:13-57
 *   CAN_CTRL::tx_routine                 src/VehicleDrive/VD_can_controller.hpp:43-55
 *   VehicleInfo publish                  src/RobotManager/RM_task_main.cpp:772-823
 */
#ifndef FMSKF_H_
#define FMSKF_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 3: fmskf_tick_inputs.angle_sum_pitch (the former unchecked `reserved` word), fmskf_config.flags,
 * the asynchronous ensemble entry points, fmskf_comm_info, fmskf_get_motor_status */
#define FMSKF_ABI_VERSION 3u

/* ---- status codes (every entry point returns one) ------------------------ */
#define FMSKF_OK 0
#define FMSKF_EINVAL 1   /* bad argument / shape / state */
#define FMSKF_ENOMEM 2   /* device or host allocation failed */
#define FMSKF_EDEVICE 3  /* HIP error, or no usable GPU */
#define FMSKF_ERCCL 4    /* collective failed (multi-GPU ensemble path) */
#define FMSKF_ENOTSUP 5  /* entry point not valid for this model */

/* ---- models --------------------------------------------------------------- */
/* RS: reference semantics.  State = the firmware's VEHICLE_CTRL pose/velocity.
 *     correct = theta hard overwrite (P == 0, R == 0), predict = the odometry
 *     integrator bit for bit (VD_vehicle_controller.cpp:11-51).
 * KF6:  6-state linear KF (px, py, theta, vx, vy, omega), fp32; z = (theta,
 *       omega, vx_world, vy_world) formed in-kernel from yaw, gyro z, wheel rpm.
 * EKF9: 9-state EKF (px, py, theta, vbx, vby, omega, gyro bias, abx, aby), fp32,
 *       nonlinear mecanum f(); z formed in-kernel from 8 raw int16 words.
 * KF12D: 12-state linear KF in fp64: KF6's base + arm tip (tx, ty, tz, tvx, tvy,
 *       tvz); z = 8 fp64 (theta, omega, vx_w, vy_w, tx, ty, tz, tvz).          */
#define FMSKF_MODEL_RS 0u
#define FMSKF_MODEL_KF6 1u
#define FMSKF_MODEL_EKF9 2u
#define FMSKF_MODEL_KF12D 3u

/* sin/cos policy for util_mymath.hpp:44-45 (arm_sin_f32 / arm_cos_f32) */
#define FMSKF_TRIG_TABLE512 0u /* CMSIS-DSP algorithm: 512-entry table + linear interpolation */
#define FMSKF_TRIG_LIBM 1u     /* device sinf/cosf */

#define FMSKF_MEM_HOST 0u
#define FMSKF_MEM_DEVICE 1u

typedef struct fmskf_ctx *fmskf_handle;

typedef struct fmskf_config {
  uint32_t abi_version;  /* = FMSKF_ABI_VERSION */
  uint32_t model;        /* FMSKF_MODEL_* */
  uint64_t n_instances;  /* N */
  int32_t device;        /* HIP device ordinal */
  uint32_t trig;         /* FMSKF_TRIG_* */
  double dt;             /* tick period [s]; the reference ticks at 1 kHz (VD_task_main.cpp:22,165) */
  /* Noise / initial covariance, packed lower triangle, row-major (k = i*(i+1)/2 + j).
   * Used by the KF models (n = 6, 9, 12; m = 4, 6, 8); ignored by RS. */
  double q[78];
  double r[36];
  double p0[78];
  int8_t motor_dir[4];   /* FL, BL, BR, FR: +1 / -1 (VD_task_main.cpp:75-78) */
  uint32_t imu_read_reg; /* register index for 0x5F REGVALUE frames; init() leaves q0 = 0x51 */
  uint32_t flags;        /* FMSKF_CFG_* (0 = the defaults) */
  uint32_t reserved;     /* must be 0 */
} fmskf_config;

/* KF6, EKF9: carry the open-loop integrals -- px, py and the position block of P (P[0][0],
 * P[1][0], P[1][1]) -- as compensated fp32 pairs (hi + lo; every addition to them a TwoSum), so
 * that they track the float64 filter over long horizons (60 s at 1 kHz within 1e-5, where plain
 * fp32 drifts to 2e-5 - 6e-5).  fmskf_get_state returns hi (hi + lo rounded is hi); the lo parts
 * are readable through fmskf_get_state_lo.  +40 B per robot-tick (KF6 232 -> 272, EKF9 456 ->
 * 496).  Off by default: the plain fp32 filters are the headline and cfg 3. */
#define FMSKF_CFG_COMP_POS 1u

/* Fill defaults for `model` with `n` instances (dt = 1 ms, TABLE512, reference motor
 * directions, model-specific Q/R/P0).  Pure host function (no GPU needed). */
int fmskf_config_init(fmskf_config *cfg, uint32_t model, uint64_t n);

/* ---- lifecycle ------------------------------------------------------------ */
int fmskf_create(const fmskf_config *cfg, fmskf_handle *out);
int fmskf_destroy(fmskf_handle h);
/* Zero-initialised state, as the firmware's static objects at boot
 * (VD_vehicle_controller.hpp:73-77), P = P0 for KF models; the
 * control state too (power off), keeping the control parameters. */
int fmskf_reset(fmskf_handle h);
int fmskf_set_stream(fmskf_handle h, void *hip_stream); /* hipStream_t; NULL = default */
int fmskf_sync(fmskf_handle h);
int fmskf_get_config(fmskf_handle h, fmskf_config *out);
const char *fmskf_strerror(int status);
/* last error message of the calling thread ("" if none) */
const char *fmskf_last_error(void);
int fmskf_abi_version(void);
/* state dimension n, measurement dimension m and state element size for a model */
int fmskf_model_dims(uint32_t model, uint32_t *n, uint32_t *m, uint32_t *elem_bytes);

/* ---- ingest: device boundary --------------------------------------------- */
/* IMU task tick (IMT::main, imu_task_main.cpp:43-82 at 100 Hz): per instance, feed one
 * poll's UART bytes through the WT901 parser (wit_c_sdk.c:132-198), then
 * IMU_IF_WT901C::update (imu_if_wt901c.cpp:83-89): is_error = no quaternion frame
 * since the last good poll; else refresh the Data page (updateData, :91-129).
 * bytes: instance i's bytes at bytes + i*stride, len[i] <= stride.
 * latch_qinit != 0 additionally latches q_init after a good poll (init(), :70-76). */
int fmskf_ingest_wt901(fmskf_handle h, const uint8_t *bytes, uint32_t stride, const uint32_t *len,
                       int latch_qinit, uint32_t mem);

/* CAN RX (VD_can_controller.hpp:65-95 -> MOTOR_IF_M2006::rx_callback): frames [N][4][8]
 * (FL, BL, BR, FR; C610 payload: angle, rpm, current big-endian), stamps [N][4]
 * (int16 us, micros() & 0x7FFF), present [N] bitmask (bit w = wheel w has a frame;
 * NULL = all four).  Updates the device-resident motor state. */
int fmskf_ingest_can(fmskf_handle h, const uint8_t *frames, const int16_t *stamps,
                     const uint8_t *present, uint32_t mem);

/* ---- per tick -------------------------------------------------------------- */
/* One robot's KF6 tick record, 16 bytes: the three KF6 inputs of one robot in one
 * contiguous record (the sensor packet a robot would ship per tick).  Passing records
 * instead of the yaw / gyro / rpm planes lets each lane fetch its inputs with one 16-byte
 * load instead of three (measured 41.6 -> 39.5 us per 2^20-robot tick on MI355X). */
typedef struct fmskf_kf6_record {
  float yaw_deg;     /* IMT::get_status_now_yaw */
  float gyro_z_dps;  /* IMU_IF::Data.gyro[2] */
  int16_t rpm[4];    /* s16_rawSpeedRpm FL, BL, BR, FR */
} fmskf_kf6_record;

/* Inputs of one tick.  Every plane pointer may be NULL: the kernel then reads the
 * device-resident value the ingest entry points produced (full pipeline). */
typedef struct fmskf_tick_inputs {
  uint32_t mem;              /* FMSKF_MEM_HOST or FMSKF_MEM_DEVICE for all pointers below */
  /* plane pitch of angle_sum in elements (single-tick calls; 0 = N, >= N otherwise).  A padded
   * pitch keeps the four sum planes off a power-of-two stride, which aliases in the memory-side
   * cache: the RS tick at 2^20 robots reads [4][2^20] sums measurably slower than [4][2^20 + 512]
   * (fmskf_tick_many takes the plane pitch from tick_stride) */
  uint32_t angle_sum_pitch;
  const float *yaw_deg;      /* [N] IMT::get_status_now_yaw (deg, [-180,180)); RS, KF6 */
  const float *gyro_z_dps;   /* [N] IMU_IF::Data.gyro[2] (deg/s, as published); KF6 */
  const int16_t *rpm;        /* [N][4] Status.s16_rawSpeedRpm FL,BL,BR,FR; RS, KF6 */
  const int64_t *angle_sum;  /* [4][angle_sum_pitch] MOTOR_IF_M2006::get_rawAngleSum; RS */
  const int16_t *raw;        /* [N][8] EKF9 words: Yaw, GZ, AX, AY registers, rpm x4 */
  const double *z;           /* [8][N] KF12D measurements */
  const uint8_t *valid;      /* [N] measurement present (0 = predict only); NULL = all */
  /* KF6 only: [N] records replacing yaw_deg, gyro_z_dps and rpm (which must then be NULL);
   * tick_many: [T][N], advancing by tick_stride records per tick */
  const fmskf_kf6_record *kf6_rec;
} fmskf_tick_inputs;

/* correct: RS -> theta = deg2rad(yaw) (VD_task_main.cpp:368); KF models -> update. */
int fmskf_correct(fmskf_handle h, const fmskf_tick_inputs *in);
/* predict: RS -> VEHICLE_CTRL::update odometry (VD_vehicle_controller.cpp:11-51);
 * KF models -> time update (x <- f(x), P <- F P F^T + Q). */
int fmskf_predict(fmskf_handle h, const fmskf_tick_inputs *in);
/* fused correct-then-predict, one kernel, one pass over the state (the hot path) */
int fmskf_tick(fmskf_handle h, const fmskf_tick_inputs *in);
/* T fused ticks in one launch, state held on chip between ticks.  Inputs are T
 * consecutive tick records: each plane pointer advances by tick_stride elements
 * per tick (tick_stride >= N; for [N][k] planes by tick_stride*k). */
int fmskf_tick_many(fmskf_handle h, const fmskf_tick_inputs *in, uint32_t n_ticks,
                    uint64_t tick_stride);

/* ---- readout --------------------------------------------------------------- */
/* VEHICLE_CTRL::get_vehicle_pos_m_latest (x m, y m, th rad).  Any pointer may be NULL. */
int fmskf_get_pose(fmskf_handle h, float *x, float *y, float *th, uint32_t mem);
/* VEHICLE_CTRL::get_vehicle_vel_mmps_latest (body frame mm/s, mm/s, rad/s) */
int fmskf_get_vel(fmskf_handle h, float *vx, float *vy, float *vth, uint32_t mem);
/* Full model state: x [n][N] and P packed [n(n+1)/2][N] in the model's element type
 * (float, or double for KF12D); RS: x = (x, y, th, vx, vy, vth) floats, P unused.
 * Hidden compensation rows are not part of x / P: EKF9's heading low part and, with
 * FMSKF_CFG_COMP_POS, KF6's position low parts.  get_state returns the hi rows; set_state
 * restarts every low part at 0, so a get_state / set_state round trip is exact only up to the
 * low parts (fmskf_get_state_lo / fmskf_set_state_lo carry them; fmskf_save_state /
 * fmskf_load_state keep everything). */
int fmskf_get_state(fmskf_handle h, void *x, void *p_packed, uint32_t mem);
int fmskf_set_state(fmskf_handle h, const void *x, const void *p_packed, uint32_t mem);
/* The hidden low-part rows [rows][N] float: EKF9's heading (1 row), then with
 * FMSKF_CFG_COMP_POS the 5 rows px, py, P[0][0], P[1][0], P[1][1] (KF6: those 5 only); *rows
 * receives the count (0: the model keeps none, and lo may be NULL).  set_state_lo after
 * set_state restores a handle bit for bit. */
int fmskf_get_state_lo(fmskf_handle h, float *lo, uint32_t *rows, uint32_t mem);
int fmskf_set_state_lo(fmskf_handle h, const float *lo, uint32_t mem);
/* RS: the int64 s64_rawAngleSumPrev [4][N] (VD_vehicle_controller.hpp:75) */
int fmskf_get_prev_sum(fmskf_handle h, int64_t *prev, uint32_t mem);
/* Checkpoint / resume: every per-robot array of the handle (estimator state,
 * RS encoder sums, NaN counters, and the IMU / motor ingest and control state when they
 * exist, with the control parameters) written byte for byte in its device layout, and read
 * back into a handle of the same model, N and ABI; resuming continues bit-identically.
 * Ingest / control state the checkpoint does not hold is reset to its initial value on load.
 * The handle's fmskf_config (noise, geometry) is its own: the saved copy is not applied.
 * Synchronous; EINVAL on I/O errors or a checkpoint that does not match the handle, in which
 * case load leaves the handle's state untouched (lengths are validated before any copy). */
int fmskf_save_state(fmskf_handle h, const char *path);
int fmskf_load_state(fmskf_handle h, const char *path);
/* IMU_IF::Data page [16][N] (accel3, gyro3, mag3, angle3, qut4) of each robot's last successful
 * poll (zeros before one), formed here from the register words that poll left (updateData,
 * imu_if_wt901c.cpp:91-129; the ingest keeps the words, not the page), is_error [N] */
int fmskf_get_imu(fmskf_handle h, float *data, uint8_t *is_error, uint32_t mem);
/* WT901 register file sReg [0x90][N] (int16) and parser bytes pending [N] */
int fmskf_get_imu_regs(fmskf_handle h, int16_t *regs, uint8_t *pending, uint32_t mem);
/* Motor state [N][4]: angle, rpm, curr (int16), angle_sum [4][N] int64,
 * speed_radps [4][N] float (MOTOR_IF_M2006::Status + s64_rawAngleSum) */
int fmskf_get_motors(fmskf_handle h, int16_t *angle, int16_t *rpm, int16_t *curr,
                     int64_t *angle_sum, float *speed_radps, uint32_t mem);
/* MOTOR_IF_M2006::get_status_latest (VD_motor_if_m2006.hpp:23-30,47-50) for every wheel of every
 * robot, [N][4] each (FL, BL, BR, FR): s16_microsec_id, s16_rawAngle, s16_rawSpeedRpm,
 * s16_rawCurr, flt_dltOutAngle_rad (VD_motor_if_m2006.cpp:64: the raw angle difference of the
 * last two frames, not wrap-corrected, as the firmware computes it -- a wheel crossing 8191 -> 0
 * reports about -2*pi/36 rad -- x OUT_RAD_PER_RAW_ANGLE x GEAR_RATIO_INV, formed at readout from
 * the last two angles), flt_SpeedRadPS.  Any pointer may be NULL. */
int fmskf_get_motor_status(fmskf_handle h, int16_t *microsec_id, int16_t *angle, int16_t *rpm,
                           int16_t *curr, float *dlt_out_angle_rad, float *speed_radps, uint32_t mem);
/* counters: [0] = instances whose state went non-finite (NaN/Inf guard); [1] = calls of
 * fmskf_isr_tick_can that ran the CAN RX as a kernel of its own before the ISR (a caller rpm /
 * angle sums / KF6 records, CAN buffers not 16-byte (frames) / 8-byte (stamps) aligned, or a
 * regime where the ISR is not one kernel); [2] = ISRs (fmskf_isr_tick or fmskf_isr_tick_can)
 * that ran as the estimator tick, the control step and the 0x200 frame in three kernels instead
 * of one (KF12D; KF6 / EKF9 past the Infinity Cache).  Results are identical either way; [1] and
 * [2] count since create / reset and are not checkpointed. */
int fmskf_get_counters(fmskf_handle h, uint64_t *counters, uint32_t n_counters);

/* ---- ensemble statistics (mean / covariance of x across instances) --------- */
/* Record layout: {count, mean[n], M2 packed[n(n+1)/2]} in fp64 (28 doubles for n=6).
 * fmskf_ensemble_partial writes this rank's record; ranks all-gather the records
 * (RCCL over xGMI, one process per GPU) and fmskf_ensemble_combine folds them in
 * rank order -> deterministic.  `out` may be host or device per mem.
 * The moment sums are accumulated about a shift vector: robot 0's state when the first
 * record after create / reset / set_state / load_state (or fmskf_graph_begin) is taken.  It
 * stays pinned until the next of those calls, so successive records of one state are bitwise
 * identical; M2 loses relative precision only if the fleet drifts many standard deviations
 * away from that snapshot (reset or set_state takes a new one). */
int fmskf_ensemble_record_len(fmskf_handle h, uint32_t *len);
int fmskf_ensemble_partial(fmskf_handle h, double *out, uint32_t mem);
/* fmskf_tick, then this rank's record of the post-tick state (as fmskf_ensemble_partial) in
 * one call.  KF6, EKF9 and KF12D (tiled state, positive-definite R): one tick kernel that also
 * reduces the state it stores, from registers, to per-block records (cross-lane swaps + DPP,
 * no second pass over x), then the fold; the RS model and the KF12D fallback updates tick,
 * then run the stand-alone record.  Records of one state are bitwise identical
 * whichever call produced them only up to fp64 rounding (same shift, different summation
 * order); each call is bitwise reproducible. */
int fmskf_tick_ensemble(fmskf_handle h, const fmskf_tick_inputs *in, double *out, uint32_t mem);
/* host-side: records [n_records][len] -> mean [n], cov packed [n(n+1)/2] (unbiased) */
int fmskf_ensemble_combine(uint32_t n_state, const double *records, uint32_t n_records,
                           double *mean, double *cov_packed);

/* Native multi-GPU path: one process per GPU, an RCCL communicator owned by
 * the handle, the ensemble record all-gathered over xGMI on the handle's stream.  RCCL
 * (librccl.so.1) is resolved at run time, so the library has no link-time dependency on it;
 * FMSKF_ERCCL when it cannot be loaded or a collective fails.
 *   rank 0: fmskf_comm_unique_id(id); distribute the 128 bytes to every rank (any channel);
 *   every rank: fmskf_comm_init(h, id, rank, world); then fmskf_ensemble_stats(h, ...). */
#define FMSKF_COMM_ID_BYTES 128
int fmskf_comm_unique_id(uint8_t id[FMSKF_COMM_ID_BYTES]);
int fmskf_comm_init(fmskf_handle h, const uint8_t id[FMSKF_COMM_ID_BYTES], int rank, int world);
/* The handle's communicator as RCCL itself reports it (ncclCommCount, ncclCommUserRank);
 * EINVAL when the handle has none. */
int fmskf_comm_info(fmskf_handle h, int *world, int *rank);
/* The file the RCCL entry points were resolved from (dladdr of ncclAllGather), or "" while no
 * communicator call has loaded RCCL yet or when it cannot be loaded.  It never loads RCCL itself,
 * and the string stays valid and unchanged for the life of the process.  FMSKF_RCCL_LIBRARY may
 * name another file for the tests' one-GPU loopback stand-in: the library is accepted only if
 * its dynamic symbol table (read from the file before it is loaded, so a rejected file's
 * constructors never run) exports `fmskf_rccl_stand_in`.  That refuses an RCCL build or another
 * collective library picked up by mistake; it is not a defence against a hostile library, which
 * can export the same marker -- an environment that can set FMSKF_RCCL_LIBRARY can already load
 * code into the process. */
const char *fmskf_rccl_library(void);
/* mean [n], cov packed [n(n+1)/2] (unbiased) over every robot of every rank (the ranks of
 * fmskf_comm_init; without a communicator, this handle's robots): device partial record,
 * ncclAllGather, fold in rank order on the host -> identical on every rank, deterministic. */
int fmskf_ensemble_stats(fmskf_handle h, double *mean, double *cov_packed);

/* Asynchronous form of the same exchange, for callers that keep ticking while the records
 * travel (record fused into the tick, gather on a separate stream overlapping
 * the next tick).  Nothing blocks the host:
 *   fmskf_tick_ensemble_begin: fmskf_tick whose kernel also writes this rank's block records
 *     of the post-tick state (KF6, EKF9, KF12D with a positive-definite R; other models tick,
 *     then run the stand-alone record), on the handle's stream;
 *   fmskf_ensemble_begin: the stand-alone record of the current state (no tick);
 *   the record's fold rides in the next begin's tick kernel (extra blocks past its tick
 *   blocks), or runs ahead of the next fmskf_tick, or at fmskf_ensemble_end when nothing
 *   came first; with a communicator of fmskf_comm_init of more than one rank, ncclAllGather
 *   and the copy of the gathered records to pinned host memory then run on the handle's side
 *   stream (one rank: the gather is the identity, the fold writes the pinned slot).  No tick on
 *   the handle's stream waits for the gather, and no call waits on the host.
 *   fmskf_ensemble_end: waits for the OLDEST pending begin and returns its mean [n] and
 *     covariance packed [n(n+1)/2] (unbiased, rank-order fold: identical on every rank,
 *     deterministic).  EINVAL when nothing is pending.
 * At most four begins may be pending (EINVAL on a fifth).  Every rank must issue the same
 * sequence of begins (it is a collective).  Not valid inside a graph capture. */
int fmskf_tick_ensemble_begin(fmskf_handle h, const fmskf_tick_inputs *in);
int fmskf_ensemble_begin(fmskf_handle h);
int fmskf_ensemble_end(fmskf_handle h, double *mean, double *cov_packed);
/* fmskf_ensemble_end that also returns the robots the gathered records count (the sum of their
 * count rows) and how many records were folded (the communicator's size; 1 without one).  Any
 * pointer may be NULL. */
int fmskf_ensemble_end_count(fmskf_handle h, double *mean, double *cov_packed, double *count,
                             uint32_t *n_records);
/* How long the exchange of the result the last fmskf_ensemble_end / _end_count collected took on
 * the handle's side stream: ncclAllGather of the record plus the copy of the gathered records to
 * pinned host memory, between two timing events recorded around them (ms).  -1 when that result
 * needed no exchange (no communicator, or one of a single rank: the fold wrote the pinned slot
 * itself) or none was collected yet.  Lets an N > 1 run say what its collective costs beside the
 * tick. */
int fmskf_ensemble_exchange_ms(fmskf_handle h, float *ms);

/* ---- vehicle control step -------------------------- */
/* Per-robot control state is allocated on the first call of any entry point below
 * (~250 B per robot); zero-initialised like the firmware's static objects, power off. */
typedef struct fmskf_ctrl_params {
  /* FF_PI_D construction (VD_task_main.cpp:86-89): built for 100 Hz (U32_VD_TASK_CTRL_FREQ_HZ)
   * although stepped by the 1 kHz ISR -- the reference's quirk, kept as the default */
  float ctrl_freq_hz;  /* 100 */
  float ff_gain;       /* 0.0075 */
  float p_gain;        /* 0.02 */
  float i_gain;        /* 0.01 */
  float d_gain;        /* 0.0 */
  float i_limit;       /* 0.5 */
  float lpf_freq_hz;   /* 10 (velocity LPF of PI_D, util_controller.hpp:99-101) */
  float ff_limit;      /* 1.0 (set_FF_limit, VD_task_main.cpp:157-160) */
  float interp_ts;     /* VelInterpConstJerk sample time 1/1000 s (VD_task_main.cpp:95-97) */
  int16_t curr_limit_raw; /* MOTOR_IF_M2006::s16_rawCurr_lim 3000 (VD_motor_if_m2006.hpp:62) */
  int16_t reserved;
} fmskf_ctrl_params;

int fmskf_ctrl_params_init(fmskf_ctrl_params *p);
/* takes effect from the next control step; controller state is kept */
int fmskf_set_ctrl_params(fmskf_handle h, const fmskf_ctrl_params *p);
/* VEHICLE_CTRL::start / stop: on [N] (nonzero = on); NULL = all on */
int fmskf_set_power(fmskf_handle h, const uint8_t *on, uint32_t mem);
/* VEHICLE_CTRL::set_target_vel -> VelInterpConstJerk::set_target_params per axis.
 * vel, acl, jrk: [3][N] planes (x mm/s, y mm/s, th rad/s); mask [N] (NULL = every robot). */
int fmskf_set_target_vel(fmskf_handle h, const float *vel, const float *acl, const float *jrk,
                         const uint8_t *mask, uint32_t mem);
/* The control half of VEHICLE_CTRL::update, one tick: interpolators, conv_Vdir_to_Mdir, the
 * four FF_PI_D loops on the measured wheel speed, set_CurrA_tgt.  rpm [N][4] (FL,BL,BR,FR
 * s16_rawSpeedRpm); NULL = the device motor state fmskf_ingest_can keeps. */
int fmskf_control(fmskf_handle h, const int16_t *rpm, uint32_t mem);
/* CAN_CTRL::tx_routine: frames [N][8] = the 0x200 payload (big-endian raw currents) */
int fmskf_can_tx(fmskf_handle h, uint8_t *frames, uint32_t mem);
/* The firmware ISR in one call (VDT::can_tx_routine_intr, VD_task_main.cpp:366-372): correct,
 * VEHICLE_CTRL::update (estimator time update, then the control half on the same rpm record),
 * M_CAN.tx_routine.  Inputs as fmskf_tick (NULL planes = the device-resident ingest state);
 * frames [N][8] receives the 0x200 payloads (NULL: no frame, the current targets are still
 * kept).  Models RS, KF6 and EKF9 run as ONE kernel (one pass over the estimator state, the
 * tick inputs and the control state; KF6 / EKF9 with their state past the Infinity Cache:
 * three); KF12D runs its tick kernel, then the control step and the frame.  Results are
 * identical to fmskf_tick + fmskf_control + fmskf_can_tx in sequence. */
int fmskf_isr_tick(fmskf_handle h, const fmskf_tick_inputs *in, uint8_t *frames, uint32_t mem);
/* The tick's CAN RX and the ISR in one call: fmskf_ingest_can(h, can_frames, can_stamps, NULL,
 * mem) -- the four C610 frames of every robot present, MOTOR_IF_M2006::rx_callback
 * (VD_motor_if_m2006.cpp) -- then fmskf_isr_tick(h, in, frames, mem).  can_frames [N][4][8],
 * can_stamps [N][4] as fmskf_ingest_can.  Models KF6 (no caller rpm / records in `in`), EKF9
 * (no caller rpm) and RS (no caller rpm / angle sums) run it as ONE kernel: the received rpm
 * (RS: and the new angle sums) feed the estimator (EKF9: the wheel loops only, its measurement
 * is the raw record) and the four wheel loops from registers (otherwise, and where the ISR
 * itself is not one kernel, the two calls run).
 * Results are identical to the two calls in sequence. */
int fmskf_isr_tick_can(fmskf_handle h, const uint8_t *can_frames, const int16_t *can_stamps,
                       const fmskf_tick_inputs *in, uint8_t *frames, uint32_t mem);
/* readout: vel_tgt [3][N] (get_vehicle_vel_tgt_mmps_latest), curr_raw [N][4]
 * (get_rawCurr_tgt), wheel_tgt / wheel_ctrl [4][N] (FF_PI_D get_target / last output), all as
 * the last control step (fmskf_control or an ISR call) left them.  Any pointer may be NULL.
 * The step itself stores only the state its next tick reads and the currents: the first readout
 * (or checkpoint, or fmskf_set_power) after a step forms vel_tgt / wheel_tgt / wheel_ctrl from
 * that state with the step's parameters, one small kernel on the handle's stream; changing the
 * parameters, targets or power flags after a step does not change what this returns. */
int fmskf_get_ctrl(fmskf_handle h, float *vel_tgt, int16_t *curr_raw, float *wheel_tgt,
                   float *wheel_ctrl, uint32_t mem);

/* ---- VehicleInfo export -------------------------------- */
/* The ROS VehicleInfo message as RM_task_main.cpp:772-823 fills it (VehicleInfo.msg,
 * VehiclePosition.msg, ImuInfo.msg, FloorDetection.msg), natural C alignment, 84 bytes. */
typedef struct fmskf_vehicle_info {
  int32_t pos_x, pos_y;   /* (int32_t)(x_m * 1000.0f): truncation, ARM saturation */
  float pos_theta;        /* rad */
  int32_t vel_x, vel_y;   /* (int32_t)(mm/s) */
  float vel_theta;        /* rad/s */
  uint8_t imu_fault;      /* 0xFF when IMU_IF::isError (every imu field 0), else 0 */
  uint8_t pad_[3];
  float imu_q[4];         /* qx qy qz qw = Data.qut[0..3] */
  float imu_g[3];         /* Data.gyro */
  float imu_a[3];         /* Data.accel */
  uint8_t floor[8];       /* right left forward back rightforward leftforward rightback leftback */
  float cam_pitch;
  uint32_t fault;
} fmskf_vehicle_info;

/* out [N] records; floor [N][8], cam_pitch [N], fault [N] come from subsystems outside the
 * path and may be NULL (zero). */
int fmskf_export_vehicle_info(fmskf_handle h, fmskf_vehicle_info *out, const uint8_t *floor,
                              const float *cam_pitch, const uint32_t *fault, uint32_t mem);

/* ---- HIP graph of a per-tick call sequence ------------------------------------- */
/* Record the device work of the entry points called between begin and end (on the handle's
 * stream, which must be a stream set with fmskf_set_stream, not the null stream) into a HIP
 * graph, then replay it: one launch per tick for launch-bound (small-N) fleets.  Only
 * device-pointer calls (FMSKF_MEM_DEVICE, or NULL planes reading the device state) can be
 * captured; a call that needs a host round trip fails during capture.  A new begin
 * replaces the previous graph. */
int fmskf_graph_begin(fmskf_handle h);
int fmskf_graph_end(fmskf_handle h);
int fmskf_graph_launch(fmskf_handle h, uint32_t times);

/* ---- diagnostics ------------------------------------------------------------ */
/* Evaluate the device sin/cos policy on x[n] (device pointers when mem = DEVICE). */
int fmskf_eval_trig(fmskf_handle h, const float *x, float *s, float *c, uint64_t n, uint32_t mem);
/* Per-launch kernel timing with HIP events recorded on the handle's stream around
 * every tick-kernel launch (enable resets the record).  fmskf_last_kernel_ms: the
 * last launch; fmskf_kernel_time_total: sum and count of all launches since
 * enable (waits for the last one).  At most 65536 launches are recorded. */
int fmskf_set_timing(fmskf_handle h, int enable);
int fmskf_last_kernel_ms(fmskf_handle h, float *ms);
int fmskf_kernel_time_total(fmskf_handle h, double *total_ms, uint32_t *count);

#ifdef __cplusplus
}
#endif
#endif /* FMSKF_H_ */
