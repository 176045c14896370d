// kernels_ctrl.hip -- the vehicle control step for gfx950:
// velocity interpolation, inverse kinematics, the four FF_PI_D wheel loops, the C610 current
// frame, and the VehicleInfo export.
//
// One robot per lane over plane-major state (fmskf_internal.hpp CtrlDev).  The control step
// is the control half of VEHICLE_CTRL::update (VD_vehicle_controller.cpp:53-98): every tick
// the three VelInterpConstJerk interpolators advance (util_vel_interp.hpp:106-133) and their
// output goes through conv_Vdir_to_Mdir (:113-118); with the power on each wheel's FF_PI_D
// (util_controller.hpp:104-120,171-177, IIR1 util_iir.hpp:39-45) turns target and measured
// motor speed into a current, narrowed like MOTOR_IF_M2006::set_CurrA_tgt (hpp:36-37,59-60);
// with the power off interpolators and controllers reset and the current is 0.  Every float
// expression keeps the reference's operation order (library built with -ffp-contract=off), so
// results are bit-identical to oracle/fmskf_oracle.c, itself pinned to the reference's own
// FF_PI_D (tests/golden/ctrl_ref.npz).  HBM-bound: ~370 B per robot-tick, no reuse.
#include "can_lane.hpp"
#include "ctrl_lane.hpp"
#include "kf6_lane.hpp"
#include "lane_rs.hpp"

#pragma clang fp contract(off)

namespace fmskf {


// set_target_vel: VEHICLE_CTRL::set_target_vel (VD_vehicle_controller.cpp:100-104) per robot
// with mask[i] != 0 (or all); vel/acl/jrk [3][N] (x mm/s, y mm/s, th rad/s)
__global__ __launch_bounds__(kBlock) void k_ctrl_set_target(CtrlDev c, const float *vel,
                                                            const float *acl, const float *jrk,
                                                            const uint8_t *mask) {
  const uint64_t n = c.n, pp = c.pitch;
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  if (mask && !mask[i]) return;
#pragma unroll
  for (int a = 0; a < 3; a++) {
    Interp s;
    // plane a * kAxF + k of robot i (tiled or planar, ctrl_lane.hpp Planes)
    auto at = [&](int k) -> uint64_t {
      const uint32_t pl = (uint32_t)(a * kAxF + k);
      return FMSKF_CTRL_TILED ? st_at(tile_w<float>(), 0, 3 * kAxF, pl, i) : pl * pp + i;
    };
#pragma unroll
    for (int k = 0; k < kAxF; k++) s.f[k] = c.ax[at(k)];
    interp_set(s, vel[a * n + i], acl[a * n + i], jrk[a * n + i]);
#pragma unroll
    for (int k = 0; k < kAxF; k++) c.ax[at(k)] = s.f[k];
  }
}

// The per-tick control step.  rpm [N][4] int16 (MOTOR_IF_M2006::Status.s16_rawSpeedRpm).
// rstride: robot i's four rpm at rpm + 4 * rstride * i (1: [N][4] planes; 2: the rpm field of
// 16-byte fmskf_kf6_record's)
template <bool SMALL, int CP = 0>
__global__ __launch_bounds__(kBlock) void k_ctrl_step(CtrlDev c, CtrlPrm p, const int16_t *rpm,
                                                      uint32_t rstride) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= (uint32_t)c.n) return;
  const uint2 rw = reinterpret_cast<const uint2 *>(rpm)[(uint64_t)i * rstride];
  CtrlLane<SMALL, CP> L;
  L.load(c, i);
  L.step(c, p, i, rw);
}

// The firmware ISR in one pass (VDT::can_tx_routine_intr, VD_task_main.cpp:366-372), reference
// semantics: correct (theta <- deg2rad(yaw)), VEHICLE_CTRL::update (velocity, odometry, then the
// control half on the same rpm record), M_CAN.tx_routine (the 0x200 frame; skipped when frames is
// NULL).  Every load of both steps is issued before either computes; results are bit-identical
// to fmskf_tick + fmskf_control + fmskf_can_tx in sequence (the same lane functions).
struct IsrRsArgs {
  uint64_t pitch;
  float *x;
  int64_t *prev;  // 64-robot tiles of wheel pairs (lane_rs.hpp rs_prev_at)
  const float *yaw_deg;      // the caller's plane, or the IMU state's Yaw words (yaw_word)
  const int16_t *rpm;
  const int64_t *angle_sum;  // [4][sum_pitch]: the caller's sums, or NULL: the motor state's
  uint64_t sum_pitch;
  const uint32_t *msum_lo;  // the motor state's sums, split (fmskf_internal.hpp m_sum_lo)
  const int32_t *msum_hi;
  const float *sintab;
  uint8_t *frames;
  uint32_t yaw_word;  // TickIn::imu_words bit 0 (fmskf_device.hpp tick_yaw)
};
// CAN (round 5, fmskf_isr_tick_can): the tick's four C610 frames per robot first (can_lane.hpp),
// the new angle sums and rpm handed to the odometry and the wheel loops in registers instead of
// read back from the motor state.
// PS (round 6, CAN only): the previous sums live in the motor state.  When the last predict read
// the motor state's sums and nothing changed them since (the host tracks it: fmskf_ctx
// rs_prev_synced), s64_rawAngleSumPrev equals the sums the CAN lane loads anyway, so the odometry
// takes those and the prev planes are neither read nor written (64 B per robot-tick: 685 -> 621 B);
// the host copies the sums into the prev planes before anything else reads them
// (rs_prev_materialize).  Mrad is the same int64 difference, so the result is bit-identical.
template <bool LIBM, bool SMALL, int CP = 0, bool CAN = false, bool CNT = false, bool PS = false>
__global__ __launch_bounds__(kBlock) void k_isr_rs(IsrRsArgs a, CtrlDev c, CtrlPrm p, CanArgs can) {
  static_assert(CAN || !PS, "the previous sums come from the CAN lane");
  const uint64_t n = c.n, pp = a.pitch;
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= (uint32_t)n) return;
  Can4Lane<CNT, CAN && !PS> cl;  // CNT: the motor state non-temporal (launchers: can_nt); the whole
                                  // new sums only where the odometry needs them (not PS)
  if constexpr (CAN) {  // the block's 256-robot chunk
    const uint32_t hb = __builtin_amdgcn_readfirstlane(i) & ~(uint32_t)(kBlock - 1);
    cl.load(can, hb, i - hb);
  }
  RsLane s;
  s.px = a.x[i];
  s.py = a.x[pp + i];
  s.th = 0.f;  // overwritten by the correct step
  if constexpr (!PS) rs_prev_load(a.prev, i, s.prev);
  const float yaw = tick_yaw(a.yaw_word != 0u, reinterpret_cast<const uint32_t *>(a.yaw_deg)[i]);
  uint2 rw;
  int64_t sum[4];
  if constexpr (!CAN) {
    rw = reinterpret_cast<const uint2 *>(a.rpm)[i];
    if (a.msum_lo) {  // the motor state's sums (wave-uniform)
      motor_sum_load(a.msum_lo, a.msum_hi, i, sum);
    } else {
#pragma unroll
      for (int w = 0; w < 4; w++) sum[w] = a.angle_sum[w * a.sum_pitch + i];
    }
  }
  CtrlLane<SMALL, CP> L;
  L.load(c, i);
  if constexpr (CAN) {
    rw = cl.step(can, true);
    if constexpr (PS) {
      // the previous sums are the stored ones, so sum - prev is this frame's delta: the odometry
      // takes (d, 0), the same int64 difference, without the whole sums
#pragma unroll
      for (int w = 0; w < 4; w++) {
        s.prev[w] = 0;
        sum[w] = cl.d[w];
      }
    } else {
#pragma unroll
      for (int w = 0; w < 4; w++) sum[w] = cl.sm[w];
    }
  }
  rs_tick1<LIBM, true, true>(s, yaw, rw, sum, a.sintab);
  const uint2 cw = L.step(c, p, i, rw);
  a.x[i] = s.px;
  a.x[pp + i] = s.py;
  a.x[2 * pp + i] = s.th;
  a.x[3 * pp + i] = s.vx;
  a.x[4 * pp + i] = s.vy;
  a.x[5 * pp + i] = s.vth;
  if constexpr (!PS) rs_prev_store(a.prev, i, s.prev);
  if (a.frames) reinterpret_cast<uint2 *>(a.frames)[i] = tx_frame(cw);
  if constexpr (CAN) cl.finish(can, true);
}

// The firmware ISR in one pass for the 6-state KF: the KF6 tick (correct with the IMU yaw /
// gyro / wheel velocity, predict), then the control half of VEHICLE_CTRL::update on the same
// rpm, then the 0x200 frame (NULL frames: none).  Lane functions shared with k_kf6t /
// k_ctrl_step / k_can_tx (kf6_lane.hpp, ctrl_lane.hpp): bit-identical to fmskf_tick +
// fmskf_control + fmskf_can_tx in sequence.  One robot per lane, the clamped-index form of
// k_kf6t (lanes past N load instance N-1 and store nothing); every load of both steps is
// issued before either computes.  CPC: the control planes' cache policy.
// CAN (round 5, fmskf_isr_tick_can): the tick's four C610 frames per robot first
// (MOTOR_IF_M2006::rx_callback, can_lane.hpp), their rpm handed to the tick and the wheel loops
// in registers -- the firmware's CAN RX ISR and 1 kHz ISR in one launch, bit-identical to
// fmskf_ingest_can + fmskf_isr_tick
template <class O, int CPC, bool CAN = false, bool CNT = false>
__global__ __launch_bounds__(kBlock) void k_isr_kf6(KfArgs<MdKF6, Kf6Params> a, CtrlDev c, CtrlPrm p,
                                                   uint8_t *frames, CanArgs can) {
  const uint64_t n = a.n;
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  const bool live = i < (uint32_t)n;
  const uint32_t ic = live ? i : (uint32_t)n - 1u;
  Can4Lane<CNT> cl;  // CNT: the motor state non-temporal (launchers: can_nt)
  if constexpr (CAN) {  // the block's 256-robot chunk (every block has a live lane)
    const uint32_t hb = __builtin_amdgcn_readfirstlane(i) & ~(uint32_t)(kBlock - 1);
    cl.load(can, hb, ic - hb);
  }
  float x[6], P[21];
  __shared__ float wtab[O::LIBM ? 1 : kBlock / 64][O::LIBM ? 1 : kWaveTab];
  float *stab = wtab[O::LIBM ? 0 : threadIdx.x >> 6];
  WaveTable<O::LIBM> tv(a.in.sintab);
  kf6_load_state<O>(a.x, a.P, a.pitch, ic, x, P);
  Kf6In m = kf6_load_in<O>(a.in, n, 0, ic);
  CtrlLane<true, CPC> L;
  L.load(c, ic);
  tv.store(stab);
  Kf6Lo<O> lo;  // O::COMP: the position low parts (FMSKF_CFG_COMP_POS)
  kf6_load_lo<O>(a.prm.lo, ic, lo);
  if constexpr (CAN) m.rpm = cl.step(can, live);  // the rpm this tick's frames carried
  kf6_tick1<O>(m, stab, a.prm, x, P, lo);
  if (live) {
    kf6_store_state<O>(a.x, a.P, a.pitch, i, x, P);
    kf6_store_lo<O>(a.prm.lo, i, lo);
  }
  nan_guard(x, P, a.counters, live);
  if (live) {
    const uint2 cw = L.step(c, p, i, m.rpm);
    if (frames) reinterpret_cast<uint2 *>(frames)[i] = tx_frame(cw);
  }
  if constexpr (CAN) cl.finish(can, live);
}

// CAN_CTRL::tx_routine, VD_can_controller.hpp:43-55: frames [N][8], big-endian raw currents
__global__ __launch_bounds__(kBlock) void k_can_tx(const int16_t *curr, uint64_t n, uint8_t *frames) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  reinterpret_cast<uint2 *>(frames)[i] = tx_frame(reinterpret_cast<const uint2 *>(curr)[i]);
}

// VehicleInfo export (RM_task_main.cpp:772-823), 84-byte records (fmskf_vehicle_info).  Each
// lane builds its record in LDS, then the block writes its 256 records as one contiguous
// run of dwords (coalesced), instead of 21 strided stores per lane.
constexpr int kViWords = 21;
struct ImuView {  // the IMU state VehicleInfo reads (the snapshot: fmskf_device.hpp imu_data_page)
  const int16_t *snap;
  const uint32_t *yg;  // the snapshot's Yaw / GZ words (DevState::imu_yg)
  const float *qinit, *qprev;
  const uint8_t *err;
};
__global__ __launch_bounds__(kBlock) void k_vehicle_info(const float *ro, ImuView im, uint64_t n,
                                                         uint32_t *out,
                                                         const uint8_t *floor,
                                                         const float *cam_pitch,
                                                         const uint32_t *fault) {
  __shared__ uint32_t rec[kBlock * kViWords];
  const uint64_t b0 = (uint64_t)blockIdx.x * kBlock;
  const uint64_t i = b0 + threadIdx.x;
  if (i < n) {
    uint32_t *r = rec + threadIdx.x * kViWords;
    const float px = ro[i], py = ro[n + i], pth = ro[2 * n + i];
    const float vx = ro[3 * n + i], vy = ro[4 * n + i], vth = ro[5 * n + i];
    r[0] = (uint32_t)f2i32_arm(px * 1000.0f);
    r[1] = (uint32_t)f2i32_arm(py * 1000.0f);
    r[2] = __builtin_bit_cast(uint32_t, pth);
    r[3] = (uint32_t)f2i32_arm(vx);
    r[4] = (uint32_t)f2i32_arm(vy);
    r[5] = __builtin_bit_cast(uint32_t, vth);
    const bool err = im.err[i] != 0;
    r[6] = err ? 0xFFu : 0u;
    // the Data page (accel 0-2, gyro 3-5, mag 6-8, angle 9-11, qut 12-15) of the last
    // successful poll, formed from its snapshot row; zeros before the first one
    float d[16];
#pragma unroll
    for (int k = 0; k < 16; k++) d[k] = 0.0f;
    uint32_t rw[6];
    snap_row_load(im.snap, i, rw);
    int16_t w[kSnapWords];
    snap_page_words(rw, 0, 0, 0, w);  // (the record takes no magnetometer field)
    if (!err && (w[14] & kSnapValid)) {
      const float *q = (w[14] & kSnapLatched) ? im.qprev : im.qinit;
      const float qi[4] = {q[i], q[n + i], q[2 * n + i], q[3 * n + i]};
      const uint32_t g = im.yg[i];
      imu_data_page(w, imu_yaw_deg(g), imu_gz_dps(g), qi, d);
    }
#pragma unroll
    for (int k = 0; k < 4; k++) r[7 + k] = err ? 0u : __builtin_bit_cast(uint32_t, d[12 + k]);
#pragma unroll
    for (int k = 0; k < 3; k++) r[11 + k] = err ? 0u : __builtin_bit_cast(uint32_t, d[3 + k]);
#pragma unroll
    for (int k = 0; k < 3; k++) r[14 + k] = err ? 0u : __builtin_bit_cast(uint32_t, d[k]);
    if (floor) {
      const uint2 f = reinterpret_cast<const uint2 *>(floor)[i];
      r[17] = f.x;
      r[18] = f.y;
    } else {
      r[17] = r[18] = 0u;
    }
    r[19] = cam_pitch ? __builtin_bit_cast(uint32_t, cam_pitch[i]) : 0u;
    r[20] = fault ? fault[i] : 0u;
  }
  __syncthreads();
  const uint64_t valid = (n - b0) < (uint64_t)kBlock ? (n - b0) : (uint64_t)kBlock;
  const uint32_t words = (uint32_t)valid * kViWords;
  uint32_t *dst = out + b0 * kViWords;
  for (uint32_t k = threadIdx.x; k < words; k += kBlock) dst[k] = rec[k];
}

static inline dim3 grid1(uint64_t n) { return dim3((unsigned)((n + kBlock - 1) / kBlock)); }

int launch_ctrl_set_target(const CtrlDev &c, const float *vel, const float *acl, const float *jrk,
                           const uint8_t *mask, hipStream_t st) {
  if (c.n == 0) return 0;
  k_ctrl_set_target<<<grid1(c.n), kBlock, 0, st>>>(c, vel, acl, jrk, mask);
  return (int)hipGetLastError();
}

int launch_ctrl_step(const CtrlDev &c, const CtrlPrm &p, const int16_t *rpm, uint32_t rstride,
                     hipStream_t st) {
  if (c.n == 0) return 0;
  if (c.pitch * 4 * 3 * kAxF < 0xFFFFFFFFull && state_nt(ctrl_state_bytes(c)))
    // 3 blocks per CU (48 KiB dynamic LDS): 2^22 239.4-239.5 -> 235.9-237.0 us
    k_ctrl_step<true, kStateNT><<<grid1(c.n), kBlock, FMSKF_LDS_CAP("FMSKF_CTRL_LDS", true, 48u * 1024u), st>>>(c, p, rpm, rstride);
  else if (c.pitch * 4 * 3 * kAxF < 0xFFFFFFFFull)
    k_ctrl_step<true><<<grid1(c.n), kBlock, 0, st>>>(c, p, rpm, rstride);
  else
    k_ctrl_step<false><<<grid1(c.n), kBlock, 0, st>>>(c, p, rpm, rstride);
  return (int)hipGetLastError();
}

// the step outputs nothing reads back, formed when a reader needs them (ctrl_lane.hpp
// ctrl_derive_lane; host: fmskf_ctx::ctrl_derived_stale)
template <bool SMALL>
__global__ __launch_bounds__(kBlock) void k_ctrl_derive(CtrlDev c, CtrlPrm p) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= (uint32_t)c.n) return;
  ctrl_derive_lane<SMALL>(c, p, i);
}

int launch_ctrl_derive(const CtrlDev &c, const CtrlPrm &p, hipStream_t st) {
  if (c.n == 0) return 0;
  if (c.pitch * 4 * 3 * kAxF < 0xFFFFFFFFull) k_ctrl_derive<true><<<grid1(c.n), kBlock, 0, st>>>(c, p);
  else k_ctrl_derive<false><<<grid1(c.n), kBlock, 0, st>>>(c, p);
  return (int)hipGetLastError();
}

template <bool CAN, bool CNT = false, bool PS = false>
static int isr_rs_l(const DevState &s, const TickIn &in, bool libm, const CtrlDev &c, const CtrlPrm &p,
                    uint8_t *frames, hipStream_t st, const CanArgs &can) {
  if (c.n == 0) return 0;
  const IsrRsArgs a{s.pitch, (float *)s.x, s.prev_sum, in.yaw_deg, in.rpm, in.angle_sum, in.sum_pitch,
                    in.msum_lo, in.msum_hi, in.sintab, frames, in.imu_words & 1u};
  const bool small = c.pitch * 4 * 3 * kAxF < 0xFFFFFFFFull;
  const bool nt = small && state_nt(ctrl_state_bytes(c) + s.n * 56);
  if (nt) {
    // 3 blocks per CU (48 KiB dynamic LDS): 2^20 75.7-76.5 -> 73.9 us (two passes)
    const unsigned lds = FMSKF_LDS_CAP("FMSKF_ISR_LDS", true, 48u * 1024u);
    if (libm) k_isr_rs<true, true, kStateNT, CAN, CNT, PS><<<grid1(c.n), kBlock, lds, st>>>(a, c, p, can);
    else k_isr_rs<false, true, kStateNT, CAN, CNT, PS><<<grid1(c.n), kBlock, lds, st>>>(a, c, p, can);
  } else if (libm) {
    if (small) k_isr_rs<true, true, 0, CAN, CNT, PS><<<grid1(c.n), kBlock, 0, st>>>(a, c, p, can);
    else k_isr_rs<true, false, 0, CAN, CNT, PS><<<grid1(c.n), kBlock, 0, st>>>(a, c, p, can);
  } else {
    if (small) k_isr_rs<false, true, 0, CAN, CNT, PS><<<grid1(c.n), kBlock, 0, st>>>(a, c, p, can);
    else k_isr_rs<false, false, 0, CAN, CNT, PS><<<grid1(c.n), kBlock, 0, st>>>(a, c, p, can);
  }
  return (int)hipGetLastError();
}

int launch_isr_rs(const DevState &s, const TickIn &in, bool libm, const CtrlDev &c,
                  const CtrlPrm &p, uint8_t *frames, hipStream_t st) {
  return isr_rs_l<false>(s, in, libm, c, p, frames, st, CanArgs{});
}

// The fused KF6 ISR where it applies: one tick of the default single-tick form (state in one
// 4 GiB window, cached, not the two-robot cache-resident kernel's layout question: one robot
// per lane), the control planes in one window.  Returns hipErrorNotSupported otherwise (the
// caller then runs the three kernels).  Past the Infinity Cache (KF6 state + control state
// > 256 MiB) the control planes are non-temporal, as in k_isr_rs.
template <bool LIBM, bool VALID, bool REC, bool COMP>
static int isr_kf6_v(const KfArgs<MdKF6, Kf6Params> &a, const CtrlDev &c, const CtrlPrm &p, uint8_t *frames,
                     bool nt, hipStream_t st, const CanArgs *can) {
  using O = Opt<LIBM, true, true, true, VALID, REC, false, false, COMP>;
  const unsigned lds = nt ? FMSKF_LDS_CAP("FMSKF_ISR_LDS", true, 48u * 1024u) : 0u;
  if constexpr (!REC) {  // with CAN the rpm comes from the frames, so the inputs are planes
    if (can && can_nt_flag(*can)) {
      if (nt) k_isr_kf6<O, kStateNT, true, true><<<grid1(c.n), kBlock, lds, st>>>(a, c, p, frames, *can);
      else k_isr_kf6<O, 0, true, true><<<grid1(c.n), kBlock, 0, st>>>(a, c, p, frames, *can);
      return (int)hipGetLastError();
    }
    if (can) {
      if (nt) k_isr_kf6<O, kStateNT, true><<<grid1(c.n), kBlock, lds, st>>>(a, c, p, frames, *can);
      else k_isr_kf6<O, 0, true><<<grid1(c.n), kBlock, 0, st>>>(a, c, p, frames, *can);
      return (int)hipGetLastError();
    }
  }
  if (can) return (int)hipErrorNotSupported;
  if (nt) k_isr_kf6<O, kStateNT><<<grid1(c.n), kBlock, lds, st>>>(a, c, p, frames, CanArgs{});
  else k_isr_kf6<O, 0><<<grid1(c.n), kBlock, 0, st>>>(a, c, p, frames, CanArgs{});
  return (int)hipGetLastError();
}

template <bool COMP>
static int isr_kf6_c(const KfArgs<MdKF6, Kf6Params> &a, const CtrlDev &c, const CtrlPrm &p, uint8_t *frames, bool nt,
                     hipStream_t st, bool libm, bool valid, bool rec, const CanArgs *can) {
  if (libm) {
    if (valid) return rec ? isr_kf6_v<true, true, true, COMP>(a, c, p, frames, nt, st, can)
                          : isr_kf6_v<true, true, false, COMP>(a, c, p, frames, nt, st, can);
    return rec ? isr_kf6_v<true, false, true, COMP>(a, c, p, frames, nt, st, can)
               : isr_kf6_v<true, false, false, COMP>(a, c, p, frames, nt, st, can);
  }
  if (valid) return rec ? isr_kf6_v<false, true, true, COMP>(a, c, p, frames, nt, st, can)
                        : isr_kf6_v<false, true, false, COMP>(a, c, p, frames, nt, st, can);
  return rec ? isr_kf6_v<false, false, true, COMP>(a, c, p, frames, nt, st, can)
             : isr_kf6_v<false, false, false, COMP>(a, c, p, frames, nt, st, can);
}

static int isr_kf6_l(const DevState &s, const TickIn &in, const Kf6Params &kp, bool libm, const CtrlDev &c,
                     const CtrlPrm &p, uint8_t *frames, hipStream_t st, const CanArgs *can) {
  if (c.n == 0) return 0;
  const bool small_state = s.pitch * 84 < 0xFFFFFFFFull;
  const bool small_ctrl = c.pitch * 4 * 3 * kAxF < 0xFFFFFFFFull;
  // the tick kernel alone streams its state non-temporal past the cache: keep that regime on
  // the three-kernel path (its own occupancy caps)
  // KF6 state bytes per robot (FMSKF_CFG_COMP_POS: + the position low parts)
  const uint64_t sb = kp.lo ? 128 : 108;
  if (!small_state || !small_ctrl || state_nt(s.n * sb)) return (int)hipErrorNotSupported;
  const KfArgs<MdKF6, Kf6Params> a{s.n, s.pitch, (float *)s.x, (float *)s.P, in, s.counters, kp};
  const bool nt = state_nt(ctrl_state_bytes(c) + s.n * sb);
  const bool valid = in.valid != nullptr, rec = in.rec != nullptr;
  return kp.lo ? isr_kf6_c<true>(a, c, p, frames, nt, st, libm, valid, rec, can)
               : isr_kf6_c<false>(a, c, p, frames, nt, st, libm, valid, rec, can);
}

int launch_isr_kf6(const DevState &s, const TickIn &in, const Kf6Params &kp, bool libm, const CtrlDev &c,
                   const CtrlPrm &p, uint8_t *frames, hipStream_t st) {
  return isr_kf6_l(s, in, kp, libm, c, p, frames, st, nullptr);
}

// fmskf_isr_tick_can: the CAN RX of the tick's frames (every wheel present) fused into the KF6
// ISR.  hipErrorNotSupported where the fused form does not apply (record inputs, the tick's
// non-temporal regime, the motor state past the cached regime or its sum planes past 4 GiB,
// unaligned frames / stamps): the caller then runs CAN RX and the ISR as two calls
int launch_isr_kf6_can(const DevState &s, const TickIn &in, const Kf6Params &kp, bool libm, const CtrlDev &c,
                       const CtrlPrm &p, uint8_t *frames, const uint8_t *can_frames, const int16_t *can_stamps,
                       const int8_t dir[4], hipStream_t st) {
  CanArgs ca;
  if (in.rec || !can_args(s, can_frames, can_stamps, dir, ca)) return (int)hipErrorNotSupported;
  ca.nt = can_nt(s);
  return isr_kf6_l(s, in, kp, libm, c, p, frames, st, &ca);
}

// the reference-semantics ISR with the tick's CAN RX fused in: the odometry reads the new sums
// and rpm from the CAN lane (the caller passes no rpm / sums: TickIn's are the motor state's).
// prev_in_sums: the previous sums equal the motor state's stored sums (k_isr_rs PS)
int launch_isr_rs_can(const DevState &s, const TickIn &in, bool libm, const CtrlDev &c, const CtrlPrm &p,
                      uint8_t *frames, const uint8_t *can_frames, const int16_t *can_stamps, const int8_t dir[4],
                      bool prev_in_sums, hipStream_t st) {
  CanArgs ca;
  if (!can_args(s, can_frames, can_stamps, dir, ca)) return (int)hipErrorNotSupported;
  if (prev_in_sums) {
    if (can_nt(s)) return isr_rs_l<true, true, true>(s, in, libm, c, p, frames, st, ca);
    return isr_rs_l<true, false, true>(s, in, libm, c, p, frames, st, ca);
  }
  if (can_nt(s)) return isr_rs_l<true, true>(s, in, libm, c, p, frames, st, ca);
  return isr_rs_l<true>(s, in, libm, c, p, frames, st, ca);
}

int launch_can_tx(const CtrlDev &c, uint8_t *frames, hipStream_t st) {
  if (c.n == 0) return 0;
  k_can_tx<<<grid1(c.n), kBlock, 0, st>>>(c.curr, c.n, frames);
  return (int)hipGetLastError();
}

int launch_vehicle_info(const DevState &s, const float *readout, void *out, const uint8_t *floor,
                        const float *cam_pitch, const uint32_t *fault, hipStream_t st) {
  if (s.n == 0) return 0;
  const ImuView im{s.imu_snap, s.imu_yg, s.imu_qinit, s.imu_qprev, s.imu_err};
  k_vehicle_info<<<grid1(s.n), kBlock, 0, st>>>(readout, im, s.n, (uint32_t *)out, floor, cam_pitch, fault);
  return (int)hipGetLastError();
}

}  // namespace fmskf
