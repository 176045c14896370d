// api_ctrl.cpp -- vehicle control step, CAN TX, the fused firmware ISR, VehicleInfo export,
// the trig evaluator and per-launch timing.
#include "api_ctx.hpp"

using namespace fmskf;
using namespace fmskf::capi;

// ============================================================================
// vehicle control step, CAN TX, VehicleInfo export
// ============================================================================
namespace {

void ctrl_params_defaults(fmskf_ctrl_params *p) {
  memset(p, 0, sizeof(*p));
  p->ctrl_freq_hz = 100.0f;  // U32_VD_TASK_CTRL_FREQ_HZ (VD_task_main.cpp:23,86-89)
  p->ff_gain = 0.0075f;
  p->p_gain = 0.02f;
  p->i_gain = 0.01f;
  p->d_gain = 0.0f;
  p->i_limit = 0.5f;
  p->lpf_freq_hz = 10.0f;
  p->ff_limit = 1.0f;                            // VD_task_main.cpp:157-160
  p->interp_ts = 1.0f / (float)1000;             // VD_task_main.cpp:95-97
  p->curr_limit_raw = 3000;                      // VD_motor_if_m2006.hpp:62
}

// the device parameter block, computed like the reference's constructors
// (util_controller.hpp:10,96-101: dt_ = 1.0f / freq, the IIR1 coefficients in float)
CtrlPrm make_ctrl_prm(const fmskf_ctx *h) {
  const fmskf_ctrl_params &c = h->cprm;
  CtrlPrm p{};
  p.freq = c.ctrl_freq_hz;
  p.dt = 1.0f / c.ctrl_freq_hz;
  p.ff_gain = c.ff_gain;
  p.p_gain = c.p_gain;
  p.i_gain = c.i_gain;
  p.d_gain = c.d_gain;
  p.i_limit = c.i_limit;
  p.ff_limit = c.ff_limit;
  p.a1 = (2.0f * c.ctrl_freq_hz - c.lpf_freq_hz) / (2.0f * c.ctrl_freq_hz + c.lpf_freq_hz);
  p.b0 = c.lpf_freq_hz / (2.0f * c.ctrl_freq_hz + c.lpf_freq_hz);
  p.b1 = c.lpf_freq_hz / (2.0f * c.ctrl_freq_hz + c.lpf_freq_hz);
  p.ts = c.interp_ts;
  p.curr_limit = c.curr_limit_raw;
  for (int w = 0; w < 4; w++) p.dir[w] = h->cfg.motor_dir[w];
  return p;
}

// the parameter block of a control-step launch: outside a capture the step leaves its derived
// outputs to be formed on demand, with these parameters (ctrl_materialize); inside one it stores
// them itself
CtrlPrm ctrl_step_prm(fmskf_ctx *h) {
  CtrlPrm p = make_ctrl_prm(h);
  p.store_derived = h->capturing ? 1u : 0u;
  if (h->capturing) {
    h->graph_has_ctrl = true;
  } else {
    h->ctrl_prm_last = p;
    h->ctrl_derived_stale = true;
  }
  return p;
}

}  // namespace

namespace fmskf {
namespace capi {

void ctrl_materialize(fmskf_ctx *h) {
  if (!h->ctrl_ready || !h->ctrl_derived_stale) return;
  launch_check(launch_ctrl_derive(h->ctrl, h->ctrl_prm_last, h->stream), "control outputs");
  h->ctrl_derived_stale = false;
}

void zero_ctrl(fmskf_ctx *h) {
  CtrlDev &c = h->ctrl;
  hip_check(hipMemsetAsync(c.ax, 0, (size_t)3 * kAxF * c.pitch * 4, h->stream), "ctrl init");
  hip_check(hipMemsetAsync(c.pid, 0, (size_t)4 * kPidF * c.pitch * 4, h->stream), "ctrl init");
  hip_check(hipMemsetAsync(c.vel_tgt, 0, (size_t)3 * c.pitch * 4, h->stream), "ctrl init");
  hip_check(hipMemsetAsync(c.rpm_prev, 0, (size_t)4 * c.n * 2, h->stream), "ctrl init");
  hip_check(hipMemsetAsync(c.curr, 0, (size_t)4 * c.n * 2, h->stream), "ctrl init");
  hip_check(hipMemsetAsync(c.power, 0, (size_t)c.n, h->stream), "ctrl init");
  ctrl_params_defaults(&h->cprm);
  h->ctrl_derived_stale = false;
}

void ensure_ctrl(fmskf_ctx *h) {
  if (h->ctrl_ready) return;
  CtrlDev &c = h->ctrl;
  c.n = h->s.n;
  // tiled interpolator / FF_PI_D arrays cover ceil(N / W) whole tiles (ctrl_lane.hpp Planes)
  const uint64_t w = tile_w_elem(4);
  c.pitch = FMSKF_CTRL_TILED ? std::max(h->s.pitch, (c.n + w - 1) / w * w) : h->s.pitch;
  c.ax = h->alloc<float>((size_t)3 * kAxF * c.pitch);
  c.pid = h->alloc<float>((size_t)4 * kPidF * c.pitch);
  c.vel_tgt = h->alloc<float>((size_t)3 * c.pitch);
  c.rpm_prev = h->alloc<int16_t>((size_t)4 * c.n);
  c.curr = h->alloc<int16_t>((size_t)4 * c.n);
  c.power = h->alloc<uint8_t>((size_t)c.n);
  zero_ctrl(h);
  h->ctrl_ready = true;
}

}  // namespace capi
}  // namespace fmskf

extern "C" {

int fmskf_ctrl_params_init(fmskf_ctrl_params *p) {
  return guarded([&] {
    if (!p) fail(FMSKF_EINVAL, "null params");
    ctrl_params_defaults(p);
  });
}

int fmskf_set_ctrl_params(fmskf_handle h, const fmskf_ctrl_params *p) {
  return guarded([&] {
    check_handle(h);
    if (!p) fail(FMSKF_EINVAL, "null params");
    if (!(p->ctrl_freq_hz > 0.0f) || !(p->interp_ts > 0.0f) || p->curr_limit_raw < 0)
      fail(FMSKF_EINVAL, "ctrl params: freq and ts must be > 0, current limit >= 0");
    DeviceGuard g(h->cfg.device);
    ensure_ctrl(h);
    h->cprm = *p;
  });
}

int fmskf_set_power(fmskf_handle h, const uint8_t *on, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    ensure_ctrl(h);
    ctrl_materialize(h);  // the last step's outputs are formed with the power flags it ran with
    const uint64_t n = h->s.n;
    if (!on) {
      hip_check(hipMemsetAsync(h->ctrl.power, 1, n, h->stream), "power");
      return;
    }
    if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
    hip_check(hipMemcpyAsync(h->ctrl.power, on, n,
                             mem == FMSKF_MEM_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice,
                             h->stream),
              "power");
    finish_out(h, mem);  // the caller's host buffer may be reused on return
  });
}

int fmskf_set_target_vel(fmskf_handle h, const float *vel, const float *acl, const float *jrk,
                         const uint8_t *mask, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (!vel || !acl || !jrk) fail(FMSKF_EINVAL, "null vel/acl/jrk");
    DeviceGuard g(h->cfg.device);
    ensure_ctrl(h);
    const uint64_t n = h->s.n;
    Stager sg(h, mem);
    const void *v = vel, *a = acl, *j = jrk, *m = mask;
    sg.add(&v, 3 * n * 4);
    sg.add(&a, 3 * n * 4);
    sg.add(&j, 3 * n * 4);
    sg.add(&m, n);
    sg.run();
    launch_check(launch_ctrl_set_target(h->ctrl, (const float *)v, (const float *)a,
                                        (const float *)j, (const uint8_t *)m, h->stream),
                 "set_target_vel launch");
  });
}

int fmskf_control(fmskf_handle h, const int16_t *rpm, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    ensure_ctrl(h);
    const void *r = rpm;
    if (r) {
      Stager sg(h, mem);
      sg.add(&r, h->s.n * 8);
      sg.run();
    } else {
      ensure_motors(h);
      r = h->s.m_rpm;
    }
    h->time_begin();
    launch_check(launch_ctrl_step(h->ctrl, ctrl_step_prm(h), (const int16_t *)r, 1, h->stream),
                 "control launch");
    h->time_end();
  });
}

int fmskf_can_tx(fmskf_handle h, uint8_t *frames, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (!frames) fail(FMSKF_EINVAL, "null frames");
    if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
    DeviceGuard g(h->cfg.device);
    ensure_ctrl(h);
    const size_t bytes = h->s.n * 8;
    uint8_t *dst = mem == FMSKF_MEM_DEVICE ? frames : (uint8_t *)host_result(h, bytes);
    launch_check(launch_can_tx(h->ctrl, dst, h->stream), "can_tx launch");
    copy_out_sync(h, frames, dst, bytes, mem);
  });
}

// FMSKF_ISR_FUSED=0: the KF6 and EKF9 ISRs as three kernels (A/B, and the tests' cross-check)
// FMSKF_RS_PREV_SKIP=0: the fused RS CAN ISR always reads and writes the prev planes (A/B)
static bool rs_prev_skip() {
  static const bool v = [] {
    const char *e = getenv("FMSKF_RS_PREV_SKIP");
    return !e || atoi(e) != 0;
  }();
  return v;
}

static bool isr_kf6_fused() {
  static const bool v = [] {
    const char *e = getenv("FMSKF_ISR_FUSED");
    return !e || atoi(e) != 0;
  }();
  return v;
}

// the ISR's launches for resolved inputs `t` (frames into `dst`, or none)
static void isr_launches(fmskf_ctx *h, const TickIn &t, uint8_t *dst) {
  const bool libm = h->cfg.trig == FMSKF_TRIG_LIBM;
  const CtrlPrm p = ctrl_step_prm(h);
  int fused = (int)hipErrorNotSupported;
  if (h->cfg.model == FMSKF_MODEL_KF6 && isr_kf6_fused()) {
    if (!t.rec && !t.rpm) ensure_motors(h);
    fused = launch_isr_kf6(h->s, t, h->kf6, libm, h->ctrl, p, dst, h->stream);
    if (fused != (int)hipErrorNotSupported) launch_check(fused, "isr launch");
  } else if (h->cfg.model == FMSKF_MODEL_EKF9 && isr_kf6_fused()) {
    if (!t.rpm) ensure_motors(h);
    fused = launch_isr_ekf9(h->s, t, h->ekf9, libm, h->ctrl, p, t.rpm ? t.rpm : h->s.m_rpm, dst, h->stream);
    if (fused != (int)hipErrorNotSupported) launch_check(fused, "isr launch");
  }
  if (h->cfg.model == FMSKF_MODEL_RS) {
    rs_prev_materialize(h);
    launch_check(launch_isr_rs(h->s, t, libm, h->ctrl, p, dst, h->stream), "isr launch");
    h->rs_prev_synced = t.msum_lo != nullptr;
  } else if (fused == (int)hipErrorNotSupported) {  // estimator tick, then the control step and the frame (three launches)
    h->isr_ctrl_split++;
    int e = 0;
    switch (h->cfg.model) {
      case FMSKF_MODEL_KF6: e = launch_kf6(h->s, t, h->kf6, libm, true, true, h->stream); break;
      case FMSKF_MODEL_EKF9: e = launch_ekf9(h->s, t, h->ekf9, libm, true, true, h->stream); break;
      case FMSKF_MODEL_KF12D: e = launch_kf12d(h->s, t, h->kf12, true, true, h->stream); break;
    }
    launch_check(e, "tick kernel launch");
    if (!t.rec && !t.rpm) ensure_motors(h);
    const int16_t *rpm = t.rec ? (const int16_t *)(t.rec + 2) : t.rpm ? t.rpm : h->s.m_rpm;
    launch_check(launch_ctrl_step(h->ctrl, p, rpm, t.rec ? 2 : 1, h->stream), "control launch");
    if (dst) launch_check(launch_can_tx(h->ctrl, dst, h->stream), "can_tx launch");
  }
}

int fmskf_isr_tick(fmskf_handle h, const fmskf_tick_inputs *in, uint8_t *frames, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (frames && mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
    DeviceGuard g(h->cfg.device);
    ensure_ctrl(h);
    const uint64_t n = h->s.n;
    const TickIn t = resolve_inputs(h, in, true, true, 1, n);
    const size_t bytes = n * 8;
    uint8_t *dst = !frames ? nullptr : mem == FMSKF_MEM_DEVICE ? frames : (uint8_t *)host_result(h, bytes);
    h->time_begin();
    isr_launches(h, t, dst);
    h->time_end();
    if (frames) copy_out_sync(h, frames, dst, bytes, mem);
  });
}

int fmskf_isr_tick_can(fmskf_handle h, const uint8_t *can_frames, const int16_t *can_stamps,
                       const fmskf_tick_inputs *in, uint8_t *frames, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (!can_frames || !can_stamps) fail(FMSKF_EINVAL, "null can_frames/can_stamps");
    if (!in) fail(FMSKF_EINVAL, "null inputs");
    if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
    DeviceGuard g(h->cfg.device);
    ensure_ctrl(h);
    ensure_motors(h);
    const uint64_t n = h->s.n;
    const void *f = can_frames, *s = can_stamps;
    std::vector<std::pair<const void **, size_t>> cf{{&f, n * 32}, {&s, n * 8}};
    // one staging round for the CAN frames and the tick inputs when they share a mem flag
    const bool together = in->mem == mem;
    const TickIn t = resolve_inputs(h, in, true, true, 1, n, together ? &cf : nullptr);
    if (!together) {
      Stager sg(h, mem);
      for (const auto &it : cf) sg.add(it.first, it.second);
      sg.run();
    }
    const bool libm = h->cfg.trig == FMSKF_TRIG_LIBM;
    const size_t bytes = n * 8;
    uint8_t *dst = !frames ? nullptr : mem == FMSKF_MEM_DEVICE ? frames : (uint8_t *)host_result(h, bytes);
    int fused = (int)hipErrorNotSupported;
    h->time_begin();
    // one launch where the tick reads the rpm (RS: and the angle sums) the frames carry: no
    // caller rpm / sums / records
    if (h->cfg.model == FMSKF_MODEL_KF6 && isr_kf6_fused() && !in->kf6_rec && !in->rpm) {
      fused = launch_isr_kf6_can(h->s, t, h->kf6, libm, h->ctrl, ctrl_step_prm(h), dst, (const uint8_t *)f,
                                 (const int16_t *)s, h->cfg.motor_dir, h->stream);
    } else if (h->cfg.model == FMSKF_MODEL_EKF9 && isr_kf6_fused() && !in->rpm) {
      fused = launch_isr_ekf9_can(h->s, t, h->ekf9, libm, h->ctrl, ctrl_step_prm(h), dst, (const uint8_t *)f,
                                  (const int16_t *)s, h->cfg.motor_dir, h->stream);
    } else if (h->cfg.model == FMSKF_MODEL_RS && !in->rpm && !in->angle_sum) {
      // the previous sums are the stored ones: take them from the CAN lane, skip the prev planes
      // (not inside a capture: a replay may start from another state)
      const bool ps = h->rs_prev_synced && !h->capturing && rs_prev_skip();
      if (!ps) rs_prev_materialize(h);
      fused = launch_isr_rs_can(h->s, t, libm, h->ctrl, ctrl_step_prm(h), dst, (const uint8_t *)f,
                                (const int16_t *)s, h->cfg.motor_dir, ps, h->stream);
      if (fused != (int)hipErrorNotSupported) {
        h->rs_prev_synced = true;  // the odometry's previous sums are the new motor sums
        h->rs_prev_stale = h->rs_prev_stale || ps;
      }
    }
    if (fused != (int)hipErrorNotSupported) {
      launch_check(fused, "isr+can launch");
      h->s.m_par ^= 1u;  // the frames' stamps and angles went over the older history slots
    }
    if (fused == (int)hipErrorNotSupported) {  // CAN RX, then the ISR of fmskf_isr_tick
      h->isr_can_split++;
      rs_prev_materialize(h);  // the CAN RX rewrites the motor sums
      h->rs_prev_synced = false;
      launch_check(launch_can(h->s, (const uint8_t *)f, (const int16_t *)s, nullptr, h->cfg.motor_dir, h->stream),
                   "can launch");
      h->s.m_par ^= 1u;
      isr_launches(h, t, dst);
    }
    h->time_end();
    if (frames) copy_out_sync(h, frames, dst, bytes, mem);
  });
}

int fmskf_get_ctrl(fmskf_handle h, float *vel_tgt, int16_t *curr_raw, float *wheel_tgt,
                   float *wheel_ctrl, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    ensure_ctrl(h);
    ctrl_materialize(h);
    const CtrlDev &c = h->ctrl;
    const size_t row = c.n * 4, pb = c.pitch * 4;
    copy_planes_out(h, vel_tgt, c.vel_tgt, row, pb, 3, mem);
    copy_out(h, curr_raw, c.curr, c.n * 8, mem);
    // wheel w's field k is plane w*kPidF + k: planes of one field are kPidF planes apart
    const float *pid = c.pid;
    size_t ppb = pb;
    if (FMSKF_CTRL_TILED && (wheel_tgt || wheel_ctrl)) {  // dense [4 * kPidF][N] copy first
      float *dense = (float *)h->stage_for((size_t)4 * kPidF * row);
      launch_check(launch_untile(c.pid, dense, 4 * kPidF, c.n, 4, h->stream), "untile pid");
      pid = dense;
      ppb = row;
    }
    copy_planes_out(h, wheel_tgt, pid + 4 * (ppb / 4), row, ppb * kPidF, 4, mem);
    copy_planes_out(h, wheel_ctrl, pid + 5 * (ppb / 4), row, ppb * kPidF, 4, mem);
    finish_out(h, mem);
  });
}

int fmskf_export_vehicle_info(fmskf_handle h, fmskf_vehicle_info *out, const uint8_t *floor,
                              const float *cam_pitch, const uint32_t *fault, uint32_t mem) {
  static_assert(sizeof(fmskf_vehicle_info) == 84, "VehicleInfo record layout");
  return guarded([&] {
    check_handle(h);
    if (!out) fail(FMSKF_EINVAL, "null out");
    DeviceGuard g(h->cfg.device);
    const uint64_t n = h->s.n;
    ensure_imu(h);
    Stager sg(h, mem);
    const void *f = floor, *c = cam_pitch, *u = fault;
    sg.add(&f, n * 8);
    sg.add(&c, n * 4);
    sg.add(&u, n * 4);
    sg.run();
    launch_check(launch_readout(h->s, h->readout, h->stream), "readout");
    const size_t bytes = n * sizeof(fmskf_vehicle_info);
    void *dst = mem == FMSKF_MEM_DEVICE ? (void *)out : host_result(h, bytes);
    launch_check(launch_vehicle_info(h->s, h->readout, dst, (const uint8_t *)f, (const float *)c,
                                     (const uint32_t *)u, h->stream),
                 "vehicle_info launch");
    copy_out_sync(h, out, dst, bytes, mem);
  });
}

int fmskf_eval_trig(fmskf_handle h, const float *x, float *s, float *c, uint64_t n, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (!x || !s || !c) fail(FMSKF_EINVAL, "null argument");
    DeviceGuard g(h->cfg.device);
    const bool libm = h->cfg.trig == FMSKF_TRIG_LIBM;
    if (mem == FMSKF_MEM_DEVICE) {
      launch_check(launch_trig(x, s, c, n, libm, h->s.sintab, h->stream), "trig launch");
      return;
    }
    if (mem != FMSKF_MEM_HOST) fail(FMSKF_EINVAL, "bad mem flag");
    if (n == 0) return;
    char *buf = (char *)h->stage_for(3 * n * 4);
    float *dx = (float *)buf, *ds = dx + n, *dc = ds + n;
    hip_check(hipMemcpyAsync(dx, x, n * 4, hipMemcpyHostToDevice, h->stream), "H2D");
    launch_check(launch_trig(dx, ds, dc, n, libm, h->s.sintab, h->stream), "trig launch");
    hip_check(hipMemcpyAsync(s, ds, n * 4, hipMemcpyDeviceToHost, h->stream), "D2H");
    hip_check(hipMemcpyAsync(c, dc, n * 4, hipMemcpyDeviceToHost, h->stream), "D2H");
    hip_check(hipStreamSynchronize(h->stream), "sync");
  });
}

int fmskf_set_timing(fmskf_handle h, int enable) {
  return guarded([&] {
    check_handle(h);
    h->timing = enable != 0;
    h->tcount = 0;
  });
}

int fmskf_kernel_time_total(fmskf_handle h, double *total_ms, uint32_t *count) {
  return guarded([&] {
    check_handle(h);
    if (!total_ms || !count) fail(FMSKF_EINVAL, "null argument");
    DeviceGuard g(h->cfg.device);
    double sum = 0.0;
    if (h->tcount) hip_check(hipEventSynchronize(h->tpool[2 * h->tcount - 1]), "hipEventSynchronize");
    for (size_t k = 0; k < h->tcount; k++) {
      float ms = 0.f;
      hip_check(hipEventElapsedTime(&ms, h->tpool[2 * k], h->tpool[2 * k + 1]), "hipEventElapsedTime");
      sum += ms;
    }
    *total_ms = sum;
    *count = (uint32_t)h->tcount;
  });
}

int fmskf_last_kernel_ms(fmskf_handle h, float *ms) {
  return guarded([&] {
    check_handle(h);
    if (!ms) fail(FMSKF_EINVAL, "null ms");
    if (!h->timing) fail(FMSKF_EINVAL, "timing not enabled");
    DeviceGuard g(h->cfg.device);
    hip_check(hipEventSynchronize(h->ev1), "hipEventSynchronize");
    hip_check(hipEventElapsedTime(ms, h->ev0, h->ev1), "hipEventElapsedTime");
  });
}

}  // extern "C"
