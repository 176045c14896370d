// api_handle.cpp -- the C ABI (include/fmskf.h) over the HIP kernels: handle lifecycle,
// host staging, ingest, the tick entry points, state get / set.
//
// Owns the device SoA state of a handle, resolves NULL input planes to the
// device-resident ingest state (full pipeline), stages host inputs with async
// copies on the handle's stream, validates shapes, and converts every failure to
// a status code (no exception crosses the ABI).  No CPU fallback exists: every
// compute entry point launches a HIP kernel or fails with FMSKF_EDEVICE.
#include "api_ctx.hpp"

using namespace fmskf;
using namespace fmskf::capi;

thread_local std::string fmskf::capi::g_last_error;

namespace {

void apply_defaults(fmskf_config *c, uint32_t model, uint64_t n) {
  memset(c, 0, sizeof(*c));
  c->abi_version = FMSKF_ABI_VERSION;
  c->model = model;
  c->n_instances = n;
  c->device = 0;
  c->trig = FMSKF_TRIG_TABLE512;
  c->dt = 0.001;
  c->motor_dir[0] = 1;   // FL  (VD_task_main.cpp:75)
  c->motor_dir[1] = 1;   // BL  (:76)
  c->motor_dir[2] = -1;  // BR  (:77)
  c->motor_dir[3] = -1;  // FR  (:78)
  c->imu_read_reg = 0x51;  // q0: IMU_IF_WT901C::init -> WitReadReg(q0, 4)
  const double dt = c->dt;
  auto setq = [&](int i, int j, double v) { c->q[i * (i + 1) / 2 + j] = v; };
  auto setr = [&](int i, int j, double v) { c->r[i * (i + 1) / 2 + j] = v; };
  auto setp = [&](int i, double v) { c->p0[i * (i + 1) / 2 + i] = v; };
  // discretised white-noise-acceleration blocks for a (pos, vel) pair with density qc
  auto cv_block = [&](int p, int v, double qc) {
    setq(p, p, qc * dt * dt * dt / 3.0);
    setq(v, p, qc * dt * dt / 2.0);
    setq(v, v, qc * dt);
  };
  switch (model) {
    case FMSKF_MODEL_KF6:
      cv_block(0, 3, 4.0);
      cv_block(1, 4, 4.0);
      cv_block(2, 5, 100.0);
      setr(0, 0, 2.5e-5);  // yaw (5 mrad)^2
      setr(1, 1, 2.5e-3);  // gyro (0.05 rad/s)^2
      setr(2, 2, 4e-4);    // wheel velocity (2 cm/s)^2
      setr(3, 3, 4e-4);
      setr(3, 2, 1e-5);
      for (int i = 0; i < 6; i++) setp(i, i < 3 ? 1.0 : 0.25);
      break;
    case FMSKF_MODEL_EKF9: {
      const double qd[9] = {1e-10, 1e-10, 1e-10, 4e-3 * dt, 4e-3 * dt, 100.0 * dt, 1e-12, 2500.0 * dt, 2500.0 * dt};
      for (int i = 0; i < 9; i++) setq(i, i, qd[i]);
      const double rd[6] = {2.5e-5, 2.5e-3, 0.25, 0.25, 4e-4, 4e-4};
      for (int i = 0; i < 6; i++) setr(i, i, rd[i]);
      for (int i = 0; i < 9; i++) setp(i, i < 3 ? 1.0 : (i == 6 ? 1e-2 : 0.25));
      break;
    }
    case FMSKF_MODEL_KF12D: {
      cv_block(0, 3, 4.0);
      cv_block(1, 4, 4.0);
      cv_block(2, 5, 100.0);
      cv_block(6, 9, 1.0);
      cv_block(7, 10, 1.0);
      cv_block(8, 11, 1.0);
      const double rd[8] = {2.5e-5, 2.5e-3, 4e-4, 4e-4, 1e-6, 1e-6, 1e-6, 1e-4};
      for (int i = 0; i < 8; i++) setr(i, i, rd[i]);
      setr(3, 2, 1e-5);
      for (int i = 0; i < 12; i++) setp(i, (i % 6) < 3 ? 1.0 : 0.25);
      break;
    }
    default: break;
  }
}

void convert_params(fmskf_ctx *h) {
  const fmskf_config &c = h->cfg;
  h->kf6.dt = (float)c.dt;
  for (int k = 0; k < 21; k++) h->kf6.q[k] = (float)c.q[k];
  for (int k = 0; k < 10; k++) h->kf6.r[k] = (float)c.r[k];
  h->ekf9.dt = (float)c.dt;
  for (int k = 0; k < 45; k++) h->ekf9.q[k] = (float)c.q[k];
  for (int k = 0; k < 21; k++) h->ekf9.r[k] = (float)c.r[k];
  h->kf12.dt = c.dt;
  for (int k = 0; k < 78; k++) h->kf12.q[k] = c.q[k];
  for (int k = 0; k < 36; k++) h->kf12.r[k] = c.r[k];
  for (int a = 0; a < 4; a++)
    for (int b = 0; b <= a; b++) h->kf12.r2[a * (a + 1) / 2 + b] = c.r[(a + 4) * (a + 5) / 2 + (b + 4)];
  h->kf12.decor = kf12d_cinv(h->kf12.r, h->kf12.cinv) ? 1 : 0;
  h->kf12.sparse = h->kf12.decor && kf12d_sparse(h->kf12.cinv, h->kf12.q) ? 1 : 0;
}

}  // namespace

namespace fmskf {
namespace capi {

// WT901 / IMU_IF state and M2006 motor state, allocated on first use (an ingest call, a NULL
// input plane that reads them, a readout of them, or a graph capture) and zero-initialised like
// the firmware's static objects
void zero_imu(fmskf_ctx *h) {
  DevState &s = h->s;
  const uint64_t n = s.n;
  hipStream_t st = h->stream;
  hip_check(hipMemsetAsync(s.imu_reg, 0, 0x90 * n * 2, st), "reset imu");
  hip_check(hipMemsetAsync(s.imu_parser, 0, 3 * n * 4, st), "reset imu");
  hip_check(hipMemsetAsync(s.imu_cnt, 0, n, st), "reset imu");
  hip_check(hipMemsetAsync(s.imu_flags, 0, n, st), "reset imu");
  hip_check(hipMemsetAsync(s.imu_err, 0, n, st), "reset imu");
  hip_check(hipMemsetAsync(s.imu_qinit, 0, 4 * n * 4, st), "reset imu");
  hip_check(hipMemsetAsync(s.imu_snap, 0, kRowWords * n * 2, st), "reset imu");
  hip_check(hipMemsetAsync(s.imu_mag, 0, 4 * n * 2, st), "reset imu");
  hip_check(hipMemsetAsync(s.imu_yg, 0, n * 4, st), "reset imu");
  hip_check(hipMemsetAsync(s.imu_qprev, 0, 4 * n * 4, st), "reset imu");
}
void zero_motors(fmskf_ctx *h) {
  DevState &s = h->s;
  const uint64_t n = s.n;
  hipStream_t st = h->stream;
  hip_check(hipMemsetAsync(s.m_micro, 0, 4 * n * 2, st), "reset motors");
  hip_check(hipMemsetAsync(s.m_angle, 0, 4 * n * 2, st), "reset motors");
  hip_check(hipMemsetAsync(s.m_prev, 0, 4 * n * 2, st), "reset motors");
  hip_check(hipMemsetAsync(s.m_rpm, 0, 4 * n * 2, st), "reset motors");
  hip_check(hipMemsetAsync(s.m_curr, 0, 4 * n * 2, st), "reset motors");
  hip_check(hipMemsetAsync(s.m_sum_lo, 0, 4 * n * 4, st), "reset motors");
  hip_check(hipMemsetAsync(s.m_sum_hi, 0, 4 * n * 4, st), "reset motors");
  hip_check(hipMemsetAsync(s.m_iir_y, 0, 4 * n * 4, st), "reset motors");
  hip_check(hipMemsetAsync(s.m_prev_micro, 0, 4 * n * 2, st), "reset motors");
}

void ensure_imu(fmskf_ctx *h) {
  DevState &s = h->s;
  if (s.imu_reg) return;
  if (h->capturing) fail(FMSKF_EINVAL, "IMU state first used inside a graph capture");
  const uint64_t n = s.n;
  s.imu_reg = h->alloc<int16_t>(0x90 * n);
  s.imu_parser = h->alloc<uint32_t>(3 * n);
  s.imu_cnt = h->alloc<uint8_t>(n);
  s.imu_flags = h->alloc<uint8_t>(n);
  s.imu_err = h->alloc<uint8_t>(n);
  s.imu_qinit = h->alloc<float>(4 * n);
  s.imu_snap = h->alloc<int16_t>(kRowWords * n);
  s.imu_mag = h->alloc<int16_t>(4 * n);
  s.imu_yg = h->alloc<uint32_t>(n);
  s.imu_qprev = h->alloc<float>(4 * n);
  zero_imu(h);
}
void rs_prev_materialize(fmskf_ctx *h) {
  if (!h->rs_prev_stale) return;
  const DevState &s = h->s;
  launch_check(launch_motor_sums(s.m_sum_lo, s.m_sum_hi, s.prev_sum, s.n, 0, true, h->stream), "previous sums");
  h->rs_prev_stale = false;
}

void ensure_motors(fmskf_ctx *h) {
  DevState &s = h->s;
  if (s.m_sum_lo) return;
  if (h->capturing) fail(FMSKF_EINVAL, "motor state first used inside a graph capture");
  const uint64_t n = s.n;
  s.m_micro = h->alloc<int16_t>(4 * n);
  s.m_angle = h->alloc<int16_t>(4 * n);
  s.m_prev = h->alloc<int16_t>(4 * n);
  s.m_rpm = h->alloc<int16_t>(4 * n);
  s.m_curr = h->alloc<int16_t>(4 * n);
  s.m_sum_lo = h->alloc<uint32_t>(4 * n);
  s.m_sum_hi = h->alloc<int32_t>(4 * n);
  s.m_iir_y = h->alloc<float>(4 * n);
  s.m_prev_micro = h->alloc<int16_t>(4 * n);
  zero_motors(h);
}

}  // namespace capi
}  // namespace fmskf

namespace {

void do_reset(fmskf_ctx *h) {
  DevState &s = h->s;
  const uint64_t n = s.n;
  const Dims d = h->d;
  const uint32_t np = d.nx * (d.nx + 1) / 2;
  hipStream_t st = h->stream;
  const uint64_t pp = s.pitch;
  hip_check(hipMemsetAsync(s.x, 0, (size_t)d.nx * pp * d.elem, st), "reset x");
  if (d.m > 0 && s.tile) {  // tiled P: every row filled with its P0 entry in one pass
    std::vector<uint64_t> bits(np);
    for (uint32_t k = 0; k < np; k++) {
      const double v = h->cfg.p0[k];
      if (d.elem == 4) {
        const float f = (float)v;
        uint32_t b;
        memcpy(&b, &f, 4);
        bits[k] = b;
      } else {
        memcpy(&bits[k], &v, 8);
      }
    }
    launch_check(launch_tiled_fill(s.P, np, n, bits.data(), d.elem, st), "reset P0");
  } else if (d.m > 0) {
    hip_check(hipMemsetAsync(s.P, 0, (size_t)np * pp * d.elem, st), "reset P");
    for (uint32_t i = 0; i < d.nx; i++) {
      for (uint32_t j = 0; j <= i; j++) {
        const double v = h->cfg.p0[i * (i + 1) / 2 + j];
        if (v == 0.0) continue;
        const size_t k = i * (i + 1) / 2 + j;
        if (d.elem == 4) {
          float f = (float)v;
          uint32_t bits;
          memcpy(&bits, &f, 4);
          hip_check(hipMemsetD32Async((hipDeviceptr_t)((float *)s.P + k * pp), bits, n, st), "reset P0");
        } else {
          uint64_t bits;
          memcpy(&bits, &v, 8);
          launch_check(launch_fill64((double *)s.P + k * pp, bits, n, st), "reset P0");
        }
      }
    }
  }
  if (s.prev_sum) hip_check(hipMemsetAsync(s.prev_sum, 0, 4 * pp * 8, st), "reset prev");
  if (s.thlo) hip_check(hipMemsetAsync(s.thlo, 0, n * 4, st), "reset heading low part");
  if (s.xlo) hip_check(hipMemsetAsync(s.xlo, 0, (size_t)kKf6LoRows * pp * 4, st), "reset position low parts");
  if (s.imu_reg) zero_imu(h);
  if (s.m_sum_lo) zero_motors(h);
  if (h->ctrl_ready) {  // the control objects are static in the firmware too: zero, power off
    const CtrlDev &c = h->ctrl;
    hip_check(hipMemsetAsync(c.ax, 0, (size_t)3 * kAxF * c.pitch * 4, st), "reset ctrl");
    hip_check(hipMemsetAsync(c.pid, 0, (size_t)4 * kPidF * c.pitch * 4, st), "reset ctrl");
    hip_check(hipMemsetAsync(c.vel_tgt, 0, (size_t)3 * c.pitch * 4, st), "reset ctrl");
    hip_check(hipMemsetAsync(c.rpm_prev, 0, (size_t)4 * c.n * 2, st), "reset ctrl");
    hip_check(hipMemsetAsync(c.curr, 0, (size_t)4 * c.n * 2, st), "reset ctrl");
    hip_check(hipMemsetAsync(c.power, 0, (size_t)c.n, st), "reset ctrl");
  }
  hip_check(hipMemsetAsync(s.counters, 0, 8 * 8, st), "reset counters");
  h->isr_can_split = h->isr_ctrl_split = 0;
  h->rs_prev_synced = h->rs_prev_stale = false;  // the prev planes were zeroed above
  h->ctrl_derived_stale = false;                  // and the control outputs
  h->ens_shift_ok = false;
}

}  // namespace

namespace fmskf {
namespace capi {

// Resolve the tick inputs of a call (NULL -> device-resident ingest state), stage host
// planes and validate what the model needs.
TickIn resolve_inputs(fmskf_ctx *h, const fmskf_tick_inputs *in, bool need_upd, bool need_pred,
                      uint32_t n_ticks, uint64_t stride,
                      const std::vector<std::pair<const void **, size_t>> *extra) {
  if (!in) fail(FMSKF_EINVAL, "null inputs");
  DevState &s = h->s;
  const uint64_t n = s.n;
  if (stride < n) fail(FMSKF_EINVAL, "tick_stride < N");
  if (n_ticks == 0) fail(FMSKF_EINVAL, "n_ticks == 0");
  TickIn t{};
  t.yaw_deg = in->yaw_deg;
  t.gyro_z = in->gyro_z_dps;
  t.rpm = in->rpm;
  t.angle_sum = in->angle_sum;
  t.raw = in->raw;
  t.z = in->z;
  t.valid = in->valid;
  t.rec = (const uint32_t *)in->kf6_rec;
  t.sintab = s.sintab;
  t.stride = stride;
  t.sum_pitch = stride;
  t.n_ticks = n_ticks;
  if (t.rec && h->cfg.model != FMSKF_MODEL_KF6) fail(FMSKF_EINVAL, "kf6_rec is a KF6 input");
  if (t.rec && (t.yaw_deg || t.gyro_z || t.rpm))
    fail(FMSKF_EINVAL, "kf6_rec replaces yaw_deg / gyro_z_dps / rpm: pass one or the other");
  if (in->angle_sum_pitch) {
    if (n_ticks != 1 || stride != n) fail(FMSKF_EINVAL, "angle_sum_pitch is for single-tick calls (tick_many: tick_stride)");
    if (in->angle_sum_pitch < n) fail(FMSKF_EINVAL, "angle_sum_pitch < N");
    t.sum_pitch = in->angle_sum_pitch;
  }
  const uint64_t span = (uint64_t)(n_ticks - 1) * stride + n;  // elements per [N] plane
  Stager sg(h, in->mem);
  sg.add((const void **)&t.yaw_deg, span * 4);
  sg.add((const void **)&t.gyro_z, span * 4);
  sg.add((const void **)&t.rpm, span * 8);
  sg.add((const void **)&t.angle_sum, ((uint64_t)(n_ticks - 1) * stride * 4 + 3 * t.sum_pitch + n) * 8);
  sg.add((const void **)&t.raw, span * 16);
  sg.add((const void **)&t.z, ((uint64_t)(n_ticks - 1) * stride * 8 + 7 * stride + n) * 8);
  sg.add((const void **)&t.valid, span);
  sg.add((const void **)&t.rec, span * 16);
  if (extra)
    for (const auto &it : *extra) sg.add(it.first, it.second);
  sg.run();
  const bool many = n_ticks > 1 || stride != n;
  auto dev_default = [&](const void *p, const char *name) {
    if (!p && many) fail(FMSKF_EINVAL, std::string("tick_many needs explicit plane ") + name);
  };
  switch (h->cfg.model) {
    case FMSKF_MODEL_RS:
      if (need_upd) {
        dev_default(t.yaw_deg, "yaw_deg");
        if (!t.yaw_deg) {
          ensure_imu(h);
          t.yaw_deg = (const float *)s.imu_yg;  // IMT::get_status_now_yaw: Data.angle[2], its Yaw word
          t.imu_words |= 1u;
        }
      }
      if (need_pred) {
        dev_default(t.rpm, "rpm");
        dev_default(t.angle_sum, "angle_sum");
        if (!t.rpm || !t.angle_sum) ensure_motors(h);
        if (!t.rpm) t.rpm = s.m_rpm;
        if (!t.angle_sum) {  // the motor state's split sums (fmskf_internal.hpp m_sum_lo)
          t.msum_lo = s.m_sum_lo;
          t.msum_hi = s.m_sum_hi;
        }
      }
      break;
    case FMSKF_MODEL_KF6:
      if (need_upd && !t.rec) {
        dev_default(t.yaw_deg, "yaw_deg");
        dev_default(t.gyro_z, "gyro_z_dps");
        dev_default(t.rpm, "rpm");
        if (!t.yaw_deg || !t.gyro_z) ensure_imu(h);
        if (!t.rpm) ensure_motors(h);
        // Data.angle[2] / Data.gyro[2]: a NULL plane reads the IMU state's Yaw / GZ word
        if (!t.yaw_deg) {
          t.yaw_deg = (const float *)s.imu_yg;
          t.imu_words |= 1u;
        }
        if (!t.gyro_z) {
          t.gyro_z = (const float *)s.imu_yg;
          t.imu_words |= 2u;
        }
        if (!t.rpm) t.rpm = s.m_rpm;
      }
      break;
    case FMSKF_MODEL_EKF9:
      if (need_upd && !t.raw) fail(FMSKF_EINVAL, "EKF9 needs raw words");
      break;
    case FMSKF_MODEL_KF12D:
      if (need_upd && !t.z) fail(FMSKF_EINVAL, "KF12D needs z");
      break;
  }
  return t;
}

void run_tick(fmskf_ctx *h, const fmskf_tick_inputs *in, bool upd, bool pred, uint32_t n_ticks,
              uint64_t stride) {
  check_handle(h);
  DeviceGuard g(h->cfg.device);
  TickIn t = resolve_inputs(h, in, upd, pred, n_ticks, stride);
  // a plain tick after an asynchronous ensemble event: the event's fold runs stand-alone
  // ahead of it (a record every K > 1 ticks gets its result one fold after its tick; only the
  // next ensemble tick's kernel carries it).  Not inside a capture: the replay would fold
  // whatever the slot holds then
  if (!h->capturing) ens_flush(h);
  const bool libm = h->cfg.trig == FMSKF_TRIG_LIBM;
  const bool rs_pred = h->cfg.model == FMSKF_MODEL_RS && pred;
  if (rs_pred) rs_prev_materialize(h);  // the predict reads the prev planes
  h->time_begin();
  int e = 0;
  switch (h->cfg.model) {
    case FMSKF_MODEL_RS: e = launch_rs(h->s, t, libm, upd, pred, h->stream); break;
    case FMSKF_MODEL_KF6: e = launch_kf6(h->s, t, h->kf6, libm, upd, pred, h->stream); break;
    case FMSKF_MODEL_EKF9: e = launch_ekf9(h->s, t, h->ekf9, libm, upd, pred, h->stream); break;
    case FMSKF_MODEL_KF12D: e = launch_kf12d(h->s, t, h->kf12, upd, pred, h->stream); break;
  }
  launch_check(e, "tick kernel launch");
  // the predict stored the sums it read as the previous ones
  if (rs_pred) h->rs_prev_synced = t.msum_lo != nullptr;
  h->time_end();
}

void copy_out(fmskf_ctx *h, void *dst, const void *src, size_t bytes, uint32_t mem) {
  if (!dst) return;
  if (mem == FMSKF_MEM_HOST) {
    hip_check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, h->stream), "D2H");
  } else if (mem == FMSKF_MEM_DEVICE) {
    hip_check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, h->stream), "D2D");
  } else {
    fail(FMSKF_EINVAL, "bad mem flag");
  }
}
// `planes` planes of `row` bytes: device planes at `dev_pitch` bytes <-> dense user planes
void copy_planes_out(fmskf_ctx *h, void *dst, const void *src, size_t row, size_t dev_pitch,
                     size_t planes, uint32_t mem) {
  if (!dst) return;
  if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
  const hipMemcpyKind k = mem == FMSKF_MEM_HOST ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
  hip_check(hipMemcpy2DAsync(dst, row, src, dev_pitch, row, planes, k, h->stream), "copy planes");
}
void copy_planes_in(fmskf_ctx *h, void *dst, const void *src, size_t row, size_t dev_pitch,
                    size_t planes, uint32_t mem) {
  if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
  const hipMemcpyKind k = mem == FMSKF_MEM_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
  hip_check(hipMemcpy2DAsync(dst, dev_pitch, src, row, row, planes, k, h->stream), "copy planes");
}
void finish_out(fmskf_ctx *h, uint32_t mem) {
  if (mem == FMSKF_MEM_HOST) hip_check(hipStreamSynchronize(h->stream), "hipStreamSynchronize");
}
// where a kernel writes a result of `bytes` bound for the caller's host memory: the pinned
// output slot itself under zero-copy staging, else device scratch
void *host_result(fmskf_ctx *h, size_t bytes) {
  if (bytes <= fmskf_ctx::kPinned && !h->capturing) return fmskf_ctx::dev_ptr(h->pinned_out());
  return h->out_for(bytes);
}
// one device buffer to the caller's host (or device) buffer, complete on return: a small host
// result goes through the pinned slot (written there by the kernel under zero-copy staging, or
// one DMA), then a CPU copy
void copy_out_sync(fmskf_ctx *h, void *dst, const void *src, size_t bytes, uint32_t mem) {
  if (mem == FMSKF_MEM_HOST && h->pin_out && src == fmskf_ctx::dev_ptr(h->pin_out)) {
    hip_check(hipStreamSynchronize(h->stream), "hipStreamSynchronize");
    memcpy(dst, h->pin_out, bytes);
    return;
  }
  if (mem == FMSKF_MEM_HOST && bytes <= fmskf_ctx::kPinned && !h->capturing) {
    char *pin = h->pinned_out();
    hip_check(hipMemcpyAsync(pin, src, bytes, hipMemcpyDeviceToHost, h->stream), "D2H");
    hip_check(hipStreamSynchronize(h->stream), "hipStreamSynchronize");
    memcpy(dst, pin, bytes);
    return;
  }
  if (mem == FMSKF_MEM_HOST) copy_out(h, dst, src, bytes, mem);
  finish_out(h, mem);
}

}  // namespace capi
}  // namespace fmskf

// ============================================================================
// C ABI
// ============================================================================
extern "C" {

int fmskf_abi_version(void) { return (int)FMSKF_ABI_VERSION; }

const char *fmskf_strerror(int status) {
  switch (status) {
    case FMSKF_OK: return "ok";
    case FMSKF_EINVAL: return "invalid argument";
    case FMSKF_ENOMEM: return "out of memory";
    case FMSKF_EDEVICE: return "device error";
    case FMSKF_ERCCL: return "collective error";
    case FMSKF_ENOTSUP: return "not supported for this model";
    default: return "unknown status";
  }
}

const char *fmskf_last_error(void) { return g_last_error.c_str(); }

int fmskf_model_dims(uint32_t model, uint32_t *n, uint32_t *m, uint32_t *elem_bytes) {
  return guarded([&] {
    Dims d = dims_of(model);
    if (n) *n = d.nx;
    if (m) *m = d.m;
    if (elem_bytes) *elem_bytes = d.elem;
  });
}

int fmskf_config_init(fmskf_config *cfg, uint32_t model, uint64_t n) {
  return guarded([&] {
    if (!cfg) fail(FMSKF_EINVAL, "null config");
    (void)dims_of(model);
    apply_defaults(cfg, model, n);
  });
}

int fmskf_create(const fmskf_config *cfg, fmskf_handle *out) {
  return guarded([&] {
    if (!cfg || !out) fail(FMSKF_EINVAL, "null argument");
    *out = nullptr;
    if (cfg->abi_version != FMSKF_ABI_VERSION) fail(FMSKF_EINVAL, "ABI version mismatch");
    const Dims d = dims_of(cfg->model);
    if (cfg->n_instances == 0) fail(FMSKF_EINVAL, "n_instances == 0");
    if (cfg->n_instances > (1ull << 30)) fail(FMSKF_EINVAL, "n_instances > 2^30 per handle");
    if (cfg->trig > FMSKF_TRIG_LIBM) fail(FMSKF_EINVAL, "bad trig policy");
    if (!(cfg->dt > 0.0) || !isfinite(cfg->dt)) fail(FMSKF_EINVAL, "dt must be > 0");
    if (cfg->imu_read_reg + 4 > 0x90) fail(FMSKF_EINVAL, "imu_read_reg out of range");
    if ((cfg->flags & ~FMSKF_CFG_COMP_POS) || cfg->reserved) fail(FMSKF_EINVAL, "unknown config flags");
    if ((cfg->flags & FMSKF_CFG_COMP_POS) && cfg->model != FMSKF_MODEL_KF6 && cfg->model != FMSKF_MODEL_EKF9)
      fail(FMSKF_ENOTSUP, "FMSKF_CFG_COMP_POS is a KF6 / EKF9 mode");
    for (int w = 0; w < 4; w++)
      if (cfg->motor_dir[w] != 1 && cfg->motor_dir[w] != -1) fail(FMSKF_EINVAL, "motor_dir must be +-1");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) fail(FMSKF_EDEVICE, "no HIP device");
    if (cfg->device < 0 || cfg->device >= ndev) fail(FMSKF_EINVAL, "bad device ordinal");
    DeviceGuard g(cfg->device);
    fmskf_ctx *h = new fmskf_ctx();
    try {
      h->cfg = *cfg;
      h->d = d;
      const uint64_t n = cfg->n_instances;
      DevState &s = h->s;
      s.n = n;
      s.model = cfg->model;
      const uint32_t np = d.nx * (d.nx + 1) / 2;
      s.tile = (FMSKF_TILED && (cfg->model == FMSKF_MODEL_EKF9 || cfg->model == FMSKF_MODEL_KF12D)) ||
                       (FMSKF_KF6_TILED && cfg->model == FMSKF_MODEL_KF6)
                   ? tile_w_elem(d.elem) : 0;
      // a tiled array's rows x pitch elements cover ceil(N / tile) whole tiles
      s.pitch = s.tile ? std::max(plane_pitch(n), (n + s.tile - 1) / s.tile * s.tile) : plane_pitch(n);
      s.x = h->alloc<char>((size_t)d.nx * s.pitch * d.elem);
      s.P = d.m ? h->alloc<char>((size_t)np * s.pitch * d.elem) : nullptr;
      s.prev_sum = cfg->model == FMSKF_MODEL_RS ? h->alloc<int64_t>(4 * s.pitch) : nullptr;
      // EKF9: the compensated heading's hidden low part (kf_generic.hpp th_add), one float a robot
      s.thlo = cfg->model == FMSKF_MODEL_EKF9 ? h->alloc<float>(n) : nullptr;
      // KF6 / EKF9 with FMSKF_CFG_COMP_POS: the position low parts, tiled like x and P
      s.xlo = (cfg->flags & FMSKF_CFG_COMP_POS) ? h->alloc<float>((size_t)kKf6LoRows * s.pitch) : nullptr;
      h->kf6.lo = s.xlo;
      // the WT901 / motor ingest state (~470 B per robot) is allocated on first use
      // (ensure_imu / ensure_motors): a handle fed tick inputs by the caller holds only x, P
      s.counters = h->alloc<unsigned long long>(8);
      s.sintab = h->alloc<float>(513);
      {
        // the fused KF6 tick + record (fmskf_tick_ensemble) writes one record per tick block
        const size_t len = 1 + d.nx + np;
        size_t nb = (size_t)ensemble_nblocks(n);
        if (cfg->model == FMSKF_MODEL_KF6 || cfg->model == FMSKF_MODEL_EKF9 || cfg->model == FMSKF_MODEL_KF12D)
          nb = std::max(nb, (size_t)((n + kBlock - 1) / kBlock));
        h->ens_blocks = h->alloc<double>(nb * len);
        h->ens_out = h->alloc<double>(91);
        h->ens_shift = h->alloc<double>(12);
      }
      h->readout = h->alloc<float>(6 * n);
      // TABLE512: CMSIS-DSP's sinTable_f32 as its published 8-decimal literals (arm_common_tables.c;
      // the firmware's arm_sin_f32 / arm_cos_f32, util_mymath.hpp:44-45), cmsis_sintab.inc
      static const float tab[513] = {
#include "cmsis_sintab.inc"
      };
      hip_check(hipMemcpy(s.sintab, tab, sizeof(tab), hipMemcpyHostToDevice), "sintab upload");
      hip_check(hipEventCreate(&h->ev0), "hipEventCreate");
      hip_check(hipEventCreate(&h->ev1), "hipEventCreate");
      convert_params(h);
      {
        double *coef = h->alloc<double>(36 + 78);
        hip_check(hipMemcpy(coef, h->kf12.cinv, 36 * sizeof(double), hipMemcpyHostToDevice), "coef upload");
        hip_check(hipMemcpy(coef + 36, h->kf12.q, 78 * sizeof(double), hipMemcpyHostToDevice), "coef upload");
        h->kf12.coef = coef;
      }
      do_reset(h);
      hip_check(hipStreamSynchronize(h->stream), "hipStreamSynchronize");
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

int fmskf_destroy(fmskf_handle h) {
  return guarded([&] {
    if (!h) return;
    DeviceGuard g(h->cfg.device);
    delete h;
  });
}

int fmskf_reset(fmskf_handle h) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    do_reset(h);
  });
}

int fmskf_set_stream(fmskf_handle h, void *stream) {
  return guarded([&] {
    check_handle(h);
    // work queued on the old stream (staging buffers, pinned slots) completes before the new
    // stream can reuse what it reads
    if (h->stream != (hipStream_t)stream && !h->capturing)
      hip_check(hipStreamSynchronize(h->stream), "hipStreamSynchronize");
    h->stream = (hipStream_t)stream;
  });
}

int fmskf_graph_begin(fmskf_handle h) {
  return guarded([&] {
    check_handle(h);
    if (!h->stream) fail(FMSKF_EINVAL, "graph capture needs a stream (fmskf_set_stream)");
    if (h->capturing) fail(FMSKF_EINVAL, "capture already open");
    if (h->timing) fail(FMSKF_EINVAL, "disable per-launch timing before capturing");
    DeviceGuard g(h->cfg.device);
    // state that is allocated on first use must exist before the capture starts
    ensure_imu(h);
    ensure_motors(h);
    ensure_ctrl(h);
    ensure_shift(h);
    // a replay starts from whatever state the handle is in then: captured RS ISRs keep the prev
    // planes themselves (no PS form inside a capture), so they must be current before it
    rs_prev_materialize(h);
    h->rs_prev_synced = false;
    // captured control steps store their derived outputs themselves (ctrl_step_prm); the ones
    // before the capture are formed now, while the host still knows their parameters
    ctrl_materialize(h);
    h->graph_has_ctrl = false;
    h->graph_par0 = h->s.m_par;  // the motor history order the captured CAN RX calls start from
    hip_check(hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal),
              "hipStreamBeginCapture");
    h->capturing = true;
  });
}

int fmskf_graph_end(fmskf_handle h) {
  return guarded([&] {
    check_handle(h);
    if (!h->capturing) fail(FMSKF_EINVAL, "no capture open");
    DeviceGuard g(h->cfg.device);
    h->capturing = false;
    h->rs_prev_synced = false;  // the captured calls moved host-side flags the replays do not
    // nor has any captured CAN RX run: the order is back where the capture started, and each
    // replay leaves it where the capture ended
    h->graph_par_end = h->s.m_par;
    h->s.m_par = h->graph_par0;
    hipGraph_t gnew = nullptr;
    hip_check(hipStreamEndCapture(h->stream, &gnew), "hipStreamEndCapture");
    if (h->graph_exec) hip_check(hipGraphExecDestroy(h->graph_exec), "hipGraphExecDestroy");
    if (h->graph) hip_check(hipGraphDestroy(h->graph), "hipGraphDestroy");
    h->graph_exec = nullptr;
    h->graph = gnew;
    hip_check(hipGraphInstantiate(&h->graph_exec, h->graph, nullptr, nullptr, 0),
              "hipGraphInstantiate");
  });
}

int fmskf_graph_launch(fmskf_handle h, uint32_t times) {
  return guarded([&] {
    check_handle(h);
    if (!h->graph_exec) fail(FMSKF_EINVAL, "no graph captured");
    if (h->capturing) fail(FMSKF_EINVAL, "capture still open");
    DeviceGuard g(h->cfg.device);
    for (uint32_t k = 0; k < times; k++) {
      if (h->s.m_par != h->graph_par0) {  // replays start from the capture's motor history order
        launch_check(launch_motor_swap(h->s, h->stream), "motor history order");
        h->s.m_par ^= 1u;
      }
      hip_check(hipGraphLaunch(h->graph_exec, h->stream), "hipGraphLaunch");
      h->s.m_par = h->graph_par_end;
    }
    h->rs_prev_synced = false;
    if (h->graph_has_ctrl && times > 0) h->ctrl_derived_stale = false;  // the replayed steps stored them
  });
}

int fmskf_sync(fmskf_handle h) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    hip_check(hipStreamSynchronize(h->stream), "hipStreamSynchronize");
  });
}

int fmskf_get_config(fmskf_handle h, fmskf_config *out) {
  return guarded([&] {
    check_handle(h);
    if (!out) fail(FMSKF_EINVAL, "null out");
    *out = h->cfg;
  });
}

int fmskf_ingest_wt901(fmskf_handle h, const uint8_t *bytes, uint32_t stride, const uint32_t *len,
                       int latch_qinit, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (!bytes || !len) fail(FMSKF_EINVAL, "null bytes/len");
    DeviceGuard g(h->cfg.device);
    const uint64_t n = h->s.n;
    if (mem == FMSKF_MEM_HOST) {
      for (uint64_t i = 0; i < n; i++)
        if (len[i] > stride) fail(FMSKF_EINVAL, "len[i] > stride");
    }
    ensure_imu(h);
    Stager sg(h, mem);
    const void *b = bytes, *l = len;
    sg.add(&b, (size_t)stride * n);
    sg.add(&l, n * 4);
    sg.run();
    launch_check(launch_wt901(h->s, (const uint8_t *)b, stride, (const uint32_t *)l, latch_qinit,
                              h->cfg.imu_read_reg, h->stream),
                 "wt901 launch");
  });
}

int fmskf_ingest_can(fmskf_handle h, const uint8_t *frames, const int16_t *stamps,
                     const uint8_t *present, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (!frames || !stamps) fail(FMSKF_EINVAL, "null frames/stamps");
    DeviceGuard g(h->cfg.device);
    const uint64_t n = h->s.n;
    ensure_motors(h);
    Stager sg(h, mem);
    const void *f = frames, *s = stamps, *p = present;
    sg.add(&f, n * 32);
    sg.add(&s, n * 8);
    sg.add(&p, n);
    sg.run();
    rs_prev_materialize(h);  // the previous sums leave the motor state now
    launch_check(launch_can(h->s, (const uint8_t *)f, (const int16_t *)s, (const uint8_t *)p,
                            h->cfg.motor_dir, h->stream),
                 "can launch");
    h->s.m_par ^= 1u;  // the frames' stamps and angles went over the older history slots
    h->rs_prev_synced = false;
  });
}

int fmskf_correct(fmskf_handle h, const fmskf_tick_inputs *in) {
  return guarded([&] { run_tick(h, in, true, false, 1, h ? h->s.n : 0); });
}

int fmskf_predict(fmskf_handle h, const fmskf_tick_inputs *in) {
  return guarded([&] { run_tick(h, in, false, true, 1, h ? h->s.n : 0); });
}

int fmskf_tick(fmskf_handle h, const fmskf_tick_inputs *in) {
  return guarded([&] { run_tick(h, in, true, true, 1, h ? h->s.n : 0); });
}

int fmskf_tick_many(fmskf_handle h, const fmskf_tick_inputs *in, uint32_t n_ticks,
                    uint64_t tick_stride) {
  return guarded([&] { run_tick(h, in, true, true, n_ticks, tick_stride); });
}

int fmskf_get_pose(fmskf_handle h, float *x, float *y, float *th, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    const uint64_t n = h->s.n;
    launch_check(launch_readout(h->s, h->readout, h->stream), "readout");
    copy_out(h, x, h->readout, n * 4, mem);
    copy_out(h, y, h->readout + n, n * 4, mem);
    copy_out(h, th, h->readout + 2 * n, n * 4, mem);
    finish_out(h, mem);
  });
}

int fmskf_get_vel(fmskf_handle h, float *vx, float *vy, float *vth, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    const uint64_t n = h->s.n;
    launch_check(launch_readout(h->s, h->readout, h->stream), "readout");
    copy_out(h, vx, h->readout + 3 * n, n * 4, mem);
    copy_out(h, vy, h->readout + 4 * n, n * 4, mem);
    copy_out(h, vth, h->readout + 5 * n, n * 4, mem);
    finish_out(h, mem);
  });
}

int fmskf_get_state(fmskf_handle h, void *x, void *p_packed, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    const uint64_t n = h->s.n;
    const Dims d = h->d;
    const size_t row = (size_t)n * d.elem, pb = (size_t)h->s.pitch * d.elem;
    const uint32_t np = d.nx * (d.nx + 1) / 2;
    if (p_packed && !d.m) fail(FMSKF_ENOTSUP, "RS model has no covariance");
    if (h->s.tile) {  // tiled state: gather into dense planes (device), then copy
      if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
      auto out = [&](void *dst, const void *src, uint32_t rows) {
        if (!dst) return;
        void *dense = mem == FMSKF_MEM_DEVICE ? dst : h->out_for(row * rows);
        launch_check(launch_untile(src, dense, rows, n, d.elem, h->stream), "untile");
        if (mem == FMSKF_MEM_HOST) {
          copy_out(h, dst, dense, row * rows, mem);
          hip_check(hipStreamSynchronize(h->stream), "get_state sync");  // scratch reused next
        }
      };
      out(x, h->s.x, d.nx);
      if (p_packed) out(p_packed, h->s.P, np);
    } else {
      copy_planes_out(h, x, h->s.x, row, pb, d.nx, mem);
      if (p_packed) copy_planes_out(h, p_packed, h->s.P, row, pb, np, mem);
    }
    finish_out(h, mem);
  });
}

int fmskf_set_state(fmskf_handle h, const void *x, const void *p_packed, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    const uint64_t n = h->s.n;
    const Dims d = h->d;
    if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
    const size_t row = (size_t)n * d.elem, pb = (size_t)h->s.pitch * d.elem;
    const uint32_t np = d.nx * (d.nx + 1) / 2;
    if (p_packed && !d.m) fail(FMSKF_ENOTSUP, "RS model has no covariance");
    if (h->s.tile) {  // dense planes (staged to the device when on the host) -> tiled state
      auto in = [&](void *dst, const void *src, uint32_t rows) {
        if (!src) return;
        const void *dense = src;
        if (mem == FMSKF_MEM_HOST) {
          void *stg = h->stage_for(row * rows);
          hip_check(hipMemcpyAsync(stg, src, row * rows, hipMemcpyHostToDevice, h->stream), "stage H2D");
          dense = stg;
        }
        launch_check(launch_tile(dense, dst, rows, n, d.elem, h->stream), "tile");
        if (mem == FMSKF_MEM_HOST) hip_check(hipStreamSynchronize(h->stream), "set_state sync");
      };
      in(h->s.x, x, d.nx);
      if (p_packed) in(h->s.P, p_packed, np);
    } else {
      if (x) copy_planes_in(h, h->s.x, x, row, pb, d.nx, mem);
      if (p_packed) copy_planes_in(h, h->s.P, p_packed, row, pb, np, mem);
    }
    if (x) h->ens_shift_ok = false;
    // a heading set from outside is exact as given: its compensation term restarts at zero
    if (x && h->s.thlo) hip_check(hipMemsetAsync(h->s.thlo, 0, n * 4, h->stream), "heading low part");
    // compensated positions: a state set from outside restarts every low part (x and P)
    if ((x || p_packed) && h->s.xlo)
      hip_check(hipMemsetAsync(h->s.xlo, 0, (size_t)kKf6LoRows * h->s.pitch * 4, h->stream), "position low parts");
    finish_out(h, mem);
  });
}

}  // extern "C"
