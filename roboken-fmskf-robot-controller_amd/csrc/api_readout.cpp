// api_readout.cpp -- readouts of the ingest and estimator state, the NaN / Inf counters, and
// the synchronous ensemble record (stand-alone partial, fused into the tick, host combine).
#include "api_ctx.hpp"

using namespace fmskf;
using namespace fmskf::capi;

extern "C" {

int fmskf_get_prev_sum(fmskf_handle h, int64_t *prev, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (!h->s.prev_sum) fail(FMSKF_ENOTSUP, "prev_sum exists in the RS model only");
    DeviceGuard g(h->cfg.device);
    if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
    rs_prev_materialize(h);
    if (!prev) return;
    // the tick's tiled layout on the device -> the ABI's [4][N] planes
    const uint64_t n = h->s.n;
    int64_t *dense = mem == FMSKF_MEM_DEVICE ? prev : (int64_t *)h->out_for((size_t)4 * n * 8);
    launch_check(launch_prev_out(h->s.prev_sum, dense, n, n, h->stream), "previous sums");
    if (mem == FMSKF_MEM_HOST) copy_out(h, prev, dense, (size_t)4 * n * 8, mem);
    finish_out(h, mem);
  });
}

int fmskf_get_imu(fmskf_handle h, float *data, uint8_t *is_error, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    ensure_imu(h);
    if (data) {  // the page formed from the last successful poll's snapshot (imu_data_page)
      if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
      float *dst = mem == FMSKF_MEM_DEVICE ? data : (float *)h->out_for(16 * h->s.n * 4);
      launch_check(launch_imu_data(h->s, dst, h->stream), "imu data");
      if (mem == FMSKF_MEM_HOST) copy_out(h, data, dst, 16 * h->s.n * 4, mem);
    }
    copy_out(h, is_error, h->s.imu_err, h->s.n, mem);
    finish_out(h, mem);
  });
}

int fmskf_get_imu_regs(fmskf_handle h, int16_t *regs, uint8_t *pending, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    ensure_imu(h);
    launch_check(launch_wt901_regs_sync(h->s, h->stream), "register file sync");
    copy_out(h, regs, h->s.imu_reg, 0x90 * h->s.n * 2, mem);
    copy_out(h, pending, h->s.imu_cnt, h->s.n, mem);
    finish_out(h, mem);
  });
}

int fmskf_get_motors(fmskf_handle h, int16_t *angle, int16_t *rpm, int16_t *curr,
                     int64_t *angle_sum, float *speed_radps, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
    const uint64_t n = h->s.n;
    ensure_motors(h);
    copy_out(h, angle, motor_slots(h->s).angle, 4 * n * 2, mem);
    copy_out(h, rpm, h->s.m_rpm, 4 * n * 2, mem);
    copy_out(h, curr, h->s.m_curr, 4 * n * 2, mem);
    if (angle_sum) {  // the split sums as whole int64 [4][N] planes
      int64_t *dense = mem == FMSKF_MEM_DEVICE ? angle_sum : (int64_t *)h->out_for((size_t)4 * n * 8);
      launch_check(launch_motor_sums(h->s.m_sum_lo, h->s.m_sum_hi, dense, n, n, false, h->stream), "motor sums");
      if (mem == FMSKF_MEM_HOST) copy_out(h, angle_sum, dense, (size_t)4 * n * 8, mem);
    }
    // Status::flt_SpeedRadPS is the IIR1 output, i.e. its state y (VD_motor_if_m2006.cpp:63):
    // [4][N] planes out of the device's [N][4] rows
    if (speed_radps) {
      if (mem == FMSKF_MEM_HOST) {
        std::vector<float> rows(4 * n);
        copy_out(h, rows.data(), h->s.m_iir_y, 4 * n * 4, mem);
        hip_check(hipStreamSynchronize(h->stream), "hipStreamSynchronize");
        for (uint64_t i = 0; i < n; i++)
          for (int w = 0; w < 4; w++) speed_radps[(size_t)w * n + i] = rows[4 * i + w];
      } else if (mem == FMSKF_MEM_DEVICE) {  // one strided copy per wheel: column w -> plane w
        for (int w = 0; w < 4; w++)
          hip_check(hipMemcpy2DAsync(speed_radps + (size_t)w * n, 4, h->s.m_iir_y + w, 16, 4, n,
                                     hipMemcpyDeviceToDevice, h->stream),
                    "speed transpose");
      } else {
        fail(FMSKF_EINVAL, "bad mem flag");
      }
    }
    finish_out(h, mem);
  });
}

int fmskf_get_motor_status(fmskf_handle h, int16_t *microsec_id, int16_t *angle, int16_t *rpm,
                           int16_t *curr, float *dlt_out_angle_rad, float *speed_radps, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
    DeviceGuard g(h->cfg.device);
    const uint64_t n = h->s.n;
    ensure_motors(h);
    const MotorSlots ms = motor_slots(h->s);
    copy_out(h, microsec_id, ms.micro, 4 * n * 2, mem);
    copy_out(h, angle, ms.angle, 4 * n * 2, mem);
    copy_out(h, rpm, h->s.m_rpm, 4 * n * 2, mem);
    copy_out(h, curr, h->s.m_curr, 4 * n * 2, mem);
    if (dlt_out_angle_rad) {
      float *dst = mem == FMSKF_MEM_DEVICE ? dlt_out_angle_rad : (float *)h->out_for(4 * n * 4);
      launch_check(launch_motor_dlt(ms.angle, ms.prev, dst, 4 * n, h->stream), "motor dlt");
      if (mem == FMSKF_MEM_HOST) copy_out(h, dlt_out_angle_rad, dst, 4 * n * 4, mem);
    }
    // Status::flt_SpeedRadPS [N][4]: the IIR1 output rows as the device keeps them
    copy_out(h, speed_radps, h->s.m_iir_y, 4 * n * 4, mem);
    finish_out(h, mem);
  });
}

int fmskf_get_state_lo(fmskf_handle h, float *lo, uint32_t *rows, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
    DeviceGuard g(h->cfg.device);
    const uint64_t n = h->s.n;
    const uint32_t rh = h->s.thlo ? 1u : 0u, rx = h->s.xlo ? kKf6LoRows : 0u;
    if (rows) *rows = rh + rx;
    if (!lo || !(rh + rx)) return;
    if (rh) copy_out(h, lo, h->s.thlo, n * 4, mem);
    if (rx) {
      float *dst = lo + (size_t)rh * n;
      void *dense = mem == FMSKF_MEM_DEVICE ? (void *)dst : h->out_for((size_t)rx * n * 4);
      launch_check(launch_untile(h->s.xlo, dense, rx, n, 4, h->stream), "untile");
      if (mem == FMSKF_MEM_HOST) copy_out(h, dst, dense, (size_t)rx * n * 4, mem);
    }
    finish_out(h, mem);
  });
}

int fmskf_set_state_lo(fmskf_handle h, const float *lo, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
    if (!lo) fail(FMSKF_EINVAL, "null lo");
    DeviceGuard g(h->cfg.device);
    const uint64_t n = h->s.n;
    const uint32_t rh = h->s.thlo ? 1u : 0u, rx = h->s.xlo ? kKf6LoRows : 0u, r = rh + rx;
    if (!r) fail(FMSKF_ENOTSUP, "this model keeps no low-part rows");
    const float *src = lo;
    if (mem == FMSKF_MEM_HOST) {
      void *stg = h->stage_for((size_t)r * n * 4);
      hip_check(hipMemcpyAsync(stg, lo, (size_t)r * n * 4, hipMemcpyHostToDevice, h->stream), "stage H2D");
      src = (const float *)stg;
    }
    if (rh) hip_check(hipMemcpyAsync(h->s.thlo, src, n * 4, hipMemcpyDeviceToDevice, h->stream), "lo");
    if (rx) launch_check(launch_tile(src + (size_t)rh * n, h->s.xlo, rx, n, 4, h->stream), "tile");
    h->ens_shift_ok = false;
    finish_out(h, FMSKF_MEM_HOST);
  });
}

int fmskf_get_counters(fmskf_handle h, uint64_t *counters, uint32_t n_counters) {
  return guarded([&] {
    check_handle(h);
    if (!counters || n_counters == 0) return;
    DeviceGuard g(h->cfg.device);
    unsigned long long tmp[8];
    hip_check(hipMemcpyAsync(tmp, h->s.counters, sizeof(tmp), hipMemcpyDeviceToHost, h->stream), "D2H");
    hip_check(hipStreamSynchronize(h->stream), "sync");
    tmp[1] = h->isr_can_split;  // host-side counters: the launch forms the ISR calls took
    tmp[2] = h->isr_ctrl_split;
    for (uint32_t k = 0; k < n_counters && k < 8; k++) counters[k] = tmp[k];
  });
}

int fmskf_ensemble_record_len(fmskf_handle h, uint32_t *len) {
  return guarded([&] {
    check_handle(h);
    if (!len) fail(FMSKF_EINVAL, "null len");
    const uint32_t nx = h->d.nx;
    *len = 1 + nx + nx * (nx + 1) / 2;
  });
}

int fmskf_ensemble_partial(fmskf_handle h, double *out, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (!out) fail(FMSKF_EINVAL, "null out");
    DeviceGuard g(h->cfg.device);
    const uint32_t nx = h->d.nx;
    const uint32_t len = 1 + nx + nx * (nx + 1) / 2;
    double *dst = mem == FMSKF_MEM_DEVICE ? out : h->ens_out;
    ensure_shift(h);
    launch_check(launch_ensemble(h->s, (int)nx, h->d.elem == 8, h->ens_blocks, h->ens_shift, dst,
                                 h->stream),
                 "ensemble launch");
    if (mem == FMSKF_MEM_HOST) {
      copy_out(h, out, h->ens_out, len * 8, mem);
      finish_out(h, mem);
    } else if (mem != FMSKF_MEM_DEVICE) {
      fail(FMSKF_EINVAL, "bad mem flag");
    }
  });
}

int fmskf_tick_ensemble(fmskf_handle h, const fmskf_tick_inputs *in, double *out, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (!out) fail(FMSKF_EINVAL, "null out");
    if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
    DeviceGuard g(h->cfg.device);
    const uint32_t nx = h->d.nx;
    const uint32_t len = 1 + nx + nx * (nx + 1) / 2;
    double *dst = mem == FMSKF_MEM_DEVICE ? out : h->ens_out;
    ensure_shift(h);
    if (fused_record(h)) {
      // one kernel: the tick writes each block's record of the state it just stored (no
      // second pass over x), then the fold
      TickIn t = resolve_inputs(h, in, true, true, 1, h->s.n);
      t.ens_blocks = h->ens_blocks;
      t.ens_shift = h->ens_shift;
      int nb = 0;
      const bool libm = h->cfg.trig == FMSKF_TRIG_LIBM;
      h->time_begin();
      if (h->cfg.model == FMSKF_MODEL_KF6)
        launch_check(launch_kf6(h->s, t, h->kf6, libm, true, true, h->stream, &nb), "tick kernel launch");
      else if (h->cfg.model == FMSKF_MODEL_EKF9)
        launch_check(launch_ekf9(h->s, t, h->ekf9, libm, true, true, h->stream, &nb), "tick kernel launch");
      else
        launch_check(launch_kf12d(h->s, t, h->kf12, true, true, h->stream, &nb), "tick kernel launch");
      h->time_end();
      launch_check(launch_ens_fold((int)nx, h->ens_blocks, nb, h->ens_shift, dst, h->stream),
                   "ensemble fold launch");
    } else {
      run_tick(h, in, true, true, 1, h->s.n);
      launch_check(launch_ensemble(h->s, (int)nx, h->d.elem == 8, h->ens_blocks, h->ens_shift, dst,
                                   h->stream),
                   "ensemble launch");
    }
    if (mem == FMSKF_MEM_HOST) {
      copy_out(h, out, h->ens_out, len * 8, mem);
      finish_out(h, mem);
    }
  });
}

int fmskf_ensemble_combine(uint32_t n_state, const double *records, uint32_t n_records,
                           double *mean, double *cov_packed) {
  return guarded([&] {
    if (n_state == 0 || n_state > 12 || !records) fail(FMSKF_EINVAL, "bad arguments");
    const uint32_t nx = n_state, np = nx * (nx + 1) / 2, len = 1 + nx + np;
    std::vector<double> acc(len, 0.0);
    for (uint32_t r = 0; r < n_records; r++) {  // fixed rank order: deterministic
      const double *b = records + (size_t)r * len;
      const double na = acc[0], nb = b[0];
      if (nb == 0.0) continue;
      if (na == 0.0) {
        acc.assign(b, b + len);
        continue;
      }
      const double nn = na + nb;
      double d[12];
      for (uint32_t k = 0; k < nx; k++) d[k] = b[1 + k] - acc[1 + k];
      const double f = na * nb / nn;
      for (uint32_t k = 0; k < nx; k++) acc[1 + k] = acc[1 + k] + d[k] * (nb / nn);
      for (uint32_t p = 0; p < nx; p++)
        for (uint32_t q = 0; q <= p; q++) {
          const uint32_t k = p * (p + 1) / 2 + q;
          acc[1 + nx + k] = acc[1 + nx + k] + b[1 + nx + k] + d[p] * d[q] * f;
        }
      acc[0] = nn;
    }
    if (mean)
      for (uint32_t k = 0; k < nx; k++) mean[k] = acc[1 + k];
    if (cov_packed)
      for (uint32_t k = 0; k < np; k++) cov_packed[k] = acc[0] > 1.0 ? acc[1 + nx + k] / (acc[0] - 1.0) : 0.0;
  });
}

}  // extern "C"
