"""BASELINE configs[0]'s full horizon at fleet size on the GPU: 60 000 ticks (60 s at 1 kHz) of
8192 KF6 robots through the bench's kernel form (k_kf6p, 16-byte fmskf_kf6_records, here with a
validity mask: one tick in 13 without a measurement), of 4096 EKF9 robots (k_ekf9p, raw IMU +
wheel records, compensated heading) and of 1024 KF12D fp64 robots (k_kf12s, cfg 5's model).  The inputs are one 1000-tick trajectory
(fmskf.synth.Trajectory), device-resident, replayed 60 times with a fresh validity mask per pass
(each replay restarts the measured motion: the filters also take the jump).  The state and the
covariance equal the oracle's (oracle/fmskf_oracle.c) bit for bit at every 1000th tick (KF12D:
within cfg 5's 1e-12, relative to each state's fleet scale): no rounding difference is allowed to
appear and compound over the horizon.  (The cfg 1 trace in
tests/test_oracle_frozen.py is one robot over the same horizon; tests/test_oracle_kf_long.py
holds the oracle itself against float64 over it.)"""
import numpy as np
import pytest

import fmskf
from fmskf import Engine
from fmskf.synth import Trajectory

pytestmark = pytest.mark.gpu

T_LONG = 60000
CHUNK = 1000


def _bits(a, b, what, t):
    ai, bi = a.view(np.uint32), b.view(np.uint32)
    if not np.array_equal(ai, bi):
        bad = np.argwhere(ai != bi)
        raise AssertionError(f"{what} differs at tick {t}: {bad.shape[0]} entries, first {bad[0].tolist()}")


def _moments(got, want, t):
    """the fused asynchronous ensemble record (the shift taken once, at the first record, while
    the fleet drifts for 60 s) against the oracle's two-pass moments of the same state: each mean
    within 1e-12 of max(|mean|, its standard deviation), each covariance entry within 1e-9 of
    sqrt(var_p var_q) (an entry near zero is judged against its variables' scale)"""
    (mg, cg), (mw, cw) = got, want
    nx = mw.size
    var = np.array([cw[p * (p + 1) // 2 + p] for p in range(nx)])
    sd = np.sqrt(np.maximum(var, 0.0))
    em = float(np.max(np.abs(mg - mw) / np.maximum(np.maximum(np.abs(mw), sd), 1e-300)))
    scale = np.array([sd[p] * sd[q] for p in range(nx) for q in range(p + 1)])
    ec = float(np.max(np.abs(cg - cw) / np.maximum(scale, 1e-300)))
    assert em <= 1e-12 and ec <= 1e-9, (t, em, ec)


def test_kf6_records_masked_60000_ticks(orc):
    import torch
    n = 8192
    cfg = fmskf.default_config("kf6", n)
    prm = orc.kf6_params(cfg.dt, np.array(cfg.q[:21]), np.array(cfg.r[:10]), orc.TRIG_TABLE512)
    xo = np.zeros((6, n), np.float32)
    Po = np.repeat(np.float32(np.array(cfg.p0[:21]))[:, None], n, 1).copy()
    rng = np.random.default_rng(1313)
    with Engine("kf6", n) as e:
        e.set_stream(torch.cuda.current_stream())
        yaw, gz, rpm = Trajectory(n, CHUNK, seed=0x464D534B ^ 7).kf6_inputs()
        rec_d = torch.from_numpy(fmskf.kf6_records(yaw, gz, rpm).view(np.int32).reshape(CHUNK, n, 4)).cuda()
        for t0 in range(0, T_LONG, CHUNK):
            valid = (rng.random((CHUNK, n)) > 1.0 / 13).astype(np.uint8)
            val_d = torch.from_numpy(valid).cuda()
            for k in range(CHUNK):
                if k == CHUNK - 1:  # the chunk's last tick also records the fleet's moments
                    e.tick_ensemble_begin(kf6_rec=rec_d[k], valid=val_d[k])
                else:
                    e.tick(kf6_rec=rec_d[k], valid=val_d[k])
                orc.kf6_tick(xo, Po, yaw[k], gz[k], rpm[k], valid[k], prm, nthreads=0)
            x, P = e.get_state()
            t = t0 + CHUNK - 1
            _bits(x, xo, "x", t)
            _bits(P, Po, "P", t)
            _moments(e.ensemble_end(), orc.ens_finalize(6, orc.ens_partial(xo)), t)
        assert e.get_counters()[0] == 0
    assert np.isfinite(xo).all() and np.abs(xo[:2]).max() > 1.0  # the robots went somewhere


def test_ekf9_masked_60000_ticks(orc):
    import torch
    n = 4096
    cfg = fmskf.default_config("ekf9", n)
    prm = orc.ekf9_params(cfg.dt, np.array(cfg.q[:45]), np.array(cfg.r[:21]), orc.TRIG_TABLE512)
    xo = np.zeros((10, n), np.float32)  # row 9: the heading's low part
    Po = np.repeat(np.float32(np.array(cfg.p0[:45]))[:, None], n, 1).copy()
    rng = np.random.default_rng(99)
    with Engine("ekf9", n) as e:
        e.set_stream(torch.cuda.current_stream())
        raw = Trajectory(n, CHUNK, seed=0x464D534B ^ 9).ekf9_raw()
        raw_d = torch.from_numpy(raw).cuda()
        for t0 in range(0, T_LONG, CHUNK):
            valid = (rng.random((CHUNK, n)) > 1.0 / 13).astype(np.uint8)
            val_d = torch.from_numpy(valid).cuda()
            for k in range(CHUNK):
                if k == CHUNK - 1:
                    e.tick_ensemble_begin(raw=raw_d[k], valid=val_d[k])
                else:
                    e.tick(raw=raw_d[k], valid=val_d[k])
                orc.ekf9_tick(xo, Po, raw[k], valid[k], prm, nthreads=0)
            x, P = e.get_state()
            t = t0 + CHUNK - 1
            _bits(x, xo[:9], "x", t)
            _bits(P, Po, "P", t)
            _moments(e.ensemble_end(), orc.ens_finalize(9, orc.ens_partial(np.ascontiguousarray(xo[:9]))), t)
        assert e.get_counters()[0] == 0


def test_kf12d_60000_ticks(orc):
    import torch
    n = 1024
    cfg = fmskf.default_config("kf12d", n)
    prm = orc.kf12d_params(cfg.dt, np.array(cfg.q[:78]), np.array(cfg.r[:36]))
    xo = np.zeros((12, n))
    Po = np.repeat(np.array(cfg.p0[:78])[:, None], n, 1).copy()
    worst = 0.0
    with Engine("kf12d", n) as e:
        e.set_stream(torch.cuda.current_stream())
        z = Trajectory(n, CHUNK, seed=0x464D534B ^ 12).kf12d_z()
        z_d = torch.from_numpy(z).cuda()
        for t0 in range(0, T_LONG, CHUNK):
            for k in range(CHUNK):
                e.tick(z=z_d[k])
                orc.kf12d_tick(xo, Po, z[k], None, prm, nthreads=0)
            x, P = e.get_state()
            scale = np.maximum(np.abs(xo).max(axis=1, keepdims=True), 1e-3)
            ex = float((np.abs(x - xo) / scale).max())
            ep = float((np.abs(P - Po) / max(np.abs(Po).max(), 1e-3)).max())
            assert ex <= 1e-12 and ep <= 1e-12, (t0 + CHUNK - 1, ex, ep)
            worst = max(worst, ex, ep)
        assert e.get_counters()[0] == 0
    print(f"kf12d 60000 ticks x {n}: max relative difference {worst:.3e}")


def test_isr_kf6_control_60000_ticks(orc):
    """The firmware ISR over the same horizon (fmskf_isr_tick: the KF6 tick, the wheel speed
    loops and the 0x200 frame in one kernel, k_isr_kf6), 2048 robots fed records with a
    validity mask, power and target-velocity events every few seconds: the estimator state, the
    FF_PI_D outputs, the current targets and the frame bytes equal the oracle's (kf6_tick +
    the control batch + can_tx) at every 1000th tick."""
    n = 2048
    rng = np.random.default_rng(4242)
    cfg = fmskf.default_config("kf6", n)
    prm = orc.kf6_params(cfg.dt, np.array(cfg.q[:21]), np.array(cfg.r[:10]), orc.TRIG_TABLE512)
    xo = np.zeros((6, n), np.float32)
    Po = np.repeat(np.float32(np.array(cfg.p0[:21]))[:, None], n, 1).copy()
    ref = orc.CtrlBatch(n)
    yaw, gz, rpm = Trajectory(n, CHUNK, seed=0x464D534B ^ 11).kf6_inputs()
    rec = fmskf.kf6_records(yaw, gz, rpm)
    with Engine("kf6", n) as e:
        for t0 in range(0, T_LONG, CHUNK):
            valid = (rng.random((CHUNK, n)) > 1.0 / 13).astype(np.uint8)
            if t0 % 6000 == 0:  # new targets (C_ACCEL / JERK_MAX_MOVE, VD_task_main.cpp:29-38)
                vel = np.stack([rng.uniform(-400, 400, n), rng.uniform(-400, 400, n),
                                rng.uniform(-6 * np.pi, 6 * np.pi, n)]).astype(np.float32)
                acl = np.array([[1000.0], [1000.0], [30.0]], np.float32).repeat(n, 1)
                jrk = np.array([[10000.0], [10000.0], [300.0]], np.float32).repeat(n, 1)
                e.set_target_vel(vel, acl, jrk)
                ref.set_target_vel(vel, acl, jrk)
            if t0 % 9000 == 0:  # power: most robots on, some off, changing every 9 s
                on = (rng.random(n) < 0.85).astype(np.uint8)
                e.set_power(on)
                ref.set_power(on)
            for k in range(CHUNK):
                last = k == CHUNK - 1
                fr = e.isr_tick(frames=last, kf6_rec=rec[k], valid=valid[k])
                orc.kf6_tick(xo, Po, yaw[k], gz[k], rpm[k], valid[k], prm, nthreads=0)
                ref.step(rpm[k])
            t = t0 + CHUNK - 1
            x, P = e.get_state()
            _bits(x, xo, "x", t)
            _bits(P, Po, "P", t)
            g = e.get_ctrl()
            cur = ref.curr()
            np.testing.assert_array_equal(g["curr"], cur, err_msg=f"currents at tick {t}")
            _bits(g["wheel_ctrl"], ref.wheel("ctrl"), "FF_PI_D output", t)
            _bits(g["vel_tgt"], ref.vel_tgt(), "velocity target", t)
            np.testing.assert_array_equal(fr, orc.can_tx(cur), err_msg=f"0x200 frames at tick {t}")
        assert e.get_counters()[0] == 0
    assert np.abs(cur).max() > 0  # the loops drove the wheels


@pytest.mark.parametrize("model", ["rs", "kf6"])
def test_firmware_pipeline_60000_ticks(orc, model):
    """The firmware's whole per-tick path for a fleet over the same horizon, device-resident:
    four C610 frames per robot every tick (fmskf_ingest_can, MOTOR_IF_M2006::rx_callback), a
    44-byte WT901 poll every 10 ticks (fmskf_ingest_wt901: WitSerialDataIn, CopeWitData,
    isComComp, updateData), and the tick on the ingested state (NULL planes: the yaw / gyro
    page, the wheel rpm and angle sums).  2048 robots; the RS model is the reference's own
    integrator (VD_vehicle_controller.cpp:36-51).  Against the batched oracle (the same
    restatements as tests/cfg1_trace.py's one robot): pose / state, covariance, the previous
    angle sums, the Data page and the motor state bit for bit at every 1000th tick."""
    import torch
    n = 2048
    tr = Trajectory(n, CHUNK, seed=0x464D534B ^ 21)
    frames = np.stack([tr.can_frames(k)[0] for k in range(CHUNK)])          # [T, N, 4, 8]
    polls = [tr.wt901_poll_rows(k) for k in range(0, CHUNK, 10)]
    frames_d = torch.from_numpy(frames).cuda()
    polls_d = [(torch.from_numpy(r).cuda(), torch.from_numpy(ln).cuda()) for r, ln in polls]
    wb, mb = orc.Wt901Batch(n), orc.MotorBatch(n)
    if model == "rs":
        pos, vel = np.zeros((3, n), np.float32), np.zeros((3, n), np.float32)
        prev = np.zeros((4, n), np.int64)
    else:
        cfg = fmskf.default_config("kf6", n)
        prm = orc.kf6_params(cfg.dt, np.array(cfg.q[:21]), np.array(cfg.r[:10]), orc.TRIG_TABLE512)
        xo = np.zeros((6, n), np.float32)
        Po = np.repeat(np.float32(np.array(cfg.p0[:21]))[:, None], n, 1).copy()
    with Engine(model, n) as e:
        e.set_stream(torch.cuda.current_stream())
        for t0 in range(0, T_LONG, CHUNK):
            g = t0 + np.arange(CHUNK)
            stamps = (((g[:, None, None] + 1) * 1000 + np.arange(4)[None, None, :] * 7) & 0x7FFF).astype(np.int16)
            stamps = np.ascontiguousarray(np.broadcast_to(stamps, (CHUNK, n, 4)))
            stamps_d = torch.from_numpy(stamps).cuda()
            for k in range(CHUNK):
                t = t0 + k
                e.ingest_can(frames_d[k], stamps_d[k])
                mb.rx(frames[k], stamps[k])
                if k % 10 == 0:
                    rows_d, lens_d = polls_d[k // 10]
                    e.ingest_wt901(rows_d, lens_d, latch_qinit=(t == 0))
                    wb.update(*polls[k // 10], latch_qinit=(t == 0))
                e.tick()
                d = wb.data
                rpm = mb.field("rpm")
                if model == "rs":
                    sums = np.ascontiguousarray(mb.field("angle_sum").T)
                    orc.rs_tick(pos, vel, prev, np.ascontiguousarray(d[11]), sums, rpm)
                else:
                    orc.kf6_tick(xo, Po, np.ascontiguousarray(d[11]), np.ascontiguousarray(d[5]), rpm, None, prm,
                                 nthreads=0)
            t = t0 + CHUNK - 1
            x, P = e.get_state()
            if model == "rs":
                _bits(x[:3], pos, "pose", t)
                _bits(x[3:], vel, "velocity", t)
                np.testing.assert_array_equal(e.get_prev_sum(), prev, err_msg=f"previous sums at tick {t}")
            else:
                _bits(x, xo, "x", t)
                _bits(P, Po, "P", t)
            data, err = e.get_imu()
            _bits(data, wb.data, "Data page", t)
            np.testing.assert_array_equal(err, wb.is_error, err_msg=f"IMU error flags at tick {t}")
            m = e.get_motors()
            np.testing.assert_array_equal(m["angle_sum"], mb.field("angle_sum").T, err_msg=f"angle sums at tick {t}")
            np.testing.assert_array_equal(m["rpm"], mb.field("rpm"), err_msg=f"rpm at tick {t}")
        assert e.get_counters()[0] == 0


def _motor_state(e, mb, t):
    """the whole C610 state (MOTOR_IF_M2006, VD_motor_if_m2006.cpp:32-72) against the oracle's:
    the int64 angle sums, every Status field (get_status_latest) incl. the IIR speed"""
    m = e.get_motors()
    st = e.get_motor_status()
    np.testing.assert_array_equal(m["angle_sum"], mb.field("angle_sum").T, err_msg=f"angle sums at tick {t}")
    for k, f in (("microsec_id", "micro"), ("angle", "angle"), ("rpm", "rpm"), ("curr", "curr")):
        np.testing.assert_array_equal(st[k], mb.field(f), err_msg=f"{k} at tick {t}")
    _bits(st["dlt_out_angle_rad"], mb.field("dlt_out_angle_rad"), "flt_dltOutAngle_rad", t)
    _bits(st["speed_radps"], mb.field("speed_radps"), "flt_SpeedRadPS", t)


@pytest.mark.parametrize("model", ["rs", "kf6", "ekf9"])
def test_isr_tick_can_firmware_60000_ticks(orc, model):
    """The default firmware call, fmskf_isr_tick_can (the millisecond's four C610 rx_callbacks and
    the whole ISR, can_tx_routine_intr, VD_task_main.cpp:366-372, in ONE kernel: k_isr_rs /
    k_isr_kf6 / k_isr_ekf9 with the C610 lane in front), over BASELINE configs[0]'s horizon
    against the oracle directly -- not against the library's own two-call path.  2048 robots,
    device-resident CAN frames every tick, a 44-byte WT901 poll every 10 ticks (RS, KF6: the
    tick reads the ingested yaw / gyro page; EKF9 reads its raw record), power and target events
    every few seconds.  At every 1000th tick, bit for bit: the motor state (orc_m2006_rx), the
    estimator state (orc_rs_tick / kf6_tick / ekf9_tick), the control state and currents
    (CtrlBatch) and the 0x200 frames (orc_can_tx).  The handle's launch-form counters show every
    tick ran as the one fused kernel."""
    import torch
    n = 2048
    rng = np.random.default_rng(0xF05ED ^ len(model))
    tr = Trajectory(n, CHUNK, seed=0x464D534B ^ 31)
    frames = np.stack([tr.can_frames(k)[0] for k in range(CHUNK)])          # [T, N, 4, 8]
    frames_d = torch.from_numpy(frames).cuda()
    wb, mb, ref = orc.Wt901Batch(n), orc.MotorBatch(n), orc.CtrlBatch(n)
    if model == "ekf9":
        raw = tr.ekf9_raw()
        raw_d = torch.from_numpy(raw).cuda()
        cfg = fmskf.default_config("ekf9", n)
        prm = orc.ekf9_params(cfg.dt, np.array(cfg.q[:45]), np.array(cfg.r[:21]), orc.TRIG_TABLE512)
        xo = np.zeros((10, n), np.float32)  # row 9: the heading's low part
        Po = np.repeat(np.float32(np.array(cfg.p0[:45]))[:, None], n, 1).copy()
    else:
        polls = [tr.wt901_poll_rows(k) for k in range(0, CHUNK, 10)]
        polls_d = [(torch.from_numpy(r).cuda(), torch.from_numpy(ln).cuda()) for r, ln in polls]
        if model == "rs":
            pos, vel = np.zeros((3, n), np.float32), np.zeros((3, n), np.float32)
            prev = np.zeros((4, n), np.int64)
        else:
            cfg = fmskf.default_config("kf6", n)
            prm = orc.kf6_params(cfg.dt, np.array(cfg.q[:21]), np.array(cfg.r[:10]), orc.TRIG_TABLE512)
            xo = np.zeros((6, n), np.float32)
            Po = np.repeat(np.float32(np.array(cfg.p0[:21]))[:, None], n, 1).copy()
    out_d = torch.empty((n, 8), dtype=torch.uint8, device="cuda")
    with Engine(model, n) as e:
        e.set_stream(torch.cuda.current_stream())
        for t0 in range(0, T_LONG, CHUNK):
            if t0 % 6000 == 0:  # new targets (C_ACCEL / JERK_MAX_MOVE, VD_task_main.cpp:29-38)
                vel_t = np.stack([rng.uniform(-400, 400, n), rng.uniform(-400, 400, n),
                                  rng.uniform(-6 * np.pi, 6 * np.pi, n)]).astype(np.float32)
                acl = np.array([[1000.0], [1000.0], [30.0]], np.float32).repeat(n, 1)
                jrk = np.array([[10000.0], [10000.0], [300.0]], np.float32).repeat(n, 1)
                e.set_target_vel(vel_t, acl, jrk)
                ref.set_target_vel(vel_t, acl, jrk)
            if t0 % 9000 == 0:  # power: most robots on, some off, changing every 9 s
                on = (rng.random(n) < 0.85).astype(np.uint8)
                e.set_power(on)
                ref.set_power(on)
            g = t0 + np.arange(CHUNK)
            stamps = (((g[:, None, None] + 1) * 1000 + np.arange(4)[None, None, :] * 7) & 0x7FFF).astype(np.int16)
            stamps = np.ascontiguousarray(np.broadcast_to(stamps, (CHUNK, n, 4)))
            stamps_d = torch.from_numpy(stamps).cuda()
            for k in range(CHUNK):
                t = t0 + k
                if model != "ekf9" and k % 10 == 0:  # the IMU task's 10 ms poll
                    rows_d, lens_d = polls_d[k // 10]
                    e.ingest_wt901(rows_d, lens_d, latch_qinit=(t == 0))
                    wb.update(*polls[k // 10], latch_qinit=(t == 0))
                last = k == CHUNK - 1
                kw = dict(raw=raw_d[k]) if model == "ekf9" else {}
                e.isr_tick_can(frames_d[k], stamps_d[k], frames=last, out=out_d if last else None, **kw)
                mb.rx(frames[k], stamps[k])
                rpm = mb.field("rpm")
                if model == "rs":
                    d = wb.data
                    orc.rs_tick(pos, vel, prev, np.ascontiguousarray(d[11]),
                                np.ascontiguousarray(mb.field("angle_sum").T), rpm)
                elif model == "kf6":
                    d = wb.data
                    orc.kf6_tick(xo, Po, np.ascontiguousarray(d[11]), np.ascontiguousarray(d[5]), rpm, None, prm,
                                 nthreads=0)
                else:
                    orc.ekf9_tick(xo, Po, raw[k], None, prm, nthreads=0)
                ref.step(rpm)
            t = t0 + CHUNK - 1
            x, P = e.get_state()
            if model == "rs":
                _bits(x[:3], pos, "pose", t)
                _bits(x[3:], vel, "velocity", t)
                np.testing.assert_array_equal(e.get_prev_sum(), prev, err_msg=f"previous sums at tick {t}")
            else:
                _bits(x, xo[:x.shape[0]], "x", t)
                _bits(P, Po, "P", t)
            _motor_state(e, mb, t)
            gc = e.get_ctrl()
            cur = ref.curr()
            np.testing.assert_array_equal(gc["curr"], cur, err_msg=f"currents at tick {t}")
            _bits(gc["wheel_ctrl"], ref.wheel("ctrl"), "FF_PI_D output", t)
            _bits(gc["wheel_tgt"], ref.wheel("tgt"), "FF_PI_D target", t)
            _bits(gc["vel_tgt"], ref.vel_tgt(), "velocity target", t)
            np.testing.assert_array_equal(out_d.cpu().numpy(), orc.can_tx(cur), err_msg=f"0x200 frames at tick {t}")
        c = e.get_counters()
        assert c[0] == 0, c[:3]
        assert c[1] == 0 and c[2] == 0, f"not every tick ran as the fused kernel: {c[:3]}"
    assert np.abs(cur).max() > 0  # the loops drove the wheels
