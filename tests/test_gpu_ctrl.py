"""GPU parity for SURVEY.md 8(f) rows 2-4: the vehicle control step, the C610 TX frame and
the VehicleInfo export, through the C ABI, against the oracle (itself pinned to the
reference's own FF_PI_D by tests/golden/ctrl_ref.npz, tests/test_oracle_ctrl.py).
Bar: bit-exact (float results compared as bit patterns, integers exactly)."""
import numpy as np
import pytest

import fmskf
from fmskf import Engine
from fmskf.synth import Trajectory

pytestmark = pytest.mark.gpu


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint32) if a.dtype == np.float32 else a


def _schedule(rng, n, T):
    """random set_target / power events: list per tick of (kind, payload)"""
    ev = {}
    for t in range(T):
        if t == 0 or rng.random() < 0.05:
            vel = np.stack([rng.uniform(-400, 400, n), rng.uniform(-400, 400, n),
                            rng.uniform(-6 * np.pi, 6 * np.pi, n)]).astype(np.float32)
            big = rng.random() < 0.5  # C_ACCEL/JERK_MAX_MOVE vs _STOP (VD_task_main.cpp:29-48)
            acl = np.array([[2000.0 if big else 1000.0], [2000.0 if big else 1000.0],
                            [70.0 if big else 30.0]], np.float32).repeat(n, 1)
            jrk = np.array([[30000.0 if big else 10000.0], [30000.0 if big else 10000.0],
                            [1000.0 if big else 300.0]], np.float32).repeat(n, 1)
            mask = (rng.random(n) < 0.7).astype(np.uint8)
            ev.setdefault(t, []).append(("target", (vel, acl, jrk, mask)))
        if t == 0 or rng.random() < 0.03:
            ev.setdefault(t, []).append(("power", (rng.random(n) < 0.85).astype(np.uint8)))
    return ev


@pytest.mark.parametrize("n,T", [(1, 50), (3001, 300)])
def test_control_step_bitexact(orc, n, T):
    rng = np.random.default_rng(1234 + n)
    ev = _schedule(rng, n, T)
    ref = orc.CtrlBatch(n)
    with Engine("kf6", n) as e:
        for t in range(T):
            for kind, pl in ev.get(t, []):
                if kind == "target":
                    e.set_target_vel(*pl)
                    ref.set_target_vel(*pl)
                else:
                    e.set_power(pl)
                    ref.set_power(pl)
            rpm = rng.integers(-9000, 9000, (n, 4)).astype(np.int16)
            e.control(rpm)
            ref.step(rpm)
        got = e.get_ctrl()
        frames = e.can_tx()
    np.testing.assert_array_equal(got["curr"], ref.curr())
    np.testing.assert_array_equal(bits(got["vel_tgt"]), bits(ref.vel_tgt()))
    np.testing.assert_array_equal(bits(got["wheel_tgt"]), bits(ref.wheel("tgt")))
    np.testing.assert_array_equal(bits(got["wheel_ctrl"]), bits(ref.wheel("ctrl")))
    np.testing.assert_array_equal(frames, orc.can_tx(ref.curr()))


def test_control_custom_params_and_d_term(orc):
    n, T = 777, 120
    rng = np.random.default_rng(5)
    kw = dict(ctrl_freq_hz=1000.0, ff_gain=0.01, p_gain=0.05, i_gain=0.2, d_gain=0.004,
              i_limit=0.8, lpf_freq_hz=25.0, ff_limit=0.7, interp_ts=np.float32(0.001),
              curr_limit_raw=2500)
    prm = orc.ctrl_params(c_freq=1000.0, ff=0.01, pg=0.05, ig=0.2, dg=0.004, ilim=0.8, lpf=25.0,
                          fflim=0.7, ts=np.float32(0.001), clim=2500)
    ref = orc.CtrlBatch(n, prm)
    vel = np.stack([rng.uniform(-400, 400, n), rng.uniform(-400, 400, n),
                    rng.uniform(-3, 3, n)]).astype(np.float32)
    acl = np.array([[1000.0], [1000.0], [30.0]], np.float32).repeat(n, 1)
    jrk = np.array([[10000.0], [10000.0], [300.0]], np.float32).repeat(n, 1)
    with Engine("rs", n) as e:
        e.set_ctrl_params(**kw)
        e.set_power(None)
        ref.set_power(np.ones(n, np.uint8))
        e.set_target_vel(vel, acl, jrk)
        ref.set_target_vel(vel, acl, jrk)
        for t in range(T):
            rpm = rng.integers(-300, 300, (n, 4)).astype(np.int16)
            e.control(rpm)
            ref.step(rpm)
        got = e.get_ctrl()
    np.testing.assert_array_equal(got["curr"], ref.curr())
    np.testing.assert_array_equal(bits(got["wheel_ctrl"]), bits(ref.wheel("ctrl")))


def test_control_outputs_formed_on_demand(orc, tmp_path):
    """Round 6: the step leaves vel_tgt and FF_PI_D now_tgt / now_ctrl to be formed when read
    (ctrl_lane.hpp ctrl_derive_lane).  A readout still returns the LAST step's outputs after the
    parameters change, after the power flags and targets change, after graph replays whose
    captured steps ran with parameters changed since, and through a checkpoint; robots switched
    off keep the interpolators' last output (VD_vehicle_controller.cpp, FF_PI_D reset)."""
    import torch
    n = 1537
    rng = np.random.default_rng(77)
    kw_b = dict(ctrl_freq_hz=1000.0, ff_gain=0.01, p_gain=0.05, i_gain=0.2, d_gain=0.004,
                i_limit=0.8, lpf_freq_hz=25.0, ff_limit=0.7, interp_ts=np.float32(0.001),
                curr_limit_raw=2500)
    prm_b = orc.ctrl_params(c_freq=1000.0, ff=0.01, pg=0.05, ig=0.2, dg=0.004, ilim=0.8, lpf=25.0,
                            fflim=0.7, ts=np.float32(0.001), clim=2500)
    prm_a = orc.ctrl_params()
    ref = orc.CtrlBatch(n, prm_a)

    def targets():
        vel = np.stack([rng.uniform(-400, 400, n), rng.uniform(-400, 400, n),
                        rng.uniform(-6, 6, n)]).astype(np.float32)
        return vel, np.full((3, n), 1000.0, np.float32), np.full((3, n), 10000.0, np.float32)

    def rpm():
        return rng.integers(-900, 900, (n, 4)).astype(np.int16)

    def check(e, what):
        got = e.get_ctrl()
        np.testing.assert_array_equal(got["curr"], ref.curr(), err_msg=what)
        np.testing.assert_array_equal(bits(got["vel_tgt"]), bits(ref.vel_tgt()), err_msg=what)
        np.testing.assert_array_equal(bits(got["wheel_tgt"]), bits(ref.wheel("tgt")), err_msg=what)
        np.testing.assert_array_equal(bits(got["wheel_ctrl"]), bits(ref.wheel("ctrl")), err_msg=what)

    st = torch.cuda.Stream()
    with Engine("kf6", n) as e:
        e.set_stream(st)
        pw = (rng.random(n) < 0.8).astype(np.uint8)
        e.set_power(pw)
        ref.set_power(pw)
        tv = targets()
        e.set_target_vel(*tv)
        ref.set_target_vel(*tv)
        for _ in range(6):
            r = rpm()
            e.control(r)
            ref.step(r)
        e.set_ctrl_params(**kw_b)  # the last step ran with the defaults
        check(e, "after set_ctrl_params")
        ref.p = prm_b
        r = rpm()
        e.control(r)
        ref.step(r)
        pw = (rng.random(n) < 0.5).astype(np.uint8)  # power and targets change after the step
        e.set_power(pw)
        ref.set_power(pw)
        tv = targets()
        e.set_target_vel(*tv)
        ref.set_target_vel(*tv)
        check(e, "after set_power / set_target_vel")
        for _ in range(2):  # steps with robots just switched off (their outputs are stored)
            r = rpm()
            e.control(r)
            ref.step(r)
        check(e, "power-off robots")
        # a graph of two steps captured with parameters B, replayed after switching to A
        rr = [rpm() for _ in range(2)]
        dev = [torch.from_numpy(x).cuda() for x in rr]
        torch.cuda.synchronize()
        e.graph_begin()
        for d in dev:
            e.control(d)
        e.graph_end()
        e.set_ctrl_params()  # defaults (A) from now on; the replays keep B
        e.graph_launch(3)
        for _ in range(3):
            for x in rr:
                ref.step(x)
        st.synchronize()
        check(e, "graph replays")
        ref.p = prm_a
        r = rpm()
        e.control(r)  # a direct step with A after the replays
        ref.step(r)
        e.save_state(tmp_path / "ctrl.ck")  # a checkpoint right after a step
        with Engine("kf6", n) as b:
            b.load_state(tmp_path / "ctrl.ck")
            check(b, "checkpoint")
        check(e, "direct step after the replays")


def test_control_reads_ingested_motor_state():
    n = 513
    T = 6
    tr = Trajectory(n, T, seed=17)
    vel = np.zeros((3, n), np.float32)
    vel[0] = 150.0
    acl = np.full((3, n), 1000.0, np.float32)
    jrk = np.full((3, n), 10000.0, np.float32)
    with Engine("kf6", n) as a, Engine("kf6", n) as b:
        for e in (a, b):
            e.set_power(None)
            e.set_target_vel(vel, acl, jrk)
        for t in range(T):
            fr, st = tr.can_frames(t)
            a.ingest_can(fr, st)
            rpm = a.get_motors()["rpm"]
            a.control()          # NULL rpm: the device-resident motor state
            b.control(rpm)
        np.testing.assert_array_equal(a.get_ctrl()["curr"], b.get_ctrl()["curr"])


def test_vehicle_info_export_bitexact(orc):
    n, T = 2049, 20
    tr = Trajectory(n, T, seed=23)
    yaw, gz, rpm = tr.kf6_inputs()
    buf = np.zeros((n, 48), np.uint8)
    lens = np.zeros(n, np.uint32)
    for i in range(n):
        b = np.frombuffer(tr.wt901_poll_bytes(0, i), np.uint8)
        buf[i, :b.size] = b
        lens[i] = b.size
    lens[::7] = 0  # no bytes this poll -> is_error, exported as imu.fault 0xFF
    rng = np.random.default_rng(3)
    floor = rng.integers(0, 2, (n, 8)).astype(np.uint8)
    cam = rng.uniform(-30, 30, n).astype(np.float32)
    fault = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    for model in ("rs", "kf6"):
        with Engine(model, n) as e:
            e.ingest_wt901(buf, lens, latch_qinit=True)
            for t in range(T):
                if model == "rs":
                    e.tick(yaw_deg=yaw[t], angle_sum=np.zeros((4, n), np.int64), rpm=rpm[t])
                else:
                    e.tick(yaw_deg=yaw[t], gyro_z_dps=gz[t], rpm=rpm[t])
            rec = e.export_vehicle_info(floor, cam, fault)
            px, py, pth = e.get_pose()
            vx, vy, vth = e.get_vel()
            data, err = e.get_imu()
        ref = orc.vehicle_info(px, py, pth, vx, vy, vth, data, err, floor=floor, cam_pitch=cam,
                               fault=fault)
        assert rec.tobytes() == ref.tobytes(), model
    assert set(np.unique(rec["imu_fault"])) <= {0, 0xFF}


def test_control_large_n_properties():
    """N = 2^20 robots, all powered, one target: every robot's interpolator reaches the
    target; currents stay within the limit; TX frames decode back to the currents."""
    import torch
    n = 1 << 20
    with Engine("kf6", n) as e:
        e.set_power(None)
        vel = np.zeros((3, n), np.float32)
        vel[0] = 200.0
        vel[2] = -1.0
        e.set_target_vel(vel, np.full((3, n), 1000.0, np.float32) * np.float32([[1], [1], [0.03]]),
                         np.full((3, n), 10000.0, np.float32) * np.float32([[1], [1], [0.03]]))
        rpm = torch.zeros((n, 4), dtype=torch.int16, device="cuda")
        for _ in range(400):
            e.control(rpm)
        got = e.get_ctrl()
        fr = e.can_tx()
    assert (got["vel_tgt"][0] == np.float32(200.0)).all()
    assert (got["vel_tgt"][2] == np.float32(-1.0)).all()
    assert np.abs(got["curr"]).max() <= 3000
    dec = ((fr[:, 0::2].astype(np.int32) << 8) | fr[:, 1::2]).astype(np.uint16).view(np.int16)
    np.testing.assert_array_equal(dec, got["curr"])


def test_fleet_loop_cpp_host_program():
    """examples/fleet_loop.cpp (C++ over the C ABI, the firmware's task structure incl. the
    wheel loops, TX frames and the VehicleInfo publish) runs and prints sane values."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "build", "fleet_loop")
    assert os.path.exists(exe), "build() makes build/fleet_loop"
    out = subprocess.run([exe, "4096", "200"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.strip().splitlines()
    assert lines[0].startswith("robots=4096 ticks=200")
    x0 = float(lines[1].split("x=")[1].split()[0])
    assert 0.0 < x0 < 1.0          # driven forward for 0.2 s
    assert "imu.fault=0" in lines[2]
    # the asynchronous ensemble every 16 ticks (fmskf_ensemble_begin / _end, two results late):
    # 12 records, the fleet mean of x between the slowest and fastest robots' x
    assert lines[3].startswith("fleet (1 rank): 12 ensemble records"), lines[3]
    mx = float(lines[3].split("mean x=")[1].split()[0])
    vx = float(lines[3].split("var x=")[1].split()[0].rstrip(","))
    assert 0.0 < mx < 1.0 and vx > 0.0
    assert lines[3].endswith("4096 robots in 1 records"), lines[3]  # fmskf_ensemble_end_count
    # MOTOR_IF_M2006::get_status_latest: robot 0's FL wheel advances 1 count (1 raw angle) a tick
    assert lines[4].startswith("robot 0 FL: microsec_id="), lines[4]
    dlt = float(lines[4].split("dlt=")[1].split()[0])
    assert abs(dlt - 2 * 3.1415926 / 8191 / 36) < 1e-6 * dlt, lines[4]


@pytest.mark.parametrize("model", ["rs", "kf6"])
def test_fleet_loop_cpp_fused_can_equals_split(model):
    """examples/fleet_loop.cpp with the tick's CAN RX inside the ISR call (fmskf_isr_tick_can,
    the default; one kernel for RS, KF6 and EKF9) prints exactly what the split form (rx_callback, then
    can_tx_routine) prints: poses, VehicleInfo, TX frame bytes, the ensemble and motor Status."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "build", "fleet_loop")
    outs = []
    for split in ("0", "1"):
        env = dict(os.environ, FLEET_MODEL=model, FLEET_SPLIT_CAN=split)
        out = subprocess.run([exe, "3000", "120"], capture_output=True, text=True, timeout=300, env=env)
        assert out.returncode == 0, out.stderr
        outs.append(out.stdout.strip().splitlines()[1:])  # line 0: wall time
    assert outs[0] == outs[1]
    assert float(outs[0][0].split("x=")[1].split()[0]) > 0.0


def test_reset_zeroes_control_state():
    n = 300
    with Engine("rs", n) as e:
        e.set_power(None)
        vel = np.full((3, n), 100.0, np.float32)
        e.set_target_vel(vel, np.full((3, n), 1000.0, np.float32), np.full((3, n), 10000.0, np.float32))
        for _ in range(20):
            e.control(np.full((n, 4), 50, np.int16))
        assert np.abs(e.get_ctrl()["curr"]).max() > 0
        e.reset()
        g = e.get_ctrl()
        assert not g["curr"].any() and not g["vel_tgt"].any() and not g["wheel_ctrl"].any()
        e.control(np.full((n, 4), 50, np.int16))   # power is off after reset
        assert not e.get_ctrl()["curr"].any()


# EKF9 (round 5): one fused kernel (k_isr_ekf9) while its state is cache-resident, with LIBM, a
# mask, COMP_POS, one robot and 2^20 + 17 robots (the control planes non-temporal).
# KF6: one fused kernel (k_isr_kf6) for planes / records, TABLE512 / LIBM, with or without a
# validity mask; at 2^20 + 17 the KF6 + control state outgrows the Infinity Cache and the
# fused kernel's control planes go non-temporal
@pytest.mark.parametrize("model,n,T", [("rs", 3001, 200), ("rs", 1, 30), ("kf6", 1000, 60),
                                       ("kf6rec", 999, 40), ("kf6libm", 777, 30), ("kf6mask", 1001, 30),
                                       ("kf6recmask", 1, 20), ("kf6rec", (1 << 20) + 17, 4),
                                       ("ekf9", 1000, 40), ("ekf9", 1, 20), ("ekf9libm", 513, 20),
                                       ("ekf9mask", 777, 30), ("ekf9comp", 600, 20), ("ekf9", (1 << 20) + 17, 3)])
def test_isr_tick_equals_tick_control_can_tx(orc, model, n, T):
    """fmskf_isr_tick (the firmware ISR in one call; one fused kernel for RS and KF6) leaves
    the estimator state, the control state and the 0x200 frames bit-identical to fmskf_tick +
    fmskf_control + fmskf_can_tx, with random power and target events; RS also against the
    oracle's pose, and both against the oracle's control batch directly."""
    rng = np.random.default_rng(99 + n)
    ev = _schedule(rng, n, T)
    tr = Trajectory(n, T, seed=31)
    trig = fmskf.TRIG_LIBM if model.endswith("libm") else fmskf.TRIG_TABLE512
    valid = (rng.random((T, n)) > 0.25).astype(np.uint8) if model.endswith("mask") else None
    vk = (lambda t: {}) if valid is None else (lambda t: dict(valid=valid[t]))  # noqa: E731
    flags = 0
    if model.startswith("ekf9"):  # the raw WT901 words + rpm; the control step reads the rpm plane
        flags = fmskf.CFG_COMP_POS if model == "ekf9comp" else 0
        raw = tr.ekf9_raw()
        _, _, rpm = tr.kf6_inputs()
        kw = [dict(raw=raw[t], rpm=rpm[t], **vk(t)) for t in range(T)]
        model = "ekf9"
    elif model == "rs":
        yaw, sums, rpm = tr.rs_inputs()
        kw = [dict(yaw_deg=yaw[t], angle_sum=sums[t], rpm=rpm[t]) for t in range(T)]
    elif not model.startswith("kf6rec"):
        yaw, gz, rpm = tr.kf6_inputs()
        kw = [dict(yaw_deg=yaw[t], gyro_z_dps=gz[t], rpm=rpm[t], **vk(t)) for t in range(T)]
        model = "kf6"
    else:  # KF6 fed 16-byte records: the control step reads the records' rpm field
        from fmskf import kf6_records
        yaw, gz, rpm = tr.kf6_inputs()
        rec = kf6_records(yaw, gz, rpm)
        kw = [dict(kf6_rec=rec[t], **vk(t)) for t in range(T)]
        model = "kf6"
    ref = orc.CtrlBatch(n)
    pos = np.zeros((3, n), np.float32)
    vel = np.zeros((3, n), np.float32)
    prev = np.zeros((4, n), np.int64)
    with Engine(model, n, trig=trig, flags=flags) as a, Engine(model, n, trig=trig, flags=flags) as b:
        for t in range(T):
            for kind, pl in ev.get(t, []):
                for e in (a, b):
                    (e.set_target_vel(*pl) if kind == "target" else e.set_power(pl))
                (ref.set_target_vel(*pl) if kind == "target" else ref.set_power(pl))
            fa = a.isr_tick(**kw[t]) if t % 7 else a.isr_tick(frames=False, **kw[t])
            b.tick(**kw[t])
            b.control(rpm[t])  # the plane rpm: equal to the records' field
            fb = b.can_tx()
            if t % 7:
                np.testing.assert_array_equal(fa, fb)
            ref.step(rpm[t])
            if model == "rs":
                orc.rs_tick(pos, vel, prev, yaw[t], np.ascontiguousarray(sums[t]), rpm[t])
        xa, Pa = a.get_state()
        xb, Pb = b.get_state()
        ga, gb = a.get_ctrl(), b.get_ctrl()
        if model == "rs":
            np.testing.assert_array_equal(a.get_prev_sum(), prev)
    np.testing.assert_array_equal(bits(xa), bits(xb))
    if Pa is not None:
        np.testing.assert_array_equal(bits(Pa), bits(Pb))
    for k in ("vel_tgt", "curr", "wheel_tgt", "wheel_ctrl"):
        np.testing.assert_array_equal(bits(ga[k]), bits(gb[k]))
    np.testing.assert_array_equal(ga["curr"], ref.curr())
    np.testing.assert_array_equal(bits(ga["wheel_ctrl"]), bits(ref.wheel("ctrl")))
    if model == "rs":
        np.testing.assert_array_equal(bits(xa[:3]), bits(pos))
        np.testing.assert_array_equal(bits(xa[3:]), bits(vel))


def test_isr_tick_device_resident_and_graph():
    """The whole firmware pipeline on device-resident state: CAN ingest -> fmskf_isr_tick with
    NULL planes (IMU yaw page, motor rpm and angle sums) into a device frame buffer, captured
    as a HIP graph and replayed: identical to direct calls."""
    import torch
    n, T = 4099, 12
    tr = Trajectory(n, T, seed=41)
    vel = np.zeros((3, n), np.float32)
    vel[1] = 120.0
    acl = np.full((3, n), 1000.0, np.float32)
    jrk = np.full((3, n), 10000.0, np.float32)
    frames = [tr.can_frames(t) for t in range(T)]
    dev = [(torch.from_numpy(np.ascontiguousarray(f)).cuda(), torch.from_numpy(np.ascontiguousarray(s)).cuda())
           for f, s in frames]
    out_a = torch.zeros((n, 8), dtype=torch.uint8, device="cuda")
    out_b = torch.zeros((n, 8), dtype=torch.uint8, device="cuda")
    st = torch.cuda.Stream()
    with Engine("rs", n) as a, Engine("rs", n) as b:
        for e in (a, b):
            e.set_stream(st)
            e.set_power(None)
            e.set_target_vel(vel, acl, jrk)
        for t in range(T):
            a.ingest_can(*dev[t])
            a.isr_tick(out=out_a)
            b.ingest_can(*dev[t])
            b.tick()
            b.control()
            b.can_tx(out=out_b)
            st.synchronize()
            assert torch.equal(out_a, out_b)
        # graph replay of the ISR alone on the final motor state, against direct calls
        a.graph_begin()
        a.isr_tick(out=out_a)
        a.graph_end()
        a.graph_launch(5)
        for _ in range(5):
            b.isr_tick(out=out_b)
        st.synchronize()
        assert torch.equal(out_a, out_b)
        np.testing.assert_array_equal(bits(a.get_state()[0]), bits(b.get_state()[0]))


@pytest.mark.parametrize("model", ["rs", "kf6", "ekf9"])
def test_checkpoint_resume_bitexact(tmp_path, model):
    """fmskf_save_state / load_state (SURVEY.md 5 checkpoint/resume): run the firmware
    pipeline (CAN + WT901 ingest, the ISR tick with control and TX frames) for T ticks in one
    handle; in another, stop halfway, checkpoint, resume in a fresh handle and finish.  Every
    readout agrees bit for bit; a checkpoint of another N is rejected."""
    import fmskf
    n, T = 777, 24
    tr = Trajectory(n, T, seed=71)
    vel = np.zeros((3, n), np.float32)
    vel[0] = 120.0
    vel[2] = 0.5
    acl = np.full((3, n), 1000.0, np.float32)
    jrk = np.full((3, n), 10000.0, np.float32)
    raw = tr.ekf9_raw() if model == "ekf9" else None

    def step(e, t):
        fr, st = tr.can_frames(t)
        e.ingest_can(fr, st)
        if t % 10 == 0:
            buf = np.zeros((n, 48), np.uint8)
            lens = np.zeros(n, np.uint32)
            for i in range(n):
                b = np.frombuffer(tr.wt901_poll_bytes(t, i), np.uint8)
                buf[i, :b.size] = b
                lens[i] = b.size
            e.ingest_wt901(buf, lens, latch_qinit=(t == 0))
        if model == "ekf9":
            e.tick(raw=raw[t])
            e.control()
            return e.can_tx()
        return e.isr_tick()

    def readout(e):
        x, P = e.get_state()
        motors = dict(e.get_motors(), **{"status_" + k: v for k, v in e.get_motor_status().items()})
        out = dict(x=x, ctrl=e.get_ctrl(), motors=motors, imu=e.get_imu())
        if P is not None:
            out["P"] = P
        return out

    with Engine(model, n) as a:
        a.set_power(None)
        a.set_target_vel(vel, acl, jrk)
        fa = [step(a, t) for t in range(T)]
        ra = readout(a)
    ck = tmp_path / "fleet.ck"
    with Engine(model, n) as b:
        b.set_power(None)
        b.set_target_vel(vel, acl, jrk)
        fb = [step(b, t) for t in range(T // 2)]
        b.save_state(ck)
    with Engine(model, n) as c:
        c.load_state(ck)
        fb += [step(c, t) for t in range(T // 2, T)]
        rc = readout(c)
    for t in range(T):
        np.testing.assert_array_equal(fa[t], fb[t])
    np.testing.assert_array_equal(bits(ra["x"]), bits(rc["x"]))
    if "P" in ra:
        np.testing.assert_array_equal(bits(ra["P"]), bits(rc["P"]))
    for k in ra["ctrl"]:
        np.testing.assert_array_equal(bits(ra["ctrl"][k]), bits(rc["ctrl"][k]))
    for k in ra["motors"]:
        np.testing.assert_array_equal(ra["motors"][k], rc["motors"][k])
    np.testing.assert_array_equal(bits(ra["imu"][0]), bits(rc["imu"][0]))
    with Engine(model, n + 1) as d:
        with pytest.raises(fmskf.FmskfError):
            d.load_state(ck)
    # a truncated file, one with trailing bytes, one with a flipped byte in the middle (the
    # checksum), a format-1 file (no recorded control / motor layout) or a format-2 one (motor
    # planes no longer kept) is rejected before any
    # copy: the handle keeps its state
    blob = ck.read_bytes()
    mid = len(blob) // 2
    flipped = blob[:mid] + bytes([blob[mid] ^ 0x40]) + blob[mid + 1:]
    v1 = b"FMSKFCK1" + blob[8:]
    v2 = b"FMSKFCK2" + blob[8:]  # format 2 kept the dlt / speed motor planes
    v3 = b"FMSKFCK3" + blob[8:]  # format 3 had no previous motor angles (ABI 2)
    v4 = b"FMSKFCK4" + blob[8:]  # format 4 kept the motor IIR state as [4][N] planes
    cases = [("cut", blob[:-5]), ("long", blob + b"\0"), ("flip", flipped), ("v1", v1), ("v2", v2), ("v3", v3),
             ("v4", v4)]
    if model == "rs":  # a round-5 RS file: header layout word 0, the previous sums as [4][N] planes
        cases.append(("rs_r5", blob[:84] + b"\0\0\0\0" + blob[88:]))
    with Engine(model, n) as e:
        e.load_state(ck)
        before = readout(e)
        for name, data in cases:
            bad = tmp_path / name
            bad.write_bytes(data)
            with pytest.raises(fmskf.FmskfError):
                e.load_state(bad)
            after = readout(e)
            np.testing.assert_array_equal(bits(before["x"]), bits(after["x"]))
            for k in before["motors"]:
                np.testing.assert_array_equal(before["motors"][k], after["motors"][k])
    # state the checkpoint does not hold is reset on load: a handle that has ingested CAN
    # frames, loaded from a checkpoint saved before any ingest, reads zero motor state
    fresh = tmp_path / "fresh.ck"
    with Engine(model, n) as f0:
        f0.save_state(fresh)
    with Engine(model, n) as g:
        step(g, 0)
        g.load_state(fresh)
        for k, v in g.get_motors().items():
            assert not np.any(v), k


_NT_SCRIPT = r"""
import sys
sys.path[:0] = sys.argv[1:4]
from oracle import oracle as orc
import test_gpu_ctrl as T
T.test_isr_tick_equals_tick_control_can_tx(orc, "rs", 3001, 60)
T.test_isr_tick_equals_tick_control_can_tx(orc, "kf6rec", 999, 30)
T.test_control_step_bitexact(orc, 3001, 100)
import test_gpu_parity as P
P.test_can_ingest_bitexact(orc, False, 777)
print("nt ok")
"""


def test_nontemporal_control_and_isr_bitexact():
    """The non-temporal control-state instantiations of k_ctrl_step and k_isr_rs, and the
    non-temporal motor-state CAN ingest k_can4<true> (chosen
    automatically once the state outgrows the Infinity Cache, fmskf_internal.hpp state_nt)
    forced on at small N in a child process: the ISR and control parity tests above, against
    the three-call sequence and the oracle."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, FMSKF_STATE_NT="1")
    out = subprocess.run([sys.executable, "-c", _NT_SCRIPT, root,
                          os.path.join(root, "roboken-fmskf-robot-controller_amd"),
                          os.path.join(root, "tests")],
                         capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "nt ok" in out.stdout
