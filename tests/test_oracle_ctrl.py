"""Oracle rows of SURVEY.md 8(f) 2-4: the vehicle control step, the C610 TX frame and the
VehicleInfo export.

* FF_PI_D (util_controller.hpp) is pinned bit for bit by tests/golden/ctrl_ref.npz, made
  by tests/golden/make_golden_ctrl.py from the reference's own header compiled here.
* VelInterpConstJerk (util_vel_interp.hpp) includes arm_math.h (CMSIS-DSP, absent): it is
  pinned by known answers derived from its own formulas (profile durations, the reached
  velocity, the no-constant-acceleration branch); arm_sqrt_f32 is parity unpinned.
* The integer conversions follow Cortex-M7 semantics (VCVT saturates, NaN -> 0, the int16
  narrowing keeps the low 16 bits) and are pinned by hand-derived known answers.
"""
import ctypes as C
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def golden_ctrl():
    d = np.load(os.path.join(ROOT, "tests", "golden", "ctrl_ref.npz"))
    return {k: d[k] for k in d.files}


def test_ffpid_matches_reference_golden(orc, golden_ctrl):
    g = golden_ctrl
    keys = [str(k) for k in g["gain_keys"]]
    assert len(g["name"]) >= 10
    for s in range(len(g["name"])):
        a = dict(zip(keys, g["gains"][s].tolist()))
        prm = orc.ctrl_params(c_freq=a["c_freq"], ff=a["ff"], pg=a["pg"], ig=a["ig"], dg=a["dg"],
                              ilim=a["ilim"], lpf=a["lpf"], fflim=a["fflim"])
        pid = orc.Pid()
        L = orc.lib()
        out = np.zeros(g["tgt"].shape[1], np.float32)
        for k in range(out.size):
            if g["reset"][s, k]:
                L.orc_pid_reset(C.byref(pid))
            pid.tgt = float(g["tgt"][s, k])
            out[k] = L.orc_pid_update(C.byref(pid), C.byref(prm), float(g["val"][s, k]))
            assert np.float32(pid.val) == g["now_val"][s, k]
        bad = np.nonzero(out.view(np.uint32) != g["ctrl"][s].view(np.uint32))[0]
        assert bad.size == 0, f"{g['name'][s]}: first mismatch at step {bad[0]}"


def _run_interp(orc, v0, vt, am, jrk, steps, ts=np.float32(0.001)):
    L = orc.lib()
    s = orc.Interp()
    L.orc_interp_reset(C.byref(s))
    s.vel_now = float(v0)
    L.orc_interp_set(C.byref(s), float(vt), float(am), float(jrk))
    vel = np.array([L.orc_interp_update(C.byref(s), float(ts)) for _ in range(steps)], np.float32)
    return s, vel


def test_interp_trapezoid_known_answer(orc):
    # 0 -> 200 mm/s, a 1000, j 10000 (C_ACCEL/JERK_MAX_MOVE.x, VD_task_main.cpp:29-38):
    # dt1 = dt3 = a/j = 0.1 s, dt2 = (200 - a*(dt1+dt3)/2)/a = 0.1 s
    s, vel = _run_interp(orc, 0.0, 200.0, 1000.0, 10000.0, 400)
    assert abs(s.dt1 - 0.1) < 1e-6 and abs(s.dt3 - 0.1) < 1e-6 and abs(s.dt2 - 0.1) < 1e-5
    assert s.jerk_p == 10000.0 and s.jerk_m == -10000.0 and s.acl_max == 1000.0
    t = np.arange(400, dtype=np.float64) * 0.001
    # jerk phase: v = j t^2 / 2 (the kernel evaluates at dt before increment)
    k = t <= 0.1
    np.testing.assert_allclose(vel[k], 0.5 * 10000.0 * t[k] ** 2, rtol=0, atol=2e-3)
    assert vel[-1] == np.float32(200.0)  # final branch sets the target exactly
    # monotone up to the last decel step; that step evaluates acl_max + jerk_m*(dt-dt1-dt2)
    # one sample past dt3 (the `<= ... + ts_` bounds), a small negative acceleration the
    # reference really produces (199.4999 -> 199.4899) before snapping to the target
    assert np.all(np.diff(vel[:301].astype(np.float64)) >= -1e-4)
    assert vel[301] < vel[300] and vel[302] == np.float32(200.0)
    assert abs(vel[200] - 150.0) < 1.5  # mid constant-accel section


def test_interp_short_move_sqrt_branch(orc):
    # 0 -> 5 mm/s: dt2 < 0 -> dt1 = sqrt(dv/j) = 0.02236, peak accel j*dt1 = 223.6
    s, vel = _run_interp(orc, 0.0, 5.0, 1000.0, 10000.0, 100)
    assert s.dt2 == 0.0
    assert abs(s.dt1 - np.sqrt(5.0 / 10000.0)) < 1e-6
    assert abs(s.acl_max - 10000.0 * np.sqrt(5.0 / 10000.0)) < 1e-3
    assert vel[-1] == np.float32(5.0)


def test_interp_decelerate_negative(orc):
    # from 300 down to -100: acl_max flips sign, jerk_p negative
    s, vel = _run_interp(orc, 300.0, -100.0, 2000.0, 30000.0, 600)
    assert s.acl_max < 0 and s.jerk_p == -30000.0 and s.jerk_m == 30000.0
    assert vel[-1] == np.float32(-100.0)
    assert vel.min() >= np.float32(-100.5) and vel.max() <= np.float32(300.5)


def test_interp_reset_then_update_is_zero(orc):
    L = orc.lib()
    s = orc.Interp()
    L.orc_interp_reset(C.byref(s))
    assert L.orc_interp_update(C.byref(s), 0.001) == 0.0
    assert s.dt > 0


def test_curr_to_raw_known_answers(orc):
    f = orc.lib().orc_curr_to_raw
    assert f(0.5, 1, 3000) == 500
    assert f(0.5, -1, 3000) == -500
    assert f(-0.0019, 1, 3000) == -1          # truncation toward zero
    assert f(3.5, 1, 3000) == 3000            # saturation at s16_rawCurr_lim
    assert f(-3.5, 1, 3000) == -3000
    assert f(float("nan"), 1, 3000) == 0      # VCVT: NaN -> 0
    assert f(40.0, 1, 30000) == -25536        # 40000 keeps its low 16 bits (int16 narrowing)
    assert f(-32.768, -1, 30000) == -30000    # -32768 * -1 = 32768 -> -32768 -> clamp
    assert f(1e20, 1, 3000) == -1             # INT32_MAX low 16 bits = 0xFFFF


def test_can_tx_packing(orc):
    out = orc.can_tx(np.array([[0x0123, -2, 3000, -3000]], np.int16))
    assert out[0].tolist() == [0x01, 0x23, 0xFF, 0xFE, 0x0B, 0xB8, 0xF4, 0x48]


def test_f2i32_arm(orc):
    assert orc.f2i32_arm(1.9) == 1
    assert orc.f2i32_arm(-1.9) == -1
    assert orc.f2i32_arm(float("nan")) == 0
    assert orc.f2i32_arm(3e9) == 2**31 - 1
    assert orc.f2i32_arm(-3e9) == -(2**31)


def test_vehicle_info_known_answers(orc):
    d = np.arange(32, dtype=np.float32).reshape(16, 2) / 8
    rec = orc.vehicle_info([1.2345, -0.0019], [-2.5, 3.0], [0.5, -3.1], [123.9, -45.5],
                           [-0.9, 7.2], [0.25, -0.5], d, [0, 1],
                           floor=np.array([[1, 0, 1, 0, 1, 0, 1, 0], [0] * 8], np.uint8),
                           cam_pitch=12.5, fault=7)
    assert rec.itemsize == 84
    assert rec["pos_x"].tolist() == [1234, -1]        # (int32)(1.2345f*1000.0f) = 1234
    assert rec["pos_y"].tolist() == [-2500, 3000]
    assert rec["vel_x"].tolist() == [123, -45]
    assert rec["vel_y"].tolist() == [0, 7]
    assert rec["imu_fault"].tolist() == [0, 0xFF]
    np.testing.assert_array_equal(rec["imu_q"][0], d[12:16, 0])
    np.testing.assert_array_equal(rec["imu_g"][0], d[3:6, 0])
    np.testing.assert_array_equal(rec["imu_a"][0], d[0:3, 0])
    assert not rec["imu_q"][1].any() and not rec["imu_g"][1].any()
    assert rec["floor"][0].tolist() == [1, 0, 1, 0, 1, 0, 1, 0]
    assert rec["cam_pitch"].tolist() == [12.5, 12.5] and rec["fault"].tolist() == [7, 7]


def test_ctrl_step_power_cycle(orc):
    b = orc.CtrlBatch(4)
    b.set_power([1, 1, 1, 0])
    vel = np.array([[200, -200, 0, 200], [0, 100, 0, 0], [0, 0, 1.0, 0]], np.float32)
    acl = np.array([[1000] * 4, [1000] * 4, [30] * 4], np.float32)
    jrk = np.array([[10000] * 4, [10000] * 4, [300] * 4], np.float32)
    b.set_target_vel(vel, acl, jrk)
    rpm = np.zeros((4, 4), np.int16)
    for _ in range(500):
        b.step(rpm)
    vt = b.vel_tgt()
    np.testing.assert_array_equal(vt[:, 0], [200, 0, 0])
    np.testing.assert_array_equal(vt[:, 1], [-200, 100, 0])
    assert vt[2, 2] == np.float32(1.0)
    # wheels at rest, targets nonzero: every powered controller saturates its FF/I terms
    cur = b.curr()
    assert (cur[3] == 0).all()          # power off: zero current, interpolators reset
    assert np.abs(cur[:3]).max() > 0 and np.abs(cur).max() <= 3000
    # reversed motors (BR, FR) flip the sign of the raw current
    assert np.sign(cur[0, 0]) == -np.sign(cur[0, 3]) or cur[0, 0] == 0
