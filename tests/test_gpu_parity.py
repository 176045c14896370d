"""GPU parity: the HIP path (through the C ABI) against the oracle.

Bar: bit-exact for every integer / byte path and for every fp32/fp64 path whose
trig policy is the table (both sides evaluate the identical IEEE operation
sequence with contraction off).  The LIBM policy compares device sinf/cosf with
glibc's, which may differ by an ulp; those runs use the north-star tolerance
(1e-5 relative per physical quantity, as in tests/test_oracle_kf_fp64.py).
"""
import numpy as np
import pytest

import fmskf
from fmskf import Engine
from fmskf.synth import Trajectory, wt901_frame
from conftest import iter_golden_streams

pytestmark = pytest.mark.gpu

TABLE, LIBM = fmskf.TRIG_TABLE512, fmskf.TRIG_LIBM


def bits_equal(a, b, what=""):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    assert a.shape == b.shape, what
    if a.dtype.kind == "f":
        ia = a.view(np.uint32 if a.dtype == np.float32 else np.uint64)
        ib = b.astype(a.dtype).view(ia.dtype)
        bad = np.nonzero(ia != ib)
        assert bad[0].size == 0, f"{what}: {bad[0].size} mismatches, first at {tuple(x[0] for x in bad)}: {a[bad][0]!r} vs {b[bad][0]!r}"
    else:
        np.testing.assert_array_equal(a, b, err_msg=what)


def rel_close(a, b, tol=1e-5, what=""):
    scale = max(np.abs(b).max(), 1e-3)
    err = np.abs(a.astype(np.float64) - b.astype(np.float64)).max() / scale
    assert err <= tol, f"{what}: {err}"


# ----------------------------------------------------------------------------- trig
def test_trig_table_bitexact(orc):
    x = np.linspace(-50, 50, 100003).astype(np.float32)
    x = np.concatenate([x, np.float32([0, -0.0, 2 * np.pi, -2 * np.pi, 1e-9, -1e-9, 6.2831855])])
    with Engine("kf6", 8, trig=TABLE) as e:
        s, c = e.eval_trig(x)
    so, co = orc.eval_trig(x, orc.TRIG_TABLE512)
    bits_equal(s, so, "sin")
    bits_equal(c, co, "cos")


# headings where the reference's float -> int casts leave the int32 range (past 2^31 turns),
# infinities, NaN, denormals and the 2^24 float-integer edge
EXTREME_RAD = np.float32([1.3493e10, 1.35e10, -1.35e10, 1.5e10, -1.5e10, 4e12, -4e12, 1e20, -1e20,
                          3.4e38, -3.4e38, np.inf, -np.inf, np.nan, 1e-40, -1e-40, 16777216.0,
                          -16777217.0, 2147483520.0, -2147483648.0, 6.2831855, -6.2831855])


def nan_aware_equal(a, b, what=""):
    """bitwise equal, except that NaN only has to meet NaN (x86 and gfx950 differ in the
    default NaN's sign bit; the firmware's value is NaN either way)"""
    a, b = np.asarray(a), np.asarray(b)
    na, nb = np.isnan(a), np.isnan(b)
    assert np.array_equal(na, nb), f"{what}: NaN positions differ"
    bits_equal(np.where(na, 0, a).astype(a.dtype), np.where(nb, 0, b).astype(a.dtype), what)


def test_trig_table_extremes_bitexact(orc):
    """The CMSIS table lookup with the M7's saturating VCVT (the floor of a heading past 2^31
    turns, the uint16_t table index): every input gives the oracle's answer, and the index stays
    inside the 513-entry table."""
    x = np.concatenate([EXTREME_RAD, -EXTREME_RAD * np.float32(0.5)])
    with Engine("kf6", 8, trig=TABLE) as e:
        s, c = e.eval_trig(x)
    so, co = orc.eval_trig(x, orc.TRIG_TABLE512)
    nan_aware_equal(s, so, "sin")
    nan_aware_equal(c, co, "cos")


def test_rs_tick_extreme_headings(orc):
    """RS tick (VD_vehicle_controller.cpp:36-51) fed IMU yaws whose radians leave the int32 turn
    range in normalize_rad_0to2pi (util_mymath.hpp:18-25), inf and NaN: pose, velocity and
    encoder state as the oracle gives them."""
    with np.errstate(over="ignore"):  # rad -> deg of the largest ones overflows to inf, as wanted
        yaw_deg = np.concatenate([EXTREME_RAD, EXTREME_RAD * np.float32(57.29578)])
    n, T = yaw_deg.size, 3
    tr = Trajectory(n, T, seed=41)
    _, sums, rpm = tr.rs_inputs()
    yaw = np.repeat(yaw_deg[None], T, 0)
    with Engine("rs", n, trig=TABLE) as e:
        for t in range(T):
            e.tick(yaw_deg=yaw[t], angle_sum=sums[t], rpm=rpm[t])
        pose = e.get_pose()
        prev = e.get_prev_sum()
    pos, velo, prevo = _rs_oracle(orc, n, yaw, sums, rpm, TABLE, T)
    nan_aware_equal(np.stack(pose), pos, "pose")
    bits_equal(prev, prevo, "prev")


def test_kf6_tick_extreme_yaw(orc):
    """KF6 correct + predict with IMU yaws far outside any heading (the trig of the state's
    heading then takes the saturating table path), inf and NaN: x and P as the oracle gives
    them, NaN meeting NaN."""
    with np.errstate(over="ignore"):  # rad -> deg of the largest ones overflows to inf, as wanted
        yaw_deg = np.concatenate([EXTREME_RAD, EXTREME_RAD * np.float32(57.29578)])
    n, T = yaw_deg.size, 3
    rng = np.random.default_rng(8)
    yaw = np.repeat(yaw_deg[None], T, 0)
    gz = rng.uniform(-300, 300, (T, n)).astype(np.float32)
    rpm = rng.integers(-9000, 9000, (T, n, 4)).astype(np.int16)
    with Engine("kf6", n, trig=TABLE) as e:
        for t in range(T):
            e.tick(yaw_deg=yaw[t], gyro_z_dps=gz[t], rpm=rpm[t])
        x, P = e.get_state()
    xo, Po = _kf6_oracle(orc, n, yaw, gz, rpm, None, orc.TRIG_TABLE512, T)
    nan_aware_equal(x, xo, "x")
    nan_aware_equal(P, Po, "P")


def test_trig_libm_close(orc):
    x = np.linspace(-10, 10, 10001).astype(np.float32)
    with Engine("kf6", 8, trig=LIBM) as e:
        s, c = e.eval_trig(x)
    assert np.abs(s - np.sin(x.astype(np.float64))).max() < 5e-7
    assert np.abs(c - np.cos(x.astype(np.float64))).max() < 5e-7


# ----------------------------------------------------------------------------- KF6
def _kf6_setup(n, T, seed):
    tr = Trajectory(n, T, seed=seed)
    yaw, gz, rpm = tr.kf6_inputs()
    rng = np.random.default_rng(seed)
    valid = (rng.random((T, n)) > 0.1).astype(np.uint8)
    return tr, yaw, gz, rpm, valid


def _kf6_oracle(orc, n, yaw, gz, rpm, valid, trig, ticks):
    cfg = fmskf.default_config("kf6", n)
    prm = orc.kf6_params(cfg.dt, np.array(cfg.q[:21]), np.array(cfg.r[:10]), trig)
    x = np.zeros((6, n), np.float32)
    P = np.repeat(np.float32(np.array(cfg.p0[:21]))[:, None], n, 1).copy()
    for t in range(ticks):
        orc.kf6_tick(x, P, yaw[t], gz[t], rpm[t], None if valid is None else valid[t], prm,
                     nthreads=0)
    return x, P


@pytest.mark.parametrize("n", [1, 1037])
def test_kf6_tick_bitexact(orc, n):
    T = 40
    _, yaw, gz, rpm, valid = _kf6_setup(n, T, 21 + n)
    with Engine("kf6", n, trig=TABLE) as e:
        for t in range(T):
            e.tick(yaw_deg=yaw[t], gyro_z_dps=gz[t], rpm=rpm[t], valid=valid[t])
        x, P = e.get_state()
        assert e.get_counters()[0] == 0
    xo, Po = _kf6_oracle(orc, n, yaw, gz, rpm, valid, orc.TRIG_TABLE512, T)
    bits_equal(x, xo, "x")
    bits_equal(P, Po, "P")


def test_kf6_libm_within_tolerance(orc):
    n, T = 777, 60
    _, yaw, gz, rpm, valid = _kf6_setup(n, T, 5)
    with Engine("kf6", n, trig=LIBM) as e:
        for t in range(T):
            e.tick(yaw_deg=yaw[t], gyro_z_dps=gz[t], rpm=rpm[t], valid=valid[t])
        x, P = e.get_state()
    xo, Po = _kf6_oracle(orc, n, yaw, gz, rpm, valid, orc.TRIG_LIBM, T)
    for grp in [(0, 1), (2,), (3, 4), (5,)]:
        rel_close(x[list(grp)], xo[list(grp)], 1e-5, f"x{grp}")
    rel_close(P, Po, 1e-5, "P")


def test_kf6_split_equals_fused_and_many():
    n, T = 1000, 12
    _, yaw, gz, rpm, valid = _kf6_setup(n, T, 8)
    with Engine("kf6", n) as a, Engine("kf6", n) as b, Engine("kf6", n) as c:
        for t in range(T):
            a.tick(yaw_deg=yaw[t], gyro_z_dps=gz[t], rpm=rpm[t], valid=valid[t])
            b.correct(yaw_deg=yaw[t], gyro_z_dps=gz[t], rpm=rpm[t], valid=valid[t])
            b.predict()
        c.tick_many(T, yaw_deg=yaw, gyro_z_dps=gz, rpm=rpm, valid=valid)
        xa, Pa = a.get_state()
        xb, Pb = b.get_state()
        xc, Pc = c.get_state()
    bits_equal(xa, xb, "split x")
    bits_equal(Pa, Pb, "split P")
    bits_equal(xa, xc, "many x")
    bits_equal(Pa, Pc, "many P")


@pytest.mark.parametrize("n,trig", [(1, TABLE), (3001, TABLE), (777, LIBM)])
def test_kf6_records_bitexact(orc, n, trig):
    """fmskf_kf6_record inputs (one 16-byte load per lane) against the oracle, against the
    plane inputs, with a validity mask; tick_many over [T][N] records; host and device."""
    import torch
    T = 30
    _, yaw, gz, rpm, valid = _kf6_setup(n, T, 77 + n)
    rec = fmskf.kf6_records(yaw, gz, rpm)
    assert rec.shape == (T, n) and rec.dtype.itemsize == 16
    drec = fmskf.kf6_records(*(torch.from_numpy(v).cuda() for v in (yaw, gz, rpm)))
    assert torch.equal(drec.cpu().view(torch.uint8).reshape(T, n, 16),
                       torch.from_numpy(rec.view(np.uint8).reshape(T, n, 16)))
    with Engine("kf6", n, trig=trig) as a, Engine("kf6", n, trig=trig) as b, \
            Engine("kf6", n, trig=trig) as c, Engine("kf6", n, trig=trig) as d:
        for t in range(T):
            a.tick(kf6_rec=rec[t], valid=valid[t])
            b.tick(yaw_deg=yaw[t], gyro_z_dps=gz[t], rpm=rpm[t], valid=valid[t])
            d.tick(kf6_rec=drec[t], valid=torch.from_numpy(valid[t]).cuda())
        c.tick_many(T, kf6_rec=rec, valid=valid)
        torch.cuda.synchronize()
        (xa, Pa), (xb, Pb), (xc, Pc), (xd, Pd) = (e.get_state() for e in (a, b, c, d))
    for x, P, what in ((xb, Pb, "planes"), (xc, Pc, "tick_many"), (xd, Pd, "device")):
        bits_equal(xa, x, "x vs " + what)
        bits_equal(Pa, P, "P vs " + what)
    if trig == TABLE:
        xo, Po = _kf6_oracle(orc, n, yaw, gz, rpm, valid, orc.TRIG_TABLE512, T)
        bits_equal(xa, xo, "x vs oracle")
        bits_equal(Pa, Po, "P vs oracle")


def test_kf6_records_rejected_where_ambiguous():
    n = 64
    rec = fmskf.kf6_records(np.zeros(n, np.float32), np.zeros(n, np.float32), np.zeros((n, 4), np.int16))
    with Engine("kf6", n) as e:
        with pytest.raises(fmskf.FmskfError):
            e.tick(kf6_rec=rec, yaw_deg=np.zeros(n, np.float32))
        with pytest.raises(ValueError):
            e.tick(kf6_rec=rec[: n - 1])
    with Engine("rs", n) as e:
        with pytest.raises(fmskf.FmskfError):
            e.tick(kf6_rec=rec)


def test_kf6_device_inputs_torch():
    import torch
    n, T = 4099, 5
    _, yaw, gz, rpm, valid = _kf6_setup(n, T, 9)
    with Engine("kf6", n) as a, Engine("kf6", n) as b:
        stream = torch.cuda.current_stream()
        b.set_stream(stream)
        dy, dg, dr = (torch.from_numpy(v).cuda() for v in (yaw, gz, rpm))
        for t in range(T):
            a.tick(yaw_deg=yaw[t], gyro_z_dps=gz[t], rpm=rpm[t])
            b.tick(yaw_deg=dy[t], gyro_z_dps=dg[t], rpm=dr[t])
        torch.cuda.synchronize()
        bits_equal(a.get_state()[0], b.get_state()[0], "x")
        bits_equal(a.get_state()[1], b.get_state()[1], "P")


def test_kf6_large_n_sampled_bitexact(orc):
    """N = 2^20 (the bench config): fused multi-tick launch on device inputs; a sample
    of 2048 instances is recomputed by the oracle bit for bit, the rest must be finite
    with a positive covariance diagonal."""
    import torch
    n, T = 1 << 20, 8
    tr = Trajectory(n, T, seed=77)
    yaw, gz, rpm = tr.kf6_inputs()
    with Engine("kf6", n) as e:
        e.tick_many(T, yaw_deg=torch.from_numpy(yaw).cuda(), gyro_z_dps=torch.from_numpy(gz).cuda(),
                    rpm=torch.from_numpy(rpm).cuda())
        x, P = e.get_state()
        assert e.get_counters()[0] == 0
    assert np.isfinite(x).all() and np.isfinite(P).all()
    diag = [0, 2, 5, 9, 14, 20]
    assert (P[diag] > 0).all()
    idx = np.sort(np.random.default_rng(0).choice(n, 2048, replace=False))
    xo, Po = _kf6_oracle(orc, idx.size, np.ascontiguousarray(yaw[:, idx]),
                         np.ascontiguousarray(gz[:, idx]), np.ascontiguousarray(rpm[:, idx]),
                         None, orc.TRIG_TABLE512, T)
    bits_equal(x[:, idx], xo, "x sample")
    bits_equal(P[:, idx], Po, "P sample")


def test_nan_guard_counts_bad_instances():
    n = 512
    _, yaw, gz, rpm, _ = _kf6_setup(n, 1, 3)
    yaw = yaw[0].copy()
    yaw[[5, 100, 300]] = np.nan
    with Engine("kf6", n) as e:
        e.tick(yaw_deg=yaw, gyro_z_dps=gz[0], rpm=rpm[0])
        assert e.get_counters()[0] == 3


# ----------------------------------------------------------------------------- RS
def _rs_oracle(orc, n, yaw, sums, rpm, trig, T):
    pos = np.zeros((3, n), np.float32)
    vel = np.zeros((3, n), np.float32)
    prev = np.zeros((4, n), np.int64)
    for t in range(T):
        orc.rs_tick(pos, vel, prev, yaw[t], np.ascontiguousarray(sums[t]), rpm[t], trig)
    return pos, vel, prev


@pytest.mark.parametrize("trig", [TABLE, LIBM])
def test_rs_tick_bitexact(orc, trig):
    n, T = 2053, 50
    tr = Trajectory(n, T, seed=31)
    yaw, sums, rpm = tr.rs_inputs()
    with Engine("rs", n, trig=trig) as e:
        for t in range(T):
            e.tick(yaw_deg=yaw[t], angle_sum=sums[t], rpm=rpm[t])
        x, _ = e.get_state()
        prev = e.get_prev_sum()
        pose = e.get_pose()
        vel = e.get_vel()
    pos, velo, prevo = _rs_oracle(orc, n, yaw, sums, rpm, trig, T)
    bits_equal(prev, prevo, "prev")
    bits_equal(x[3:6], velo, "vel")
    bits_equal(vel, velo, "vel readout")
    bits_equal(x[2], pos[2], "theta")  # the IMU overwrite involves no trig
    if trig == TABLE:
        bits_equal(x[:3], pos, "pos")
        bits_equal(pose, pos, "pose readout")
    else:  # device sinf/cosf vs glibc: ulp-level differences only
        rel_close(x[:2], pos[:2], 1e-5, "pos")
        rel_close(pose[:2], pos[:2], 1e-5, "pose readout")


def test_rs_many_and_split():
    n, T = 600, 16
    tr = Trajectory(n, T, seed=32)
    yaw, sums, rpm = tr.rs_inputs()
    with Engine("rs", n) as a, Engine("rs", n) as b, Engine("rs", n) as c:
        for t in range(T):
            a.tick(yaw_deg=yaw[t], angle_sum=sums[t], rpm=rpm[t])
            b.correct(yaw_deg=yaw[t])
            b.predict(angle_sum=sums[t], rpm=rpm[t])
        c.tick_many(T, yaw_deg=yaw, angle_sum=sums, rpm=rpm)
        for o in (b, c):
            bits_equal(a.get_state()[0], o.get_state()[0], "x")
            bits_equal(a.get_prev_sum(), o.get_prev_sum(), "prev")


# ----------------------------------------------------------------------------- EKF9 / KF12D
# EKF9 R cases: the default (diagonal: the sequential scalar update), and correlated wheel
# velocities and accelerations (the joint LDL^T update)
EKF9_R_CASES = {"diagonal": {}, "correlated": {(5, 4): 1e-4, (3, 2): 0.05, (1, 0): 1e-5}}


def _ekf9_r(cfg, terms):
    r = np.array(cfg.r[:21])
    for (i, j), v in terms.items():
        r[i * (i + 1) // 2 + j] = v
    return r


@pytest.mark.parametrize("case", list(EKF9_R_CASES))
def test_ekf9_bitexact(orc, case):
    n, T = 1500, 30
    tr = Trajectory(n, T, seed=41)
    raw = tr.ekf9_raw()
    cfg = fmskf.default_config("ekf9", n)
    r = _ekf9_r(cfg, EKF9_R_CASES[case])
    with Engine("ekf9", n, trig=TABLE, r=r) as e:
        for t in range(T):
            e.tick(raw=raw[t])
        x, P = e.get_state()
        rec = e.tick_ensemble(raw=raw[0])  # the fused record kernel takes the same update path
        x2, P2 = e.get_state()
    prm = orc.ekf9_params(cfg.dt, np.array(cfg.q[:45]), r, orc.TRIG_TABLE512)
    xo = np.zeros((10, n), np.float32)  # row 9: the heading's low part
    Po = np.repeat(np.float32(np.array(cfg.p0[:45]))[:, None], n, 1).copy()
    for t in range(T):
        orc.ekf9_tick(xo, Po, raw[t], None, prm, nthreads=0)
    bits_equal(x, xo[:9], "x")
    bits_equal(P, Po, "P")
    orc.ekf9_tick(xo, Po, raw[0], None, prm, nthreads=0)
    bits_equal(x2, xo[:9], "x (tick_ensemble)")
    bits_equal(P2, Po, "P (tick_ensemble)")
    assert rec[0] == n


@pytest.mark.parametrize("n,T,case", [(1000, 9, "diagonal"), (257, 4, "diagonal"), (1000, 5, "correlated")])
def test_ekf9_many_split_mask_bitexact(orc, n, T, case):
    """EKF9 over the tiled state: T ticks in one tick_many launch (the ping-pong loop kernel,
    odd T exercising its tail), per-tick ticks and correct-then-predict calls, all with a
    validity mask at ragged N, bit-identical to each other and to the oracle."""
    tr = Trajectory(n, T, seed=43)
    raw = tr.ekf9_raw()
    rng = np.random.default_rng(n)
    valid = (rng.random((T, n)) > 0.2).astype(np.uint8)
    cfg = fmskf.default_config("ekf9", n)
    r = _ekf9_r(cfg, EKF9_R_CASES[case])
    with Engine("ekf9", n, r=r) as a, Engine("ekf9", n, r=r) as b, Engine("ekf9", n, r=r) as c:
        a.tick_many(T, raw=raw, valid=valid)
        for t in range(T):
            b.tick(raw=raw[t], valid=valid[t])
            c.correct(raw=raw[t], valid=valid[t])
            c.predict()
        (xa, Pa), (xb, Pb), (xc, Pc) = (e.get_state() for e in (a, b, c))
    prm = orc.ekf9_params(cfg.dt, np.array(cfg.q[:45]), r, orc.TRIG_TABLE512)
    xo = np.zeros((10, n), np.float32)  # row 9: the heading's low part
    Po = np.repeat(np.float32(np.array(cfg.p0[:45]))[:, None], n, 1).copy()
    for t in range(T):
        orc.ekf9_tick(xo, Po, raw[t], valid[t], prm, nthreads=0)
    for x, P, what in ((xa, Pa, "tick_many"), (xb, Pb, "tick"), (xc, Pc, "split")):
        bits_equal(x, xo[:9], "x " + what)
        bits_equal(P, Po, "P " + what)


def test_ekf9_libm_within_tolerance(orc):
    n, T = 600, 30
    tr = Trajectory(n, T, seed=44)
    raw = tr.ekf9_raw()
    cfg = fmskf.default_config("ekf9", n)
    with Engine("ekf9", n, trig=LIBM) as e:
        for t in range(T):
            e.tick(raw=raw[t])
        x, P = e.get_state()
    prm = orc.ekf9_params(cfg.dt, np.array(cfg.q[:45]), np.array(cfg.r[:21]), orc.TRIG_LIBM)
    xo = np.zeros((10, n), np.float32)
    Po = np.repeat(np.float32(np.array(cfg.p0[:45]))[:, None], n, 1).copy()
    for t in range(T):
        orc.ekf9_tick(xo, Po, raw[t], None, prm, nthreads=0)
    # device sinf/cosf vs glibc differ by ulps; the north-star tolerance 1e-5 relative
    for grp in [(0, 1), (2,), (3, 4), (5, 6), (7, 8)]:
        rel_close(x[list(grp)], xo[list(grp)], 1e-5, f"x{grp}")
    rel_close(P, Po, 1e-5, "P")


def test_kf12d_many_equals_ticks():
    """KF12D T ticks in one launch (state held in registers across ticks) == T single ticks,
    with a validity mask, over the tiled state at ragged N."""
    n, T = 513, 6
    tr = Trajectory(n, T, seed=52)
    z = np.ascontiguousarray(tr.kf12d_z())
    valid = (np.random.default_rng(5).random((T, n)) > 0.25).astype(np.uint8)
    with Engine("kf12d", n) as a, Engine("kf12d", n) as b:
        a.tick_many(T, z=z, valid=valid)
        for t in range(T):
            b.tick(z=z[t], valid=valid[t])
        (xa, Pa), (xb, Pb) = a.get_state(), b.get_state()
    bits_equal(xa, xb, "x")
    bits_equal(Pa, Pb, "P")


KF12D_R_CASES = {
    # R positive definite -> decorrelated scalar-sequential update (canonical KF12D order)
    "blockdiag_R_decorrelated": {},
    "cross_R_decorrelated": {(4, 0): 1e-6, (7, 3): -2e-6, (5, 1): 3e-7},
    # R not positive definite (S = H P H^T + R still invertible) -> LDL^T fallbacks
    "cross_R_indefinite_joint": {(4, 0): 1e-5, (7, 3): -2e-5},
    "blockdiag_R_semidefinite_groups": {(7, 7): 0.0},
}


@pytest.mark.parametrize("case", list(KF12D_R_CASES))
def test_kf12d_vs_oracle(orc, case):
    n, T = 700, 20
    tr = Trajectory(n, T, seed=51)
    z = tr.kf12d_z()
    cfg = fmskf.default_config("kf12d", n)
    r = np.array(cfg.r[:36])
    for (i, j), v in KF12D_R_CASES[case].items():
        r[i * (i + 1) // 2 + j] = v
    assert bool(orc.kf12d_cinv(r)[0]) == ("decorrelated" in case)
    with Engine("kf12d", n, r=r) as e:
        for t in range(T):
            e.tick(z=z[t])
        x, P = e.get_state()
    prm = orc.kf12d_params(cfg.dt, np.array(cfg.q[:78]), r)
    xo = np.zeros((12, n))
    Po = np.repeat(np.array(cfg.p0[:78])[:, None], n, 1).copy()
    for t in range(T):
        orc.kf12d_tick(xo, Po, np.ascontiguousarray(z[t]), None, prm, nthreads=0)
    # fp64: tolerance 1e-12 relative (config 5); the device follows the oracle's operation
    # order, so in practice the results are bit exact
    for k in range(12):
        rel_close(x[k], xo[k], 1e-12, f"x{k}")
    rel_close(P, Po, 1e-12, "P")
    assert np.array_equal(x.view(np.uint64), xo.view(np.uint64))
    assert np.array_equal(P.view(np.uint64), Po.view(np.uint64))


# ----------------------------------------------------------------------------- WT901 ingest
def test_wt901_ingest_matches_reference_golden(orc, golden_wt901):
    streams = list(iter_golden_streams(golden_wt901))
    for rri in sorted({s[0] for s in streams}):
        group = [s for s in streams if s[0] == rri]
        n = len(group)
        maxp = max(len(s[2]) for s in group)
        stride = max(len(p) for s in group for p in s[2]) + 16
        orcs = [orc.Wt901(rri) for _ in group]
        with Engine("rs", n, imu_read_reg=rri) as e:
            for k in range(maxp):
                buf = np.zeros((n, stride), np.uint8)
                lens = np.zeros(n, np.uint32)
                for i, s in enumerate(group):
                    if k < len(s[2]):
                        b = np.frombuffer(s[2][k], np.uint8)
                        buf[i, :b.size] = b
                        lens[i] = b.size
                    orcs[i].update(buf[i, :lens[i]])
                e.ingest_wt901(buf, lens)
                regs, pending = e.get_imu_regs()
                data, err = e.get_imu()
                for i, s in enumerate(group):
                    kk = min(k, len(s[2]) - 1)
                    np.testing.assert_array_equal(regs[:, i], s[3][kk], err_msg=f"{s[1]} poll {k}")
                    assert err[i] == orcs[i].is_error
                    assert pending[i] == len(orcs[i].parser)
                    bits_equal(data[:, i], orcs[i].data, f"data {s[1]} poll {k}")


@pytest.mark.parametrize("stride", [48, 64, 96])
def test_wt901_ingest_random_streams(orc, stride):
    """Mixed clean / noisy / damaged / short-frame polls.  Strides 48 and 64 take the
    vector-row kernel (and its whole-frame fast path for clean polls with an empty window),
    96 the byte-load kernel."""
    n, polls = 3000, 6
    rng = np.random.default_rng(99 + stride)
    orcs = [orc.Wt901(0x51) for _ in range(n)]
    with Engine("kf6", n) as e:
        for k in range(polls):
            buf = np.zeros((n, stride), np.uint8)
            lens = rng.integers(0, stride + 1, n).astype(np.uint32)
            for i in range(n):
                kind = rng.integers(0, 4)
                if kind == 0:  # clean poll
                    b = b"".join(wt901_frame(t, rng.integers(0, 65536, 4)) for t in (0x51, 0x52, 0x53, 0x59))
                    b = np.frombuffer(b, np.uint8)
                elif kind == 3:  # 0-5 whole frames of any type, or a torn tail
                    ts = rng.choice([0x50, 0x51, 0x52, 0x53, 0x54, 0x59, 0x5A, 0x5F, 0x61], int(rng.integers(0, 6)))
                    b = b"".join(wt901_frame(int(t), rng.integers(0, 65536, 4)) for t in ts)
                    if rng.random() < 0.3:
                        b = b[:int(rng.integers(0, len(b) + 1))]
                    b = np.frombuffer(b, np.uint8)
                elif kind == 1:  # noisy
                    b = rng.integers(0, 256, int(lens[i]), dtype=np.uint8)
                    b[rng.random(b.size) < 0.2] = 0x55
                else:  # frames with errors
                    fr = [bytearray(wt901_frame(int(rng.choice([0x51, 0x59, 0x5F, 0x50])), rng.integers(0, 65536, 4))) for _ in range(6)]
                    for f in fr:
                        if rng.random() < 0.3:
                            f[int(rng.integers(0, 11))] ^= 0xA5
                    b = np.frombuffer(bytes(b"".join(fr)), np.uint8)
                b = b[:stride]
                lens[i] = b.size
                buf[i, :b.size] = b
                orcs[i].update(b, latch_qinit=(k == 0))
            e.ingest_wt901(buf, lens, latch_qinit=(k == 0))
        regs, pending = e.get_imu_regs()
        data, err = e.get_imu()
    for i in range(0, n, 7):
        np.testing.assert_array_equal(regs[:, i], orcs[i].regs)
        assert pending[i] == len(orcs[i].parser)
        assert err[i] == orcs[i].is_error
        bits_equal(data[:, i], orcs[i].data, f"data {i}")


@pytest.mark.parametrize("stride", [48, 96])
def test_wt901_data_page_across_latches(orc, stride):
    """The Data page is formed at readout from the last successful poll's snapshot row (round
    5): after EVERY poll it equals the oracle's eagerly written page bit for bit -- before the
    first successful poll (all zeros), on the poll that latches q_init (its page uses the OLD
    q_init, kept as qprev), on the polls after it, across a second latch, and for robots whose
    poll failed (the page of their last success stays).  VehicleInfo reads the same page.  The
    register file too, on every third poll: the standard poll writes eleven registers into the
    snapshot row only (round 6), and a failed poll, a 0x5F register reply (Q0-Q3) or another
    frame mix after it must see them (wit_c_sdk.c:90-130).  And the tick's yaw: an RS handle fed
    the same polls takes Data.angle[2] from the Yaw / GZ words (round 6) in its correct step
    (theta = deg2rad(yaw), VD_task_main.cpp:368), so theta follows the page, not the register."""
    n, polls = 1537, 9
    rng = np.random.default_rng(41 + stride)
    orcs = [orc.Wt901(0x51) for _ in range(n)]
    latch = {1, 5}
    deg2rad = np.float32(np.float32(3.14159265358979) / np.float32(180.0))  # util_mymath.hpp:14
    with Engine("kf6", n) as e, Engine("rs", n) as rs:
        for k in range(polls):
            buf = np.zeros((n, stride), np.uint8)
            lens = np.zeros(n, np.uint32)
            for i in range(n):
                r = rng.random()
                if k == 0 and i % 3:  # most robots have no successful poll before the first latch
                    ts = (0x51, 0x52, 0x53)
                elif r < 0.7:  # the standard poll (fast path)
                    ts = (0x51, 0x52, 0x53, 0x59)
                elif r < 0.80:  # no quaternion frame: the poll fails, the page stays
                    ts = (0x51, 0x53)
                elif r < 0.85:  # a failed poll that writes the magnetometer: the page keeps the
                    ts = (0x54, 0x51)  # earlier HX-HZ (round 6: F_MAGDET, imu_mag)
                elif r < 0.92:  # a register-read reply (0x5F at imu_read_reg 0x51: Q0-Q3) alone
                    ts = (0x5F,)
                else:  # a quaternion frame among others, through the parser
                    ts = (0x54, 0x59, 0x52)
                b = np.frombuffer(b"".join(wt901_frame(t, rng.integers(0, 65536, 4)) for t in ts), np.uint8)
                buf[i, :b.size] = b
                lens[i] = b.size
                orcs[i].update(b, latch_qinit=(k in latch))
            e.ingest_wt901(buf, lens, latch_qinit=(k in latch))
            rs.ingest_wt901(buf, lens, latch_qinit=(k in latch))
            rs.correct()  # NULL yaw plane: the ingested Data.angle[2]
            th = rs.get_pose()[2]
            data, err = e.get_imu()
            for i in range(n):
                assert err[i] == orcs[i].is_error
                bits_equal(data[:, i], orcs[i].data, f"data {i} poll {k}")
            yaw = np.array([orcs[i].data[11] for i in range(n)], np.float32)
            bits_equal(th, yaw * deg2rad, f"theta poll {k}")
            if k % 3 == 1:  # the register file (round 6: the standard poll keeps eleven of its
                # registers in the snapshot row only; the readout writes them back), on some polls,
                # so that later polls also start from row-resident registers
                regs, _ = e.get_imu_regs()
                for i in range(0, n, 3):
                    np.testing.assert_array_equal(regs[:, i], orcs[i].regs, err_msg=f"regs {i} poll {k}")
        vi = e.export_vehicle_info()
    for i in range(0, n, 5):
        d = orcs[i].data
        if orcs[i].is_error:
            assert vi["imu_fault"][i] == 0xFF and not np.any(vi["imu_q"][i])
        else:
            bits_equal(vi["imu_q"][i], d[12:16], f"vi q {i}")
            bits_equal(vi["imu_g"][i], d[3:6], f"vi g {i}")
            bits_equal(vi["imu_a"][i], d[0:3], f"vi a {i}")


# ----------------------------------------------------------------------------- CAN ingest
@pytest.mark.parametrize("masked", [True, False, "mixed"])
def test_can_ingest_bitexact(orc, masked, n=1001):
    """masked: every tick with a `present` mask (k_can, wheel per lane); False: every wheel
    present (k_can4, robot per lane); "mixed": one masked tick in three, so the robots' Status
    ring heads fall out of step and k_can4 blocks meet robots whose wheels sit in other slots
    of the angle ring than the block's first robot."""
    T = 25
    rng = np.random.default_rng(7)
    dirs = [1, 1, -1, -1]
    motors = [[orc.M2006(d) for d in dirs] for _ in range(n)]
    with Engine("rs", n) as e:
        for t in range(T):
            frames = rng.integers(0, 256, (n, 4, 8), dtype=np.uint8)
            frames[:, :, 0] &= 0x1F  # mostly in-range 13-bit angles
            frames[rng.random((n, 4)) < 0.05, 0] |= 0x80  # some out-of-range / negative
            stamps = rng.integers(0, 0x8000, (n, 4)).astype(np.int16)
            stamps[rng.random((n, 4)) < 0.05] = 1234  # equal stamps -> usec_dlt == 0
            mask_now = masked is True or (masked == "mixed" and t % 3 == 1)
            present = rng.integers(0, 16, n).astype(np.uint8) if mask_now else np.full(n, 15, np.uint8)
            e.ingest_can(frames, stamps, present if mask_now else None)
            for i in range(n):
                for w in range(4):
                    if (present[i] >> w) & 1:
                        motors[i][w].rx(frames[i, w], int(stamps[i, w]))
        m = e.get_motors()
        st = e.get_motor_status()
    for i in range(n):
        for w in range(4):
            s = motors[i][w].s
            assert m["angle"][i, w] == s.angle and m["rpm"][i, w] == s.rpm
            assert m["curr"][i, w] == s.curr and m["angle_sum"][w, i] == s.angle_sum
            bits_equal(m["speed_radps"][w, i:i + 1], np.float32([s.speed_radps]), "speed")
            # MOTOR_IF_M2006::get_status_latest: the full Status (VD_motor_if_m2006.hpp:23-30),
            # flt_dltOutAngle_rad formed at readout from the last two angles
            assert st["microsec_id"][i, w] == s.micro and st["angle"][i, w] == s.angle
            assert st["rpm"][i, w] == s.rpm and st["curr"][i, w] == s.curr
            bits_equal(st["dlt_out_angle_rad"][i, w:w + 1], np.float32([s.dlt_out_angle_rad]), "dlt")
            bits_equal(st["speed_radps"][i, w:w + 1], np.float32([s.speed_radps]), "status speed")


def test_full_pipeline_rs_device_resident(orc):
    """CAN ingest every tick + IMU ingest every 10 ticks + tick with NULL planes (the
    device-resident state), against the same sequence through the oracle."""
    n, T = 257, 40
    tr = Trajectory(n, T, seed=61)
    with Engine("rs", n) as e:
        imus = [orc.Wt901(0x51) for _ in range(n)]
        mot = [[orc.M2006(d) for d in (1, 1, -1, -1)] for _ in range(n)]
        pos = np.zeros((3, n), np.float32)
        vel = np.zeros((3, n), np.float32)
        prev = np.zeros((4, n), np.int64)
        for t in range(T):
            fr, st = tr.can_frames(t)
            e.ingest_can(fr, st)
            for i in range(n):
                for w in range(4):
                    mot[i][w].rx(fr[i, w], int(st[i, w]))
            if t % 10 == 0:
                buf = np.zeros((n, 48), np.uint8)
                lens = np.zeros(n, np.uint32)
                for i in range(n):
                    b = np.frombuffer(tr.wt901_poll_bytes(t, i), np.uint8)
                    buf[i, :b.size] = b
                    lens[i] = b.size
                    imus[i].update(b, latch_qinit=(t == 0))
                e.ingest_wt901(buf, lens, latch_qinit=(t == 0))
            e.tick()
            yaw = np.array([imus[i].data[11] for i in range(n)], np.float32)
            sums = np.array([[mot[i][w].s.angle_sum for i in range(n)] for w in range(4)], np.int64)
            rpm = np.array([[mot[i][w].s.rpm for w in range(4)] for i in range(n)], np.int16)
            orc.rs_tick(pos, vel, prev, yaw, sums, rpm)
        x, _ = e.get_state()
    bits_equal(x[:3], pos, "pose")
    bits_equal(x[3:], vel, "vel")


# ----------------------------------------------------------------------------- ensemble
# 2^20 (KF6 / EKF9: one pass of 4 robots per lane over 1024 blocks) and 3 * 2^20 + 5 (past the
# 2048-block cap: grid-stride passes, a ragged last pass)
@pytest.mark.parametrize("model,n", [("kf6", 100003), ("ekf9", 5000), ("kf12d", 3000), ("kf6", 1 << 20),
                                     ("ekf9", 1 << 20), ("kf6", 3 * (1 << 20) + 5), ("kf12d", 300001)])
def test_ensemble_partial(orc, model, n):
    rng = np.random.default_rng(5)
    with Engine(model, n) as e:
        x = (rng.normal(size=(e.nx, n)) * np.arange(1, e.nx + 1)[:, None] + 3.0).astype(e.dtype)
        e.set_state(x, None)
        r1 = e.ensemble_partial()
        r2 = e.ensemble_partial()
    bits_equal(r1, r2, "deterministic")
    ro = orc.ens_partial(x)
    assert r1[0] == n
    np.testing.assert_allclose(r1[1:1 + x.shape[0]], ro[1:1 + x.shape[0]], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(r1[1 + x.shape[0]:], ro[1 + x.shape[0]:], rtol=1e-9)


# ----------------------------------------------------------------------------- edge cases
def test_edge_rpm_extremes_and_single_instance(orc):
    rpm = np.array([[-32768, 32767, -1, 0]], np.int16)
    yaw = np.float32([179.99])
    gz = np.float32([-2000.0])
    with Engine("kf6", 1) as e:
        e.tick(yaw_deg=yaw, gyro_z_dps=gz, rpm=rpm)
        x, P = e.get_state()
    xo, Po = _kf6_oracle(orc, 1, yaw[None], gz[None], rpm[None], None, orc.TRIG_TABLE512, 1)
    bits_equal(x, xo)
    bits_equal(P, Po)


def test_bad_inputs_rejected():
    with Engine("kf6", 64) as e:
        with pytest.raises(fmskf.FmskfError):
            e.tick_many(2, yaw_deg=np.zeros((2, 64), np.float32))  # missing planes
        with pytest.raises(fmskf.FmskfError):
            e.get_prev_sum()  # RS only
        # extents are checked before any kernel can read past a short buffer
        with pytest.raises(ValueError):
            e.tick_many(4, yaw_deg=np.zeros((2, 64), np.float32),
                        gyro_z_dps=np.zeros((4, 64), np.float32), rpm=np.zeros((4, 64, 4), np.int16))
        with pytest.raises(ValueError):
            e.tick(yaw_deg=np.zeros(63, np.float32), gyro_z_dps=np.zeros(64, np.float32),
                   rpm=np.zeros((64, 4), np.int16))
        with pytest.raises(TypeError):
            e.tick(yaw=np.zeros(64, np.float32))


# ----------------------------------------------------------------------------- fused ensemble
# KF6 at 2^20 runs the two-robots-per-lane tick (k_kf6p) with the record epilogue; at
# 3 * 2^20 + 5 the state outgrows the Infinity Cache and the one-robot-per-lane tick (k_kf6t)
# carries it, 6145 block records
@pytest.mark.parametrize("model,n", [("kf6", 100003), ("kf6", 1), ("kf6", 70000), ("ekf9", 3000),
                                     ("kf6", 1 << 20), ("kf6", 3 * (1 << 20) + 5), ("ekf9", 1),
                                     ("ekf9", 700), ("ekf9", 1 << 20), ("ekf9", 1300001),
                                     ("kf12d", 1), ("kf12d", 3001), ("kf12d", 1 << 20), ("kf12d", 300001)])
def test_tick_ensemble_fused(orc, model, n):
    """fmskf_tick_ensemble = fmskf_tick + the record of the post-tick state: state bit-exact
    vs a plain tick, record vs the oracle's two-pass moments of that state, and bitwise
    reproducible."""
    T = 6
    tr = Trajectory(n, T, seed=88)
    if model == "kf6":
        yaw, gz, rpm = tr.kf6_inputs()
        kw = lambda t: dict(yaw_deg=yaw[t], gyro_z_dps=gz[t], rpm=rpm[t])  # noqa: E731
    elif model == "ekf9":
        raw = tr.ekf9_raw()
        kw = lambda t: dict(raw=raw[t])  # noqa: E731
    else:  # KF12D: the decorrelated fp64 tick with the record epilogue (past the Infinity
        # Cache at 2^20: the non-temporal instantiation)
        z = np.ascontiguousarray(tr.kf12d_z())
        kw = lambda t: dict(z=np.ascontiguousarray(z[t]))  # noqa: E731
    with Engine(model, n) as a, Engine(model, n) as b, Engine(model, n) as c:
        for t in range(T - 1):
            for e in (a, b, c):
                e.tick(**kw(t))
        a.tick(**kw(T - 1))
        rb = b.tick_ensemble(**kw(T - 1))
        rc = c.tick_ensemble(**kw(T - 1))
        xa, Pa = a.get_state()
        xb, Pb = b.get_state()
        rp = b.ensemble_partial()
    bits_equal(xa, xb, "x")
    bits_equal(Pa, Pb, "P")
    bits_equal(rb, rc, "deterministic")
    assert rb[0] == n
    mo, co = orc.ens_finalize(xb.shape[0], orc.ens_partial(xb))
    mf, cf = fmskf.ensemble_combine(xb.shape[0], rb[None, :])
    np.testing.assert_allclose(mf, mo, rtol=1e-12, atol=1e-12)
    if n > 1:
        np.testing.assert_allclose(cf, co, rtol=1e-9, atol=1e-15)
    # same statistics as the stand-alone partial record of the same state
    mp, cp = fmskf.ensemble_combine(xb.shape[0], rp[None, :])
    np.testing.assert_allclose(mf, mp, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("n,trig,masked,records", [(70000, LIBM, False, False), (70000, TABLE, True, False),
                                                   (3001, TABLE, True, True), (3 * (1 << 20) + 5, TABLE, True, True)])
def test_tick_ensemble_fused_libm_and_mask(orc, n, trig, masked, records):
    """The fused KF6 tick + record under the LIBM sin/cos policy, with a validity mask, with
    16-byte tick records, and past the Infinity Cache (k_kf6t): the state bit-exact against a
    plain tick of the same inputs, the record against the oracle's moments of that state."""
    import torch
    T = 3
    tr = Trajectory(n, T, seed=91)
    yaw, gz, rpm = tr.kf6_inputs()
    valid = (np.random.default_rng(n).random((T, n)) > 0.3).astype(np.uint8) if masked else None
    if records:
        recs = fmskf.kf6_records(*(torch.from_numpy(a).cuda() for a in (yaw, gz, rpm)))
        kw = lambda t: dict(kf6_rec=recs[t], **({"valid": torch.from_numpy(valid[t]).cuda()}  # noqa: E731
                                                if masked else {}))
    else:
        kw = lambda t: dict(yaw_deg=yaw[t], gyro_z_dps=gz[t], rpm=rpm[t],  # noqa: E731
                            **({"valid": valid[t]} if masked else {}))
    with Engine("kf6", n, trig=trig) as a, Engine("kf6", n, trig=trig) as b:
        for e in (a, b):
            e.set_stream(torch.cuda.current_stream())
        for t in range(T - 1):
            a.tick(**kw(t))
            b.tick(**kw(t))
        a.tick(**kw(T - 1))
        rb = b.tick_ensemble(**kw(T - 1))
        xa, Pa = a.get_state()
        xb, Pb = b.get_state()
    bits_equal(xa, xb, "x")
    bits_equal(Pa, Pb, "P")
    assert rb[0] == n
    mo, co = orc.ens_finalize(6, orc.ens_partial(xb))
    mf, cf = fmskf.ensemble_combine(6, rb[None, :])
    np.testing.assert_allclose(mf, mo, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(cf, co, rtol=1e-9, atol=1e-15)


@pytest.mark.parametrize("n", [5000, 1300001])
def test_tick_ensemble_fused_ekf9_libm_mask(orc, n):
    """EKF9 fused tick + record with the LIBM policy (the one-robot-per-lane kernel) and with a
    validity mask under TABLE512 (two robots per lane below the Infinity Cache size, one per
    lane past it): state bit-exact against plain ticks, the record against the oracle."""
    T = 3
    tr = Trajectory(n, T, seed=92)
    raw = tr.ekf9_raw()
    valid = (np.random.default_rng(n).random((T, n)) > 0.3).astype(np.uint8)
    for trig, masked in ((LIBM, False), (TABLE, True)):
        kw = lambda t: dict(raw=raw[t], **({"valid": valid[t]} if masked else {}))  # noqa: E731
        with Engine("ekf9", n, trig=trig) as a, Engine("ekf9", n, trig=trig) as b:
            for t in range(T - 1):
                a.tick(**kw(t))
                b.tick(**kw(t))
            a.tick(**kw(T - 1))
            rb = b.tick_ensemble(**kw(T - 1))
            xa, Pa = a.get_state()
            xb, Pb = b.get_state()
        bits_equal(xa, xb, "x")
        bits_equal(Pa, Pb, "P")
        assert rb[0] == n
        mo, co = orc.ens_finalize(9, orc.ens_partial(xb))
        mf, cf = fmskf.ensemble_combine(9, rb[None, :])
        np.testing.assert_allclose(mf, mo, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(cf, co, rtol=1e-9, atol=1e-15)


# ----------------------------------------------------------------------------- state layout
@pytest.mark.parametrize("model,n", [("kf6", 1000), ("ekf9", 1), ("ekf9", 1000), ("kf12d", 257),
                                     ("kf12d", 3 * 256), ("rs", 300)])
def test_state_round_trip_and_reset(model, n):
    """fmskf_set_state / get_state round-trip the dense planes bit for bit whatever the device
    layout (tiled for EKF9 / KF12D, planar pitch for KF6 / RS), from host and from device
    memory, at ragged N; fmskf_reset restores x = 0 and P = P0 in every row."""
    import torch
    rng = np.random.default_rng(n)
    with Engine(model, n) as e:
        nx, np_ = e.nx, e.np_
        x = rng.normal(size=(nx, n)).astype(e.dtype)
        P = rng.normal(size=(np_, n)).astype(e.dtype) if e.m else None
        e.set_state(x, P)
        gx, gP = e.get_state()
        bits_equal(gx, x, "x host")
        if P is not None:
            bits_equal(gP, P, "P host")
        x2 = (x * 2).astype(e.dtype)
        e.set_state(torch.from_numpy(x2).cuda(), None)
        torch.cuda.synchronize()
        bits_equal(e.get_state()[0], x2, "x device")
        if P is not None:
            bits_equal(e.get_state()[1], P, "P kept")
        pose = e.get_pose()
        bits_equal(pose, x2[:3], "pose readout")
        e.reset()
        gx, gP = e.get_state()
        assert not gx.any()
        if P is not None:
            p0 = np.array(fmskf.default_config(model, n).p0[:np_], dtype=e.dtype)
            bits_equal(gP, np.repeat(p0[:, None], n, 1), "P0")


def test_tick_many_strided_rings_and_edge_sizes(orc):
    """tick_many over rings whose per-tick stride exceeds N (records and planes), N = 1 for
    the tiled models, and an all-zero validity mask (predict only) -- each equal to the same
    ticks issued one by one."""
    n, T, pad = 300, 5, 77
    _, yaw, gz, rpm, valid = _kf6_setup(n, T, 90)
    st = n + pad
    rec = fmskf.kf6_records(yaw, gz, rpm)
    ring = np.zeros((T, st), rec.dtype)
    ring[:, :n] = rec
    y2, g2, r2 = (np.zeros((T, st) + a.shape[2:], a.dtype) for a in (yaw, gz, rpm))
    y2[:, :n], g2[:, :n], r2[:, :n] = yaw, gz, rpm
    v2 = np.zeros((T, st), np.uint8)
    v2[:, :n] = valid
    with Engine("kf6", n) as a, Engine("kf6", n) as b, Engine("kf6", n) as c:
        a.tick_many(T, tick_stride=st, kf6_rec=ring, valid=v2)
        b.tick_many(T, tick_stride=st, yaw_deg=y2, gyro_z_dps=g2, rpm=r2, valid=v2)
        for t in range(T):
            c.tick(kf6_rec=rec[t], valid=valid[t])
        (xa, Pa), (xb, Pb), (xc, Pc) = (e.get_state() for e in (a, b, c))
    for x, P, what in ((xa, Pa, "records"), (xb, Pb, "planes")):
        bits_equal(x, xc, "x " + what)
        bits_equal(P, Pc, "P " + what)
    # N = 1, tiled models, tick_many vs ticks; an all-zero mask skips every update
    tr = Trajectory(1, 4, seed=91)
    raw = tr.ekf9_raw()
    z = np.ascontiguousarray(tr.kf12d_z())
    zero = np.zeros((4, 1), np.uint8)
    for model, kw_many, kw_t in (("ekf9", dict(raw=raw), lambda t: dict(raw=raw[t])),
                                 ("kf12d", dict(z=z), lambda t: dict(z=z[t]))):
        with Engine(model, 1) as a, Engine(model, 1) as b, Engine(model, 1) as c, \
                Engine(model, 1) as d:
            a.tick_many(4, **kw_many)
            c.tick_many(4, valid=zero, **kw_many)
            for t in range(4):
                b.tick(**kw_t(t))
                d.predict()
            bits_equal(a.get_state()[0], b.get_state()[0], model + " x")
            bits_equal(a.get_state()[1], b.get_state()[1], model + " P")
            bits_equal(c.get_state()[0], d.get_state()[0], model + " masked x")
            bits_equal(c.get_state()[1], d.get_state()[1], model + " masked P")


_VARIANT_SCRIPT = r"""
import sys, numpy as np
sys.path[:0] = sys.argv[1:3]
import fmskf
from fmskf import Engine
from fmskf.synth import Trajectory
from oracle import oracle as orc
for n in (1, 777, 5000):
    T = 6
    tr = Trajectory(n, T, seed=n)
    yaw, gz, rpm = tr.kf6_inputs()
    valid = (np.random.default_rng(n).random((T, n)) > 0.2).astype(np.uint8)
    rec = fmskf.kf6_records(yaw, gz, rpm)
    with Engine("kf6", n) as e:
        for t in range(T):
            e.tick(kf6_rec=rec[t], valid=valid[t]) if t % 2 else e.tick(yaw_deg=yaw[t], gyro_z_dps=gz[t], rpm=rpm[t], valid=valid[t])
        x, P = e.get_state()
    cfg = fmskf.default_config("kf6", n)
    prm = orc.kf6_params(cfg.dt, np.array(cfg.q[:21]), np.array(cfg.r[:10]))
    xo = np.zeros((6, n), np.float32)
    Po = np.repeat(np.float32(np.array(cfg.p0[:21]))[:, None], n, 1).copy()
    for t in range(T):
        orc.kf6_tick(xo, Po, yaw[t], gz[t], rpm[t], valid[t], prm, nthreads=0)
    assert np.array_equal(x.view(np.uint32), xo.view(np.uint32)), n
    assert np.array_equal(P.view(np.uint32), Po.view(np.uint32)), n
print("variant ok")
"""


@pytest.mark.parametrize("variant", ["15", "12"])
def test_kf6_single_tick_variants_bitexact(variant):
    """The single-tick KF6 kernels forced at small N (the launcher picks k_kf6p with 2 robots
    per lane at these sizes): k_kf6t (one robot per lane, the choice past the Infinity Cache)
    and k_kf6p with 2 robots per lane without the occupancy cap, forced through
    FMSKF_KF6_VARIANT in a child process, bit-exact against the oracle with planes, records
    and a validity mask."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, FMSKF_KF6_VARIANT=variant)
    out = subprocess.run([sys.executable, "-c", _VARIANT_SCRIPT, root,
                          os.path.join(root, "roboken-fmskf-robot-controller_amd")],
                         capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "variant ok" in out.stdout


_NT_SCRIPT = r"""
import sys, numpy as np
sys.path[:0] = sys.argv[1:3]
import fmskf
from fmskf import Engine
from fmskf.synth import Trajectory
from oracle import oracle as orc
for n in (1, 700, 1000):
    T = 5
    tr = Trajectory(n, T, seed=60 + n)
    valid = (np.random.default_rng(n).random((T, n)) > 0.2).astype(np.uint8)
    raw = tr.ekf9_raw()
    cfg = fmskf.default_config("ekf9", n)
    with Engine("ekf9", n) as e:
        for t in range(T):
            e.tick(raw=raw[t], valid=valid[t])
        x, P = e.get_state()
    prm = orc.ekf9_params(cfg.dt, np.array(cfg.q[:45]), np.array(cfg.r[:21]), orc.TRIG_TABLE512)
    xo = np.zeros((10, n), np.float32)
    Po = np.repeat(np.float32(np.array(cfg.p0[:45]))[:, None], n, 1).copy()
    for t in range(T):
        orc.ekf9_tick(xo, Po, raw[t], valid[t], prm, nthreads=0)
    assert np.array_equal(x.view(np.uint32), xo[:9].view(np.uint32)), ("ekf9", n)
    assert np.array_equal(P.view(np.uint32), Po.view(np.uint32)), ("ekf9", n)
    z = np.ascontiguousarray(tr.kf12d_z())
    for cross in (False, True):
        cfg = fmskf.default_config("kf12d", n)
        r = np.array(cfg.r[:36])
        if cross:
            r[4 * 5 // 2 + 0] = 1e-6
        with Engine("kf12d", n, r=r) as e:
            for t in range(T):
                e.tick(z=z[t], valid=valid[t])
            x, P = e.get_state()
        prm = orc.kf12d_params(cfg.dt, np.array(cfg.q[:78]), r)
        xo = np.zeros((12, n))
        Po = np.repeat(np.array(cfg.p0[:78])[:, None], n, 1).copy()
        for t in range(T):
            orc.kf12d_tick(xo, Po, np.ascontiguousarray(z[t]), valid[t], prm, nthreads=0)
        assert np.array_equal(x.view(np.uint64), xo.view(np.uint64)), ("kf12d", n, cross)
        assert np.array_equal(P.view(np.uint64), Po.view(np.uint64)), ("kf12d", n, cross)
print("nt ok")
"""


def test_nontemporal_state_kernels_bitexact():
    """The non-temporal state instantiations (chosen automatically once the state outgrows the
    Infinity Cache, fmskf_internal.hpp state_nt) forced on at small N in a child process:
    EKF9 and KF12D (block-diagonal and correlated R) with a validity mask, and KF6's k_kf6t
    through the variant script, bit-exact against the oracle."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, FMSKF_STATE_NT="1", FMSKF_KF6_VARIANT="15")
    args = [root, os.path.join(root, "roboken-fmskf-robot-controller_amd")]
    for script, ok in ((_NT_SCRIPT, "nt ok"), (_VARIANT_SCRIPT, "variant ok")):
        out = subprocess.run([sys.executable, "-c", script] + args,
                             capture_output=True, text=True, timeout=240, env=env)
        assert out.returncode == 0, out.stderr[-3000:]
        assert ok in out.stdout


@pytest.mark.parametrize("ekf9", ["4", "2"])
def test_ekf9_kernel_variants_bitexact(ekf9):
    """Both EKF9 single-tick kernels (FMSKF_EKF9_VARIANT: 2 two robots per lane -- the default
    while the state fits the Infinity Cache --, 4 one robot per lane), forced in a child
    process, with a validity mask at N = 1, 700 (an odd tile count: the last two-robot block
    has no second tile) and 1000, bit-exact against the oracle."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, FMSKF_EKF9_VARIANT=ekf9)
    out = subprocess.run([sys.executable, "-c", _NT_SCRIPT, root,
                          os.path.join(root, "roboken-fmskf-robot-controller_amd")],
                         capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "nt ok" in out.stdout


def test_rs_one_robot_per_lane_bitexact():
    """FMSKF_RS_TWO=0 (k_rs, one robot per lane, instead of k_rs2) in a child process: the RS
    tick parity test against the oracle, both trig policies."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = (
        "import sys\n"
        "sys.path[:0] = sys.argv[1:4]\n"
        "from oracle import oracle as orc\n"
        "import test_gpu_parity as T\n"
        "T.test_rs_tick_bitexact(orc, T.TABLE)\n"
        "T.test_rs_tick_bitexact(orc, T.LIBM)\n"
        "print('rs ok')\n")
    env = dict(os.environ, FMSKF_RS_TWO="0")
    out = subprocess.run([sys.executable, "-c", script, root,
                          os.path.join(root, "roboken-fmskf-robot-controller_amd"),
                          os.path.join(root, "tests")],
                         capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "rs ok" in out.stdout


_WT901_TR_SCRIPT = r"""
import sys, numpy as np
sys.path[:0] = sys.argv[1:3]
from fmskf import Engine
from fmskf.synth import wt901_frame
from oracle import oracle as orc
rng = np.random.default_rng(4242)
stride = 48


def clean(m):
    fr = np.zeros((m, 4, 11), np.uint8)
    fr[:, :, 0] = 0x55
    fr[:, :, 1] = np.array([0x51, 0x52, 0x53, 0x59], np.uint8)
    fr[:, :, 2:10] = rng.integers(0, 256, (m, 4, 8), dtype=np.uint8)
    fr[:, :, 10] = (fr[:, :, :10].sum(axis=2, dtype=np.uint32) & 0xFF).astype(np.uint8)
    return fr.reshape(m, 44)


# n % 8 == 0 with a partial last wave, n % 8 != 0 (per-lane stores only), one full wave
for n in (2584, 2585, 64):
    nw = -(-n // 64)
    ob = orc.Wt901Batch(n)
    with Engine("kf6", n) as e:
        for k in range(6):
            buf = np.zeros((n, stride), np.uint8)
            buf[:, :44] = clean(n)
            lens = np.full(n, 44, np.uint32)
            for w in range(nw):
                lo, hi = 64 * w, min(64 * w + 64, n)
                kind = (w + k) % 5
                if kind == 1:  # one damaged byte in one lane
                    buf[lo + (w % (hi - lo)), 7] ^= 0x5A
                elif kind == 2:  # a torn poll: its tail is pending in the next poll's window
                    lens[lo + (3 * w) % (hi - lo)] = 30
                elif kind == 3:  # a different frame order in one lane
                    r = lo + (5 * w) % (hi - lo)
                    buf[r, :44] = np.frombuffer(b"".join(wt901_frame(t, rng.integers(0, 65536, 4))
                                                         for t in (0x59, 0x51, 0x52, 0x53)), np.uint8)
                # kind 0 and 4: every lane a clean standard poll (the transposed store)
            ob.update(buf, lens, latch_qinit=(k == 0))
            e.ingest_wt901(buf, lens, latch_qinit=(k == 0))
            regs, pending = e.get_imu_regs()
            data, err = e.get_imu()
            st = orc._struct_view(ob.s, orc.Wt901State)
            assert np.array_equal(regs, st["reg"].T), (n, k)
            assert np.array_equal(pending, st["cnt"].astype(np.uint8)), (n, k)
            assert np.array_equal(err, st["is_error"]), (n, k)
            assert np.array_equal(data.view(np.uint32), ob.data.view(np.uint32)), (n, k)
print("wt901 ok")
"""


def test_wt901_wave_patterns_bitexact():
    """k_wt901 on wave-structured polls (round 4 measured LDS-transposed stores for waves of
    standard polls and kept the per-lane form; this pattern set checked all three bit-exact):
    waves of clean standard polls next to waves with one damaged, torn or reordered lane, a
    partial last wave, N % 8 != 0 and a single wave; every robot's register file, parser backlog,
    error flag and Data page against the oracle after every poll, bit for bit (child process)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", _WT901_TR_SCRIPT, root,
                          os.path.join(root, "roboken-fmskf-robot-controller_amd")],
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "wt901 ok" in out.stdout


def test_can_rs_per_plane_descriptor_forms_bitexact():
    """The per-plane descriptor form of k_rs2 (FMSKF_RS_VARIANT=0; the default reaches every plane
    of an array through one descriptor and soffset) in a child process: the RS tick parity tests
    against the oracle, with the CAN ingest tests beside them (round 6: k_can4 has one form)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = (
        "import sys\n"
        "sys.path[:0] = sys.argv[1:4]\n"
        "from oracle import oracle as orc\n"
        "import test_gpu_parity as T\n"
        "T.test_can_ingest_bitexact(orc, False)\n"
        "T.test_can_ingest_bitexact(orc, 'mixed')\n"
        "T.test_rs_tick_bitexact(orc, T.TABLE)\n"
        "T.test_rs_tick_bitexact(orc, T.LIBM)\n"
        "print('planes ok')\n")
    env = dict(os.environ, FMSKF_RS_VARIANT="0")
    out = subprocess.run([sys.executable, "-c", script, root,
                          os.path.join(root, "roboken-fmskf-robot-controller_amd"),
                          os.path.join(root, "tests")],
                         capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "planes ok" in out.stdout
