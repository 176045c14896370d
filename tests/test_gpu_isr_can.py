"""fmskf_isr_tick_can: the tick's CAN RX and the firmware ISR in one call (one kernel for RS, KF6
and EKF9, k_isr_rs / k_isr_kf6 / k_isr_ekf9 with the C610 lane of can_lane.hpp in front) against the two calls it replaces,
fmskf_ingest_can + fmskf_isr_tick, on random targets / power events.  Bar: bit-exact for the
estimator state, the control state, the 0x200 frames and the whole motor state
(MOTOR_IF_M2006::rx_callback, VD_motor_if_m2006.cpp; the two-call path is itself held to the
oracle by test_gpu_parity / test_gpu_ctrl)."""
import numpy as np
import pytest

import fmskf
from fmskf import Engine
from fmskf.synth import Trajectory

pytestmark = pytest.mark.gpu


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint32) if a.dtype == np.float32 else a


# kf6* / rs* / ekf9*: the fused kernels (planes, LIBM, validity mask, compensated positions,
# device-resident frames, a ragged last block, the non-temporal control regime past the Infinity
# Cache); kf6rpm / kf6rec / rssum / ekf9rpm: the documented two-call fallback (a caller rpm,
# records, caller sums)
CASES = [("kf6", 4099, 40), ("kf6", 1, 20), ("kf6libm", 777, 20), ("kf6mask", 1001, 20),
         ("kf6comp", 513, 20), ("kf6dev", 2048 + 5, 20), ("kf6rpm", 300, 12), ("kf6rec", 257, 12),
         ("rs", 999, 30), ("rs", 1, 12), ("rslibm", 700, 12), ("rssum", 333, 12),
         ("kf6mixmem", 3000, 12), ("rsmixmem", 3000, 12),
         ("ekf9", 1000, 20), ("ekf9", 1, 12), ("ekf9libm", 513, 12), ("ekf9rpm", 400, 12),
         ("ekf9", (1 << 20) + 17, 3),
         ("kf6", (1 << 20) + 17, 3), ("rs", (1 << 20) + 17, 3)]


FALLBACK = ("kf6rpm", "kf6rec", "rssum", "ekf9rpm")


@pytest.mark.parametrize("case,n,T", CASES)
def test_isr_tick_can_equals_ingest_then_isr(case, n, T):
    import torch
    rng = np.random.default_rng(7 + n)
    tr = Trajectory(n, T, seed=53)
    trig = fmskf.TRIG_LIBM if case.endswith("libm") else fmskf.TRIG_TABLE512
    flags = fmskf.CFG_COMP_POS if case == "kf6comp" else 0
    model = "rs" if case.startswith("rs") else "ekf9" if case.startswith("ekf9") else "kf6"
    raw = tr.ekf9_raw() if model == "ekf9" else None
    dev_in = case.endswith("mixmem")  # host CAN frames, device tick inputs: two staging flags
    sums = np.ascontiguousarray(tr.rs_inputs()[1]) if case == "rssum" else None
    yaw, gz, rpm = tr.kf6_inputs()
    valid = (rng.random((T, n)) > 0.25).astype(np.uint8) if case == "kf6mask" else None

    def kw(t):
        if model == "ekf9":  # the raw WT901 words; ekf9rpm: the caller's rpm plane (two calls)
            return dict(raw=raw[t], rpm=rpm[t]) if case == "ekf9rpm" else dict(raw=raw[t])
        if case == "rssum":  # the caller's sums: CAN RX, then the ISR on them
            return dict(yaw_deg=yaw[t], angle_sum=sums[t])
        if model == "rs" and not dev_in:
            return dict(yaw_deg=yaw[t])  # sums and rpm: the device motor state
        if case == "kf6rec":
            return dict(kf6_rec=fmskf.kf6_records(yaw, gz, rpm)[t])
        if dev_in:
            d = dict(yaw_deg=torch.from_numpy(yaw[t]).cuda())
            if model == "kf6":
                d["gyro_z_dps"] = torch.from_numpy(gz[t]).cuda()
            return d
        d = dict(yaw_deg=yaw[t], gyro_z_dps=gz[t])
        if case == "kf6rpm":
            d["rpm"] = rpm[t]
        if valid is not None:
            d["valid"] = valid[t]
        return d

    vel = np.stack([rng.uniform(-400, 400, n), rng.uniform(-400, 400, n),
                    rng.uniform(-3, 3, n)]).astype(np.float32)
    acl = np.full((3, n), 1000.0, np.float32)
    jrk = np.full((3, n), 10000.0, np.float32)
    with Engine(model, n, trig=trig, flags=flags) as a, Engine(model, n, trig=trig, flags=flags) as b:
        on = (rng.random(n) < 0.9).astype(np.uint8)
        for e in (a, b):
            e.set_power(on)
            e.set_target_vel(vel, acl, jrk)
        for t in range(T):
            f, s = tr.can_frames(t)
            if case == "kf6dev":
                f, s = (torch.from_numpy(np.ascontiguousarray(f)).cuda(),
                        torch.from_numpy(np.ascontiguousarray(s)).cuda())
            last = t == T - 1 or t % 5 == 1
            fa = a.isr_tick_can(f, s, frames=last, **kw(t))
            b.ingest_can(f, s)
            if case != "kf6dev":
                fb = b.isr_tick(frames=last, **kw(t))
            elif last:
                fb = b.isr_tick(out=torch.empty((n, 8), dtype=torch.uint8, device="cuda"), **kw(t)).cpu().numpy()
                fa = fa.cpu().numpy()
            else:
                b.isr_tick(frames=False, **kw(t))
            if last:
                np.testing.assert_array_equal(fa, fb)
        xa, Pa = a.get_state()
        xb, Pb = b.get_state()
        ga, gb = a.get_ctrl(), b.get_ctrl()
        ma, mb = a.get_motors(), b.get_motors()
        ca, cb = a.get_counters(), b.get_counters()
    # which launch form ran (fmskf_get_counters [1]: CAN RX as its own kernel, [2]: the ISR as
    # three kernels): the fused cases really ran one kernel per tick, the documented fallbacks
    # (a caller rpm / records / sums) ran the two calls every tick
    if case in FALLBACK:
        assert ca[1] == T, (case, ca[:3])
    else:
        assert ca[1] == 0 and ca[2] == 0, (case, ca[:3])
    assert cb[1] == 0 and cb[2] == ca[2], (case, ca[:3], cb[:3])
    np.testing.assert_array_equal(bits(xa), bits(xb))
    if Pa is not None:
        np.testing.assert_array_equal(bits(Pa), bits(Pb))
    for k in ("vel_tgt", "curr", "wheel_tgt", "wheel_ctrl"):
        np.testing.assert_array_equal(bits(ga[k]), bits(gb[k]))
    for k in ma:
        np.testing.assert_array_equal(bits(ma[k]), bits(mb[k]), err_msg=k)


def test_isr_tick_can_errors():
    """null CAN buffers and a bad mem flag are refused before any launch (the handle stays usable)"""
    import ctypes as C
    n = 64
    with Engine("kf6", n) as e:
        L = fmskf._lib.load()
        assert L.fmskf_isr_tick_can(e.h, None, None, None, None, fmskf.MEM_HOST) == fmskf._lib.EINVAL
        f = np.zeros((n, 4, 8), np.uint8)
        s = np.zeros((n, 4), np.int16)
        assert L.fmskf_isr_tick_can(e.h, f.ctypes.data_as(C.c_void_p), s.ctypes.data_as(C.c_void_p),
                                    None, None, 7) == fmskf._lib.EINVAL
        e.isr_tick_can(f, s, frames=False)
        import torch
        with pytest.raises(TypeError):  # host CAN frames, device TX buffer: one mem flag covers both
            e.isr_tick_can(f, s, out=torch.empty((n, 8), dtype=torch.uint8, device="cuda"))
        with pytest.raises(ValueError):  # short CAN arrays are caught before the C call
            e.isr_tick_can(f[: n // 2], s)


def test_isr_tick_can_kf12d_counts_three_kernels():
    """KF12D has no fused ISR: fmskf_isr_tick_can runs CAN RX, the tick, the control step and the
    frame as separate kernels, and the handle's counters say so"""
    n, T = 300, 3
    tr = Trajectory(n, T, seed=5)
    z = tr.kf12d_z()
    with Engine("kf12d", n) as e:
        for t in range(T):
            f, s = tr.can_frames(t)
            e.isr_tick_can(f, s, frames=False, z=z[t])
        c = e.get_counters()
    assert c[1] == T and c[2] == T, c[:3]


# the scripted sequence of test_rs_prev_in_motor_sums: every transition of where the RS
# odometry's previous sums live (fmskf_ctx rs_prev_synced / rs_prev_stale)
RS_OPS = (["fused"] * 3 + ["prev"] + ["split"] + ["fused"] * 2 + ["caller_sums"] + ["fused"] * 2 + ["ckpt"]
          + ["fused"] * 2 + ["graph"] + ["fused"] + ["predict_only"] + ["fused"] * 2 + ["prev", "fused", "reset"]
          + ["fused"] * 3 + ["ingest_only", "fused", "fused", "prev"])


def test_rs_prev_in_motor_sums(orc, tmp_path):
    """fmskf_isr_tick_can, reference semantics: once the last predict read the motor state's sums,
    the fused kernel takes the previous sums (s64_rawAngleSumPrev) from the motor state and skips
    the prev planes (k_isr_rs PS); every other reader / writer brings them back first.  A scripted
    mix of fused ticks, the two-call form, a tick on caller sums, a checkpoint round trip, a graph
    capture and replay, a predict on the motor sums, a stand-alone CAN RX and a reset, against the
    oracle (orc_m2006_rx + orc_rs_tick, VD_motor_if_m2006.cpp:32-72, VD_vehicle_controller.cpp:
    36-51): the pose after every step and the previous sums at the `prev` steps, bit for bit."""
    import torch
    n = 1001
    T = len(RS_OPS) + 2
    tr = Trajectory(n, T, seed=77)
    yaw = tr.kf6_inputs()[0]
    csum = tr.rs_inputs()[1]  # [T][4][N] sums unrelated to the motor state's
    rpm_c = tr.rs_inputs()[2]
    mb = orc.MotorBatch(n)
    pos, vel, prev = np.zeros((3, n), np.float32), np.zeros((3, n), np.float32), np.zeros((4, n), np.int64)
    prev_stream = torch.cuda.current_stream()
    stream = torch.cuda.Stream()  # graph capture needs a real stream; the copies below queue on it too
    torch.cuda.set_stream(stream)
    e = Engine("rs", n)
    e.set_stream(stream)

    def oracle_tick(t, sums=None, rpm=None, correct=True):
        r = mb.field("rpm") if rpm is None else rpm
        s = np.ascontiguousarray(mb.field("angle_sum").T) if sums is None else np.ascontiguousarray(sums)
        orc.rs_tick(pos, vel, prev, yaw[t], s, r, do_correct=correct)

    t = 0
    try:
        for op in RS_OPS:
            f, s = tr.can_frames(t)
            if op == "fused":
                e.isr_tick_can(f, s, frames=False, yaw_deg=yaw[t])
                mb.rx(f, s)
                oracle_tick(t)
            elif op == "split":
                e.ingest_can(f, s)
                e.isr_tick(frames=False, yaw_deg=yaw[t])
                mb.rx(f, s)
                oracle_tick(t)
            elif op == "caller_sums":  # the odometry on the caller's sums: prev = those
                e.ingest_can(f, s)
                e.tick(yaw_deg=yaw[t], angle_sum=csum[t], rpm=rpm_c[t])
                mb.rx(f, s)
                oracle_tick(t, csum[t], rpm_c[t])
            elif op == "predict_only":  # predict on the motor state's sums (no correct)
                e.ingest_can(f, s)
                e.predict()
                mb.rx(f, s)
                oracle_tick(t, correct=False)
            elif op == "ingest_only":  # CAN RX with no tick: the motor sums move ahead of prev
                e.ingest_can(f, s)
                mb.rx(f, s)
                t += 1
                continue
            elif op == "ckpt":
                path = str(tmp_path / "rs.ck")
                e.save_state(path)
                e.close()
                e = Engine("rs", n)
                e.set_stream(stream)
                e.load_state(path)
                e.isr_tick_can(f, s, frames=False, yaw_deg=yaw[t])
                mb.rx(f, s)
                oracle_tick(t)
            elif op == "graph":  # capture one fused call on device buffers, replay it twice
                fd = torch.from_numpy(np.ascontiguousarray(f)).cuda()
                sd = torch.from_numpy(np.ascontiguousarray(s)).cuda()
                yd = torch.from_numpy(np.ascontiguousarray(yaw[t])).cuda()
                e.graph_begin()
                e.isr_tick_can(fd, sd, frames=False, yaw_deg=yd)
                e.graph_end()
                for k in range(2):
                    f2, s2 = tr.can_frames(t + k)
                    fd.copy_(torch.from_numpy(np.ascontiguousarray(f2)))
                    sd.copy_(torch.from_numpy(np.ascontiguousarray(s2)))
                    yd.copy_(torch.from_numpy(np.ascontiguousarray(yaw[t + k])))
                    e.graph_launch(1)
                    mb.rx(f2, s2)
                    oracle_tick(t + k)
                t += 1
            elif op == "reset":
                e.reset()
                mb = orc.MotorBatch(n)
                pos[:], vel[:], prev[:] = 0, 0, 0
                t += 1
                continue
            elif op == "prev":
                np.testing.assert_array_equal(e.get_prev_sum(), prev, err_msg=f"previous sums after tick {t}")
                continue
            x, _ = e.get_state()
            np.testing.assert_array_equal(bits(x[:3]), bits(pos), err_msg=f"pose after {op} at tick {t}")
            np.testing.assert_array_equal(bits(x[3:]), bits(vel), err_msg=f"velocity after {op} at tick {t}")
            t += 1
        m = e.get_motors()
        np.testing.assert_array_equal(m["angle_sum"], mb.field("angle_sum").T)
    finally:
        e.close()
        torch.cuda.set_stream(prev_stream)


# ---- the split angle sums across 2^32 (round 6: low words every frame, high words on a carry)
_M64 = (1 << 64) - 1


def _ck_hash(body: bytes) -> int:
    """api_checkpoint.cpp CkHash: 64-bit multiply-xor over 8-byte little-endian words, the tail
    zero-padded, xor the length"""
    h = 0x9E3779B97F4A7C15
    pad = body + b"\0" * (-len(body) % 8)
    for (w,) in __import__("struct").iter_unpack("<Q", pad):
        h = ((h ^ w) * 0x100000001B3) & _M64
        h ^= h >> 29
    return h ^ len(body)


def _split_sums(sums):
    """fmskf_internal.hpp m_sum_lo / m_sum_hi: sum = hi * 2^32 + lo read as int32"""
    s = np.asarray(sums, np.int64)
    lo = ((s + (1 << 31)) & 0xFFFFFFFF) - (1 << 31)  # the signed low word
    return lo.astype(np.int32), ((s - lo) >> 32).astype(np.int32)


def _patch_motor_sums(path, n, sums):
    """rewrite the motor group's angle sums of an RS checkpoint (groups 1 | 4 | 8) to `sums`
    ([N][4] int64) and fix the checksum: a test-side forge of the split low / high words"""
    import struct
    from fmskf._lib import Config, CtrlParams
    blob = bytearray(open(path, "rb").read())
    groups = struct.unpack_from("<I", blob, 40)[0]
    assert groups == 1 | 4 | 8, groups
    pos = 88 + C_sizeof(Config) + C_sizeof(CtrlParams)
    secs = []
    while pos < len(blob):
        b = struct.unpack_from("<Q", blob, pos)[0]
        secs.append((pos + 8, b))
        pos += 8 + b
    # estimator group (RS: x, prev sums, counters), then the motor group: micro, angle, prev,
    # prev_micro, rpm, curr, sum_lo, sum_hi, iir_y
    (lo_off, lo_b), (hi_off, hi_b) = secs[3 + 6], secs[3 + 7]
    assert lo_b == hi_b == 16 * n
    lo, hi = _split_sums(sums)
    blob[lo_off:lo_off + lo_b] = lo.reshape(n, 4).tobytes()
    blob[hi_off:hi_off + hi_b] = hi.reshape(n, 4).tobytes()
    body = bytes(blob[88:])
    struct.pack_into("<QQ", blob, 64, len(body), _ck_hash(body))
    open(path, "wb").write(bytes(blob))


def C_sizeof(t):
    import ctypes
    return ctypes.sizeof(t)


def test_angle_sums_carry_across_2p32(orc, tmp_path):
    """s64_rawAngleSum (VD_motor_if_m2006.cpp:66-69) is kept as a signed low 32-bit word and a high
    word, and a frame writes the high word only when its delta carries the low word out of the
    int32 range.  Sums forged next to the carry boundaries (odd multiples of 2^31, with negative
    and positive high words) and next to 0 and 2^32 (no carry) are driven across them for a dozen
    ticks by +-3000..4000-count steps through every CAN path -- the fused RS CAN+ISR (its PS and
    whole-sum forms), fmskf_ingest_can (k_can4) with the RS tick on the motor state, and the
    masked wheel-per-lane kernel -- against the oracle's int64 sums, the previous sums and the
    pose, bit for bit."""
    n, T = 515, 14
    rng = np.random.default_rng(2032)
    dirs = np.array([1, 1, -1, -1])
    raw0 = rng.integers(0, 8192, (n, 4))
    step = rng.choice([4000, -4000, 3000, -3500], (n, 4))

    def frames(t):
        raw = (raw0 + t * step) % 8192
        fr = np.zeros((n, 4, 8), np.uint8)
        for k, v in enumerate((raw, rng.integers(-900, 900, (n, 4)) * dirs, np.full((n, 4), 100))):
            u = np.asarray(v, np.int64) & 0xFFFF
            fr[:, :, 2 * k] = (u >> 8).astype(np.uint8)
            fr[:, :, 2 * k + 1] = (u & 0xFF).astype(np.uint8)
        st = np.ascontiguousarray(np.broadcast_to(((t + 1) * 1000 + np.arange(4) * 7) & 0x7FFF, (n, 4))).astype(np.int16)
        return fr, st

    yaw = rng.uniform(-180, 180, (T + 2, n)).astype(np.float32)
    mb = orc.MotorBatch(n)
    ck = str(tmp_path / "rs.ck")
    with Engine("rs", n) as e:  # two warm-up ticks, then the checkpoint
        for t in range(2):
            f, s = frames(t)
            e.isr_tick_can(f, s, frames=False, yaw_deg=yaw[t])
            mb.rx(f, s)
        e.save_state(ck)
    lo = rng.choice([(1 << 32) - 6000, 6000, (1 << 31) - 5000, (1 << 31) + 5000], (n, 4)).astype(np.int64)
    hi = rng.integers(-3, 3, (n, 4)).astype(np.int64)
    sums = (hi << 32) + lo
    _patch_motor_sums(ck, n, sums)
    orc._struct_view(mb.m, orc.M2006State)["angle_sum"][:] = sums.reshape(-1)
    pos, vel = np.zeros((3, n), np.float32), np.zeros((3, n), np.float32)
    with Engine("rs", n) as e:
        e.load_state(ck)
        x, _ = e.get_state()
        pos[:], vel[:] = x[:3], x[3:]
        prev = e.get_prev_sum()
        np.testing.assert_array_equal(e.get_motors()["angle_sum"], sums.T)
        for t in range(2, T):
            f, s = frames(t)
            kind = t % 4
            if kind in (0, 1):  # the fused call (whole sums on its first tick, PS after)
                e.isr_tick_can(f, s, frames=False, yaw_deg=yaw[t])
                mb.rx(f, s)
            elif kind == 2:  # k_can4, then the RS tick on the motor state's sums
                e.ingest_can(f, s)
                mb.rx(f, s)
                e.tick(yaw_deg=yaw[t])
            else:  # the masked wheel-per-lane kernel (every wheel present), then the ISR
                e.ingest_can(f, s, present=np.full(n, 15, np.uint8))
                mb.rx(f, s)
                e.isr_tick(frames=False, yaw_deg=yaw[t])
            orc.rs_tick(pos, vel, prev, yaw[t], np.ascontiguousarray(mb.field("angle_sum").T), mb.field("rpm"))
            np.testing.assert_array_equal(e.get_motors()["angle_sum"], mb.field("angle_sum").T, err_msg=f"tick {t}")
            x, _ = e.get_state()
            np.testing.assert_array_equal(bits(x[:3]), bits(pos), err_msg=f"pose tick {t}")
        np.testing.assert_array_equal(e.get_prev_sum(), prev)
    moved = _split_sums(mb.field("angle_sum"))[1] != _split_sums(sums)[1]
    assert moved.sum() > n // 2, moved.sum()  # many wheels carried into another high word
