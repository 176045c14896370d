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
