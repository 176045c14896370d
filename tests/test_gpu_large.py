"""GPU parity at sizes past the 4 GiB buffer window: the kernels' SMALL instantiations
address every plane array through one buffer descriptor with 32-bit offsets; beyond 4 GiB of
planes they switch to 64-bit addressing.  These runs take the large path and check a sample
of robots (first, last and random ones) against the oracle bit for bit."""
import numpy as np
import pytest

import fmskf
from fmskf import Engine

pytestmark = pytest.mark.gpu


def _sample(n, k=2048, seed=0):
    rng = np.random.default_rng(seed)
    idx = np.concatenate([np.arange(64), np.arange(n - 64, n), rng.choice(n, k, replace=False)])
    return np.unique(idx)


def test_kf6_past_the_buffer_window(orc):
    import torch
    from fmskf.synth import kf6_ring_torch
    n, T = 52_000_000, 3          # pitch * 84 B > 4 GiB -> 64-bit plane addressing
    assert fmskf_pitch(n) * 84 > 0xFFFFFFFF
    yaw, gz, rpm = kf6_ring_torch(n, T, seed=99, device="cuda")
    with Engine("kf6", n) as e:
        for t in range(T):
            e.tick(yaw_deg=yaw[t], gyro_z_dps=gz[t], rpm=rpm[t])
        x, P = e.get_state()
        assert e.get_counters()[0] == 0
    idx = _sample(n)
    ys, gs, rs = (a[:, torch.from_numpy(idx).cuda()].cpu().numpy() for a in (yaw, gz, rpm))
    cfg = fmskf.default_config("kf6", idx.size)
    prm = orc.kf6_params(cfg.dt, np.array(cfg.q[:21]), np.array(cfg.r[:10]))
    xo = np.zeros((6, idx.size), np.float32)
    Po = np.repeat(np.float32(np.array(cfg.p0[:21]))[:, None], idx.size, 1).copy()
    for t in range(T):
        orc.kf6_tick(xo, Po, np.ascontiguousarray(ys[t]), np.ascontiguousarray(gs[t]),
                     np.ascontiguousarray(rs[t]), None, prm, nthreads=0)
    np.testing.assert_array_equal(x[:, idx].view(np.uint32), xo.view(np.uint32))
    np.testing.assert_array_equal(P[:, idx].view(np.uint32), Po.view(np.uint32))


def test_kf6_headline_instantiation_2p20(orc):
    """The bench's exact headline kernel: the single fused tick fed 16-byte fmskf_kf6_records at
    exactly 2^20 robots (k_kf6p<4, 2, Opt<TABLE512, UPD, PRED, SMALL, !VALID, REC>>, two robots per
    lane while the state fits the Infinity Cache), fed by the bench's own input generator (the
    64-tick HBM ring of kf6_ring_torch) for 70 ticks (the ring wraps), sampled bit-exact
    against the oracle."""
    import torch
    from fmskf.synth import kf6_ring_torch
    n, R, T = 1 << 20, 64, 70
    yaw, gz, rpm = kf6_ring_torch(n, R, seed=2024, device="cuda")
    recs = fmskf.kf6_records(yaw, gz, rpm)
    with Engine("kf6", n) as e:
        e.set_stream(torch.cuda.current_stream())
        prepared = [e.prepare(kf6_rec=recs[r]) for r in range(R)]
        for t in range(T):
            e.tick_prepared(prepared[t % R])
        x, P = e.get_state()
        assert e.get_counters()[0] == 0
    idx = _sample(n, seed=20)
    ti = torch.from_numpy(idx).cuda()
    ys, gs, rs = (a[:, ti].cpu().numpy() for a in (yaw, gz, rpm))
    cfg = fmskf.default_config("kf6", idx.size)
    prm = orc.kf6_params(cfg.dt, np.array(cfg.q[:21]), np.array(cfg.r[:10]))
    xo = np.zeros((6, idx.size), np.float32)
    Po = np.repeat(np.float32(np.array(cfg.p0[:21]))[:, None], idx.size, 1).copy()
    for t in range(T):
        r = t % R
        orc.kf6_tick(xo, Po, np.ascontiguousarray(ys[r]), np.ascontiguousarray(gs[r]),
                     np.ascontiguousarray(rs[r]), None, prm, nthreads=0)
    np.testing.assert_array_equal(x[:, idx].view(np.uint32), xo.view(np.uint32))
    np.testing.assert_array_equal(P[:, idx].view(np.uint32), Po.view(np.uint32))


@pytest.mark.parametrize("n", [36_000_000, 46_000_000])
def test_control_past_the_buffer_window(orc, n):
    """36M: the 36 interpolator planes (144 B per robot) pass 4 GiB while the 24 FF_PI_D planes
    do not (the SMALL choice must follow the larger array); 46M: both pass."""
    import torch
    T = 40
    assert fmskf_pitch(n) * 4 * 36 > 0xFFFFFFFF
    g = torch.Generator(device="cuda").manual_seed(4)
    vel = torch.stack([torch.rand(n, generator=g, device="cuda") * 800 - 400,
                       torch.rand(n, generator=g, device="cuda") * 800 - 400,
                       torch.rand(n, generator=g, device="cuda") * 6 - 3])
    acl = torch.tensor([[1000.0], [1000.0], [30.0]], device="cuda").expand(3, n).contiguous()
    jrk = torch.tensor([[10000.0], [10000.0], [300.0]], device="cuda").expand(3, n).contiguous()
    rpm = torch.randint(-3000, 3000, (T, n, 4), generator=g, device="cuda", dtype=torch.int16)
    with Engine("kf6", n) as e:
        e.set_power(None)
        e.set_target_vel(vel, acl, jrk)
        for t in range(T):
            e.control(rpm[t])
        got = e.get_ctrl()
    idx = _sample(n, seed=1)
    ti = torch.from_numpy(idx).cuda()
    ref = orc.CtrlBatch(idx.size)
    ref.set_power(np.ones(idx.size, np.uint8))
    ref.set_target_vel(vel[:, ti].cpu().numpy(), acl[:, ti].cpu().numpy(), jrk[:, ti].cpu().numpy())
    rs = rpm[:, ti].cpu().numpy()
    for t in range(T):
        ref.step(np.ascontiguousarray(rs[t]))
    np.testing.assert_array_equal(got["curr"][idx], ref.curr())
    np.testing.assert_array_equal(got["vel_tgt"][:, idx].view(np.uint32), ref.vel_tgt().view(np.uint32))
    np.testing.assert_array_equal(got["wheel_ctrl"][:, idx].view(np.uint32),
                                  ref.wheel("ctrl").view(np.uint32))


def fmskf_pitch(n):
    return ((n + 511) // 512) * 512 + 256


@pytest.mark.parametrize("n", [1 << 20, 1 << 22])
def test_ekf9_sampled_with_mask(orc, n):
    """cfg 3's model with a random validity mask: a sample bit for bit. At 2^20 the state fits
    the Infinity Cache; at 2^22 (cfg 3's size) the tick streams it non-temporal."""
    from fmskf.synth import Trajectory
    T = 4
    tr = Trajectory(n, T, seed=12)
    raw = tr.ekf9_raw()
    valid = (np.random.default_rng(5).random((T, n)) > 0.2).astype(np.uint8)
    with Engine("ekf9", n) as e:
        for t in range(T):
            e.tick(raw=raw[t], valid=valid[t])
        x, P = e.get_state()
    idx = _sample(n, seed=2)
    cfg = fmskf.default_config("ekf9", idx.size)
    prm = orc.ekf9_params(cfg.dt, np.array(cfg.q[:45]), np.array(cfg.r[:21]), orc.TRIG_TABLE512)
    xo = np.zeros((10, idx.size), np.float32)  # row 9: the heading's low part
    Po = np.repeat(np.float32(np.array(cfg.p0[:45]))[:, None], idx.size, 1).copy()
    for t in range(T):
        orc.ekf9_tick(xo, Po, np.ascontiguousarray(raw[t][idx]), np.ascontiguousarray(valid[t][idx]),
                      prm, nthreads=0)
    np.testing.assert_array_equal(x[:, idx].view(np.uint32), xo[:9].view(np.uint32))
    np.testing.assert_array_equal(P[:, idx].view(np.uint32), Po.view(np.uint32))


def test_rs_2p20_sampled(orc):
    from fmskf.synth import Trajectory
    n, T = 1 << 20, 5
    tr = Trajectory(n, T, seed=13)
    yaw, sums, rpm = tr.rs_inputs()
    with Engine("rs", n) as e:
        for t in range(T):
            e.tick(yaw_deg=yaw[t], angle_sum=sums[t], rpm=rpm[t])
        pose = e.get_pose()
        prev = e.get_prev_sum()
    idx = _sample(n, seed=3)
    pos = np.zeros((3, idx.size), np.float32)
    vel = np.zeros((3, idx.size), np.float32)
    pv = np.zeros((4, idx.size), np.int64)
    for t in range(T):
        orc.rs_tick(pos, vel, pv, np.ascontiguousarray(yaw[t][idx]),
                    np.ascontiguousarray(sums[t][:, idx]), np.ascontiguousarray(rpm[t][idx]))
    np.testing.assert_array_equal(np.stack(pose)[:, idx].view(np.uint32), pos.view(np.uint32))
    np.testing.assert_array_equal(prev[:, idx], pv)


@pytest.mark.parametrize("n", [1 << 18, 1 << 20])
def test_kf12d_sampled(orc, n):
    """KF12D sampled against the oracle; 2^20 is cfg 5's size (non-temporal state stream)."""
    from fmskf.synth import Trajectory
    T = 4
    tr = Trajectory(n, T, seed=14)
    z = tr.kf12d_z()
    with Engine("kf12d", n) as e:
        for t in range(T):
            e.tick(z=z[t])
        x, P = e.get_state()
    idx = _sample(n, seed=4)
    cfg = fmskf.default_config("kf12d", idx.size)
    prm = orc.kf12d_params(cfg.dt, np.array(cfg.q[:78]), np.array(cfg.r[:36]))
    xo = np.zeros((12, idx.size))
    Po = np.repeat(np.array(cfg.p0[:78])[:, None], idx.size, 1).copy()
    for t in range(T):
        orc.kf12d_tick(xo, Po, np.ascontiguousarray(z[t][:, idx]), None, prm, nthreads=0)
    scale = np.maximum(np.abs(xo).max(axis=1, keepdims=True), 1e-3)
    assert (np.abs(x[:, idx] - xo) / scale).max() <= 1e-12
    assert (np.abs(P[:, idx] - Po) / max(np.abs(Po).max(), 1e-3)).max() <= 1e-12


def test_kf6_records_and_planes_past_2p28(orc):
    """N = 2^28 + 777 KF6 robots (29 GB of state; feasible because the ingest state is only
    allocated on first use): record and plane inputs are addressed from each block's first
    robot, so no 32-bit lane offset wraps (robot i's record sits at i * 16 B > 4 GiB here).
    Both input forms give the same pose bit for bit; a sample matches the oracle."""
    import torch
    from fmskf.synth import kf6_ring_torch
    n, T = (1 << 28) + 777, 2
    yaw, gz, rpm = kf6_ring_torch(n, T, seed=5, device="cuda")
    rec = fmskf.kf6_records(yaw, gz, rpm)
    assert rec.numel() * 4 > 0xFFFFFFFF
    with Engine("kf6", n) as e:
        for t in range(T):
            e.tick(kf6_rec=rec[t])
        pose_rec = e.get_pose()
        assert e.get_counters()[0] == 0
        e.reset()
        del rec
        for t in range(T):
            e.tick(yaw_deg=yaw[t], gyro_z_dps=gz[t], rpm=rpm[t])
        pose_pl = e.get_pose()
    np.testing.assert_array_equal(pose_rec.view(np.uint32), pose_pl.view(np.uint32))
    idx = _sample(n, seed=3)
    ys, gs, rs = (a[:, torch.from_numpy(idx).cuda()].cpu().numpy() for a in (yaw, gz, rpm))
    cfg = fmskf.default_config("kf6", idx.size)
    prm = orc.kf6_params(cfg.dt, np.array(cfg.q[:21]), np.array(cfg.r[:10]))
    xo = np.zeros((6, idx.size), np.float32)
    Po = np.repeat(np.float32(np.array(cfg.p0[:21]))[:, None], idx.size, 1).copy()
    for t in range(T):
        orc.kf6_tick(xo, Po, np.ascontiguousarray(ys[t]), np.ascontiguousarray(gs[t]),
                     np.ascontiguousarray(rs[t]), None, prm, nthreads=0)
    np.testing.assert_array_equal(pose_rec[:, idx].view(np.uint32), xo[:3].view(np.uint32))


def _wt901_polls(n, stride, rng):
    """One poll per robot at the benchmark shape (44 B = four frames 0x51 acc,
    0x52 gyro, 0x53 angle, 0x59 quaternion per 10 ms), built vectorised: 60% clean, 15% with one
    byte damaged (a checksum failure and the resync of wit_c_sdk.c:142-156), 15% torn (the tail
    carried into the next poll), 10% noise with 0x55 sprinkled in."""
    fr = np.zeros((n, 4, 11), np.uint8)
    fr[:, :, 0] = 0x55
    fr[:, :, 1] = np.array([0x51, 0x52, 0x53, 0x59], np.uint8)
    fr[:, :, 2:10] = rng.integers(0, 256, (n, 4, 8), dtype=np.uint8)
    fr[:, :, 10] = (fr[:, :, :10].sum(axis=2, dtype=np.uint32) & 0xFF).astype(np.uint8)
    buf = np.zeros((n, stride), np.uint8)
    buf[:, :44] = fr.reshape(n, 44)
    lens = np.full(n, 44, np.uint32)
    kind = rng.choice(4, n, p=[0.6, 0.15, 0.15, 0.1])
    d = np.flatnonzero(kind == 1)
    buf[d, rng.integers(0, 44, d.size)] ^= 0xA5
    t = np.flatnonzero(kind == 2)
    lens[t] = rng.integers(0, 44, t.size)
    z = np.flatnonzero(kind == 3)
    noise = rng.integers(0, 256, (z.size, stride), dtype=np.uint8)
    noise[rng.random(noise.shape) < 0.2] = 0x55
    buf[z] = noise
    lens[z] = rng.integers(0, stride + 1, z.size)
    return buf, lens


def test_wt901_ingest_2p20_sampled(orc):
    """The batched WT901 decoder at the benchmark size, 2^20 robots x 4 polls
    of mixed clean / damaged / torn / noisy bytes at the 48-byte stride: register file, parser
    backlog, error flag and the scaled Data page of a sample bit for bit against the oracle's
    restatement of wit_c_sdk.c:90-198 and imu_if_wt901c.cpp:91-143."""
    n, polls, stride = 1 << 20, 4, 48
    rng = np.random.default_rng(2024)
    idx = _sample(n, k=1024, seed=4)
    orcs = [orc.Wt901(0x51) for _ in idx]
    with Engine("kf6", n) as e:
        for k in range(polls):
            buf, lens = _wt901_polls(n, stride, rng)
            e.ingest_wt901(buf, lens, latch_qinit=(k == 0))
            for o, i in zip(orcs, idx):
                o.update(buf[i, :lens[i]], latch_qinit=(k == 0))
        regs, pending = e.get_imu_regs()
        data, err = e.get_imu()
    for o, i in zip(orcs, idx):
        np.testing.assert_array_equal(regs[:, i], o.regs, err_msg=f"robot {i}")
        assert pending[i] == len(o.parser) and err[i] == o.is_error, f"robot {i}"
        np.testing.assert_array_equal(data[:, i].view(np.uint32), o.data.view(np.uint32),
                                      err_msg=f"robot {i}")


@pytest.mark.parametrize("n,masked", [(1 << 22, False), (1 << 20, True)])
def test_can_ingest_large_sampled(orc, n, masked):
    """C610 RX decode (VD_motor_if_m2006.cpp:32-72) at bench sizes: 2^22 robots takes the
    robot-per-lane kernel with the non-temporal state, 2^20 with `present` masks the wheel-per-lane
    kernel; a sample of robots bit for bit (angle, rpm, current, the int64 angle sum, the speed
    IIR) after 4 ticks with out-of-range angles and equal stamps (ARM x/0 -> 0)."""
    T = 4
    rng = np.random.default_rng(77 + masked)
    dirs = [1, 1, -1, -1]
    idx = _sample(n, k=1024, seed=5)
    motors = [[orc.M2006(d) for d in dirs] for _ in idx]
    with Engine("rs", n) as e:
        for t in range(T):
            frames = rng.integers(0, 256, (n, 4, 8), dtype=np.uint8)
            frames[:, :, 0] &= 0x1F
            frames[rng.random((n, 4)) < 0.05, 0] |= 0x80
            stamps = rng.integers(0, 0x8000, (n, 4)).astype(np.int16)
            stamps[rng.random((n, 4)) < 0.05] = 1234
            present = rng.integers(0, 16, n).astype(np.uint8) if masked else None
            e.ingest_can(frames, stamps, present)
            for m, i in zip(motors, idx):
                for w in range(4):
                    if present is None or (present[i] >> w) & 1:
                        m[w].rx(frames[i, w], int(stamps[i, w]))
        got = e.get_motors()
    for m, i in zip(motors, idx):
        for w in range(4):
            s = m[w].s
            assert (got["angle"][i, w], got["rpm"][i, w], got["curr"][i, w], got["angle_sum"][w, i]) == \
                (s.angle, s.rpm, s.curr, s.angle_sum), f"robot {i} wheel {w}"
            assert got["speed_radps"][w, i].view(np.uint32) == np.float32(s.speed_radps).view(np.uint32)
