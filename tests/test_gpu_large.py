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


def test_control_past_the_buffer_window(orc):
    import torch
    n, T = 46_000_000, 40         # pitch * 4 B * 24 FF_PI_D planes > 4 GiB
    assert fmskf_pitch(n) * 4 * 24 > 0xFFFFFFFF
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
