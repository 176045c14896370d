"""Host-resident inputs and outputs of up to 1 MiB per call go through the handle's pinned slots
(api_ctx.hpp `Stager`, api_handle.cpp `copy_out_sync`): by default the kernels read the
packed inputs and write their host-bound frames in place over PCIe.  The boundary's contract
(caller-owned pointers, no retention after return) must hold whatever the
staging: a caller may overwrite its host buffer as soon as a call returns, and asynchronous
ticks may queue far ahead of the GPU without a slot being rewritten under a kernel that still
reads it.  Every result bit-exact against the oracle."""
import numpy as np
import pytest

from fmskf import Engine
from fmskf.synth import Trajectory
from test_gpu_parity import _kf6_oracle, bits_equal

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [777, 65536, 65537])  # 65536: exactly the 1 MiB slot; 65537: past it
def test_async_ticks_reuse_one_host_buffer(orc, n):
    """40 asynchronous ticks fed from ONE host buffer, rewritten right after each call returns
    (no synchronisation in between), then the wheel loops and frames of a final ISR tick."""
    T = 40
    tr = Trajectory(n, T, seed=91)
    yaw, gz, rpm = tr.kf6_inputs()
    by = np.empty(n, np.float32)
    bg = np.empty(n, np.float32)
    br = np.empty((n, 4), np.int16)
    with Engine("kf6", n) as e:
        for t in range(T):
            by[:], bg[:], br[:] = yaw[t], gz[t], rpm[t]
            e.tick(yaw_deg=by, gyro_z_dps=bg, rpm=br)
            by[:], bg[:], br[:] = 1e30, -1e30, 32767  # the caller reuses its buffer at once
        x, P = e.get_state()
    xo, Po = _kf6_oracle(orc, n, yaw, gz, rpm, None, orc.TRIG_TABLE512, T)
    bits_equal(x, xo, "x")
    bits_equal(P, Po, "P")


def test_isr_host_frames_match_three_calls_device():
    """fmskf_isr_tick with host inputs and host frames (the pinned output slot) against the
    same ticks fed from device buffers into device frames, for the KF6 and RS models."""
    import torch
    n, T = 4099, 25
    tr = Trajectory(n, T, seed=92)
    yaw, gz, rpm = tr.kf6_inputs()
    vel = np.zeros((3, n), np.float32)
    vel[0] = 120.0
    acl = np.full((3, n), 1000.0, np.float32)
    jrk = np.full((3, n), 10000.0, np.float32)
    for model in ("kf6", "rs"):
        if model == "kf6":
            kw = {"yaw_deg": yaw, "gyro_z_dps": gz, "rpm": rpm}
        else:
            ry, rs, rr = tr.rs_inputs()
            kw = {"yaw_deg": ry, "angle_sum": rs, "rpm": rr}
        with Engine(model, n) as a, Engine(model, n) as b:
            for e in (a, b):
                e.set_power(None)
                e.set_target_vel(vel, acl, jrk)
            dev = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in kw.items()}
            out = torch.empty((n, 8), dtype=torch.uint8, device="cuda")
            for t in range(T):
                fa = a.isr_tick(**{k: v[t] for k, v in kw.items()})
                b.isr_tick(out=out, **{k: v[t] for k, v in dev.items()})
                np.testing.assert_array_equal(fa, out.cpu().numpy(), err_msg=f"{model} tick {t}")
            xa, xb = a.get_state()[0], b.get_state()[0]
            np.testing.assert_array_equal(xa.view(np.uint32), xb.view(np.uint32))

