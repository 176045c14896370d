"""Independent handles (threading row): each handle owns its state and stream,
one handle per host thread, distinct handles independent.  Two handles ticked interleaved on
two HIP streams with device-resident inputs (no host synchronisation between their launches),
and four host threads driving a handle each through the C ABI at once (ctypes drops the GIL
for the call), every result bit-exact against the oracle."""
import threading

import numpy as np
import pytest
import torch

import fmskf
from fmskf import Engine
from fmskf.synth import Trajectory
from test_gpu_parity import _kf6_oracle, bits_equal

pytestmark = pytest.mark.gpu


def _ekf9_oracle(orc, n, raw):
    cfg = fmskf.default_config("ekf9", n)
    prm = orc.ekf9_params(cfg.dt, np.array(cfg.q[:45]), np.array(cfg.r[:21]), orc.TRIG_TABLE512)
    x = np.zeros((10, n), np.float32)  # row 9: the heading's low part
    P = np.repeat(np.float32(np.array(cfg.p0[:45]))[:, None], n, 1).copy()
    for t in range(raw.shape[0]):
        orc.ekf9_tick(x, P, raw[t], None, prm, nthreads=0)
    return np.ascontiguousarray(x[:9]), P


def test_two_handles_two_streams_interleaved(orc):
    na, nb, T = 70001, 5003, 12
    ta, tb = Trajectory(na, T, seed=61), Trajectory(nb, T, seed=62)
    yaw, gz, rpm = ta.kf6_inputs()
    raw = tb.ekf9_raw()
    dev = torch.device("cuda", 0)
    dy, dg, dr = (torch.from_numpy(v).to(dev) for v in (yaw, gz, rpm))
    draw = torch.from_numpy(raw).to(dev)
    torch.cuda.synchronize()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    with Engine("kf6", na) as a, Engine("ekf9", nb) as b:
        a.set_stream(sa)
        b.set_stream(sb)
        for t in range(T):  # launches alternate between the two streams, nothing waits
            a.tick(yaw_deg=dy[t], gyro_z_dps=dg[t], rpm=dr[t])
            b.tick(raw=draw[t])
        xa, Pa = a.get_state()
        xb, Pb = b.get_state()
    xo, Po = _kf6_oracle(orc, na, yaw, gz, rpm, None, orc.TRIG_TABLE512, T)
    bits_equal(xa, xo, "kf6 x")
    bits_equal(Pa, Po, "kf6 P")
    xo, Po = _ekf9_oracle(orc, nb, raw)
    bits_equal(xb, xo, "ekf9 x")
    bits_equal(Pb, Po, "ekf9 P")


def test_one_handle_per_host_thread(orc):
    T = 10
    sizes = [4099, 20011, 777, 65536]
    trajs = [Trajectory(n, T, seed=70 + k) for k, n in enumerate(sizes)]
    inputs = [tr.kf6_inputs() for tr in trajs]
    results = [None] * len(sizes)
    errors = []
    start = threading.Barrier(len(sizes))

    def worker(k):
        try:
            torch.cuda.set_device(0)
            with Engine("kf6", sizes[k]) as e:
                e.set_stream(torch.cuda.Stream())
                yaw, gz, rpm = inputs[k]
                start.wait()
                for t in range(T):  # host inputs: each call stages them on the handle's stream
                    e.tick(yaw_deg=yaw[t], gyro_z_dps=gz[t], rpm=rpm[t])
                results[k] = e.get_state()
        except Exception as ex:  # noqa: BLE001 -- reported by the main thread
            errors.append((k, repr(ex)))

    threads = [threading.Thread(target=worker, args=(k,)) for k in range(len(sizes))]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    assert not any(th.is_alive() for th in threads), "a handle thread did not finish"
    assert not errors, errors
    for k, n in enumerate(sizes):
        yaw, gz, rpm = inputs[k]
        xo, Po = _kf6_oracle(orc, n, yaw, gz, rpm, None, orc.TRIG_TABLE512, T)
        bits_equal(results[k][0], xo, f"thread {k} x")
        bits_equal(results[k][1], Po, f"thread {k} P")
