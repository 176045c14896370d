"""Freeze the oracle's answers for the rows the reference build cannot pin.

The reference sources of these rows -- imu_if_wt901c.cpp:91-143 (A3/A4: validity flag, Data
page scaling, axis flips, q_init product), VD_motor_if_m2006.cpp:32-72 (A8: C610 frame decode,
angle unwrap, int64 angle sum, speed IIR) and VD_vehicle_controller.cpp:36-51 with
util_mymath.hpp:18-25 (A9-A12: the odometry integrator and heading normalisation) -- include
global_config.hpp:4, which pulls in Arduino.h; the image has no Arduino / CMSIS-DSP headers, so
they stay "parity unpinned" against the firmware.  What this script pins is the restatement
itself: tests/golden/oracle_frozen.npz holds seeded inputs and the oracle's outputs, so a
later edit of oracle/fmskf_oracle.c that changes any of these answers fails
tests/test_oracle_frozen.py, and the GPU tests check the library against the same data.

  python tests/golden/make_golden_oracle.py      (CPU only; ~1 minute)
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "roboken-fmskf-robot-controller_amd"), os.path.dirname(HERE)):
    sys.path.insert(0, p)

from oracle import oracle as orc  # noqa: E402
from fmskf.synth import wt901_frame  # noqa: E402
import cfg1_trace  # noqa: E402

OUT = os.path.join(HERE, "oracle_frozen.npz")


def imu_streams(n=48, polls=12, stride=64, seed=2024):
    """Mixed clean / torn / noisy / damaged WT901 polls (A1-A4 through the Data page)."""
    rng = np.random.default_rng(seed)
    buf = np.zeros((polls, n, stride), np.uint8)
    lens = np.zeros((polls, n), np.uint32)
    for k in range(polls):
        for i in range(n):
            kind = int(rng.integers(0, 4))
            if kind == 0:
                b = b"".join(wt901_frame(t, rng.integers(0, 65536, 4)) for t in (0x51, 0x52, 0x53, 0x59))
            elif kind == 1:
                ts = rng.choice([0x50, 0x51, 0x52, 0x53, 0x54, 0x59, 0x5A, 0x5F], int(rng.integers(0, 6)))
                b = b"".join(wt901_frame(int(t), rng.integers(0, 65536, 4)) for t in ts)
                if rng.random() < 0.4:
                    b = b[:int(rng.integers(0, len(b) + 1))]
            elif kind == 2:
                a = rng.integers(0, 256, int(rng.integers(0, stride + 1)), dtype=np.uint8)
                a[rng.random(a.size) < 0.2] = 0x55
                b = a.tobytes()
            else:
                fr = [bytearray(wt901_frame(int(rng.choice([0x51, 0x59, 0x53])), rng.integers(0, 65536, 4)))
                      for _ in range(5)]
                for f in fr:
                    if rng.random() < 0.3:
                        f[int(rng.integers(0, 11))] ^= 0x5A
                b = bytes(b"".join(fr))
            b = np.frombuffer(b, np.uint8)[:stride]
            buf[k, i, :b.size] = b
            lens[k, i] = b.size
    return buf, lens


def imu_answers(buf, lens):
    P, n, _ = buf.shape
    imus = [orc.Wt901(0x51) for _ in range(n)]
    data = np.zeros((P, 16, n), np.float32)
    err = np.zeros((P, n), np.uint8)
    for k in range(P):
        for i in range(n):
            imus[i].update(buf[k, i, :lens[k, i]], latch_qinit=(k == 0))
            data[k, :, i] = imus[i].data
            err[k, i] = imus[i].is_error
    return data, err


def can_streams(n=64, T=30, seed=610):
    rng = np.random.default_rng(seed)
    frames = rng.integers(0, 256, (T, n, 4, 8), dtype=np.uint8)
    frames[..., 0] &= 0x1F
    frames[rng.random((T, n, 4)) < 0.05, 0] |= 0x80
    stamps = rng.integers(0, 0x8000, (T, n, 4)).astype(np.int16)
    stamps[rng.random((T, n, 4)) < 0.05] = 777
    present = rng.integers(0, 16, (T, n)).astype(np.uint8)
    present[0] = 15
    return frames, stamps, present


def can_answers(frames, stamps, present):
    T, n = present.shape
    mot = [[orc.M2006(d) for d in (1, 1, -1, -1)] for _ in range(n)]
    out = {k: np.zeros((T, n, 4), np.int16) for k in ("angle", "rpm", "curr")}
    out["angle_sum"] = np.zeros((T, 4, n), np.int64)
    out["speed"] = np.zeros((T, 4, n), np.float32)
    for t in range(T):
        for i in range(n):
            for w in range(4):
                if (present[t, i] >> w) & 1:
                    mot[i][w].rx(frames[t, i, w], int(stamps[t, i, w]))
                s = mot[i][w].s
                out["angle"][t, i, w] = s.angle
                out["rpm"][t, i, w] = s.rpm
                out["curr"][t, i, w] = s.curr
                out["angle_sum"][t, w, i] = s.angle_sum
                out["speed"][t, w, i] = s.speed_radps
    return out


def main():
    orc.build()
    res = {}
    inp = cfg1_trace.Cfg1Inputs()
    res["cfg1_digest"] = np.array(inp.digest)
    for model in ("rs", "kf6"):
        s, extra = cfg1_trace.run_oracle(orc, inp, model)
        res[f"cfg1_{model}_samples"] = s
        for k, v in extra.items():
            res[f"cfg1_{model}_{k}"] = v
    buf, lens = imu_streams()
    data, err = imu_answers(buf, lens)
    res.update(imu_bytes=buf, imu_lens=lens, imu_data=data, imu_err=err)
    frames, stamps, present = can_streams()
    res.update(can_frames=frames, can_stamps=stamps, can_present=present)
    for k, v in can_answers(frames, stamps, present).items():
        res[f"can_{k}"] = v
    np.savez_compressed(OUT, **res)
    print(f"wrote {OUT}: {os.path.getsize(OUT)} bytes; cfg1 digest {inp.digest[:16]}")


if __name__ == "__main__":
    main()
