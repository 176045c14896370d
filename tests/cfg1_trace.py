"""BASELINE.json configs[0] / SURVEY.md 8(d) cfg 1: one robot, 60 000 ticks (60 s of the 1 kHz
ISR), fed the way the firmware feeds it -- four C610 CAN frames every tick
(MOTOR_IF_M2006::rx_callback, VD_motor_if_m2006.cpp:32-72), a 44-byte WT901 poll every 10
ticks (IMT::main, imu_task_main.cpp:43-82, 100 Hz) and the tick reading both from the
ingested state (VDT::can_tx_routine_intr, VD_task_main.cpp:366-372: correct, then predict).

The same loop runs through the oracle (CPU) and through the library (the device-resident
path: tick inputs left NULL), for the RS model (the reference's integrator) and the KF6
filter.  The headings wrap ~10 times in 60 s, so normalize_rad_0to2pi (util_mymath.hpp:18-25)
and the KF heading wrap run on every branch.  tests/golden/make_golden_oracle.py freezes the
oracle's trajectory (sampled every 100 ticks) in tests/golden/oracle_frozen.npz.
"""
from __future__ import annotations

import hashlib

import numpy as np

T_CFG1 = 60000
SAMPLE_EVERY = 100
SEED_CFG1 = 0x464D534B ^ 1  # seed "FMSK" xor config id


class Cfg1Inputs:
    """Pre-built per-tick device traffic of the cfg 1 trace (frames, stamps, polls)."""

    def __init__(self, ticks: int = T_CFG1):
        from fmskf.synth import Trajectory
        tr = Trajectory(1, ticks, seed=SEED_CFG1)
        self.ticks = ticks
        self.frames = []
        self.stamps = []
        self.polls = {}
        h = hashlib.sha256()
        for t in range(ticks):
            fr, st = tr.can_frames(t)
            self.frames.append(np.ascontiguousarray(fr))
            self.stamps.append(np.ascontiguousarray(st))
            h.update(fr.tobytes())
            h.update(st.tobytes())
            if t % 10 == 0:
                b = tr.wt901_poll_bytes(t, 0)
                self.polls[t] = b
                h.update(b)
        self.digest = h.hexdigest()


def run_oracle(orc, inp: Cfg1Inputs, model: str):
    """The firmware loop through the oracle.  Returns (samples [S, 6] f32, extra dict)."""
    import fmskf
    imu = orc.Wt901(0x51)
    mot = [orc.M2006(d) for d in (1, 1, -1, -1)]
    samples = []
    if model == "rs":
        pos = np.zeros((3, 1), np.float32)
        vel = np.zeros((3, 1), np.float32)
        prev = np.zeros((4, 1), np.int64)
    else:
        cfg = fmskf.default_config("kf6", 1)
        prm = orc.kf6_params(cfg.dt, np.array(cfg.q[:21]), np.array(cfg.r[:10]))
        x = np.zeros((6, 1), np.float32)
        P = np.float32(np.array(cfg.p0[:21]))[:, None].copy()
    for t in range(inp.ticks):
        fr, st = inp.frames[t], inp.stamps[t]
        for w in range(4):
            mot[w].rx(fr[0, w], int(st[0, w]))
        if t in inp.polls:
            imu.update(np.frombuffer(inp.polls[t], np.uint8), latch_qinit=(t == 0))
        d = imu.data
        rpm = np.array([[m.s.rpm for m in mot]], np.int16)
        if model == "rs":
            sums = np.array([[m.s.angle_sum] for m in mot], np.int64)
            orc.rs_tick(pos, vel, prev, np.float32([d[11]]), sums, rpm)
            state = np.concatenate([pos[:, 0], vel[:, 0]])
        else:
            orc.kf6_tick(x, P, np.float32([d[11]]), np.float32([d[5]]), rpm, None, prm)
            state = x[:, 0].copy()
        if t % SAMPLE_EVERY == SAMPLE_EVERY - 1:
            samples.append(state.copy())
    extra = {"prev": prev[:, 0].copy()} if model == "rs" else {"P": P[:, 0].copy()}
    return np.stack(samples).astype(np.float32), extra


def run_engine(inp: Cfg1Inputs, model: str):
    """The same loop through the library (C ABI), device-resident tick inputs."""
    from fmskf import Engine
    samples = []
    with Engine(model, 1) as e:
        for t in range(inp.ticks):
            e.ingest_can(inp.frames[t], inp.stamps[t])
            if t in inp.polls:
                b = np.frombuffer(inp.polls[t], np.uint8)
                buf = np.zeros((1, 48), np.uint8)
                buf[0, :b.size] = b
                e.ingest_wt901(buf, np.array([b.size], np.uint32), latch_qinit=(t == 0))
            e.tick()
            if t % SAMPLE_EVERY == SAMPLE_EVERY - 1:
                x, _ = e.get_state()
                samples.append(x[:, 0].copy())
        x, P = e.get_state()
        extra = {"prev": e.get_prev_sum()[:, 0].copy()} if model == "rs" else {"P": P[:, 0].copy()}
    return np.stack(samples).astype(np.float32), extra
