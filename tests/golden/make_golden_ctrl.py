"""Generate tests/golden/ctrl_ref.npz from the REFERENCE's own motor speed controller.

Runs UTIL::FF_PI_D (src/Utility/util_controller.hpp with the UTIL::IIR1 velocity LPF of
util_iir.hpp; compiled unmodified from /root/reference by oracle/Makefile into
oracle/_ref/libctrl_ref.so) over seeded set_target / update / reset sequences and records
what it returns after every step: the control output, get_now_val() and get_target().

Sequences cover the firmware's construction (VD_task_main.cpp:86-89,157-160: 100 Hz, FF
0.0075, P 0.02, I 0.01, D 0, I-limit 0.5, LPF 10 Hz, FF limit 1), random gains with a
nonzero D term, integrator and feed-forward saturation, and resets mid-sequence.

Run only where /root/reference exists:  python tests/golden/make_golden_ctrl.py
The output is data (inputs and expected outputs), committed; nothing of the reference
travels with it.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle  # noqa: E402

OUT = os.path.join(HERE, "ctrl_ref.npz")
STEPS = 400
FIRMWARE = dict(c_freq=100.0, ff=0.0075, pg=0.02, ig=0.01, dg=0.0, ilim=0.5, lpf=10.0, fflim=1.0)
KEYS = list(FIRMWARE)


def sequences(rng):
    seqs = []
    # 1. firmware gains, a motor-speed step response (motor rad/s x 36, as VEHICLE_CTRL feeds)
    t = np.zeros(STEPS, np.float32)
    t[20:] = 300.0
    v = np.float32(300.0) * (1 - np.exp(-np.arange(STEPS, dtype=np.float32) / 40.0)).astype(np.float32)
    seqs.append(("firmware_step", dict(FIRMWARE), t, v, None))
    # 2. firmware gains, noisy tracking with resets (power off/on)
    t = (rng.normal(0, 400, STEPS)).astype(np.float32)
    v = (t + rng.normal(0, 30, STEPS)).astype(np.float32)
    rs = (rng.random(STEPS) < 0.02).astype(np.uint8)
    seqs.append(("firmware_noisy_resets", dict(FIRMWARE), t, v, rs))
    # 3. integrator saturation: large persistent error
    t = np.full(STEPS, 2000.0, np.float32)
    v = np.zeros(STEPS, np.float32)
    seqs.append(("integrator_saturates", dict(FIRMWARE), t, v, None))
    # 4. negative saturation of FF and I
    seqs.append(("negative_saturation", dict(FIRMWARE), -t, v, None))
    # 5-10. random gains incl. a D term (the LPF path), random limits
    for k in range(6):
        g = dict(c_freq=float(rng.choice([100.0, 1000.0, 250.0])), ff=float(rng.uniform(0, 0.02)),
                 pg=float(rng.uniform(0, 0.1)), ig=float(rng.uniform(0, 0.5)),
                 dg=float(rng.uniform(0, 0.01)), ilim=float(rng.uniform(0.05, 2.0)),
                 lpf=float(rng.uniform(1.0, 50.0)), fflim=float(rng.uniform(0.1, 2.0)))
        t = np.repeat(rng.normal(0, 500, STEPS // 20), 20).astype(np.float32)
        v = (np.convolve(t, np.ones(15) / 15, mode="same") + rng.normal(0, 10, STEPS)).astype(np.float32)
        rs = (rng.random(STEPS) < 0.01).astype(np.uint8) if k % 2 else None
        seqs.append((f"random_gains_{k}", g, t, v, rs))
    return seqs


def main():
    oracle.build()
    rng = np.random.default_rng(0x464D534B)
    names, gains, tgt, val, rst, ctrl, now_val, target = [], [], [], [], [], [], [], []
    for name, g, t, v, rs in sequences(rng):
        c, nv, tg = oracle.RefFfPiD.run(t, v, rs, **g)
        names.append(name)
        gains.append([g[k] for k in KEYS])
        tgt.append(t)
        val.append(v)
        rst.append(np.zeros(STEPS, np.uint8) if rs is None else rs)
        ctrl.append(c)
        now_val.append(nv)
        target.append(tg)
    np.savez_compressed(OUT, name=np.array(names), gain_keys=np.array(KEYS),
                        gains=np.array(gains, np.float32), tgt=np.stack(tgt), val=np.stack(val),
                        reset=np.stack(rst), ctrl=np.stack(ctrl), now_val=np.stack(now_val),
                        target=np.stack(target))
    print(f"wrote {OUT}: {len(names)} sequences x {STEPS} steps")


if __name__ == "__main__":
    main()
