"""Generate tests/golden/wt901_ref.npz from the REFERENCE's own WT901 SDK.

Runs lib/wt901c/wit_c_sdk.c (compiled unmodified from /root/reference by
oracle/Makefile into oracle/_ref/libwit_ref.so) over seeded byte streams and
records, after every poll, the full register file sReg[0x90] and the sequence
of register-update callbacks (reg, count) the SDK fired.  Those callbacks are
what IMU_IF_WT901C's SensorDataUpdata turns into update flags
(src/Imu/imu_if_wt901c.cpp:23-48), so the fixture pins the parser (A1), the
register file (A2) and the flag inputs of A3.

Run only where /root/reference exists:  python tests/golden/make_golden_wt901.py
The output is data (inputs and expected outputs), committed; nothing of the
reference travels with it.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "roboken-fmskf-robot-controller_amd"))

from oracle import oracle  # noqa: E402
from fmskf.synth import wt901_frame  # noqa: E402

OUT = os.path.join(HERE, "wt901_ref.npz")
TYPES_STD = [0x51, 0x52, 0x53, 0x59]
TYPES_ALL = [0x50, 0x51, 0x52, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5A, 0x5F]
TYPES_UNKNOWN = [0x00, 0x4F, 0x5B, 0x5C, 0x5E, 0x60, 0xFF]


def rwords(rng):
    return rng.integers(0, 65536, 4)


def frame(rng, t):
    return wt901_frame(t, rwords(rng))


def corrupt(rng, fr: bytes) -> bytes:
    b = bytearray(fr)
    k = int(rng.integers(1, 11))
    b[k] = (b[k] + int(rng.integers(1, 256))) & 0xFF
    return bytes(b)


def scenario(rng, kind: str):
    """Returns a list of polls (bytes each)."""
    polls = []
    if kind == "standard":
        for _ in range(8):
            polls.append(b"".join(frame(rng, t) for t in TYPES_STD))
    elif kind == "all_types":
        for _ in range(8):
            ts = rng.choice(TYPES_ALL + TYPES_UNKNOWN, size=int(rng.integers(1, 7)))
            polls.append(b"".join(frame(rng, int(t)) for t in ts))
    elif kind == "garbage_between":
        for _ in range(8):
            p = b""
            for t in TYPES_STD:
                g = rng.integers(0, 256, int(rng.integers(0, 6)), dtype=np.uint8)
                g[rng.random(g.size) < 0.3] = 0x55
                p += bytes(g) + frame(rng, t)
            polls.append(p)
    elif kind == "bad_checksum":
        for _ in range(8):
            p = b""
            for t in TYPES_STD:
                fr = frame(rng, t)
                p += corrupt(rng, fr) if rng.random() < 0.4 else fr
            polls.append(p)
    elif kind == "split":
        stream = b"".join(frame(rng, int(rng.choice(TYPES_STD))) for _ in range(40))
        cuts = np.sort(rng.choice(np.arange(1, len(stream)), size=12, replace=False))
        prev = 0
        for c in list(cuts) + [len(stream)]:
            polls.append(stream[prev:c])
            prev = c
    elif kind == "random":
        for _ in range(8):
            g = rng.integers(0, 256, int(rng.integers(0, 120)), dtype=np.uint8)
            g[rng.random(g.size) < 0.15] = 0x55
            polls.append(bytes(g))
    elif kind == "partial_and_empty":
        fr = [frame(rng, t) for t in TYPES_STD]
        polls = [b"", fr[0][:5], fr[0][5:] + fr[1], b"", fr[2] + fr[3][:10], fr[3][10:], b"",
                 b"\x55" * 13, fr[0]]
    elif kind == "resync_lag":
        # a checksum failure leaves 10 bytes in the window that drain one per arrival
        fr = [frame(rng, t) for t in TYPES_STD]
        polls = [corrupt(rng, fr[0]) + fr[1], fr[2] + fr[3], b"\x55" + fr[3], fr[3] + fr[0]]
    else:
        raise ValueError(kind)
    return polls


KINDS = ["standard", "all_types", "garbage_between", "bad_checksum", "split", "random",
         "partial_and_empty", "resync_lag"]
RRIS = [0x51, 0x00, 0x34, 0x8C]


def main():
    oracle.build()
    rng = np.random.default_rng(0x57543901)
    rri_l, npolls, plen, allb, regs, cb_reg, cb_num, cb_cnt, kinds = [], [], [], [], [], [], [], [], []
    for rep in range(3):
        for kind in KINDS:
            rri = RRIS[(rep + len(kinds)) % len(RRIS)] if kind in ("all_types", "random") else 0x51
            polls = scenario(rng, kind)
            ref = oracle.RefWt901(rri)
            rri_l.append(rri)
            npolls.append(len(polls))
            kinds.append(kind)
            for p in polls:
                ref.feed(p)
                plen.append(len(p))
                allb.append(np.frombuffer(p, np.uint8))
                regs.append(ref.regs())
                cbs = ref.take_cb()
                cb_cnt.append(len(cbs))
                cb_reg += [c[0] for c in cbs]
                cb_num += [c[1] for c in cbs]
    np.savez_compressed(
        OUT,
        read_reg_index=np.array(rri_l, np.uint32),
        n_polls=np.array(npolls, np.uint32),
        poll_len=np.array(plen, np.uint32),
        bytes=np.concatenate(allb).astype(np.uint8),
        regs=np.stack(regs).astype(np.int16),
        cb_count=np.array(cb_cnt, np.uint32),
        cb_reg=np.array(cb_reg, np.uint16),
        cb_num=np.array(cb_num, np.uint16),
        kind=np.array(kinds),
    )
    print(f"wrote {OUT}: {len(npolls)} streams, {len(plen)} polls, {sum(plen)} bytes, "
          f"{len(cb_reg)} callbacks")


if __name__ == "__main__":
    main()
