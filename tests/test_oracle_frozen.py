"""The frozen oracle answers (tests/golden/oracle_frozen.npz, made by
tests/golden/make_golden_oracle.py) against the oracle (CPU) and against the library (GPU).

Rows covered: A3/A4 (WT901 validity flag + Data page: scaling, flips, q_init product,
imu_if_wt901c.cpp:91-143), A8 (C610 decode, unwrap, int64 angle sum, speed IIR,
VD_motor_if_m2006.cpp:32-72) and the config 1 trace (one robot, 60 000 ticks, RS integrator and
KF6 fed from the ingested state; VD_vehicle_controller.cpp:36-51, util_mymath.hpp:18-25).
These rows are parity unpinned against the firmware (its sources include Arduino.h via
global_config.hpp:4); the fixture pins the restatement so it cannot drift silently, and the
GPU tests hold the library to the same bits.
"""
import os

import numpy as np
import pytest

import cfg1_trace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def frozen():
    d = np.load(os.path.join(ROOT, "tests", "golden", "oracle_frozen.npz"))
    return {k: d[k] for k in d.files}


@pytest.fixture(scope="module")
def cfg1_inputs(frozen):
    inp = cfg1_trace.Cfg1Inputs()
    assert inp.digest == str(frozen["cfg1_digest"]), \
        "cfg 1 input stream changed (fmskf.synth or numpy's generator): regenerate the fixture"
    return inp


def bits(a, b, what):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b).astype(a.dtype)
    if a.dtype.kind == "f":
        a = a.view(np.uint32 if a.dtype == np.float32 else np.uint64)
        b = b.view(a.dtype)
    bad = np.argwhere(a != b)
    assert bad.size == 0, f"{what}: {len(bad)} mismatches, first at {tuple(bad[0])}"


# ----------------------------------------------------------------------------- oracle (CPU)
@pytest.mark.parametrize("model", ["rs", "kf6"])
def test_oracle_cfg1_trace_frozen(orc, frozen, cfg1_inputs, model):
    s, extra = cfg1_trace.run_oracle(orc, cfg1_inputs, model)
    bits(s, frozen[f"cfg1_{model}_samples"], f"{model} trajectory")
    for k, v in extra.items():
        bits(v, frozen[f"cfg1_{model}_{k}"], f"{model} {k}")
    # the heading wraps through +-pi several times in the 60 s (the long-run normalisation path)
    th = s[:, 2]
    assert (np.abs(np.diff(th)) > 3.0).sum() >= 3


def test_oracle_imu_frozen(orc, frozen):
    from golden.make_golden_oracle import imu_answers
    data, err = imu_answers(frozen["imu_bytes"], frozen["imu_lens"])
    bits(data, frozen["imu_data"], "Data page")
    bits(err, frozen["imu_err"], "is_error")


def test_oracle_can_frozen(orc, frozen):
    from golden.make_golden_oracle import can_answers
    out = can_answers(frozen["can_frames"], frozen["can_stamps"], frozen["can_present"])
    for k, v in out.items():
        bits(v, frozen[f"can_{k}"], k)


# ----------------------------------------------------------------------------- library (GPU)
@pytest.mark.gpu
@pytest.mark.parametrize("model", ["rs", "kf6"])
def test_gpu_cfg1_trace_frozen(frozen, cfg1_inputs, model):
    """60 000 ticks of one robot through the C ABI, device-resident inputs, bit-exact against
    the frozen oracle trajectory every 100 ticks and in the final state."""
    s, extra = cfg1_trace.run_engine(cfg1_inputs, model)
    bits(s, frozen[f"cfg1_{model}_samples"], f"{model} trajectory")
    for k, v in extra.items():
        bits(v, frozen[f"cfg1_{model}_{k}"], f"{model} {k}")


@pytest.mark.gpu
def test_gpu_imu_frozen(frozen):
    from fmskf import Engine
    buf, lens = frozen["imu_bytes"], frozen["imu_lens"]
    P, n, _ = buf.shape
    with Engine("kf6", n) as e:
        for k in range(P):
            e.ingest_wt901(buf[k], lens[k], latch_qinit=(k == 0))
            data, err = e.get_imu()
            bits(data, frozen["imu_data"][k], f"Data page poll {k}")
            bits(err.astype(np.uint8), frozen["imu_err"][k], f"is_error poll {k}")


@pytest.mark.gpu
def test_gpu_can_frozen(frozen):
    from fmskf import Engine
    fr, st, pr = frozen["can_frames"], frozen["can_stamps"], frozen["can_present"]
    T, n = pr.shape
    with Engine("rs", n) as e:
        for t in range(T):
            e.ingest_can(fr[t], st[t], pr[t])
            m = e.get_motors()
            for k, key in (("angle", "angle"), ("rpm", "rpm"), ("curr", "curr"),
                           ("angle_sum", "angle_sum"), ("speed_radps", "speed")):
                bits(m[k], frozen[f"can_{key}"][t], f"{key} tick {t}")
