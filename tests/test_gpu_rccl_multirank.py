"""libfmskf's communicator at world > 1 on the one-GPU test box.

RCCL refuses two ranks on one GPU, so the ranks here load tests/native/loopback_rccl.cpp
through FMSKF_RCCL_LIBRARY: the same five entry points, the all-gather staged through a
directory.  What runs is the library's own multi-rank code -- result slots sized by world,
ncclAllGather of each rank's fused record on the side stream, the copy-out of `world`
records and their fold in rank order -- which the driver's 8-GPU run otherwise executes for
the first time.  Each rank (tests/native/rccl_rank_worker.py, one process per rank, no torch)
ticks its own shard and a twin handle without a communicator; every collected result must
equal fmskf_ensemble_combine of the twins' local records in rank order, bit for bit, on
every rank.  RCCL itself is exercised at world 1 in tests/test_gpu_rccl.py and by
bench.py at world N on the driver's node."""
import os
import subprocess
import sys

import numpy as np
import pytest

import fmskf

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LOOPBACK = os.path.join(ROOT, "build", "libloopback_rccl.so")
WORKER = os.path.join(ROOT, "tests", "native", "rccl_rank_worker.py")


def run_ranks(tmp_path, model, sizes, T, every, mode="sync"):
    assert os.path.exists(LOOPBACK), "build() makes build/libloopback_rccl.so"
    world = len(sizes)
    env = dict(os.environ, FMSKF_RCCL_LIBRARY=LOOPBACK, LOOPBACK_RCCL_DIR=str(tmp_path), LOOPBACK_RCCL_MODE=mode)
    id_file = str(tmp_path / "uid")
    procs = [subprocess.Popen([sys.executable, WORKER, model, str(r), str(world), str(n), str(T), str(every),
                               id_file, str(tmp_path / f"rank{r}.npz")], env=env)
             for r, n in enumerate(sizes)]
    try:
        rcs = [p.wait(timeout=150) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    assert rcs == [0] * world, rcs
    return [dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(world)]


@pytest.mark.parametrize("model,sizes,every,mode", [("kf6", [70001, 65536], 1, "sync"),
                                                    ("kf6", [1 << 20, 1000, 4097], 2, "sync"),
                                                    ("kf6", [70001, 65536, 3], 1, "callback"),
                                                    ("ekf9", [5001, 30000], 1, "sync"),
                                                    ("ekf9", [5001, 30000], 1, "callback"),
                                                    ("kf12d", [3001, 2000], 2, "sync"),
                                                    ("rs", [4097, 1023, 512], 1, "sync")])
def test_native_communicator_world_gt_1(tmp_path, model, sizes, every, mode):
    """mode "callback": the stand-in enqueues its exchange on the side stream as a host function
    between two asynchronous copies, so the library's ordering (gather behind the fold, the copy
    of the gathered records and the slot's event behind the gather) is exercised with no host
    wait inside ncclAllGather."""
    T = 7
    outs = run_ranks(tmp_path, model, sizes, T, every, mode)
    L = outs[0]["local"].shape[1]
    nx = next(k for k in range(1, 16) if 1 + k + k * (k + 1) // 2 == L)  # record {count, mean, M2}
    events = T // every
    for r, o in enumerate(outs):
        assert bool(o["same_state"]), f"rank {r}: the communicator changed the tick"
        assert o["got_mean"].shape[0] == events
        # the communicator's own size and rank (fmskf_comm_info: ncclCommCount / ncclCommUserRank)
        assert tuple(o["comm_info"]) == (len(sizes), r)
        # every gathered result counts the whole fleet, folded from `world` records
        assert o["counts"].shape == (events, 2)
        assert np.all(o["counts"][:, 0] == float(sum(sizes))) and np.all(o["counts"][:, 1] == len(sizes))
        assert str(o["rccl_library"]) == LOOPBACK
        # every collected result went through the side stream's exchange, and its time is known
        # (fmskf_ensemble_exchange_ms, the N > 1 bench line's scaling_diag.exchange_ms)
        assert o["exchange_ms"].shape == (events,) and np.all(o["exchange_ms"] >= 0.0), o["exchange_ms"]
    for k in range(events):
        want_m, want_c = fmskf.ensemble_combine(nx, np.stack([o["local"][k] for o in outs]))
        for r, o in enumerate(outs):
            np.testing.assert_array_equal(o["got_mean"][k], want_m, err_msg=f"rank {r} event {k}")
            np.testing.assert_array_equal(o["got_cov"][k], want_c, err_msg=f"rank {r} event {k}")
    assert outs[0]["got_mean"].shape == (events, nx)
    # the synchronous fmskf_ensemble_stats and a stand-alone asynchronous record of the final
    # state: the rank-order fold of every rank's stand-alone partial
    want_m, want_c = fmskf.ensemble_combine(nx, np.stack([o["final"] for o in outs]))
    for o in outs:
        for m, c in ((o["sync_mean"], o["sync_cov"]), (o["alone_mean"], o["alone_cov"])):
            np.testing.assert_array_equal(m, want_m)
            np.testing.assert_array_equal(c, want_c)
    assert float(np.stack([o["final"] for o in outs])[:, 0].sum()) == float(sum(sizes))


def test_fleet_loop_cpp_two_ranks(tmp_path):
    """examples/fleet_loop.cpp, the C++ caller, at world 2: rank 0 writes fmskf_comm_unique_id
    to FLEET_ID, both ranks fmskf_comm_init and collect fmskf_ensemble_begin / _end every 16
    ticks.  Both ranks drive the same synthetic traffic, so the two-rank fold has the one-rank
    run's mean and every rank prints the same fleet line."""
    exe = os.path.join(ROOT, "build", "fleet_loop")
    assert os.path.exists(exe), "build() makes build/fleet_loop"
    one = subprocess.run([exe, "4096", "200"], capture_output=True, text=True, timeout=150)
    assert one.returncode == 0, one.stderr
    env = dict(os.environ, FMSKF_RCCL_LIBRARY=LOOPBACK, LOOPBACK_RCCL_DIR=str(tmp_path), FLEET_WORLD="2",
               FLEET_ID=str(tmp_path / "fleet_id"), FLEET_DEVICE="0")
    procs = [subprocess.Popen([exe, "4096", "200"], env=dict(env, FLEET_RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(2)]
    try:
        outs = [p.communicate(timeout=150) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    assert [p.returncode for p in procs] == [0, 0], [o[1] for o in outs]
    fleet = [o[0].strip().splitlines()[3] for o in outs]
    assert fleet[0] == fleet[1], fleet
    assert fleet[0].startswith("fleet (2 ranks): 12 ensemble records"), fleet[0]
    solo = one.stdout.strip().splitlines()[3]
    mean = lambda line: line.split("last mean ")[1].split(", var")[0]  # noqa: E731
    assert mean(fleet[0]) == mean(solo), (fleet[0], solo)
    assert fleet[0].endswith("8192 robots in 2 records"), fleet[0]  # both ranks' robots, two records
