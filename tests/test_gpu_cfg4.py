"""Config 4 (BASELINE.json configs[3]: 2^24 KF6 robots over 8 GPUs, ensemble mean / covariance
all-gathered over RCCL) on the one-GPU test box.

* the per-GPU shard (2^21 robots, 16-byte tick records) ticked and recorded by the fused
  tick + ensemble kernel, sampled bit-exact against the oracle, the record against the oracle's
  two-pass moments of the same state;
* bench.py's distributed code path under torch.distributed.run at world size 1, for each
  gather mode (torch all-gather on RCCL's stream, in the tick stream, and the handle-owned
  communicator fmskf_comm_init / fmskf_ensemble_stats that C callers bind): the gathered
  record must fold to the statistics of the rank's stand-alone record.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import fmskf
from fmskf import Engine
from fmskf.synth import Trajectory

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cfg4_shard_2p21_records_and_record(orc):
    import torch
    n, T = 1 << 21, 4
    tr = Trajectory(n, T, seed=404)
    yaw, gz, rpm = tr.kf6_inputs()
    dy, dg, dr = (torch.from_numpy(a).cuda() for a in (yaw, gz, rpm))
    recs = fmskf.kf6_records(dy, dg, dr)
    with Engine("kf6", n) as e:
        e.set_stream(torch.cuda.current_stream())
        for t in range(T - 1):
            e.tick(kf6_rec=recs[t])
        rec = e.tick_ensemble(kf6_rec=recs[T - 1])
        x, P = e.get_state()
        assert e.get_counters()[0] == 0
    idx = np.sort(np.random.default_rng(4).choice(n, 2048, replace=False))
    cfg = fmskf.default_config("kf6", idx.size)
    prm = orc.kf6_params(cfg.dt, np.array(cfg.q[:21]), np.array(cfg.r[:10]))
    xo = np.zeros((6, idx.size), np.float32)
    Po = np.repeat(np.float32(np.array(cfg.p0[:21]))[:, None], idx.size, 1).copy()
    for t in range(T):
        orc.kf6_tick(xo, Po, np.ascontiguousarray(yaw[t, idx]), np.ascontiguousarray(gz[t, idx]),
                     np.ascontiguousarray(rpm[t, idx]), None, prm)
    assert np.array_equal(x[:, idx].view(np.uint32), xo.view(np.uint32))
    assert np.array_equal(P[:, idx].view(np.uint32), Po.view(np.uint32))
    assert rec[0] == n
    mo, co = orc.ens_finalize(6, orc.ens_partial(x))
    mf, cf = fmskf.ensemble_combine(6, rec[None, :])
    np.testing.assert_allclose(mf, mo, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(cf, co, rtol=1e-9, atol=1e-15)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("gather", ["async", "stream", "native"])
@pytest.mark.parametrize("ensemble", ["fused", "separate"])
def test_bench_distributed_path_world1(gather, ensemble):
    if gather == "native" and ensemble == "separate":
        pytest.skip("the native path records through fmskf_tick_ensemble_begin itself")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "1",
           "--steps", "40", "--warmup", "5", "--ensemble-every", "8", "--no-cpu-baseline", "--no-fused",
           "--no-secondary", "--gather", gather, "--ensemble", ensemble, "--check-ensemble"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 1
    chk = out["ensemble_check"]
    assert chk["count"] == 1 << 20
    assert chk["mean_max_rel"] < 1e-12, chk
    assert chk["cov_max_rel"] < 1e-9, chk
    assert out["nonfinite_instances"] == 0
    assert out["value"] > 1e9
    assert out["parity_sampled"]["bitexact"], out["parity_sampled"]
    assert out["config"]["gather"] == gather


def test_bench_spawns_ranks_without_launcher():
    """`python bench.py --gpus 2` with no launcher (the driver's BENCH command form): bench.py
    starts torch.distributed.run itself, two ranks (gloo, both on the one GPU of the test box),
    the line reports n_gpus 2, a green ensemble check and the post-timing parity sample."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--backend", "gloo", "--same-device", "--steps", "20",
           "--warmup", "5", "--n-per-gpu", str(1 << 18), "--ensemble-every", "8", "--no-fused",
           "--no-secondary", "--check-ensemble", "--cpu-sample-s", "1"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["n_gpus"] == 2 and out["config"]["global_instances"] == 2 << 18
    chk = out["ensemble_check"]
    assert chk["count"] == 2 << 18 and chk["mean_max_rel"] < 1e-12 and chk["cov_max_rel"] < 1e-9, chk
    assert out["parity_sampled"]["bitexact"]
    assert out["cpu_baseline"]["value"] > 0 and out["cpu_baseline"]["affinity_cpus"] >= 1


@pytest.mark.parametrize("strong,gather", [(False, "async"), (True, "async"), (False, "native"), (True, "native")])
def test_bench_world2_rehearsal_same_gpu(strong, gather, tmp_path):
    """bench.py's N > 1 code path with two ranks (torch.distributed.run, gloo, both ranks on the
    one GPU of the test box; RCCL refuses two ranks on one device): per-rank shards with their
    own seeds, fused records all-gathered every 8 ticks, max-over-ranks timing, the whole-job
    count, and every rank's gathered records folding to the statistics of the stand-alone
    records.  strong: cfg 4's strong-scaling form (--n-total, an odd total split unevenly).
    native: the driver's default at N > 1 -- libfmskf's own communicator (comm id broadcast over
    the process group, fmskf_tick_ensemble_begin / fmskf_ensemble_end) -- with the loopback
    stand-in for RCCL (tests/native/loopback_rccl.cpp, FMSKF_RCCL_LIBRARY)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    if gather == "native":
        env.update(FMSKF_RCCL_LIBRARY=os.path.join(ROOT, "build", "libloopback_rccl.so"),
                   LOOPBACK_RCCL_DIR=str(tmp_path))
    n = 1 << 18
    total = 2 * n + 3 if strong else 2 * n
    size = ["--n-total", str(total)] if strong else ["--n-per-gpu", str(n)]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--steps", "32", "--warmup", "4", "--ensemble-every", "8", *size,
           "--no-cpu-baseline", "--no-fused", "--no-secondary", "--backend", "gloo", "--same-device",
           "--check-ensemble", "--gather", gather, "--cfg4-steps", "32"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["n_gpus"] == 2 and out["config"]["global_instances"] == total
    assert out["scaling"] == ("strong" if strong else "weak")
    chk = out["ensemble_check"]
    assert chk["count"] == total
    assert chk["mean_max_rel"] < 1e-12, chk
    assert chk["cov_max_rel"] < 1e-9, chk
    assert out["ensemble"]["count"] == total  # the gathered records' own count rows
    assert out["nonfinite_instances"] == 0
    assert out["config"]["gather"] == gather
    if gather == "native":
        # what the communicator itself reports, from every rank (ncclCommCount / UserRank)
        assert out["rccl_ranks"] == 2 and out["rccl"]["user_ranks"] == [0, 1], out["rccl"]
        assert out["rccl"]["library"].endswith("libloopback_rccl.so")
        assert out["ensemble"]["records_folded"] == 2
    # BASELINE configs[3] in the same invocation: 2^24 robots over the two ranks
    c4 = out["cfg4_16M"]
    assert c4["instances_total"] == 1 << 24 and c4["n_gpus"] == 2
    assert c4["gathered_count"] == 1 << 24 and c4["records_folded"] == 2, c4
    assert c4["ensemble_every_16"]["steps_per_s"] > 0 and c4["ensemble_every_1"]["steps_per_s"] > 0
    if gather == "native":
        assert c4["rccl_ranks"] == 2


def test_bench_native_gather_falls_back_together(tmp_path):
    """When libfmskf's communicator cannot come up (here FMSKF_RCCL_LIBRARY names a missing
    library, so fmskf_comm_unique_id fails on rank 0), every rank learns it over torch's group and
    all of them measure with torch's all-gather instead; the line says so (`gather_fallback`, the
    config's gather "async"), the ensemble check stays green and cfg4_16M measures the same way,
    instead of the 8-GPU run dying or its ranks disagreeing."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1",
               FMSKF_RCCL_LIBRARY=str(tmp_path / "missing_librccl.so"))
    n = 1 << 18
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--steps", "16", "--warmup", "4", "--ensemble-every", "8", "--n-per-gpu", str(n),
           "--no-cpu-baseline", "--no-fused", "--no-secondary", "--backend", "gloo", "--same-device",
           "--check-ensemble", "--gather", "native", "--cfg4-steps", "16"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    fb = out["gather_fallback"]
    assert fb["from"] == "native" and fb["to"] == "async" and fb["errors"], fb
    assert out["config"]["gather"] == "async" and "rccl_ranks" not in out
    chk = out["ensemble_check"]
    assert chk["count"] == 2 * n and chk["mean_max_rel"] < 1e-12 and chk["cov_max_rel"] < 1e-9, chk
    c4 = out["cfg4_16M"]
    assert c4["gather"] == "async", c4  # the run had already fallen back
    assert c4["gathered_count"] == 1 << 24

