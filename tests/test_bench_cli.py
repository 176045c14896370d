"""bench.py's launcher decision (CPU only): `--gpus N > 1` without a launcher runs N ranks
through torch.distributed.run as a child process; under a launcher, or at N = 1, it runs in
place."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402  (module import touches no GPU and no torch)


def test_spawns_n_ranks_without_launcher():
    cmd = bench.launcher_cmd(["--gpus", "4", "--steps", "20", "--warmup", "5"], {})
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    i = cmd.index("--master-addr")
    assert cmd[i + 1] == "127.0.0.1" and int(cmd[i + 3]) > 0
    assert cmd[-7:] == [os.path.abspath(bench.__file__), "--gpus", "4", "--steps", "20", "--warmup", "5"]


def test_no_spawn_under_launcher_or_single_gpu():
    assert bench.launcher_cmd(["--gpus", "8"], {"WORLD_SIZE": "8"}) is None
    assert bench.launcher_cmd(["--gpus", "1"], {}) is None
    assert bench.launcher_cmd([], {}) is None
    assert bench.launcher_cmd(["--gpus=2", "--backend", "gloo"], {})[4] == "--nproc-per-node=2"


def test_cpu_share_reports_affinity():
    s = bench.cpu_share()
    assert s["affinity_cpus"] >= 1 and s["host_cpus"] >= s["affinity_cpus"]


def test_scaling_diag_fields():
    """the N > 1 line's self-explanation (bench.scaling_diag): per-rank plain-tick times, the sum
    of the ranks' plain-tick rates, scaling_self = value / that sum, and the side-stream exchange
    times max over ranks"""
    per_rank = [(0, 1 << 20, 0.0370), (1, 1 << 20, 0.0380)]
    rates = (1 << 20) / 0.0370e-3 + (1 << 20) / 0.0380e-3
    value = 0.9 * rates
    d = bench.scaling_diag(per_rank, [[0.020, 0.031], [0.025]], value, 0.0400, 0.0380)
    assert d["tick_kernel_ms_min"] == 0.0370 and d["tick_kernel_ms_max"] == 0.0380
    assert abs(d["rank_local_rate_sum"] - rates) < 1e-6 * rates
    assert abs(d["scaling_self"] - 0.9) < 1e-12
    assert abs(d["ms_per_step_over_tick_kernel"] - 0.0400 / 0.0380) < 1e-12
    x = d["exchange_ms"]
    assert x["max_over_ranks"] == 0.031 and x["per_rank_max"] == [0.031, 0.025] and x["events_per_rank"] == 2
    assert bench.scaling_diag(per_rank, [[], []], value, 0.04, 0.038)["exchange_ms"] is None


def test_mall_regime_and_traffic_provenance():
    assert bench.mall_regime(124 * (1 << 20)) == "hbm+mall"
    assert bench.mall_regime(124 * (1 << 24)) == "hbm"
    import json
    tj = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    b, src = bench.traffic_of(tj)
    assert b == tj["hbm_bytes_per_launch"] and "FETCH_SIZE" in src and tj["source"]["round"] in src
    for f in tj["source"]["committed_as"]:
        assert os.path.exists(os.path.join(ROOT, f)), f
    assert bench.traffic_of({"kernel": "x"}) == (None, None)


def test_path_byte_models_agree():
    """The path rows' algorithmic bytes per robot (bench.PATH_BYTES, the `roofline.achieved`
    numerator) and the read / write split tools/pmc_traffic.py checks the FETCH / WRITE counters
    against are one model: every row both name sums to the same bytes, and so does the committed
    profiles/pmc_traffic_paths.json (bytes per launch at 2^20 robots)."""
    import json
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import pmc_traffic  # noqa: E402
    secondary = {"cfg2_kf6_comp_pos_2p20": 272}
    seen = 0
    for key, _kernel, rd, wr in pmc_traffic.PATHS:
        want = bench.PATH_BYTES.get(key, secondary.get(key))
        assert want is not None, key
        assert rd + wr == want, (key, rd, wr, want)
        seen += 1
    assert seen >= 10
    committed = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic_paths.json")))
    for key, _kernel, rd, wr in pmc_traffic.PATHS:
        if key in committed:
            assert committed[key]["algorithmic_bytes_per_launch"] == (rd + wr) << 20, key
