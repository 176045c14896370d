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
