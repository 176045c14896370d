"""The driver's bench command (`python bench.py --gpus 1 --steps 20 --warmup 5`) on the GPU box:
the one JSON line it prints keeps the contract the round's records are judged on -- BASELINE's
metric and unit, the cfg 2 workload, whole-job `value` consistent with `ms_per_step`, a
`roofline` whose `frac` is `achieved / peak` with the PMC `traffic`, the `cpu_baseline` with its
core count, kind and sample, the post-timing parity sample bit-exact, and every `secondary` /
`path_rows` entry with SURVEY §8(d)'s algorithmic bytes."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SECONDARY_BYTES = {"cfg3_ekf9_2p22": 448, "cfg5_kf12d_2p20": 1504, "cfg2_kf6_2p24": 232,
                   "cfg2_kf6_comp_pos_2p20": 272, "cfg3_ekf9_comp_pos_2p22": 488, "cfg4_shard_kf6_2p21": 232}
PATH_BYTES = {"rs_tick_2p20": 140, "rs_tick_2p20_padded_sums": 140, "rs_tick_2p20_device_state": 140,
              "wt901_ingest_2p20": 88, "can_ingest_2p20": 168, "control_step_2p20": 297,
              "isr_kf6_2p20": 529, "firmware_loop_kf6_2p20": 701.8, "isr_can_kf6_2p20": 689,
              "isr_ekf9_2p20": 753, "isr_can_ekf9_2p20": 913, "isr_rs_2p20": 437, "isr_can_rs_2p20": 501,
              "firmware_loop_rs_fused_2p20": 509.8, "firmware_loop_kf6_fused_2p20": 693.8}


def test_driver_bench_line_contract():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "1", "--steps", "20", "--warmup", "5"],
                       cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert out["metric"] == base["metric"] and out["unit"] == "steps/s"
    assert (out["n_gpus"], out["steps"], out["warmup"]) == (1, 20, 5)
    assert out["higher_is_better"] is True and out["scaling"] == "weak" and out["vs_baseline"] is None
    assert out["dtype"] == "f32" and "synthetic" in out["data"]
    cfg = out["config"]
    assert cfg["workload"].startswith("cfg2") and cfg["instances_per_gpu"] == 1 << 20
    assert cfg["global_instances"] == 1 << 20
    # whole-job steps/s over the timed wall clock
    assert out["value"] == pytest.approx((1 << 20) / (out["ms_per_step"] * 1e-3), rel=1e-6)
    assert out["value"] > 1e9
    rf = out["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0 and rf["bytes_per_step"] == 232
    assert rf["frac"] == pytest.approx(rf["achieved"] / rf["peak"], rel=1e-9)
    assert rf["achieved"] == pytest.approx(232 * (1 << 20) / (rf["kernel_ms"] * 1e-3) / 1e9, rel=1e-6)
    assert 0.5 < rf["frac"] < 1.0
    assert rf["traffic"] == pytest.approx(232 * (1 << 20), rel=0.05)  # PMC bytes per launch
    assert "FETCH_SIZE" in rf["traffic_source"] and rf["traffic_source"].startswith("profiles/pmc_traffic.json")
    # the roofline's denominator is consistent with the run's own clock: the kernel's average
    # (>= 200 prequeued plain ticks) cannot exceed the timed region's GPU time per step (which
    # also holds the ensemble ticks' record epilogue), and frac follows from that region
    assert rf["kernel_ticks_timed"] >= 200
    assert rf["kernel_ms"] <= 1.01 * rf["timed_region_ms_per_step"], rf
    assert rf["kernel_ms"] <= 1.01 * out["ms_per_step"], (rf, out["ms_per_step"])
    region_frac = 232 * (1 << 20) / (rf["timed_region_ms_per_step"] * 1e-3) / 8e12
    assert rf["frac"] == pytest.approx(region_frac, rel=0.03), (rf["frac"], region_frac)
    assert rf["regime"] == "hbm+mall"  # 124 B x 2^20 fits the 256 MiB Infinity Cache
    cb = out["cpu_baseline"]
    assert cb["value"] > 0 and cb["unit"] == "steps/s" and cb["cores"] >= 1
    assert cb["kind"] == "port" and cb["sample"]
    # the tuned port is bitwise the checker on the sample, and both rates are reported
    assert cb["bitexact_vs_checker"] is True and cb["value_checker"] > 0 and cb["value_1core"] > 0
    assert cb["rs_tick"]["steps_per_s"] > 0 and cb["rs_tick"]["steps_per_s_1core"] > 0
    assert out["parity_sampled"]["bitexact"] and out["parity_sampled"]["mismatched_robots"] == 0
    assert out["nonfinite_instances"] == 0
    assert out["ensemble"]["count"] == 1 << 20
    for key, b in SECONDARY_BYTES.items():
        sec = out["secondary"][key]["roofline"]
        assert sec["bytes_per_step"] == b, key
        assert 0.3 < sec["frac"] < 1.0, (key, sec)
    assert out["secondary"]["cfg2_kf6_2p24"]["roofline"]["regime"] == "hbm"
    for key in ("cfg3_ekf9_2p22", "cfg5_kf12d_2p20", "cfg2_kf6_2p24"):
        assert out["secondary"][key]["roofline"]["traffic_source"], key
    for key, b in PATH_BYTES.items():
        row = out["path_rows"][key]["roofline"]
        assert row["bytes_per_step"] == pytest.approx(b), key
        assert 0.3 < row["frac"] < 1.0, (key, row)
    # the firmware loop with the tick's CAN RX inside the ISR call is not slower than the split
    # form (the fused kernel moves 8 B less per robot and saves a launch)
    pr = out["path_rows"]
    assert pr["firmware_loop_kf6_fused_2p20"]["kernel_ms"] <= 1.02 * pr["firmware_loop_kf6_2p20"]["kernel_ms"]
