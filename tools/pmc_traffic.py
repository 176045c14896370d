"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-launch HBM traffic for the KF6 tick.

gfx950 counter calibration (MI355X_MICROARCH.md, HBM section): FETCH_SIZE is exact only for
known access widths, so the same counters are collected for tools/membench.hip's
pattern_ipl1_dword kernel, which issues exactly the KF6 tick's loads and stores (27 dword
state planes read + written, yaw/gyro dword planes and the [N][4] int16 rpm plane read:
232 B per instance) with no arithmetic.  Its counter readings divided by its known bytes
give the correction factors, applied to the tick kernel's readings.

  python tools/pmc_traffic.py gpurun_out [profiles/pmc_traffic.json] [records|planes]
  python tools/pmc_traffic.py secondary gpurun_out [profiles/pmc_traffic_secondary.json]
  python tools/pmc_traffic.py paths gpurun_out [profiles/pmc_traffic_paths.json]
"""
import csv
import glob
import json
import os
import sys

# the round the counters were collected in (PMC_TAG=r5 ...): recorded as each file's `source`,
# which bench.py reports beside the traffic figure (`traffic_source`)
TAG = os.environ.get("PMC_TAG", "")


def source(root, dirs, kernel):
    return {"round": TAG, "kernel": kernel, "passes": [f"{os.path.relpath(root)}/{d}" for d in dirs],
            "committed_as": [f"profiles/{TAG}_{d}.csv" for d in dirs] if TAG else []}


def read(dirname, kernel_substr):
    vals = []
    for f in glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel_substr in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]))
    return vals


# HBM-regime lines of the bench (secondary): the tick kernel and, for calibration, the
# tools/membench.hip `caps` pattern with the same access widths and cache policy (non-temporal
# state rows of 4 or 8 bytes per lane, a 16-byte record), at the same N.  Per config:
# (bench key, kernel substring, pattern substring, pattern N, pattern read / write bytes per
# robot, algorithmic read / write bytes per robot of the tick, N)
SECONDARY = [
    ("cfg3_ekf9_2p22", "k_ekf9t", "k_tiled_probe<54, 256, 2, float>", 1 << 22, 232, 216, 236, 220, 1 << 22),
    ("cfg5_kf12d_2p20", "k_kf12s", "k_tiled_probe<90, 256, 2, double>", 1 << 20, 736, 720, 784, 720, 1 << 20),
    ("cfg2_kf6_2p24", "k_kf6t", "k_pitch_nt<27>", 1 << 24, 124, 108, 124, 108, 1 << 24),
]


def read_grid(dirname, kernel_substr, grid):
    vals = []
    for f in glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel_substr in r["Kernel_Name"] and int(r["Grid_Size"]) == grid:
                vals.append(float(r["Counter_Value"]))
    return vals


def secondary(root, out):
    """profiles/pmc_traffic_secondary.json: calibrated HBM bytes per launch of the cfg 3 / cfg 5 /
    2^24 tick kernels (gpurun_out/pmc_sec_{kernel,pattern}_{FETCH,WRITE}_SIZE)."""
    res = {"unit": "bytes per launch", "calibration": "tools/membench.hip caps patterns, same widths, same N"}
    for key, ksub, psub, pn, prd, pwr, ard, awr, n in SECONDARY:
        ent = {"n_instances": n, "kernel": ksub, "pattern": psub,
               "source": source(root, [f"pmc_sec_{key}_FETCH_SIZE", f"pmc_sec_{key}_WRITE_SIZE"], ksub)}
        for c, pbytes, abytes in (("FETCH_SIZE", prd * pn, ard * n), ("WRITE_SIZE", pwr * pn, awr * n)):
            pat = read_grid(os.path.join(root, f"pmc_sec_pattern_{c}"), psub, pn)
            kf = read(os.path.join(root, f"pmc_sec_{key}_{c}"), ksub)
            if not pat or not kf:
                print(f"missing data for {key} {c}: pattern {len(pat)} kernel {len(kf)}")
                return 1
            pv = sorted(pat)[len(pat) // 2] * 1024.0
            kv = sorted(kf)[len(kf) // 2] * 1024.0
            factor = pbytes / pv
            ent[c] = {"raw_kernel_bytes": kv, "raw_pattern_bytes": pv, "pattern_algorithmic_bytes": pbytes,
                      "calibration_factor": factor, "kernel_bytes_calibrated": kv * factor}
        ent["hbm_bytes_per_launch"] = ent["FETCH_SIZE"]["kernel_bytes_calibrated"] + \
            ent["WRITE_SIZE"]["kernel_bytes_calibrated"]
        ent["algorithmic_bytes_per_launch"] = (ard + awr) * n
        ent["traffic_over_algorithmic"] = ent["hbm_bytes_per_launch"] / ent["algorithmic_bytes_per_launch"]
        res[key] = ent
    print(json.dumps(res, indent=1))
    if out:
        json.dump(res, open(out, "w"), indent=1)
    return 0


# The rows either side of the tick at 2^20 (bench path_rows): (bench key, kernel substring,
# kernel read / write bytes per robot).  RS: px, py, prev, sums, yaw, rpm read (84), x and prev
# written (56); WT901 standard poll: row, len, parser count / flags read (54),
# flags, error, 2 registers (round 6: the other thirteen only in the snapshot row and the Yaw /
# GZ words), the 24-byte snapshot row, the Yaw / GZ words written (34; the empty parser window is
# neither read nor written, and round 6 reads no magnetometer register); CAN RX, four wheels: frame, stamp, micro, angle, previous angle / stamp, IIR y,
# the sums' low words read (104), the new stamp and angle over the older history slots, IIR y, the
# sums' low words, rpm and curr written (64; round 6: the sums' high words only on a carry); the KF6 with FMSKF_CFG_COMP_POS (k_kf6p at
# 2^20): the tick's 124 / 108 plus the five low-part rows read and written (144 / 128); the fused
# ISR with and without the CAN RX (below).  The
# counters are corrected with the KF6 calibration of profiles/pmc_traffic.json (the same
# streaming dword / 8- / 16-byte lane accesses: FETCH_SIZE counts half, WRITE_SIZE exact).
PATHS = [
    ("rs_tick_2p20", "k_rs2", 84, 56),
    ("rs_tick_2p20_padded_sums", "k_rs2", 84, 56),
    ("wt901_ingest_2p20", "k_wt901", 54, 34),
    ("can_ingest_2p20", "k_can4", 104, 64),
    # the control step (k_ctrl_step): power 1, interpolators 132, FF_PI_D 48, the last step's rpm 8,
    # rpm 8 read; the interpolators' time / speed / accel 36, FF_PI_D 48, the rpm 8 and the
    # currents 8 written (round 6)
    ("control_step_2p20", "k_ctrl_step", 1 + 132 + 48 + 8 + 8, 36 + 48 + 8 + 8),
    ("cfg2_kf6_comp_pos_2p20", "k_kf6p", 144, 128),
    # the fused KF6 ISR (k_isr_kf6, planes): the tick's 124 / 108, the control step's reads
    # without its rpm (189; 209 before round 6 also read the interpolators' acceleration and the
    # four float now_val) and writes (100; 152 before round 6 formed vel_tgt / now_tgt / now_ctrl
    # on demand and kept now_val as the step's rpm), the 0x200 frame (8 w)
    ("isr_kf6_2p20", "k_isr_kf6", 124 + 189, 108 + 100 + 8),
    # with the tick's CAN RX fused in (fmskf_isr_tick_can): + the CAN row's 104 / 64, the rpm
    # plane no longer read
    ("isr_can_kf6_2p20", "k_isr_kf6", 124 - 8 + 189 + 104, 108 + 100 + 8 + 64),
    # the reference-semantics ISR (k_isr_rs) on the motor state: the RS tick's 84 / 56 with the
    # control step's 189 / 100 and the frame; with the CAN RX fused in, the rpm and sums not read
    ("isr_rs_2p20", "k_isr_rs", 84 + 189, 56 + 100 + 8),
    # the EKF9 ISR (k_isr_ekf9): the tick's 232 / 216 (cfg 3's count; the heading's hidden row,
    # 4 + 4 B, is traffic above it) with the control step's 197 / 100 (its own rpm plane) and the
    # frame
    ("isr_ekf9_2p20", "k_isr_ekf9", 232 + 197, 216 + 100 + 8),
    # round 6: the previous sums neither read nor written while they equal the motor sums (PS)
    ("isr_can_rs_2p20", "k_isr_rs", 84 - 8 - 32 - 32 + 189 + 104, 56 - 32 + 100 + 8 + 64),
    # the EKF9 ISR with the tick's CAN RX fused in: + the CAN row's 104 / 64, the control step's
    # rpm plane no longer read
    ("isr_can_ekf9_2p20", "k_isr_ekf9", 232 + 197 - 8 + 104, 216 + 100 + 8 + 64),
]


def paths(root, out, calib="profiles/pmc_traffic.json"):
    """profiles/pmc_traffic_paths.json: memory-side bytes per launch of the path-row kernels at
    2^20 (gpurun_out/pmc_path_{key}_{FETCH,WRITE}_SIZE, tools/kbench.py runs)."""
    cj = json.load(open(calib))
    fac = {c: cj[c]["calibration_factor"] for c in ("FETCH_SIZE", "WRITE_SIZE")}
    n = 1 << 20
    res = {"unit": "bytes per launch", "n_instances": n,
           "calibration": f"{calib} (KF6 pattern): FETCH x {fac['FETCH_SIZE']:.4f}, WRITE x {fac['WRITE_SIZE']:.4f}"}
    for key, ksub, rd, wr in PATHS:
        ent = {"kernel": ksub,
               "source": source(root, [f"pmc_path_{key}_FETCH_SIZE", f"pmc_path_{key}_WRITE_SIZE"], ksub)}
        for c, algo in (("FETCH_SIZE", rd * n), ("WRITE_SIZE", wr * n)):
            kv = read(os.path.join(root, f"pmc_path_{key}_{c}"), ksub)
            if not kv:
                print(f"missing data for {key} {c}")
                return 1
            k = sorted(kv)[len(kv) // 2] * 1024.0
            ent[c] = {"raw_bytes": k, "calibrated_bytes": k * fac[c], "kernel_algorithmic_bytes": algo,
                      "over_algorithmic": k * fac[c] / algo}
        ent["hbm_bytes_per_launch"] = ent["FETCH_SIZE"]["calibrated_bytes"] + ent["WRITE_SIZE"]["calibrated_bytes"]
        ent["algorithmic_bytes_per_launch"] = (rd + wr) * n
        ent["traffic_over_algorithmic"] = ent["hbm_bytes_per_launch"] / ent["algorithmic_bytes_per_launch"]
        res[key] = ent
    print(json.dumps(res, indent=1))
    if out:
        json.dump(res, open(out, "w"), indent=1)
    return 0


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "paths":
        return paths(sys.argv[2] if len(sys.argv) > 2 else "gpurun_out",
                     sys.argv[3] if len(sys.argv) > 3 else None)
    if len(sys.argv) > 1 and sys.argv[1] == "secondary":
        return secondary(sys.argv[2] if len(sys.argv) > 2 else "gpurun_out",
                         sys.argv[3] if len(sys.argv) > 3 else None)
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    out = sys.argv[2] if len(sys.argv) > 2 else None
    n = 1 << 20
    inputs = sys.argv[3] if len(sys.argv) > 3 else "records"
    res = {"n_instances": n, "kernel": "k_kf6 (tick, TABLE512, N=2^20)", "inputs": inputs,
           "unit": "bytes per launch",
           "source": source(root, ["pmc_kf6_FETCH_SIZE", "pmc_kf6_WRITE_SIZE"], "k_kf6p (tools/kbench.py --packed)")}
    for c, algo in (("FETCH_SIZE", 124 * n), ("WRITE_SIZE", 108 * n)):
        pat = read(os.path.join(root, f"pmc_pat_{c}"), "k_pattern<1>")
        kf = read(os.path.join(root, f"pmc_kf6_{c}"), "k_kf6")
        if not pat or not kf:
            print(f"missing data for {c}: pattern {len(pat)} kf6 {len(kf)}")
            return 1
        p = sorted(pat)[len(pat) // 2] * 1024.0  # counters are in KiB
        k = sorted(kf)[len(kf) // 2] * 1024.0
        factor = algo / p
        res[c] = {"raw_kf6_bytes": k, "raw_pattern_bytes": p, "pattern_algorithmic_bytes": algo,
                  "calibration_factor": factor, "kf6_bytes_calibrated": k * factor}
    res["hbm_bytes_per_launch"] = res["FETCH_SIZE"]["kf6_bytes_calibrated"] + \
        res["WRITE_SIZE"]["kf6_bytes_calibrated"]
    res["algorithmic_bytes_per_launch"] = 232 * n
    res["traffic_over_algorithmic"] = res["hbm_bytes_per_launch"] / res["algorithmic_bytes_per_launch"]
    print(json.dumps(res, indent=1))
    if out:
        json.dump(res, open(out, "w"), indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
