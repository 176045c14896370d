"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-launch HBM traffic for the KF6 tick.

gfx950 counter calibration (MI355X_MICROARCH.md, HBM section): FETCH_SIZE is exact only for
known access widths, so the same counters are collected for tools/membench.hip's
pattern_ipl1_dword kernel, which issues exactly the KF6 tick's loads and stores (27 dword
state planes read + written, yaw/gyro dword planes and the [N][4] int16 rpm plane read:
232 B per instance) with no arithmetic.  Its counter readings divided by its known bytes
give the correction factors, applied to the tick kernel's readings.

  python tools/pmc_traffic.py gpurun_out [profiles/pmc_traffic.json] [records|planes]
"""
import csv
import glob
import json
import os
import sys


def read(dirname, kernel_substr):
    vals = []
    for f in glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel_substr in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]))
    return vals


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    out = sys.argv[2] if len(sys.argv) > 2 else None
    n = 1 << 20
    inputs = sys.argv[3] if len(sys.argv) > 3 else "records"
    res = {"n_instances": n, "kernel": "k_kf6 (tick, TABLE512, N=2^20)", "inputs": inputs,
           "unit": "bytes per launch"}
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
