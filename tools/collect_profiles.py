"""Copy the profiling session's outputs from gpurun_out/ into profiles/ under a round prefix:
    python tools/collect_profiles.py r3 [--pmc-kf6] [--secondary]
always: bench.log / prof.log lines, the rocprofv3 kernel / domain stats and the fmskf kernel trace
of the driver's command, and the path-row PMC passes (pmc_path_*, tools/session.sh) when
present; --pmc-kf6: the headline kernel's FETCH / WRITE passes and their calibration pattern
(tools/session.sh); --secondary: the HBM-regime PMC passes and the prof_* kernel stats"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")
P = os.path.join(ROOT, "profiles")


def last_json(path):
    for line in reversed(open(path).read().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no JSON line in {path}")


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r1"
    if not tag.isidentifier():  # a round prefix such as r2, never an option
        raise SystemExit(__doc__)
    pmc_kf6 = "--pmc-kf6" in sys.argv
    secondary = "--secondary" in sys.argv
    json.dump(last_json(os.path.join(G, "bench.log")), open(os.path.join(P, f"{tag}_bench.json"), "w"), indent=1)
    json.dump(last_json(os.path.join(G, "prof.log")), open(os.path.join(P, f"{tag}_prof_bench_line.json"), "w"),
              indent=1)
    for k in ("kernel_stats", "domain_stats"):
        shutil.copy(os.path.join(G, "prof", f"run_{k}.csv"), os.path.join(P, f"{tag}_bench_{k}.csv"))
    with open(os.path.join(G, "prof", "run_kernel_trace.csv")) as fi, \
            open(os.path.join(P, f"{tag}_bench_kernel_trace_fmskf.csv"), "w", newline="") as fo:
        r = csv.reader(fi)
        w = csv.writer(fo)
        hdr = next(r)
        w.writerow(hdr)
        col = hdr.index("Kernel_Name")
        for row in r:
            if "fmskf::" in row[col]:
                w.writerow(row)
    if pmc_kf6:
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            for kind in ("kf6", "pat"):
                src = glob.glob(os.path.join(G, f"pmc_{kind}_{c}", "**", "*counter_collection.csv"), recursive=True)[0]
                shutil.copy(src, os.path.join(P, f"{tag}_pmc_{'kf6' if kind == 'kf6' else 'pattern'}_{c}.csv"))
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), G,
                        os.path.join(P, "pmc_traffic.json"), "records"], check=True, stdout=subprocess.DEVNULL)
    # the rows either side of the tick (tools/session.sh paths): calibrated traffic + the counter rows
    if glob.glob(os.path.join(G, "pmc_path_*")):
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), "paths", G,
                        os.path.join(P, "pmc_traffic_paths.json")], check=True, stdout=subprocess.DEVNULL)
        for d in sorted(glob.glob(os.path.join(G, "pmc_path_*"))):
            f = os.path.join(d, "run_counter_collection.csv")
            if not os.path.isdir(d) or not os.path.exists(f):
                continue
            rows_in = list(csv.reader(open(f)))
            col = rows_in[0].index("Kernel_Name")
            keep = [r for r in rows_in[1:] if "fmskf::" in r[col]]
            with open(os.path.join(P, f"{tag}_{os.path.basename(d)}.csv"), "w", newline="") as fo:
                w = csv.writer(fo)
                w.writerow(rows_in[0])
                w.writerows(keep)
    # wave-state counters of the path-row kernels (tools/session.sh sq) and their per-kernel summary
    sq = []
    for d in sorted(glob.glob(os.path.join(G, "sq_*"))):
        f = os.path.join(d, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        rows_in = list(csv.reader(open(f)))
        hdr = rows_in[0]
        col, cn, cv = hdr.index("Kernel_Name"), hdr.index("Counter_Name"), hdr.index("Counter_Value")
        keep = [r for r in rows_in[1:] if "fmskf::" in r[col]]
        with open(os.path.join(P, f"{tag}_{os.path.basename(d)}.csv"), "w", newline="") as fo:
            w = csv.writer(fo)
            w.writerow(hdr)
            w.writerows(keep)
        tot, calls = {}, {}
        for r in keep:
            k = (r[col], r[cn])
            tot[k] = tot.get(k, 0.0) + float(r[cv])
            calls[k] = calls.get(k, 0) + 1
        for name in sorted({k[0] for k in tot}):
            if calls.get((name, "SQ_WAVES"), 0) < 5:  # warm-up launches of other kernels
                continue
            a = {c: tot[(name, c)] / calls[(name, c)] for (nm, c) in tot if nm == name}
            wc = a["SQ_WAVE_CYCLES"]
            sq.append({"run": os.path.basename(d), "kernel": name, "launches": calls[(name, "SQ_WAVES")],
                       "waves": a["SQ_WAVES"], "valu_per_wave": a["SQ_INSTS_VALU"] / a["SQ_WAVES"],
                       "salu_per_wave": a["SQ_INSTS_SALU"] / a["SQ_WAVES"],
                       "wait_frac": a["SQ_WAIT_ANY"] / wc, "issue_wait_frac": a["SQ_WAIT_INST_ANY"] / wc,
                       "active_frac": a["SQ_ACTIVE_INST_ANY"] / wc})
    if sq:
        json.dump(sq, open(os.path.join(P, f"{tag}_sq_summary.json"), "w"), indent=1)
    # HBM-regime bench lines (tools/session.sh sec): calibrated traffic + the counter rows
    if secondary and glob.glob(os.path.join(G, "pmc_sec_*")):
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), "secondary", G,
                        os.path.join(P, "pmc_traffic_secondary.json")], check=True, stdout=subprocess.DEVNULL)
        for d in sorted(glob.glob(os.path.join(G, "pmc_sec_*"))):
            f = os.path.join(d, "run_counter_collection.csv")
            if not os.path.isdir(d) or not os.path.exists(f):
                continue
            rows_in = list(csv.reader(open(f)))
            col = rows_in[0].index("Kernel_Name")
            keep = [r for r in rows_in[1:] if any(k in r[col] for k in ("fmskf::", "k_tiled_probe", "k_pitch_nt"))]
            with open(os.path.join(P, f"{tag}_{os.path.basename(d)}.csv"), "w", newline="") as fo:
                w = csv.writer(fo)
                w.writerow(rows_in[0])
                w.writerows(keep)
    rows = []
    for d in sorted(glob.glob(os.path.join(G, "prof_*")) if secondary else []):
        if not os.path.isdir(d):
            continue
        f = glob.glob(os.path.join(d, "*kernel_stats.csv"))
        if not f:
            continue
        for r in csv.DictReader(open(f[0])):
            if "fmskf::" in r["Name"]:
                rows.append([os.path.basename(d)[5:], r["Name"], r["Calls"], r["AverageNs"], r["MinNs"], r["MaxNs"]])
    if rows:
        with open(os.path.join(P, f"{tag}_secondary_kernel_stats.csv"), "w", newline="") as fo:
            w = csv.writer(fo)
            w.writerow(["workload", "kernel", "calls", "avg_ns", "min_ns", "max_ns"])
            w.writerows(rows)
    print(f"profiles/{tag}_* refreshed: {len(rows)} secondary kernel rows")


if __name__ == "__main__":
    main()
