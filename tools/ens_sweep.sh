#!/usr/bin/env bash
# GPU-box sweep of the stand-alone ensemble record (k_ens_partial + k_ens_fold) under the
# rocprofv3 kernel trace: each "model n" entry of CFGS (';'-separated) at each robots-per-lane
# setting of RS (FMSKF_ENS_R; "auto" leaves it unset), then the per-kernel averages.
#   CFGS="kf6 1048576; ekf9 4194304" RS="auto 4 8" bash tools/ens_sweep.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ens
IFS=';' read -ra CFG <<< "${CFGS:-kf6 1048576; kf6 2097152; kf6 4194304; ekf9 1048576; ekf9 2097152; ekf9 4194304}"
for p in $(seq 1 "${PASSES:-1}"); do
  for cfg in "${CFG[@]}"; do
    read -r model n <<< "$cfg"
    for r in ${RS:-auto 4 8}; do
      d=gpurun_out/ens/${model}_${n}_r${r}_p$p
      envs=()
      [ "$r" = auto ] || envs=(FMSKF_ENS_R=$r)
      env "${envs[@]}" timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run -- \
        python tools/kbench.py --model "$model" --n "$n" --op ensemble --ticks 50 > "$d.log" 2>&1
      rc=$?
      if [ $rc -ne 0 ]; then echo "!!! $model $n r=$r rc=$rc"; tail -n 5 "$d.log"; exit $rc; fi
    done
  done
done
python - <<'EOF'
import csv, glob, os
for d in sorted(glob.glob("gpurun_out/ens/*_r*_p*/")):
    out = []
    for r in csv.DictReader(open(d + "run_kernel_stats.csv")):
        nm = r["Name"].split("<")[0].split("::")[-1]
        if nm in ("k_ens_partial", "k_ens_fold"):
            out.append(f"{nm} {float(r['AverageNs']) / 1000:.2f}")
    print(os.path.basename(d.rstrip("/")), ", ".join(out))
EOF
