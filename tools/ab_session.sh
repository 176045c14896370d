#!/usr/bin/env bash
# A/B kernel sweeps on the GPU box: optional selected parity tests, then one kbench line per
# entry of AB (entries separated by ';', each "[VAR=value ...] kbench args"), each pass of the
# list PASSES times.  Every GPU step runs under its own limit; any rc other than 0 ends it.
#   AB="FMSKF_ENS_VEC=0 --model kf6 --op ensemble; --model kf6 --op ensemble" PASSES=2 \
#   TEST_K="ensemble" bash tools/ab_session.sh
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT"
LOG="$OUT/ab.log"
: > "$LOG"
if [ -n "${TEST_K:-}" ]; then
  timeout -k 10 "${TEST_LIMIT:-600}" python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -rf -k "$TEST_K" > "$OUT/ab_tests.log" 2>&1
  rc=$?
  tail -n 5 "$OUT/ab_tests.log"
  if [ $rc -ne 0 ]; then echo "!!! tests rc=$rc: stopping"; exit $rc; fi
fi
IFS=';' read -ra ENTRIES <<< "${AB:-}"
for p in $(seq 1 "${PASSES:-1}"); do
  for ent in "${ENTRIES[@]}"; do
    envs=()
    args=()
    for w in $ent; do
      if [[ "$w" == *=* && ${#args[@]} -eq 0 ]]; then envs+=("$w"); else args+=("$w"); fi
    done
    line=$(env "${envs[@]}" timeout -k 10 "${KB_LIMIT:-180}" python tools/kbench.py "${args[@]}" 2>>"$OUT/ab_err.log" | tail -n 1)
    rc=$?
    echo "{\"pass\": $p, \"env\": \"${envs[*]}\", \"args\": \"${args[*]}\", \"out\": ${line:-null}}" | tee -a "$LOG"
    if [ $rc -ne 0 ]; then echo "!!! kbench rc=$rc: stopping"; exit $rc; fi
  done
done
echo "=== ab done"
