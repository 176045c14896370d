#!/usr/bin/env bash
# Round-2 GPU session: parity tests, the driver's bench command, its kernel trace.
# Every GPU step has its own limit; any rc other than 0/1 ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT"
STEPS="${STEPS:-tests bench prof}"
run() {
  local name=$1 limit=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 6 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "!!! $name rc=$rc: stopping"; exit $rc; fi
  return 0
}
for s in $STEPS; do
  case $s in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run pytest_gpu 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf ${TEST_ARGS:-} ;;
    tsel)  run pytest_sel 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rf -k "${TEST_K}" ;;
    bench) run bench 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench2) run bench2 600 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary ;;
    prof)  run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
             python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline ;;
    kb)    i=0; IFS=';' read -ra KBL <<< "${KB_LIST:-}"; for a in "${KBL[@]}"; do
             i=$((i+1)); run kb$i 240 python tools/kbench.py $a
           done ;;
  esac
done
echo "=== session done"
