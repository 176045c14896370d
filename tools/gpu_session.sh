#!/usr/bin/env bash
# One GPU-box session: smoke -> GPU parity tests -> bench -> rocprofv3 kernel trace.
# Each GPU step has its own time limit; a crash/abort/timeout (rc not in {0,1}) ends
# the session immediately (no further GPU work after a fault).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT"
STEPS="${STEPS:-smoke tests bench prof}"

run() {  # name limit cmd...
  local name=$1 limit=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "!!! $name ended with rc=$rc: stopping the session"
    exit $rc
  fi
  return 0
}

for s in $STEPS; do
  case $s in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run pytest_gpu 1200 python -m pytest tests -m gpu -q --timeout 600 -rf ;;
    bench) run bench 600 python bench.py ${BENCH_ARGS:-} ;;
    dist1) run dist1 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
             --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --steps 200 \
             --warmup 20 --no-cpu-baseline --no-fused ;;
    kb)    i=0; IFS=';' read -ra KBL <<< "${KB_LIST:-}"; for a in "${KBL[@]}"; do
             i=$((i+1)); run kb$i 240 python tools/kbench.py $a
           done ;;
    sweep) for v in ${VARIANTS:-0 2 3 4}; do
             export FMSKF_KF6_VARIANT=$v
             run kb_v$v 180 python tools/kbench.py ${KB_ARGS:-}
           done
           unset FMSKF_KF6_VARIANT ;;
    prof)  run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
             python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-fused ;;
    pmc)   run pmc 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
             python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-fused &&
           run pmc2 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
             python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-fused ;;
  esac
done
echo "=== session done"
