#!/usr/bin/env bash
# Round-4 profile refresh (one per round, at the end): the driver's bench command, its
# rocprofv3 kernel trace, FETCH_SIZE / WRITE_SIZE passes (one counter per run) of the headline
# kernel and its calibration pattern, of the HBM-regime secondary lines and of the path rows
# (incl. the FMSKF_CFG_COMP_POS KF6 at 2^20), and wave-state counters of the path-row kernels.
# Each GPU step runs under its own limit; a crash / abort / timeout (rc not in {0,1}) ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT" build
run() {
  local name=$1 limit=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 3 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "!!! $name rc=$rc: stopping"; exit $rc; fi
  return 0
}
[ -x build/membench ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/membench.hip -o build/membench
STEPS="${STEPS:-bench prof pmc sec paths sq}"
for s in $STEPS; do
  case $s in
    bench) run bench 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    prof)  run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
             python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline ;;
    pmc)   for c in FETCH_SIZE WRITE_SIZE; do
             run pmc_kf6_$c 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_kf6_$c" -o run -- \
               python tools/kbench.py --ticks 30 --packed
             run pmc_pat_$c 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_pat_$c" -o run -- build/membench 20
           done ;;
    sec)   for c in FETCH_SIZE WRITE_SIZE; do
             run pmc_sec_pattern_$c 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_sec_pattern_$c" -o run -- \
               build/membench 22 1 caps
             run pmc_sec_cfg3_ekf9_2p22_$c 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_sec_cfg3_ekf9_2p22_$c" -o run -- \
               python tools/kbench.py --model ekf9 --n 4194304 --ticks 8
             run pmc_sec_cfg5_kf12d_2p20_$c 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_sec_cfg5_kf12d_2p20_$c" -o run -- \
               python tools/kbench.py --model kf12d --ticks 8
             run pmc_sec_cfg2_kf6_2p24_$c 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_sec_cfg2_kf6_2p24_$c" -o run -- \
               python tools/kbench.py --model kf6 --packed --n 16777216 --ticks 6
           done ;;
    paths) for c in FETCH_SIZE WRITE_SIZE; do
             run pmc_path_rs_tick_2p20_$c 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_path_rs_tick_2p20_$c" -o run -- \
               python tools/kbench.py --model rs --ticks 30
             run pmc_path_rs_tick_2p20_padded_sums_$c 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_path_rs_tick_2p20_padded_sums_$c" -o run -- \
               python tools/kbench.py --model rs --pad 512 --ticks 30
             run pmc_path_wt901_ingest_2p20_$c 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_path_wt901_ingest_2p20_$c" -o run -- \
               python tools/kbench.py --op wt901 --ticks 30
             run pmc_path_can_ingest_2p20_$c 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_path_can_ingest_2p20_$c" -o run -- \
               python tools/kbench.py --op can --ticks 30
             run pmc_path_cfg2_kf6_comp_pos_2p20_$c 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_path_cfg2_kf6_comp_pos_2p20_$c" -o run -- \
               python tools/kbench.py --packed --comp --ticks 30
           done ;;
    sq)    SQC="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
           run sq_kf6 120 rocprofv3 --pmc $SQC --output-format csv -d "$OUT/sq_kf6" -o run -- python tools/kbench.py --packed --ticks 30
           run sq_rs 120 rocprofv3 --pmc $SQC --output-format csv -d "$OUT/sq_rs" -o run -- python tools/kbench.py --model rs --pad 512 --ticks 30
           run sq_wt901 120 rocprofv3 --pmc $SQC --output-format csv -d "$OUT/sq_wt901" -o run -- python tools/kbench.py --op wt901 --ticks 30
           run sq_can 120 rocprofv3 --pmc $SQC --output-format csv -d "$OUT/sq_can" -o run -- python tools/kbench.py --op can --ticks 30
           ;;
  esac
done
echo "=== profile session done"
