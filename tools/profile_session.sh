#!/usr/bin/env bash
# GPU-box profiling session for the headline kernel:
#   1. bench.py (the driver's default command) -> gpurun_out/bench.log
#   2. rocprofv3 --kernel-trace --stats of the same bench -> gpurun_out/prof/
#   3. rocprofv3 --pmc FETCH_SIZE and (separate pass) WRITE_SIZE of the tick kernel at the bench
#      shape and of tools/membench.hip's pattern kernel (same access pattern, known bytes:
#      the calibration the MI355X guide asks for before trusting absolute counter values)
# Each GPU step has its own limit; a crash/timeout (rc not in {0,1}) ends the session.
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
  tail -n 4 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "!!! stopping"; exit $rc; fi
}
[ -x build/membench ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/membench.hip -o build/membench
run bench 600 python bench.py --gpus 1 --steps 20 --warmup 5
# the driver's command under the kernel trace (its secondary cfg 3 / 5 / 2^24 lines included)
run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
for c in FETCH_SIZE WRITE_SIZE; do
  run pmc_kf6_$c 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_kf6_$c" -o run -- \
    python tools/kbench.py --ticks 30 --packed
  run pmc_pat_$c 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_pat_$c" -o run -- \
    build/membench 20
done
# the HBM-regime secondary lines (cfg 3, cfg 5, KF6 at 2^24): tick kernels and their
# same-width calibration patterns, one counter per pass (PMC_SEC=1)
if [ "${PMC_SEC:-0}" = 1 ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    run pmc_sec_pattern_$c 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_sec_pattern_$c" -o run -- \
      build/membench 22 1 caps
    run pmc_sec_cfg3_ekf9_2p22_$c 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_sec_cfg3_ekf9_2p22_$c" -o run -- \
      python tools/kbench.py --model ekf9 --n 4194304 --ticks 8
    run pmc_sec_cfg5_kf12d_2p20_$c 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_sec_cfg5_kf12d_2p20_$c" -o run -- \
      python tools/kbench.py --model kf12d --ticks 8
    run pmc_sec_cfg2_kf6_2p24_$c 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_sec_cfg2_kf6_2p24_$c" -o run -- \
      python tools/kbench.py --model kf6 --packed --n 16777216 --ticks 6
  done
fi
echo "=== session done"
# secondary rows: every tick model and the rows either side of the tick, one rocprofv3 kernel
# trace each (PROF_ALL=1)
if [ "${PROF_ALL:-0}" = 1 ]; then
  for spec in "kf6_2p24:--model kf6 --packed --n 16777216 --ticks 20" "kf6_planes:--model kf6 --ring 64 --ticks 200" \
              "kf6_2p21:--model kf6 --packed --n 2097152 --ticks 100" "isr_rs:--model rs --op isr --ticks 200" \
              "ekf9:--model ekf9 --ticks 100" \
              "ekf9_2p22:--model ekf9 --n 4194304 --ticks 30" "kf12d:--model kf12d --ticks 30" \
              "rs:--model rs --ticks 200" "control:--op control --ticks 100" "control_2p22:--op control --n 4194304 --ticks 30" \
              "wt901:--op wt901 --ticks 50" "can:--op can --ticks 100" "ensemble:--op ensemble --ticks 100" \
              "ens_ekf9:--op ensemble --model ekf9 --ticks 100" "ens_kf12d:--op ensemble --model kf12d --ticks 50" \
              "ens_ekf9_2p22:--op ensemble --model ekf9 --n 4194304 --ticks 50" "rs_2p24:--model rs --n 16777216 --ticks 20" \
              "pipeline_graph_4096:--op pipeline_graph --n 4096 --ticks 1000" \
              "tick_ens_kf6:--model kf6 --packed --op tick_ensemble --ticks 100" \
              "tick_ens_ekf9:--model ekf9 --op tick_ensemble --ticks 100" \
              "tick_ens_kf12d:--model kf12d --op tick_ensemble --ticks 30" \
              "isr_kf6:--model kf6 --packed --op isr --ticks 200" \
              "isr_kf6_4096:--model kf6 --packed --op isr --n 4096 --ticks 1000"; do
    name=${spec%%:*}; args=${spec#*:}
    run prof_$name 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o run -- \
      python tools/kbench.py $args
  done
fi
echo "=== session done (all)"
