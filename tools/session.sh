#!/usr/bin/env bash
# One GPU-box session, parametrised by STEPS (run on the box through gpurun):
#   STEPS="smoke tests bench" tools/session.sh
# Steps:
#   smoke   __graft_entry__.smoke()
#   tests   the -m gpu suite (PYTEST_K narrows it)
#   bench   the driver's bench command (BENCH_ARGS replaces its arguments)
#   prof    rocprofv3 --kernel-trace --stats of the driver's bench command
#   pmc     FETCH_SIZE / WRITE_SIZE passes of the headline kernel and its calibration pattern
#   sec     the same for the HBM-regime secondary lines (cfg 3, cfg 5, KF6 2^24)
#   paths   the same for the path rows at 2^20 (RS, WT901, CAN, COMP KF6, the fused ISR with / without CAN)
#   sq      wave-state counters (7 SQ + GRBM, one pass) of the tick and path-row kernels
#   sqab    the same per SQ_LIST entry "name|VAR=v ...|kbench args" (';'-separated)
#   mix     tools/membench.hip byte-mix streaming ceilings at 2^20 and 2^22
#   kb      tools/kbench.py per KB_LIST entry "[VAR=v ...] kbench args" (';'-separated),
#           KB_PASSES passes, one JSON line per run appended to gpurun_out/kb.jsonl
#   dist1   the distributed code at world 1 under torch.distributed.run (real RCCL, native gather)
#   world4  four ranks on the one GPU through the loopback RCCL stand-in (rehearsal of the
#           driver's --gpus N line; rates meaningless)
# Each GPU step runs under its own time limit; a crash / abort / timeout (rc not in {0, 1})
# ends the session: no further GPU work after a fault.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT" build
STEPS="${STEPS:-smoke tests bench}"
SQC="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
DRIVER=(python bench.py --gpus 1 --steps 20 --warmup 5)

run() {  # name limit cmd...
  local name=$1 limit=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 3 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "!!! $name ended with rc=$rc: stopping the session"
    exit $rc
  fi
  return 0
}

pmc2() {  # name limit kbench-args...: one FETCH_SIZE and one WRITE_SIZE pass of a kbench run
  local name=$1 limit=$2; shift 2
  for c in FETCH_SIZE WRITE_SIZE; do
    run ${name}_$c "$limit" rocprofv3 --pmc $c --output-format csv -d "$OUT/${name}_$c" -o run -- \
      python tools/kbench.py "$@"
  done
}

membench() {
  [ -x build/membench ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/membench.hip -o build/membench
}

for s in $STEPS; do
  case $s in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) if [ -n "${PYTEST_K:-}" ]; then KARGS=(-k "$PYTEST_K"); else KARGS=(); fi
           run pytest_gpu 1100 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
             -rf "${KARGS[@]}" ;;
    bench) if [ -n "${BENCH_ARGS:-}" ]; then run bench 600 python bench.py $BENCH_ARGS
           else run bench 600 "${DRIVER[@]}"; fi ;;
    prof)  run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
             "${DRIVER[@]}" --no-cpu-baseline ;;
    pmc)   membench
           pmc2 pmc_kf6 300 --ticks 30 --packed
           for c in FETCH_SIZE WRITE_SIZE; do
             run pmc_pat_$c 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_pat_$c" -o run -- build/membench 20
           done ;;
    sec)   membench
           for c in FETCH_SIZE WRITE_SIZE; do
             run pmc_sec_pattern_$c 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_sec_pattern_$c" -o run -- \
               build/membench 22 1 caps
           done
           pmc2 pmc_sec_cfg3_ekf9_2p22 300 --model ekf9 --n 4194304 --ticks 8
           pmc2 pmc_sec_cfg5_kf12d_2p20 300 --model kf12d --ticks 8
           pmc2 pmc_sec_cfg2_kf6_2p24 300 --model kf6 --packed --n 16777216 --ticks 6 ;;
    paths) pmc2 pmc_path_rs_tick_2p20 120 --model rs --ticks 30
           pmc2 pmc_path_rs_tick_2p20_padded_sums 120 --model rs --pad 512 --ticks 30
           pmc2 pmc_path_wt901_ingest_2p20 120 --op wt901 --ticks 30
           pmc2 pmc_path_can_ingest_2p20 120 --op can --ticks 30
           pmc2 pmc_path_control_step_2p20 120 --op control --ticks 30
           pmc2 pmc_path_cfg2_kf6_comp_pos_2p20 120 --packed --comp --ticks 30
           pmc2 pmc_path_isr_kf6_2p20 120 --op isr --ticks 30
           pmc2 pmc_path_isr_can_kf6_2p20 120 --op isr_can --ticks 30
           pmc2 pmc_path_isr_rs_2p20 120 --model rs --op isr --ticks 30
           pmc2 pmc_path_isr_can_rs_2p20 120 --model rs --op isr_can --ticks 30
           pmc2 pmc_path_isr_ekf9_2p20 120 --model ekf9 --op isr --ticks 30
           pmc2 pmc_path_isr_can_ekf9_2p20 120 --model ekf9 --op isr_can --ticks 30 ;;
    sq)    for ent in "kf6|--packed --ticks 30" "rs|--model rs --pad 512 --ticks 30" "wt901|--op wt901 --ticks 30" \
                      "can|--op can --ticks 30"; do
             IFS='|' read -r nm ka <<< "$ent"
             run sq_$nm 120 rocprofv3 --pmc $SQC --output-format csv -d "$OUT/sq_$nm" -o run -- python tools/kbench.py $ka
           done ;;
    sqab)  IFS=';' read -ra SQL <<< "${SQ_LIST:-}"; for ent in "${SQL[@]}"; do
             IFS='|' read -r nm ev ka <<< "$ent"
             for kv in $ev; do export "$kv"; done
             run sq_$nm 120 rocprofv3 --pmc $SQC --output-format csv -d "$OUT/sq_$nm" -o run -- python tools/kbench.py $ka
             for kv in $ev; do unset "${kv%%=*}"; done
           done ;;
    mix)   membench
           run mix20 120 build/membench 20 1 mix
           run mix22 120 build/membench 22 1 mix ;;
    kb)    for p in $(seq 1 "${KB_PASSES:-1}"); do
             i=0; IFS=';' read -ra KBL <<< "${KB_LIST:-}"; for ent in "${KBL[@]}"; do
               i=$((i+1)); envs=(); args=()
               for w in $ent; do
                 if [[ "$w" == *=* && ${#args[@]} -eq 0 ]]; then envs+=("$w"); else args+=("$w"); fi
               done
               run kb${p}_$i 240 env "${envs[@]}" python tools/kbench.py "${args[@]}"
               echo "{\"pass\": $p, \"env\": \"${envs[*]}\", \"args\": \"${args[*]}\", \"out\": $(tail -n 1 $OUT/kb${p}_$i.log)}" >> "$OUT/kb.jsonl"
             done
           done ;;
    dist1) run dist1 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
             --master-port 29531 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline --no-fused --no-secondary ;;
    world4) run world4 600 env FMSKF_RCCL_LIBRARY="$PWD/build/libloopback_rccl.so" LOOPBACK_RCCL_DIR=/tmp \
              LOOPBACK_RCCL_MODE=callback python bench.py --gpus 4 --backend gloo --same-device --gather native \
              --steps 64 --warmup 8 --no-cpu-baseline --no-fused --no-secondary --cfg4-steps 16 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "=== session done"
