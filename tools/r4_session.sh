#!/usr/bin/env bash
# Round-4 GPU session: parity tests, the driver's bench command, its rocprofv3 kernel trace,
# and FETCH_SIZE / WRITE_SIZE passes (one counter per run) of the path-row kernels at 2^20.
# Each GPU step has its own limit; a crash / abort / timeout (rc not in {0,1}) ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT"
STEPS="${STEPS:-tests bench prof pmc}"
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
    tests) if [ -n "${PYTEST_K:-}" ]; then KARGS=(-k "$PYTEST_K"); else KARGS=(); fi
           run pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -rf "${KARGS[@]}" ;;
    bench) run bench 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    prof)  run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
             python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline ;;
    pmc)   for c in FETCH_SIZE WRITE_SIZE; do
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
    sqab)  # wave-state counters per SQ_LIST entry "name|VAR=v ...|kbench args" (';'-separated)
           SQC="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
           IFS=';' read -ra SQL <<< "${SQ_LIST:-}"; for ent in "${SQL[@]}"; do
             IFS='|' read -r nm ev ka <<< "$ent"
             for kv in $ev; do export "$kv"; done
             run sq_$nm 120 rocprofv3 --pmc $SQC --output-format csv -d "$OUT/sq_$nm" -o run -- python tools/kbench.py $ka
             for kv in $ev; do unset "${kv%%=*}"; done
           done ;;
    sq)    # one pass of wave-state counters per path-row kernel (7 SQ + 1 GRBM: within one pass)
           SQC="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
           run sq_kf6 120 rocprofv3 --pmc $SQC --output-format csv -d "$OUT/sq_kf6" -o run -- python tools/kbench.py --packed --ticks 30
           run sq_rs 120 rocprofv3 --pmc $SQC --output-format csv -d "$OUT/sq_rs" -o run -- python tools/kbench.py --model rs --pad 512 --ticks 30
           run sq_wt901 120 rocprofv3 --pmc $SQC --output-format csv -d "$OUT/sq_wt901" -o run -- python tools/kbench.py --op wt901 --ticks 30
           run sq_can 120 rocprofv3 --pmc $SQC --output-format csv -d "$OUT/sq_can" -o run -- python tools/kbench.py --op can --ticks 30
           ;;
    mix)   # streaming ceilings of the path rows' byte mixes (tools/membench.hip k_mix) at 2^20 and 2^22
           [ -x build/membench ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/membench.hip -o build/membench
           run mix20 120 build/membench 20 1 mix
           run mix22 120 build/membench 22 1 mix ;;
    kb)    # KB_LIST: entries separated by ';', each "[VAR=value ...] kbench args"; KB_PASSES passes
           for p in $(seq 1 "${KB_PASSES:-1}"); do
             i=0; IFS=';' read -ra KBL <<< "${KB_LIST:-}"; for ent in "${KBL[@]}"; do
               i=$((i+1)); envs=(); args=()
               for w in $ent; do
                 if [[ "$w" == *=* && ${#args[@]} -eq 0 ]]; then envs+=("$w"); else args+=("$w"); fi
               done
               run kb${p}_$i 240 env "${envs[@]}" python tools/kbench.py "${args[@]}"
               echo "{\"pass\": $p, \"env\": \"${envs[*]}\", \"args\": \"${args[*]}\", \"out\": $(tail -n 1 $OUT/kb${p}_$i.log)}" >> "$OUT/kb.jsonl"
             done
           done ;;
  esac
done
echo "=== session done"
