# bench three times (diagnostic: value, ms_per_step, GPU region, host split, K=1)
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_$i.log 2>&1 || exit $?
  grep '^{' gpurun_out/bench_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['timed_region_ms_per_step'], d['timed_region_host'], d['ensemble_every_1']['ms_per_step'])"
done
