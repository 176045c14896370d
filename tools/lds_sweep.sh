# the plain k_kf6p tick at the launcher's default cap against the 32 KiB cap, alternating
cd "${GRAFT_REPO_ROOT}"
for r in 1 2 3; do
  for b in default 32768; do
    printf "%s " "$b"
    if [ $b = default ]; then envs=""; else envs="FMSKF_KF6P_LDS=$b"; fi
    env $envs timeout -k 10 120 python tools/kbench.py --packed --ticks 400 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_tick']*1e3,2))" || exit 1
  done
done
