#!/bin/bash
# Same-box A/B of bench.py configs under environment switches:
#   AB_A / AB_B = env assignments (e.g. "LEASTEREO_WINO2_WALK=1"), CONFIGS, ROUNDS
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in ${CONFIGS:-c2}; do
    for side in A B; do
      if [ $side = A ]; then envs="${AB_A:-}"; else envs="${AB_B:-}"; fi
      env $envs timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 --cpu-baseline 0 --epe 0 --pair-check 0 \
        > gpurun_out/ab_${side}_${c}_$r.json 2> gpurun_out/ab_${side}_${c}_$r.err
      rc=$?; [ $rc -eq 0 ] || { echo "bench $side $c rc=$rc"; tail -3 gpurun_out/ab_${side}_${c}_$r.err; exit $rc; }
      python3 -c "import json; d=json.load(open('gpurun_out/ab_${side}_${c}_$r.json')); print('$r $side [$envs] $c', round(d['value'],1), round(d['step_ms']['median'],3))"
    done
  done
done
