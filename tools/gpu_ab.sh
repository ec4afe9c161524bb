#!/bin/bash
# Same-box A/B(/C...) of bench.py configs under environment switches, interleaved ROUNDS times:
#   AB_A / AB_B = env assignments (e.g. "LEASTEREO_WINO2_WALK=1"), or AB_VARIANTS = "envs;envs;..."
#   (',' inside a variant separates assignments), CONFIGS, ROUNDS, STEPS
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "${AB_VARIANTS:-}" ]; then IFS=';' read -r -a VARS <<< "$AB_VARIANTS"; else VARS=("${AB_A:-}" "${AB_B:-}"); fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in ${CONFIGS:-c2}; do
    # reverse the variant order on even rounds so a first-run/second-run bias cancels
    idx=("${!VARS[@]}"); [ $((r % 2)) -eq 0 ] && idx=($(printf '%s\n' "${idx[@]}" | tac))
    for i in "${idx[@]}"; do
      envs=$(echo "${VARS[$i]}" | tr ',' ' ')
      env $envs timeout -k 10 300 python3 bench.py --config $c --steps ${STEPS:-20} --warmup 5 --cpu-baseline 0 --epe 0 --pair-check 0 --extra-configs "" \
        > gpurun_out/ab_${i}_${c}_$r.json 2> gpurun_out/ab_${i}_${c}_$r.err
      rc=$?; [ $rc -eq 0 ] || { echo "bench $i $c rc=$rc"; tail -3 gpurun_out/ab_${i}_${c}_$r.err; exit $rc; }
      python3 -c "import json; d=json.load(open('gpurun_out/ab_${i}_${c}_$r.json')); print('$r $i [$envs] $c', round(d['value'],1), round(d['step_ms']['median'],3))"
    done
  done
done
