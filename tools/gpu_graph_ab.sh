#!/bin/bash
# same-box A/B of bench.py's eager launches vs a HIP-graph replay of the forward (C2)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2 3; do
  for g in 0 1; do
    timeout -k 10 200 python3 bench.py --graph $g --steps 50 --warmup 5 --cpu-baseline 0 --epe 0 --pair-check 0 --extra-configs= \
      > gpurun_out/graph_ab_${g}_$i.json 2> gpurun_out/graph_ab_${g}_$i.err || { tail -5 gpurun_out/graph_ab_${g}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/graph_ab_${g}_$i.json')); print('graph=$g run $i', round(d['value'],2), round(d['ms_per_step'],3), d['step_ms'] if 'step_ms' in d else '')"
  done
done
