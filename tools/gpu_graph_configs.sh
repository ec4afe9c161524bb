#!/bin/bash
# bench.py's default (HIP-graph replay) on every config, plus the bench tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in c2 c3 c4 c5; do
  timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 3 --cpu-baseline 0 > gpurun_out/graph_$c.json 2> gpurun_out/graph_$c.err \
    || { tail -8 gpurun_out/graph_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/graph_$c.json')); print('$c', round(d['value'],1), round(d['ms_per_step'],3), d['config'].get('launch'), round(d['roofline']['frac'],3), d.get('pair_check', {}).get('max') if isinstance(d.get('pair_check'), dict) else '')"
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bench.py tests/test_gpu_wino.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_bench.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_bench.log; exit $rc
