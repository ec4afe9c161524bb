#!/bin/bash
# scratch lease script for the current experiment (overwritten per experiment; results
# worth keeping are copied into profiles/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench.py -x -q -m gpu --timeout 200 --timeout-method thread -k "e2e or full or bench or c1" > gpurun_out/t_q.log 2>&1
rc=$?; tail -2 gpurun_out/t_q.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-baseline 0 --epe 0 --pair-check 0 > gpurun_out/q.json 2> gpurun_out/q.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/q.err; exit $rc; }
  python3 -c "import json; d=json.load(open('gpurun_out/q.json')); print('c2', round(d['value'],1), round(d['step_ms']['median'],3), round(d['roofline']['frac'],3))"
done
