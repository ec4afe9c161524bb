#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wino.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_wino.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_wino.log; [ $rc -eq 0 ] || exit $rc
for gr in 1 0; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-baseline 0 --graph $gr > gpurun_out/bench_graph$gr.json 2> gpurun_out/bench_graph$gr.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_graph$gr.err; exit $rc; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_graph$gr.json')); print('graph=$gr', round(d['value'],2), round(d['ms_per_step'],3), d['roofline']['frac'])"
done
