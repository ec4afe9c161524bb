#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wino.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_wino.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_wino.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --breakdown 1 --cpu-baseline 0 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/bench_c2.json')); print(round(d['value'],2), round(d['ms_per_step'],3), d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['mfma_executed_frac'], d['epe_px']['max_over_ranks'])"; grep -v amdgpu.ids gpurun_out/bench_c2.err | head -14; exit $rc
