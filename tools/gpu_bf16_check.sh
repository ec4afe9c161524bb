#!/bin/bash
# bf16 parity tests, then the c4 forward under rocprofv3 and a c3/c4 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_bf16.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_bf16.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof_c4.sh || exit $?
for c in c3 c4; do
  timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$c.err; exit $rc; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_$c.json')); print('$c', round(d['value'],1), round(d['ms_per_step'],2), d['epe_px']['max_over_ranks'])"
done
