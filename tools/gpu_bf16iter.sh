#!/bin/bash
# bf16 engine iteration: bf16 + evalio parity tests, c4/c3 benches with per-kernel breakdown
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_evalio.py -x -q -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_iter.log 2>&1
rc=$?; tail -8 gpurun_out/pytest_iter.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/bf16_layer_bench.py 2>/dev/null; rc=$?; [ $rc -eq 0 ] || exit $rc

for c in ${CONFIGS:-c4 c3}; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --breakdown 1 --cpu-baseline 0 \
    > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err
  rc=$?; python -c "import json,sys; d=json.load(open('gpurun_out/bench_$c.json')); print('$c', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('path_roofline',{}).get('frac'), d['epe_px']['max_over_ranks'])"
  [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_$c.err; exit $rc; }
  grep -v amdgpu.ids gpurun_out/bench_$c.err | head -14
done
