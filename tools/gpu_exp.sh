#!/bin/bash
# scratch lease script for the current experiment (overwritten per experiment; results
# worth keeping are copied into profiles/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bf16.py -x -q -m gpu --timeout 120 --timeout-method thread -k "disp or e2e or c1 or full or batch or tapsum" > gpurun_out/t_disp.log 2>&1
rc=$?; tail -2 gpurun_out/t_disp.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for c in c2 c4; do for v in 0 1; do
  LEASTEREO_TAPSUM_ROWS=$v timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 3 --breakdown 1 --cpu-baseline 0 --epe 0 --pair-check 0 \
    > gpurun_out/d_$v.json 2> gpurun_out/d_$v.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/d_$v.err; exit $rc; }
  python3 -c "import json; d=json.load(open('gpurun_out/d_$v.json')); print('$c rows=$v', round(d['value'],1), round(d['step_ms']['median'],3))"
  grep tapsum gpurun_out/d_$v.err | head -2
done; done; done
