#!/bin/bash
# Re-validation of HEAD: parity tests, c2 bench (default workload), c3/c4 bf16 benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
for c in c2 c3 c4; do
  timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 5 --breakdown 1 --cpu-baseline $([ $c = c2 ] && echo 1 || echo 0) \
    > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err
  rc=$?; cat gpurun_out/bench_$c.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_$c.err; exit $rc; }
done
