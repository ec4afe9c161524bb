#!/bin/bash
# Winograd engine: its parity tests, the end-to-end parity file, then the c2 bench with breakdown
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wino.py -x -q -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_wino.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_wino.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_parity.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --breakdown 1 --cpu-baseline 0 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
rc=$?; cat gpurun_out/bench_c2.json; grep -v amdgpu.ids gpurun_out/bench_c2.err | head -24; exit $rc
