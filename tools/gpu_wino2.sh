#!/bin/bash
# W x D Winograd engine: its parity tests (wino2 cases only), then the variant sweep
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wino.py -x -q -m gpu -k wino2 --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_wino2.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_wino2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/wino2_sweep.py --iters 10 ${SWEEP_ARGS:-} > gpurun_out/wino2_sweep.txt 2> gpurun_out/wino2_sweep.err
rc=$?; grep -v '^{' gpurun_out/wino2_sweep.txt; tail -3 gpurun_out/wino2_sweep.err; exit $rc
