#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wino.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_wino.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_wino.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 tools/wino2_sweep.py --iters 10 --variants 5 ${SWEEP:-} > gpurun_out/walk_sweep2.txt 2>&1
rc=$?; grep -v amdgpu gpurun_out/walk_sweep2.txt | grep -v '^{'; exit $rc
