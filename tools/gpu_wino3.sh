#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wino.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_wino.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_wino.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/wino_sweep.py --iters 10 --only cell_16to48_k3_L1_s1grp 2>&1 | grep -v "^{" | grep -v amdgpu.ids
