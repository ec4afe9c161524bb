#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 180 python3 tools/resample_probe.py > gpurun_out/rs_probe.txt 2>&1; rc=$?; grep -v amdgpu gpurun_out/rs_probe.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -m pytest tests/test_gpu_bf16.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
