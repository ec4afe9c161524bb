#!/bin/bash
# bf16 parity tests, then the D-streaming vs tile kernel comparison on the single-chunk layers
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_bf16.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_bf16.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bf16_stream_bench.py > gpurun_out/bf16_stream.txt 2>&1
rc=$?; grep -v amdgpu gpurun_out/bf16_stream.txt; exit $rc
