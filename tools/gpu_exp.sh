#!/bin/bash
# scratch lease script for the current experiment (overwritten per experiment; results
# worth keeping are copied into profiles/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_heads.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_split.log 2>&1
rc=$?; tail -2 gpurun_out/t_split.log; [ $rc -eq 0 ] || exit $rc
AB_A="LEASTEREO_SPLIT_GROUP48=0" AB_B="LEASTEREO_SPLIT_GROUP48=1" ROUNDS=3 bash tools/gpu_ab.sh
