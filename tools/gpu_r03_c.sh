#!/bin/bash
# Round 3: cout-block-fastest grid order (A = var_base.so, the previous build) + breakdown.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wino.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_wino.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_wino.log; [ $rc -eq 0 ] || exit $rc
AB_A="LEASTEREO_HIP_LIB=leastereo_amd/var_base.so" AB_B="LEASTEREO_X=1" ROUNDS=2 CONFIGS=c2 bash tools/gpu_ab.sh || exit $?
timeout -k 10 300 python3 bench.py --breakdown 1 --cpu-baseline 0 --epe 0 --pair-check 0 > gpurun_out/bench_bd.json 2> gpurun_out/bench_bd.err
rc=$?; grep -v amdgpu.ids gpurun_out/bench_bd.err | head -30; exit $rc
