#!/bin/bash
# Round 3: the W x D engine's 16-byte halo staging -- tests, phase stamps, same-box A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wino.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_wino.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_wino.log; [ $rc -eq 0 ] || exit $rc
LEASTEREO_HIP_LIB=leastereo_amd/var_stamps.so timeout -k 10 300 python3 tools/wino2_stamps.py \
  > gpurun_out/stamps_h16.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/stamps_h16.txt | cut -c1-330; [ $rc -eq 0 ] || exit $rc
AB_A="LEASTEREO_HALO16=0" AB_B="LEASTEREO_HALO16=1" ROUNDS=2 CONFIGS=c2 bash tools/gpu_ab.sh
