#!/bin/bash
# Round 3: tests; L2 32->32 cells on the pipelined W x D tile (A/B on WINO_MIN_VOXELS);
# 48-cout blocks on the W x D tile (sweep)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wino.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_wino.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_wino.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/wino2_sweep.py --variants 0 --iters 20 --block48 1,0 \
  --only stem1_32to32_k3_L0,cell_16to48_k3_L1_s1grp,cell_16to16_k3_L1,cell_8to8_k3_L0 > gpurun_out/sweep_b48.txt 2>&1
rc=$?; grep -v "^{" gpurun_out/sweep_b48.txt | grep -v amdgpu.ids | cut -c1-150; [ $rc -eq 0 ] || exit $rc
AB_A="LEASTEREO_X=0" AB_B="LEASTEREO_WINO_MIN_VOXELS=0" ROUNDS=2 CONFIGS=c2 bash tools/gpu_ab.sh
