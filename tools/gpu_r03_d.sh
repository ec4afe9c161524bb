#!/bin/bash
# Round 3: the one-barrier pipelined W x D tile -- tests, then same-box A/B and breakdown.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wino.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_wino.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_wino.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/wino2_sweep.py --variants 0 --iters 20 \
  --only stem1_32to32_k3_L0,conv12_128to64_k3_L1,cell_32to32_k3_L2,cell_32to96_k3_L2_s1grp,cell_8to24_k3_L0_s1grp,stem1_32to32_k3_L0 \
  > gpurun_out/sweep_pipe.txt 2>&1
rc=$?; grep -v "^{" gpurun_out/sweep_pipe.txt | grep -v amdgpu.ids | cut -c1-140; [ $rc -eq 0 ] || exit $rc
LEASTEREO_WINO2_PIPE=0 timeout -k 10 200 python3 tools/wino2_sweep.py --variants 0 --iters 20 \
  --only stem1_32to32_k3_L0,conv12_128to64_k3_L1,cell_32to32_k3_L2,cell_32to96_k3_L2_s1grp,cell_8to24_k3_L0_s1grp,stem1_32to32_k3_L0 \
  > gpurun_out/sweep_nopipe.txt 2>&1
rc=$?; grep -v "^{" gpurun_out/sweep_nopipe.txt | grep -v amdgpu.ids | cut -c1-140; [ $rc -eq 0 ] || exit $rc
AB_A="LEASTEREO_WINO2_PIPE=0" AB_B="LEASTEREO_WINO2_PIPE=1" ROUNDS=2 CONFIGS=c2 bash tools/gpu_ab.sh
