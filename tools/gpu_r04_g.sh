#!/bin/bash
# Round 4 (g): the per-lane tile's fenced step schedule (PV = 5) vs PV = 4.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wino.py -x -q --timeout 120 --timeout-method thread -k lane_halo16 \
  > gpurun_out/r04_g_tests.txt 2>&1 || { tail -30 gpurun_out/r04_g_tests.txt; exit 1; }
tail -1 gpurun_out/r04_g_tests.txt
for v in 1 2 1 2; do
  LEASTEREO_LANE_HALO16=$v timeout -k 10 200 python -u tools/wino2_sweep.py --variants 0 --walks 0,2 --iters 30 \
    --only cell_16to16_k3_L1 > gpurun_out/r04_g_sweep_$v.txt 2>&1 || { tail -20 gpurun_out/r04_g_sweep_$v.txt; exit 1; }
  grep -v "^{" gpurun_out/r04_g_sweep_$v.txt | grep -v amdgpu.ids | cut -c1-130
done
