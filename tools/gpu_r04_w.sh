#!/bin/bash
# Round 4 (w): planner re-check of the L0 cell ops after the round's kernel changes -- the
# 8 -> 8 cells on the depth-paired 1-D tile vs 16-row W x D blocks and depth walks, the 8 -> 24
# group on the two-barrier tile vs the pipeline (LEASTEREO_WINO2_PIPE=2), walks.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/wino2_sweep.py --variants 0 --iters 20 --small 0,1 --walks 0,1,2,4 \
  --only cell_8to8_k3_L0 > gpurun_out/r04_w_8to8.txt 2>&1 || { tail -20 gpurun_out/r04_w_8to8.txt; exit 1; }
grep -v "^{" gpurun_out/r04_w_8to8.txt | grep -v amdgpu.ids | cut -c1-150
for pipe in 1 2; do
  LEASTEREO_WINO2_PIPE=$pipe timeout -k 10 200 python3 tools/wino2_sweep.py --variants 0 --iters 20 --walks 0,1,2,4 \
    --only cell_8to24_k3_L0_s1grp > gpurun_out/r04_w_8to24_$pipe.txt 2>&1 || { tail -20 gpurun_out/r04_w_8to24_$pipe.txt; exit 1; }
  grep -v "^{" gpurun_out/r04_w_8to24_$pipe.txt | grep -v amdgpu.ids | sed "s/^/pipe=$pipe /" | cut -c1-150
done
