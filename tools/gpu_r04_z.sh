#!/bin/bash
# Round 4 (z): depth-walk re-check of the pipelined tile's mid-size launches (L1 16 -> 32 groups, L2
# 32 -> 96 groups, L1 16 -> 16 per-lane tile): each walk measured twice in one process (the first rows
# of a process run at a lower clock).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/wino2_sweep.py --variants 0 --iters 40 --walks 4,1,2,4,1,2 \
  --only conv12_128to64_k3_L1,cell_16to32_k3_L1_s1grp2,cell_32to96_k3_L2_s1grp,cell_16to16_k3_L1 > gpurun_out/r04_z_walks.txt 2>&1 \
  || { tail -20 gpurun_out/r04_z_walks.txt; exit 1; }
grep -v "^{" gpurun_out/r04_z_walks.txt | grep -v amdgpu.ids | cut -c1-150
