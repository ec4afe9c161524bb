#!/bin/bash
# Round 4 (s): where the small-launch (L2, 1/12 resolution) layers of the pipelined tile spend
# their time -- phase ablations (timing only) on the L2 32->32 cell op and 32->96 group, with
# conv1/2 and the L1 16->16 per-lane tile for reference; depth-walk sweep of the L2 layers.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export VARS="base: nohalo: nowdma: novpass: nobar1: nomfma: nouxf: noldsrd: mfmaonly: skel:"
ONLY=cell_32to32_k3_L2,cell_32to96_k3_L2_s1grp,conv12_128to64_k3_L1,cell_16to16_k3_L1 bash tools/wino2_ablate.sh run \
  > gpurun_out/r04_s_ablate.txt 2>&1 || { tail -20 gpurun_out/r04_s_ablate.txt; exit 1; }
cat gpurun_out/r04_s_ablate.txt
timeout -k 10 200 python3 tools/wino2_sweep.py --variants 0 --iters 20 --walks 1,2,4 \
  --only cell_32to32_k3_L2,cell_32to96_k3_L2_s1grp,cell_16to16_k3_L1 > gpurun_out/r04_s_walks.txt 2>&1 \
  || { tail -20 gpurun_out/r04_s_walks.txt; exit 1; }
grep -v "^{" gpurun_out/r04_s_walks.txt | grep -v amdgpu.ids | cut -c1-150
