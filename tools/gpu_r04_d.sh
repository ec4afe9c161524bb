#!/bin/bash
# Round 4 (d): planner audit -- every f32 3x3x3 layer shape at C2 on each Winograd tile
# variant and depth walk (tools/wino2_sweep.py), the bf16 batch-8 tests with the recorded
# figures (error-injection checks), the default bench line.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/wino2_sweep.py --variants 0,1,5,6,7 --walks 0,1,2,4 --iters 10 \
  > gpurun_out/r04_d_sweep.txt 2>&1 || { tail -20 gpurun_out/r04_d_sweep.txt; exit 1; }
grep -v "^{" gpurun_out/r04_d_sweep.txt | grep -v amdgpu.ids | cut -c1-140
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py -x -q --timeout 500 --timeout-method thread \
  -k "batch8" > gpurun_out/r04_d_bf16.txt 2>&1 || { tail -30 gpurun_out/r04_d_bf16.txt; exit 1; }
tail -1 gpurun_out/r04_d_bf16.txt
