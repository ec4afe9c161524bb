#!/bin/bash
# Round 4 (b): the per-lane 16-byte halo tile (PV = 4) -- bit-identity tests, then the C2
# forward's per-kernel breakdown with the tile on and off (same box); the bf16 batch-8
# tests recording the HIP figures (LEA_BF16_RECORD=1).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_wino.py -x -q --timeout 120 --timeout-method thread \
  -k "lane_halo16 or wino2_vs_torch or depth_walk or buffer_epilogue or e2e_golden" > gpurun_out/r04_b_wino.txt 2>&1 \
  || { tail -30 gpurun_out/r04_b_wino.txt; exit 1; }
tail -1 gpurun_out/r04_b_wino.txt
for on in 1 0 1 0; do
  LEASTEREO_LANE_HALO16=$on timeout -k 10 300 python -u bench.py --breakdown 1 --cpu-baseline 0 --gpu-eager "" \
    --pair-check 0 --epe 0 --steps 30 > gpurun_out/r04_b_bench_$on.json 2> gpurun_out/r04_b_bench_$on.err \
    || { tail -20 gpurun_out/r04_b_bench_$on.err; exit 1; }
  echo "lane16=$on $(python -c "import json;d=json.loads(open('gpurun_out/r04_b_bench_$on.json').read());print(round(d['value'],2), round(d['step_ms']['median'],3))")"
  grep "conv3d_wino2_kernel<8, 1, 1" gpurun_out/r04_b_bench_$on.err
done
LEA_BF16_RECORD=1 timeout -k 10 1500 python -u -m pytest tests/test_gpu_bf16.py -x -v --timeout 1400 --timeout-method thread \
  -k "batch8" > gpurun_out/r04_b_bf16.txt 2>&1 || { tail -30 gpurun_out/r04_b_bf16.txt; exit 1; }
tail -3 gpurun_out/r04_b_bf16.txt
cat gpurun_out/bf16_hip_measured.json | head -60
