#!/bin/bash
# Round 4 (f): b128 halo reads in the per-lane 16-cout tile (PV = 4) and the depth-paired
# 1-D tile -- bit-identity tests, per-layer times, PMC (bank conflicts), same-box bench A/B.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_wino.py tests/test_gpu_parity.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r04_f_tests.txt 2>&1 || { tail -30 gpurun_out/r04_f_tests.txt; exit 1; }
tail -1 gpurun_out/r04_f_tests.txt
timeout -k 10 300 python -u tools/wino2_sweep.py --variants 0 --walks 0 --iters 20 \
  --only stem1_32to32_k3_L0,cell_16to16_k3_L1,cell_8to8_k3_L0,cell_16to16_k3_L1 > gpurun_out/r04_f_sweep.txt 2>&1 \
  || { tail -20 gpurun_out/r04_f_sweep.txt; exit 1; }
grep -v "^{" gpurun_out/r04_f_sweep.txt | grep -v amdgpu.ids | cut -c1-130
SWEEP_ARGS="--variants 0 --only cell_16to16_k3_L1,cell_8to8_k3_L0" FILTERS="conv3d_wino" bash tools/gpu_pmc_layer.sh \
  > gpurun_out/r04_f_pmc.txt 2>&1 || { tail -20 gpurun_out/r04_f_pmc.txt; exit 1; }
grep -E "^lea" gpurun_out/r04_f_pmc.txt
for on in 1 0 1 0; do
  LEASTEREO_LANE_HALO16=$on LEASTEREO_HALO16=$on timeout -k 10 300 python -u bench.py --breakdown 1 --cpu-baseline 0 \
    --gpu-eager "" --pair-check 0 --epe 0 --steps 50 > gpurun_out/r04_f_bench_$on.json 2> gpurun_out/r04_f_bench_$on.err \
    || { tail -20 gpurun_out/r04_f_bench_$on.err; exit 1; }
  echo "b128=$on $(python -c "import json;d=json.loads(open('gpurun_out/r04_f_bench_$on.json').read());print(round(d['value'],2), round(d['step_ms']['median'],3))")"
done
grep -E "conv3d_wino2_kernel<8, 1, 1|conv3d_wino_kernel<4, 16, 0" gpurun_out/r04_f_bench_1.err gpurun_out/r04_f_bench_0.err
