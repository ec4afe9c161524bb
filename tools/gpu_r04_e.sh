#!/bin/bash
# Round 4 (e): the C2 L2 32->32 cells on the pipelined W x D tile -- parity tests, then
# same-box A/B of the whole bench (LEASTEREO_WINO_SMALL32_MIN huge = the direct engine).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wino.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r04_e_tests.txt 2>&1 || { tail -30 gpurun_out/r04_e_tests.txt; exit 1; }
tail -1 gpurun_out/r04_e_tests.txt
for v in 32768 1000000000 32768 1000000000 32768 1000000000; do
  LEASTEREO_WINO_SMALL32_MIN=$v timeout -k 10 300 python -u bench.py --breakdown 1 --cpu-baseline 0 --gpu-eager "" \
    --pair-check 0 --epe 0 --steps 50 > gpurun_out/r04_e_bench_$v.json 2> gpurun_out/r04_e_bench_$v.err \
    || { tail -20 gpurun_out/r04_e_bench_$v.err; exit 1; }
  echo "small32_min=$v $(python -c "import json;d=json.loads(open('gpurun_out/r04_e_bench_$v.json').read());print(round(d['value'],2), round(d['step_ms']['median'],3), round(d['roofline']['frac'],3))")"
done
grep -E "conv3d_dma_kernel<2, 2, 16, 1, 3|wino2p" gpurun_out/r04_e_bench_32768.err gpurun_out/r04_e_bench_1000000000.err
