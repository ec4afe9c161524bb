#!/bin/bash
# Round 4 (o): the wide 2D Winograd tile (stem0's maps) -- parity + cv_stem tests, per-launch
# list, same-box C2 bench A/B (LEASTEREO_CONV2D_WINO 0/1).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cv_stem.py -x -q --timeout 300 --timeout-method thread \
  -k "conv2d or cv_stem or e2e or full" > gpurun_out/r04_o_tests.txt 2>&1 || { tail -30 gpurun_out/r04_o_tests.txt; exit 1; }
tail -1 gpurun_out/r04_o_tests.txt
timeout -k 10 300 python -u tools/layer_list.py --reps 5 > gpurun_out/r04_o_layer_list.txt 2>&1 || { tail -20 gpurun_out/r04_o_layer_list.txt; exit 1; }
grep "wino22\|conv3d_dma_kernel<[34]\|conv launches" gpurun_out/r04_o_layer_list.txt
for side in old new old new; do
  if [ $side = old ]; then export LEASTEREO_CONV2D_WINO=0; else unset LEASTEREO_CONV2D_WINO; fi
  timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --cpu-baseline 0 --epe 0 > gpurun_out/r04_o_bench_$side.json 2> gpurun_out/r04_o_bench_$side.err \
    || { tail -20 gpurun_out/r04_o_bench_$side.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r04_o_bench_$side.json $side
done
