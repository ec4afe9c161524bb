#!/bin/bash
# Round 4 (k): the few-channel 2D tile -- parity + training tests, per-launch list, and a
# same-box bench A/B of this round's new defaults against their previous values
# (old: LEASTEREO_CONV2D_SMALL=0 LEASTEREO_RESAMPLE_MODE=1 LEASTEREO_WINO_FENCE=0).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_training.py -x -q --timeout 120 \
  --timeout-method thread -k "conv2d or resample or feature or whole_model or train" > gpurun_out/r04_k_tests.txt 2>&1 \
  || { tail -30 gpurun_out/r04_k_tests.txt; exit 1; }
tail -1 gpurun_out/r04_k_tests.txt
timeout -k 10 300 python -u tools/layer_list.py --reps 5 > gpurun_out/r04_k_layer_list.txt 2>&1 || { tail -20 gpurun_out/r04_k_layer_list.txt; exit 1; }
grep "conv2d_small\|conv launches" gpurun_out/r04_k_layer_list.txt | head -40
for side in old new old new; do
  if [ $side = old ]; then export LEASTEREO_CONV2D_SMALL=0 LEASTEREO_RESAMPLE_MODE=1 LEASTEREO_WINO_FENCE=0
  else unset LEASTEREO_CONV2D_SMALL LEASTEREO_RESAMPLE_MODE LEASTEREO_WINO_FENCE; fi
  timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --cpu-baseline 0 --epe 0 > gpurun_out/r04_k_bench_$side.json 2> gpurun_out/r04_k_bench_$side.err \
    || { tail -20 gpurun_out/r04_k_bench_$side.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'])" gpurun_out/r04_k_bench_$side.json $side
done
