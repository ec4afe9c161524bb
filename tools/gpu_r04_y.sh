#!/bin/bash
# Round 4 (y): a feature cell's two ops on s0 as one launch (lea_conv2d_bnrelu_pair), op2 with them (lea_conv2d_bnrelu_split) -- 2D / feature /
# e2e / capi tests, per-launch list, same-box C2 bench A/B: LEASTEREO_PAIR_S0=2 (the pair alone) vs the default.


set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_capi.py -x -q --timeout 300 \
  --timeout-method thread -k "conv2d or feature or e2e or golden or pair or split or capi" > gpurun_out/r04_y_tests.txt 2>&1 \
  || { tail -30 gpurun_out/r04_y_tests.txt; exit 1; }
tail -1 gpurun_out/r04_y_tests.txt
timeout -k 10 300 python -u tools/layer_list.py --reps 5 > gpurun_out/r04_y_layer_list.txt 2>&1 || { tail -20 gpurun_out/r04_y_layer_list.txt; exit 1; }
grep "conv2d_small\|conv launches" gpurun_out/r04_y_layer_list.txt | sort -k7 | uniq -c -f6 | head -6
for side in old new old new; do
  if [ $side = old ]; then export LEASTEREO_PAIR_S0=2; else unset LEASTEREO_PAIR_S0; fi
  timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --cpu-baseline 0 --epe 0 > gpurun_out/r04_y_bench_$side.json 2> gpurun_out/r04_y_bench_$side.err \
    || { tail -20 gpurun_out/r04_y_bench_$side.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r04_y_bench_$side.json $side
done
