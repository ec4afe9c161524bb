#!/bin/bash
# Round 4 (q): batched staging loads in the feature stem and the row-staged tap-sum pass --
# tests (feature net, heads, e2e), per-launch list, same-box C2 bench A/B against
# ab/lib_head.so (the previous commit).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_heads.py tests/test_gpu_bf16.py -x -q --timeout 300 \
  --timeout-method thread -k "feature or stem or tapsum or head or e2e or golden or resampled or conv_resampled" > gpurun_out/r04_q_tests.txt 2>&1 \
  || { tail -30 gpurun_out/r04_q_tests.txt; exit 1; }
tail -1 gpurun_out/r04_q_tests.txt
timeout -k 10 300 python -u tools/layer_list.py --reps 5 > gpurun_out/r04_q_layer_list.txt 2>&1 || { tail -20 gpurun_out/r04_q_layer_list.txt; exit 1; }
grep "feature_stem\|tapsum\|conv3d_reg\|conv launches" gpurun_out/r04_q_layer_list.txt
for side in old new old new; do
  if [ $side = old ]; then export LEASTEREO_HIP_LIB=$PWD/ab/lib_head.so; else unset LEASTEREO_HIP_LIB; fi
  timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --cpu-baseline 0 --epe 0 > gpurun_out/r04_q_bench_$side.json 2> gpurun_out/r04_q_bench_$side.err \
    || { tail -20 gpurun_out/r04_q_bench_$side.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r04_q_bench_$side.json $side
done
