#!/bin/bash
# Round 4 (n): separable c8 resample -- bf16 resample tests, per-launch list at C4, and a
# same-box C4 / C3 bench A/B (LEASTEREO_RESAMPLE_K=0: the gather kernel's default).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py -x -q --timeout 300 --timeout-method thread -k "resample or conv1x1_resampled" \
  > gpurun_out/r04_n_tests.txt 2>&1 || { tail -30 gpurun_out/r04_n_tests.txt; exit 1; }
tail -1 gpurun_out/r04_n_tests.txt
timeout -k 10 300 python -u tools/layer_list.py --config c4 --reps 3 > gpurun_out/r04_n_layer_list_c4.txt 2>&1 || { tail -20 gpurun_out/r04_n_layer_list_c4.txt; exit 1; }
grep "resample\|conv launches" gpurun_out/r04_n_layer_list_c4.txt
for c in c4 c3; do
for side in old new old new; do
  if [ $side = old ]; then export LEASTEREO_RESAMPLE_K=0; else unset LEASTEREO_RESAMPLE_K; fi
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 --cpu-baseline 0 --epe 0 > gpurun_out/r04_n_bench_${c}_$side.json 2> gpurun_out/r04_n_bench_${c}_$side.err \
    || { tail -20 gpurun_out/r04_n_bench_${c}_$side.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r04_n_bench_${c}_$side.json "$c $side"
done
done
