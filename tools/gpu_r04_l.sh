#!/bin/bash
# Round 4 (l): depth-walking separable resample -- bit identity, per-launch list; same-box
# bench A/B of the few-channel 2D tile alone (LEASTEREO_CONV2D_SMALL) and of the walk
# (LEASTEREO_RESAMPLE_MODE=3: per-plane separable).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "resample" \
  > gpurun_out/r04_l_tests.txt 2>&1 || { tail -30 gpurun_out/r04_l_tests.txt; exit 1; }
tail -1 gpurun_out/r04_l_tests.txt
timeout -k 10 300 python -u tools/layer_list.py --reps 5 > gpurun_out/r04_l_layer_list.txt 2>&1 || { tail -20 gpurun_out/r04_l_layer_list.txt; exit 1; }
grep "resample\|conv launches" gpurun_out/r04_l_layer_list.txt
for side in s0 s1 r3 new s0 s1 r3 new; do
  unset LEASTEREO_CONV2D_SMALL LEASTEREO_RESAMPLE_MODE
  case $side in s0) export LEASTEREO_CONV2D_SMALL=0;; s1) export LEASTEREO_CONV2D_SMALL=1;; r3) export LEASTEREO_RESAMPLE_MODE=3;; esac
  timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --cpu-baseline 0 --epe 0 > gpurun_out/r04_l_bench_$side.json 2> gpurun_out/r04_l_bench_$side.err \
    || { tail -20 gpurun_out/r04_l_bench_$side.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r04_l_bench_$side.json $side
done
