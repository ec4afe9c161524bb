#!/bin/bash
# Round 4 (r): loop-counter item walk and per-channel halo bases by compare / select / add in the
# pipelined W x D tile and the per-lane 16-cout tile (SALU per item ~170 -> ~110 / ~200 -> ~130) --
# Winograd tests, e2e golden, per-launch list, same-box C2 bench A/B against ab/lib_head.so.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_wino.py tests/test_gpu_parity.py -x -q --timeout 300 \
  --timeout-method thread -k "wino or halo or lane or e2e or golden or full" > gpurun_out/r04_r_tests.txt 2>&1 \
  || { tail -30 gpurun_out/r04_r_tests.txt; exit 1; }
tail -1 gpurun_out/r04_r_tests.txt
timeout -k 10 300 python -u tools/layer_list.py --reps 5 > gpurun_out/r04_r_layer_list.txt 2>&1 || { tail -20 gpurun_out/r04_r_layer_list.txt; exit 1; }
grep "wino\|conv launches" gpurun_out/r04_r_layer_list.txt | sort -k7 | uniq -c -f6 | head -5
for side in old new old new; do
  if [ $side = old ]; then export LEASTEREO_HIP_LIB=$PWD/ab/lib_head.so; else unset LEASTEREO_HIP_LIB; fi
  timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --cpu-baseline 0 --epe 0 > gpurun_out/r04_r_bench_$side.json 2> gpurun_out/r04_r_bench_$side.err \
    || { tail -20 gpurun_out/r04_r_bench_$side.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r04_r_bench_$side.json $side
done
