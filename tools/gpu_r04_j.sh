#!/bin/bash
# Round 4 (j): bench A/B of this round's default switches against their previous values on
# one box (LEASTEREO_RESAMPLE_MODE=1: the row-staged resample; LEASTEREO_WINO_FENCE=0: the
# depth-paired tile's compiler schedule), interleaved.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for side in old new old new; do
  if [ $side = old ]; then export LEASTEREO_RESAMPLE_MODE=1 LEASTEREO_WINO_FENCE=0; else unset LEASTEREO_RESAMPLE_MODE LEASTEREO_WINO_FENCE; fi
  timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --cpu-baseline 0 --epe 0 > gpurun_out/r04_j_bench_$side.json 2> gpurun_out/r04_j_bench_$side.err \
    || { tail -20 gpurun_out/r04_j_bench_$side.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'])" gpurun_out/r04_j_bench_$side.json $side
done
