#!/bin/bash
# Round 4 (m): side-stream schedule of the split L1 cells (op0 on s0 beside s1's preprocess
# and group) -- parity / graph tests, then a same-box bench A/B (LEASTEREO_CELL_STREAMS 0/1).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench.py tests/test_gpu_wino.py -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/r04_m_tests.txt 2>&1 || { tail -30 gpurun_out/r04_m_tests.txt; exit 1; }
tail -1 gpurun_out/r04_m_tests.txt
for side in s0 s1 s0 s1; do
  if [ $side = s0 ]; then export LEASTEREO_CELL_STREAMS=0; else unset LEASTEREO_CELL_STREAMS; fi
  timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --cpu-baseline 0 --epe 0 > gpurun_out/r04_m_bench_$side.json 2> gpurun_out/r04_m_bench_$side.err \
    || { tail -20 gpurun_out/r04_m_bench_$side.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('pair_check', {}))" gpurun_out/r04_m_bench_$side.json $side | cut -c1-200
done
