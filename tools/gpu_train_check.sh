#!/bin/bash
# training-backward tests, then the rest of the GPU suite, the default bench, and the
# training-step timings (tools/train_bench.py) at C1 and C2 sizes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_training.py -x -v -s --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_training.log 2>&1
rc=$?; grep -E "passed|failed|worst" gpurun_out/pytest_training.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/train_bench.py --steps 3 --warmup 1 > gpurun_out/train_bench_c1.jsonl 2> gpurun_out/train_bench_c1.err
rc=$?; cat gpurun_out/train_bench_c1.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/train_bench_c1.err; exit $rc; }
timeout -k 10 400 python3 -u tools/train_bench.py --height 576 --width 960 --maxdisp 192 --steps 2 --warmup 1 --impl hip \
  > gpurun_out/train_bench_c2.jsonl 2> gpurun_out/train_bench_c2.err
rc=$?; tail -1 gpurun_out/train_bench_c2.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/train_bench_c2.err; exit $rc; }
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_default.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
