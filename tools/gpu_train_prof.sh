#!/bin/bash
# training tests + train-step timings + a rocprofv3 kernel summary of the HIP train step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_training.py -x -q -s --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_training.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/pytest_training.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/train_bench.py --steps 3 --warmup 1 --impl hip > gpurun_out/train_bench_c1.jsonl 2> gpurun_out/train_bench_c1.err
rc=$?; cat gpurun_out/train_bench_c1.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/train_bench_c1.err; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_train -o run -- \
  python3 tools/train_bench.py --height 576 --width 960 --maxdisp 192 --steps 2 --warmup 1 --impl hip \
  > gpurun_out/train_bench_c2.jsonl 2> gpurun_out/train_bench_c2.err
rc=$?; tail -1 gpurun_out/train_bench_c2.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/train_bench_c2.err; exit $rc; }
f=$(find gpurun_out/prof_train -name "*kernel_stats.csv" | head -1); head -25 "$f" | cut -d, -f1-4
