#!/bin/bash
# Round 4: feature-net backward and the whole-model train step -- GPU training tests,
# then the whole-model step timed at C1 and C2.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_training.py -x -v --timeout 300 --timeout-method thread -s \
  > gpurun_out/r04_train_tests.txt 2>&1 || { tail -40 gpurun_out/r04_train_tests.txt; exit 1; }
grep -E "passed|failed|disp max" gpurun_out/r04_train_tests.txt | tail -5
timeout -k 10 300 python -u tools/train_bench.py --whole 1 > gpurun_out/r04_train_whole.jsonl 2>&1 || { tail -20 gpurun_out/r04_train_whole.jsonl; exit 1; }
timeout -k 10 300 python -u tools/train_bench.py --whole 1 --height 576 --width 960 --maxdisp 192 --steps 3 >> gpurun_out/r04_train_whole.jsonl 2>&1 || { tail -20 gpurun_out/r04_train_whole.jsonl; exit 1; }
grep "^{" gpurun_out/r04_train_whole.jsonl
