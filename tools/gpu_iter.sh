#!/bin/bash
# iteration loop: parity tests -> bench -> per-layer conv microbench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_check.sh; rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 tools/conv_bench.py --iters 20 > gpurun_out/conv_bench.txt 2>&1; rc=$?
head -16 gpurun_out/conv_bench.txt
exit $rc
