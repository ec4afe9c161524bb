#!/bin/bash
# One GPU session: parity tests, then a bench run.  Every GPU step has its own
# time limit; a crash/timeout/abort stops the script (no further GPU work).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop_if_fatal() {  # $1 = exit code of the previous GPU step
  case "$1" in
    0|1) return 0 ;;                     # pass / test failures: keep going
    *) echo "fatal exit $1: stopping GPU work" ; exit "$1" ;;
  esac
}
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -q -m gpu ${PYTEST_ARGS:-} \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_gpu.log; stop_if_fatal $rc
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:---steps 10 --warmup 3 --breakdown 1} \
  > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; cat gpurun_out/bench.json; tail -40 gpurun_out/bench.err; exit $rc
