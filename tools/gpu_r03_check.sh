#!/bin/bash
# Round 3: smoke, the full GPU suite, then the default bench line (C2 with the CPU
# baseline legs) and the C4 per-GPU shard.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
[ -n "${SKIP_BENCH:-}" ] && exit 0
timeout -k 10 400 python3 bench.py --breakdown 1 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
rc=$?; echo "bench c2 rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_c2.err; exit $rc; }
timeout -k 10 400 python3 bench.py --config c4 --breakdown 1 --cpu-baseline 0 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
rc=$?; echo "bench c4 rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_c4.err; exit $rc; }
