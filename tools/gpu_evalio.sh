#!/bin/bash
# evalio kernels: parity tests, HIP-event bench, rocprof kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_evalio.py tests/test_capi.py -x -q -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_evalio.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_evalio.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/evalio_bench.py > gpurun_out/evalio_bench.jsonl 2> gpurun_out/evalio_bench.err
rc=$?; cat gpurun_out/evalio_bench.jsonl; [ $rc -eq 0 ] || { tail gpurun_out/evalio_bench.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_evalio -o run -- \
  python3 tools/evalio_bench.py > /dev/null 2> gpurun_out/prof_evalio.err
rc=$?; find gpurun_out/prof_evalio -name "*kernel_stats.csv" | xargs -r cat | grep -E "Name|u8_|metrics" ; exit $rc
