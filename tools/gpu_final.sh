#!/bin/bash
# round-end confirmation: smoke, bench.py's default line, the bench/launcher tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_final.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], d['config']['launch'], r['frac'], r['launches_per_step'], d['cpu_baseline']['value'])"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bench.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_bench.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_bench.log; exit $rc
