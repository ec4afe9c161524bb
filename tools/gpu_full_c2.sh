#!/bin/bash
# whole GPU parity suite, then the c2 bench with per-kernel breakdown
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --breakdown 1 ${BENCH_EXTRA:-} > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/bench_c2.json')); r=d['roofline']; print(round(d['value'],2), round(d['ms_per_step'],3), r['kernel'], round(r['frac'],3), round(r['mfma_executed_frac'],3), d['epe_px']['max_over_ranks'], d.get('cpu_baseline',{}).get('value'))"; grep -v amdgpu.ids gpurun_out/bench_c2.err | head -24; exit $rc
