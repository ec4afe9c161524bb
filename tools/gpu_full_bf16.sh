#!/bin/bash
# whole GPU parity suite, then the c3/c4 (bf16) benches with per-kernel breakdown
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head; exit $rc; }
for c in c4 c3; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --breakdown 1 --cpu-baseline 0 > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$c.err; exit $rc; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_$c.json')); r=d['roofline']; print('$c', round(d['value'],1), round(d['ms_per_step'],2), r['kernel'], round(r['frac'],3), d.get('path_roofline',{}).get('frac'), d['epe_px'])"
done
