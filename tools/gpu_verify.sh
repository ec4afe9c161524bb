#!/bin/bash
# Full GPU parity suite, then c2/c3/c4 bench lines (TAG names the outputs).  Each GPU
# step is time-limited; a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-cur}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu_$TAG.log; [ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-c2 c3 c4}; do
  timeout -k 10 400 python3 bench.py --config $c --steps 20 --warmup 5 --breakdown 1 --cpu-baseline 0 \
    > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err
  rc=$?; echo "bench $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_${TAG}_$c.err; exit $rc; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$c.json')); r=d['roofline']; print('$c', round(d['value'],1), round(d['ms_per_step'],2), r['kernel'], round(r['frac'],3), r.get('mfma_executed_frac'), d.get('path_roofline',{}).get('frac'))"
done
