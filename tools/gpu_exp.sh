#!/bin/bash
# scratch lease script for the current experiment (overwritten per experiment; results
# worth keeping are copied into profiles/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/abl
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wino.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_wino.log 2>&1
rc=$?; tail -2 gpurun_out/t_wino.log; [ $rc -eq 0 ] || exit $rc
for h in 0 1 0 1; do
  LEASTEREO_HALO16=$h timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/abl/h$h -o run -- python3 tools/wino2_sweep.py --variants 0 --iters 20 --only cell_16to16_k3_L1 \
    > gpurun_out/abl/h$h.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "h$h rc=$rc"; tail -3 gpurun_out/abl/h$h.log; exit $rc; }
  f=$(ls gpurun_out/abl/h$h/*kernel_stats.csv | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'wino2_kernel' in r['Name']: print('halo16=$h', r['Name'][:70], 'calls', r['Calls'], 'avg_us', round(float(r['AverageNs'])/1e3,1))
"
  rm -rf gpurun_out/abl/h$h
done
