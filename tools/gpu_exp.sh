#!/bin/bash
# scratch lease script for the current experiment (overwritten per experiment; results
# worth keeping are copied into profiles/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/abl
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_wino.py tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread -k "halo16 or walk or small_cout or e2e or full or wino_vs" > gpurun_out/t_dp.log 2>&1
rc=$?; tail -2 gpurun_out/t_dp.log; [ $rc -eq 0 ] || exit $rc
for n in w1base w1new w1base w1new; do
  LEASTEREO_HIP_LIB=leastereo_amd/var_$n.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/abl/$n -o run -- python3 tools/wino2_sweep.py --variants 0 --iters 20 --only cell_8to8_k3_L0 \
    > gpurun_out/abl/$n.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$n rc=$rc"; tail -3 gpurun_out/abl/$n.log; exit $rc; }
  f=$(ls gpurun_out/abl/$n/*kernel_stats.csv | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'wino_kernel' in r['Name']: print('$n', r['Name'][:70], 'calls', r['Calls'], 'avg_us', round(float(r['AverageNs'])/1e3,1))
"
  rm -rf gpurun_out/abl/$n
done
