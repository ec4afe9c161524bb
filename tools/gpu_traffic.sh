#!/bin/bash
# HBM traffic: two separate --pmc passes (FETCH_SIZE, WRITE_SIZE) over a short bench run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/traffic
B="python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 --epe 0"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/traffic/fetch -o run -- $B > gpurun_out/traffic/fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/traffic/write -o run -- $B > gpurun_out/traffic/write.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -le 1 ] || exit $rc
python3 tools/traffic_report.py gpurun_out/traffic/fetch gpurun_out/traffic/write gpurun_out/traffic/hbm_traffic.json
