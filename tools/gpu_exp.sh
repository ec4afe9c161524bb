#!/bin/bash
# scratch lease script for the current experiment (overwritten per experiment; results
# worth keeping are copied into profiles/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 --epe 0 --pair-check 0 > gpurun_out/bs.json 2> gpurun_out/bs.err
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/bs.err; exit $rc; }
python3 -c "
import json; d=json.load(open('gpurun_out/bs.json')); r=d['roofline']
print(round(d['value'],1), r['kernel'], round(r['frac'],3))
for x in r['by_shape']: print(x)
"
