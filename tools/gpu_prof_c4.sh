#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o run -- \
  python3 bench.py --config c4 --steps 3 --warmup 2 --cpu-baseline 0 --epe 0 --pair-check 0 --extra-configs= > gpurun_out/prof_c4.json 2> gpurun_out/prof_c4.err
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/trace_report.py gpurun_out/prof_c4 > gpurun_out/prof_c4_forward.txt; head -30 gpurun_out/prof_c4_forward.txt
