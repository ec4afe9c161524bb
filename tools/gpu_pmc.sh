#!/bin/bash
# Counter passes (each its own rocprofv3 run, --pmc only with --kernel-trace/--stats,
# never with sys/runtime traces).  CMD = the program to profile (default: conv_bench).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
export TMPDIR=/tmp
TAG=${TAG:-pmc}
CMD=${CMD:-python3 tools/conv_bench.py --iters 5}
mkdir -p gpurun_out/$TAG
if [ "${LIST:-0}" = 1 ]; then
  timeout -k 10 120 rocprofv3 -L > gpurun_out/$TAG/counters.txt 2>&1
fi
i=0
for pass in "${PASSES[@]:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE}"; do :; done
IFS=';' read -ra P <<< "${PMC_PASSES:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE}"
for pass in "${P[@]}"; do
  i=$((i+1))
  timeout -k 10 ${PMC_TIMEOUT:-300} rocprofv3 --pmc $pass --kernel-trace --output-format csv \
    -d gpurun_out/$TAG/pass$i -o run -- $CMD > gpurun_out/$TAG/pass$i.log 2>&1
  rc=$?
  echo "pass $i ($pass): rc=$rc"
  case $rc in 0) ;; 1|2) tail -5 gpurun_out/$TAG/pass$i.log ;; *) echo "fatal: stop"; exit $rc ;; esac
done
