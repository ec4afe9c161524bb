#!/bin/bash
# HBM traffic passes (FETCH_SIZE, WRITE_SIZE: one rocprofv3 --pmc run each) over the
# benches of CONFIGS (default: the c3 and c4 bf16 ones) -> gpurun_out/traffic_<cfg>.json
# (merge: tools/traffic_merge.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/traffic_bf16
for c in ${CONFIGS:-c3 c4}; do
  B="python3 bench.py --config $c --steps 2 --warmup 1 --cpu-baseline 0 --epe 0 --pair-check 0 --extra-configs="
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d gpurun_out/traffic_bf16/${c}_$ctr -o run -- $B \
      > gpurun_out/traffic_bf16/${c}_$ctr.log 2>&1
    rc=$?; echo "$c $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python3 tools/traffic_report.py gpurun_out/traffic_bf16/${c}_FETCH_SIZE gpurun_out/traffic_bf16/${c}_WRITE_SIZE \
    gpurun_out/traffic_$c.json | head -4
done
