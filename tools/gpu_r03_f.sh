#!/bin/bash
# Round 3: H-fastest tile order on the W x D tiles: tests, traffic (c2 bench) and A/B
# against the previous build (leastereo_amd/var_base.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tr_f
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wino.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_wino.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_wino.log; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 --epe 0 --pair-check 0"
for v in new base; do
  lib=leastereo_amd/libleastereo_hip.so; [ $v = base ] && lib=leastereo_amd/var_base.so
  for ctr in FETCH_SIZE WRITE_SIZE; do
    LEASTEREO_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d gpurun_out/tr_f/${v}_$ctr -o run -- $B \
      > gpurun_out/tr_f/${v}_$ctr.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$v $ctr rc=$rc"; exit $rc; }
  done
  python3 tools/traffic_report.py gpurun_out/tr_f/${v}_FETCH_SIZE gpurun_out/tr_f/${v}_WRITE_SIZE gpurun_out/tr_f/$v.json | head -3 | sed "s/^/$v /"
done
AB_A="LEASTEREO_HIP_LIB=leastereo_amd/var_base.so" AB_B="LEASTEREO_X=1" ROUNDS=2 CONFIGS=c2 bash tools/gpu_ab.sh
