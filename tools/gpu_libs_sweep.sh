#!/bin/bash
# tools/wino2_sweep.py (SWEEP_ARGS) under the in-tree library and every var_*.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in leastereo_amd/libleastereo_hip.so leastereo_amd/var_*.so; do
  echo "== $lib"
  LEASTEREO_HIP_LIB=$PWD/$lib timeout -k 10 120 python3 tools/wino2_sweep.py $SWEEP_ARGS 2>&1 | grep -v "^{" ; rc=${PIPESTATUS[0]}
  [ $rc -eq 0 ] || { echo "$lib rc=$rc"; exit $rc; }
done
