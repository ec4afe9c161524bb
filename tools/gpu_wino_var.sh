#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for lib in leastereo_amd/libleastereo_hip.so leastereo_amd/var_*.so; do
  echo "== $lib"
  LEASTEREO_HIP_LIB=$PWD/$lib timeout -k 10 200 python3 tools/wino_sweep.py --iters 10 --only stem0_64to32_k3_L0,conv12_128to64_k3_L1,cell_16to48_k3_L1_s1grp,cell_16to16_k3_L1 2>/dev/null | grep "default"
  rc=$?; [ $rc -le 1 ] || exit $rc
done
