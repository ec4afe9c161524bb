#!/bin/bash
# Round 3, first box: the validation run (tools/gpu_r03_check.sh), then the W x D kernel's
# per-phase stamps (diagnostic build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_r03_check.sh || exit $?
LEASTEREO_HIP_LIB=leastereo_amd/var_stamps.so timeout -k 10 300 python3 tools/wino2_stamps.py \
  > gpurun_out/stamps.txt 2>&1
rc=$?; cat gpurun_out/stamps.txt | cut -c1-400; exit $rc
