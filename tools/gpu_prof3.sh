#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/bw_probe.py > gpurun_out/bw_probe.txt 2>&1; rc=$?; grep -v amdgpu gpurun_out/bw_probe.txt; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof2.sh
