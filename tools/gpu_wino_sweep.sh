#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python3 tools/wino_sweep.py --iters 10 > gpurun_out/wino_sweep.txt 2>&1
rc=$?; grep -v "^{" gpurun_out/wino_sweep.txt | grep -v amdgpu.ids; exit $rc
