#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/cv_stem_probe.py > gpurun_out/cv_probe.txt 2>&1; rc=$?; grep -v amdgpu gpurun_out/cv_probe.txt; exit $rc
