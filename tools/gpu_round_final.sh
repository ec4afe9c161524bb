#!/bin/bash
# Full GPU parity suite, then the round's profile set (tools/gpu_profile_all.sh, TAG).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-v19} bash tools/gpu_profile_all.sh
