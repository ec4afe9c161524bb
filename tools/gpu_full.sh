#!/bin/bash
# tests -> bench -> rocprof kernel trace (each step time-limited; fatal codes stop the script)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_check.sh; rc=$?
[ $rc -le 1 ] || exit $rc
TAG=${TAG:-cur} bash tools/gpu_profile.sh > /dev/null 2>&1; rc=$?
echo "profile rc=$rc"
exit $rc
