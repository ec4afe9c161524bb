#!/bin/bash
# scratch lease script for the current experiment (overwritten per experiment; results
# worth keeping are copied into profiles/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CONFIGS=c5 bash tools/gpu_traffic_bf16.sh || exit $?
python3 tools/traffic_merge.py c5 gpurun_out/traffic_c5.json && cp profiles/hbm_traffic.json gpurun_out/hbm_traffic_c5merged.json
