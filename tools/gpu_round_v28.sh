#!/bin/bash
# Round-2 closing profile set: smoke, full GPU parity suite, c2 traffic / kernel stats /
# c2-c3-c4 benches (tools/gpu_profile_all.sh), then the bf16 traffic passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-v28} bash tools/gpu_round_final.sh || exit $?
bash tools/gpu_traffic_bf16.sh
