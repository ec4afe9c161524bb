#!/bin/bash
# Round-2 closing profile set (after the iglp_opt hint): full GPU parity suite, smoke,
# c2 traffic / kernel stats / c2-c3-c4 benches (tools/gpu_profile_all.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-v26} bash tools/gpu_round_final.sh
