#!/bin/bash
# Round-2 final profile set: full GPU parity suite, c2 traffic/kernel stats/benches
# (tools/gpu_profile_all.sh), then the bf16 traffic passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-v25} bash tools/gpu_round_final.sh || exit $?
bash tools/gpu_traffic_bf16.sh
