#!/bin/bash
# tools/wino2_sweep.py (SWEEP_ARGS) under each environment of ENVS ("A=1 B=2;C=3", ";"-separated)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=';' read -ra sets <<< "${ENVS:-}"
for r in $(seq 1 ${ROUNDS:-1}); do
  for e in "${sets[@]}"; do
    echo "== [$e] round $r"
    env $e timeout -k 10 120 python3 tools/wino2_sweep.py $SWEEP_ARGS 2>&1 | grep -v "^{\|amdgpu.ids" ; rc=${PIPESTATUS[0]}
    [ $rc -eq 0 ] || { echo "[$e] rc=$rc"; exit $rc; }
  done
done
