#!/bin/bash
# Same-box A/B of library builds (a change that is not behind a switch): runs PROG under each
# LEASTEREO_HIP_LIB in LIBS, interleaved ROUNDS times.  Build the other side first, e.g.
#   cp leastereo_amd/libleastereo_hip.so ab/lib_base.so   (before the change), then make
#   LIBS="ab/lib_base.so leastereo_amd/libleastereo_hip.so" PROG="tools/pair_bf16_probe.py --iters 20" bash tools/ab_libs.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq 1 ${ROUNDS:-2}); do
  # the library order reversed on even rounds so a first-run/second-run bias cancels
  LL=(${LIBS:-leastereo_amd/libleastereo_hip.so}); [ $((r % 2)) -eq 0 ] && LL=($(printf '%s\n' "${LL[@]}" | tac))
  for L in "${LL[@]}"; do
    echo "== round $r $L"
    LEASTEREO_HIP_LIB=$L timeout -k 10 ${STEP_TIMEOUT:-120} python3 ${PROG:-tools/pair_bf16_probe.py --iters 20} || exit 1
  done
done
