#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run (no PMC here: counters get
# their own passes, see tools/gpu_pmc.sh).  Output under gpurun_out/prof_<tag>.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
TAG=${TAG:-r01}
mkdir -p gpurun_out
timeout -k 10 ${PROF_TIMEOUT:-600} rocprofv3 --kernel-trace --stats --output-format csv \
  -d gpurun_out/prof_${TAG} -o run -- \
  python3 bench.py --steps ${STEPS:-5} --warmup 2 --cpu-baseline 0 --epe 0 ${BENCH_EXTRA:-} \
  > gpurun_out/prof_${TAG}.json 2> gpurun_out/prof_${TAG}.err
rc=$?
cat gpurun_out/prof_${TAG}.json
find gpurun_out/prof_${TAG} -name "*kernel_stats.csv" | head -1 | xargs -r head -40
exit $rc
