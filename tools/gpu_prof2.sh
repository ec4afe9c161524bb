#!/bin/bash
# cv_stem tests, then rocprofv3 kernel traces of c2 and c4 bench runs with per-forward
# breakdowns (gpurun_out/prof_<TAG>_<cfg>_forward.txt).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-cur}
timeout -k 10 300 python -u -m pytest tests/test_gpu_cv_stem.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_cvs.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_cvs.log; [ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-c2 c4}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_$c -o run -- \
    python3 bench.py --config $c --steps 5 --warmup 2 --cpu-baseline 0 --epe 0 > gpurun_out/prof_${TAG}_$c.json 2> gpurun_out/prof_${TAG}_$c.err
  rc=$?; echo "prof $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/trace_report.py gpurun_out/prof_${TAG}_$c > gpurun_out/prof_${TAG}_${c}_forward.txt
  head -30 gpurun_out/prof_${TAG}_${c}_forward.txt
done
