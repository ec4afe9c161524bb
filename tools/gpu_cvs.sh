set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_cv_stem.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_cvs.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_cvs.log; [ $rc -eq 0 ] || exit $rc
TAG=cvs1 bash tools/gpu_verify.sh
