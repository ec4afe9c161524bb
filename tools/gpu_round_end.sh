#!/bin/bash
# Round-end evidence on one box: the GPU suite, smoke, the C2/C3/C4 bench lines with
# breakdowns, and a C2 rocprofv3 kernel-stats pass.  Outputs under gpurun_out/ (TAG names them).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-end}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$T.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$T.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$T.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 || { tail -20 gpurun_out/smoke_$T.log; exit 1; }
tail -1 gpurun_out/smoke_$T.log
timeout -k 10 400 python3 bench.py > gpurun_out/bench_${T}_c2.json 2> gpurun_out/bench_${T}_c2.err || { tail -5 gpurun_out/bench_${T}_c2.err; exit 1; }
for c in c3 c4; do
  timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 --breakdown 1 --cpu-baseline 0 --extra-configs= > gpurun_out/bench_${T}_$c.json 2> gpurun_out/bench_${T}_$c.err || { tail -5 gpurun_out/bench_${T}_$c.err; exit 1; }
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T}_c2 -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline 0 --epe 0 --pair-check 0 --extra-configs= > gpurun_out/prof_${T}_c2.json 2> gpurun_out/prof_${T}_c2.err || exit 1
python3 tools/trace_report.py gpurun_out/prof_${T}_c2 > gpurun_out/prof_${T}_c2_forward.txt
