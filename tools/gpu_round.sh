#!/bin/bash
# The round's closing profile set (TAG): smoke, the GPU suite, HBM traffic passes (c2 fp32,
# c3/c4 bf16) merged into profiles/hbm_traffic.json, rocprofv3 kernel stats of the c2
# bench, then the c2 (with the CPU baseline legs), c3, c4 and c5 bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
mkdir -p gpurun_out/traffic
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
B="python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 --epe 0 --pair-check 0 --extra-configs="
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d gpurun_out/traffic/c2_$ctr -o run -- $B \
    > gpurun_out/traffic/c2_$ctr.log 2>&1
  rc=$?; echo "c2 $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/traffic_report.py gpurun_out/traffic/c2_FETCH_SIZE gpurun_out/traffic/c2_WRITE_SIZE gpurun_out/traffic/c2.json > gpurun_out/traffic/c2.txt
head -6 gpurun_out/traffic/c2.txt
python3 -c "import json; o=json.load(open('profiles/hbm_traffic.json')); n=json.load(open('gpurun_out/traffic/c2.json')); o={k: v for k, v in o.items() if '@' in k}; o.update(n); json.dump(o, open('profiles/hbm_traffic.json', 'w'), indent=1, sort_keys=True)"
TC=${TRAFFIC_CONFIGS:-c3 c4 c5}
if [ -n "$TC" ]; then
  CONFIGS="$TC" bash tools/gpu_traffic_bf16.sh || exit $?
  for c in $TC; do python3 tools/traffic_merge.py $c gpurun_out/traffic_$c.json; done
fi
cp profiles/hbm_traffic.json gpurun_out/traffic/hbm_traffic_merged.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python3 bench.py --steps 5 --warmup 2 --cpu-baseline 0 --epe 0 --pair-check 0 --extra-configs= > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.err
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/trace_report.py gpurun_out/prof_$TAG > gpurun_out/prof_${TAG}_forward.txt; head -8 gpurun_out/prof_${TAG}_forward.txt
for c in ${BENCH_CONFIGS:-c2 c3 c4 c5}; do
  timeout -k 10 500 python3 bench.py --config $c --steps 20 --warmup 5 --breakdown 1 --cpu-baseline $([ $c = c2 ] && echo 1 || echo 0) \
    $([ $c = c2 ] || echo --extra-configs=) \
    > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err
  rc=$?; echo "bench $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_${TAG}_$c.err; exit $rc; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$c.json')); r=d['roofline']; print('$c', round(d['value'],1), round(d['ms_per_step'],2), r['kernel'], round(r['frac'],3), r['traffic'], round(d['path_roofline']['frac'],3))"
done
