#!/bin/bash
# Round profile set: HBM traffic passes (FETCH_SIZE, WRITE_SIZE) -> profiles/hbm_traffic.json
# on this box, rocprofv3 kernel-trace stats of the c2 bench, then the c2/c3/c4 benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/traffic
TAG=${TAG:-v19}
B="python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 --epe 0 --pair-check 0"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/traffic/fetch -o run -- $B > gpurun_out/traffic/fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/traffic/write -o run -- $B > gpurun_out/traffic/write.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/traffic_report.py gpurun_out/traffic/fetch gpurun_out/traffic/write gpurun_out/traffic/hbm_traffic.json | head -12
# c2 entries (plain kernel names) replace the old ones; per-config "@c3"/"@c4" entries
# (tools/gpu_traffic_bf16.sh + tools/traffic_merge.py) are kept
python3 -c "import json; o=json.load(open('profiles/hbm_traffic.json')); n=json.load(open('gpurun_out/traffic/hbm_traffic.json')); o={k: v for k, v in o.items() if '@' in k}; o.update(n); json.dump(o, open('profiles/hbm_traffic.json', 'w'), indent=1, sort_keys=True)"
cp profiles/hbm_traffic.json gpurun_out/traffic/hbm_traffic_merged.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python3 bench.py --steps 5 --warmup 2 --cpu-baseline 0 --epe 0 --pair-check 0 > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.err
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/trace_report.py gpurun_out/prof_$TAG > gpurun_out/prof_${TAG}_forward.txt; head -14 gpurun_out/prof_${TAG}_forward.txt
for c in c2 c3 c4 c5; do
  timeout -k 10 400 python3 bench.py --config $c --steps 20 --warmup 5 --breakdown 1 --cpu-baseline $([ $c = c2 ] && echo 1 || echo 0) \
    > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err
  rc=$?; echo "bench $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_${TAG}_$c.err; exit $rc; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$c.json')); r=d['roofline']; print('$c', round(d['value'],1), round(d['ms_per_step'],2), r['kernel'], round(r['frac'],3), r.get('mfma_executed_frac'), r['traffic'], d.get('path_roofline',{}).get('frac'))"
done
