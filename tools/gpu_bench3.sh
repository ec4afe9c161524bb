#!/bin/bash
# c2 / c3 / c4 benches (c2 with the CPU baseline) -> gpurun_out/bench_<TAG>_<cfg>.json
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-v19}
for c in c2 c3 c4; do
  timeout -k 10 400 python3 bench.py --config $c --steps 20 --warmup 5 --breakdown 1 --cpu-baseline $([ $c = c2 ] && echo 1 || echo 0) \
    > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err
  rc=$?; echo "bench $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_${TAG}_$c.err; exit $rc; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$c.json')); r=d['roofline']; print('$c', round(d['value'],1), round(d['ms_per_step'],2), r['kernel'], round(r['frac'],3), r['traffic'], d.get('path_roofline',{}).get('frac'))"
done
