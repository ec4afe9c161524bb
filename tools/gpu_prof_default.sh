#!/bin/bash
# rocprofv3 kernel summary of bench.py's default command (HIP-graph replay) at C2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_v32 -o run -- \
  python3 bench.py --steps 10 --warmup 2 --cpu-baseline 0 --epe 0 --pair-check 0 > gpurun_out/prof_v32.json 2> gpurun_out/prof_v32.err
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/prof_v32.err; exit $rc; }
f=$(find gpurun_out/prof_v32 -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/prof_v32_kernel_stats.csv
python3 -c "
import csv, json
d = json.load(open('gpurun_out/prof_v32.json'))
r = d['roofline']
print('bench', round(d['value'], 2), 'pairs/s', r['kernel'], 'HIP-event avg ms', r.get('avg_ms', r.get('ms_per_launch')))
for x in csv.DictReader(open('gpurun_out/prof_v32_kernel_stats.csv')):
    if 'wino2p' in x['Name']:
        print('rocprof', x['Name'][:50], x['Calls'], float(x['AverageNs']) / 1e6, 'ms avg')
"
