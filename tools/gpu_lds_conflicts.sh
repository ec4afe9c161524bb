#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
for c in c2 c4; do
  timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES --kernel-trace --output-format csv -d gpurun_out/conf_$c -o run -- python3 bench.py --config $c --steps 2 --warmup 1 --cpu-baseline 0 --epe 0 --pair-check 0 --extra-configs= > gpurun_out/conf_$c.log 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 - $c <<'PY'
import csv, collections, sys
c=sys.argv[1]
agg=collections.defaultdict(lambda: collections.Counter()); n=collections.Counter()
for r in csv.DictReader(open(f"gpurun_out/conf_{c}/run_counter_collection.csv")):
    k=r["Kernel_Name"].split("(")[0].replace("void ","")[:70]
    agg[k][r["Counter_Name"]]+=float(r["Counter_Value"])
for k,v in sorted(agg.items(), key=lambda kv: -kv[1]["SQ_LDS_BANK_CONFLICT"])[:12]:
    if v["SQ_LDS_BANK_CONFLICT"]>0:
        print(f"{c} {k:70s} conflict {v['SQ_LDS_BANK_CONFLICT']/1e6:8.2f}M  lds_active {v['SQ_LDS_IDX_ACTIVE']/1e6:8.2f}M  wave_cycles {v['SQ_WAVE_CYCLES']/1e6:9.1f}M")
PY
done
