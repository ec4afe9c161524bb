#!/bin/bash
# LDS bank-conflict cycles per kernel over any program (PROG), one rocprofv3 counter pass
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/conf_prog; rm -rf $D
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $D -o run -- python3 $PROG > $D.log 2>&1
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -5 $D.log; exit $rc; }
python3 - <<'PY'
import csv, collections
agg=collections.defaultdict(collections.Counter); n=collections.Counter()
for r in csv.DictReader(open("gpurun_out/conf_prog/run_counter_collection.csv")):
    k=r["Kernel_Name"].split("(")[0].replace("void ","")[:70]
    agg[k][r["Counter_Name"]]+=float(r["Counter_Value"])
for k,v in sorted(agg.items(), key=lambda kv: -kv[1]["SQ_LDS_BANK_CONFLICT"])[:12]:
    print(f"{k:70s} conflict {v['SQ_LDS_BANK_CONFLICT']/1e6:8.2f}M  lds_active {v['SQ_LDS_IDX_ACTIVE']/1e6:8.2f}M  wave_cycles {v['SQ_WAVE_CYCLES']/1e6:9.1f}M")
PY
