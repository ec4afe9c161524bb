#!/bin/bash
# Which loads of the pipelined W x D tile reach HBM: FETCH_SIZE / WRITE_SIZE passes of the
# conv1/2 and stem1 shapes on the full build and on builds without the halo DMA or the
# weight loads (timing-only variants, tools/wino2_ablate.sh switches)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/traffic_ablate; mkdir -p $D
for v in base nohalo nowdma; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    LEASTEREO_HIP_LIB=leastereo_amd/var_$v.so timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv \
      -d $D/${v}_$ctr -o run -- python3 tools/wino2_sweep.py --variants 0 --iters 2 \
      --only conv12_128to64_k3_L1,stem1_32to32_k3_L0 > $D/${v}_$ctr.log 2>&1
    rc=$?; echo "$v $ctr rc=$rc"; [ $rc -eq 0 ] || { tail -3 $D/${v}_$ctr.log; exit $rc; }
  done
  python3 tools/traffic_report.py $D/${v}_FETCH_SIZE $D/${v}_WRITE_SIZE $D/$v.json | head -3
done
