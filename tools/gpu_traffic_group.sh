#!/bin/bash
# HBM bytes per launch of the F(4,3) x F(4,3) tile under each workgroup order
# (lea_conv3d_wino44_set_group, ORDERS) on the conv1/2 and stem1 shapes: one FETCH_SIZE and
# one WRITE_SIZE pass per order and layer (tools/setter_ab.py as the program)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/traffic_group; mkdir -p $D
for layer in ${LAYERS:-conv12_128to64_k3_L1 stem1_32to32_k3_L0}; do
  for g in ${ORDERS:-0 2 4 8}; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv \
        -d $D/${layer}_g${g}_$ctr -o run -- python3 tools/setter_ab.py --setter lea_conv3d_wino44_set_group \
        --values $g --only $layer --rounds 1 --iters 2 --exact 0 > $D/${layer}_g${g}_$ctr.log 2>&1
      rc=$?; echo "$layer g=$g $ctr rc=$rc"; [ $rc -eq 0 ] || { tail -3 $D/${layer}_g${g}_$ctr.log; exit $rc; }
    done
    echo "== $layer g=$g"
    python3 tools/traffic_report.py $D/${layer}_g${g}_FETCH_SIZE $D/${layer}_g${g}_WRITE_SIZE $D/${layer}_g$g.json | grep -i wino44
  done
done
