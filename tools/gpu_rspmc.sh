#!/bin/bash
# counter passes over the c8 up-sampling probe (one case, one k)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/pmc_rs
rm -rf $D; mkdir -p $D
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR" \
            "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INSTS_SALU" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $D/pass$i -o run -- \
    python3 tools/resample_probe.py "${CASE:-up 8ch}" ${KS:-4} > $D/pass$i.log 2>&1
  rc=$?; echo "pass $i: rc=$rc"; [ $rc -eq 0 ] || { tail -5 $D/pass$i.log; exit $rc; }
done
python3 tools/pmc_kernel_report.py $D resample_c8
