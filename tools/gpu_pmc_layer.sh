#!/bin/bash
# counter passes over a layer program (PMC_PROG, default tools/wino2_sweep.py on one layer,
# SWEEP_ARGS), per kernel summary
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/pmc_layer
rm -rf $D; mkdir -p $D
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
            "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD" \
            "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU" \
            ${EXTRA_PASSES:-}; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $D/pass$i -o run -- \
    python3 ${PMC_PROG:-tools/wino2_sweep.py --iters 3 $SWEEP_ARGS} > $D/pass$i.log 2>&1
  rc=$?; echo "pass $i: rc=$rc"; [ $rc -eq 0 ] || { tail -5 $D/pass$i.log; exit $rc; }
done
for f in ${FILTERS:-conv3d_wino}; do python3 tools/pmc_kernel_report.py $D $f; done
