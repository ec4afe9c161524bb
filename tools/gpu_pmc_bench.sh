#!/bin/bash
# counter passes over a short c2 bench (one rocprofv3 run per pass), summarised per kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/pmc_bench
mkdir -p $D
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
            "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $D/pass$i -o run -- \
    python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 --epe 0 --extra-configs= > $D/pass$i.log 2>&1
  rc=$?; echo "pass $i: rc=$rc"; [ $rc -eq 0 ] || { tail -5 $D/pass$i.log; exit $rc; }
done
for f in ${FILTERS:-conv3d_wino_kernel conv3d_dma_kernel}; do python3 tools/pmc_kernel_report.py $D $f; done
