#!/bin/bash
# counter passes over the bf16 layer set (tools/bf16_layer_pmc.py), one rocprofv3 run per pass
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/pmc_bf16
mkdir -p $D
timeout -k 10 120 python3 tools/bf16_layer_pmc.py run > $D/plain.log 2>&1; rc=$?; cat $D/plain.log; [ $rc -eq 0 ] || exit $rc
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD" \
            "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU" \
            "TCC_HIT_sum TCC_MISS_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $D/pass$i -o run -- \
    python3 tools/bf16_layer_pmc.py run > $D/pass$i.log 2>&1
  rc=$?; echo "pass $i: rc=$rc"; [ $rc -eq 0 ] || { tail -5 $D/pass$i.log; exit $rc; }
done
python3 tools/bf16_layer_pmc.py report $D
