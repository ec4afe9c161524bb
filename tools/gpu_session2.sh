#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/conv_bench.py --iters 20 > gpurun_out/conv_bench.txt 2>&1
rc=$?; cat gpurun_out/conv_bench.txt | head -14; [ $rc -le 1 ] || exit $rc
LIST=1 TAG=pmc1 PMC_PASSES="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD;SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY;SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE" bash tools/gpu_pmc.sh
