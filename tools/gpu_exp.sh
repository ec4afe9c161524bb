#!/bin/bash
# scratch lease script for the current experiment (overwritten per experiment; results
# worth keeping are copied into profiles/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wino.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_wino.log 2>&1
rc=$?; tail -3 gpurun_out/t_wino.log; [ $rc -eq 0 ] || exit $rc
VARS="base: gs28: base: gs28:" ONLY=stem1_32to32_k3_L0,conv12_128to64_k3_L1,cell_32to96_k3_L2_s1grp,cell_8to24_k3_L0_s1grp \
  bash tools/wino2_ablate.sh run > gpurun_out/exp.txt 2>&1
rc=$?; cat gpurun_out/exp.txt; [ $rc -eq 0 ] || exit $rc
SWEEP_ARGS="--only stem1_32to32_k3_L0,conv12_128to64_k3_L1 --variants 0 --iters 10" FILTERS="conv3d_wino2p" \
  bash tools/gpu_pmc_layer.sh > gpurun_out/pmc_dom.txt 2>&1
rc=$?; tail -2 gpurun_out/pmc_dom.txt; exit $rc
