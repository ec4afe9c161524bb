#!/bin/bash
# Ablation of the W x D transform-pass kernel (timing only, outputs wrong): builds
# leastereo_amd/var_<name>.so with one phase knocked out each, then times the 32-cout
# layers on each build (tools/wino2_sweep.py, planner's variant, HIP events).  NOWDMA
# drops the weight DMA (two-barrier tile) or the per-lane weight loads (pipelined tile).
#   build here:  bash tools/wino2_ablate.sh build
#   run on GPU:  bash tools/wino2_ablate.sh run   (ONLY=<layer,...> picks the layers)
set -u
cd "$(dirname "$0")/.."
VARS=${VARS:-"base: nohalo:-DLEA_EXP_NOHALO nowdma:-DLEA_EXP_NOWDMA novpass:-DLEA_EXP_NOVPASS nobar2:-DLEA_EXP_NOBAR2 nomfma:-DLEA_EXP_NOMFMA nodma:-DLEA_EXP_NOHALO_-DLEA_EXP_NOWDMA"}
if [ "${1:-run}" = build ]; then
  specs=""
  for v in $VARS; do n=${v%%:*}; f=${v#*:}; specs="$specs $n:-fno-slp-vectorize ${f//_-D/ -D}"; done
  # shellcheck disable=SC2086
  eval bash tools/build_variants.sh conv3d_wino2 $(for v in $VARS; do n=${v%%:*}; f=${v#*:}; printf '"%s:-fno-slp-vectorize %s" ' "$n" "${f//_-D/ -D}"; done)
  exit $?
fi
mkdir -p gpurun_out
for v in $VARS; do
  n=${v%%:*}
  LEASTEREO_HIP_LIB=leastereo_amd/var_$n.so timeout -k 10 200 python3 tools/wino2_sweep.py --variants 0 --iters 20 \
    --only ${ONLY:-stem1_32to32_k3_L0,conv12_128to64_k3_L1,cell_32to32_k3_L2,cell_8to24_k3_L0_s1grp} > gpurun_out/ablate_$n.txt 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$n rc=$rc"; tail -3 gpurun_out/ablate_$n.txt; exit $rc; }
  grep -v "^{" gpurun_out/ablate_$n.txt | grep -v amdgpu.ids | sed "s/^/$n /" | cut -c1-150
done
