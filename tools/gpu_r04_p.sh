#!/bin/bash
# Round 4 (p): ablations of conv3d_wino2p_kernel (timing only, wrong outputs) -- the MFMA-only
# skeleton (no halo DMA, weight loads, V-pass, U transform or V reads), with and without the
# per-item barrier, and no-LDS-read / no-barrier alone.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in base onlymfma onlymfmanobar noldsrd nobar base; do
  if [ $v = base ]; then unset LEASTEREO_HIP_LIB; else export LEASTEREO_HIP_LIB=$PWD/leastereo_amd/var_$v.so; fi
  timeout -k 10 300 python -u tools/wino2_sweep.py --variants 0 --walks 0 --iters 30 --only conv12_128to64_k3_L1,stem1_32to32_k3_L0 \
    > gpurun_out/r04_p_$v.txt 2>&1 || { tail -20 gpurun_out/r04_p_$v.txt; exit 1; }
  grep -v '^{' gpurun_out/r04_p_$v.txt | grep -v amdgpu.ids | sed "s/^/$v /" | cut -c1-140
done
