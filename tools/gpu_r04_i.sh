#!/bin/bash
# Round 4 (i): fenced step schedules (lea_conv3d_wino_set_fence bit mask) -- bit identity,
# then same-box timing of the L0 8 -> 8 depth-paired tile (bit 0) and the pipelined W x D
# tile's layers (bit 1) against the compiler's schedules.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_wino.py -x -q --timeout 120 --timeout-method thread -k halo16 \
  > gpurun_out/r04_i_tests.txt 2>&1 || { tail -30 gpurun_out/r04_i_tests.txt; exit 1; }
tail -1 gpurun_out/r04_i_tests.txt
L=cell_8to8_k3_L0,conv12_128to64_k3_L1,stem1_32to32_k3_L0,cell_32to96_k3_L2_s1grp
for f in 0 3 0 3; do
  LEASTEREO_WINO_FENCE=$f timeout -k 10 300 python -u tools/wino2_sweep.py --variants 0 --walks 0 --iters 30 --only $L \
    > gpurun_out/r04_i_f$f.txt 2>&1 || { tail -20 gpurun_out/r04_i_f$f.txt; exit 1; }
  grep -v '^{' gpurun_out/r04_i_f$f.txt | grep -v amdgpu.ids | sed "s/^/fence=$f /" | cut -c1-140
done
# ablations of the pipelined tile with the slice-major weights (timing only: wrong outputs)
for v in base nouxf nowdma novpass nohalo nomfma; do
  if [ $v = base ]; then unset LEASTEREO_HIP_LIB; else export LEASTEREO_HIP_LIB=$PWD/leastereo_amd/var_$v.so; fi
  timeout -k 10 300 python -u tools/wino2_sweep.py --variants 0 --walks 0 --iters 30 --only conv12_128to64_k3_L1,stem1_32to32_k3_L0 \
    > gpurun_out/r04_i_abl_$v.txt 2>&1 || { tail -20 gpurun_out/r04_i_abl_$v.txt; exit 1; }
  grep -v '^{' gpurun_out/r04_i_abl_$v.txt | grep -v amdgpu.ids | sed "s/^/$v /" | cut -c1-140
done
unset LEASTEREO_HIP_LIB
timeout -k 10 300 python -u tools/layer_list.py --reps 5 > gpurun_out/r04_i_layer_list.txt 2>&1 || { tail -20 gpurun_out/r04_i_layer_list.txt; exit 1; }
tail -1 gpurun_out/r04_i_layer_list.txt
for f in 0 4 6 0 4 6; do
  LEASTEREO_WINO_FENCE=$f timeout -k 10 300 python -u tools/wino2_sweep.py --variants 0 --walks 0 --iters 30 --only conv12_128to64_k3_L1,stem1_32to32_k3_L0,cell_32to96_k3_L2_s1grp \
    > gpurun_out/r04_i_u$f.txt 2>&1 || { tail -20 gpurun_out/r04_i_u$f.txt; exit 1; }
  grep -v '^{' gpurun_out/r04_i_u$f.txt | grep -v amdgpu.ids | sed "s/^/ufence=$f /" | cut -c1-140
done
