#!/bin/bash
# Round 4 (u): the pipelined tile's 8-wave x-split form (conv3d_wino2p8_kernel) -- Winograd tests
# (bit-identity to the 4-wave pipeline), e2e golden, the L2 / L1 layers with the form forced on
# and off, per-launch list, same-box C2 bench A/B against ab/lib_head.so.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_wino.py tests/test_gpu_parity.py -x -q --timeout 300 \
  --timeout-method thread -k "wino or halo or lane or xsplit or e2e or golden or full" > gpurun_out/r04_u_tests.txt 2>&1 \
  || { tail -30 gpurun_out/r04_u_tests.txt; exit 1; }
tail -1 gpurun_out/r04_u_tests.txt
for xs in 0 2 1; do
  LEASTEREO_WINO2_XSPLIT=$xs timeout -k 10 200 python3 tools/wino2_sweep.py --variants 0 --iters 20 \
    --only cell_32to32_k3_L2,cell_32to96_k3_L2_s1grp,cell_16to32_k3_L1_s1grp2,conv12_128to64_k3_L1 > gpurun_out/r04_u_sweep_$xs.txt 2>&1 \
    || { tail -20 gpurun_out/r04_u_sweep_$xs.txt; exit 1; }
  grep -v "^{" gpurun_out/r04_u_sweep_$xs.txt | grep -v amdgpu.ids | sed "s/^/xsplit=$xs /" | cut -c1-150
done
timeout -k 10 300 python -u tools/layer_list.py --reps 5 > gpurun_out/r04_u_layer_list.txt 2>&1 || { tail -20 gpurun_out/r04_u_layer_list.txt; exit 1; }
grep "wino2p\|conv launches" gpurun_out/r04_u_layer_list.txt | sort -k7 | uniq -c -f6 | head -6
for side in old new old new; do
  if [ $side = old ]; then export LEASTEREO_HIP_LIB=$PWD/ab/lib_head.so; else unset LEASTEREO_HIP_LIB; fi
  timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --cpu-baseline 0 --epe 0 > gpurun_out/r04_u_bench_$side.json 2> gpurun_out/r04_u_bench_$side.err \
    || { tail -20 gpurun_out/r04_u_bench_$side.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r04_u_bench_$side.json $side
done
