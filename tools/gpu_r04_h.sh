#!/bin/bash
# Round 4 (h): (1) wino tests with the slice-major per-lane weights of the pipelined tile;
# (2) the per-lane tile's fenced schedule (PV = 5) vs PV = 4 on the 16 -> 16 cells;
# (3) same-box A/B of the pipelined tile's weight layout (ab/lib_r04_lanemajor.so = HEAD~0
#     before the change) on its layers, then the C2 bench with each library.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_wino.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r04_h_tests.txt 2>&1 || { tail -30 gpurun_out/r04_h_tests.txt; exit 1; }
tail -1 gpurun_out/r04_h_tests.txt
for v in 1 2 1 2; do
  LEASTEREO_LANE_HALO16=$v timeout -k 10 200 python -u tools/wino2_sweep.py --variants 0 --walks 0 --iters 30 \
    --only cell_16to16_k3_L1 > gpurun_out/r04_h_pv_$v.txt 2>&1 || { tail -20 gpurun_out/r04_h_pv_$v.txt; exit 1; }
  echo "lane16=$v $(grep -v '^{' gpurun_out/r04_h_pv_$v.txt | grep -v amdgpu.ids | cut -c1-130)"
done
L=conv12_128to64_k3_L1,stem1_32to32_k3_L0,cell_32to96_k3_L2_s1grp
for lib in old new old new; do
  if [ $lib = old ]; then export LEASTEREO_HIP_LIB=$PWD/ab/lib_r04_lanemajor.so; else unset LEASTEREO_HIP_LIB; fi
  timeout -k 10 300 python -u tools/wino2_sweep.py --variants 0 --walks 0 --iters 30 --only $L \
    > gpurun_out/r04_h_ab_$lib.txt 2>&1 || { tail -20 gpurun_out/r04_h_ab_$lib.txt; exit 1; }
  grep -v '^{' gpurun_out/r04_h_ab_$lib.txt | grep -v amdgpu.ids | sed "s/^/$lib /" | cut -c1-140
done
for lib in old new old new; do
  if [ $lib = old ]; then export LEASTEREO_HIP_LIB=$PWD/ab/lib_r04_lanemajor.so; else unset LEASTEREO_HIP_LIB; fi
  timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --cpu-baseline 0 --epe 0 > gpurun_out/r04_h_bench_$lib.json 2> gpurun_out/r04_h_bench_$lib.err \
    || { tail -20 gpurun_out/r04_h_bench_$lib.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'])" gpurun_out/r04_h_bench_$lib.json $lib
done
