#!/bin/bash
# Round 4 (t): the f32 disparity register form with buffer loads (scalar plane offsets) and the
# device library's expf sequence minus its overflow select -- disparity tests, bit-identity of
# the output against ab/lib_head.so on random costs, per-launch time.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "disparity or e2e or golden" > gpurun_out/r04_t_tests.txt 2>&1 || { tail -30 gpurun_out/r04_t_tests.txt; exit 1; }
tail -1 gpurun_out/r04_t_tests.txt
for scale in 3 30; do
  PYTHONPATH=$PWD LEASTEREO_HIP_LIB=$PWD/ab/lib_head.so timeout -k 10 120 python -u tools/disp_dump.py gpurun_out/disp_old.npy $scale || exit 1
  PYTHONPATH=$PWD timeout -k 10 120 python -u tools/disp_dump.py gpurun_out/disp_new.npy $scale || exit 1
  python3 -c "import numpy as np; a=np.load('gpurun_out/disp_old.npy'); b=np.load('gpurun_out/disp_new.npy'); print('scale $scale bit-identical:', np.array_equal(a.view(np.uint32), b.view(np.uint32)), a.size)"
done
