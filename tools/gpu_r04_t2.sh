#!/bin/bash
# Round 4 (t2): disparity register form, three builds timed and compared bit for bit:
# old (ab/lib_head.so), exp-only (leastereo_amd/var_dexp.so), buffer loads + exp (in-tree).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for rep in 1 2; do
for side in old dexp both; do
  case $side in old) L=$PWD/ab/lib_head.so;; dexp) L=$PWD/leastereo_amd/var_dexp.so;; both) L=$PWD/leastereo_amd/libleastereo_hip.so;; esac
  PYTHONPATH=$PWD LEASTEREO_HIP_LIB=$L timeout -k 10 120 python -u tools/disp_dump.py gpurun_out/disp_$side.npy 3 || exit 1
done
done
python3 -c "import numpy as np; a=np.load('gpurun_out/disp_old.npy'); [print(s, 'bit-identical:', np.array_equal(a.view(np.uint32), np.load('gpurun_out/disp_%s.npy' % s).view(np.uint32))) for s in ('dexp','both')]"
