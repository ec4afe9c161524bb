#!/bin/bash
# Round 4 (c): record the HIP bf16 figures at C3 and C4 (LEA_BF16_RECORD=1).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
rm -f gpurun_out/bf16_hip_measured.json
LEA_BF16_RECORD=1 timeout -k 10 1000 python -u -m pytest tests/test_gpu_bf16.py -x -v --timeout 900 --timeout-method thread \
  -k "batch8" > gpurun_out/r04_c_bf16.txt 2>&1 || { tail -30 gpurun_out/r04_c_bf16.txt; exit 1; }
tail -3 gpurun_out/r04_c_bf16.txt
python -c "
import json; d=json.load(open('gpurun_out/bf16_hip_measured.json'))
for k,v in d['cases'].items(): print(k, v['epe_max'], max(v['stage_rel_l2_pair0'].values()))"
