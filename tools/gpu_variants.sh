#!/bin/bash
# time every leastereo_amd/var_*.so on the bf16 layer set, then bench VARIANT_BENCH configs with each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in leastereo_amd/libleastereo_hip.so leastereo_amd/var_*.so; do
  LEASTEREO_HIP_LIB=$PWD/$lib timeout -k 10 120 python3 tools/bf16_layer_bench.py 2>/dev/null; rc=$?
  [ $rc -eq 0 ] || { echo "$lib rc=$rc"; exit $rc; }
done
for lib in leastereo_amd/libleastereo_hip.so leastereo_amd/var_*.so; do
  for c in ${VARIANT_BENCH:-c4}; do
    LEASTEREO_HIP_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --config $c --steps 10 --warmup 3 --cpu-baseline 0 --epe 1 \
      > gpurun_out/vb.json 2>/dev/null; rc=$?
    [ $rc -eq 0 ] || { echo "$lib $c rc=$rc"; exit $rc; }
    python3 -c "import json; d=json.load(open('gpurun_out/vb.json')); print('$lib', '$c', round(d['value'],1), round(d['ms_per_step'],2), d['epe_px']['max_over_ranks'])"
  done
done
