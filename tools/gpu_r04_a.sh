#!/bin/bash
# Round 4, first confirmation: parity/head tests after the tapsum row bound, the bench
# line with the torch GPU-eager leg (both MIOpen modes), the train-step tool's torch modes.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_heads.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r04_a_tests.txt 2>&1 || { tail -20 gpurun_out/r04_a_tests.txt; exit 1; }
tail -2 gpurun_out/r04_a_tests.txt
timeout -k 10 600 python -u bench.py --gpu-eager default,benchmark > gpurun_out/r04_a_bench.json 2> gpurun_out/r04_a_bench.err \
  || { tail -20 gpurun_out/r04_a_bench.err; exit 1; }
python - <<'P'
import json
d = json.loads(open("gpurun_out/r04_a_bench.json").read().strip().splitlines()[-1])
print("value", d["value"], "frac", d["roofline"]["frac"])
print(json.dumps(d["cpu_baseline"].get("torch_gpu_eager"), indent=1))
print(d["per_rank_step_ms"], d["host_threads_per_rank"])
P
timeout -k 10 500 python -u tools/train_bench.py > gpurun_out/r04_a_train.jsonl 2>&1 || { tail -20 gpurun_out/r04_a_train.jsonl; exit 1; }
cat gpurun_out/r04_a_train.jsonl | grep "^{"
