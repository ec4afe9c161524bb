#!/bin/bash
# One GPU call as a list of steps (replaces the round-4 one-off tools/gpu_r04_*.sh scripts):
#   bash tools/gpu_steps.sh STEP [STEP ...]
# Steps (each under its own time limit; the call stops at the first failing step):
#   smoke                    __graft_entry__.smoke()
#   suite                    the whole -m gpu suite
#   tests=EXPR               pytest -m gpu -k EXPR (EXPR: a -k expression)
#   file=PATH[@EXPR]         pytest PATH [-k EXPR]
#   bench=CFG[@ARGS]         bench.py --config CFG (ARGS: extra flags, '+' for ' ')
#   ab=CFG@ENV_A@ENV_B[@..]  same-box A/B/.., interleaved rounds (tools/gpu_ab.sh; ENV ',' for ' ', '-' none)
#   layers                   per-launch conv list of the C2 forward (tools/layer_list.py)
#   prof=TAG                 rocprofv3 kernel stats + forward breakdown of the default C2 bench
#   py=SCRIPT[@ARGS]         python SCRIPT ARGS ('+' for ' ')
# Outputs under gpurun_out/steps/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/steps
mkdir -p $O
PYT="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread"
for step in "$@"; do
  key=${step%%=*}; val=${step#*=}
  tag=$(echo "$step" | tr -c 'A-Za-z0-9_.-' '_' | cut -c1-60)
  log=$O/$tag.log
  echo "== $step"
  case $key in
    smoke) timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $log 2>&1 ;;
    suite) timeout -k 10 1000 $PYT tests -m gpu > $log 2>&1 ;;
    tests) timeout -k 10 900 $PYT tests -m gpu -k "$val" > $log 2>&1 ;;
    file)
      f=${val%%@*}; k=""; [ "$f" != "$val" ] && k=$(echo "${val#*@}" | tr "+" " ")
      if [ -n "$k" ]; then timeout -k 10 900 $PYT "$f" -k "$k" > $log 2>&1
      else timeout -k 10 900 $PYT "$f" > $log 2>&1; fi ;;
    bench)
      cfg=${val%%@*}; extra=""; [ "$cfg" != "$val" ] && extra=$(echo "${val#*@}" | tr '+' ' ')
      timeout -k 10 900 python3 bench.py --config $cfg $extra > $O/$tag.json 2> $log ;;
    ab)  # ab=CFG@VARIANT@VARIANT[@...]: each variant a ','-separated env list ('-' = none)
      cfg=${val%%@*}; vars=$(echo "${val#*@}" | tr '@' ';' | sed 's/^-;/;/; s/;-;/;;/g; s/;-$/;/')
      CONFIGS=$cfg ROUNDS=${ROUNDS:-2} AB_VARIANTS="$vars" timeout -k 10 1100 bash tools/gpu_ab.sh > $log 2>&1 ;;
    layers) timeout -k 10 300 python3 -u tools/layer_list.py --reps 5 > $log 2>&1 ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$val -o run -- \
        python3 bench.py --steps 5 --warmup 2 --cpu-baseline 0 --epe 0 --pair-check 0 > $O/prof_$val.json 2> $log \
        && python3 tools/trace_report.py $O/prof_$val > $O/prof_${val}_forward.txt ;;
    py)
      s=${val%%@*}; extra=""; [ "$s" != "$val" ] && extra=$(echo "${val#*@}" | tr '+' ' ')
      timeout -k 10 600 python3 -u $s $extra > $log 2>&1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  tail -${TAIL:-4} $log
  [ -f $O/$tag.json ] && python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('value', round(d['value'],2), 'ms', round(d['ms_per_step'],3), 'pair', d.get('pair_epe_px',{}) and d['pair_epe_px'].get('max'))" $O/$tag.json 2>/dev/null
  [ $rc -eq 0 ] || { echo "step $step rc=$rc"; exit $rc; }
done
