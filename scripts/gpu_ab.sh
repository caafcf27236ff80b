#!/bin/bash
# Bench A/B on one box (replaces the round-4 one-off wrappers): each variant is a space-free env assignment list
# ("MMS_X=1,MMS_Y=0" or "base"; the item P=<preset> selects bench.py --precision instead of setting a variable), run
# REPS times interleaved, one JSON line per run in gpurun_out/ab_<tag>_<variant>_<rep>.json
#   usage: TAG=x VARIANTS="base MMS_X=0" REPS=2 ARGS="--no-cpu-baseline --secondary ''" bash scripts/gpu_ab.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
TAG=${TAG:-ab}
for rep in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-base}; do
    envs=()
    prec=()
    if [ "$v" != "base" ]; then
      IFS=',' read -ra items <<< "$v"
      for it in "${items[@]}"; do
        if [[ $it == P=* ]]; then prec=(--precision "${it#P=}"); else envs+=("$it"); fi
      done
    fi
    out=gpurun_out/ab_${TAG}_$(echo "$v" | tr "=,/." "____")_$rep
    env "${envs[@]}" timeout -k 10 300 python -u bench.py ${ARGS:---no-cpu-baseline --secondary ''} "${prec[@]}" > $out.json 2> $out.err
    echo "$v rep $rep: $(python -c "import json,sys; d=json.loads(open('$out.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
  done
done
