#!/bin/bash
# rocprofv3 kernel-trace + stats of bench.py (one precision preset) -> gpurun_out/prof_<tag>/
# usage: bash scripts/gpu_prof.sh <tag> <precision> [extra bench args]
set -e
TAG=$1; PREC=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing --precision $PREC "$@" \
  > $R/gpurun_out/prof_$TAG.log 2>&1
