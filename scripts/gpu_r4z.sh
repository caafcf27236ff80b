#!/bin/bash
# weight gradients on a side stream beside the hash-grid backward with atomic-free split-K partials
# (MMS_SYNC_WGRAD=0 MMS_TN_WS=1) vs the default (inline, atomics), twice each
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
for rep in 1 2; do for v in "0 1" "1 0"; do
  set -- $v
  MMS_SYNC_WGRAD=$1 MMS_TN_WS=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --secondary '' \
    > gpurun_out/r4z_bench_$1$2_$rep.json 2> gpurun_out/r4z_bench_$1$2_$rep.err
done; done
