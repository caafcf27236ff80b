#!/bin/bash
# iteration: step A/B of the wide weight-gradient engine's slice reduction (float atomics vs workspace + reduce launch)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
for v in "X=0" "MMS_TN_WS=1" "MMS_TN_WS=1 MMS_TN_BLOCKS=512" "X=0" "MMS_TN_WS=1" "MMS_TN_WS=1 MMS_TN_BLOCKS=512" "X=0"; do
  echo "$v" >> gpurun_out/iter11_ab.jsonl
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-timing --steps 60 --warmup 10 >> gpurun_out/iter11_ab.jsonl 2>> gpurun_out/iter11_ab.err
done
