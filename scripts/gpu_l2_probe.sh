#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
for args in "0 2048 8 64" "4 2048 8 64" "5 2048 8 64 1" "5 2048 8 64 0" "5 2048 4 64 1" "5 2048 4 64 0"; do
  timeout -k 5 60 ./scripts/l2_probe $args >> gpurun_out/l2_probe.log 2>&1 || exit 1
done
