#!/bin/bash
# Iteration pass: the default bench line (no CPU baseline), then every gpu test.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/b_iter.json 2> gpurun_out/b_iter.err || exit $?
bash scripts/gpu_tests.sh
