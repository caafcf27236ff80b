#!/bin/bash
# Round-3 GPU iteration: the listed parity tests (stop at the first failure), then the bench (graph mode, fast preset,
# no CPU baseline) with its secondary grid_raw5 line.  usage: TESTS="tests/x.py ..." bash scripts/gpu_r3.sh <tag>
TAG=${1:-iter}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/bench_$TAG.json \
  2> gpurun_out/bench_$TAG.err
