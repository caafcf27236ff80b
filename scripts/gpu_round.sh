#!/bin/bash
# GPU iteration: selected parity tests, then the bench in graph and eager mode (fast preset, no CPU baseline).
# usage: TESTS="tests/x.py ..." bash scripts/gpu_round.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_round.log 2>&1
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/b_graph.json 2> gpurun_out/b_graph.err
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --mode eager > gpurun_out/b_eager.json 2> gpurun_out/b_eager.err
