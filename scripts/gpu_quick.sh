#!/bin/bash
# Quick GPU iteration: selected parity tests + one bench line (fast preset).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_chain.py} -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --precision fast --no-cpu-baseline > gpurun_out/b_fast.json 2> gpurun_out/b_fast.err
