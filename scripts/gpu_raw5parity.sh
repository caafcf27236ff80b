#!/bin/bash
# the raw5 training-parity test alone, printing its per-checkpoint mean dPSNR lines
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest "tests/test_gpu_train_parity.py::test_train_parity_grid_raw_5mod" -x -v -s --timeout 300 --timeout-method thread > gpurun_out/raw5parity_$1.log 2>&1
