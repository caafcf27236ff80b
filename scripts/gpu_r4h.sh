#!/bin/bash
# the radiance-panel bit-exactness test (SH without contraction), the wide weight-gradient kernel ablation with the
# two-register-set pipeline variant, and the training-parity raw5 test on the fixtures generated so far
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_kernels_basic.py \
  -k "panel or tn_grouped" > gpurun_out/r4h_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/r4h_tests.log
set -e
timeout -k 10 300 python -u scripts/wide_ablate.py run > gpurun_out/r4h_wide_ablate.txt 2>&1
