#!/bin/bash
# iteration: gradient sum-of-squares launch shape (unroll / grid) -- optimizer tests, kernel-trace profiles per variant
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
V=$R/multimodalstudio_amd/_variants
timeout -k 10 300 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_graph.py -x -v --timeout 200 --timeout-method thread > gpurun_out/iter21_tests.log 2>&1
bash scripts/gpu_prof.sh i21_base fast --secondary ""
for v in ssg512 ssg512u8 ssg256u8 ssg1k; do
  MMS_HIP_LIB=$V/libmms_$v.so bash scripts/gpu_prof.sh i21_$v fast --secondary ""
done
