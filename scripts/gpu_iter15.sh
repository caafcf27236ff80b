#!/bin/bash
# iteration: glue copies with 32-bit index math vs 64-bit (variant library) -- parity tests, kernel-trace profiles
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_glue.py tests/test_gpu_graph.py -x -v --timeout 300 --timeout-method thread > gpurun_out/iter15_tests.log 2>&1
bash scripts/gpu_prof.sh r3e fast --secondary ""
MMS_HIP_LIB=$R/multimodalstudio_amd/_variants/libmms_g64.so bash scripts/gpu_prof.sh r3e_g64 fast --secondary ""
