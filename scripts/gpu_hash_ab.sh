#!/bin/bash
# hash backward A/B: abtest/libmms_hip_old.so (the previous walk kernel) vs the tree's library, + hash parity tests
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels_basic.py -k hashgrid -x -q --timeout 120 --timeout-method thread > gpurun_out/hash_tests.log 2>&1
timeout -k 10 120 python scripts/hash_bench.py > gpurun_out/hash_new.log 2>&1
MMS_HIP_LIB=$R/abtest/libmms_hip_old.so timeout -k 10 120 python scripts/hash_bench.py > gpurun_out/hash_old.log 2>&1
