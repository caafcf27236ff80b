#!/bin/bash
# hash merge v2 A/B + hash / chain / e2e tests, then the x3 `fast` preset's bench line
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels_basic.py -k hashgrid -x -q --timeout 120 --timeout-method thread > gpurun_out/hash_tests.log 2>&1
timeout -k 10 120 python scripts/hash_bench.py > gpurun_out/hash_new.log 2>&1
MMS_HIP_LIB=$R/abtest/libmms_hip_old.so timeout -k 10 120 python scripts/hash_bench.py > gpurun_out/hash_old.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_e2e.py -q --timeout 200 --timeout-method thread > gpurun_out/chain_e2e_tests.log 2>&1 || true
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 --warmup 10 > gpurun_out/bench_fastx3.json 2> gpurun_out/bench_fastx3.err
