#!/bin/bash
# chain kernels: GPU tests for both SDF chain kernels, then the chain microbenchmark with each
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -m gpu -v -s --timeout 120 --timeout-method thread \
  > gpurun_out/c16_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/c16_tests.log
grep -q "failed\|error" gpurun_out/c16_tests.log && grep -q "FAILED\|ERROR" gpurun_out/c16_tests.log && exit 1
for v in 1 0; do
  MMS_CHAIN16=$v timeout -k 10 200 python -u scripts/chain_bench.py --sweep > gpurun_out/c16_bench_$v.log 2>&1 || exit 1
done
