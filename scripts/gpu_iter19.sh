#!/bin/bash
# iteration: backward chain epilogues' first Y tiles prefetched a layer early (MMS_CHAIN_YPRE) -- tests, A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
V=$R/multimodalstudio_amd/_variants
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_e2e.py -x -v --timeout 200 --timeout-method thread > gpurun_out/iter19_tests.log 2>&1
for v in "X=0" "MMS_HIP_LIB=$V/libmms_ypre0.so"; do
  echo "$v" >> gpurun_out/iter19_chain.txt
  env $v timeout -k 10 300 python -u scripts/chain_bench.py >> gpurun_out/iter19_chain.txt 2>&1
done
for v in "X=0" "MMS_HIP_LIB=$V/libmms_ypre0.so" "X=0" "MMS_HIP_LIB=$V/libmms_ypre0.so" "X=0" "MMS_HIP_LIB=$V/libmms_ypre0.so"; do
  echo "$v" >> gpurun_out/iter19_ab.jsonl
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 60 --warmup 10 >> gpurun_out/iter19_ab.jsonl 2>> gpurun_out/iter19_ab.err
done
