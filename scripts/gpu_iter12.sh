#!/bin/bash
# iteration: backward chain epilogue Y-prefetch depth -- chain tests on the default build, then step A/B over variants
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_e2e.py -x -v --timeout 200 --timeout-method thread > gpurun_out/iter12_tests.log 2>&1
V=multimodalstudio_amd/_variants
for v in "X=0" "MMS_HIP_LIB=$V/libmms_y1_1.so" "MMS_HIP_LIB=$V/libmms_y4_4.so" "MMS_HIP_LIB=$V/libmms_y2_2.so" "X=0" "MMS_HIP_LIB=$V/libmms_y1_1.so" "MMS_HIP_LIB=$V/libmms_y4_4.so"; do
  echo "$v" >> gpurun_out/iter12_ab.jsonl
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 60 --warmup 10 >> gpurun_out/iter12_ab.jsonl 2>> gpurun_out/iter12_ab.err
done
