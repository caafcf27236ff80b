#!/bin/bash
# iteration: hash-grid kernels in XCD-contiguous block order -- hash tests, then step A/B vs the plain order
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels_basic.py -k "hash" tests/test_gpu_e2e.py -x -v --timeout 200 --timeout-method thread > gpurun_out/iter13_tests.log 2>&1
V=multimodalstudio_amd/_variants
for v in "X=0" "MMS_HIP_LIB=$V/libmms_hx0.so" "X=0" "MMS_HIP_LIB=$V/libmms_hx0.so" "X=0" "MMS_HIP_LIB=$V/libmms_hx0.so"; do
  echo "$v" >> gpurun_out/iter13_ab.jsonl
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 60 --warmup 10 >> gpurun_out/iter13_ab.jsonl 2>> gpurun_out/iter13_ab.err
done
