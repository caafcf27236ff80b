#!/bin/bash
# iteration: hash tests on the fine-level bypass, hash variants, bench A/B against the all-merge library
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels_basic.py tests/test_gpu_e2e.py tests/test_gpu_plugins.py -x -v --timeout 200 --timeout-method thread > gpurun_out/iter7_tests.log 2>&1
timeout -k 10 200 python -u scripts/hash_variants.py run > gpurun_out/iter7_hash.log 2>&1
timeout -k 10 200 python -u scripts/hash_bench.py > gpurun_out/iter7_hash_bench.log 2>&1
F16=$R/multimodalstudio_amd/_variants/libmms_hip_fine16.so
for v in "X=0" "MMS_HIP_LIB=$F16" "X=0" "MMS_HIP_LIB=$F16"; do
  echo "$v" >> gpurun_out/iter7_ab.jsonl
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-timing --secondary "" --steps 60 --warmup 10 >> gpurun_out/iter7_ab.jsonl 2>> gpurun_out/iter7_ab.err
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/iter7_bench.json 2> gpurun_out/iter7_bench.err
