#!/bin/bash
# iteration: wgrad / e2e tests, hash-backward variants, weight-gradient workspace sweep, bench A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels_basic.py tests/test_gpu_e2e.py tests/test_gpu_chain.py -x -v --timeout 200 --timeout-method thread > gpurun_out/iter6_tests.log 2>&1
timeout -k 10 200 python -u scripts/hash_variants.py run > gpurun_out/iter6_hash.log 2>&1
timeout -k 10 200 python -u scripts/tn_wide_bench.py > gpurun_out/iter6_tn.log 2>&1
for v in "X=0" "MMS_TN_WS=0" "X=0" "MMS_TN_WS=0"; do
  echo "$v" >> gpurun_out/iter6_ab.jsonl
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-timing --secondary "" --steps 60 --warmup 10 >> gpurun_out/iter6_ab.jsonl 2>> gpurun_out/iter6_ab.err
done
