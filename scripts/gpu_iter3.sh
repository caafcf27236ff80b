#!/bin/bash
# iteration: chain / small-linear / hash / e2e tests, then bench A/B over environment variants, then the full bench line
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 500 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_e2e.py tests/test_gpu_kernels_basic.py -x -v --timeout 200 --timeout-method thread > gpurun_out/iter3_tests.log 2>&1
for v in "X=0" "MMS_TN_ENGINE=wide" "MMS_SYNC_WGRAD=1" "MMS_TN_ENGINE=wide MMS_SYNC_WGRAD=1" "MMS_TAP_WGRAD=0" "X=0"; do
  echo "$v" >> gpurun_out/iter3_ab.jsonl
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-timing --secondary "" --steps 60 --warmup 10 >> gpurun_out/iter3_ab.jsonl 2>> gpurun_out/iter3_ab.err
done
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 --warmup 10 > gpurun_out/iter3_bench.json 2> gpurun_out/iter3_bench.err
