#!/bin/bash
# iteration: kernel / e2e / train-parity tests, then bench A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels_basic.py tests/test_gpu_e2e.py tests/test_gpu_chain.py tests/test_gpu_train_parity.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/iter5_tests.log 2>&1
for v in "X=0" "MMS_SYNC_WGRAD=0 MMS_TN_BLOCKS=128" "MMS_FUSED_LOSS=0" "X=0" "MMS_SYNC_WGRAD=0 MMS_TN_BLOCKS=128"; do
  echo "$v" >> gpurun_out/iter5_ab.jsonl
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-timing --secondary "" --steps 60 --warmup 10 >> gpurun_out/iter5_ab.jsonl 2>> gpurun_out/iter5_ab.err
done
