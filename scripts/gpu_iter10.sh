#!/bin/bash
# iteration: wide weight-gradient engine with a 3-deep register pipeline -- tests, microbenchmark, bench A/B vs depth 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels_basic.py -k "tn_grouped or tn_wide" -x -v --timeout 120 --timeout-method thread > gpurun_out/iter10_tests.log 2>&1
timeout -k 10 300 python -u scripts/tn_wide_bench.py > gpurun_out/iter10_tnbench.txt 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_train_parity.py tests/test_gpu_graph.py -x -v --timeout 300 --timeout-method thread >> gpurun_out/iter10_tests.log 2>&1
for v in "X=0" "MMS_TN_DEPTH=2" "X=0" "MMS_TN_DEPTH=2"; do
  echo "$v" >> gpurun_out/iter10_ab.jsonl
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-timing --secondary "" --steps 60 --warmup 10 >> gpurun_out/iter10_ab.jsonl 2>> gpurun_out/iter10_ab.err
done
