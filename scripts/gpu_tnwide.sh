#!/bin/bash
# wide weight-gradient engine: kernel test, engine/stage/blocks sweep on the step's item sets, then bench lines
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels_basic.py tests/test_gpu_chain.py -k "tn_grouped or small_linear or chain_head" -x -v --timeout 120 --timeout-method thread > gpurun_out/tnwide_tests.log 2>&1
timeout -k 10 300 python -u scripts/tn_wide_bench.py > gpurun_out/tnwide_bench.log 2>&1
for v in "wide 16" "tiled 16" "wide 32" "wide 16" "tiled 16"; do
  set -- $v
  MMS_TN_ENGINE=$1 MMS_TN_STAGE=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-timing --secondary "" --steps 60 --warmup 10 >> gpurun_out/bench_tn_ab.jsonl 2>> gpurun_out/bench_tn_ab.err
done
