#!/bin/bash
# one-launch reported inv_s (mms_inv_variance): glue / e2e / graph tests, bench twice
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_glue.py \
  tests/test_gpu_e2e.py tests/test_gpu_graph.py > gpurun_out/r5h_tests.log 2>&1
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --secondary '' > gpurun_out/r5h_bench_$rep.json \
    2> gpurun_out/r5h_bench_$rep.err
done
