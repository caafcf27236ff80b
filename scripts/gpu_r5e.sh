#!/bin/bash
# the tail's hit count in one launch (mms_count_hits): graph / e2e tests, bench A/B twice (MMS_FUSED_COUNT)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_graph.py \
  tests/test_gpu_ddp.py > gpurun_out/r5e_tests.log 2>&1
for rep in 1 2; do for v in 1 0; do
  MMS_FUSED_COUNT=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --secondary '' \
    > gpurun_out/r5e_bench_${v}_$rep.json 2> gpurun_out/r5e_bench_${v}_$rep.err
done; done
