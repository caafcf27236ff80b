#!/bin/bash
# main-stream weight gradients deferred to the end of the backward (MMS_DEFER_WGRAD): graph / e2e tests under it, bench
# A/B twice
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
MMS_DEFER_WGRAD=1 timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread \
  tests/test_gpu_graph.py tests/test_gpu_e2e.py > gpurun_out/r5d_tests.log 2>&1
for rep in 1 2; do for v in 1 0; do
  MMS_DEFER_WGRAD=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --secondary grid_raw5 \
    > gpurun_out/r5d_bench_${v}_$rep.json 2> gpurun_out/r5d_bench_${v}_$rep.err
done; done
