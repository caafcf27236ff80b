#!/bin/bash
# stream-order A/B: the background branch issued after the foreground sampler (MMS_BG_AFTER=1) and/or the step graphs
# captured on a high-priority stream (MMS_STREAM_PRIO=1), twice each; graph tests under both flags first
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread \
  tests/test_gpu_graph.py tests/test_gpu_e2e.py > gpurun_out/r4k_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/r4k_tests.log
set -e
for rep in 1 2; do for v in "0 0" "1 0" "0 1" "1 1"; do
  set -- $v
  MMS_BG_AFTER=$1 MMS_STREAM_PRIO=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --secondary grid_raw5 \
    > gpurun_out/r4k_bench_$1$2_$rep.json 2> gpurun_out/r4k_bench_$1$2_$rep.err
done; done
