#!/bin/bash
# round-4c full checkpoint: every -m gpu test, the default bench line (CPU baselines included), a rocprofv3
# kernel-trace of the bench workload
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 1100 python -u -m pytest tests -m gpu -v -s --timeout 900 --timeout-method thread \
  > gpurun_out/r4y_tests.log 2>&1
timeout -k 10 500 python -u bench.py > gpurun_out/r4y_bench.json 2> gpurun_out/r4y_bench.err
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r4y -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing --secondary '' \
  > $R/gpurun_out/prof_r4y.log 2>&1
