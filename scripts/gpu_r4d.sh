#!/bin/bash
# round-4 checkpoint: every -m gpu test except the training-parity ones (their fixtures are being regenerated), the
# default bench line with the CPU baselines, and a rocprofv3 kernel-trace of the bench workload
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "not train_parity" \
  > gpurun_out/r4d_tests.log 2>&1
timeout -k 10 500 python -u bench.py > gpurun_out/r4d_bench.json 2> gpurun_out/r4d_bench.err
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r4d -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing --secondary '' \
  > $R/gpurun_out/prof_r4d.log 2>&1
