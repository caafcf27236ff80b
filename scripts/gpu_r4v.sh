#!/bin/bash
# pose / variance gradients in place, composite without the padded row: e2e / graph / ddp / glue / plugin / eval
# tests, the bench twice, one kernel trace
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e

timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_e2e.py \
  tests/test_gpu_graph.py tests/test_gpu_ddp.py tests/test_gpu_glue.py tests/test_gpu_plugins.py tests/test_gpu_eval.py > gpurun_out/r4v_tests.log 2>&1
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --secondary grid_raw5 > gpurun_out/r4v_bench_$rep.json \
    2> gpurun_out/r4v_bench_$rep.err
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_r4v -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing --secondary '' \
  > $R/gpurun_out/prof_r4v.log 2>&1
