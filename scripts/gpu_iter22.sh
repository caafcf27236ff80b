#!/bin/bash
# iteration: sumsq launch shape under the optimizer / training-parity tests; config-5 (grid_bg5) bench line; default bench
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_train_parity.py tests/test_gpu_ddp.py -x -v --timeout 300 --timeout-method thread > gpurun_out/iter22_tests.log 2>&1
timeout -k 10 300 python -u bench.py --config grid_bg5 --secondary "" > gpurun_out/bench_grid_bg5.json 2> gpurun_out/bench_grid_bg5.err
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 60 --warmup 10 > gpurun_out/iter22_bench.json 2> gpurun_out/iter22_bench.err
