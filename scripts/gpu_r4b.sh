#!/bin/bash
# round-4 weight-gradient engine A/B: the LDS-DMA streamed kernel (mms_gemm_tn_stream) -- its fp64 test, the engine
# microbenchmark on the bench step's item sets, and the default bench line with each engine; then the mesh-pyramid
# parity and config-5 fast-preset tests
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels_basic.py \
  -k "tn_grouped" > gpurun_out/r4b_tests.log 2>&1
timeout -k 10 300 python -u scripts/tn_wide_bench.py > gpurun_out/r4b_tnbench.txt 2>&1
for e in wide stream; do
  MMS_TN_ENGINE=$e timeout -k 10 300 python -u bench.py --no-cpu-baseline --secondary grid_raw5 \
    > gpurun_out/r4b_bench_$e.json 2> gpurun_out/r4b_bench_$e.err
done
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_mesh.py \
  "tests/test_gpu_e2e.py::test_e2e_fast_preset_deviation" > gpurun_out/r4b_tests2.log 2>&1
