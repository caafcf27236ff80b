#!/bin/bash
# fused radiance panel: its bit-exactness test, the GPU kernel / e2e / graph tests, and a bench A/B of the fused
# radiance panel (MMS_FUSED_RAD=0: input-column kernel + hash gather) twice each
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_kernels_basic.py \
  tests/test_gpu_e2e.py tests/test_gpu_plugins.py tests/test_gpu_graph.py > gpurun_out/r4g_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/r4g_tests.log
set -e
for rep in 1 2; do for f in 1 0; do
  MMS_FUSED_RAD=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --secondary grid_raw5 \
    > gpurun_out/r4g_bench_rad${f}_$rep.json 2> gpurun_out/r4g_bench_rad${f}_$rep.err
done; done
timeout -k 10 300 python -u scripts/wide_ablate.py run > gpurun_out/r4g_wide_ablate.txt 2>&1
