#!/bin/bash
# LDS-staged panel rows: bit-exact tests under both settings, the launches alone A/B, the bench twice per setting
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
for v in 1 0; do
  MMS_RAD_STAGED=$v timeout -k 10 200 python -u -m pytest -v --timeout 100 --timeout-method thread \
    tests/test_gpu_kernels_basic.py -k "panel" > gpurun_out/r4o_tests_$v.log 2>&1
  MMS_RAD_STAGED=$v timeout -k 10 200 python -u scripts/panel_bench.py >> gpurun_out/r4o_panel.txt 2>&1
done
for rep in 1 2; do for v in 1 0; do
  MMS_RAD_STAGED=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --secondary '' \
    > gpurun_out/r4o_bench_${v}_$rep.json 2> gpurun_out/r4o_bench_${v}_$rep.err
done; done
