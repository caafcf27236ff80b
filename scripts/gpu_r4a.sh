#!/bin/bash
# round-4 check: the data-parallel split-graph path (2-rank gloo test), graph tests, the config-5 e2e fixtures, the
# default bench line, and an A/B of the LDS-staged background input backward (variant bg1) on the grid_bg5 workload
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ddp.py \
  tests/test_gpu_graph.py tests/test_gpu_e2e.py > gpurun_out/r4a_tests.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --secondary "" > gpurun_out/r4a_bench.json 2> gpurun_out/r4a_bench.err
for v in base bg1; do
  lib=""; [ $v = bg1 ] && lib=multimodalstudio_amd/_variants/libmms_bg1.so
  env ${lib:+MMS_HIP_LIB=$lib} timeout -k 10 300 python -u bench.py --config grid_bg5 --no-cpu-baseline --secondary "" \
    > gpurun_out/r4a_bg5_$v.json 2> gpurun_out/r4a_bg5_$v.err
done
