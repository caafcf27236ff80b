#!/bin/bash
# in-step A/B of the wide weight-gradient kernel's two-register-set pipeline (default) vs the round-3 loop (variant
# wpipe0), twice each, plus the weight-gradient and e2e tests on the default library
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_kernels_basic.py \
  tests/test_gpu_e2e.py tests/test_gpu_graph.py > gpurun_out/r4i_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/r4i_tests.log
set -e
for rep in 1 2; do for v in pipe wpipe0; do
  lib=""; [ $v = wpipe0 ] && lib=multimodalstudio_amd/_variants/libmms_wpipe0.so
  env ${lib:+MMS_HIP_LIB=$lib} timeout -k 10 300 python -u bench.py --no-cpu-baseline --secondary grid_raw5 \
    > gpurun_out/r4i_bench_${v}_$rep.json 2> gpurun_out/r4i_bench_${v}_$rep.err
done; done
