#!/bin/bash
# sampler panels formed from the spacing bins (mms_sdf_panel_rays_fwd): bit-exact panel tests, the sampler / e2e /
# graph tests, then the bench twice with and without (MMS_FUSED_SAMPLER)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_kernels_basic.py \
  tests/test_gpu_sampler.py tests/test_gpu_e2e.py tests/test_gpu_graph.py > gpurun_out/r4q_tests.log 2>&1
for rep in 1 2; do for v in 1 0; do
  MMS_FUSED_SAMPLER=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --secondary '' \
    > gpurun_out/r4q_bench_${v}_$rep.json 2> gpurun_out/r4q_bench_${v}_$rep.err
done; done
