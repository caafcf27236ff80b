#!/bin/bash
# the step loss in one launch each way (MMS_FUSED_STEP_LOSS) and the composite keeping the background rows itself:
# e2e / graph / ddp / glue / eval / plugin tests, bench A/B twice
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_e2e.py \
  tests/test_gpu_graph.py tests/test_gpu_ddp.py tests/test_gpu_glue.py tests/test_gpu_eval.py tests/test_gpu_plugins.py \
  > gpurun_out/r5b_tests.log 2>&1
for rep in 1 2; do for v in 1 0; do
  MMS_FUSED_STEP_LOSS=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --secondary '' \
    > gpurun_out/r5b_bench_${v}_$rep.json 2> gpurun_out/r5b_bench_${v}_$rep.err
done; done
