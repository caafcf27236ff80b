#!/bin/bash
# background-branch issue point A/B: MMS_BG_AT=-1 (after the sampler, the default), 0, 1, 2 (after that sampler
# iteration), twice each; the background-stream e2e test under each non-default point first
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
for at in 0 2; do
  MMS_BG_AT=$at timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread \
    tests/test_gpu_e2e.py -k "background_stream or fast_preset" tests/test_gpu_graph.py \
    > gpurun_out/r4n_tests_$at.log 2>&1
done
for rep in 1 2; do for at in -1 0 1 2; do
  MMS_BG_AT=$at timeout -k 10 300 python -u bench.py --no-cpu-baseline --secondary grid_raw5 \
    > gpurun_out/r4n_bench_${at}_$rep.json 2> gpurun_out/r4n_bench_${at}_$rep.err
done; done
