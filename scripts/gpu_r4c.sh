#!/bin/bash
# weight-gradient launch shape A/B in the bench step: K-slice partial tiles by float atomics vs the workspace + reduce
# launch (MMS_TN_WS), at 256 and 512 blocks (MMS_TN_BLOCKS); then the mesh-pyramid parity test
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
for ws in 0 1; do for nb in 256 512; do
  MMS_TN_WS=$ws MMS_TN_BLOCKS=$nb timeout -k 10 300 python -u bench.py --no-cpu-baseline --secondary grid_raw5 \
    > gpurun_out/r4c_bench_ws${ws}_$nb.json 2> gpurun_out/r4c_bench_ws${ws}_$nb.err
done; done
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_mesh.py \
  > gpurun_out/r4c_mesh.log 2>&1
