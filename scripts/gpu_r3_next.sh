#!/bin/bash
# round-3 measurement batch: parity scatter at checkpoints, clean kernel traces of grid_rgb and grid_raw5, new GPU tests
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_mesh.py tests/test_gpu_eval.py tests/test_gpu_ddp.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r3_newtests.log 2>&1 || true
for s in 95000 50000; do
  timeout -k 10 240 python scripts/parity_scatter.py --config raw5 --start-step $s --runs 4 --eps 1e-15 --checkpoints 0 25 50 100 > gpurun_out/scatter_ck_$s.log 2>&1
done
bash scripts/gpu_prof.sh r3b fast --secondary ''
bash scripts/gpu_prof.sh r3b5 fast --config grid_raw5 --secondary ''
