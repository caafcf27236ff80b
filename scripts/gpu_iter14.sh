#!/bin/bash
# iteration: glue kernels without per-element 64-bit index divisions -- parity tests, bench, kernel-trace profile
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_glue.py tests/test_gpu_train_parity.py tests/test_gpu_graph.py -x -v --timeout 300 --timeout-method thread > gpurun_out/iter14_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 60 --warmup 10 >> gpurun_out/iter14_ab.jsonl 2>> gpurun_out/iter14_ab.err
done
bash scripts/gpu_prof.sh r3d fast
