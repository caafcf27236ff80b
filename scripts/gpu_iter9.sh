#!/bin/bash
# iteration: graph / e2e / train-parity / ddp tests on the side-stream radiance grid backward, then bench A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_e2e.py tests/test_gpu_train_parity.py tests/test_gpu_ddp.py tests/test_gpu_optim.py -x -v --timeout 300 --timeout-method thread > gpurun_out/iter9_tests.log 2>&1
for v in "X=0" "MMS_RAD_GRID_SIDE=0" "X=0" "MMS_RAD_GRID_SIDE=0"; do
  echo "$v" >> gpurun_out/iter9_ab.jsonl
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-timing --secondary "" --steps 60 --warmup 10 >> gpurun_out/iter9_ab.jsonl 2>> gpurun_out/iter9_ab.err
done
echo "serial background" >> gpurun_out/iter9_ab.jsonl
timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-timing --secondary "" --steps 60 --warmup 10 --serial-background >> gpurun_out/iter9_ab.jsonl 2>> gpurun_out/iter9_ab.err
