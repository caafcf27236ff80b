#!/bin/bash
# banked optimizer (one zero / clip / AdamW launch for both groups, the zero arena in the same zero launch, arena-carved
# step outputs, persistent backward seed): optimizer / graph / e2e / ddp / glue tests, bench A/B (MMS_BANKED_OPTIM),
# one kernel trace
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_optim.py \
  tests/test_gpu_graph.py tests/test_gpu_e2e.py tests/test_gpu_ddp.py tests/test_gpu_glue.py \
  > gpurun_out/r4r_tests.log 2>&1
for rep in 1 2; do for v in 1 0; do
  MMS_BANKED_OPTIM=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --secondary '' \
    > gpurun_out/r4r_bench_${v}_$rep.json 2> gpurun_out/r4r_bench_${v}_$rep.err
done; done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_r4r -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing --secondary '' \
  > $R/gpurun_out/prof_r4r.log 2>&1
