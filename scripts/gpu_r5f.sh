#!/bin/bash
# round-4 final checkpoint: every -m gpu test, smoke(), the default bench line (CPU baselines included), a rocprofv3
# kernel-trace of the bench workload
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 1100 python -u -m pytest tests -m gpu -v -s --timeout 900 --timeout-method thread \
  > gpurun_out/r5f_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5f_smoke.log 2>&1
timeout -k 10 500 python -u bench.py > gpurun_out/r5f_bench.json 2> gpurun_out/r5f_bench.err
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r5f -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing --secondary '' \
  > $R/gpurun_out/prof_r5f.log 2>&1
cd $R
# the fused next-step hit count (MMS_FUSED_COUNT=1, opt-in): its tests and a bench A/B, twice
MMS_FUSED_COUNT=1 timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread \
  tests/test_gpu_graph.py tests/test_gpu_ddp.py > gpurun_out/r5f_count_tests.log 2>&1
for rep in 1 2; do for v in 1 0; do
  MMS_FUSED_COUNT=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --secondary '' \
    > gpurun_out/r5f_count_${v}_$rep.json 2> gpurun_out/r5f_count_${v}_$rep.err
done; done
