#!/bin/bash
# round-4 checkpoint: the fused SDF panel test, every other -m gpu test except the training-parity ones (their
# fixtures are still being generated), the default bench line with CPU baselines, the unfused-panel A/B, and a
# rocprofv3 kernel-trace of the bench workload
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "not train_parity" \
  > gpurun_out/r4e_tests.log 2>&1
timeout -k 10 500 python -u bench.py > gpurun_out/r4e_bench.json 2> gpurun_out/r4e_bench.err
MMS_FUSED_PANEL=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --secondary "" \
  > gpurun_out/r4e_bench_unfused.json 2> gpurun_out/r4e_bench_unfused.err
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r4e -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing --secondary '' \
  > $R/gpurun_out/prof_r4e.log 2>&1
