#!/bin/bash
# Round checkpoint on the GPU box: every -m gpu test, the default bench line (as the driver runs it), a rocprofv3
# kernel-trace summary and an MFMA-busy PMC pass of the bench workload.  Each GPU step has its own time limit and the
# steps stop at the first failure.
# usage: TAG=r02a bash scripts/gpu_full.sh   (SKIP_PYTEST=1: bench and profiles only)
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-run}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
[ -n "$SKIP_PYTEST" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed" >> gpurun_out/pytest_$TAG.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing --secondary '' \
  > $R/gpurun_out/prof_$TAG.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY \
  --output-format csv -d $R/gpurun_out/pmc_mfma_$TAG -o run -- \
  python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-kernel-timing --secondary '' \
  > $R/gpurun_out/pmc_mfma_$TAG.log 2>&1
