#!/bin/bash
# quick parity subset on the current tree, the default bench line, a rocprofv3 kernel-trace profile of the bench,
# and the FETCH / WRITE traffic passes.  usage: bash scripts/gpu_r3prof.sh <tag>
TAG=${1:-r3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_graph.py tests/test_gpu_glue.py tests/test_gpu_chain.py tests/test_gpu_sampler.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
bash scripts/gpu_prof.sh $TAG fast || exit $?
bash scripts/gpu_pmc.sh fast || exit $?
