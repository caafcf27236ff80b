#!/bin/bash
# Measurement pass (no tests): the default bench line with the CPU baseline, a rocprofv3 kernel-trace --stats profile
# of the bench, and the FETCH_SIZE / WRITE_SIZE passes.  usage: bash scripts/gpu_measure.sh <tag>
TAG=${1:-measure}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
bash scripts/gpu_prof.sh $TAG fast || exit $?
bash scripts/gpu_pmc.sh fast || exit $?
