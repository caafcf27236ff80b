#!/bin/bash
# Round-end GPU pass: every -m gpu test, the default bench line (CPU baseline included), a rocprofv3 kernel-trace
# --stats profile of the bench, and the FETCH_SIZE / WRITE_SIZE passes.  Stops at the first fault / timeout.
# usage: bash scripts/gpu_final.sh <tag>
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_$TAG.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
bash scripts/gpu_prof.sh $TAG fast || exit $?
bash scripts/gpu_pmc.sh fast || exit $?
