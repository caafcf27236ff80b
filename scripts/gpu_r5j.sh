#!/bin/bash
# HIP runtime knob A/B: kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1) vs the default, twice each
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
for rep in 1 2; do for v in 1 0; do
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --secondary '' \
    > gpurun_out/r5j_bench_${v}_$rep.json 2> gpurun_out/r5j_bench_${v}_$rep.err
done; done
