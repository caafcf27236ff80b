#!/bin/bash
# round-3d evidence on the current tree: the default bench line (with the CPU baseline), a rocprofv3 kernel-trace
# profile of the bench, the FETCH / WRITE traffic passes and the MFMA-busy pass
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r3d_final.json 2> gpurun_out/bench_r3d_final.err
bash scripts/gpu_prof.sh r3d_final fast
bash scripts/gpu_pmc.sh fast
bash scripts/gpu_pmc_mfma.sh r3d
