#!/bin/bash
# Quick GPU iteration: kernel parity tests + one bench line (fast preset) + PSNR noise probe.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels_basic.py tests/test_gpu_e2e.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --precision fast --no-cpu-baseline > gpurun_out/b_fast.json 2> gpurun_out/b_fast.err
timeout -k 10 300 python scripts/train_psnr.py --steps 300 --every 100 --precision fp32 --start-step 95000 --runs 3 > gpurun_out/noise_300.log 2>&1
