#!/bin/bash
# hash backward A/B + hash tests, then converged PSNR (grid_raw5, 3000 steps, 3 seeds) with the non-SDF families on
# mode 4 (split-bf16x3 forward, bf16 backward) and on the all-x3 preset
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels_basic.py -k hashgrid -x -q --timeout 120 --timeout-method thread > gpurun_out/hash_tests.log 2>&1
timeout -k 10 120 python scripts/hash_bench.py > gpurun_out/hash_new.log 2>&1
MMS_HIP_LIB=$R/abtest/libmms_hip_old.so timeout -k 10 120 python scripts/hash_bench.py > gpurun_out/hash_old.log 2>&1
for s in 1 2 3; do
  timeout -k 10 200 python scripts/converge_psnr.py --precision fast --override radiance=4 heads=4 background=4 \
    --steps 3000 --max-iters 3000 --eval-every 3000 --seed $s --out gpurun_out/conv3k_fast_m4_s$s.json > gpurun_out/conv3k_fast_m4_s$s.log 2>&1
done
for s in 1 2 3; do
  timeout -k 10 200 python scripts/converge_psnr.py --precision bf16x3 \
    --steps 3000 --max-iters 3000 --eval-every 3000 --seed $s --out gpurun_out/conv3k_bf16x3_s$s.json > gpurun_out/conv3k_bf16x3_s$s.log 2>&1
done
