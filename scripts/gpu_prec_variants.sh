#!/bin/bash
# which part of the fast preset costs converged PSNR: 3000-step grid_raw5 runs (3 seeds) with single MLP families
# moved back to split-bf16x3
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
set -e
for v in "heads=2" "radiance=2" "background=2"; do
  tag=$(echo $v | tr '=' '_')
  for s in 1 2 3; do
    timeout -k 10 200 python scripts/converge_psnr.py --precision fast --override $v --steps 3000 --max-iters 3000 \
      --eval-every 3000 --seed $s --out gpurun_out/conv3k_fast_${tag}_s$s.json > gpurun_out/conv3k_fast_${tag}_s$s.log 2>&1
  done
done
