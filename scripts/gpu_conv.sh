#!/bin/bash
# converged PSNR runs (grid_raw5, 3000 steps = the whole schedule, FullViewEvaluator on 5 held-out views)
# usage: bash scripts/gpu_conv.sh "fast:1 fp32:4 fast:2:sdf=0 ..."   (job = precision:seed[:PRECISION override])
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
for job in $1; do
  IFS=: read p s ov <<< "$job"
  tag=$p${ov:+_${ov/=/}}
  timeout -k 10 300 python -u scripts/converge_psnr.py --precision $p --steps 3000 --max-iters 3000 --eval-every 3000 \
    --seed $s ${ov:+--override $ov} --out gpurun_out/conv3k_${tag}_s$s.json > gpurun_out/conv3k_${tag}_s$s.log 2>&1
done
