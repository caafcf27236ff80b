#!/bin/bash
# hash variants (SDF walk + plain walk), the MFMA-utilisation PMC pass, one more converged-PSNR seed of the fast preset
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 200 python -u scripts/hash_variants.py run > gpurun_out/iter8_hash.log 2>&1
bash scripts/gpu_pmc_mfma.sh fast
bash scripts/gpu_conv.sh "fast:9"
