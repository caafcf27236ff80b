#!/bin/bash
# iteration: LDS-staged background input backward (variant bg1: MMS_BG_BWD_STAGED=1) -- e2e / glue / train-parity tests on
# the variant library, per-step profiles and bench A/B against the default build
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
V=$R/multimodalstudio_amd/_variants
MMS_HIP_LIB=$V/libmms_bg1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_glue.py tests/test_gpu_train_parity.py -x -v --timeout 300 --timeout-method thread > gpurun_out/iter23_tests.log 2>&1
bash scripts/gpu_prof.sh i23_base fast --secondary ""
MMS_HIP_LIB=$V/libmms_bg1.so bash scripts/gpu_prof.sh i23_bg1 fast --secondary ""
for v in "X=0" "MMS_HIP_LIB=$V/libmms_bg1.so" "X=0" "MMS_HIP_LIB=$V/libmms_bg1.so"; do
  echo "$v" >> gpurun_out/iter23_ab.jsonl
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-timing --steps 60 --warmup 10 >> gpurun_out/iter23_ab.jsonl 2>> gpurun_out/iter23_ab.err
done
