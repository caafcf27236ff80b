#!/bin/bash
# the config-5 training-parity test (fp32 and the benchmarked preset), per-seed lines streamed
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -v -s --timeout 900 --timeout-method thread \
  "tests/test_gpu_train_parity.py::test_train_parity_config5" > gpurun_out/r4l_parity.log 2>&1
echo "pytest rc=$?" >> gpurun_out/r4l_parity.log
