#!/bin/bash
# isolate the first-run e2e failure: the rgb e2e test alone, 3 fresh processes with the shared accumulators and one
# without
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 1 0; do
  MMS_GRAD_ACC=$v timeout -k 10 200 python -u -m pytest -q --timeout 100 --timeout-method thread \
    "tests/test_gpu_e2e.py::test_e2e_train_step" >> gpurun_out/r4t_tests.log 2>&1
  echo "acc=$v rc=$?" >> gpurun_out/r4t_tests.log
done
exit 0
