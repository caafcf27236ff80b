#!/bin/bash
# GPU parity tests only (no -x: every failure is reported).  usage: TESTS="tests/x.py ..." bash scripts/gpu_tests.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_tests.log
exit $rc
