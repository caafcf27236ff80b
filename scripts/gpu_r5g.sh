#!/bin/bash
# final verification of the committed defaults (fused hit count on): every -m gpu test, smoke(), the default bench
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
timeout -k 10 1100 python -u -m pytest tests -m gpu -v -s --timeout 900 --timeout-method thread \
  > gpurun_out/r5g_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5g_smoke.log 2>&1
timeout -k 10 500 python -u bench.py > gpurun_out/r5g_bench.json 2> gpurun_out/r5g_bench.err
