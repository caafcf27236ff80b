#!/bin/bash
# Round check on one MI355X: GPU parity tests, smoke, bench (fast + fp32 presets, with CPU baseline on one).
# A failing test does not stop the bench; a timeout / abort / crash of any GPU step ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
set -e
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --precision fast > gpurun_out/b_fast.json 2> gpurun_out/b_fast.err
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --precision fp32 --no-cpu-baseline > gpurun_out/b_fp32.json 2> gpurun_out/b_fp32.err
