#!/bin/bash
# fp16-panel presets checkpoint (PRESET, default fast_h16d): the kernel / chain unit tests, the envelope-gated e2e,
# full-size and graph-vs-eager tests under PRESET, a graph-replayed NaN probe, then a bench A/B of fast_h16b against
# VARIANTS.  Test failures (exit 1) still run the rest; anything else (a fault, abort, time limit) ends the script.
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out && export TMPDIR=/tmp
P=${PRESET:-fast_h16d}
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_kernels_basic.py \
  tests/test_gpu_chain.py -k "wide16 or tn_grouped or fp16_backward or antisymmetric" > gpurun_out/w16_unit.log 2>&1
rc=$?; echo "unit rc=$rc"; [ $rc -le 1 ] || exit $rc
MMS_FAST_PRESET=$P timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_e2e.py tests/test_gpu_fullsize.py tests/test_gpu_graph.py -k "fast_preset or matches_eager" \
  > gpurun_out/w16_e2e.log 2>&1
rc=$?; echo "e2e rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u scripts/nan_probe.py $P 12 graph > gpurun_out/nan_probe.log 2>&1 || exit 1
grep "^step" gpurun_out/nan_probe.log | tail -1
TAG=w16 VARIANTS=${VARIANTS:-"base P=fast_h16c P=$P"} REPS=2 timeout -k 10 600 bash scripts/gpu_ab.sh
