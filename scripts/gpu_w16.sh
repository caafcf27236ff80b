#!/bin/bash
# fast_h16c (fp16 hidden-layer weight gradients) checkpoint: the kernel / chain unit tests, the envelope-gated e2e and
# full-size preset tests, a graph-replayed NaN probe, then a bench A/B against fast_h16b.  Test failures (exit 1)
# still run the rest; anything else (a fault, abort, time limit) ends the script.
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_kernels_basic.py \
  tests/test_gpu_chain.py -k "wide16 or tn_grouped or fp16_backward or antisymmetric" > gpurun_out/w16_unit.log 2>&1
rc=$?; echo "unit rc=$rc"; [ $rc -le 1 ] || exit $rc
MMS_FAST_PRESET=fast_h16c timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_e2e.py tests/test_gpu_fullsize.py tests/test_gpu_graph.py -k "fast_preset or matches_eager" > gpurun_out/w16_e2e.log 2>&1
rc=$?; echo "e2e rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u scripts/nan_probe.py fast_h16c 12 graph > gpurun_out/nan_h16c_g.log 2>&1 || exit 1
grep "^step" gpurun_out/nan_h16c_g.log | tail -2
TAG=w16 VARIANTS="base P=fast_h16c" REPS=2 timeout -k 10 500 bash scripts/gpu_ab.sh
