#!/bin/bash
# full GPU suite on the current defaults, then a repeated bench A/B of the weight-gradient engine / stream
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/iter4_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/iter4_tests.log
[ $rc -le 1 ] || exit $rc
set -e
for v in "X=0" "MMS_TN_ENGINE=tiled MMS_SYNC_WGRAD=0" "X=0" "MMS_TN_ENGINE=tiled MMS_SYNC_WGRAD=0" "MMS_SYNC_WGRAD=0" "X=0"; do
  echo "$v" >> gpurun_out/iter4_ab.jsonl
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-timing --secondary "" --steps 60 --warmup 10 >> gpurun_out/iter4_ab.jsonl 2>> gpurun_out/iter4_ab.err
done
