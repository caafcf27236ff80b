#!/bin/bash
# kernel traces of the bench step with the background branch issued after sampler iteration 0 / 2 / after the
# sampler (MMS_BG_AT), for one-step timelines
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
set -e
for at in -1 0 2; do
  MMS_BG_AT=$at timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_r4p_$at -o run -- \
    python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing --secondary '' \
    > $R/gpurun_out/prof_r4p_$at.log 2>&1
done
