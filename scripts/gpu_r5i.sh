#!/bin/bash
# final tree: rocprofv3 kernel-trace + stats of the bench workload
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r5i -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing --secondary '' \
  > $R/gpurun_out/prof_r5i.log 2>&1
