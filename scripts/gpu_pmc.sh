#!/bin/bash
# HBM traffic counters for the bench workload: one rocprofv3 --pmc pass per counter (FETCH_SIZE and WRITE_SIZE
# do not fit one pass on gfx950), kernel-trace only, no other trace domains.
# usage: bash scripts/gpu_pmc.sh <precision>
set -e
PREC=${1:-fast}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/pmc_${PREC}_$C -o run -- \
    python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing --secondary "" --precision $PREC \
    > $R/gpurun_out/pmc_${PREC}_$C.log 2>&1
done
