#!/bin/bash
# MFMA-pipe utilisation of the bench workload's kernels: one rocprofv3 --pmc pass (4 SQ + 1 GRBM counters),
# kernel dispatches only.  usage: bash scripts/gpu_pmc_mfma.sh <tag>   -> gpurun_out/pmc_mfma_<tag>/
set -e
TAG=${1:-fast}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE \
  --output-format csv -d $R/gpurun_out/pmc_mfma_$TAG -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing --secondary "" \
  > $R/gpurun_out/pmc_mfma_$TAG.log 2>&1
