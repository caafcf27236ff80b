#!/bin/bash
# PMC counters of the chain microbenchmark's kernels (diagnostics): LDS array activity / conflicts, waits, MFMA busy
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
for v in 1 0; do
  MMS_CHAIN16=$v timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY \
    SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    --output-format csv -d $R/gpurun_out/pmc_chain_$v -o run -- python3 $R/scripts/chain_bench.py --sweep \
    > $R/gpurun_out/pmc_chain_$v.log 2>&1 || exit 1
done
