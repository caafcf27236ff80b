#!/bin/bash
# diagnostic: chain-kernel wave-time shares from the stamp build (scripts/chain_stamps.py)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
MMS_HIP_LIB=$R/multimodalstudio_amd/_variants/libmms_stamps.so timeout -k 10 300 python -u scripts/chain_stamps.py > gpurun_out/iter16_stamps.txt 2>&1
