#!/bin/bash
# chain16 variants (scripts/lib_variants.py) through the chain microbenchmark: VARIANTS="base c16d2 ..."
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
export MMS_CHAIN16=${MMS_CHAIN16:-1}
for v in ${VARIANTS:-base}; do
  echo "== $v" >> gpurun_out/abl.log
  if [ $v = base ]; then
    timeout -k 10 120 python -u scripts/chain_bench.py --sweep 2>&1 | grep -v amdgpu.ids >> gpurun_out/abl.log || exit 1
  else
    MMS_HIP_LIB=multimodalstudio_amd/_variants/libmms_$v.so timeout -k 10 120 python -u scripts/chain_bench.py --sweep \
      2>&1 | grep -v amdgpu.ids >> gpurun_out/abl.log || exit 1
  fi
done
