#!/bin/bash
# wide weight-gradient kernel A/B: the kernel tests under the product library, then a bench A/B against the
# variant libraries named in VARIANTS (scripts/lib_variants.py)
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_kernels_basic.py -k "wide16 or tn_grouped" > gpurun_out/wd_unit.log 2>&1 || exit 1
TAG=wd VARIANTS=${VARIANTS:-"MMS_HIP_LIB=multimodalstudio_amd/_variants/libmms_wd2.so base"} REPS=3 timeout -k 10 800 bash scripts/gpu_ab.sh
