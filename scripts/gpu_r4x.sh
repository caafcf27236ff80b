#!/bin/bash
# weight-gradient engine knobs in the step (MMS_TN_BLOCKS / MMS_TN_STAGE / MMS_TN_WS), one bench each
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
set -e
for cfg in "256 16 0" "384 16 0" "512 16 0" "192 16 0" "256 32 0" "256 16 1" "512 16 1" "256 16 0"; do
  set -- $cfg
  MMS_TN_BLOCKS=$1 MMS_TN_STAGE=$2 MMS_TN_WS=$3 timeout -k 10 300 python -u bench.py --no-cpu-baseline \
    --secondary '' > gpurun_out/r4x_bench_$1_$2_$3.json 2> gpurun_out/r4x_bench_$1_$2_$3.err
  python - "$1 $2 $3" gpurun_out/r4x_bench_$1_$2_$3.json <<'PY' >> gpurun_out/r4x_summary.txt
import json, sys
d = json.load(open(sys.argv[2]))
w = [k for k in d["roofline_kernels"] if k["kernel"].startswith("mms_gemm_tn_wide")]
print(sys.argv[1], round(d["value"]), d["ms_per_step"], w[0]["ms_per_step"] if w else None)
PY
done
