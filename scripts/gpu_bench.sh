set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --precision fp32 > gpurun_out/b_fp32.json 2> gpurun_out/b_fp32.err
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --precision bf16x3 > gpurun_out/b_x3.json 2> gpurun_out/b_x3.err
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --precision fast > gpurun_out/b_fast.json 2> gpurun_out/b_fast.err
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof2 -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing --precision fp32 > $R/gpurun_out/prof2.log 2>&1
