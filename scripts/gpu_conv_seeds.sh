set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mesh.py tests/test_gpu_e2e.py -v -s --timeout 200 --timeout-method thread > gpurun_out/mesh_e2e.log 2>&1 || true
for s in 1 2 3; do
  timeout -k 10 200 python scripts/converge_psnr.py --precision fast --steps 3000 --max-iters 3000 --eval-every 3000 --seed $s --out gpurun_out/conv3k_fast_s$s.json > gpurun_out/conv3k_fast_s$s.log 2>&1
done
for s in 1 2 3; do
  timeout -k 10 300 python scripts/converge_psnr.py --precision fp32 --steps 3000 --max-iters 3000 --eval-every 3000 --seed $s --out gpurun_out/conv3k_fp32_s$s.json > gpurun_out/conv3k_fp32_s$s.log 2>&1
done
