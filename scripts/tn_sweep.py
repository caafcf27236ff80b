"""Weight-gradient (TN) GEMM time vs split-K count on the step's shapes (bf16 operands, fp32 accumulate, colsum)."""
import sys
import torch
sys.path.insert(0, ".")
from multimodalstudio_amd import hip_ops, functions as fx

dev = torch.device("cuda", 0)
shapes = [(256, 256, 32768), (256, 283, 32768), (128, 256, 32768), (256, 39, 32768), (256, 256, 110000),
          (256, 317, 110000), (64, 256, 110000), (256, 256, 550000)]
for prec in (1, 2):
    for N, K, M in shapes:
        if prec == 2 and M < 500000:
            continue
        A = fx._alloc(M, N, dev).normal_()
        B = fx._alloc(M, K, dev).normal_()
        C = torch.zeros(N, K, device=dev)
        db = torch.zeros(N, device=dev)
        res = []
        for splits in (4, 8, 16, 32, 64, 128, 256):
            if M // splits < 128:
                continue
            for _ in range(3):
                hip_ops.gemm(hip_ops.TN, N, K, M, A, A.stride(0), B, B.stride(0), C, K, accumulate=True,
                             splits=splits, prec=prec, colsum=db)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                hip_ops.gemm(hip_ops.TN, N, K, M, A, A.stride(0), B, B.stride(0), C, K, accumulate=True,
                             splits=splits, prec=prec, colsum=db)
            e1.record()
            torch.cuda.synchronize()
            res.append((splits, e0.elapsed_time(e1) / 20 * 1e3))
        tiles = ((N + 127) // 128) * ((K + 127) // 128)
        print(f"prec {prec} N {N} K {K} M {M} (default splits {hip_ops._splits_for(M, tiles)}): " +
              " ".join(f"s{s}={t:.1f}us" for s, t in res), flush=True)
