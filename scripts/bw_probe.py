#!/usr/bin/env python
"""HBM calibration on the box: torch copy / reduction / hipBLASLt GEMMs on the SDF-layer shapes."""
import torch

dev = torch.device("cuda", 0)


def t(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


M, K = 269760, 256
a = torch.randn(M, K, device=dev)
b = torch.empty_like(a)
us = t(lambda: b.copy_(a))
print(f"copy 276MB: {us:.1f} us  {2 * a.numel() * 4 / us / 1e3:.0f} GB/s")
us = t(lambda: torch.add(a, 1.0, out=b))
print(f"add  276MB: {us:.1f} us  {2 * a.numel() * 4 / us / 1e3:.0f} GB/s")
us = t(lambda: a.sum(dim=1))
print(f"rowsum 276MB: {us:.1f} us  {a.numel() * 4 / us / 1e3:.0f} GB/s")
w = torch.randn(256, K, device=dev)
us = t(lambda: torch.mm(a, w.T))
print(f"fp32 mm 270k x256x256: {us:.1f} us")
ab, wb = a.bfloat16(), w.bfloat16()
us = t(lambda: torch.mm(ab, wb.T))
print(f"bf16 mm 270k x256x256: {us:.1f} us")
us = t(lambda: torch.nn.functional.softplus(a, beta=100, threshold=20))
print(f"softplus 276MB: {us:.1f} us  {2 * a.numel() * 4 / us / 1e3:.0f} GB/s")
