#!/usr/bin/env python
"""GEMM microbenchmark on the exact shapes one training step issues.

Records every hip_ops.gemm call of one bench-config training step, then times each distinct
(mode, M, N, K, strides, splits) in isolation for the requested precisions, next to torch.mm
(hipBLASLt) fp32 / bf16 for orientation.  Prints one line per shape and the per-step totals.

    python scripts/gemm_bench.py [--precs=0,1,2] [--reps 20] [--torch]
"""
from __future__ import annotations

import argparse
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precs", default="0,1,2")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--torch", action="store_true")
    ap.add_argument("--rays", type=int, default=2048)
    a = ap.parse_args()
    from multimodalstudio_amd import hip_ops, functions
    from multimodalstudio_amd.pipeline import Trainer, TrainConfig
    dev = torch.device("cuda", 0)
    tr = Trainer(TrainConfig(method="grid", modalities=("rgb",), num_rays_per_modality=a.rays, log2T=19), dev)
    tr.set_step(95000)
    tr.train_step()
    calls = []
    orig = hip_ops.gemm

    def rec(mode, M, N, K, A, lda, B, ldb, C, ldc, **kw):
        calls.append((mode, M, N, K, lda, ldb, ldc, kw.get("splits", 1), kw.get("bias") is not None,
                      kw.get("act", 0), kw.get("aux") is not None, bool(kw.get("accumulate", False))))
        return orig(mode, M, N, K, A, lda, B, ldb, C, ldc, **kw)

    hip_ops.gemm = rec
    functions.gemm = rec
    tr.train_step()
    torch.cuda.synchronize()
    hip_ops.gemm = orig
    functions.gemm = orig
    cnt = collections.Counter(calls)
    precs = [int(p) for p in a.precs.split(",")]
    names = {0: "NT", 1: "NN", 2: "TN"}
    tot = collections.defaultdict(float)
    flops_tot = 0.0
    print(f"{len(calls)} gemm calls/step, {len(cnt)} distinct")
    hdr = f"{'mode':4s} {'M':>7s} {'N':>5s} {'K':>7s} {'spl':>4s} {'n':>2s} {'GFLOP':>7s} " + \
        " ".join(f"{'p' + str(p) + ' us':>9s} {'TF':>6s}" for p in precs) + ("   torch32 us  torch16 us" if a.torch else "")
    print(hdr)
    for key, n in sorted(cnt.items(), key=lambda kv: -kv[0][1] * kv[0][2] * kv[0][3] * kv[1]):
        mode, M, N, K, lda, ldb, ldc, splits, has_b, act, has_aux, accum = key
        # operand extents (rows x ld) per mode
        if mode == 0:
            A = torch.randn(M, lda, device=dev); B = torch.randn(N, ldb, device=dev); C = torch.empty(M, ldc, device=dev)
        elif mode == 1:
            A = torch.randn(M, lda, device=dev); B = torch.randn(K, ldb, device=dev); C = torch.empty(M, ldc, device=dev)
        else:
            A = torch.randn(K, lda, device=dev); B = torch.randn(K, ldb, device=dev); C = torch.zeros(M, ldc, device=dev)
        bias = torch.randn(N, device=dev) if has_b else None
        Z = torch.empty(M, N, device=dev) if act else None
        aux = torch.randn(M, ldc, device=dev) if has_aux else None
        fl = 2.0 * M * N * K
        flops_tot += fl * n
        line = f"{names[mode]:4s} {M:7d} {N:5d} {K:7d} {splits:4d} {n:2d} {fl / 1e9:7.2f} "
        for p in precs:
            def run():
                orig(mode, M, N, K, A, lda, B, ldb, C, ldc, bias=bias, Z=Z, ldz=N, aux=aux, ldaux=ldc, act=act,
                     dact=act, accumulate=accum, splits=splits, prec=p)
            for _ in range(3):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.reps
            tot[p] += us * n
            line += f"{us:9.1f} {fl / us / 1e6:6.1f} "
        if a.torch:
            for dt in (torch.float32, torch.bfloat16):
                if mode == 0:
                    x, y = A[:, :K].to(dt), B[:, :K].to(dt).T
                elif mode == 1:
                    x, y = A[:, :K].to(dt), B[:, :N].to(dt)
                else:
                    x, y = A[:, :M].to(dt).T, B[:, :N].to(dt)
                for _ in range(3):
                    torch.mm(x, y)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    torch.mm(x, y)
                e1.record()
                torch.cuda.synchronize()
                line += f" {e0.elapsed_time(e1) * 1e3 / a.reps:10.1f}"
        print(line, flush=True)
    print(f"per-step GEMM: {flops_tot / 1e9:.1f} GFLOP; " +
          ", ".join(f"prec{p}: {tot[p] / 1e3:.2f} ms ({flops_tot / tot[p] / 1e6:.1f} TF/s)" for p in precs))


if __name__ == "__main__":
    main()
