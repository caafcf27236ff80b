#!/usr/bin/env python
"""Weight-gradient engines on the bench step's item sets (diagnostics): mms_gemm_tn_grouped (128 x 128 tiles) vs
mms_gemm_tn_wide (256 x 256 tiles) at several block targets, split-bf16x3 and bf16, with the algorithmic bytes rate.

    python scripts/tn_wide_bench.py
"""
from __future__ import annotations

import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

M = 55360   # centre rows of the grid_rgb bench step (865 hit rays x 64 samples)
SETS = {
    # (N_out, K_in, rows, dZ row offset): the SDF MLP (taps: 4 M more rows), the radiance MLP, the background base
    "sdf": [(256, 71, 5 * M), (256, 256, 5 * M), (257, 256, M), (1, 256, 4 * M)],
    "radiance": [(256, 317, M), (256, 256, M), (256, 256, M)],
    "bg_head": [(256, 283, 131072), (256, 256, 131072), (256, 256, 131072), (128, 256, 131072)],
}


def timeit(fn, reps=10):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    from multimodalstudio_amd import hip_ops
    from multimodalstudio_amd.functions import _alloc
    dev = torch.device("cuda", 0)
    for name, spec in SETS.items():
        items, nbytes, ref = [], 0, None
        for N, K, R in spec:
            dZ = _alloc(R, N, dev).normal_()
            X = _alloc(R, K, dev).normal_()
            dW = torch.zeros(N, K, device=dev)
            db = torch.zeros(N, device=dev)
            items.append((N, K, R, dZ, X, dW, db))
            nbytes += R * 4 * (N + K)
        for prec in (2,):
            outs = {}
            for engine, sr, targets in (("tiled", None, (None,)), ("wide", 16, (256, 512)), ("wide-ws", 16, (256, 512))):
                hip_ops.TN_WORKSPACE = engine == "wide-ws"
                engine = "wide" if engine == "wide-ws" else engine
                for tb in targets:
                    for it in items:
                        it[5].zero_()
                    run = lambda: hip_ops.gemm_tn_grouped(items, prec, target_blocks=tb, engine=engine, stage_rows=sr)
                    run()
                    torch.cuda.synchronize()
                    outs[(engine, sr, tb, hip_ops.TN_WORKSPACE)] = [it[5].clone() for it in items]
                    us = timeit(run)
                    ref = outs[("tiled", None, None, False)]
                    err = max(((a - b).abs().max() / b.abs().max()).item()
                              for a, b in zip(outs[(engine, sr, tb, hip_ops.TN_WORKSPACE)], ref))
                    tag = engine + ("+ws" if engine == "wide" and hip_ops.TN_WORKSPACE else "")
                    print(f"{name:9s} prec {prec} {tag:8s}/{str(sr):4s} blocks {str(tb):5s} {us:8.1f} us "
                          f"{nbytes / us / 1e3:7.1f} GB/s algorithmic  (vs tiled: {err:.1e})", flush=True)


if __name__ == "__main__":
    main()
