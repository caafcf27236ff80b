#!/usr/bin/env python
"""Fused MLP chain microbenchmark at the bench workload's sizes (diagnostics).

SDF chain (71-256-256-257, split bf16x3) over [centre M | 4 taps M] rows with rows_full = M, its backward, the
sampler's inference form (rows_full = 0), and the radiance chain (317-256-256-256, bf16) fwd/bwd.  Prints time per
launch and the MFMA-rate of the algorithmic flops (bench.py chain_work).

    python scripts/chain_bench.py [--centres 54400]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


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


def params(dims, dev, g):
    out = []
    for k, n in zip(dims[:-1], dims[1:]):
        v = torch.randn(n, k, generator=g) / k ** 0.5
        out += [torch.linalg.vector_norm(v, dim=1, keepdim=True).to(dev).requires_grad_(True),
                v.to(dev).requires_grad_(True), (torch.randn(n, generator=g) * 0.1).to(dev).requires_grad_(True)]
    return out


def kernel_us(fn, reps=10):
    """Average duration of the mms_mlp_chain launches fn makes, from HIP events around each launch (_lib.TIMER), so
    the weight-norm / pack launches of ChainRun.forward are not counted."""
    from multimodalstudio_amd import _lib
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    sys.path.insert(0, ROOT)
    from bench import chain_work
    _lib.TIMER.start({"mms_mlp_chain": chain_work})
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    _lib.TIMER.stop()
    summ = _lib.TIMER.summary()
    return {k: ms * 1e3 for k, (n, ms, _) in summ.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--centres", type=int, default=54400)
    ap.add_argument("--sweep", action="store_true", help="sampler-form chain at 1 block, 1 and 2 block rounds")
    a = ap.parse_args()
    from multimodalstudio_amd import functions as fx
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    M = a.centres

    def run_case(name, dims, acts, prec, rows, rows_full):
        p = params(dims, dev, g)
        X = fx._alloc(rows, dims[0], dev)
        X.copy_(torch.randn(rows, dims[0], generator=g) * 0.3)
        dy = fx._alloc(rows, dims[-1], dev)
        dy.copy_(torch.randn(rows, dims[-1], generator=g))
        run = fx.ChainRun(p, acts, prec)
        keep = rows_full != 0
        tf = timeit(lambda: run.forward(X, keep=keep, rows_full=rows_full))
        K0, N0, N1, N2 = dims
        rf = rows_full
        fl = 2.0 * rows * (K0 * N0 + N0 * N1) + 2.0 * (rf * N2 + (rows - rf)) * N1
        peak = 2500.0 / (3 if prec == 2 else 1)
        print(f"{name:28s} fwd {tf:9.1f} us  {fl / tf / 1e6:7.1f} TF/s ({100 * fl / tf / 1e6 / peak:5.1f}% of {peak:.0f})",
              flush=True)
        if keep:
            def bwd():
                run.forward(X, keep=True, rows_full=rows_full)
                run.backward(dy)
            tb = timeit(bwd) - tf
            flb = 2.0 * (rf * N2 + (rows - rf)) * N1 + 2.0 * rows * (N1 * N0 + N0 * K0)
            print(f"{name:28s} bwd {tb:9.1f} us  (incl. weight-gradient GEMMs; chain-only flops "
                  f"{flb / 1e9:.1f} GFLOP)", flush=True)

    if a.sweep:
        p = params((71, 256, 256, 257), dev, g)
        run = fx.ChainRun(p, fx.SDF_ACTS, 2)
        for rows in [128, 256 * 128, 512 * 128, 2048 * 128]:
            X = fx._alloc(rows, 71, dev)
            X.copy_(torch.randn(rows, 71, generator=g) * 0.3)
            us = kernel_us(lambda: run.forward(X, keep=False, rows_full=0))
            print(f"sdf infer-form chain rows={rows:8d} blocks={rows // 128:5d}  kernel {us}", flush=True)
        for rows_full_frac in [1.0, 0.2, 0.0]:
            rows = 5 * M
            X = fx._alloc(rows, 71, dev)
            X.copy_(torch.randn(rows, 71, generator=g) * 0.3)
            rf = int(rows * rows_full_frac)
            dy = fx._alloc(rows, 257, dev)
            dy.copy_(torch.randn(rows, 257, generator=g))

            def fb():
                run.forward(X, keep=True, rows_full=rf)
                run.backward(dy)
            us = kernel_us(fb)
            print(f"sdf train-form chain rows={rows} rows_full={rf}  kernel {us}", flush=True)
        return
    run_case("sdf 5M (centre+taps)", (71, 256, 256, 257), fx.SDF_ACTS, 2, 5 * M, M)
    run_case("sdf sampler (32 rows/ray)", (71, 256, 256, 257), fx.SDF_ACTS, 2, M // 2, 0)
    run_case("radiance", (317, 256, 256, 256), fx.RAD_ACTS, 1, M, M)


if __name__ == "__main__":
    main()
