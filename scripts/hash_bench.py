#!/usr/bin/env python
"""Hash-grid microbenchmark at the bench workload's sizes (diagnostics).

Points are laid out as the SDF batch is: [centre M | 4 taps M] with the taps (2/1024)/sqrt(3) away, centres
sampled along rays (64 per ray) so consecutive rows are neighbouring samples, as in the training step.
Times forward, and backward with/without the table and position gradients, grouped (G=5) and plain.

    python scripts/hash_bench.py [--rays 880] [--log2T 19]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=880)
    ap.add_argument("--log2T", type=int, default=19)
    a = ap.parse_args()
    from multimodalstudio_amd import functions as F
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    R, S = a.rays, 64
    o = torch.nn.functional.normalize(torch.randn(R, 3, generator=g), dim=-1) * 3.0
    d = torch.nn.functional.normalize(-o + 0.3 * torch.randn(R, 3, generator=g), dim=-1)
    t = torch.sort(torch.rand(R, S, generator=g) * 2.0 + 2.0, dim=-1).values
    c = (o[:, None, :] + t[..., None] * d[:, None, :]).reshape(-1, 3).clamp(-1, 1)
    M = c.shape[0]
    delta = 2.0 / 1024 / 3 ** 0.5
    dirs = torch.tensor([[1., -1., -1.], [-1., -1., 1.], [-1., 1., -1.], [1., 1., 1.]])
    x = torch.cat([c] + [c + delta * k for k in dirs], 0).contiguous().to(dev)
    L = 16
    scales = [float(int(16 * (1.3195079 ** l))) for l in range(L)]
    cfg = F.GridCfg(scales, a.log2T, 1.0)
    table = ((torch.rand(L << a.log2T, 2, generator=g) * 2 - 1) * 1e-2).to(dev)
    out = torch.empty(5 * M, 32, device=dev)
    dout = torch.randn(5 * M, 32, generator=g).to(dev)
    dtable = torch.zeros_like(table)
    dpos = torch.zeros_like(x)
    lookups = 5 * M
    print(f"M = {M} centres, {lookups} lookups per pass")

    def rep(name, us, nbytes_per_lookup):
        print(f"{name:44s} {us:9.1f} us  {lookups * nbytes_per_lookup / us / 1e3:8.1f} GB/s algorithmic", flush=True)

    rep("fwd", timeit(lambda: F.grid_fwd(cfg, x, 3, 5 * M, table, L, out, 0)), 1164)
    rep("bwd plain  (dtable + dpos)", timeit(lambda: F.grid_bwd(cfg, x, 3, 5 * M, table, L, dout, 0, dtable, dpos)), 2188)
    rep("bwd plain  (dtable only)", timeit(lambda: F.grid_bwd(cfg, x, 3, 5 * M, table, L, dout, 0, dtable, None)), 2188)
    rep("bwd plain  (dpos only)", timeit(lambda: F.grid_bwd(cfg, x, 3, 5 * M, table, L, dout, 0, None, dpos)), 1164)
    rep("bwd G=5    (dtable + dpos)", timeit(lambda: F.grid_bwd(cfg, x, 3, 5 * M, table, L, dout, 0, dtable, dpos,
                                                               group=5)), 2188)
    rep("bwd G=5    (dtable only)", timeit(lambda: F.grid_bwd(cfg, x, 3, 5 * M, table, L, dout, 0, dtable, None,
                                                             group=5)), 2188)
    rep("dpos gather G=5", timeit(lambda: F._lib.call(
        "mms_hashgrid_dpos_grouped", x.data_ptr(), M, 5, M, 3, table.data_ptr(), cfg.L, cfg.log2T, cfg.F, cfg.interp,
        cfg.scales_ptr, cfg.radius, L, dout.data_ptr(), dout.stride(0), dpos.data_ptr(), 3, F._s())), 1164)
    rep("dpos gather plain (radiance-like, 1/5 rows)", timeit(lambda: F._lib.call(
        "mms_hashgrid_dpos_grouped", x.data_ptr(), M, 1, M, 3, table.data_ptr(), cfg.L, cfg.log2T, cfg.F, cfg.interp,
        cfg.scales_ptr, cfg.radius, L, dout.data_ptr(), dout.stride(0), dpos.data_ptr(), 3, F._s())) * 5, 1164)
    rep("bwd plain 1/5 rows (dtable + dpos) x5", timeit(lambda: F.grid_bwd(cfg, x, 3, M, table, L, dout, 0, dtable,
                                                                           dpos)) * 5, 2188)
    rep("zero dtable (64 MiB memset)", timeit(lambda: dtable.zero_()), 0)


if __name__ == "__main__":
    main()
