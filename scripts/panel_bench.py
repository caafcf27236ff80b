#!/usr/bin/env python
"""MLP input-panel launches alone at the bench step's sizes (diagnostics): mms_rad_panel_fwd (radiance rows, M =
880 rays x 64 samples) and mms_sdf_panel_fwd (the SDF batch, centre + 4 taps).  Run once per MMS_RAD_STAGED /
MMS_SDF_STAGED setting (read once per process by the library) to A/B the LDS-staged row writes.

    python scripts/panel_bench.py
"""
from __future__ import annotations

import os
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    from multimodalstudio_amd import _lib, functions as fx
    from multimodalstudio_amd.functions import _alloc
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    R, S = 880, 64
    o = torch.nn.functional.normalize(torch.randn(R, 3, generator=g), dim=-1) * 3.0
    d = torch.nn.functional.normalize(-o + 0.3 * torch.randn(R, 3, generator=g), dim=-1)
    t = torch.sort(torch.rand(R, S, generator=g) * 2.0 + 2.0, dim=-1).values
    pos = (o[:, None, :] + t[..., None] * d[:, None, :]).reshape(-1, 3).clamp(-1, 1).contiguous().to(dev)
    M, G = R * S, 256
    dirs = d.to(dev)
    normals = torch.nn.functional.normalize(torch.randn(M, 3, generator=g), dim=-1).to(dev)
    out = torch.randn(M, 264, generator=g).to(dev)
    geo = out[:, 1:1 + G]
    L, log2T = 16, 19
    cfg = fx.GridCfg([float(int(16 * (1.3195079 ** l))) for l in range(L)], log2T, 1.0)
    table = ((torch.rand(L << log2T, 2, generator=g) * 2 - 1) * 1e-2).to(dev)
    Xr = _alloc(M, 3 + 25 + G + 1 + 32, dev)
    Xs = _alloc(5 * M, 71, dev)
    delta = 2.0 / 1024 / 3 ** 0.5

    def rad():
        _lib.call("mms_rad_panel_fwd", pos.data_ptr(), 3, dirs.data_ptr(), normals.data_ptr(), geo.data_ptr(),
                  geo.stride(0), M, S, G, table.data_ptr(), cfg.L, cfg.log2T, cfg.F, cfg.interp, cfg.scales_ptr,
                  cfg.radius, L, Xr.data_ptr(), Xr.stride(0), fx._s())

    def sdf():
        _lib.call("mms_sdf_panel_fwd", pos.data_ptr(), 3, M, 4, delta, 6, table.data_ptr(), cfg.L, cfg.log2T, cfg.F,
                  cfg.interp, cfg.scales_ptr, cfg.radius, L, Xs.data_ptr(), Xs.stride(0), fx._s())

    tag = f"rad_staged={os.environ.get('MMS_RAD_STAGED', '1')} sdf_staged={os.environ.get('MMS_SDF_STAGED', '1')}"
    for name, fn, rows, ld in (("rad_panel", rad, M, Xr.stride(0)), ("sdf_panel", sdf, 5 * M, Xs.stride(0))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000.0 / 20
        print(f"{tag} {name}: {us:7.1f} us  ({rows} rows, ld {ld})", flush=True)


if __name__ == "__main__":
    main()
