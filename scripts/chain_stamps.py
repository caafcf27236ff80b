#!/usr/bin/env python
"""Where a chain kernel's waves spend their cycles (diagnostics): runs the SDF and radiance chains of the bench
workload on the stamp build of the library (scripts/lib_variants.py stamps: csrc/mlp_chain.hip MMS_CHAIN_STAMPS=1)
and prints, per layer, the share of wave time in the k-steps' wait + barrier, the ring / input issue + get_b, the
fragment reads + MFMA issue, and the layer entry (the previous layer's last MFMAs + the work between layers).

    MMS_HIP_LIB=multimodalstudio_amd/_variants/libmms_stamps.so python scripts/chain_stamps.py
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
K = 17
SEG = ["wait", "get_b", "mfma", "entry"]


def read(lib, nwaves):
    buf = (ctypes.c_ulonglong * (nwaves * K))()
    assert lib.mms_chain_stamps(buf, nwaves * K, 0) == 0
    return np.frombuffer(buf, dtype=np.uint64).reshape(nwaves, K).astype(np.float64)


def report(name, st, groups):
    for gname, sel in groups.items():
        s = st[sel]
        tot = s.sum(1).mean()
        parts = []
        for l in range(4):
            v = s[:, 4 * l:4 * l + 4].mean(0)
            if v.sum() == 0:
                continue
            parts.append(f"L{l}: " + " ".join(f"{SEG[k]} {100 * v[k] / tot:4.1f}%" for k in range(4)))
        print(f"{name:10s} {gname:8s} {tot:9.0f} clk/wave | " + " | ".join(parts) +
              f" | tail {100 * s[:, 16].mean() / tot:4.1f}%", flush=True)


def main():
    from multimodalstudio_amd import _lib, functions as fx
    fx.PRECISION["bwd16"] = int(os.environ.get("MMS_STAMP_BWD16", "1"))   # the backward chains on prec 6 (fast_h16b)
    lib = _lib.lib()
    lib.mms_chain_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int]
    lib.mms_chain_stamps.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    M = 55360
    for name, dims, acts, rows, rf in (("sdf", (71, 256, 256, 257), fx.SDF_ACTS, 5 * M, M),
                                       ("radiance", (317, 256, 256, 256), fx.RAD_ACTS, M, M)):
        p = []
        for k, n in zip(dims[:-1], dims[1:]):
            v = torch.randn(n, k, generator=g) / k ** 0.5
            p += [torch.linalg.vector_norm(v, dim=1, keepdim=True).to(dev).requires_grad_(True),
                  v.to(dev).requires_grad_(True), (torch.randn(n, generator=g) * 0.1).to(dev).requires_grad_(True)]
        X = fx._alloc(rows, dims[0], dev)
        X.copy_(torch.randn(rows, dims[0], generator=g) * 0.3)
        dy = fx._alloc(rows, dims[-1], dev)
        dy.copy_(torch.randn(rows, dims[-1], generator=g))
        run = fx.ChainRun(p, acts, 2)
        nb = (rows + 127) // 128
        groups = {"all": slice(0, 4 * nb)}
        if rf != rows:
            groups = {"centre": slice(0, 4 * (rf // 128)), "taps": slice(4 * (rf // 128 + 1), 4 * nb)}
        for _ in range(3):
            run.forward(X, keep=True, rows_full=rf)
            run.backward(dy)
        torch.cuda.synchronize()
        assert lib.mms_chain_stamps(None, 0, 1) == 0
        run.forward(X, keep=True, rows_full=rf)
        torch.cuda.synchronize()
        report(name + " fwd", read(lib, 4 * nb), groups)
        assert lib.mms_chain_stamps(None, 0, 1) == 0
        run.backward(dy)
        torch.cuda.synchronize()
        report(name + " bwd", read(lib, 4 * nb), groups)


if __name__ == "__main__":
    main()
