#!/usr/bin/env python
"""GEMM phase ablation (diagnostics only; cdna_hip_programming.md §7 'Ablate').

    python scripts/gemm_ablate.py build      # CPU container: compile variants into build/ablate/
    python scripts/gemm_ablate.py run        # GPU box: time every variant on the SDF-MLP shapes

Variants compile csrc/gemm.hip alone with -DMMS_GEMM_ABLATE=<bits>: 1 = no epilogue stores,
2 = no MFMA, 4 = no global loads.  Timing-only builds: their outputs are wrong by design.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
OUT = ROOT / "build" / "ablate"
VARIANTS = {"full": 0, "no_store": 1, "no_mfma": 2, "no_load": 4, "only_epi": 6, "only_load": 3, "only_mfma": 5}


def build():
    OUT.mkdir(parents=True, exist_ok=True)
    src = ROOT / "multimodalstudio_amd" / "csrc" / "gemm.hip"
    procs = []
    for name, bits in VARIANTS.items():
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-shared",
               "-munsafe-fp-atomics", f"-DMMS_GEMM_ABLATE={bits}", str(src), "-o", str(OUT / f"gemm_{name}.so")]
        procs.append(subprocess.Popen(cmd))
    for p in procs:
        if p.wait() != 0:
            raise SystemExit("ablation build failed")
    print("built", sorted(os.listdir(OUT)))


def run():
    import torch
    dev = torch.device("cuda", 0)
    libs = {}
    for name in VARIANTS:
        L = ctypes.CDLL(str(OUT / f"gemm_{name}.so"), mode=os.RTLD_LOCAL)
        f = L.mms_gemm
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_int] * 3 + [ctypes.c_int64] * 3 + [ctypes.c_void_p, ctypes.c_int64] * 3 + \
            [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
             ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int,
             ctypes.c_void_p, ctypes.c_void_p]
        libs[name] = f
    M = 269760
    shapes = [  # (label, ta, tb, M, N, K, act/Z, aux, splits)
        ("NT fwd 256x256 +act+Z", 0, 0, M, 256, 256, True, False, 1),
        ("NN dX 256x256 +aux", 0, 1, M, 256, 256, False, True, 1),
        ("TN dW 256x256 split", 1, 1, 256, 256, M, False, False, 256),
        ("NT fwd K=72", 0, 0, M, 256, 72, True, False, 1),
    ]
    for prec in (0, 1, 2):
        for label, ta, tb, m, n, k, act, aux, splits in shapes:
            A = torch.randn(k, m, device=dev) if ta else torch.randn(m, k, device=dev)
            B = torch.randn(k, n, device=dev) if tb else torch.randn(n, k, device=dev)
            C = torch.zeros(m, n, device=dev)
            Z = torch.empty(m, n, device=dev) if act else None
            X = torch.randn(m, n, device=dev) if aux else None
            bias = torch.randn(n, device=dev) if act else None
            s = torch.cuda.current_stream().cuda_stream
            line = f"prec{prec} {label:24s}"
            for name, f in libs.items():
                def call():
                    rc = f(prec, ta, tb, m, n, k, A.data_ptr(), A.shape[1], B.data_ptr(), B.shape[1], C.data_ptr(), n,
                           None if bias is None else bias.data_ptr(), None if Z is None else Z.data_ptr(), n,
                           None if X is None else X.data_ptr(), n, 2 if act else 0, 2 if aux else 0, 100.0, 20.0,
                           1 if splits > 1 else 0, splits, -1, None, s)
                    assert rc == 0
                for _ in range(3):
                    call()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    call()
                e1.record()
                torch.cuda.synchronize()
                line += f" {name}={e0.elapsed_time(e1) * 100:.0f}us"
            print(line, flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
