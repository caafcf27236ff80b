#!/usr/bin/env python
"""Weight-gradient (TN) GEMM diagnostics: split-K tile map x phase ablation x split count, on the step's shapes.

    python scripts/wgrad_bench.py build   # CPU container: compile csrc/gemm.hip variants into scratch/lib/
    python scripts/wgrad_bench.py run     # GPU box: time every variant; a read-bandwidth reference per shape

Variants: xcd{0,1} (-DMMS_GEMM_XCDSPLIT: the split-K slices' tiles on one XCD or spread), ablation bits
(-DMMS_GEMM_ABLATE: 1 = no epilogue stores / atomics, 2 = no MFMA, 4 = no global loads).  Timing-only builds.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
OUT = ROOT / "scratch" / "lib"
VARIANTS = {"x0_full": (0, 0), "x1_full": (1, 0), "x1_nostore": (1, 1), "x1_nomfma": (1, 2), "x1_noload": (1, 4)}
SHAPES = [  # (prec, N, K, M rows)
    (1, 256, 256, 110000), (1, 256, 320, 110000), (1, 256, 256, 32768), (1, 256, 288, 32768), (1, 64, 256, 110000),
    (2, 256, 256, 550000), (2, 256, 72, 550000)]


def build():
    OUT.mkdir(parents=True, exist_ok=True)
    src = ROOT / "multimodalstudio_amd" / "csrc" / "gemm.hip"
    procs = []
    for name, (x, ab) in VARIANTS.items():
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-shared",
               "-munsafe-fp-atomics", f"-DMMS_GEMM_ABLATE={ab}", f"-DMMS_GEMM_XCDSPLIT={x}",
               "-I", str(ROOT / "include"), str(src), "-o", str(OUT / f"gemm_{name}.so")]
        procs.append(subprocess.Popen(cmd))
    for p in procs:
        if p.wait() != 0:
            raise SystemExit("variant build failed")
    print("built", sorted(os.listdir(OUT)))


def run():
    import torch
    sys.path.insert(0, str(ROOT))
    from multimodalstudio_amd import functions as fx, hip_ops
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
    s = torch.cuda.current_stream().cuda_stream

    def timeit(fn, reps=20):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3

    for prec, N, K, M in SHAPES:
        A = fx._alloc(M, N, dev).normal_()
        B = fx._alloc(M, K, dev).normal_()
        C = torch.zeros(N, K, device=dev)
        db = torch.zeros(N, device=dev)
        tiles = ((N + 127) // 128) * ((K + 127) // 128)
        dflt = hip_ops._splits_for(M, tiles, prec)
        nbytes = M * (A.stride(0) + B.stride(0)) * 4
        t_rd = timeit(lambda: (A.sum(), B.sum()))
        print(f"prec {prec} N {N} K {K} M {M}: {nbytes / 1e6:.0f} MB operands, torch read {t_rd:.1f} us "
              f"({nbytes / t_rd / 1e3:.0f} GB/s); default splits {dflt}", flush=True)
        for splits in sorted({dflt, max(1, dflt // 2), dflt * 2, max(1, dflt // 4)}):
            line = f"   splits {splits:4d}:"
            for name, f in libs.items():
                def call():
                    rc = f(prec, 1, 1, N, K, M, A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), C.data_ptr(), K,
                           None, None, 0, None, 0, 0, 0, 1.0, 20.0, 1, splits, -1, db.data_ptr(), s)
                    assert rc == 0
                t = timeit(call)
                line += f" {name}={t:.1f}us"
                if name == "x1_full":
                    line += f"({nbytes / t / 1e3:.0f}GB/s)"
            print(line, flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
