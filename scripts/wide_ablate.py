#!/usr/bin/env python
"""Wide weight-gradient kernel phase ablation (diagnostics only; cdna_hip_programming.md §7 'Ablate').

    python scripts/wide_ablate.py build      # CPU container: compile variants into multimodalstudio_amd/_variants/
    python scripts/wide_ablate.py run        # GPU box: time every variant on the bench step's SDF / radiance item sets

Variants compile csrc/gemm.hip alone with -DMMS_WIDE_ABLATE=<bits>: 1 = no output atomics, 2 = no MFMA, 4 = no global
loads, 8 = no LDS image stores.  Timing-only builds: their outputs are wrong by design.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
OUT = ROOT / "multimodalstudio_amd" / "_variants"
VARIANTS = {"full": 0, "no_atomic": 1, "no_mfma": 2, "no_load": 4, "no_lds_store": 8,
            "mfma_only": 1 | 4 | 8, "no_load_no_atomic": 1 | 4, "pipe": 0, "pipe_no_atomic": 1}
PIPE = {"pipe", "pipe_no_atomic"}   # built with MMS_WIDE_PIPE=1
M = 55360


def build():
    OUT.mkdir(parents=True, exist_ok=True)
    src = ROOT / "multimodalstudio_amd" / "csrc" / "gemm.hip"
    procs = []
    for name, bits in VARIANTS.items():
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-shared",
               "-munsafe-fp-atomics", f"-DMMS_WIDE_ABLATE={bits}", f"-DMMS_WIDE_PIPE={int(name in PIPE)}", "-I", str(ROOT / "include"), str(src), "-o",
               str(OUT / f"wide_{name}.so")]
        procs.append(subprocess.Popen(cmd))
    for p in procs:
        if p.wait() != 0:
            raise SystemExit("ablation build failed")
    print("built", sorted(os.listdir(OUT)))


def run():
    import torch
    sys.path.insert(0, str(ROOT))
    from multimodalstudio_amd import _lib
    from multimodalstudio_amd.functions import _alloc
    dev = torch.device("cuda", 0)
    restype, argtypes = _lib.SIGNATURES["mms_gemm_tn_wide"]
    sets = {"sdf": [(256, 71, 5 * M), (256, 256, 5 * M), (257, 256, M)],
            "radiance": [(256, 317, M), (256, 256, M), (256, 256, M)]}
    for sname, spec in sets.items():
        items = []
        nbytes = 0
        for N, K, R in spec:
            dZ = _alloc(R, N, dev).normal_()
            X = _alloc(R, K, dev).normal_()
            items.append((N, K, R, dZ, X, torch.zeros(N, K, device=dev), torch.zeros(N, device=dev)))
            nbytes += 4 * R * (N + K)
        n = len(items)
        I64, VP = ctypes.c_int64 * n, ctypes.c_void_p * n
        args = (2, n, I64(*[it[0] for it in items]), I64(*[it[1] for it in items]), I64(*[it[2] for it in items]),
                VP(*[it[3].data_ptr() for it in items]), I64(*[it[3].stride(0) for it in items]),
                VP(*[it[4].data_ptr() for it in items]), I64(*[it[4].stride(0) for it in items]),
                VP(*[it[5].data_ptr() for it in items]), I64(*[it[5].stride(0) for it in items]),
                VP(*[it[6].data_ptr() for it in items]), 256, 16, None, 0)
        line = f"{sname:9s} ({nbytes / 1e6:.0f} MB)"
        ref = None
        for name in VARIANTS:
            lib = ctypes.CDLL(str(OUT / f"wide_{name}.so"), mode=os.RTLD_LOCAL)
            f = lib.mms_gemm_tn_wide
            f.restype, f.argtypes = restype, argtypes
            s = torch.cuda.current_stream().cuda_stream
            for _ in range(3):
                assert f(*args, s) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                f(*args, s)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 100
            line += f" {name}={us:.0f}us"
            if name in ("full", "pipe"):
                # one clean launch: the pipelined kernel's dW / db against the baseline kernel's
                for it in items:
                    it[5].zero_()
                    it[6].zero_()
                assert f(*args, s) == 0
                torch.cuda.synchronize()
                got = [torch.cat([it[5].flatten(), it[6]]) for it in items]
                if ref is None:
                    ref = got
                else:
                    err = max(float((a - b).abs().max() / b.abs().max()) for a, b in zip(got, ref))
                    line += f" (pipe vs full rel {err:.1e})"
        print(line, flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
