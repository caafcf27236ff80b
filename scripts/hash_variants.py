#!/usr/bin/env python
"""Hash-grid backward variants on the bench step's SDF batch (diagnostics): merge-table size, samples per block and
the level from which pending corner gradients bypass the LDS merge (csrc/hashgrid.hip MMS_HASH_* macros).

    python scripts/hash_variants.py build   # CPU container: compile the variants into scratch/lib/
    python scripts/hash_variants.py run     # GPU box: time each variant (table gradient + position gradient)
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
OUT = ROOT / "multimodalstudio_amd" / "_variants"   # travels to the GPU box (scratch/ does not)
VARIANTS = {  # name: (log2 lines, samples per block, first direct level) of the SDF batch's [centre | 4 taps] walk
    "merge_all": (9, 4, 16), "fine14": (9, 4, 14), "fine13": (9, 4, 13), "fine12": (9, 4, 12), "fine11": (9, 4, 11),
    "ch2_fine12": (9, 2, 12), "ch8_fine12": (9, 8, 12), "l8_fine12": (8, 4, 12),
}
PLAIN = {  # name: (points per block, first direct level) of the plain walk (the radiance grid)
    "p_ch8_f16": (8, 16), "p_ch8_f12": (8, 12), "p_ch8_f8": (8, 8), "p_ch8_f4": (8, 4), "p_ch8_f0": (8, 0),
    "p_ch16_f8": (16, 8), "p_ch16_f4": (16, 4), "p_ch32_f4": (32, 4),
    "p_ch16_f12": (16, 12), "p_ch32_f12": (32, 12), "p_ch32_f8": (32, 8), "p_ch64_f8": (64, 8), "p_ch64_f12": (64, 12),
}


def build():
    OUT.mkdir(parents=True, exist_ok=True)
    src = ROOT / "multimodalstudio_amd" / "csrc" / "hashgrid.hip"
    procs = []
    for name, (ll, ch, fine) in VARIANTS.items():
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-shared",
               "-munsafe-fp-atomics", f"-DMMS_HASH_LOG_LINES={ll}", f"-DMMS_HASH_CH5={ch}", f"-DMMS_HASH_FINE={fine}",
               "-I", str(ROOT / "include"), str(src), "-o", str(OUT / f"hash_{name}.so")]
        procs.append(subprocess.Popen(cmd))
    for name, (ch, fine) in PLAIN.items():
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-shared",
               "-munsafe-fp-atomics", f"-DMMS_HASH_CH1={ch}", f"-DMMS_HASH_FINE1={fine}",
               "-I", str(ROOT / "include"), str(src), "-o", str(OUT / f"hash_{name}.so")]
        procs.append(subprocess.Popen(cmd))
    for p in procs:
        if p.wait() != 0:
            raise SystemExit("variant build failed")
    print("built", sorted(os.listdir(OUT)))


def run():
    import torch
    sys.path.insert(0, str(ROOT))
    from multimodalstudio_amd import _lib, functions as F
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    R, S = 880, 64
    o = torch.nn.functional.normalize(torch.randn(R, 3, generator=g), dim=-1) * 3.0
    d = torch.nn.functional.normalize(-o + 0.3 * torch.randn(R, 3, generator=g), dim=-1)
    t = torch.sort(torch.rand(R, S, generator=g) * 2.0 + 2.0, dim=-1).values
    c = (o[:, None, :] + t[..., None] * d[:, None, :]).reshape(-1, 3).clamp(-1, 1)
    M = c.shape[0]
    delta = 2.0 / 1024 / 3 ** 0.5
    dirs = torch.tensor([[1., -1., -1.], [-1., -1., 1.], [-1., 1., -1.], [1., 1., 1.]])
    x = torch.cat([c] + [c + delta * k for k in dirs], 0).contiguous().to(dev)
    L, log2T = 16, 19
    cfg = F.GridCfg([float(int(16 * (1.3195079 ** l))) for l in range(L)], log2T, 1.0)
    table = ((torch.rand(L << log2T, 2, generator=g) * 2 - 1) * 1e-2).to(dev)
    dout = torch.randn(5 * M, 32, generator=g).to(dev)
    restype, argtypes = _lib.SIGNATURES["mms_hashgrid_bwd_grouped"]
    ref = None
    for name in list(VARIANTS) + list(PLAIN):
        plain = name in PLAIN
        G = 1 if plain else 5   # the plain walk runs the centre rows alone: the radiance grid's batch
        lib = ctypes.CDLL(str(OUT / f"hash_{name}.so"), mode=os.RTLD_LOCAL)
        fn = lib.mms_hashgrid_bwd_grouped
        fn.restype, fn.argtypes = restype, argtypes
        dtable = torch.zeros_like(table)
        dpos = torch.zeros_like(x)

        def call():
            rc = fn(x.data_ptr(), M, G, M, 3, table.data_ptr(), L, log2T, 2, 0, cfg.scales_ptr, 1.0, L,
                    dout.data_ptr(), dout.stride(0), dtable.data_ptr(), dpos.data_ptr(), 3,
                    torch.cuda.current_stream().cuda_stream)
            assert rc == 0
        call()
        torch.cuda.synchronize()
        got = (dtable.clone(), dpos.clone())
        if ref is None or name == next(iter(PLAIN)):
            ref = got
        err = max(((a - b).abs().max() / b.abs().max()).item() for a, b in zip(got, ref))
        for _ in range(2):
            call()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            call()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 100.0
        first = next(iter(PLAIN if plain else VARIANTS))
        print(f"{name:12s} {(PLAIN if plain else VARIANTS)[name]}  {us:8.1f} us  (vs {first} {err:.1e})", flush=True)


def split():
    """The product library's walk with both gradients vs the split pair: the walk without the position gradient +
    mms_hashgrid_dpos_grouped (the gather-shaped position gradient), for the SDF batch (G = 5) and the plain walk."""
    import torch
    sys.path.insert(0, str(ROOT))
    from multimodalstudio_amd import _lib, functions as F
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    R, S = 880, 64
    o = torch.nn.functional.normalize(torch.randn(R, 3, generator=g), dim=-1) * 3.0
    d = torch.nn.functional.normalize(-o + 0.3 * torch.randn(R, 3, generator=g), dim=-1)
    t = torch.sort(torch.rand(R, S, generator=g) * 2.0 + 2.0, dim=-1).values
    c = (o[:, None, :] + t[..., None] * d[:, None, :]).reshape(-1, 3).clamp(-1, 1)
    M = c.shape[0]
    delta = 2.0 / 1024 / 3 ** 0.5
    dirs = torch.tensor([[1., -1., -1.], [-1., -1., 1.], [-1., 1., -1.], [1., 1., 1.]])
    x = torch.cat([c] + [c + delta * k for k in dirs], 0).contiguous().to(dev)
    L, log2T = 16, 19
    cfg = F.GridCfg([float(int(16 * (1.3195079 ** l))) for l in range(L)], log2T, 1.0)
    table = ((torch.rand(L << log2T, 2, generator=g) * 2 - 1) * 1e-2).to(dev)
    dout = torch.randn(5 * M, 32, generator=g).to(dev)
    s = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    for G in (5, 1):
        dtable, dpos = torch.zeros_like(table), torch.zeros_like(x)

        def both():
            _lib.call("mms_hashgrid_bwd_grouped", x.data_ptr(), M, G, M, 3, table.data_ptr(), L, log2T, 2, 0,
                      cfg.scales_ptr, 1.0, L, dout.data_ptr(), 32, dtable.data_ptr(), dpos.data_ptr(), 3, s())

        def walk_only():
            _lib.call("mms_hashgrid_bwd_grouped", x.data_ptr(), M, G, M, 3, table.data_ptr(), L, log2T, 2, 0,
                      cfg.scales_ptr, 1.0, L, dout.data_ptr(), 32, dtable.data_ptr(), None, 3, s())

        def dpos_only():
            _lib.call("mms_hashgrid_dpos_grouped", x.data_ptr(), M, G, M, 3, table.data_ptr(), L, log2T, 2, 0,
                      cfg.scales_ptr, 1.0, L, dout.data_ptr(), 32, dpos.data_ptr(), 3, s())
        for name, fn in (("both", both), ("walk_only", walk_only), ("dpos_only", dpos_only),
                         ("split", lambda: (walk_only(), dpos_only()))):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            torch.cuda.synchronize()
            print(f"G={G} {name:10s} {e0.elapsed_time(e1) * 100.0:8.1f} us", flush=True)


if __name__ == "__main__":
    {"build": build, "run": run, "split": split}[sys.argv[1]]()
