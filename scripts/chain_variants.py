#!/usr/bin/env python
"""Chain-kernel build variants for step A/B runs (diagnostics): the backward epilogue's Y-tile prefetch depth
(csrc/mlp_chain.hip MMS_CHAIN_YAHEAD for 3-layer chains, MMS_CHAIN_YAHEAD4 for 4-layer chains).  Each variant is the
product library with mlp_chain.hip rebuilt under the macros, selected at run time with MMS_HIP_LIB.

    python scripts/chain_variants.py            # CPU container: build multimodalstudio_amd/_variants/libmms_y*.so
    MMS_HIP_LIB=multimodalstudio_amd/_variants/libmms_y1_1.so python bench.py ...   # GPU box
"""
from __future__ import annotations

import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from multimodalstudio_amd import build as b   # noqa: E402

OUT = ROOT / "multimodalstudio_amd" / "_variants"
VARIANTS = {"y1_1": (1, 1), "y2_2": (2, 2), "y4_4": (4, 4), "y8_4": (8, 4)}


def main():
    b.build()
    OUT.mkdir(parents=True, exist_ok=True)
    others = [o for o in sorted(b.BUILD.glob("*.o")) if o.stem != "mlp_chain"]
    procs = {}
    for name, (y3, y4) in VARIANTS.items():
        obj = OUT / f"mlp_chain_{name}.o"
        cmd = [b.HIPCC, *b.CFLAGS, f"-DMMS_CHAIN_YAHEAD={y3}", f"-DMMS_CHAIN_YAHEAD4={y4}", "-c",
               str(b.CSRC / "mlp_chain.hip"), "-o", str(obj)]
        procs[name] = (subprocess.Popen(cmd, stderr=subprocess.DEVNULL), obj)
    for name, (p, obj) in procs.items():
        if p.wait() != 0:
            raise SystemExit(f"variant {name} failed")
        lib = OUT / f"libmms_{name}.so"
        subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", str(lib), str(obj),
                        *map(str, others)], check=True)
        obj.unlink()
        print("built", lib)


if __name__ == "__main__":
    main()
