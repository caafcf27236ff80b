#!/usr/bin/env python
"""Product-library build variants for step A/B runs (diagnostics): one translation unit rebuilt under macros -- the
backward chain epilogue's Y-tile prefetch depth (csrc/mlp_chain.hip MMS_CHAIN_YAHEAD / MMS_CHAIN_YAHEAD4), the
hash-grid kernels' block order (csrc/hashgrid.hip MMS_HASH_XCD) -- linked with the other objects and selected at run
time with MMS_HIP_LIB.

    python scripts/lib_variants.py [name ...]   # CPU container: build multimodalstudio_amd/_variants/libmms_<name>.so
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
VARIANTS = {  # name: (translation unit, macro definitions)
    "y1_1": ("mlp_chain", {"MMS_CHAIN_YAHEAD": 1, "MMS_CHAIN_YAHEAD4": 1}),
    "y2_2": ("mlp_chain", {"MMS_CHAIN_YAHEAD": 2, "MMS_CHAIN_YAHEAD4": 2}),
    "y8_4": ("mlp_chain", {"MMS_CHAIN_YAHEAD": 8, "MMS_CHAIN_YAHEAD4": 4}),
    "hx0": ("hashgrid", {"MMS_HASH_XCD": 0}),
    "stamps": ("mlp_chain", {"MMS_CHAIN_STAMPS": 1}),   # scripts/chain_stamps.py
    "ahead0": ("mlp_chain", {"MMS_CHAIN_AHEAD": 0}),
    "ss2k": ("loss_optim", {"MMS_SUMSQ_GRID": 2048, "MMS_SUMSQ_UNROLL": 4}),   # the round-3c launch shape
    "wpipe0": ("gemm", {"MMS_WIDE_PIPE": 0}),   # the wide weight-gradient kernel's one-register-set loop (round 3)
    "d3": ("mlp_chain", {"MMS_CHAIN_DEPTH": 3}),  # the chains' weight / input ring three k-steps deep (where LDS allows)
    "d4": ("mlp_chain", {"MMS_CHAIN_DEPTH": 4}),
    "nw2": ("mlp_chain", {"MMS_CHAIN_NW": 2}),    # 64-row chain blocks (two per CU where the LDS holds them)
}
# the wide weight-gradient kernel's phase ablations in the step (MMS_WIDE_ABLATE bits: 2 no MFMAs, 4 no global loads,
# 8 no LDS image stores; results wrong, timing only -- round 6's fp16 mixed launch)
VARIANTS.update({f"wabl{n}": ("gemm", {"MMS_WIDE_ABLATE": n}) for n in (2, 4, 8, 12)})
VARIANTS.update({f"wd{n}": ("gemm", {"MMS_WIDE_DEPTH16": n}) for n in (2, 4)})   # the fp16 items' register sets
VARIANTS["wk16"] = ("gemm", {"MMS_WIDE_WK16": 16, "MMS_WIDE_DEPTH16": 3})   # 16-row stages for the fp16 items
VARIANTS.update({f"x3c{int(10 * c)}": ("gemm", {"MMS_WIDE_X3COST": c}) for c in (1.0, 1.5, 2.0)})   # slice cost weights
# the backward epilogue's ablations on the stamp build (MMS_CHAIN_EPI_ABL bits: 1 no Y loads, 2 no dZ stores, 4 no
# scratch round trips)
VARIANTS.update({f"stampsE{n}": ("mlp_chain", {"MMS_CHAIN_STAMPS": 1, "MMS_CHAIN_EPI_ABL": n}) for n in (1, 2, 4, 3, 7)})
# (round 5's two-waves-per-SIMD chain, csrc/chain16.hip, and its ablation variants were removed from the tree after
# measuring -2 % in the step; DESIGN §3 keeps the record, git history the source)


def main():
    names = sys.argv[1:] or list(VARIANTS)
    b.build()
    OUT.mkdir(parents=True, exist_ok=True)
    procs = {}
    for name in names:
        unit, macros = VARIANTS[name]
        obj = OUT / f"{unit}_{name}.o"
        cmd = [b.HIPCC, *b.CFLAGS, *[f"-D{k}={v}" for k, v in macros.items()], "-c", str(b.CSRC / f"{unit}.hip"),
               "-o", str(obj)]
        procs[name] = (subprocess.Popen(cmd, stderr=subprocess.DEVNULL), obj, unit)
    for name, (p, obj, unit) in procs.items():
        if p.wait() != 0:
            raise SystemExit(f"variant {name} failed")
        others = [o for o in sorted(b.BUILD.glob("*.o")) if o.stem != unit]
        lib = OUT / f"libmms_{name}.so"
        subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", str(lib), str(obj),
                        *map(str, others)], check=True)
        obj.unlink()
        print("built", lib)


if __name__ == "__main__":
    main()
