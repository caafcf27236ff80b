"""Build the C-ABI HIP library ``libmms_hip.so`` for gfx950 with hipcc (no torch in the ABI).

Each ``csrc/*.hip`` translation unit is compiled to an object in ``build/`` (in parallel) and
linked into ``multimodalstudio_amd/libmms_hip.so``.  hipcc cross-compiles without a GPU, so this
runs in the CPU container too; the built ``.so`` travels to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import concurrent.futures
import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
INCLUDE = PKG.parent / "include"
BUILD = PKG.parent / "build" / "mms_hip"
LIB = PKG / "libmms_hip.so"
ARCH = os.environ.get("MMS_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

CFLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-fPIC",
    "-std=c++17",
    "-fvisibility=hidden",
    "-Wall",
    "-Wno-unused-function",
    "-munsafe-fp-atomics",  # hardware global_atomic_add_f32 (no CAS loop)
    f"-I{INCLUDE}",         # common.h includes the C-ABI header: definitions are checked against it
]


def _compile(src: Path) -> Path:
    obj = BUILD / (src.stem + ".o")
    deps = [src] + sorted(CSRC.glob("*.h")) + sorted(INCLUDE.glob("*.h"))
    if obj.exists() and all(obj.stat().st_mtime >= d.stat().st_mtime for d in deps):
        return obj
    cmd = [HIPCC, *CFLAGS, "-c", str(src), "-o", str(obj)]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{res.stdout}\n{res.stderr}")
    return obj


def build(verbose: bool = False) -> Path:
    BUILD.mkdir(parents=True, exist_ok=True)
    srcs = sorted(CSRC.glob("*.hip"))
    if not srcs:
        raise RuntimeError("no HIP sources found")
    jobs = min(len(srcs), max(1, min(16, os.cpu_count() or 1)))
    with concurrent.futures.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(_compile, srcs))
    newest = max(o.stat().st_mtime for o in objs)
    if not LIB.exists() or LIB.stat().st_mtime < newest:
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(LIB), *map(str, objs)]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed:\n{res.stdout}\n{res.stderr}")
    if verbose:
        print(f"built {LIB}")
    return LIB


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
