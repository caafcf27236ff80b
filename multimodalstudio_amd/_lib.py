"""ctypes binding of the C-ABI library ``libmms_hip.so``.

The argument types are derived from the declarations in ``include/mms_hip.h`` (the single source of
truth for the boundary), so the header and the binding cannot drift apart.  There is no fallback:
if the library or header is missing every op raises.
Streams: each call passes ``torch.cuda.current_stream().cuda_stream`` (a hipStream_t) so kernels
are ordered with PyTorch's own work; the library never synchronises or allocates.
"""
from __future__ import annotations

import ctypes
import os
import re
from pathlib import Path

_PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("MMS_HIP_LIB", _PKG / "libmms_hip.so"))
HEADER = _PKG.parent / "include" / "mms_hip.h"

_DECL = re.compile(r"^\s*(int|const char\*)\s+(mms_\w+)\s*\(([^;]*?)\)\s*;", re.S | re.M)


def _ctype(arg: str):
    a = arg.strip()
    if a == "void" or not a:
        return None
    if "*" in a:
        return ctypes.c_void_p
    t = a.rsplit(" ", 1)[0].strip()
    return {"int64_t": ctypes.c_int64, "int": ctypes.c_int, "float": ctypes.c_float, "double": ctypes.c_double,
            "uint64_t": ctypes.c_uint64, "uint32_t": ctypes.c_uint32}[t]


def parse_header(path: Path = HEADER):
    """Return {name: (restype, [argtypes])} for every mms_* declaration in the header."""
    text = path.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    out = {}
    for ret, name, args in _DECL.findall(text):
        argtypes = [t for t in (_ctype(x) for x in args.replace("\n", " ").split(",")) if t is not None]
        out[name] = (ctypes.c_char_p if ret.startswith("const char") else ctypes.c_int, argtypes)
    return out


SIGNATURES = parse_header() if HEADER.exists() else {}

_lib = None


class HipLibraryError(RuntimeError):
    pass


def lib():
    """Load (once) and return the ctypes library; raise loudly if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise HipLibraryError(
            f"{LIB_PATH} not found: build it with `python -m multimodalstudio_amd.build` "
            "(there is no CPU or PyTorch fallback for the MMS hot path)")
    if not SIGNATURES:
        raise HipLibraryError(f"C-ABI header {HEADER} not found")
    L = ctypes.CDLL(str(LIB_PATH), mode=ctypes.RTLD_GLOBAL)
    for name, (restype, argtypes) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.argtypes = argtypes
        fn.restype = restype
    _lib = L
    return L


class KernelTimer:
    """Live per-launch timing of selected entry points with HIP events on the launching stream.

    ``watch[name] = work_fn(args) -> algorithmic bytes or flops of that launch`` (or ``(label, work)`` to
    split one entry point into several records, e.g. the GEMM per precision).  Used by bench.py for
    the roofline fractions; disabled (zero overhead beyond a dict lookup) unless ``active``.
    """

    def __init__(self):
        self.active = False
        self.watch = {}
        self.records = []

    def start(self, watch):
        self.watch = dict(watch)
        self.records = []
        self.active = True

    def stop(self):
        self.active = False

    def summary(self):
        """{name: (launches, mean_ms, mean_work)} — call after a device synchronise.  ``mean_work`` is a
        float, or a tuple of floats when the work function returns several quantities (e.g. flops, bytes)."""
        out = {}
        for name, ev0, ev1, work in self.records:
            ms = ev0.elapsed_time(ev1)
            n, t, w = out.get(name, (0, 0.0, None))
            if isinstance(work, tuple):
                w = work if w is None else tuple(a + b for a, b in zip(w, work))
            else:
                w = work if w is None else w + work
            out[name] = (n + 1, t + ms, w)
        res = {}
        for k, (n, t, w) in out.items():
            res[k] = (n, t / n, tuple(x / n for x in w) if isinstance(w, tuple) else w / n)
        return res


TIMER = KernelTimer()
# debugging: synchronise after every entry point and name the first one whose kernel faulted (MMS_SYNC_CALLS=1; the
# previous calls' argument summaries are printed with it)
SYNC_CALLS = os.environ.get("MMS_SYNC_CALLS", "0") == "1"
_RECENT: list = []


def call(name: str, *args) -> None:
    """Invoke ``name`` and raise RuntimeError with mms_last_error() on a non-zero status."""
    L = lib()
    if name not in SIGNATURES:
        # an undeclared entry point would be called with ctypes' default (32-bit int) argument conversion
        raise HipLibraryError(f"{name} is not declared in {HEADER.name}: refusing an untyped call")
    timed = TIMER.active and name in TIMER.watch
    if timed:
        import torch
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
    rc = getattr(L, name)(*args)
    if timed:
        e1.record()
        w = TIMER.watch[name](args)
        key = name
        if isinstance(w, tuple) and isinstance(w[0], str):
            key, w = f"{name}:{w[0]}", w[1]
        TIMER.records.append((key, e0, e1, tuple(float(x) for x in w) if isinstance(w, tuple) else float(w)))
    if rc != 0:
        msg = L.mms_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed ({rc}): {msg}")
    if SYNC_CALLS:
        import torch
        _RECENT.append(f"{name}{tuple(a if isinstance(a, (int, float)) else type(a).__name__ for a in args)}")
        del _RECENT[:-4]
        try:
            torch.cuda.synchronize()
            import time
            time.sleep(0.02)        # a memory fault can be reported after the faulting kernel's completion
            torch.cuda.synchronize()
        except Exception as e:
            raise RuntimeError(f"kernel fault in or before {name} (last calls: {_RECENT})") from e


def exported_symbols():
    return list(SIGNATURES.keys())
