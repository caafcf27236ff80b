"""ctypes binding of the C-ABI library ``libmms_hip.so`` (declared in include/mms_hip.h).

The product path has no fallback: if the library is missing or fails to load, every op raises.
Streams: each call passes ``torch.cuda.current_stream().cuda_stream`` (a hipStream_t) so kernels
are ordered with PyTorch's own work; the library never synchronises or allocates.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

_PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("MMS_HIP_LIB", _PKG / "libmms_hip.so"))

_p = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int
_f32 = ctypes.c_float

# name -> argtypes (restype is always int status, except mms_last_error / mms_version)
SIGNATURES = {
    "mms_hashgrid_fwd": [_p, _i64, _i64, _p, _i32, _i32, _i32, _p, _f32, _i32, _p, _i64, _p],
    "mms_hashgrid_bwd": [_p, _i64, _i64, _p, _i32, _i32, _i32, _p, _f32, _i32, _p, _i64, _p, _p, _i64, _p],
    "mms_gemm_f32": [_i32, _i64, _i64, _i64, _p, _i64, _p, _i64, _p, _i64, _p, _p, _i64, _p, _i64,
                     _i32, _i32, _f32, _f32, _i32, _i32, _p],
}

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
    L = ctypes.CDLL(str(LIB_PATH), mode=ctypes.RTLD_GLOBAL)
    for name, argtypes in SIGNATURES.items():
        fn = getattr(L, name)
        fn.argtypes = argtypes
        fn.restype = ctypes.c_int
    L.mms_last_error.argtypes = []
    L.mms_last_error.restype = ctypes.c_char_p
    L.mms_version.argtypes = []
    L.mms_version.restype = ctypes.c_char_p
    _lib = L
    return L


def call(name: str, *args) -> None:
    """Invoke ``name`` and raise RuntimeError with mms_last_error() on a non-zero status."""
    L = lib()
    rc = getattr(L, name)(*args)
    if rc != 0:
        msg = L.mms_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed ({rc}): {msg}")


def exported_symbols():
    return list(SIGNATURES.keys()) + ["mms_last_error", "mms_version"]
