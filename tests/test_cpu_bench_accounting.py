"""bench.py's algorithmic-work accounting (the roofline denominators) on the launch arguments the C-ABI
receives -- no GPU: the argument tuples are built as multimodalstudio_amd/functions.py builds them."""
import ctypes
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def _chain_args(prec, bwd, Ns, K0, M, rows_full, stored):
    """mms_mlp_chain's positional arguments (include/mms_hip.h), pointers as truthy placeholders."""
    n = len(Ns)
    outs = (ctypes.c_void_p * n)(*[(1 if s else None) for s in stored])
    ns = (ctypes.c_int * n)(*Ns)
    a = [prec, bwd, n, 1, K0, K0, M, rows_full] + [None] * 10 + [ctypes.cast(outs, ctypes.c_void_p).value, None,
                                                                 ctypes.cast(ns, ctypes.c_void_p).value]
    return a, (outs, ns)


@pytest.mark.parametrize("prec,label", [(2, "bf16x3"), (5, "fp16"), (6, "fp16-rowscaled")])
def test_chain_work_sdf(prec, label):
    M, rf = 5 * 1000, 1000
    if prec == 6:   # a backward mode: the SDF backward 257 -> 256 -> 256 -> 71
        a, keep = _chain_args(prec, 1, [256, 256, 71], 257, M, rf, [True, True, True])
        name, (flops, nbytes) = bench.chain_work(a)
        assert name == f"{label}:sdf_bwd"
        # first layer: 257 inputs on the centre rows, 1 on the taps; then 256x256 and 256x71 on every row
        assert flops == 2.0 * (rf * 257 + (M - rf)) * 256 + 2.0 * M * (256 * 256 + 256 * 71)
    else:
        a, keep = _chain_args(prec, 0, [256, 256, 257], 71, M, rf, [True, True, True])
        name, (flops, nbytes) = bench.chain_work(a)
        assert name == f"{label}:sdf_fwd"
        # the taps need only the sdf column of the last layer
        assert flops == 2.0 * M * (71 * 256 + 256 * 256) + 2.0 * (rf * 257 + (M - rf)) * 256
    assert nbytes > 0


def test_every_chain_mode_has_a_peak():
    for p, name in bench.PREC_NAMES.items():
        assert name in bench.MFMA_PEAK_TF, (p, name)
