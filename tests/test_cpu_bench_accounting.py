"""bench.py's algorithmic-work accounting (the roofline denominators) on the launch arguments the C-ABI
receives -- no GPU: the argument tuples are built as multimodalstudio_amd/functions.py builds them."""
import ctypes
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def _chain_args(prec, bwd, Ns, K0, M, rows_full, stored, fp16=None, f16=None):
    """mms_mlp_chain's positional arguments (include/mms_hip.h), pointers as truthy placeholders; ``fp16``: per layer,
    whether its out is a prec-6 fp16 dZ store (rinv[l] set); ``f16``: per layer, fp16 activation rows (forward out /
    backward aux)."""
    n = len(Ns)
    outs = (ctypes.c_void_p * n)(*[(1 if s else None) for s in stored])
    ns = (ctypes.c_int * n)(*Ns)
    rinv = None if fp16 is None else (ctypes.c_void_p * n)(*[(1 if f else None) for f in fp16])
    a = [prec, bwd, n, 1, K0, K0, M, rows_full] + [None] * 10 + [ctypes.cast(outs, ctypes.c_void_p).value, None,
                                                                 ctypes.cast(ns, ctypes.c_void_p).value]
    fl = None if f16 is None else (ctypes.c_int * n)(*[int(f) for f in f16])
    a += [None] * 6 + [None if rinv is None else ctypes.cast(rinv, ctypes.c_void_p).value, None if fp16 is None else 1,
                       None if fl is None else ctypes.cast(fl, ctypes.c_void_p).value, None]
    assert len(a) == 31       # ... tap_part, ld_tap, rinv, emax, f16, stream
    return a, (outs, ns, rinv, fl)


@pytest.mark.parametrize("prec,label", [(2, "bf16x3"), (5, "fp16"), (6, "fp16-rowscaled")])
def test_chain_work_sdf(prec, label):
    M, rf = 5 * 1000, 1000
    if prec == 6:   # a backward mode: the SDF backward 257 -> 256 -> 256 -> 71
        a, keep = _chain_args(prec, 1, [256, 256, 71], 257, M, rf, [True, True, True])
        name, (flops, nbytes, eq) = bench.chain_work(a)
        assert name == f"{label}:sdf_bwd"
        # first layer: 257 inputs on the centre rows, 1 on the taps; then 256x256 and 256x71 on every row
        f0 = 2.0 * (rf * 257 + (M - rf)) * 256
        assert flops == f0 + 2.0 * M * (256 * 256 + 256 * 71)
        # its mode ceiling: the first layer split-bf16x3 (three MFMAs per product), the rest one fp16 MFMA
        assert eq == flops + 2.0 * f0
    else:
        a, keep = _chain_args(prec, 0, [256, 256, 257], 71, M, rf, [True, True, True])
        name, (flops, nbytes) = bench.chain_work(a)
        assert name == f"{label}:sdf_fwd"
        # the taps need only the sdf column of the last layer
        assert flops == 2.0 * M * (71 * 256 + 256 * 256) + 2.0 * (rf * 257 + (M - rf)) * 256
    assert nbytes > 0


def test_every_chain_mode_has_a_peak():
    for p, name in bench.PREC_NAMES.items():
        assert name in bench.MFMA_PEAK_TF or p == 6, (p, name)    # prec 6 is priced per launch (chain_work)


def test_rowscaled_mode_peak_is_priced_per_layer():
    """a prec-6 backward chain's mode ceiling weights its split-bf16x3 first layer at a third of the peak."""
    a, keep = _chain_args(6, 1, [256, 256, 256], 256, 4096, 4096, [True, True, True])
    name, work = bench.chain_work(a)
    recs = bench.kernel_records({"mms_mlp_chain:" + name: (1, 0.1, work)}, 1, "fast_h16b")
    r = recs[0]
    assert abs(r["mode_peak"] - bench.BF16_MFMA_PEAK_TF * 3 / 5) < 0.1      # 3 equal layers: 1/(3/3 + 1/3 + 1/3)
    assert r["frac_of_mode_peak"] > r["frac"]


def test_fp16_dz_stores_and_wide16_bytes():
    """Preset fast_h16c: a prec-6 backward chain's fp16 hidden-layer dZ stores count 2 B per element + the row's 4-B
    inverse scale; mms_gemm_tn_wide16 counts its fp16 A rows the same way and fp32 X."""
    M = 4096
    a32, k32 = _chain_args(6, 1, [256, 256, 71], 257, M, M, [True, True, True])
    a16, k16 = _chain_args(6, 1, [256, 256, 71], 257, M, M, [True, True, True], fp16=[True, True, False])
    _, (f32, b32, _) = bench.chain_work(a32)
    _, (f16, b16, _) = bench.chain_work(a16)
    assert f16 == f32
    assert b32 - b16 == 2 * (M * 256 * 2.0 - M * 4.0)
    n = 3
    I64 = ctypes.c_int64 * n
    ainv = (ctypes.c_void_p * n)(1, 1, None)          # two fp16-dZ items and an fp32 one (the output layer)
    b16 = (ctypes.c_int * n)(0, 1, 1)                 # the input panel fp32, hidden activations fp16
    w = [n, I64(256, 256, 257), I64(71, 256, 256), I64(M, M, M), None, None,
         ctypes.cast(ainv, ctypes.c_void_p).value, None, None, None, ctypes.cast(b16, ctypes.c_void_p).value] + \
        [None] * 5
    name, (flops, nbytes) = bench.gemm_wide16_work(w)
    assert name == "fp16:TN_grouped"
    assert flops == 2.0 * M * (256 * 71 + 256 * 256 + 257 * 256)
    assert nbytes == (2.0 * M * 256 + 4.0 * M + 4.0 * M * 71 + 8.0 * 256 * 71) + \
        (2.0 * M * 256 + 4.0 * M + 2.0 * M * 256 + 8.0 * 256 * 256) + (4.0 * M * 257 + 2.0 * M * 256 + 8.0 * 257 * 256)
    rec = bench.kernel_records({"mms_gemm_tn_wide16:" + name: (1, 0.1, (flops, nbytes))}, 1, "fast_h16c")[0]
    assert rec["peak"] == bench.BF16_MFMA_PEAK_TF


def test_fp16_activation_rows_bytes():
    """Preset fast_h16d: the forward's fp16 hidden activation rows count 2 B per element, and so do the backward's
    activation (aux) reads of them."""
    M = 4096
    f32, _ = _chain_args(2, 0, [256, 256, 257], 71, M, M, [True, True, True])
    f16, _ = _chain_args(2, 0, [256, 256, 257], 71, M, M, [True, True, True], f16=[True, True, False])
    assert bench.chain_work(f32)[1][1] - bench.chain_work(f16)[1][1] == 2 * M * 256 * 2.0
    b32, _ = _chain_args(6, 1, [256, 256, 71], 257, M, M, [True, True, True], fp16=[True, True, False])
    b16, _ = _chain_args(6, 1, [256, 256, 71], 257, M, M, [True, True, True], fp16=[True, True, False],
                         f16=[True, True, False])
    assert bench.chain_work(b32)[1][1] - bench.chain_work(b16)[1][1] == 2 * M * 256 * 2.0
