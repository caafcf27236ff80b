"""torch.autograd bridges onto the C-ABI HIP kernels (libmms_hip.so).

Tensors are PyTorch-owned device memory; kernels receive raw pointers and the current HIP stream.
Every function here requires CUDA(HIP) tensors and raises otherwise: there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

from . import _lib

ACT_IDS = {None: 0, "None": 0, "Identity": 0, "ReLU": 1, "Softplus": 2, "Sigmoid": 3}
NT, NN, TN = 0, 1, 2


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _check_dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("MMS HIP ops require device (cuda/hip) tensors; no CPU fallback exists")


# ----------------------------------------------------------------------------------------------
# hash grid
# ----------------------------------------------------------------------------------------------
def _f32_array(vals):
    arr = (ctypes.c_float * len(vals))(*[float(v) for v in vals])
    return arr


INTERP = {None: 0, "Linear": 0, "Smoothstep": 1}   # HashEncodingConfig.interpolation (encodings.py:64-67)


def hashgrid_forward(pos: torch.Tensor, table: torch.Tensor, scales, log2T: int, radius: float,
                     active_levels: int, out: Optional[torch.Tensor] = None, interp: int = 0) -> torch.Tensor:
    """Raw forward launch; pos [M, >=3] (row stride pos.stride(0)), out [M, >=2L]; interp 0 Linear, 1 Smoothstep."""
    _check_dev(pos, table)
    L = len(scales)
    M = pos.shape[0]
    if out is None:
        out = torch.empty(M, 2 * L, device=pos.device, dtype=torch.float32)
    assert pos.stride(1) == 1 and out.stride(1) == 1 and table.is_contiguous()
    sc = _f32_array(scales)
    _lib.call("mms_hashgrid_fwd", pos.data_ptr(), M, pos.stride(0), table.data_ptr(), L, log2T, table.shape[1],
              int(interp), ctypes.cast(sc, ctypes.c_void_p), float(radius), int(active_levels), out.data_ptr(), out.stride(0),
              _stream())
    return out


def hashgrid_backward(pos, table, scales, log2T, radius, active_levels, dout, dtable=None, dpos=None, interp: int = 0):
    _check_dev(pos, table, dout)
    L = len(scales)
    sc = _f32_array(scales)
    assert dout.stride(1) == 1
    _lib.call("mms_hashgrid_bwd", pos.data_ptr(), pos.shape[0], pos.stride(0), table.data_ptr(), L, log2T,
              table.shape[1], int(interp), ctypes.cast(sc, ctypes.c_void_p), float(radius), int(active_levels),
              dout.data_ptr(), dout.stride(0), _ptr(dtable), _ptr(dpos), 0 if dpos is None else dpos.stride(0),
              _stream())


class HashGridFunction(torch.autograd.Function):
    """FeatureGrid(HashEncoding) forward/backward on the HIP kernels."""

    @staticmethod
    def forward(ctx, pos, table, scales, log2T, radius, active_levels, interp: int = 0):
        pos_c = pos.contiguous()
        out = hashgrid_forward(pos_c, table, scales, log2T, radius, active_levels, interp=interp)
        ctx.save_for_backward(pos_c, table)
        ctx.cfg = (scales, log2T, radius, active_levels, interp)
        return out

    @staticmethod
    def backward(ctx, dout):
        pos, table = ctx.saved_tensors
        scales, log2T, radius, active_levels, interp = ctx.cfg
        dtable = torch.zeros_like(table) if ctx.needs_input_grad[1] else None
        dpos = torch.zeros_like(pos) if ctx.needs_input_grad[0] else None
        hashgrid_backward(pos, table, scales, log2T, radius, active_levels, dout.contiguous(), dtable, dpos,
                          interp=interp)
        return dpos, dtable, None, None, None, None, None


# ----------------------------------------------------------------------------------------------
# GEMM
# ----------------------------------------------------------------------------------------------
_MODE_TRANS = {NT: (0, 0), NN: (0, 1), TN: (1, 1)}
PREC_IDS = {"fp32": 0, "bf16": 1, "bf16x3": 2}


def gemm(mode: int, M: int, N: int, K: int, A: torch.Tensor, lda: int, B: torch.Tensor, ldb: int,
         C: torch.Tensor, ldc: int, bias=None, Z=None, ldz=0, aux=None, ldaux=0, act=0, dact=0,
         beta=1.0, thr=20.0, accumulate=False, splits=1, prec: int = 0, ones_col: int = -1, colsum=None):
    """NT: C = A B^T (A [M,K], B [N,K]); NN: C = A B (B [K,N]); TN: C = A^T B (A [K,M], B [K,N]).

    ``colsum`` (TN only): colsum[m] += sum_k A[k, m] fused into the same pass (bias gradients)."""
    ta, tb = _MODE_TRANS[mode]
    _lib.call("mms_gemm", int(prec), ta, tb, int(M), int(N), int(K), A.data_ptr(), int(lda), B.data_ptr(), int(ldb),
              C.data_ptr(), int(ldc), _ptr(bias), _ptr(Z), int(ldz), _ptr(aux), int(ldaux), int(act), int(dact),
              float(beta), float(thr), int(bool(accumulate)), int(splits), int(ones_col), _ptr(colsum), _stream())


def weight_norm_fwd(g, v, W, norms):
    N, K = v.shape
    _lib.call("mms_weight_norm_fwd", g.data_ptr(), v.data_ptr(), N, K, W.data_ptr(), W.stride(0), norms.data_ptr(),
              _stream())


def weight_norm_bwd(g, v, norms, dW, dg, dv):
    N, K = v.shape
    _lib.call("mms_weight_norm_bwd", g.data_ptr(), v.data_ptr(), norms.data_ptr(), N, K, dW.data_ptr(), dW.stride(0),
              dg.data_ptr(), dv.data_ptr(), _stream())


def colsum_(A, out):
    M, N = A.shape
    _lib.call("mms_colsum", A.data_ptr(), M, N, A.stride(0), out.data_ptr(), _stream())


def act_bwd(dY, Z, act, beta, thr, dZ):
    M, N = dY.shape
    _lib.call("mms_act_bwd", dY.data_ptr(), dY.stride(0), Z.data_ptr(), Z.stride(0), M, N, int(act), float(beta),
              float(thr), dZ.data_ptr(), dZ.stride(0), _stream())


# split-K target: blocks per weight-gradient GEMM (measured, scripts/tn_sweep.py): one 128x128-tile block per CU for
# bf16 operands (more splits only add float atomics), two for split-bf16x3 (3 MFMAs per product), four for fp32
_SPLIT_BLOCKS = {0: 1024, 1: 256, 2: 512}


def _splits_for(M_rows: int, tiles: int, prec: int = 0) -> int:
    """K slices of a split-K weight gradient: a multiple of 8 (mms_gemm spreads each tile's slices over the 8 XCDs and
    pads the count to a multiple of 8: a padded count loads some XCDs with one slice more) within the block target."""
    target = max(1, _SPLIT_BLOCKS.get(int(prec), 1024) // max(1, tiles))
    if target >= 8:
        target = target // 8 * 8
    return int(max(1, min(target, M_rows // 512)))


# grouped weight-gradient launches (mms_gemm_tn_grouped): blocks per launch for all the MLP's layers together
_GROUP_BLOCKS = {0: 1024, 1: 256, 2: 512}


# weight-gradient engine of the bf16 modes: "wide" (mms_gemm_tn_wide: 256 x 256 tiles, operand rows read once per
# slice; SDF MLP 0.52 -> 0.36 ms alone, scripts/tn_wide_bench.py) or "tiled" (mms_gemm_tn_grouped: 128 x 128 tiles);
# MMS_TN_ENGINE overrides (A/B measurement)
TN_ENGINE = os.environ.get("MMS_TN_ENGINE", "wide")
_WIDE_BLOCKS = 256
TN_STAGE_ROWS = int(os.environ.get("MMS_TN_STAGE", "16"))
TN_WORKSPACE = os.environ.get("MMS_TN_WS", "0") == "1"


def _aligned_item(it) -> bool:
    A, B = it[3], it[4]
    return all(t.data_ptr() % 16 == 0 and t.stride(0) % 4 == 0 and t.stride(1) == 1 for t in (A, B))


def gemm_tn_grouped(items, prec: int, target_blocks: Optional[int] = None, engine: Optional[str] = None,
                    stage_rows: Optional[int] = None):
    """items = [(N_out, K_in, rows, dZ [rows, >=N_out], X [rows, >=K_in], dW [N_out, K_in], db [N_out] or None)]:
    dW += dZ^T X and db += colsum(dZ) for every item in one launch (<= 5 items)."""
    n = len(items)
    I64 = ctypes.c_int64 * n
    VP = ctypes.c_void_p * n
    engine = engine or TN_ENGINE
    # the wide engine's 256-row tiles pay for MLPs with 256-wide layers; the 64-wide modality heads stay on 128 tiles
    wide = engine == "wide" and int(prec) in (1, 2) and all(_aligned_item(it) for it in items) and \
        max(it[0] for it in items) >= 128
    if wide:
        entry = "mms_gemm_tn_wide"
        target = int(os.environ.get("MMS_TN_BLOCKS", "0")) or target_blocks or _WIDE_BLOCKS
    else:
        entry = "mms_gemm_tn_grouped"
        target = int(os.environ.get("MMS_TN_BLOCKS", "0")) or target_blocks or _GROUP_BLOCKS.get(int(prec), 512)
    extra = ()
    if wide:
        # the slices' partial tiles go through a scratch buffer and a deterministic reduce launch (plain stores instead
        # of 256 KB of float atomics per block); MMS_TN_WS=0 keeps the atomics
        ws = torch.empty((target + 16) * 65536, device=items[0][3].device) if TN_WORKSPACE else None
        extra = (int(stage_rows or TN_STAGE_ROWS), None if ws is None else ws.data_ptr(),
                 0 if ws is None else ws.numel())
    _lib.call(entry, int(prec), n, I64(*[it[0] for it in items]), I64(*[it[1] for it in items]),
              I64(*[it[2] for it in items]), VP(*[it[3].data_ptr() for it in items]),
              I64(*[it[3].stride(0) for it in items]), VP(*[it[4].data_ptr() for it in items]),
              I64(*[it[4].stride(0) for it in items]), VP(*[it[5].data_ptr() for it in items]),
              I64(*[it[5].stride(0) for it in items]),
              VP(*[(it[6].data_ptr() if it[6] is not None else None) for it in items]), target, *extra, _stream())


def gemm_tn_wide16(items, target_blocks: Optional[int] = None):
    """items = [(N_out, K_in, rows, dZ, rinv or None, emax or None, X, dW, db or None)] in ONE launch
    (mms_gemm_tn_wide16): dW += dZ^T X and db += colsum(dZ).  dZ fp16 row-scaled with rinv / emax (mms_mlp_chain prec
    6 with rinv; emax a 1-element int32 view): one fp16 MFMA per product; dZ fp32 (rinv None): split bf16x3.  X fp32 or
    fp16 rows (its dtype).  <= 5 items."""
    n = len(items)
    I64 = ctypes.c_int64 * n
    VP = ctypes.c_void_p * n
    target = int(os.environ.get("MMS_TN_BLOCKS", "0")) or target_blocks or _WIDE_BLOCKS
    _lib.call("mms_gemm_tn_wide16", n, I64(*[it[0] for it in items]), I64(*[it[1] for it in items]),
              I64(*[it[2] for it in items]), VP(*[it[3].data_ptr() for it in items]),
              I64(*[it[3].stride(0) for it in items]), VP(*[_ptr(it[4]) for it in items]),
              VP(*[_ptr(it[5]) for it in items]), VP(*[it[6].data_ptr() for it in items]),
              I64(*[it[6].stride(0) for it in items]),
              (ctypes.c_int * n)(*[int(it[6].dtype == torch.float16) for it in items]),
              VP(*[it[7].data_ptr() for it in items]), I64(*[it[7].stride(0) for it in items]),
              VP(*[_ptr(it[8]) for it in items]), target, _stream())


def _ptr(t):
    return None if t is None else t.data_ptr()
