"""Twice-differentiable matrix products on the HIP GEMM engine, for the analytic-gradient MLP fields.

The ``mlp`` / ``mlp_raw`` methods take the SDF gradient by autograd with create_graph=True and put it into the
eikonal loss (SurfaceModel.gradient, /root/reference/src/model_components/surface_model.py:192-198), so the
training step differentiates the MLP's backward pass a second time.  ``MatMul`` is a torch.autograd.Function whose
forward is one mms_gemm launch and whose backward is again expressed with ``MatMul`` -- autograd records the
backward's products when create_graph is set, and the double backward runs on the same HIP kernels.  The
element-wise parts of those MLPs (weight norm, Softplus / ReLU, the skip concatenation) are the torch operators the
reference uses, which are twice differentiable by construction.
"""
from __future__ import annotations

import torch

from . import functions as fx


def _operand(t: torch.Tensor):
    """(stored-transposed flag, leading dimension, tensor) for a 2-D operand the GEMM reads in place: row-major rows
    (trans 0) or a transposed view of row-major rows (trans 1); anything else is copied."""
    if t.stride(1) == 1 and t.stride(0) >= t.shape[1]:
        return 0, t.stride(0), t
    if t.stride(0) == 1 and t.stride(1) >= t.shape[0]:
        return 1, t.stride(1), t
    t = t.contiguous()
    return 0, t.stride(0), t


def hip_mm(a: torch.Tensor, b: torch.Tensor, prec: int = 0) -> torch.Tensor:
    """a [M, K] @ b [K, N] on mms_gemm (fp32 MFMA in the parity preset)."""
    M, K = a.shape
    N = b.shape[1]
    ta, lda, a = _operand(a)
    # mms_gemm: trans_b = 0 reads B as [N, K] rows (b^T row-major = b stored column-major), 1 as [K, N] rows
    tbt, ldb, b = _operand(b)
    tb = 1 - tbt
    out = fx._alloc(M, N, a.device)
    gemm_mode = (ta, tb)
    _gemm_any(gemm_mode, M, N, K, a, lda, b, ldb, out, prec)
    return out


def _gemm_any(mode, M, N, K, a, lda, b, ldb, out, prec):
    from . import _lib
    _lib.call("mms_gemm", int(prec), int(mode[0]), int(mode[1]), int(M), int(N), int(K), a.data_ptr(), int(lda),
              b.data_ptr(), int(ldb), out.data_ptr(), int(out.stride(0)), None, None, 0, None, 0, 0, 0, 1.0, 20.0, 0,
              1, -1, None, fx._s())


class MatMul(torch.autograd.Function):
    """a @ b with a backward that is itself differentiable (double backward through the HIP GEMM)."""

    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a, b)
        return hip_mm(a, b, fx.PRECISION["mlp"])

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        ga = MatMul.apply(g, b.t()) if ctx.needs_input_grad[0] else None
        gb = MatMul.apply(a.t(), g) if ctx.needs_input_grad[1] else None
        return ga, gb


def linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
    """nn.Linear: x @ W^T + b."""
    return MatMul.apply(x, weight.t()) + bias


__all__ = ["MatMul", "linear", "hip_mm"]
