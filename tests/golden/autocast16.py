"""CUDA fp16 autocast restated on the CPU for the reference's model forward (THIS CONTAINER ONLY; test infrastructure).

Every BASELINE YAML trains with ``mixed_precision: True`` (/root/reference/confs/grid.yaml:17 and the others), which the
reference turns into Lightning Fabric's ``"16-mixed"`` precision (/root/reference/src/engine/trainer.py:51,57-62):
``fabric.setup(model)`` (/root/reference/src/pipelines/base_pipeline.py:208-217) runs the model's forward under
``torch.autocast("cuda", dtype=torch.float16)`` and ``fabric.backward`` scales the loss by a dynamic GradScaler
(unscaled before the gradient clip, base_pipeline.py:148-149,232-248).  The ray generator and the loss run outside the
autocast region (they are not the wrapped module's forward, base_pipeline.py:141-145).

CPU autocast follows a different op policy than CUDA autocast, and the CPU's fp16 GEMM is a slow scalar loop, so this
module restates the CUDA policy as a TorchFunctionMode over the reference's Python calls:

* lower-precision ops (``linear``, ``matmul`` / ``@``, ``mm``, ``bmm``, ``addmm``, ``baddbmm``, ``einsum``): operands
  rounded to fp16, product accumulated in fp32 (fp16 x fp16 products are exact in fp32, like the tensor cores' fp32
  accumulation), the result rounded to fp16 once -- an fp16 tensor, as CUDA's autocast returns.  Their backward takes
  the incoming gradient in fp16 (the gradient of an fp16 tensor is fp16), computes each operand gradient with fp32
  accumulation and rounds it to fp16 once, then casts it to the operand's own dtype (the backward of autocast's cast);
* the fp32-list ops of CUDA autocast (``exp``, ``log``, ``pow``, ``softplus``, ``sum``, ``cumprod``, norms, losses,
  ...): fp16 tensor arguments are cast to fp32 first (differentiably, as autocast's cast), so they return fp32;
* everything else runs in the dtypes it is given -- fp16 elementwise arithmetic on the CPU computes in fp32 and rounds
  to fp16 per op, like the CUDA kernels; mixed fp16 / fp32 arguments promote to fp32 (``cat``, ``stack`` and the
  binary ops promote natively on both devices).

``FP16_SEEN`` collects every (function, argument dtypes) pair that received an fp16 tensor, so a generator can show that
no op outside these lists consumed one where CUDA's policy would differ.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch.overrides import TorchFunctionMode

H = torch.float16


def _tensors(x):
    if isinstance(x, torch.Tensor):
        yield x
    elif isinstance(x, (list, tuple)):
        for y in x:
            yield from _tensors(y)
    elif isinstance(x, dict):
        for y in x.values():
            yield from _tensors(y)


def _map(x, fn):
    if isinstance(x, torch.Tensor):
        return fn(x)
    if isinstance(x, (list, tuple)):
        return type(x)(_map(y, fn) for y in x)
    if isinstance(x, dict):
        return {k: _map(v, fn) for k, v in x.items()}
    return x


class _Lower16(torch.autograd.Function):
    """op(*tensors) with fp16-rounded operands, fp32 accumulation, one fp16 rounding of the result; backward: fp16
    incoming gradient, fp32-accumulated operand gradients rounded to fp16 once, then cast to each operand's dtype."""

    @staticmethod
    def forward(ctx, op, n, *args):
        ts = args[:n]
        rest = args[n:]
        hs = [t.to(H) if (t is not None and t.is_floating_point()) else t for t in ts]
        ctx.op, ctx.rest = op, rest
        ctx.dtypes = [None if t is None else t.dtype for t in ts]
        ctx.save_for_backward(*[h for h in hs if h is not None])
        ctx.present = [h is not None for h in hs]
        with torch.no_grad():
            out = op(*[None if h is None else h.float() for h in hs], *rest)
        return out.to(H)

    @staticmethod
    def backward(ctx, g):
        saved = iter(ctx.saved_tensors)
        hs = [next(saved) if p else None for p in ctx.present]
        with torch.enable_grad():
            fs = [None if h is None else h.float().requires_grad_(True) for h in hs]
            out = ctx.op(*fs, *ctx.rest)
            need = [f for f in fs if f is not None]
            grads = torch.autograd.grad(out, need, g.to(H).float(), allow_unused=True)
        it = iter(grads)
        res = []
        for f, dt in zip(fs, ctx.dtypes):
            if f is None:
                res.append(None)
                continue
            gr = next(it)
            res.append(None if gr is None else gr.to(H).to(dt))
        return (None, None, *res)


def _linear(x, w, b=None):
    return _Lower16.apply(F.linear, 3, x, w, b)


def _binary(op):
    def f(a, b, *rest):
        return _Lower16.apply(op, 2, a, b, *rest)
    return f


def _addmm(inp, a, b, *, beta=1, alpha=1):
    return _Lower16.apply(lambda i, x, y: torch.addmm(i, x, y, beta=beta, alpha=alpha), 3, inp, a, b)


def _einsum(eq, *ops):
    if len(ops) == 1 and isinstance(ops[0], (list, tuple)):
        ops = tuple(ops[0])
    return _Lower16.apply(lambda *t: torch.einsum(eq, *t), len(ops), *ops)


LOWER = {
    F.linear: _linear,
    torch.matmul: _binary(torch.matmul),
    torch.Tensor.matmul: _binary(torch.matmul),
    torch.Tensor.__matmul__: _binary(torch.matmul),
    torch.Tensor.__rmatmul__: lambda a, b: _binary(torch.matmul)(b, a),
    torch.mm: _binary(torch.mm),
    torch.Tensor.mm: _binary(torch.mm),
    torch.bmm: _binary(torch.bmm),
    torch.Tensor.bmm: _binary(torch.bmm),
    torch.addmm: _addmm,
    torch.einsum: _einsum,
}

# CUDA autocast's fp32 list (ops that autocast to float32) as the reference's Python reaches them
_FP32_NAMES = [
    "exp", "expm1", "log", "log10", "log2", "log1p", "reciprocal", "rsqrt", "acos", "asin", "cosh", "sinh", "tan",
    "erfinv", "pow", "sum", "prod", "cumsum", "cumprod", "norm", "logsumexp", "softmax", "log_softmax", "dist", "cdist",
    "renorm",
]
FP32 = set()
for _n in _FP32_NAMES:
    for _ns in (torch, torch.Tensor):
        if hasattr(_ns, _n):
            FP32.add(getattr(_ns, _n))
FP32 |= {torch.Tensor.__pow__, torch.Tensor.__rpow__, torch.linalg.vector_norm, torch.linalg.norm,
         torch.linalg.matrix_norm, F.softplus, F.layer_norm, F.group_norm, F.l1_loss, F.mse_loss, F.smooth_l1_loss,
         F.huber_loss, F.binary_cross_entropy_with_logits, F.cosine_similarity, F.softmax, F.log_softmax, F.kl_div,
         F.nll_loss}

FP16_SEEN: dict = {}


def _is_fp16_arg(args, kwargs):
    return any(t.dtype == H for t in _tensors(args)) or any(t.dtype == H for t in _tensors(kwargs))


class CudaAutocastFp16(TorchFunctionMode):
    """``with CudaAutocastFp16(): outputs = model(ray_bundle)`` -- the reference's forward under CUDA's fp16 autocast
    policy (module docstring)."""

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func in LOWER:
            return LOWER[func](*args, **kwargs)
        if func in FP32 and _is_fp16_arg(args, kwargs):
            up = lambda t: t.float() if t.dtype == H else t   # noqa: E731
            return func(*_map(args, up), **_map(kwargs, up))
        if _is_fp16_arg(args, kwargs):
            name = getattr(func, "__qualname__", None) or getattr(func, "__name__", str(func))
            key = (name, tuple(str(t.dtype).replace("torch.", "") for t in _tensors(args)))
            FP16_SEEN[key] = FP16_SEEN.get(key, 0) + 1
        return func(*args, **kwargs)


def fp16_finite(params) -> bool:
    """GradScaler's inf / nan check over the (still scaled) gradients."""
    return all(p.grad is None or bool(torch.isfinite(p.grad).all()) for p in params)
