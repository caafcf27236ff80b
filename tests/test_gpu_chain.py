"""GPU parity of the fused MLP chain kernels (mms_mlp_chain: all three layers of the SDF / radiance MLP in one
launch, bf16 or split-bf16x3 operands) against the reference's golden MLP vectors (tests/golden/mlp_*.npz) and,
for the SDF's tap-row mode (rows_full), against an fp64 PyTorch restatement.

Tolerances (scale-relative, written per mode): split-bf16x3 operands carry ~2^-16 relative precision, so outputs
and gradients are held to 1e-4; plain bf16 operands (8 bits) to 3e-2.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
TOL = {2: 1e-4, 1: 3e-2}
CASES = {"geo": [(2, 100.0, 20.0), (2, 100.0, 20.0), (0, 1.0, 20.0)],
         "rad": [(1, 1.0, 20.0), (1, 1.0, 20.0), (1, 1.0, 20.0)]}
PKEYS = ["parametrizations.weight.original0", "parametrizations.weight.original1", "bias"]


def rel(actual, ref):
    a = np.asarray(actual, dtype=np.float64)
    r = np.asarray(ref, dtype=np.float64)
    return np.abs(a - r).max() / max(np.abs(r).max(), 1e-30)


def _params(f, dev):
    return [torch.from_numpy(f[f"p:layers.{l}.{k}"]).to(dev).requires_grad_(True) for l in range(3) for k in PKEYS]


def _panel(x, dev):
    from multimodalstudio_amd.functions import _alloc
    X = _alloc(x.shape[0], x.shape[1], dev)
    X.copy_(torch.as_tensor(x))
    return X


def _masked_ref(x, params, acts, Y, dy):
    """fp64 backward of the weight-normed MLP with every activation derivative taken at the kernel's OWN forward
    outputs Y[l] (act' from the output, as the kernel does).  With bf16 operands a pre-activation within rounding of
    zero can land on the other side of a ReLU than in fp32; such sign flips are forward precision, not backward
    errors, so the bf16 backward is checked against this reference.  Returns dx and the parameter gradients."""
    ins = [torch.as_tensor(x).double(), Y[0].double().cpu(), Y[1].double().cpu()]
    d = torch.as_tensor(dy).double()
    out = [None] * 9
    for l in (2, 1, 0):
        act, beta, thr = acts[l]
        y = (Y[l] if l < 2 else Y[2]).double().cpu()
        if act == 1:
            d = d * (y > 0)
        elif act == 2:
            d = d * torch.where(y * beta > thr, torch.ones_like(y), 1.0 - torch.exp(-beta * y))
        g64 = params[3 * l].detach().double().cpu().requires_grad_(True)
        v64 = params[3 * l + 1].detach().double().cpu().requires_grad_(True)
        W = torch._weight_norm(v64, g64, 0)
        W.backward(d.T @ ins[l])
        out[3 * l], out[3 * l + 1], out[3 * l + 2] = g64.grad, v64.grad, d.sum(0)
        d = d @ W.detach()
    return d, out


@pytest.mark.parametrize("prec", [2, 1])
@pytest.mark.parametrize("name", list(CASES))
def test_chain_vs_golden(dev, name, prec):
    """Forward vs the reference's golden output; backward vs the golden gradients (split bf16x3) or, for plain bf16,
    vs an fp64 backward taken at the kernel's own activations (see _masked_ref)."""
    from multimodalstudio_amd import functions as fx
    f = dict(np.load(os.path.join(GOLD, f"mlp_{name}.npz")))
    params = _params(f, dev)
    X = _panel(f["x"], dev)
    run = fx.ChainRun(params, CASES[name], prec)
    y = run.forward(X, keep=True)
    Y = [t.detach().clone() for t in run.Y]
    dy = _panel(f["dy"], dev)
    dx = run.backward(dy)
    torch.cuda.synchronize()
    tol = TOL[prec]
    errs = {"y": rel(y.cpu(), f["y"])}
    if prec == 2:
        ref_dx = f["dx"]
        ref_g = [f[f"g:layers.{l}.{k}"] for l in range(3) for k in PKEYS]
    else:
        ref_dx, ref_g = _masked_ref(f["x"], params, CASES[name], Y, f["dy"])
    errs["dx"] = rel(dx.cpu(), ref_dx)
    for i, p in enumerate(params):
        l, k = divmod(i, 3)
        errs[f"g{l}.{PKEYS[k][-9:]}"] = rel(p.grad.cpu(), ref_g[i])
    print(name, prec, {k: f"{v:.1e}" for k, v in errs.items()})
    for k, v in errs.items():
        assert v < tol, f"{name} prec={prec} {k}: {v:.2e}"


def test_sdf_chain_split_activations(dev):
    """mms_mlp_chain prec 3 (the SDF chain of `fast_x2`, a measured but non-parity preset): bf16 weights W~ = bf16(W) times split-bf16 (hi + lo)
    activations.  The chain must be the MLP of the ROUNDED weights at ~2^-16 activation precision: forward vs an fp64
    forward through W~, backward (dx, every parameter gradient) vs the fp64 backward through W~ at the kernel's own
    activations, both to 1e-4 -- i.e. the rounding is the weights' alone, and the SDF's tap differences remain exact
    differences of one function."""
    from multimodalstudio_amd import functions as fx
    f = dict(np.load(os.path.join(GOLD, "mlp_geo.npz")))
    params = _params(f, dev)
    acts = CASES["geo"]
    X = _panel(f["x"], dev)
    run = fx.ChainRun(params, acts, 2, chain_prec=3)
    y = run.forward(X, keep=True)
    Y = [t.detach().clone() for t in run.Y]
    dy = _panel(f["dy"], dev)
    dx = run.backward(dy)
    torch.cuda.synchronize()
    Wt = []
    for l in range(3):
        g, v = [p.detach().float().cpu() for p in params[3 * l: 3 * l + 2]]
        Wt.append(torch._weight_norm(v, g, 0).to(torch.bfloat16).double())
    h = torch.as_tensor(f["x"]).double()
    for l in range(3):
        h = h @ Wt[l].T + params[3 * l + 2].detach().double().cpu()
        act, beta, thr = acts[l]
        if act == 2:
            h = torch.nn.functional.softplus(h, beta=beta, threshold=thr)
    errs = {"y": rel(y.cpu(), h)}
    ins = [torch.as_tensor(f["x"]).double(), Y[0].double().cpu(), Y[1].double().cpu()]
    d = torch.as_tensor(f["dy"]).double()
    for l in (2, 1, 0):
        act, beta, thr = acts[l]
        if act == 2:
            yl = Y[l].double().cpu()
            d = d * torch.where(yl * beta > thr, torch.ones_like(yl), 1.0 - torch.exp(-beta * yl))
        g64 = params[3 * l].detach().double().cpu().requires_grad_(True)
        v64 = params[3 * l + 1].detach().double().cpu().requires_grad_(True)
        torch._weight_norm(v64, g64, 0).backward(d.T @ ins[l])
        errs[f"g{l}"] = rel(params[3 * l].grad.cpu(), g64.grad)
        errs[f"v{l}"] = rel(params[3 * l + 1].grad.cpu(), v64.grad)
        errs[f"b{l}"] = rel(params[3 * l + 2].grad.cpu(), d.sum(0))
        d = d @ Wt[l]
    errs["dx"] = rel(dx.cpu(), d)
    print("split activations", {k: f"{v:.1e}" for k, v in errs.items()})
    for k, v in errs.items():
        assert v < 1e-4, f"prec=3 {k}: {v:.2e}"


def _ref_mlp(x, params, acts, leaves=None):
    """fp64 forward; ``leaves``: fp64 CPU copies of params to differentiate through (else detached copies)."""
    h = x
    for l in range(3):
        g, v, b = leaves[3 * l: 3 * l + 3] if leaves is not None else \
            [p.detach().double().cpu() for p in params[3 * l: 3 * l + 3]]
        w = torch._weight_norm(v, g, 0)
        h = h @ w.T + b
        act, beta, thr = acts[l]
        if act == 1:
            h = torch.relu(h)
        elif act == 2:
            h = torch.nn.functional.softplus(h, beta=beta, threshold=thr)
    return h


@pytest.mark.parametrize("M,rows_full", [(1000, 200), (777, 777), (640, 0), (20000, 4000), (20013, 3990)])
def test_chain_sdf_tap_rows(dev, M, rows_full):
    """SDF chain with tap rows (>= rows_full): column 0 for every row, all 257 columns for the rows below; the
    backward reads only column 0 of the tap rows (the rest of those rows is garbage on purpose).  Parameter gradients
    too: the taps' share of the last layer's row 0 is summed inside the backward chain (dw_row0 / db_row0)."""
    from multimodalstudio_amd import functions as fx
    g = torch.Generator().manual_seed(M + rows_full)
    f = dict(np.load(os.path.join(GOLD, "mlp_geo.npz")))
    params = _params(f, dev)
    x = torch.randn(M, 71, generator=g) * 0.5
    X = _panel(x, dev)
    run = fx.ChainRun(params, CASES["geo"], 2)
    keep = rows_full > 0
    y = run.forward(X, keep=keep, rows_full=rows_full)
    xr = x.double().requires_grad_(True)
    leaves = [p.detach().double().cpu().requires_grad_(True) for p in params]
    ref = _ref_mlp(xr, params, CASES["geo"], leaves)
    yc = y.detach().cpu().double()
    assert rel(yc[:, 0], ref[:, 0].detach()) < TOL[2]
    if rows_full > 0:
        assert rel(yc[:rows_full], ref[:rows_full].detach()) < TOL[2]
    if not keep:
        return
    dy = torch.randn(M, 257, generator=g)
    dy[rows_full:, 1:] = float("nan")            # never read
    dyd = _panel(dy, dev)
    for p in params:
        p.grad = None
    dx = run.backward(dyd)
    torch.cuda.synchronize()
    dyr = dy.double().clone()
    dyr[rows_full:, 1:] = 0.0
    ref.backward(dyr)
    assert rel(dx.cpu(), xr.grad) < TOL[2]
    assert torch.isfinite(dx).all()
    for i, (p, q) in enumerate(zip(params, leaves)):
        assert rel(p.grad.cpu(), q.grad) < TOL[2], (i, rel(p.grad.cpu(), q.grad))


def test_sdf_only_fast_matches_fp32(dev):
    """The sampler's inference SDF (functions.sdf_only) on the chain kernel (fast preset) vs the fp32 GEMM path:
    same values, returned as a dense [M] vector (mms_neus_step reads it densely)."""
    from multimodalstudio_amd import functions as fx
    f = dict(np.load(os.path.join(GOLD, "mlp_geo.npz")))
    params = _params(f, dev)
    g = torch.Generator().manual_seed(3)
    pos = (torch.rand(3000, 3, generator=g) * 2 - 1).to(dev)
    grid = fx.GridCfg([float(int(16 * 1.3195079 ** l)) for l in range(16)], 12, 1.0)
    table = ((torch.rand(16 << 12, 2, generator=g) * 2 - 1) * 1e-2).to(dev)
    ref = fx.sdf_only(pos, table, grid, 16, params)
    fx.set_precision("fast")
    try:
        out = fx.sdf_only(pos, table, grid, 16, params)
    finally:
        fx.set_precision("fp32")
    torch.cuda.synchronize()
    assert out.is_contiguous() and out.shape == ref.shape
    # a bf16-weight SDF chain (prec 3, fast_x2) moves the sdf by the weights' rounding (2^-9 relative): looser bound
    tol = TOL[2] if fx.PRESETS["fast"]["sdf_chain"] in (0, 2) else 1e-2
    assert rel(out.cpu(), ref.cpu()) < tol


def _masked_ref_n(x, params, acts, Y, dy):
    """_masked_ref for any layer count (ReLU / none activations)."""
    L = len(params) // 3
    ins = [torch.as_tensor(x).double()] + [Y[l].double().cpu() for l in range(L - 1)]
    d = torch.as_tensor(dy).double()
    out = [None] * (3 * L)
    for l in range(L - 1, -1, -1):
        if acts[l][0] == 1:
            d = d * (Y[l].double().cpu() > 0)
        g64 = params[3 * l].detach().double().cpu().requires_grad_(True)
        v64 = params[3 * l + 1].detach().double().cpu().requires_grad_(True)
        W = torch._weight_norm(v64, g64, 0)
        W.backward(d.T @ ins[l])
        out[3 * l], out[3 * l + 1], out[3 * l + 2] = g64.grad, v64.grad, d.sum(0)
        d = d @ W.detach()
    return d, out


@pytest.mark.parametrize("prec", [1, 4])
@pytest.mark.parametrize("dims", [[39, 256, 256, 256, 256], [283, 256, 256, 256, 128], [283, 256, 256, 256, 256],
                                  [317, 256, 256, 256]])
def test_chain_relu_layers(dev, dims, prec):
    """ReLU chains in bf16 (prec 1) and in mode 4 (split-bf16x3 forward, bf16 backward) -- the background NeRF's
    4-layer MLPs and the radiance MLP -- at a row count that is not a multiple of the 128-row block (the clamped rows
    past M must store exactly row M - 1's values): forward vs an fp64 restatement, backward (dx and every weight-norm /
    bias gradient, i.e. every stored dZ) vs the fp64 backward at the kernel's own activations; the last layer writes
    into a caller-owned strided view (the background panel)."""
    from multimodalstudio_amd import functions as fx
    g = torch.Generator().manual_seed(sum(dims))
    M = 1500
    L = len(dims) - 1
    params = []
    for l in range(L):
        k, n = dims[l], dims[l + 1]
        v = torch.randn(n, k, generator=g) / np.sqrt(k)
        params += [v.norm(dim=1, keepdim=True).clone(), v, torch.randn(n, generator=g) * 0.1]
    params = [p.to(dev).requires_grad_(True) for p in params]
    acts = [(1, 1.0, 20.0)] * L
    x = torch.randn(M, dims[0], generator=g)
    X = _panel(x, dev)
    panel = fx._alloc(M, dims[L] + 27, dev)
    assert fx._chain_shape(params, acts, prec)
    run = fx.ChainRun(params, acts, prec)
    y = run.forward(X, keep=True, last_out=panel[:, :dims[L]])
    assert y.data_ptr() == panel.data_ptr()
    h = x.double()
    for l in range(L):
        gg, v, b = [p.detach().double().cpu() for p in params[3 * l: 3 * l + 3]]
        h = torch.relu(h @ torch._weight_norm(v, gg, 0).T + b)
    assert rel(y.detach().cpu(), h) < (TOL[2] if prec == 4 else TOL[1])
    Y = [t.detach().clone() for t in run.Y]
    dy = torch.randn(M, dims[L], generator=g)
    dx = run.backward(_panel(dy, dev))
    torch.cuda.synchronize()
    ref_dx, ref_g = _masked_ref_n(x, params, acts, Y, dy)
    assert rel(dx.cpu(), ref_dx) < TOL[1]
    for i, p in enumerate(params):
        assert rel(p.grad.cpu(), ref_g[i]) < TOL[1], (i, rel(p.grad.cpu(), ref_g[i]))


@pytest.mark.parametrize("prec,C,out", [(1, 3, 3), (1, 1, 3), (1, 5, 3), (4, 3, 3), (4, 1, 3), (4, 5, 3), (2, 3, 0),
                                        (1, 3, 0)])
def test_chain_head(dev, C, prec, out):
    """A modality head 256-64-64-C (ReLU, ReLU, Sigmoid: field_heads.py:71-88; or no output activation: the
    polarization heads' Stokes, :90-106) on the chain kernel: forward vs fp64, backward (dx, every parameter gradient)
    vs the fp64 backward at the kernel's own activations (Sigmoid' from the output), at a row count that is not a
    multiple of the 128-row block."""
    from multimodalstudio_amd import functions as fx
    dims = [256, 64, 64, C]
    g = torch.Generator().manual_seed(C)
    M = 1500
    params = []
    for l in range(3):
        k, n = dims[l], dims[l + 1]
        v = torch.randn(n, k, generator=g) / np.sqrt(k)
        params += [v.norm(dim=1, keepdim=True).clone(), v, torch.randn(n, generator=g) * 0.1]
    params = [p.to(dev).requires_grad_(True) for p in params]
    acts = [(1, 1.0, 20.0), (1, 1.0, 20.0), (out, 1.0, 20.0)]
    assert fx._chain_shape(params, acts, prec)
    x = torch.randn(M, 256, generator=g)
    run = fx.ChainRun(params, acts, prec)
    y = run.forward(_panel(x, dev), keep=True)
    h = x.double()
    for l in range(3):
        gg, v, b = [p.detach().double().cpu() for p in params[3 * l: 3 * l + 3]]
        h = h @ torch._weight_norm(v, gg, 0).T + b
        h = torch.relu(h) if l < 2 else (torch.sigmoid(h) if out == 3 else h)
    assert rel(y.detach().cpu(), h) < (TOL[2] if prec in (2, 4) else TOL[1])
    Y = [t.detach().clone().double().cpu() for t in run.Y]
    dy = torch.randn(M, C, generator=g)
    dx = run.backward(_panel(dy, dev))
    torch.cuda.synchronize()
    d = dy.double() * Y[2] * (1 - Y[2]) if out == 3 else dy.double()
    ins = [x.double(), Y[0], Y[1]]
    ref = [None] * 9
    for l in (2, 1, 0):
        if l < 2:
            d = d * (Y[l] > 0)
        g64 = params[3 * l].detach().double().cpu().requires_grad_(True)
        v64 = params[3 * l + 1].detach().double().cpu().requires_grad_(True)
        W = torch._weight_norm(v64, g64, 0)
        W.backward(d.T @ ins[l])
        ref[3 * l], ref[3 * l + 1], ref[3 * l + 2] = g64.grad, v64.grad, d.sum(0)
        d = d @ W.detach()
    assert rel(dx.cpu(), d) < TOL[1]
    for i, p in enumerate(params):
        assert rel(p.grad.cpu(), ref[i]) < TOL[1], (i, rel(p.grad.cpu(), ref[i]))


@pytest.mark.parametrize("dims,acts", [
    ([317, 256, 256, 256], [(1, 1.0, 20.0)] * 3),                                   # radiance
    ([256, 64, 64, 3], [(1, 1.0, 20.0), (1, 1.0, 20.0), (3, 1.0, 20.0)]),         # plain head (Sigmoid)
    ([256, 64, 64, 3], [(1, 1.0, 20.0), (1, 1.0, 20.0), (0, 1.0, 20.0)]),         # polarization head (Stokes)
    ([39, 256, 256, 256, 256], [(1, 1.0, 20.0)] * 4),                              # background base
    ([283, 256, 256, 256, 128], [(1, 1.0, 20.0)] * 4)])                            # background head
def test_chain_fp16_forward(dev, dims, acts):
    """Preset fast_h16: the radiance / head / background forward chains on fp16 operands (mms_mlp_chain prec 5, one
    fp16 MFMA per product, fp32 accumulation -- the reference GPU's autocast precision).  Forward vs fp64 within 3e-3
    of each output's scale (fp16's 11-bit operands over K <= 317); the backward chain of the same run is split-bf16x3
    and is checked against the fp64 backward taken at the kernel's own activations to the split-bf16x3 bound."""
    from multimodalstudio_amd import functions as fx
    g = torch.Generator().manual_seed(sum(dims))
    L = len(dims) - 1
    params = []
    for k, n in zip(dims[:-1], dims[1:]):
        v = torch.randn(n, k, generator=g) / k ** 0.5
        params += [torch.linalg.vector_norm(v, dim=1, keepdim=True).to(dev).requires_grad_(True),
                   v.to(dev).requires_grad_(True), (torch.randn(n, generator=g) * 0.1).to(dev).requires_grad_(True)]
    assert fx._chain_shape(params, acts, 5)
    M = 3000
    x = torch.randn(M, dims[0], generator=g) * 0.5
    run = fx.ChainRun(params, acts, 5)
    assert run.cprec == 5 and run.bcprec == 2
    y = run.forward(_panel(x, dev), keep=True)
    Y = [t.detach().clone() for t in run.Y]
    h = x.double()
    for l in range(L):
        gg, v, b = [p.detach().double().cpu() for p in params[3 * l: 3 * l + 3]]
        h = h @ torch._weight_norm(v, gg, 0).T + b
        act = acts[l][0]
        h = torch.relu(h) if act == 1 else (torch.sigmoid(h) if act == 3 else h)
    e_fwd = rel(y.detach().cpu(), h)
    dy = torch.randn(M, dims[-1], generator=g)
    dx = run.backward(_panel(dy, dev))
    torch.cuda.synchronize()
    # fp64 backward at the kernel's own activations (ReLU / Sigmoid derivatives from its outputs)
    ins = [x.double()] + [t.double().cpu() for t in Y[:L - 1]]
    d = dy.double()
    errs = {}
    for l in range(L - 1, -1, -1):
        act = acts[l][0]
        yl = Y[l].double().cpu()
        if act == 1:
            d = d * (yl > 0)
        elif act == 3:
            d = d * yl * (1 - yl)
        gg = params[3 * l].detach().double().cpu().requires_grad_(True)
        v = params[3 * l + 1].detach().double().cpu().requires_grad_(True)
        W = torch._weight_norm(v, gg, 0)
        W.backward(d.T @ ins[l])
        errs[f"v{l}"] = rel(params[3 * l + 1].grad.cpu(), v.grad)
        errs[f"b{l}"] = rel(params[3 * l + 2].grad.cpu(), d.sum(0))
        d = d @ W.detach()
    errs["dx"] = rel(dx.cpu(), d)
    print(dims, f"fp16 forward rel {e_fwd:.2e}", {k: f"{v:.1e}" for k, v in errs.items()})
    assert e_fwd < 3e-3
    for k, v in errs.items():
        assert v < TOL[2], (k, v)


@pytest.mark.parametrize("dims,acts,M,rows_full", [
    ([71, 256, 256, 257], CASES["geo"], 777, 777),                                 # SDF
    ([71, 256, 256, 257], CASES["geo"], 20013, 3990),                              # SDF with tap rows
    ([317, 256, 256, 256], [(1, 1.0, 20.0)] * 3, 3000, None),                      # radiance
    ([256, 64, 64, 3], [(1, 1.0, 20.0), (1, 1.0, 20.0), (3, 1.0, 20.0)], 3000, None),   # plain head (Sigmoid)
    ([256, 64, 64, 3], [(1, 1.0, 20.0), (1, 1.0, 20.0), (0, 1.0, 20.0)], 3000, None),   # polarization head
    ([39, 256, 256, 256, 256], [(1, 1.0, 20.0)] * 4, 3000, None),                  # background base
    ([283, 256, 256, 256, 128], [(1, 1.0, 20.0)] * 4, 3000, None)],                # background head
    ids=["sdf", "sdf_taps", "radiance", "head", "pol_head", "bg_base", "bg_head"])
@pytest.mark.parametrize("w16", [0, 1, 2], ids=["wgrad_x3", "wgrad16", "wgrad16_y16"])
def test_chain_fp16_backward(dev, dims, acts, M, rows_full, w16):
    """Preset fast_h16b: every backward-data chain on mms_mlp_chain prec 6 -- its first layer (B = dY from memory)
    split-bf16x3, the register-fed layers on fp16 operands with a per-row power-of-two scale (the reference GPU's fp16
    autocast backward, without its global loss scale); w16 (preset fast_h16c): the hidden layers' weight gradients
    from the chain's fp16 row-scaled dZ stores (mms_gemm_tn_wide16; the 64-wide heads keep the fp32 panels); w16 = 2
    (fast_h16d): the forward's hidden activations stored as fp16 rows too (the reference below is taken at them).  dX and
    every parameter gradient vs the fp64 backward taken at
    the kernel's own forward activations within 3e-3 of each tensor's scale (fp16's 11-bit operands over K <= 256;
    split-bf16x3 measures ~1e-5 here), finite everywhere; rows of very different magnitude (1e-6 .. 1e3 in dY) keep
    that relative accuracy per row (the row scale), and the tap rows read only column 0."""
    from multimodalstudio_amd import functions as fx
    g = torch.Generator().manual_seed(sum(dims) + M)
    L = len(dims) - 1
    params = []
    for k, n in zip(dims[:-1], dims[1:]):
        v = torch.randn(n, k, generator=g) / k ** 0.5
        params += [torch.linalg.vector_norm(v, dim=1, keepdim=True).to(dev).requires_grad_(True),
                   v.to(dev).requires_grad_(True), (torch.randn(n, generator=g) * 0.1).to(dev).requires_grad_(True)]
    sdf = dims[0] == 71
    prec = 2 if sdf else 5
    old = dict(fx.PRECISION)
    fx.PRECISION["bwd16"] = 1
    fx.PRECISION["wgrad16"] = int(w16 > 0)
    fx.PRECISION["y16"] = int(w16 == 2)
    try:
        run = fx.ChainRun(params, acts, prec)
        assert run.bcprec == 6
        x = torch.randn(M, dims[0], generator=g) * 0.5
        run.forward(_panel(x, dev), keep=True, rows_full=rows_full)
        Y = [t.detach().clone() for t in run.Y]
        dy = torch.randn(M, dims[-1], generator=g)
        dy *= 10.0 ** torch.randint(-6, 4, (M, 1), generator=g).double().float()    # per-row magnitudes
        dy[1::17] = 0.0           # all-zero rows (fixed-capacity padding rows: fp16 weight gradients' rinv 0)
        rf = M if rows_full is None else rows_full
        dyr = dy.double().clone()
        dyr[rf:, 1:] = 0.0
        dy[rf:, 1:] = float("nan")          # never read
        dx = run.backward(_panel(dy, dev))
        torch.cuda.synchronize()
    finally:
        fx.PRECISION.clear()
        fx.PRECISION.update(old)
    ins = [x.double()] + [t.double().cpu() for t in Y[:L - 1]]
    d = dyr
    errs = {}
    for l in range(L - 1, -1, -1):
        act, beta, _ = acts[l]
        if l < L - 1 or act != 0:
            yl = Y[l].double().cpu()
            if act == 1:
                d = d * (yl > 0)
            elif act == 2:
                d = d * (1 - torch.exp(-beta * yl))
            elif act == 3:
                d = d * yl * (1 - yl)
        gg = params[3 * l].detach().double().cpu().requires_grad_(True)
        v = params[3 * l + 1].detach().double().cpu().requires_grad_(True)
        W = torch._weight_norm(v, gg, 0)
        W.backward(d.T @ ins[l])
        errs[f"v{l}"] = rel(params[3 * l + 1].grad.cpu(), v.grad)
        errs[f"g{l}"] = rel(params[3 * l].grad.cpu(), gg.grad)
        errs[f"b{l}"] = rel(params[3 * l + 2].grad.cpu(), d.sum(0))
        d = d @ W.detach()
    assert torch.isfinite(dx).all()
    errs["dx"] = rel(dx.cpu(), d)
    # per-row relative error of dX (the row scale keeps small rows as accurate as large ones)
    dxc = dx.cpu().double()
    row_err = ((dxc - d).abs().amax(1) / d.abs().amax(1).clamp_min(1e-300)).max().item()
    print(dims, rows_full, {k: f"{v:.1e}" for k, v in errs.items()}, f"row max {row_err:.1e}")
    for k, v in errs.items():
        assert v < 3e-3, (k, v)
    assert row_err < 1e-2


def _autocast_sdf_backward(x, params, acts, Y, dyr):
    """The reference GPU's fp16-autocast backward of the SDF MLP (trainer.py:51: nn.Linear in fp16 -- operands rounded
    to fp16, fp32 accumulation, fp16 results --, Softplus upcast to fp32 and its input gradient cast back to fp16, the
    loss scaled by the largest power of two that keeps every fp16 gradient finite, GradScaler-style, and unscaled at
    the end) restated in float64 with fp16 rounding at those points, at the kernel's own forward activations Y.
    Returns dx and the (g, v, b) gradients of each layer, like _masked_ref."""
    h16 = lambda t: t.half().double()    # noqa: E731
    L = len(params) // 3
    Ws = []
    for l in range(L):
        g64 = params[3 * l].detach().double().cpu()
        v64 = params[3 * l + 1].detach().double().cpu()
        Ws.append(torch._weight_norm(v64, g64, 0))
    ins = [x.double()] + [Y[l].double().cpu() for l in range(L - 1)]
    # largest |gradient| anywhere in the chain (fp64), to pick the scale
    d, peak = dyr.clone(), dyr.abs().max().item()
    for l in range(L - 1, -1, -1):
        if l < L - 1:
            d = d * (1 - torch.exp(-acts[l][1] * ins[l + 1]))
        peak = max(peak, d.abs().max().item(), (d.T @ ins[l]).abs().max().item())
        d = d @ Ws[l]
        peak = max(peak, d.abs().max().item())
    S = 2.0 ** np.floor(np.log2(32768.0 / peak))
    d = h16(dyr * S)
    out = [None] * (3 * L)
    for l in range(L - 1, -1, -1):
        if l < L - 1:      # Softplus in fp32 on the fp16 pre-activation, its input gradient cast back to fp16
            d = h16(d * (1 - torch.exp(-acts[l][1] * ins[l + 1])))
        dW = h16(d.T @ h16(ins[l])) / S
        g64 = params[3 * l].detach().double().cpu().requires_grad_(True)
        v64 = params[3 * l + 1].detach().double().cpu().requires_grad_(True)
        torch._weight_norm(v64, g64, 0).backward(dW)
        out[3 * l], out[3 * l + 1], out[3 * l + 2] = g64.grad, v64.grad, h16(d.sum(0)) / S
        d = h16(d @ h16(Ws[l]))
    return d / S, out


@pytest.mark.parametrize("delta", [1e-3, 2.5e-4])
def test_sdf_backward_fp16_on_antisymmetric_taps(dev, delta):
    """presets fast_h16b / fast_h16c run the SDF backward-data chain on prec 6 (fp16 register-fed layers with a per-row
    scale).  The SDF's real dY is not random per row: the eikonal loss puts k_t . g / (4 delta) on the 4 tap rows of a
    sample and the curvature loss c / (2 delta^2) on each tap and -2 c / delta^2 on the centre
    (/root/reference/src/model_components/surface_model.py:137-151), and the tap rows' inputs differ from the centre's
    by O(delta) -- so the weight gradients are sums of large, nearly cancelling per-row terms.  On that pattern the
    prec-6 dX and parameter gradients (vs fp64 at the kernel's own activations) must stay within 2x the error of the
    reference GPU's own fp16-autocast backward of the same chain (_autocast_sdf_backward) -- prec 6 rounds each row to
    fp16 like the autocast does, but with a per-row instead of a global scale.  The split-bf16x3 backward is reported
    beside it."""
    from multimodalstudio_amd import functions as fx
    g = torch.Generator().manual_seed(int(1 / delta))
    f = dict(np.load(os.path.join(GOLD, "mlp_geo.npz")))
    params = _params(f, dev)
    acts = CASES["geo"]
    C = 2000
    xc = torch.randn(C, 71, generator=g) * 0.5
    A = torch.randn(71, 3, generator=g)                      # d panel / d position
    k = torch.tensor([[1., -1., -1.], [-1., -1., 1.], [-1., 1., -1.], [1., 1., 1.]])
    x = torch.cat([xc] + [xc + delta * (A @ k[t]) for t in range(4)])
    M = 5 * C
    gv = torch.randn(C, 3, generator=g)                      # d loss / d gradient (eikonal)
    cv = torch.randn(C, 1, generator=g) * 1e-3               # d loss / d hessian (curvature)
    dy = torch.randn(M, 257, generator=g)
    dy[:C, :1] += -2.0 * cv / delta ** 2
    for t in range(4):
        dy[C * (t + 1): C * (t + 2), :1] = (gv @ k[t])[:, None] / (4 * delta) + cv / (2 * delta ** 2)
    dyr = dy.double().clone()
    dyr[C:, 1:] = 0.0
    dy[C:, 1:] = float("nan")                # never read
    errs = {}
    for name, bwd16, w16 in (("x3", 0, 0), ("prec6", 1, 0), ("prec6w16", 1, 1), ("prec6y16", 1, 2)):
        old = dict(fx.PRECISION)
        fx.PRECISION["bwd16"] = bwd16
        fx.PRECISION["wgrad16"] = int(w16 > 0)
        fx.PRECISION["y16"] = int(w16 == 2)
        try:
            for p in params:
                p.grad = None
            run = fx.ChainRun(params, acts, 2)
            assert run.bcprec == (6 if bwd16 else 2)
            run.forward(_panel(x, dev), keep=True, rows_full=C)
            Y = [t.detach().clone() for t in run.Y]
            dx = run.backward(_panel(dy, dev))
            torch.cuda.synchronize()
        finally:
            fx.PRECISION.clear()
            fx.PRECISION.update(old)
        grads = [p.grad.detach().cpu().double().clone() for p in params]
        ref_dx, ref_g = _masked_ref(x, params, acts, Y, dyr)
        e = {"dx": rel(dx.cpu(), ref_dx)}
        e.update({f"p{i}": rel(grads[i], ref_g[i]) for i in range(len(params))})
        errs[name] = e
    am_dx, am_g = _autocast_sdf_backward(x, params, acts, Y, dyr)
    e = {"dx": rel(am_dx, ref_dx)}
    e.update({f"p{i}": rel(am_g[i], ref_g[i]) for i in range(len(params))})
    errs["autocast"] = e
    for q in errs["x3"]:
        print(f"  delta {delta:.1e} {q:4s} x3 {errs['x3'][q]:.2e}  prec6 {errs['prec6'][q]:.2e}  "
              f"prec6 + fp16 wgrad {errs['prec6w16'][q]:.2e}  + fp16 Y {errs['prec6y16'][q]:.2e}  "
              f"ref-fp16-autocast {errs['autocast'][q]:.2e}")
    for mode in ("prec6", "prec6w16", "prec6y16"):
        for q, v in errs[mode].items():
            assert np.isfinite(v) and v <= 2.0 * errs["autocast"][q] + 1e-6, (mode, q, v, errs["autocast"][q])
