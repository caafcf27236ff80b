"""Stored dZ of the 4-layer chain backward vs an fp64 restatement, per hidden layer (error location)."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from multimodalstudio_amd import functions as fx

dev = torch.device("cuda", 0)
dims = [39, 256, 256, 256, 256]
g = torch.Generator().manual_seed(sum(dims))
M = 1500
params = []
for l in range(4):
    k, n = dims[l], dims[l + 1]
    v = torch.randn(n, k, generator=g) / np.sqrt(k)
    params += [v.norm(dim=1, keepdim=True).clone(), v, torch.randn(n, generator=g) * 0.1]
params = [p.to(dev).requires_grad_(True) for p in params]
acts = [(1, 1.0, 20.0)] * 4
x = torch.randn(M, dims[0], generator=g)
X = fx._alloc(M, 39, dev); X.copy_(x)
run = fx.ChainRun(params, acts, 1)
y = run.forward(X, keep=True)
Y = [t.detach().clone().double().cpu() for t in run.Y]
dy = torch.randn(M, dims[4], generator=g)
DY = fx._alloc(M, 256, dev); DY.copy_(dy)
captured = {}
orig = fx.gemm
def spy(mode, N, K, Mr, A, lda, B, ldb, C, ldc, **kw):
    if mode == fx.TN:
        captured.setdefault("A", []).append(A.detach().clone().double().cpu())
    return orig(mode, N, K, Mr, A, lda, B, ldb, C, ldc, **kw)
fx.gemm = spy
dx = run.backward(DY)
torch.cuda.synchronize()
d = dy.double()
refs = [None] * 4
for l in range(3, -1, -1):
    d = d * (Y[l] > 0)
    refs[l] = d
    gg, v = params[3 * l].detach().double().cpu(), params[3 * l + 1].detach().double().cpu()
    d = d @ torch._weight_norm(v, gg, 0)
for l, A in enumerate(captured["A"]):
    r = refs[l]
    e = (A - r).abs()
    rows = (e.max(1).values > 0.05 * r.abs().max()).nonzero().flatten()
    cols = (e.max(0).values > 0.05 * r.abs().max()).nonzero().flatten()
    print(f"layer {l}: rel {float(e.max() / r.abs().max()):.3e}; bad rows {rows[:20].tolist()} (n={len(rows)}); "
          f"bad cols {cols[:40].tolist()} (n={len(cols)})")
print("dx rel", float((dx.double().cpu() - d).abs().max() / d.abs().max()))
