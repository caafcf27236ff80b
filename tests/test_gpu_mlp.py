"""GPU parity: weight-normed MLP (fp32 MFMA GEMMs) vs the reference's golden vectors (tests/golden/mlp_*.npz)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")

CASES = {
    # name: (layers, [(act, beta, thr) per layer])
    "geo": (3, [(2, 100.0, 20.0), (2, 100.0, 20.0), (0, 1.0, 20.0)]),
    "rad": (3, [(1, 1.0, 20.0), (1, 1.0, 20.0), (1, 1.0, 20.0)]),
    "head": (3, [(1, 1.0, 20.0), (1, 1.0, 20.0), (3, 1.0, 20.0)]),
}


def close(actual, ref, rel, what):
    actual = np.asarray(actual, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    scale = np.abs(ref).max()
    err = np.abs(actual - ref).max()
    assert err <= rel * scale + 1e-12, f"{what}: max err {err:.3e} vs scale {scale:.3e}"


@pytest.mark.parametrize("name", list(CASES))
def test_mlp_golden(dev, name):
    from multimodalstudio_amd import functions as fx
    f = dict(np.load(os.path.join(GOLD, f"mlp_{name}.npz")))
    L, acts = CASES[name]
    params = []
    for l in range(L):
        for k in ["parametrizations.weight.original0", "parametrizations.weight.original1", "bias"]:
            params.append(torch.from_numpy(f[f"p:layers.{l}.{k}"]).to(dev).requires_grad_(True))
    x = torch.from_numpy(f["x"]).to(dev).requires_grad_(True)
    y = fx.MLPFunction.apply(x, tuple(acts), "heads", *params)
    y.backward(torch.from_numpy(f["dy"]).to(dev))
    torch.cuda.synchronize()
    close(y.detach().cpu(), f["y"], 2e-6, "y")
    close(x.grad.cpu(), f["dx"], 2e-6, "dx")
    i = 0
    for l in range(L):
        for k in ["parametrizations.weight.original0", "parametrizations.weight.original1", "bias"]:
            close(params[i].grad.cpu(), f[f"g:layers.{l}.{k}"], 5e-6, f"layer{l}.{k}")
            i += 1
