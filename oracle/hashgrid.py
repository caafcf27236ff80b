"""ORACLE (test infrastructure only) — CPU restatement of the reference hash-grid encoding.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
The product path (multimodalstudio_amd) never imports it.

Follows the reference's torch implementation:
  * FeatureGrid.forward           /root/reference/src/field_components/feature_structures.py:78-83
  * FeatureGrid.update_mask       /root/reference/src/field_components/feature_structures.py:85-88
  * HashEncoding.__init__ scalings /root/reference/src/field_components/encodings.py:189-233
  * HashEncoding.hash_fn          /root/reference/src/field_components/encodings.py:244-261
  * HashEncoding.pytorch_fwd      /root/reference/src/field_components/encodings.py:263-304
Pinned by tests/golden/hashgrid_*.npz (generated from the reference by tests/golden/make_golden.py).
"""
from __future__ import annotations

import numpy as np
import torch

P1 = 2654435761
P2 = 805459861


def growth_factor(min_res: int, max_res: int, num_levels: int) -> float:
    """encodings.py:192-194: exp((ln max - ln min) / (L - 1)), computed in float64 like numpy."""
    return float(np.exp((np.log(max_res) - np.log(min_res)) / (num_levels - 1)))


def level_scales(min_res: int = 16, max_res: int = 1024, num_levels: int = 16) -> torch.Tensor:
    """encodings.py:227: floor(min_res * g ** arange(L)), in float32 (torch default dtype)."""
    g = growth_factor(min_res, max_res, num_levels)
    levels = torch.arange(num_levels)
    return torch.floor(min_res * g ** levels).to(torch.float32)


def corner_indices(scaled_c: torch.Tensor, scaled_f: torch.Tensor, log2T: int) -> list:
    """Eight hashed corner indices in reference order (encodings.py:274-281), int64 [..., L]."""
    T = 1 << log2T
    L = scaled_c.shape[-2]
    offs = torch.arange(L, dtype=torch.int64) * T

    def h(cx, cy, cz):
        x = cx.to(torch.int64) * 1
        y = cy.to(torch.int64) * P1
        z = cz.to(torch.int64) * P2
        v = torch.bitwise_xor(torch.bitwise_xor(x, y), z)
        return torch.remainder(v, T) + offs

    c, f = scaled_c, scaled_f
    X, Y, Z = 0, 1, 2
    return [
        h(c[..., X], c[..., Y], c[..., Z]),
        h(c[..., X], f[..., Y], c[..., Z]),
        h(f[..., X], f[..., Y], c[..., Z]),
        h(f[..., X], c[..., Y], c[..., Z]),
        h(c[..., X], c[..., Y], f[..., Z]),
        h(c[..., X], f[..., Y], f[..., Z]),
        h(f[..., X], f[..., Y], f[..., Z]),
        h(f[..., X], c[..., Y], f[..., Z]),
    ]


def hash_encode(x_hat: torch.Tensor, table: torch.Tensor, scales: torch.Tensor, log2T: int,
                interpolation: str = "Linear") -> torch.Tensor:
    """HashEncoding.pytorch_fwd on normalised inputs x_hat [..., 3] -> [..., L * F] (differentiable).

    interpolation "Smoothstep": the tcnn mode of HashEncodingConfig.interpolation (encodings.py:64-67,207-221), which
    the reference's torch path rejects (:235-238): the trilinear weights of the fractions t become S(t) =
    t^2 (3 - 2 t) (tiny-cuda-nn's published grid encoding; tcnn is absent here, so this restatement is unpinned)."""
    xs = x_hat[..., None, :] * scales.view(-1, 1)                  # [..., L, 3]
    sc = torch.ceil(xs).to(torch.int32)
    sf = torch.floor(xs).to(torch.int32)
    off = xs - sf                                                  # int promoted; grad flows via xs
    if interpolation == "Smoothstep":
        off = off * off * (3.0 - 2.0 * off)
    idx = corner_indices(sc, sf, log2T)
    f = [table[i] for i in idx]                                    # each [..., L, F]
    ox, oy, oz = off[..., 0:1], off[..., 1:2], off[..., 2:3]
    f03 = f[0] * ox + f[3] * (1 - ox)
    f12 = f[1] * ox + f[2] * (1 - ox)
    f56 = f[5] * ox + f[6] * (1 - ox)
    f47 = f[4] * ox + f[7] * (1 - ox)
    f0312 = f03 * oy + f12 * (1 - oy)
    f4756 = f47 * oy + f56 * (1 - oy)
    enc = f0312 * oz + f4756 * (1 - oz)
    return torch.flatten(enc, start_dim=-2, end_dim=-1)


def level_mask(num_levels: int, features: int, active_levels: int) -> torch.Tensor:
    """FeatureGrid.update_mask (feature_structures.py:85-88)."""
    m = torch.ones(num_levels * features, dtype=torch.float32)
    m[active_levels * features:] = 0
    return m


def feature_grid(x: torch.Tensor, table: torch.Tensor, scales: torch.Tensor, log2T: int, radius: float,
                 active_levels: int, interpolation: str = "Linear") -> torch.Tensor:
    """FeatureGrid.forward: rescale to [0, 1], encode, multiply by coarse-to-fine mask."""
    x_hat = (x + radius) / (2 * radius)
    feats = hash_encode(x_hat, table, scales, log2T, interpolation)
    L = scales.shape[0]
    F = table.shape[-1]
    return feats * level_mask(L, F, active_levels)


def deterministic_table(num_levels: int, log2T: int, features: int = 2) -> torch.Tensor:
    """A reproducible non-trivial table used by the full-size (log2T=19) golden vectors.

    value[i, f] = 1e-3 * sin(0.37 * i + 1.3 * f + 0.11) computed in float64 then cast, so it is
    identical in numpy, torch and on the GPU without storing 64 MiB.
    """
    n = num_levels << log2T
    i = np.arange(n, dtype=np.float64)[:, None]
    f = np.arange(features, dtype=np.float64)[None, :]
    return torch.from_numpy((1e-3 * np.sin(0.37 * i + 1.3 * f + 0.11)).astype(np.float32))
