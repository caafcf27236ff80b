"""ORACLE (test infrastructure only) — encodings, weight-normed MLPs, heads, polarizer, fields.

Restates (paths under /root/reference/src):
  NeRFEncoding.forward               field_components/encodings.py:161-182
  components_from_spherical_harmonics utils/math.py:21-83  (SHEncoding, encodings.py:368-392)
  MLP.forward / weight_norm          field_components/mlp.py:152-171, 206-209
  SDFField.forward                   fields/surface_field.py:99-116
  FeatureGridAndMLP.forward          field_components/feature_structures.py:153-169
  RadianceField.forward              fields/radiance_field.py:72-77
  ModalityHead / PolarizationHead    field_components/field_heads.py:71-106
  align_polarization_filters         model_components/polarizer.py:54-82
  stokes_to_intensity                model_components/polarizer.py:84-101
  NeRFField.forward                  fields/nerf_field.py:92-105
  SceneContraction.forward           field_components/spatial_distortions.py:90-97
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from . import hashgrid as ohg


# ------------------------------------------------------------------------------------------------
# encodings
# ------------------------------------------------------------------------------------------------
def nerf_encoding(x: torch.Tensor, num_frequencies: int, min_freq: float, max_freq: float,
                  include_input: bool = True) -> torch.Tensor:
    """encodings.py:161-182 — [x, sin(x_i 2^k) (i-major), sin(x_i 2^k + pi/2)]."""
    freqs = 2 ** torch.linspace(min_freq, max_freq, num_frequencies)
    scaled = x[..., None] * freqs
    scaled = scaled.view(*scaled.shape[:-2], -1)
    enc = torch.sin(torch.cat([scaled, scaled + torch.pi / 2.0], dim=-1))
    if include_input:
        enc = torch.cat([x, enc], dim=-1)
    return enc


SH_C = {
    "c0": 0.28209479177387814, "c1": 0.4886025119029199, "c2a": 1.0925484305920792,
    "c2b": 0.9461746957575601, "c2c": 0.31539156525251999, "c2d": 0.5462742152960396,
    "c3a": 0.5900435899266435, "c3b": 2.890611442640554, "c3c": 0.4570457994644658,
    "c3d": 0.3731763325901154, "c3e": 1.445305721320277, "c4a": 2.5033429417967046,
    "c4b": 1.7701307697799304, "c4c": 0.9461746957575601, "c4d": 0.6690465435572892,
    "c4e": 0.10578554691520431, "c4f": 0.47308734787878004, "c4g": 0.4425326924449826,
}


def sh_encoding(d: torch.Tensor, levels: int = 5) -> torch.Tensor:
    """utils/math.py:21-83 with levels = degree + 1 (SURVEY §8(c) patch (2))."""
    x, y, z = d[..., 0], d[..., 1], d[..., 2]
    xx, yy, zz = x ** 2, y ** 2, z ** 2
    c = SH_C
    comps = [torch.full_like(x, c["c0"])]
    if levels > 1:
        comps += [c["c1"] * y, c["c1"] * z, c["c1"] * x]
    if levels > 2:
        comps += [c["c2a"] * x * y, c["c2a"] * y * z, c["c2b"] * zz - c["c2c"], c["c2a"] * x * z,
                  c["c2d"] * (xx - yy)]
    if levels > 3:
        comps += [c["c3a"] * y * (3 * xx - yy), c["c3b"] * x * y * z, c["c3c"] * y * (5 * zz - 1),
                  c["c3d"] * z * (5 * zz - 3), c["c3c"] * x * (5 * zz - 1), c["c3e"] * z * (xx - yy),
                  c["c3a"] * x * (xx - 3 * yy)]
    if levels > 4:
        comps += [c["c4a"] * x * y * (xx - yy), c["c4b"] * y * z * (3 * xx - yy), c["c4c"] * x * y * (7 * zz - 1),
                  c["c4d"] * y * (7 * zz - 3), c["c4e"] * (35 * zz * zz - 30 * zz + 3),
                  c["c4d"] * x * z * (7 * zz - 3), c["c4f"] * (xx - yy) * (7 * zz - 1),
                  c["c4b"] * x * z * (xx - 3 * yy), c["c4g"] * (xx * (xx - 3 * yy) - yy * (3 * xx - yy))]
    return torch.stack(comps, dim=-1)


# ------------------------------------------------------------------------------------------------
# MLP with weight norm
# ------------------------------------------------------------------------------------------------
def wn_weight(g: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    """torch weight_norm(dim=0): w = v * (g / ||v||_row)  (mlp.py:206-209).

    Uses the same ATen primitive the reference's parametrization calls (torch._weight_norm), so the
    effective weights are bit-identical to the reference's.
    """
    return torch._weight_norm(v, g, 0)


def activation(name: Optional[str], x: torch.Tensor, params: Optional[dict] = None) -> torch.Tensor:
    params = params or {}
    if name in (None, "None"):
        return x
    if name == "ReLU":
        return F.relu(x)
    if name == "Softplus":
        return F.softplus(x, beta=params.get("beta", 1.0), threshold=params.get("threshold", 20.0))
    if name == "Sigmoid":
        return torch.sigmoid(x)
    raise ValueError(name)


def mlp_forward(x: torch.Tensor, P: Dict[str, torch.Tensor], prefix: str, num_layers: int, act: str,
                act_params: Optional[dict], out_act: Optional[str], skips: Sequence[int] = ()) -> torch.Tensor:
    """MLP.forward (mlp.py:152-171) for weight-normed layers named like the reference state_dict."""
    inp = x
    for i in range(num_layers):
        if i in skips:
            x = torch.cat([x, inp], -1) / np.sqrt(2)
        base = f"{prefix}.layers.{i}"
        w = wn_weight(P[base + ".parametrizations.weight.original0"], P[base + ".parametrizations.weight.original1"])
        x = F.linear(x, w, P[base + ".bias"])
        if i < num_layers - 1:
            x = activation(act, x, act_params)
    return activation(out_act, x)


# ------------------------------------------------------------------------------------------------
# grid + MLP fields
# ------------------------------------------------------------------------------------------------
class GridSpec:
    def __init__(self, num_levels=16, min_res=16, max_res=1024, log2T=19, radius=1.0, features=2):
        self.num_levels, self.min_res, self.max_res = num_levels, min_res, max_res
        self.log2T, self.radius, self.features = log2T, radius, features
        self.scales = ohg.level_scales(min_res, max_res, num_levels)


def feature_grid_and_mlp(x: torch.Tensor, P, prefix: str, grid: GridSpec, active_levels: int, mlp_kw: dict):
    """FeatureGridAndMLP.forward: [x, aux, grid(x)] -> MLP (feature_structures.py:153-169)."""
    aux = x[..., 3:] if x.shape[-1] > 3 else None
    pos = x[..., :3]
    feats = ohg.feature_grid(pos, P[prefix + ".feature_grid.encoding.hash_table"], grid.scales, grid.log2T,
                             grid.radius, active_levels)
    mlp_in = torch.cat([pos, aux, feats], -1) if aux is not None else torch.cat([pos, feats], -1)
    return mlp_forward(mlp_in, P, prefix + ".mlp_head", **mlp_kw)


SDF_MLP = dict(num_layers=3, act="Softplus", act_params={"beta": 100}, out_act=None)
RAD_MLP = dict(num_layers=3, act="ReLU", act_params=None, out_act="ReLU")


def sdf_field(x: torch.Tensor, P, grid: GridSpec, active_levels: int, prefix="surface_model.surface_field"):
    """SDFField.forward (surface_field.py:99-116): PE(6 freqs) -> FeatureGridAndMLP -> split [1, 256]."""
    pe = nerf_encoding(x, 6, 0.0, 5.0, True)
    out = feature_grid_and_mlp(pe, P, prefix + ".field", grid, active_levels, SDF_MLP)
    return out[..., :1], out[..., 1:]


def radiance_field(pos, sh, additional, P, grid: GridSpec, active_levels: int,
                   prefix="radiance_model.radiance_field.base_field"):
    """RadianceField.forward (radiance_field.py:72-77) -> FeatureGridAndMLP 317 -> 256."""
    inp = torch.cat([pos, sh, additional], -1)
    return feature_grid_and_mlp(inp, P, prefix, grid, active_levels, RAD_MLP)


# the mlp / mlp_raw methods' fields (method_configs.py:303-353): 8-layer, 256-wide MLPs with a skip into layer 4
SDF_MLP8 = dict(num_layers=8, act="Softplus", act_params={"beta": 100}, out_act=None, skips=(4,))
RAD_MLP8 = dict(num_layers=8, act="ReLU", act_params=None, out_act="ReLU", skips=(4,))


def sdf_field_mlp(x: torch.Tensor, P, prefix="surface_model.surface_field"):
    """SDFField.forward (surface_field.py:99-116) with an MLP field: PE(6 freqs, input included) -> MLP -> [1, 256]."""
    out = mlp_forward(nerf_encoding(x, 6, 0.0, 5.0, True), P, prefix + ".field", **SDF_MLP8)
    return out[..., :1], out[..., 1:]


def radiance_field_mlp(pos, sh, additional, P, prefix="radiance_model.radiance_field.base_field"):
    """RadianceField.forward (radiance_field.py:72-77) with an MLP base field on [x, SH, geo, n.v] (285 -> 256)."""
    return mlp_forward(torch.cat([pos, sh, additional], -1), P, prefix, **RAD_MLP8)


# ------------------------------------------------------------------------------------------------
# heads and polarizer
# ------------------------------------------------------------------------------------------------
def align_polarization_filters(stokes, directions, up):
    """polarizer.py:54-82."""
    z = torch.tensor([0.0, 0.0, 1.0], dtype=directions.dtype)[None, ...].expand(directions.shape)
    n = F.normalize(torch.linalg.cross(directions, z), dim=-1)
    cos_t = torch.clamp(torch.sum(n * up, dim=-1), min=-1 + 1e-4, max=1 - 1e-4)
    theta = torch.acos(cos_t) - np.pi / 2
    c = torch.cos(2 * theta)
    s = torch.sin(2 * theta)
    one, zero = torch.ones_like(c), torch.zeros_like(c)
    rot = torch.stack([one, zero, zero, zero, c, s, zero, -s, c], dim=-1).view(-1, 3, 3)
    return (rot @ stokes[..., None]).squeeze()


def stokes_to_intensity(stokes):
    """polarizer.py:84-101 (returns the 4 polarised channels)."""
    m = 0.5 * torch.tensor([[1., 1., 0.], [1., 0., 1.], [1., -1., 0.], [1., 0., -1.]], dtype=stokes.dtype)
    return (m[None, ...] @ stokes[..., None]).squeeze()


def modality_head(x, P, prefix, kind: str, num_layers: int, directions=None, up=None):
    """ModalityHead.forward / PolarizationHead.forward (field_heads.py:71-106)."""
    if kind == "polarization":
        stokes = mlp_forward(x, P, prefix + ".field", num_layers, "ReLU", None, None)
        stokes = stokes.clone()
        stokes[..., 0] = F.leaky_relu(stokes[..., 0].clone())
        aligned = align_polarization_filters(stokes, directions, up)
        return stokes_to_intensity(aligned)
    return mlp_forward(x, P, prefix + ".field", num_layers, "ReLU", None, "Sigmoid")


# ------------------------------------------------------------------------------------------------
# background NeRF field
# ------------------------------------------------------------------------------------------------
def scene_contraction_linf(x: torch.Tensor) -> torch.Tensor:
    """SceneContraction(order=inf).forward (spatial_distortions.py:90-97)."""
    mag = torch.linalg.norm(x, ord=float("inf"), dim=-1)
    mask = mag >= 1
    out = x.clone()
    out[mask] = (2 - (1 / mag[mask][..., None])) * (x[mask] / mag[mask][..., None])
    return out


# the config-5 background base field (method_configs.py:430-441): FeatureGridAndMLP, hash grid r = 2, MLP 71-128-128-256
BG_GRID_MLP = dict(num_layers=3, act="ReLU", act_params=None, out_act="ReLU")


def nerf_field(x, d, P, prefix="background_model.background_field", base_layers=4, head_layers=4,
               grid: "GridSpec" = None, active_levels: int = 16):
    """NeRFField.forward (nerf_field.py:92-105) for the 'grid' method background (method_configs.py:187-212); with
    ``grid`` the base field is 'grid_raw_grid_bg_unbalanced''s FeatureGridAndMLP on the PE of the contracted position
    (method_configs.py:428-445; feature_structures.py:153-169 splits x = PE[:3] off for the grid)."""
    xe = nerf_encoding(x, 6, 0.0, 5.0, True)
    de = nerf_encoding(d, 4, 0.0, 3.0, True)
    if grid is not None:
        feat = feature_grid_and_mlp(xe, P, prefix + ".base_field", grid, active_levels, BG_GRID_MLP)
    else:
        feat = mlp_forward(xe, P, prefix + ".base_field", base_layers, "ReLU", None, "ReLU")
    density = mlp_forward(feat, P, prefix + ".density_head.field", 1, "ReLU", None, "Softplus")
    head = mlp_forward(torch.cat([feat, de], -1), P, prefix + ".head_field", head_layers, "ReLU", None, "ReLU")
    return density, head
