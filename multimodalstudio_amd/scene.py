"""Synthetic MMS-DATA-shaped scene — cameras, intrinsics, mosaick patterns, frames.

The reference loads meta_data.json + per-modality frames (src/data/datasets.py:485-529) written by
src/preprocessing/utils.py:437-571.  No real scene exists offline, so this module builds one with the
same schema-level properties:
  * views on a radius-3 sphere looking at the origin, small per-modality rig offsets;
  * W x H = 640 x 512 for every modality, pixel_offset 0.0 (preprocessing/utils.py:473);
  * distortion stored in READER order [k1, k2, k3, k4, p1, p2] (cameras/camera_utils.py:302-307);
  * raw mosaick patterns per modality (preprocess_mmsdata.py:43-47): rgb Bayer 2x2 (3 bands),
    polarization 2x2 (4), multispectral 3x3 (9), mono / infrared 1x1;
  * frames rendered analytically from an SDF scene (sphere r=0.5 + torus), values in [0, 1].
Everything is deterministic from ``seed``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch

CHANNELS = {"rgb": 3, "infrared": 1, "mono": 1, "polarization": 4, "multispectral": 9}
MOSAICK = {
    "rgb": [[0, 1], [1, 2]],
    "infrared": [[0]],
    "mono": [[0]],
    "polarization": [[0, 1], [3, 2]],
    "multispectral": [[0, 1, 2], [3, 4, 5], [6, 7, 8]],
}
EVAL_VIEWS = [9, 19, 29, 39, 49]


@dataclass
class ModalityCameras:
    c2w: torch.Tensor          # [C, 3, 4]
    fx: torch.Tensor           # [C]
    fy: torch.Tensor
    cx: torch.Tensor
    cy: torch.Tensor
    distortion: torch.Tensor   # [C, 6] reader order
    width: int
    height: int
    view_ids: List[int]        # frame index of each camera (train split)


def look_at(cam_pos: np.ndarray) -> np.ndarray:
    """OpenGL-style c2w (camera looks down -z, +y up) towards the origin."""
    fwd = -cam_pos / np.linalg.norm(cam_pos)
    z = -fwd
    world_up = np.array([0.0, 0.0, 1.0])
    x = np.cross(world_up, z)
    if np.linalg.norm(x) < 1e-6:
        x = np.array([1.0, 0.0, 0.0])
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    return np.stack([x, y, z, cam_pos], axis=1)


def make_cameras(modalities: List[str], n_views: int = 50, width: int = 640, height: int = 512,
                 seed: int = 0, train: Optional[bool] = True) -> Dict[str, ModalityCameras]:
    """Cameras of the train split (train=True), the eval split (EVAL_VIEWS, train=False) or every view (None)."""
    rng = np.random.default_rng(seed)
    views = [v for v in range(n_views) if train is None or (v not in EVAL_VIEWS) == train]
    golden = np.pi * (3.0 - np.sqrt(5.0))
    out = {}
    for mi, mod in enumerate(modalities):
        rig = rng.normal(scale=0.02, size=3)
        c2ws = []
        for v in views:
            zc = 0.15 + 0.7 * (v + 0.5) / n_views          # upper hemisphere band
            rr = np.sqrt(1 - zc * zc)
            th = golden * v
            pos = 3.0 * np.array([rr * np.cos(th), rr * np.sin(th), zc]) + rig
            c2ws.append(look_at(pos))
        C = len(views)
        f = 600.0 + 10.0 * mi
        dist = np.array([0.01, -0.005, 0.001, 0.0, 0.0005, -0.0003], dtype=np.float64)
        out[mod] = ModalityCameras(
            c2w=torch.tensor(np.stack(c2ws), dtype=torch.float32),
            fx=torch.full((C,), f), fy=torch.full((C,), f),
            cx=torch.full((C,), width / 2.0), cy=torch.full((C,), height / 2.0),
            distortion=torch.tensor(np.tile(dist, (C, 1)), dtype=torch.float32),
            width=width, height=height, view_ids=views)
    return out


def select_views(cams: ModalityCameras, view_ids: List[int]) -> ModalityCameras:
    """The cameras of the given frame ids (a dataset split / skip_image_indices_per_modality)."""
    keep = [cams.view_ids.index(v) for v in view_ids]
    t = torch.tensor(keep, dtype=torch.long)
    return ModalityCameras(cams.c2w[t], cams.fx[t], cams.fy[t], cams.cx[t], cams.cy[t], cams.distortion[t],
                           cams.width, cams.height, list(view_ids))


def mosaick_mask(mod: str, width: int, height: int) -> torch.Tensor:
    """RawDataset.build_mosaick_mask (datasets.py:229-254): tiled pattern cropped to H x W, int8."""
    pat = torch.tensor(MOSAICK[mod])
    nh, nw = -(-height // pat.shape[0]), -(-width // pat.shape[1])
    return pat.repeat((nh, nw))[:height, :width].to(torch.int8)


def analytic_radiance(origins: np.ndarray, dirs: np.ndarray, channels: int) -> np.ndarray:
    """Shade rays against a sphere (r = 0.5): hit -> normal-based colour, miss -> direction gradient."""
    b = np.sum(origins * dirs, -1)
    c = np.sum(origins * origins, -1) - 0.25
    disc = b * b - c
    hit = disc > 0
    t = -b - np.sqrt(np.maximum(disc, 0))
    p = origins + dirs * t[..., None]
    n = p / 0.5
    base = 0.5 + 0.5 * np.stack([n[..., 0], n[..., 1], n[..., 2]], -1)
    bgc = 0.5 + 0.4 * np.stack([dirs[..., 2], dirs[..., 0], dirs[..., 1]], -1)
    col3 = np.where(hit[..., None], base, bgc)
    k = np.arange(channels)
    w = 0.6 + 0.4 * np.cos(k * 0.7)
    out = (col3[..., k % 3] * w)
    return np.clip(out, 0.0, 1.0).astype(np.float32)


POL_LIGHT = (0.48, -0.36, 0.8)    # unit light direction of the polarization frames' specular highlight


def polarization_intensities(n: torch.Tensor, hit: torch.Tensor, d: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
    """Four polarizer-filtered intensities [..., 4] (0, 45, 90, 135 deg) of a Stokes field that the reference's
    PolarizationHead can represent exactly: world-frame Stokes S = s0 (1, p cos 2psi, p sin 2psi) that depend on
    the hit normal n (the direction d for misses), rotated into the camera frame by align_polarization_filters'
    angle theta = acos(clamp(normalize(d x z) . up, +-(1 - 1e-4))) - pi/2 and split by stokes_to_intensity
    (/root/reference/src/model_components/polarizer.py:54-101), so I0 + I2 = I1 + I3 = s0 as a real polarization
    camera measures (Malus).  A specular highlight pushes s0 past 1 on a small patch: those pixels clip at 1.0 and
    are what SkipSaturationLoss (losses.py:152-164) exists for."""
    L = torch.tensor(POL_LIGHT, device=d.device, dtype=d.dtype)
    L = L / L.norm()
    ndl = (n * L).sum(-1)
    s0_fg = 0.15 + 0.55 * (0.5 + 0.5 * ndl) + 1.1 * torch.clamp(ndl, min=0.0) ** 6
    p_fg = 0.1 + 0.4 * (1.0 - (n * -d).sum(-1).abs())
    psi_fg = torch.atan2(n[..., 1], n[..., 0])
    s0_bg = 0.45 + 0.35 * d[..., 2]
    psi_bg = torch.atan2(d[..., 1], d[..., 0])
    s0 = torch.where(hit, s0_fg, s0_bg)
    p = torch.where(hit, p_fg, torch.full_like(s0_bg, 0.2))
    psi = torch.where(hit, psi_fg, psi_bg)
    s1, s2 = s0 * p * torch.cos(2 * psi), s0 * p * torch.sin(2 * psi)
    zaxis = torch.zeros_like(d)
    zaxis[..., 2] = 1.0
    plane = torch.nn.functional.normalize(torch.linalg.cross(d, zaxis), dim=-1)
    cos_t = torch.clamp((plane * up).sum(-1), min=-1 + 1e-4, max=1 - 1e-4)
    theta = torch.acos(cos_t) - np.pi / 2
    c, s = torch.cos(2 * theta), torch.sin(2 * theta)
    a1, a2 = c * s1 + s * s2, -s * s1 + c * s2
    return 0.5 * torch.stack([s0 + a1, s0 + a2, s0 - a1, s0 - a2], -1)


def render_frames(cams: ModalityCameras, channels: int, device, raw_mod: Optional[str] = None) -> torch.Tensor:
    """Analytic frames [C, H, W, channels] (or mosaicked [C, H, W, 1] when raw_mod is given) on `device`.

    Data preparation only (the reference loads frames from disk into RAM, dataloaders.py:135-162); uses
    plain tensor math on the chosen device.  Four-channel (polarization) frames are polarizer intensities of a
    Stokes field (polarization_intensities); every other modality is a normal-shaded sphere with per-band gains.
    """
    H, W = cams.height, cams.width
    ys, xs = torch.meshgrid(torch.arange(H, device=device, dtype=torch.float32),
                            torch.arange(W, device=device, dtype=torch.float32), indexing="ij")
    frames = []
    k = torch.arange(channels, device=device)
    wk = 0.6 + 0.4 * torch.cos(k * 0.7)
    mm = mosaick_mask(raw_mod, W, H).to(device).long() if raw_mod is not None else None
    for c in range(cams.c2w.shape[0]):
        c2w = cams.c2w[c].to(device)
        dc = torch.stack([(xs - cams.cx[c]) / cams.fx[c], -(ys - cams.cy[c]) / cams.fy[c], -torch.ones_like(xs)], -1)
        d = torch.nn.functional.normalize(dc @ c2w[:, :3].T, dim=-1)
        o = c2w[:, 3].expand_as(d)
        b = (o * d).sum(-1)
        cc = (o * o).sum(-1) - 0.25
        disc = b * b - cc
        hit = disc > 0
        t = -b - torch.sqrt(torch.clamp(disc, min=0))
        n = (o + d * t[..., None]) / 0.5
        base = 0.5 + 0.5 * n
        bgc = 0.5 + 0.4 * torch.stack([d[..., 2], d[..., 0], d[..., 1]], -1)
        if channels == CHANNELS["polarization"]:
            up = c2w[:, 1].expand_as(d)     # R (0, 1, 0) (cameras.py:680-682)
            img = torch.clamp(polarization_intensities(n, hit, d, up), 0.0, 1.0)
        else:
            col3 = torch.where(hit[..., None], base, bgc)
            img = torch.clamp(col3[..., k % 3] * wk, 0.0, 1.0)
        if mm is not None:
            img = torch.gather(img, -1, mm[..., None])
        frames.append(img)
    return torch.stack(frames, 0)
