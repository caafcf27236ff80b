"""Mesh extraction: dense SDF evaluation on the inference chain + iso-surface on the HIP kernels, PLY export.

Mirrors MeshExtractor.extract / get_surface_sliding (/root/reference/src/evaluator_components/mesh_extractors.py:
30-70, utils/marching_cubes.py:35-185): an SDF grid of ``resolution`` points per axis over the scene box, the zero
level set triangulated, optional world -> GT transform (gt_scale), ``<output>/meshes/<step:08>.ply``.
MI355X-first differences (documented, parity unpinned: skimage / trimesh are absent offline):
  * the SDF is evaluated densely (fp32 points, chunks of 4M on the fused chain kernel) instead of the reference's
    fp16-point coarse-to-fine pyramid, which only evaluates near-surface points at full resolution -- near the
    surface the values are the same SDF; 512^3 points take ~0.2 s on one MI355X;
  * marching tetrahedra (mms_iso_count / mms_iso_emit) instead of skimage's Lewiner marching cubes: the same level
    set, watertight, ~2-3x more triangles; vertices welded by grid edge (trimesh merge_vertices).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Callable, Optional, Tuple

import numpy as np
import torch

from . import _lib


def _s():
    return torch.cuda.current_stream().cuda_stream


@torch.no_grad()
def sdf_grid(sdf_fn: Callable[[torch.Tensor], torch.Tensor], resolution: int, bbox_min, bbox_max, device,
             chunk: int = 1 << 22) -> torch.Tensor:
    """SDF values on a resolution^3 grid (x-major), point (i, j, k) = bbox_min + (bbox_max - bbox_min) * (i, j, k) /
    (resolution - 1) (the reference's np.linspace grid)."""
    n = int(resolution)
    lo = torch.tensor(bbox_min, dtype=torch.float64)
    hi = torch.tensor(bbox_max, dtype=torch.float64)
    axes = [torch.linspace(float(lo[d]), float(hi[d]), n, dtype=torch.float64).to(torch.float32).to(device)
            for d in range(3)]
    out = torch.empty(n * n * n, device=device)
    total = n * n * n
    for s in range(0, total, chunk):
        e = min(total, s + chunk)
        idx = torch.arange(s, e, device=device)
        k = idx % n
        j = (idx // n) % n
        i = idx // (n * n)
        pts = torch.stack([axes[0][i], axes[1][j], axes[2][k]], -1).contiguous()
        out[s:e] = sdf_fn(pts).reshape(-1)
    return out


@torch.no_grad()
def iso_surface(values: torch.Tensor, shape: Tuple[int, int, int], origin, spacing, level: float = 0.0,
                weld: bool = True):
    """Triangulate the level set of a device grid: (vertices [V, 3] float32, faces [F, 3] int64) on the device."""
    nx, ny, nz = (int(x) for x in shape)
    dev = values.device
    cells = (nx - 1) * (ny - 1) * (nz - 1)
    counts = torch.empty(cells, dtype=torch.int32, device=dev)
    _lib.call("mms_iso_count", values.data_ptr(), nx, ny, nz, float(level), counts.data_ptr(), _s())
    c64 = counts.to(torch.int64)
    offsets = torch.cumsum(c64, 0) - c64
    T = int(c64.sum())
    verts = torch.empty(max(T, 1) * 3, 3, device=dev)
    keys = torch.empty(max(T, 1) * 3, dtype=torch.int64, device=dev)
    if T > 0:
        o = (ctypes.c_float * 3)(*[float(x) for x in origin])
        sp = (ctypes.c_float * 3)(*[float(x) for x in spacing])
        _lib.call("mms_iso_emit", values.data_ptr(), nx, ny, nz, float(level), ctypes.cast(o, ctypes.c_void_p),
                  ctypes.cast(sp, ctypes.c_void_p), offsets.data_ptr(), verts.data_ptr(), keys.data_ptr(), _s())
    verts, keys = verts[:3 * T], keys[:3 * T]
    if not weld:
        return verts, torch.arange(3 * T, device=dev).view(T, 3)
    uniq, inv = torch.unique(keys, return_inverse=True)
    first = torch.full((uniq.numel(),), 3 * T, dtype=torch.int64, device=dev)
    first.scatter_reduce_(0, inv, torch.arange(3 * T, device=dev), reduce="amin")
    return verts[first], inv.view(T, 3)


def write_ply(path: str, verts: np.ndarray, faces: np.ndarray) -> None:
    """Binary little-endian PLY (float32 vertices, uchar-count int32 face lists)."""
    verts = np.ascontiguousarray(verts, dtype="<f4")
    faces = np.asarray(faces, dtype="<i4")
    header = (f"ply\nformat binary_little_endian 1.0\nelement vertex {len(verts)}\nproperty float x\n"
              f"property float y\nproperty float z\nelement face {len(faces)}\nproperty list uchar int vertex_indices\n"
              "end_header\n")
    rec = np.empty(len(faces), dtype=[("n", "u1"), ("v", "<i4", (3,))])
    rec["n"] = 3
    rec["v"] = faces
    with open(path, "wb") as f:
        f.write(header.encode("ascii"))
        f.write(verts.tobytes())
        f.write(rec.tobytes())


@dataclass
class MeshExtractorConfig:
    """MeshExtractorConfig (mesh_extractors.py:14-27)."""
    resolution: int = 512
    marching_cube_threshold: float = 0.0
    gt_scale: bool = True


class MeshExtractor:
    """MeshExtractor(config, scene_box aabb [2, 3], w2gt [4, 4], output_path).extract(sdf_fn, step)."""

    def __init__(self, config: MeshExtractorConfig, aabb, w2gt, output_path: str):
        self.config = config
        self.aabb = torch.as_tensor(aabb, dtype=torch.float32)
        self.w2gt = np.asarray(w2gt, dtype=np.float64)
        self.output_path = output_path

    def extract(self, sdf_fn: Callable[[torch.Tensor], torch.Tensor], step: int, device=None) -> str:
        device = device or torch.device("cuda", torch.cuda.current_device())
        n = self.config.resolution
        lo, hi = self.aabb[0].tolist(), self.aabb[1].tolist()
        vals = sdf_grid(sdf_fn, n, lo, hi, device)
        spacing = [(hi[d] - lo[d]) / (n - 1) for d in range(3)]
        verts, faces = iso_surface(vals, (n, n, n), lo, spacing, self.config.marching_cube_threshold)
        v = verts.double().cpu().numpy()
        if self.config.gt_scale:
            v = v @ self.w2gt[:3, :3].T + self.w2gt[:3, 3]
        out_dir = os.path.join(self.output_path, "meshes")
        os.makedirs(out_dir, exist_ok=True)
        path = os.path.join(out_dir, f"{step:08}.ply")
        write_ply(path, v.astype(np.float32), faces.cpu().numpy())
        return path


def model_sdf_fn(model) -> Callable[[torch.Tensor], torch.Tensor]:
    """The trained BaseModel's SDF (SurfaceModel.get_sdf on the inference chain), for MeshExtractor.extract."""
    return lambda x: model.surface_model.get_sdf(x)
