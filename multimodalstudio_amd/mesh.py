"""Mesh extraction: the reference's coarse-to-fine SDF pyramid on the inference chain + marching cubes on the HIP
kernels, PLY export.

Mirrors MeshExtractor.extract / get_surface_sliding (/root/reference/src/evaluator_components/mesh_extractors.py:
38-79, utils/marching_cubes.py:35-188) step by step:
  * the box is cut into (resolution / 256)^3 crops of 256^3 points (np.linspace per crop: neighbouring crops share
    their boundary plane), the points cast to float16 as the reference builds them (marching_cubes.py:96);
  * per crop a 4-level point pyramid by 2x average pooling (32^3 .. 256^3, in float16 like AvgPool3d on the half
    tensor); the 32^3 level is evaluated everywhere, each finer level only where the nearest-upsampled coarser
    |sdf| < threshold (threshold = 2 * crop / 256 * 8, halved per level), other points keep the upsampled coarse
    value (marching_cubes.py:118-155);
  * crops whose values do not straddle the level are skipped; the others are triangulated by marching cubes
    (mms_mc_count / mms_mc_emit: skimage.measure.marching_cubes's role; skimage is absent offline, so the
    triangulation is parity-unpinned -- the face-ambiguity rule is Lewiner's asymptotic decider, interior ambiguities
    take the no-tunnel choice) at level 0 (the reference hard-codes level = 0: MeshExtractorConfig's
    marching_cube_threshold is not passed on, mesh_extractors.py:63-75), vertices offset by the crop minimum, welded
    within the crop (skimage returns an indexed mesh);
  * the crops are concatenated (trimesh.util.concatenate) without merging: extract() asks for return_mesh=True, and
    only the return_mesh=False path calls merge_vertices(digits_vertex=6) (marching_cubes.py:180-188);
  * optional world -> GT transform (gt_scale), ``<output>/meshes/<step:08>.ply``.
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
    """SDF values on a dense resolution^3 grid (x-major), point (i, j, k) = bbox_min + (bbox_max - bbox_min) *
    (i, j, k) / (resolution - 1) (np.linspace).  For tests and small grids; extraction uses the pyramid."""
    n = int(resolution)
    axes = [torch.tensor(np.linspace(float(bbox_min[d]), float(bbox_max[d]), n), dtype=torch.float32, device=device)
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
def marching_cubes(values: torch.Tensor, shape: Tuple[int, int, int], origin, spacing, level: float = 0.0,
                   weld: bool = True):
    """Triangulate the level set of a device grid (mms_mc_count / mms_mc_emit): (vertices [V, 3] float32, faces [F, 3]
    int64) on the device, faces facing increasing values; weld: vertices shared by neighbouring cubes merged (by the
    grid edge they lie on)."""
    nx, ny, nz = (int(x) for x in shape)
    dev = values.device
    values = values.contiguous()
    cubes = (nx - 1) * (ny - 1) * (nz - 1)
    counts = torch.empty(cubes, dtype=torch.int32, device=dev)
    _lib.call("mms_mc_count", values.data_ptr(), nx, ny, nz, float(level), counts.data_ptr(), _s())
    c64 = counts.to(torch.int64)
    offsets = torch.cumsum(c64, 0) - c64
    T = int(c64.sum())
    verts = torch.empty(max(T, 1) * 3, 3, device=dev)
    keys = torch.empty(max(T, 1) * 3, dtype=torch.int64, device=dev)
    if T > 0:
        o = (ctypes.c_float * 3)(*[float(x) for x in origin])
        sp = (ctypes.c_float * 3)(*[float(x) for x in spacing])
        _lib.call("mms_mc_emit", values.data_ptr(), nx, ny, nz, float(level), ctypes.cast(o, ctypes.c_void_p),
                  ctypes.cast(sp, ctypes.c_void_p), offsets.data_ptr(), verts.data_ptr(), keys.data_ptr(), _s())
    verts, keys = verts[:3 * T], keys[:3 * T]
    if not weld:
        return verts, torch.arange(3 * T, device=dev).view(T, 3)
    uniq, inv = torch.unique(keys, return_inverse=True)
    first = torch.full((uniq.numel(),), 3 * T, dtype=torch.int64, device=dev)
    first.scatter_reduce_(0, inv, torch.arange(3 * T, device=dev), reduce="amin")
    return verts[first], inv.view(T, 3)


CROP = 256


@torch.no_grad()
def crop_sdf_pyramid(sdf_fn, lo, hi, device, chunk: int = 1 << 21, stats: Optional[dict] = None) -> torch.Tensor:
    """One crop's SDF values [256^3] (x-major) by the reference's coarse-to-fine pyramid (marching_cubes.py:81-155)."""
    n = CROP
    axes = [torch.tensor(np.linspace(lo[d], hi[d], n), dtype=torch.float16, device=device) for d in range(3)]
    pts = torch.stack(torch.meshgrid(*axes, indexing="ij"), 0)            # [3, n, n, n] float16
    pyramid = [pts]
    for _ in range(3):
        pts = torch.nn.functional.avg_pool3d(pts[None], 2, stride=2)[0]
        pyramid.append(pts)
    pyramid = pyramid[::-1]

    def evaluate(p):
        out = torch.empty(p.shape[0], device=device)
        for s in range(0, p.shape[0], chunk):
            out[s:s + chunk] = sdf_fn(p[s:s + chunk].float().contiguous()).reshape(-1)
        if stats is not None:
            stats["evaluated"] = stats.get("evaluated", 0) + int(p.shape[0])
        return out

    mask, sdf = None, None
    threshold = 2 * (hi[0] - lo[0]) / n * 8
    for pid, p in enumerate(pyramid):
        cn = p.shape[-1]
        p = p.reshape(3, -1).permute(1, 0)
        if mask is None:
            sdf = evaluate(p)
            count = p.shape[0]
        else:
            m = mask.reshape(-1)
            count = int(m.sum())
            if count:
                sdf[m] = evaluate(p[m])
        if stats is not None:
            stats.setdefault("levels", []).append(count)      # points this pyramid level evaluated
        if pid < 3:
            mask = (torch.abs(sdf) < threshold).reshape(1, 1, cn, cn, cn)
            mask = torch.nn.functional.interpolate(mask.float(), scale_factor=2, mode="nearest").bool()
            sdf = torch.nn.functional.interpolate(sdf.reshape(1, 1, cn, cn, cn), scale_factor=2,
                                                  mode="nearest").reshape(-1)
        threshold /= 2.0
    return sdf


@torch.no_grad()
def get_surface_sliding(sdf_fn: Callable[[torch.Tensor], torch.Tensor], resolution: int = 512,
                        bounding_box_min=(-1.0, -1.0, -1.0), bounding_box_max=(1.0, 1.0, 1.0), device=None,
                        merge: bool = False, stats: Optional[dict] = None):
    """get_surface_sliding (marching_cubes.py:35-188) -> (vertices [V, 3] float32, faces [F, 3] int64) on the device.
    merge: weld the crops' shared boundary vertices as merge_vertices(digits_vertex=6) does (the return_mesh=False
    path); ``stats`` receives the number of SDF evaluations ("evaluated") and of dense points ("points")."""
    assert resolution % CROP == 0
    device = device or torch.device("cuda", torch.cuda.current_device())
    N = resolution // CROP
    grid = [np.linspace(float(bounding_box_min[d]), float(bounding_box_max[d]), N + 1) for d in range(3)]
    verts, faces, nv = [], [], 0
    for i in range(N):
        for j in range(N):
            for k in range(N):
                lo = (grid[0][i], grid[1][j], grid[2][k])
                hi = (grid[0][i + 1], grid[1][j + 1], grid[2][k + 1])
                z = crop_sdf_pyramid(sdf_fn, lo, hi, device, stats=stats)
                if stats is not None:
                    stats["points"] = stats.get("points", 0) + CROP ** 3
                if float(z.min()) > 0.0 or float(z.max()) < 0.0:
                    continue                                      # no surface in this crop
                sp = [(hi[d] - lo[d]) / (CROP - 1) for d in range(3)]
                v, f = marching_cubes(z, (CROP, CROP, CROP), lo, sp, 0.0)
                verts.append(v)
                faces.append(f + nv)
                nv += v.shape[0]
    if not verts:
        return torch.zeros(0, 3, device=device), torch.zeros(0, 3, dtype=torch.int64, device=device)
    V, F = torch.cat(verts), torch.cat(faces)
    if merge:
        key = torch.round(V.double() * 1e6).to(torch.int64)
        _, first_of, inv = _unique_rows(key)
        V, F = V[first_of], inv[F]
    return V, F


def _unique_rows(key: torch.Tensor):
    """(unique rows, index of each unique row's first occurrence, inverse) of an int64 [n, 3] tensor."""
    uniq, inv = torch.unique(key, dim=0, return_inverse=True)
    n = key.shape[0]
    first = torch.full((uniq.shape[0],), n, dtype=torch.int64, device=key.device)
    first.scatter_reduce_(0, inv, torch.arange(n, device=key.device), reduce="amin")
    return uniq, first, inv


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
    """MeshExtractorConfig (mesh_extractors.py:27-37)."""
    resolution: int = 512
    marching_cube_threshold: float = 0.0   # carried, not used: the reference's extract() never passes it on
    gt_scale: bool = True


class MeshExtractor:
    """MeshExtractor(config, scene_box aabb [2, 3], w2gt [4, 4], output_path).extract(sdf_fn, step)
    (mesh_extractors.py:38-79)."""

    def __init__(self, config: MeshExtractorConfig, aabb, w2gt, output_path: str):
        self.config = config
        self.aabb = torch.as_tensor(aabb, dtype=torch.float32)
        self.w2gt = np.asarray(w2gt, dtype=np.float64)
        self.output_path = output_path
        self.last_stats: dict = {}

    def extract(self, sdf_fn: Callable[[torch.Tensor], torch.Tensor], step: int, device=None) -> str:
        device = device or torch.device("cuda", torch.cuda.current_device())
        self.last_stats = {}
        verts, faces = get_surface_sliding(lambda x: sdf_fn(x).reshape(-1), self.config.resolution,
                                           self.aabb[0].tolist(), self.aabb[1].tolist(), device,
                                           stats=self.last_stats)
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
