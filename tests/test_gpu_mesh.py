"""Mesh extraction (mesh.py: dense SDF grid + marching tetrahedra on the HIP kernels).

The reference's mesh path (utils/marching_cubes.py, skimage + trimesh) is not importable offline, so the mesh is
checked against geometry instead (parity unpinned): on an analytic sphere SDF the welded mesh is a closed
2-manifold of genus 0 (every edge in exactly two faces, V - E + F = 2), its vertices lie on the sphere to the
linear-interpolation error, every triangle faces outward, and its area is 4 pi r^2 within 1 %.  The model path
exports a PLY from a geometric-init SDF field (a sphere of radius ~0.4 by construction, mlp.py:173-198).
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_sphere_iso_surface(dev):
    from multimodalstudio_amd import mesh
    n, r = 64, 0.5
    vals = mesh.sdf_grid(lambda p: p.norm(dim=-1) - r, n, [-1, -1, -1], [1, 1, 1], dev)
    h = 2.0 / (n - 1)
    V, F = mesh.iso_surface(vals, (n, n, n), [-1, -1, -1], [h, h, h])
    v = V.double().cpu().numpy()
    f = F.cpu().numpy()
    assert len(f) > 1000
    assert np.abs(np.linalg.norm(v, axis=1) - r).max() < 0.5 * h * h / r + 1e-5
    e = np.sort(np.concatenate([f[:, [0, 1]], f[:, [1, 2]], f[:, [2, 0]]]), axis=1)
    _, cnt = np.unique(e, axis=0, return_counts=True)
    assert (cnt == 2).all()
    assert len(v) - len(cnt) + len(f) == 2
    a, b, c = v[f[:, 0]], v[f[:, 1]], v[f[:, 2]]
    nrm = np.cross(b - a, c - a)
    assert ((nrm * (a + b + c)).sum(1) > 0).all()
    area = 0.5 * np.linalg.norm(nrm, axis=1).sum()
    assert abs(area / (4 * np.pi * r * r) - 1) < 0.01


def test_model_mesh_export(dev, tmp_path):
    from multimodalstudio_amd import mesh
    from multimodalstudio_amd import model as mm
    torch.manual_seed(0)
    model = mm.BaseModel(mm.ModelSpec({"rgb": 3}, log2T=14)).to(dev)
    ex = mesh.MeshExtractor(mesh.MeshExtractorConfig(resolution=64, gt_scale=True), [[-1, -1, -1], [1, 1, 1]],
                            np.diag([2.0, 2.0, 2.0, 1.0]), str(tmp_path))
    path = ex.extract(mesh.model_sdf_fn(model), step=1234)
    assert path.endswith(os.path.join("meshes", "00001234.ply"))
    with open(path, "rb") as fh:
        head = fh.read(400).split(b"end_header\n")[0].decode()
    nv = int(head.split("element vertex ")[1].split()[0])
    nf = int(head.split("element face ")[1].split()[0])
    assert nv > 100 and nf > 100
    size = os.path.getsize(path)
    assert size == len(head) + len("end_header\n") + 12 * nv + 13 * nf
