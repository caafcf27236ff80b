"""Mesh extraction (mesh.py: the reference's coarse-to-fine SDF pyramid + marching cubes on the HIP kernels).

The reference's mesh path (utils/marching_cubes.py: skimage's marching cubes + trimesh) is not importable offline, so
the mesh is checked against geometry (parity unpinned): on analytic sphere and torus SDFs the welded mesh
is a closed 2-manifold (every edge in exactly two faces) of the right genus (V - E + F = 2 and 0), its vertices lie
on the surface to the linear-interpolation error, every triangle faces outward, its area matches, and its triangle
count is marching cubes' (about 2 triangles per surface cube, half of marching tetrahedra's).  The pyramid evaluates
only the near-surface points at full resolution.  The model path exports a PLY from a geometric-init SDF field (a
sphere of radius ~0.4 by construction, mlp.py:173-198).
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def sphere(r):
    return lambda p: p.norm(dim=-1) - r


def torus(R, r):
    return lambda p: torch.sqrt((torch.sqrt(p[:, 0] ** 2 + p[:, 1] ** 2) - R) ** 2 + p[:, 2] ** 2) - r


def _check_closed(v, f, euler):
    e = np.sort(np.concatenate([f[:, [0, 1]], f[:, [1, 2]], f[:, [2, 0]]]), axis=1)
    _, cnt = np.unique(e, axis=0, return_counts=True)
    assert (cnt == 2).all(), np.bincount(cnt)
    assert len(v) - len(cnt) + len(f) == euler


@pytest.mark.parametrize("shape", ["sphere", "torus"])
def test_marching_cubes_analytic(dev, shape):
    from multimodalstudio_amd import mesh
    n = 96
    fn = sphere(0.5) if shape == "sphere" else torus(0.5, 0.2)
    vals = mesh.sdf_grid(fn, n, [-1, -1, -1], [1, 1, 1], dev)
    h = 2.0 / (n - 1)
    V, F = mesh.marching_cubes(vals, (n, n, n), [-1, -1, -1], [h, h, h])
    v = V.double().cpu().numpy()
    f = F.cpu().numpy()
    _check_closed(v, f, 2 if shape == "sphere" else 0)
    sdf = fn(torch.from_numpy(v)).numpy()
    assert np.abs(sdf).max() < 0.5 * h * h / 0.2 + 1e-5          # linear interpolation of a curved surface
    a, b, c = v[f[:, 0]], v[f[:, 1]], v[f[:, 2]]
    nrm = np.cross(b - a, c - a)
    cen = torch.from_numpy((a + b + c) / 3).requires_grad_(True)
    fn(cen).sum().backward()
    assert ((nrm * cen.grad.numpy()).sum(1) > 0).all()         # outward: along the SDF gradient
    area = 0.5 * np.linalg.norm(nrm, axis=1).sum()
    ref = 4 * np.pi * 0.25 if shape == "sphere" else 4 * np.pi ** 2 * 0.5 * 0.2
    assert abs(area / ref - 1) < 0.01
    # marching cubes' triangle density: ~2 triangles per surface cube (tetrahedra gave 2-3x more)
    cubes = int(((vals.view(n, n, n) < 0).float().unfold(0, 2, 1).unfold(1, 2, 1).unfold(2, 2, 1)
                 .reshape(n - 1, n - 1, n - 1, 8).sum(-1).remainder(8) != 0).sum())
    assert 1.5 * cubes <= len(f) <= 2.5 * cubes, (len(f), cubes)


def test_pyramid_extraction_evaluates_near_surface_only(dev):
    """get_surface_sliding at resolution 512 (8 crops of 256^3): far fewer SDF evaluations than 512^3, and the same
    surface as the dense grid -- the merged mesh is closed and on the sphere."""
    from multimodalstudio_amd import mesh
    r = 0.6
    stats = {}
    V, F = mesh.get_surface_sliding(sphere(r), 512, (-1, -1, -1), (1, 1, 1), dev, merge=True, stats=stats)
    assert stats["points"] == 512 ** 3
    assert stats["evaluated"] < 0.1 * 512 ** 3, stats
    v = V.double().cpu().numpy()
    f = F.cpu().numpy()
    h = 2.0 / 511
    assert np.abs(np.linalg.norm(v, axis=1) - r).max() < 1e-3 + 0.5 * h * h / r
    _check_closed(v, f, 2)
    # without the merge (MeshExtractor.extract's return_mesh path) the crops' boundary vertices stay duplicated
    V2, F2 = mesh.get_surface_sliding(sphere(r), 512, (-1, -1, -1), (1, 1, 1), dev)
    assert F2.shape == F.shape and V2.shape[0] > V.shape[0]


def test_model_mesh_export(dev, tmp_path):
    from multimodalstudio_amd import mesh
    from multimodalstudio_amd import model as mm
    torch.manual_seed(0)
    model = mm.BaseModel(mm.ModelSpec({"rgb": 3}, log2T=14)).to(dev)
    ex = mesh.MeshExtractor(mesh.MeshExtractorConfig(resolution=256, gt_scale=True), [[-1, -1, -1], [1, 1, 1]],
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
    assert ex.last_stats["evaluated"] < 0.25 * 256 ** 3


def _fixture_sdf(p):
    """tests/golden/make_golden.py analytic_sdf (sphere united with a torus), the same float32 expression."""
    p = p.float()
    c = torch.tensor([0.1, -0.05, 0.2], dtype=torch.float32, device=p.device)
    sph = torch.sqrt(((p - c) ** 2).sum(-1)) - 0.45
    q = torch.sqrt(p[:, 0] ** 2 + p[:, 1] ** 2) - 0.6
    tor = torch.sqrt(q ** 2 + p[:, 2] ** 2) - 0.12
    return torch.minimum(sph, tor)


def test_pyramid_matches_reference_crops(dev):
    """The coarse-to-fine SDF pyramid of every 256^3 crop against the reference's get_surface_sliding run on the same
    analytic SDF (tests/golden/mesh_pyramid.npz, marching_cubes.py:35-171 with skimage's marching_cubes intercepted):
    the points each pyramid level evaluates (the |sdf| < threshold masks, level by level) and the final volume handed
    to marching cubes (sign census, sum, a fixed sample of entries).  The triangulation itself stays unpinned."""
    from multimodalstudio_amd import mesh
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mesh_pyramid.npz")
    f = np.load(path)
    res = int(f["resolution"])
    n = res // mesh.CROP
    grid = [np.linspace(-1.0, 1.0, n + 1) for _ in range(3)]
    idx = torch.from_numpy(f["sample_index"]).to(dev)
    ci = 0
    for i in range(n):
        for j in range(n):
            for k in range(n):
                lo = (grid[0][i], grid[1][j], grid[2][k])
                hi = (grid[0][i + 1], grid[1][j + 1], grid[2][k + 1])
                stats = {}
                z = mesh.crop_sdf_pyramid(_fixture_sdf, lo, hi, dev, stats=stats)
                ref_levels = f["level_counts"][ci].tolist()
                # masks from |sdf| < threshold: a point within float rounding of a threshold may flip; none did here
                assert stats["levels"] == ref_levels, (ci, stats["levels"], ref_levels)
                if ci in set(f["surface_crops"].tolist()):
                    zc = z.double()
                    assert int((z < 0).sum()) == int(f[f"crop{ci}:neg"]), ci
                    assert abs(float(zc.sum()) - float(f[f"crop{ci}:sum"])) <= 1e-6 * float(zc.abs().sum()), ci
                    got = z[idx].cpu().numpy()
                    np.testing.assert_allclose(got, f[f"crop{ci}:sample"], rtol=3e-7, atol=3e-7,
                                               err_msg=f"crop {ci}")   # sqrt to 1 ulp (4 of 65536 entries)
                ci += 1
