"""Evaluation render path (evaluate.py) against the reference's eval-mode full-view rendering.

tests/golden/eval_grid_rgb.npz (make_golden.py:gen_eval) holds the reference BaseModel's eval-mode outputs for every
pixel of one 24 x 20 view (no jitter anywhere).  The HIP FullViewEvaluator renders the same view in chunks of 128 rays
(the chunking must not change any ray's result) and must reproduce the images (fp32 preset, 1e-4 of each tensor's
scale; normals and depth follow the same SDF as in test_gpu_e2e.py) and the PSNR computed from the reference rendering
(0.01 dB).  A smoke case runs eval_split on a small synthetic trainer.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def rel_err(actual, ref):
    a = np.asarray(actual, dtype=np.float64)
    r = np.asarray(ref, dtype=np.float64)
    s = np.abs(r).max()
    return np.abs(a - r).max() / s if s > 0 else np.abs(a - r).max()


def test_full_view_matches_reference(dev):
    from multimodalstudio_amd import evaluate as ev
    from multimodalstudio_amd import functions as fx
    from multimodalstudio_amd import model as mm
    from multimodalstudio_amd import pipeline as pl
    from multimodalstudio_amd import scene as ms
    fx.set_precision("fp32")
    f = dict(np.load(os.path.join(GOLD, "eval_grid_rgb.npz")))
    mods = [str(m) for m in f["mods"]]
    H, W = int(f["H"]), int(f["W"])
    log2T = int(np.log2(f["p:surface_model.surface_field.field.feature_grid.encoding.hash_table"].shape[0] // 16))
    model = mm.BaseModel(mm.ModelSpec({m: ms.CHANNELS[m] for m in mods}, log2T=log2T)).to(dev)
    model.load_state_dict({k[2:]: torch.from_numpy(v) for k, v in f.items() if k.startswith("p:")}, strict=True)
    model.set_step(int(f["step"]))
    cams = {m: pl.DeviceCameras(ms.ModalityCameras(
        torch.from_numpy(f[f"{m}:c2w"]), torch.from_numpy(f[f"{m}:fx"]), torch.from_numpy(f[f"{m}:fy"]),
        torch.from_numpy(f[f"{m}:cx"]), torch.from_numpy(f[f"{m}:cy"]), torch.from_numpy(f[f"{m}:distortion"]),
        W, H, []), dev) for m in mods}
    pose = pl.CameraOptimizer(mods, {m: cams[m].num for m in mods}).to(dev)
    with torch.no_grad():
        for m in mods:
            pose.pose_adjustment[m].copy_(torch.from_numpy(f[f"{m}:pose"]))
    evaluator = ev.FullViewEvaluator(model, pl.RayGenerator(cams, pose, 0.0), H, W, eval_num_rays_per_chunk=128)
    model.train()
    rend = evaluator.render_view({m: int(f["view"]) for m in mods})
    assert model.training        # restored after the eval query
    assert evaluator.last_rays_per_sec > 0
    for m in mods:
        for k in [m, "accumulation", "depth", "normals"]:
            got = rend[m][k].cpu().numpy()
            ref = f[f"{m}:out:{k}"]
            assert got.shape == ref.shape, (k, got.shape, ref.shape)
            tol = 2e-3 if k == "normals" else 1e-4
            assert rel_err(got, ref) < tol, (m, k, rel_err(got, ref))
    gt = torch.from_numpy(f["gt"]).to(dev)
    ours = evaluator.compute_metrics(rend, {mods[0]: gt})[mods[0]]["PSNR"]
    r = np.clip(f[f"{mods[0]}:out:{mods[0]}"].astype(np.float64), 0, 1)
    ref_psnr = 10 * np.log10(1.0 / np.mean((r - f["gt"].astype(np.float64)) ** 2))
    assert abs(ours - ref_psnr) < 0.01, (ours, ref_psnr)


def test_eval_split_smoke(dev):
    from multimodalstudio_amd import evaluate as ev
    from multimodalstudio_amd import functions as fx
    from multimodalstudio_amd.pipeline import TrainConfig, Trainer
    fx.set_precision("fast")
    try:
        t = Trainer(TrainConfig(method="grid_raw", modalities=("rgb", "polarization"), num_rays_per_modality=256,
                                log2T=14, width=64, height=48), dev)
        t.set_step(95000)
        t.train_step()
        scores, rate = ev.eval_split(t, n_views=1, eval_num_rays_per_chunk=1024)
    finally:
        fx.set_precision("fp32")
    assert set(scores) == {"rgb", "polarization"}
    for m, s in scores.items():
        assert np.isfinite(s) and s > 0, (m, s)
    assert rate > 0


def test_raw_eval_renderings(dev):
    """RawEvaluator's extras (evaluator.py:621-700): every head aligned to the first modality's view and mosaicked with
    each modality's pattern, degree / angle of polarization of the aligned polarization rendering, SSIM beside PSNR."""
    from multimodalstudio_amd import evaluate as ev
    from multimodalstudio_amd import scene as ms
    from multimodalstudio_amd.pipeline import DeviceCameras, RayGenerator, TrainConfig, Trainer
    t = Trainer(TrainConfig(method="grid_raw", modalities=("rgb", "polarization"), num_rays_per_modality=256,
                            log2T=14, width=48, height=40), dev)
    t.set_step(95000)
    cams = ms.make_cameras(t.modalities, 50, 48, 40, seed=0, train=False)
    dcams = {m: DeviceCameras(cams[m], dev) for m in t.modalities}
    e = ev.FullViewEvaluator(t.model, RayGenerator(dcams, t.pose, 0.0), 40, 48, 512, t.masks)
    rend = e.render_view({"rgb": 0, "polarization": 0})
    al = rend["_aligned"]
    assert al["rgb"].shape == (40, 48, 3) and al["polarization"].shape == (40, 48, 4)
    assert al["rgb:mosaicked"].shape == (40, 48, 1) and al["polarization:mosaicked"].shape == (40, 48, 1)
    # the aligned heads are the first modality's own renderings
    assert torch.equal(al["rgb"], rend["rgb"]["rgb"])
    dop, aop = al["degree_of_polarization"], al["angle_of_polarization"]
    assert dop.shape == (40, 48) and torch.isfinite(aop).all() and (aop >= 0).all() and (aop <= 1).all()
    gt = {m: ms.render_frames(ev._one_view(cams[m], 0), ms.CHANNELS[m], dev, m)[0] for m in t.modalities}
    met = e.compute_metrics(rend, gt)
    for m in t.modalities:
        assert np.isfinite(met[m]["PSNR"]) and -1.0 <= met[m]["SSIM"] <= 1.0, met
