"""PSNR / trajectory parity: 100 training steps of the `grid` model through the HIP path,
replaying the exact inputs and uniform draws of the CPU restatement's run (tests/golden/make_train_parity.py),
then eval-ray PSNR on held-out views.  fp32 mode: |dPSNR| <= 0.1 dB and the loss trajectory within 1e-3;
the `fast` preset (bf16 / split-bf16x3 MFMA) is held to |dPSNR| <= 0.1 dB as well."""
from __future__ import annotations

import ast
import os

import numpy as np
import pytest
import torch

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "train_parity_rgb.npz")


def _rng(f, tag, m, dev, mm):
    return mm.RNG(uniform={m: torch.from_numpy(f[f"{tag}:{m}:uniform"]).to(dev)},
                  pdf={m: [t.to(dev) for t in torch.from_numpy(f[f"{tag}:{m}:pdf"])]},
                  background={m: torch.from_numpy(f[f"{tag}:{m}:bg"]).to(dev)})


def run_parity(dev, precision: str):
    from multimodalstudio_amd import functions as fx
    from multimodalstudio_amd import model as mm
    from multimodalstudio_amd import pipeline as pl
    from multimodalstudio_amd import scene as ms
    f = np.load(GOLD)
    cfg = ast.literal_eval(f["cfg_json"].tobytes().decode())
    fx.set_precision(precision)
    try:
        tc = pl.TrainConfig(method=cfg["method"], modalities=tuple(cfg["modalities"]),
                            num_rays_per_modality=cfg["rays"], log2T=cfg["log2T"], width=cfg["width"],
                            height=cfg["height"], n_views=cfg["n_views"])
        tr = pl.Trainer(tc, dev)
        ck = float(sum(float(v.detach().double().abs().sum()) for v in tr.model.state_dict().values()))
        assert ck == pytest.approx(float(f["init_checksum"]), rel=1e-9), "model init drifted from the fixture"
        tr.set_step(cfg["start_step"])
        tr.fields.step_count = 0          # fresh optimizer state, as the oracle run
        if tr.poses is not None:
            tr.poses.step_count = 0
        mods = list(cfg["modalities"])
        losses = []
        for k in range(cfg["steps"]):
            coords = {m: torch.from_numpy(f[f"s{k}:{m}:coords"]) for m in mods}
            targets = {m: torch.from_numpy(f[f"s{k}:{m}:targets"]) for m in mods}
            rng = mm.RNG({}, {}, {})
            for m in mods:
                r = _rng(f, f"s{k}", m, dev, mm)
                rng.uniform.update(r.uniform), rng.pdf.update(r.pdf), rng.background.update(r.background)
            _, total, _ = tr.train_step(coords, targets, rng)
            losses.append(float(total))
        # eval: held-out views, zero pose delta, no grad
        ecams = ms.make_cameras(mods, cfg["n_views"], cfg["width"], cfg["height"], seed=0, train=False)
        dcams = {m: pl.DeviceCameras(ecams[m], dev) for m in mods}
        gen = pl.RayGenerator(dcams, pl.CameraOptimizer(mods, {m: dcams[m].num for m in mods}, mode="off"), 0.0)
        tr.model.set_step(tr.step, tc.max_iters)
        psnr = {}
        preds = {}
        with torch.no_grad():
            for m in mods:
                coords = {m: torch.from_numpy(f[f"eval:{m}:coords"]).to(dev)}
                outs = tr.model(gen(coords), _rng(f, "eval", m, dev, mm))
                pred = outs[m][m].float().cpu()
                tgt = torch.from_numpy(f[f"eval:{m}:targets"])
                psnr[m] = -10.0 * float(np.log10(float(((pred - tgt) ** 2).mean())))
                preds[m] = pred.numpy()
        return f, cfg, np.array(losses), psnr, preds
    finally:
        fx.set_precision("fp32")


@pytest.mark.gpu
def test_train_parity_fp32(dev):
    f, cfg, losses, psnr, preds = run_parity(dev, "fp32")
    ref = np.array([float(f[f"s{k}:loss"]) for k in range(cfg["steps"])])
    rel = np.abs(losses - ref) / np.abs(ref)
    k = int(rel.argmax())
    print("fp32 per-step loss (hip, oracle):", [(i, round(float(losses[i]), 6), round(float(ref[i]), 6))
                                                 for i in range(min(6, len(ref)))], "worst", k, losses[k], ref[k])
    print(f"fp32: max loss rel err {rel.max():.2e}; PSNR {psnr} vs oracle "
          f"{ {m: float(f[f'eval:{m}:psnr']) for m in cfg['modalities']} }")
    assert rel.max() < 1e-3
    for m in cfg["modalities"]:
        assert abs(psnr[m] - float(f[f"eval:{m}:psnr"])) <= 0.1
        err = np.abs(preds[m] - f[f"eval:{m}:pred"]).max()
        assert err < 1e-2, f"eval prediction max abs err {err}"


@pytest.mark.gpu
def test_train_parity_fast_preset(dev):
    f, cfg, losses, psnr, _ = run_parity(dev, "fast")
    ref = np.array([float(f[f"s{k}:loss"]) for k in range(cfg["steps"])])
    print(f"fast: loss rel err mean {np.mean(np.abs(losses - ref) / ref):.2e}; PSNR {psnr} vs oracle "
          f"{ {m: float(f[f'eval:{m}:psnr']) for m in cfg['modalities']} }")
    for m in cfg["modalities"]:
        assert abs(psnr[m] - float(f[f"eval:{m}:psnr"])) <= 0.1
