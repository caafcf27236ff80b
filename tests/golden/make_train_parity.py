#!/usr/bin/env python
"""Training-trajectory fixture for the PSNR-parity test (SURVEY §8(d) 'PSNR parity').

The CPU restatement (oracle/, pinned bit-exact to the reference by tests/test_oracle_golden.py) trains
the `grid` model on the synthetic scene from a seeded init for K steps; every input of every step
(pixel coords, targets, the sampler/background uniform draws) and the oracle's per-step losses are
stored, plus the eval-ray predictions and PSNR after training.  tests/test_gpu_train_parity.py replays
the same K steps through the HIP path and compares.

    python tests/golden/make_train_parity.py        (CPU, ~1 min on 8 threads; writes tests/golden/train_parity_rgb.npz)
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

CFG = dict(method="grid", modalities=("rgb",), rays=256, log2T=12, width=160, height=128, n_views=10,
           start_step=20000, steps=100, eval_rays=1024, init_seed=654824, sampler_seed=654824, rng_seed=11,
           eval_seed=5)


def param_checksum(sd):
    return float(sum(float(v.double().abs().sum()) for v in sd.values()))


def main():
    from multimodalstudio_amd import scene as ms
    from multimodalstudio_amd.model import BaseModel, ModelSpec
    from multimodalstudio_amd.pipeline import UniformPixelSampler
    from oracle import model as om
    from oracle import rays as orr
    from oracle.train import OracleTrainer

    torch.set_num_threads(min(8, os.cpu_count() or 1))
    mods = list(CFG["modalities"])
    channels = {m: ms.CHANNELS[m] for m in mods}
    torch.manual_seed(CFG["init_seed"])
    model = BaseModel(ModelSpec(channels, log2T=CFG["log2T"]))
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    cams = ms.make_cameras(mods, CFG["n_views"], CFG["width"], CFG["height"], seed=0, train=True)
    ecams = ms.make_cameras(mods, CFG["n_views"], CFG["width"], CFG["height"], seed=0, train=False)
    images = {m: ms.render_frames(cams[m], channels[m], torch.device("cpu")) for m in mods}
    eimages = {m: ms.render_frames(ecams[m], channels[m], torch.device("cpu")) for m in mods}
    frames = {m: {"shape": (cams[m].c2w.shape[0], CFG["height"], CFG["width"]),
                  "indexes": torch.arange(cams[m].c2w.shape[0], dtype=torch.int32)} for m in mods}
    sampler = UniformPixelSampler(CFG["rays"], CFG["sampler_seed"])
    ot = OracleTrainer(sd, channels, cams, CFG["log2T"], CFG["start_step"], raw=False)
    gen = torch.Generator().manual_seed(CFG["rng_seed"])
    rec = {}

    def rng_hook(n_hit, n_rays):
        uni = {m: torch.rand(n_hit[m], 1, generator=gen) for m in mods}
        pdf = {m: [torch.rand(n_hit[m], 1, generator=gen) for _ in range(4)] for m in mods}
        bg = {m: torch.rand(n_rays[m], ot.spec.bg_samples + 1, generator=gen) for m in mods}
        rec["rng"] = (uni, pdf, bg)
        return om.RNG(uni, pdf, bg)

    ot.rng = rng_hook
    out = {"cfg_json": np.frombuffer(repr(CFG).encode(), dtype=np.uint8), "init_checksum": param_checksum(sd)}
    # eval on held-out view rays (pose delta zero: the field is evaluated, not the pose)
    def evaluate(tag):
        eg = torch.Generator().manual_seed(CFG["eval_seed"])
        st = om.StepState(step=ot.step)
        for m in mods:
            c = ecams[m]
            n = CFG["eval_rays"]
            ci = torch.randint(0, c.c2w.shape[0], (n, 1), generator=eg, dtype=torch.int32)
            px = torch.randint(0, CFG["width"], (n, 1), generator=eg, dtype=torch.int32)
            py = torch.randint(0, CFG["height"], (n, 1), generator=eg, dtype=torch.int32)
            coords = torch.cat([ci, py, px], -1)
            tgt = eimages[m][ci[:, 0].long(), py[:, 0].long(), px[:, 0].long()]
            rays = {m: orr.generate_rays(coords, c.fx, c.fy, c.cx, c.cy, c.c2w, c.distortion, torch.zeros(1, 6), 0.0)}
            with torch.no_grad():
                hit = int(orr.sphere_collider(rays[m].origins, rays[m].directions)[2].sum())
                uni = {m: torch.rand(hit, 1, generator=eg)}
                pdf = {m: [torch.rand(hit, 1, generator=eg) for _ in range(4)]}
                bg = {m: torch.rand(n, ot.spec.bg_samples + 1, generator=eg)}
                outs = om.model_forward(rays, ot.P, ot.spec, st, om.RNG(uni, pdf, bg))
            pred = outs[m][m]
            mse = float(((pred - tgt) ** 2).mean())
            psnr = -10.0 * np.log10(mse)
            print(f"{tag} {m}: PSNR {psnr:.4f} dB", flush=True)
            out[f"{tag}:{m}:coords"] = coords.numpy()
            out[f"{tag}:{m}:targets"] = tgt.numpy()
            out[f"{tag}:{m}:uniform"] = uni[m].numpy()
            out[f"{tag}:{m}:pdf"] = torch.stack(pdf[m]).numpy()
            out[f"{tag}:{m}:bg"] = bg[m].numpy()
            out[f"{tag}:{m}:pred"] = pred.numpy()
            out[f"{tag}:{m}:psnr"] = np.float64(psnr)

    evaluate("eval0")
    t0 = time.time()
    for k in range(CFG["steps"]):
        coords, sel = sampler.sample(frames)
        targets = {m: images[m][sel[m].long(), coords[m][:, 1].long(), coords[m][:, 2].long()] for m in mods}
        loss = ot.train_step(coords, targets)
        uni, pdf, bg = rec["rng"]
        for m in mods:
            out[f"s{k}:{m}:coords"] = coords[m].numpy()
            out[f"s{k}:{m}:targets"] = targets[m].numpy()
            out[f"s{k}:{m}:uniform"] = uni[m].numpy()
            out[f"s{k}:{m}:pdf"] = torch.stack(pdf[m]).numpy()
            out[f"s{k}:{m}:bg"] = bg[m].numpy()
        out[f"s{k}:loss"] = np.float64(loss)
        print(f"step {k}: loss {loss:.6f} ({time.time() - t0:.1f}s)", flush=True)
    evaluate("eval")
    # untrained PSNR for scale (how far training moved the field)
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "train_parity_rgb.npz"), **out)


if __name__ == "__main__":
    main()
