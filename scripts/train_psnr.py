#!/usr/bin/env python
"""Train the `grid` model on the synthetic scene through the HIP path and report held-out PSNR every
--every steps (diagnostics for the PSNR-parity test: how fast PSNR plateaus, and the run-to-run spread that
float-atomic reduction order alone produces).

    python scripts/train_psnr.py [--steps 1000] [--every 100] [--precision fp32] [--start-step 20000] [--runs 2]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--every", type=int, default=100)
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--start-step", type=int, default=20000)
    ap.add_argument("--rays", type=int, default=256)
    ap.add_argument("--runs", type=int, default=2)
    a = ap.parse_args()
    from multimodalstudio_amd import functions as fx
    from multimodalstudio_amd import model as mm
    from multimodalstudio_amd import pipeline as pl
    from multimodalstudio_amd import scene as ms
    dev = torch.device("cuda", 0)
    fx.set_precision(a.precision)
    mods = ["rgb"]
    W, H, V = 160, 128, 10
    ecams = ms.make_cameras(mods, V, W, H, seed=0, train=False)
    eimg = ms.render_frames(ecams["rgb"], 3, dev)
    dcams = {m: pl.DeviceCameras(ecams[m], dev) for m in mods}
    gen = pl.RayGenerator(dcams, pl.CameraOptimizer(mods, {m: dcams[m].num for m in mods}, mode="off"), 0.0)
    eg = torch.Generator().manual_seed(5)
    n = 4096
    ci = torch.randint(0, ecams["rgb"].c2w.shape[0], (n, 1), generator=eg, dtype=torch.int32)
    px = torch.randint(0, W, (n, 1), generator=eg, dtype=torch.int32)
    py = torch.randint(0, H, (n, 1), generator=eg, dtype=torch.int32)
    coords = torch.cat([ci, py, px], -1).to(dev)
    tgt = eimg[ci[:, 0].long().to(dev), py[:, 0].long().to(dev), px[:, 0].long().to(dev)]
    for run in range(a.runs):
        tc = pl.TrainConfig(method="grid", modalities=tuple(mods), num_rays_per_modality=a.rays, log2T=12, width=W,
                            height=H, n_views=V)
        tr = pl.Trainer(tc, dev)
        tr.set_step(a.start_step)
        tr.fields.step_count = 0
        if tr.poses is not None:
            tr.poses.step_count = 0
        hist = []
        for k in range(1, a.steps + 1):
            tr.train_step()
            if k % a.every == 0:
                tr.model.set_step(tr.step, tc.max_iters)
                with torch.no_grad():
                    g = torch.Generator(device="cpu").manual_seed(9)
                    rng = mm.RNG({"rgb": torch.rand(n, 1, generator=g).to(dev)},
                                 {"rgb": [torch.rand(n, 1, generator=g).to(dev) for _ in range(4)]},
                                 {"rgb": torch.rand(n, 17, generator=g).to(dev)})
                    # the model compacts to hit rays: pass full-length draws, it slices what it needs
                    out = tr.model(gen({"rgb": coords}), rng)["rgb"]["rgb"]
                psnr = -10 * float(np.log10(float(((out - tgt) ** 2).mean())))
                hist.append((k, round(psnr, 3)))
        print(f"run {run} ({a.precision}): " + " ".join(f"{k}:{p}" for k, p in hist), flush=True)


if __name__ == "__main__":
    main()
