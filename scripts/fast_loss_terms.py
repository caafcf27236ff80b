"""Loss terms of the rgb train-parity trajectory (seed-0 fixture) under fp32 and the fast preset: which part of the
total separates the presets.  usage: python scripts/fast_loss_terms.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_gpu_train_parity as tp  # noqa: E402
from multimodalstudio_amd import pipeline as pl  # noqa: E402

orig = pl.Trainer.train_step
rec = []


def wrapped(self, *a, **k):
    out = orig(self, *a, **k)
    rec.append({n: float(v) for n, v in out[0].items()})
    return out


pl.Trainer.train_step = wrapped
dev = torch.device("cuda", 0)
for prec in (sys.argv[1:] or ["fp32", tp.FAST]):
    rec.clear()
    f, cfg, losses, psnr = tp.run_parity(dev, prec, tp.GOLD)
    keys = rec[0].keys()
    means = {n: np.mean([r[n] for r in rec]) for n in keys}
    last = {n: np.mean([r[n] for r in rec[-20:]]) for n in keys}
    ref = np.array([float(f[f"s{k}:loss"]) for k in range(cfg["steps"])])
    print(prec, "total", losses.mean(), "oracle", ref.mean(), "terms mean", means, "last20", last, "psnr", psnr,
          flush=True)
