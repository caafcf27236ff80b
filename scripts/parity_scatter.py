#!/usr/bin/env python
"""Run-to-run scatter of the HIP path's held-out PSNR on one parity fixture (no oracle): the same seeded training
problem replayed R times, for each AdamW eps given.  Float-atomic reduction order is the only difference between the
runs, so the spread measures how chaotic the trajectory is -- the floor under any paired HIP-vs-oracle comparison.

    python scripts/parity_scatter.py [--fixture train_parity_raw5.npz] [--runs 3] [--eps 1e-15 1e-8] [--precision fp32]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fixture", default="train_parity_raw5v.npz")
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--eps", type=float, nargs="+", default=[1e-15, 1e-8])
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--config", default=None, help="a make_train_parity.CONFIGS name instead of --fixture")
    ap.add_argument("--start-step", type=int, default=None)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--checkpoints", type=int, nargs="*", default=[25, 50, 100])
    a = ap.parse_args()
    from test_gpu_train_parity import run_parity
    dev = torch.device("cuda", 0)
    gold = os.path.join(ROOT, "tests", "golden", a.fixture)
    cfg = None
    if a.config is not None:
        sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
        from make_train_parity import CONFIGS
        cfg = dict(CONFIGS[a.config])
        if a.start_step is not None:
            cfg["start_step"] = a.start_step
        if a.steps is not None:
            cfg["steps"] = a.steps
    for eps in a.eps:
        hists = []
        for r in range(a.runs):
            hist = []
            _, cfg, losses, psnr = run_parity(dev, a.precision, gold, eps=eps, cfg=cfg, history=hist,
                                              checkpoints=tuple(a.checkpoints))
            hists.append(dict(hist))
            print(f"eps {eps:g} run {r}: mean loss {losses.mean():.6f} PSNR " +
                  " ".join(f"{m}:{v:.4f}" for m, v in psnr.items()), flush=True)
        for step in sorted(hists[0]):
            rows = [h[step] for h in hists]
            mods = list(rows[0])
            mean = {m: float(np.mean([p[m] for p in rows])) for m in mods}
            sd = {m: float(np.std([p[m] for p in rows], ddof=1)) for m in mods}
            print(f"eps {eps:g} step {step}: mean " + " ".join(f"{m}:{v:.3f}" for m, v in mean.items()) +
                  " | run-to-run sd " + " ".join(f"{m}:{v:.4f}" for m, v in sd.items()), flush=True)


if __name__ == "__main__":
    main()
