#!/usr/bin/env python
"""Converged-quality PSNR of a precision preset: train a method on the synthetic MMS-DATA-shaped scene from step 0
through the benchmarked path (graph-captured step, device pixel sampler) and score held-out full views with
evaluate.FullViewEvaluator every --eval-every steps.  The schedules (LR warm-up / milestones, coarse-to-fine levels,
tap delta, cos anneal, curvature warm-up) follow --max-iters, so a short run covers the whole schedule.

    python scripts/converge_psnr.py --precision fast --steps 6000 --max-iters 6000 [--method grid_raw] [--out f.json]

Prints one progress line per evaluation (and every 250 steps) so a long run is never silent.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ALL5 = ("rgb", "infrared", "mono", "polarization", "multispectral")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--method", default="grid_raw")
    ap.add_argument("--modalities", default=",".join(ALL5))
    ap.add_argument("--precision", default="fast")
    ap.add_argument("--steps", type=int, default=6000)
    ap.add_argument("--max-iters", type=int, default=6000)
    ap.add_argument("--rays", type=int, default=2048)
    ap.add_argument("--log2T", type=int, default=19)
    ap.add_argument("--eval-every", type=int, default=2000)
    ap.add_argument("--eval-views", type=int, default=5)
    ap.add_argument("--seed", type=int, default=654824)
    ap.add_argument("--out", default=None)
    ap.add_argument("--override", nargs="*", default=[],
                    help="PRECISION entries to change after the preset, e.g. heads=2 radiance=2 (functions.PRESETS)")
    a = ap.parse_args()
    from multimodalstudio_amd import evaluate as ev
    from multimodalstudio_amd import functions as fx
    from multimodalstudio_amd import graphs as gr
    from multimodalstudio_amd import pipeline as pl
    dev = torch.device("cuda", 0)
    fx.set_precision(a.precision)
    for kv in a.override:
        k, v = kv.split("=")
        fx.PRECISION[k] = int(v)
    mods = tuple(a.modalities.split(","))
    tc = pl.TrainConfig(method=a.method, modalities=mods, num_rays_per_modality=a.rays, log2T=a.log2T,
                        max_iters=a.max_iters, gpu_sampler=True, seed=a.seed)
    tr = pl.Trainer(tc, dev)
    gt = gr.GraphTrainer(tr)
    hist = []
    t0 = time.time()
    for k in range(1, a.steps + 1):
        gt.step()
        if k % 250 == 0 and k % a.eval_every != 0:
            torch.cuda.synchronize()
            print(f"[{a.precision}] step {k} ({time.time() - t0:.0f}s)", flush=True)
        if k % a.eval_every == 0 or k == a.steps:
            torch.cuda.synchronize()
            tr.model.set_step(tr.step, tc.max_iters)
            psnr, rate = ev.eval_split(tr, n_views=a.eval_views)
            hist.append({"step": k, "psnr": psnr, "test_rays_per_sec": rate, "wall_s": time.time() - t0})
            print(f"[{a.precision}] step {k}: " + " ".join(f"{m} {v:.3f}" for m, v in psnr.items()) +
                  f"  ({time.time() - t0:.0f}s, eval {rate / 1e6:.2f} Mrays/s)", flush=True)
    res = {"precision": a.precision, "overrides": a.override, "method": a.method, "modalities": mods, "rays": a.rays, "steps": a.steps,
           "max_iters": a.max_iters, "log2T": a.log2T, "graph_stats": gt.stats, "history": hist}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
