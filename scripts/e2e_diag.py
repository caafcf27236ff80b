#!/usr/bin/env python
"""Where an end-to-end fixture's parameter-gradient error comes from: per parameter tensor, the scale-relative max
error, its 99.9th percentile and the number of elements above 1e-3 of the scale, plus the loss terms vs the
reference's (tests/golden/e2e_*.npz).  A handful of outlying elements points at a discrete flip (a ReLU / L1 sign at
a near-zero argument); a broad error at a systematic difference.

    python scripts/e2e_diag.py e2e_grid_raw_5mod_sat_s95000 [fp32|fast]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from test_gpu_e2e import load, run_hip_e2e
    from multimodalstudio_amd import functions as fx
    name = sys.argv[1]
    fx.set_precision(sys.argv[2] if len(sys.argv) > 2 else "fp32")
    f = load(name)
    mods, model, pose, outs, losses, total = run_hip_e2e(f, torch.device("cuda", 0))
    for k, v in losses.items():
        ref = f.get("loss:" + k)
        if ref is not None:
            print(f"loss {k:20s} hip {float(v):.7e} ref {float(ref):.7e} rel {abs(float(v) - float(ref)) / max(abs(float(ref)), 1e-30):.2e}")
    rows = []
    for k, p in model.named_parameters():
        if "g:" + k not in f or p.grad is None:
            continue
        ref = f["g:" + k].astype(np.float64)
        got = p.grad.detach().cpu().numpy().astype(np.float64)
        scale = np.abs(ref).max() + 1e-30
        e = np.abs(got - ref) / scale
        i = int(np.argmax(e))
        rows.append((e.max(), np.quantile(e, 0.999), int((e > 1e-3).sum()), e.size, k, np.unravel_index(i, ref.shape),
                     got.flat[i], ref.flat[i], scale))
    rows.sort(key=lambda r: -r[0])
    for r in rows[:10]:
        print(f"{r[0]:.2e} p99.9 {r[1]:.2e} n>1e-3 {r[2]}/{r[3]}  {r[4]}  at {r[5]} hip {r[6]:.4e} ref {r[7]:.4e} "
              f"scale {r[8]:.3e}")


if __name__ == "__main__":
    main()
