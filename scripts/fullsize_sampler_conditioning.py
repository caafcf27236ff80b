#!/usr/bin/env python
"""How well conditioned a full-size fixture's NeuS sampling is (CPU, this container): the oracle run free-running in
float64 (nothing injected) against the reference's float32 bins.  On the rough fixture (e2e_full_grid_rgb_l19) float32
vs float64 summation moves ~14 % of the rays' bins; a smooth fixture must keep >= 99 % of them within 2e-5, or the
free-running parity test on it (tests/test_gpu_fullsize.py::test_fullsize_smooth_free_running) would pin nothing.

    python scripts/fullsize_sampler_conditioning.py e2e_full_grid_rgb_l19_smooth
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

from oracle import model as om  # noqa: E402
from oracle import rays as orr  # noqa: E402
from test_oracle_golden import e2e_inputs  # noqa: E402


def main(name):
    from multimodalstudio_amd.scene import CHANNELS
    f = e2e_inputs(name)
    mods = [str(m) for m in f["mods"]]
    dt = torch.float64
    T = lambda a: torch.from_numpy(np.asarray(a)).to(dt if np.asarray(a).dtype.kind == "f" else None)  # noqa
    key = "p:surface_model.surface_field.field.feature_grid.encoding.hash_table"
    spec = om.spec_grid({m: CHANNELS[m] for m in mods}, log2T=int(np.log2(f[key].shape[0] // 16)), raw=bool(f["raw"]))
    st = om.StepState(step=int(f["step"]))
    P = {k[2:]: T(v) for k, v in f.items() if k.startswith("p:")}
    torch.set_default_dtype(dt)
    with torch.no_grad():
        poses = {m: T(f[f"{m}:pose"]) for m in mods}
        rays = {m: orr.generate_rays(T(f[f"{m}:coords"]), T(f[f"{m}:fx"]), T(f[f"{m}:fy"]), T(f[f"{m}:cx"]),
                                     T(f[f"{m}:cy"]), T(f[f"{m}:c2w"]), T(f[f"{m}:distortion"]), poses[m], 0.0)
                for m in mods}
        draws = [T(f[f"rand:{i}"]) for i in range(len([k for k in f if k.startswith("rand:")]))]
        nm = len(mods)
        rng = om.RNG(uniform={m: draws[i] for i, m in enumerate(mods)},
                     pdf={m: draws[nm + 4 * i: nm + 4 * i + 4] for i, m in enumerate(mods)},
                     background={m: draws[5 * nm + i] for i, m in enumerate(mods)})
        outs = om.model_forward(rays, P, spec, st, rng)
    for m in mods:
        db = np.abs(outs[m]["bins"].numpy() - f[f"{m}:bins"]).max(1)
        e = np.abs(outs[m][m].numpy() - f[f"{m}:out:{m}"]).max(1) / np.abs(f[f"{m}:out:{m}"]).max()
        print(f"{name} {m}: float64 oracle vs the reference's float32 bins: rays within 2e-5 {np.mean(db <= 2e-5):.4f}"
              f", largest shift {db.max():.2e}; radiance worst ray {e.max():.2e}")


if __name__ == "__main__":
    torch.set_num_threads(8)
    main(sys.argv[1] if len(sys.argv) > 1 else "e2e_full_grid_rgb_l19_smooth")
