"""Which bf16 stage moves the fast preset's training PSNR: raw5 parity runs with one stage at a time promoted."""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, ".."))
import test_gpu_train_parity as T  # noqa: E402
from multimodalstudio_amd import functions as fx  # noqa: E402

fast = dict(fx.PRESETS["fast"])
fx.PRESETS["fast_rad3"] = dict(fast, radiance=2)
fx.PRESETS["fast_heads3"] = dict(fast, heads=2)
fx.PRESETS["fast_bg3"] = dict(fast, background=2)
fx.PRESETS["fast_rad32"] = dict(fast, radiance=0)
dev = torch.device("cuda", 0)
reps = int(os.environ.get("REPS", "4"))
for prec in sys.argv[1:]:
    ds = []
    for rep in range(reps):
        f, cfg, losses, psnr = T.run_parity(dev, prec, T.GOLD_RAW5)
        oracle = {m: float(f[f"eval:{m}:psnr"]) for m in cfg["modalities"]}
        ds.append([psnr[m] - oracle[m] for m in cfg["modalities"]])
    ds = np.array(ds)
    print(prec, "mean dPSNR", np.round(ds.mean(0), 3), "overall", round(float(ds.mean()), 3), "sd",
          round(float(ds.std(0).mean()), 3), flush=True)
