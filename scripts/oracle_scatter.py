#!/usr/bin/env python
"""Oracle-vs-oracle' scatter of the raw5 training-parity window (CPU, test infrastructure): each seed's fixture run
(the oracle as committed) and the same run with every gradient perturbed by a relative 2^-22 per step (oracle', the
size of float-atomic / GEMM reordering differences), held-out PSNR (raw and clipped as compute_metrics takes it) at
the checkpoints.  The paired oracle' - oracle differences are the reference algorithm's own sensitivity: the floor
under the HIP - oracle gate of tests/test_gpu_train_parity.py.

    python scripts/oracle_scatter.py run <seed> <perturb> <out.json>      (one run)
    python scripts/oracle_scatter.py summary <dir>                          (table of the paired differences)
"""
from __future__ import annotations

import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
CHECKPOINTS = (10, 25, 40)


def run(seed: int, perturb: float, out: str, name: str = "raw5"):
    import make_train_parity as mtp
    res = mtp.main(name, seed, perturb, checkpoints=CHECKPOINTS, save=False)
    json.dump({k: float(v) for k, v in res.items() if k.endswith("psnr") or k.endswith("psnr_clip") or
               k.endswith(":loss")}, open(out, "w"))


def summary(d: str):
    runs = {}
    for p in glob.glob(os.path.join(d, "*.json")):
        seed, pert = os.path.basename(p)[:-5].split("_")
        runs.setdefault(int(seed), {})[float(pert)] = json.load(open(p))
    perts = sorted({k for r in runs.values() for k in r if k > 0})
    for pert in perts:
        seeds = sorted(s for s in runs if 0.0 in runs[s] and pert in runs[s])
        keys = sorted({k.rsplit(":", 2)[0] for k in runs[seeds[0]][0.0] if "psnr" in k},
                      key=lambda t: int(t[4:] or 10 ** 6))
        mods = sorted({k.split(":")[1] for k in runs[seeds[0]][0.0] if "psnr" in k})
        print(f"perturb {pert:g}: {len(seeds)} seeds")
        for kind in ("psnr", "psnr_clip"):
            for tag in keys:
                d_ = {m: np.array([runs[s][pert][f"{tag}:{m}:{kind}"] - runs[s][0.0][f"{tag}:{m}:{kind}"] for s in seeds])
                      for m in mods}
                print(f"  {kind:9s} {tag:7s} mean " + " ".join(f"{m[:5]} {v.mean():+.4f}" for m, v in d_.items()) +
                      " | sd " + " ".join(f"{m[:5]} {v.std(ddof=1):.4f}" for m, v in d_.items()))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]), float(sys.argv[3]), sys.argv[4])
    else:
        summary(sys.argv[2])
