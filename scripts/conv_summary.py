#!/usr/bin/env python
"""Paired converged-PSNR comparison of precision presets (scripts/converge_psnr.py outputs, gpurun_out/conv3k_*.json):
per modality, the mean over seeds of (variant - fp32) held-out PSNR with its standard error, for every variant that
shares seeds with fp32.  Earlier runs recorded in an existing summary (--prev) are merged in (fp32 seeds 1-3 of the
round-3 file).

    python scripts/conv_summary.py --prev profiles/round3_converged_psnr.json --out profiles/round3_converged_psnr.json
"""
from __future__ import annotations

import argparse
import glob
import json
import math
import os
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", default="gpurun_out/conv3k_*_s*.json")
    ap.add_argument("--prev", default=None)
    ap.add_argument("--keep-prev", nargs="*", default=["fp32"], help="variants of --prev merged in")
    ap.add_argument("--base", default="fp32", help="the variant the others are paired against")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    runs = {}
    if a.prev and os.path.exists(a.prev):
        prev = json.load(open(a.prev))
        for v in a.keep_prev:
            for s, r in prev.get("runs", {}).get(v, {}).items():
                runs.setdefault(v, {})[str(s)] = r
    for path in sorted(glob.glob(a.runs)):
        m = re.search(r"conv3k_(.+)_s(\d+)\.json$", path)
        d = json.load(open(path))
        last = d["history"][-1]
        runs.setdefault(m.group(1), {})[m.group(2)] = {"psnr": last["psnr"], "wall_s": last["wall_s"]}
    summary = {}
    base = runs.get(a.base, {})
    for v, rs in sorted(runs.items()):
        if v == a.base:
            continue
        seeds = sorted(set(rs) & set(base), key=int)
        if not seeds:
            continue
        mods = list(rs[seeds[0]]["psnr"])
        per = {}
        for m in mods:
            d = [rs[s]["psnr"][m] - base[s]["psnr"][m] for s in seeds]
            mean = sum(d) / len(d)
            sd = math.sqrt(sum((x - mean) ** 2 for x in d) / max(1, len(d) - 1))
            per[m] = {"mean": round(mean, 4), "se": round(sd / math.sqrt(len(d)), 4), "n": len(d)}
        allm = [sum(rs[s]["psnr"][m] - base[s]["psnr"][m] for m in mods) / len(mods) for s in seeds]
        mean = sum(allm) / len(allm)
        sd = math.sqrt(sum((x - mean) ** 2 for x in allm) / max(1, len(allm) - 1))
        summary[v] = {"seeds": seeds, f"paired_dpsnr_vs_{a.base}": per, "all_modality_mean": round(mean, 4),
                      "all_modality_se": round(sd / math.sqrt(len(allm)), 4)}
        print(f"{v:22s} seeds {','.join(seeds):18s} " + " ".join(f"{m} {p['mean']:+.3f}±{p['se']:.3f}"
                                                               for m, p in per.items()) +
              f" | all {mean:+.3f}±{sd / math.sqrt(len(allm)):.3f}")
    if a.out:
        out = {"what": "grid_raw5 (5 mosaicked modalities) trained from step 0 for 3000 steps (max_iters 3000: full LR / "
                       "coarse-to-fine schedule) on the synthetic scene, held-out PSNR (FullViewEvaluator, 5 views) per "
                       "modality; scripts/converge_psnr.py, seed = pixel sampler / draw seed (same init); paired "
                       "differences vs the fp32 preset with standard errors (scripts/conv_summary.py)",
               "runs": runs, "summary": summary}
        if a.prev and os.path.exists(a.prev):
            out["earlier"] = {k: v for k, v in json.load(open(a.prev)).items() if k in ("variants", "summary")}
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
