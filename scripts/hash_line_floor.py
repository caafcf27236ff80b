#!/usr/bin/env python
"""The radiance hash walk's HBM-traffic floor (CPU, this container): for the samples of the
benchmarked step (e2e_full_grid_rgb_l19: 2048 rays, 876 hits, 64 samples each -- the bench's per-step radiance batch)
count the DISTINCT table cache lines the 8 corners x 16 levels touch.  With an unbounded cache and a perfect sample
order every such line still moves once from HBM (forward: read; backward: read-modify-write of the gradient line by the
float atomics), so (distinct lines x line size) is a floor no reordering of the walk can go below.  Compared with the
SURVEY §8(d) algorithmic bytes (8 B per corner) and the PMC traffic per launch in profiles/pmc_traffic_fast_h16b.json.

    python scripts/hash_line_floor.py
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import hashgrid as oh  # noqa: E402
from oracle import rays as orr  # noqa: E402
from test_oracle_golden import e2e_inputs  # noqa: E402


def main():
    f = e2e_inputs("e2e_full_grid_rgb_l19")
    T = lambda a: torch.from_numpy(np.asarray(a))  # noqa: E731
    m = "rgb"
    smp = orr.make_samples(T(f[f"{m}:bins"]), T(f[f"{m}:hit:nears"]), T(f[f"{m}:hit:fars"]), "uniform")
    o, d = T(f[f"{m}:hit:origins"]), T(f[f"{m}:hit:directions"])
    pos = (o[:, None, :] + d[:, None, :] * smp.starts[..., None].reshape(o.shape[0], -1, 1)).reshape(-1, 3)
    x_hat = (pos + 1.0) / 2.0
    log2T = 19
    scales = oh.level_scales()
    xs = x_hat[:, None, :] * scales.view(-1, 1)
    idx = torch.stack(oh.corner_indices(torch.ceil(xs).to(torch.int32), torch.floor(xs).to(torch.int32), log2T), 0)
    n = pos.shape[0]
    out = {"samples": n}
    alg_fwd = n * 16 * 8 * 8          # float2 per corner
    rows = []
    for line in (64, 128):
        lines = (idx * 8) // line      # [8, n, L] byte offset of the float2 entry -> line
        per_level = [int(torch.unique(lines[:, :, l]).numel()) for l in range(16)]
        total = sum(per_level)
        rows.append((line, per_level, total))
        out[f"distinct_lines_{line}B"] = total
        out[f"floor_fwd_MB_{line}B"] = total * line / 1e6
        out[f"floor_bwd_MB_{line}B"] = 2 * total * line / 1e6
    out["algorithmic_corner_MB"] = alg_fwd / 1e6
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic_fast_h16b.json")
    if os.path.exists(pmc):
        out["pmc"] = {k: v for k, v in json.load(open(pmc)).items() if "radiance" in k or "hash" in k}
    for line, per_level, total in rows:
        print(f"{line:3d}-B lines: distinct per level {per_level}")
        print(f"      total {total} lines = {total * line / 1e6:.1f} MB read (forward floor), "
              f"{2 * total * line / 1e6:.1f} MB read + written (backward floor)")
    print(f"{n} samples; corner bytes (8 B x 8 corners x 16 levels): {alg_fwd / 1e6:.1f} MB")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
