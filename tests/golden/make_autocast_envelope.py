"""The reference's own fp16-autocast deviation ("16-mixed", the mode every BASELINE YAML trains in) on the end-to-end
fixtures, written to tests/golden/autocast_envelope.npz (THIS CONTAINER ONLY: it imports the reference).

    python tests/golden/make_autocast_envelope.py [fixture ...]

For each fixture the reference step is re-run exactly as make_golden.py ran it (same parameters, camera rig, pixels
and every uniform draw), but with the model forward under CUDA's fp16 autocast policy (autocast16.py) and the loss
scaled by Fabric's GradScaler (/root/reference/src/engine/trainer.py:51,57-62; base_pipeline.py:148-149): the scale is
the largest power of two <= 2^24 whose scaled gradients are all finite -- where the dynamic scaler settles (it doubles
after 2000 finite steps and halves on an overflow) and the scale with the least fp16 underflow, i.e. the TIGHTEST
envelope the reference's mode allows.  Not included (so the envelope is a lower bound of the reference GPU's own
deviation): the TF32 matmuls that ``matmul_precision: high`` (trainer.py:55) enables outside the autocast region (ray
generation, pose composition) and tcnn's fp16 hash tables (tcnn is absent; the torch grid is pinned).  The full-size fixtures
are re-run on the fp32 reference's own samples (its final NeuS bins injected, gen_end_to_end ``inject_bins``), as the
HIP side is then run: their rough tables make a free-running sampler chaotic (tests/test_gpu_fullsize.py).

Every quantity tests/test_gpu_e2e.py compares is recorded as the reference-fp16-vs-reference-fp32 distance, with the
same metric the test uses: ``q|max`` = max|a - ref| / max|ref| (scale-relative), ``q|l2`` = ||a - ref|| / ||ref||, and
for the rendered radiance ``q|mean_rel`` / ``q|max_rel`` = mean / max of |a - ref| / max(|ref|, 1e-2).
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import make_golden as mg  # noqa: E402
from fullsize_state import fullsize_state, with_fullsize_params  # noqa: E402

OUT = os.path.join(HERE, "autocast_envelope.npz")
RAW5 = ["rgb", "infrared", "mono", "polarization", "multispectral"]
FIXTURES = {
    # name: gen_end_to_end arguments, as make_golden.py's __main__ wrote the fixture
    "e2e_grid_rgb_s95000": (("grid", "grid.yaml", ["rgb"], 95000), {}),
    "e2e_grid_rgb_s30000": (("grid", "grid.yaml", ["rgb"], 30000), {}),
    "e2e_grid_raw_5mod_s95000": (("grid_raw", "grid_raw.yaml", RAW5, 95000), {"raw": True}),
    "e2e_grid_raw_5mod_sat_s95000": (("grid_raw", "grid_raw.yaml", RAW5, 95000),
                                     {"n_rays": 16, "raw": True, "saturate": 0.2}),
    "e2e_grid_raw_gridbg_s95000": (("grid_raw_grid_bg_unbalanced", "grid_raw_rgb_all_views_pol_10_views.yaml",
                                    ["rgb", "polarization"], 95000), {"raw": True, "grid_bg": True}),
    # the full-size fixtures are compared on the reference's own samples (bins injected on both sides): their rough
    # tables make the free-running sampler chaotic (tests/test_gpu_fullsize.py), which would swamp the precision
    "e2e_full_grid_rgb_l19": (("grid", "grid.yaml", ["rgb"], 95000),
                              {"n_rays": 2048, "log2T": 19, "W": 640, "H": 512, "n_views": 50, "cam_seed": 0,
                               "compact": True, "state": lambda: fullsize_state(["rgb"], 19), "inject": True}),
}


def rel_err(a, r):
    a, r = np.asarray(a, np.float64), np.asarray(r, np.float64)
    s = np.abs(r).max() if r.size else 0.0
    return float(np.abs(a - r).max() / s) if s > 0 else float(np.abs(a - r).max())


def rel_l2(a, r):
    a, r = np.asarray(a, np.float64), np.asarray(r, np.float64)
    n = np.linalg.norm(r)
    return float(np.linalg.norm(a - r) / n) if n > 0 else float(np.linalg.norm(a - r))


def deviations(amp: dict, ref: dict, full_grads: dict) -> dict:
    """Every compared quantity of tests/test_gpu_e2e.py, reference-fp16 vs reference-fp32 (the fixture)."""
    d = {"loss|rel": abs(float(amp["loss"]) - float(ref["loss"])) / abs(float(ref["loss"]))}
    mods = [str(m) for m in ref["mods"]]
    for m in mods:
        got, want = amp[f"{m}:out:{m}"].astype(np.float64), ref[f"{m}:out:{m}"].astype(np.float64)
        rel = np.abs(got - want) / np.maximum(np.abs(want), 1e-2)
        d[f"{m}:{m}|mean_rel"], d[f"{m}:{m}|max_rel"] = float(rel.mean()), float(rel.max())
        d[f"{m}:{m}|max"] = rel_err(got, want)
        for k in ["normals", "accumulation", "depth", "gradients", "hessians"]:
            if f"{m}:out:{k}" in ref:
                d[f"{m}:{k}|max"] = rel_err(amp[f"{m}:out:{k}"], ref[f"{m}:out:{k}"])
        d[f"{m}:dpose|max"] = rel_err(amp[f"{m}:dpose"], ref[f"{m}:dpose"])
        a_b, r_b = amp[f"{m}:bins"], ref[f"{m}:bins"]
        d[f"{m}:bins|abs"] = float(np.abs(a_b - r_b).max()) if a_b.shape == r_b.shape else float("inf")
    for k in ref:
        if k.startswith("g:"):
            d[f"{k}|l2"], d[f"{k}|max"] = rel_l2(amp[k], ref[k]), rel_err(amp[k], ref[k])
        elif k.startswith("gtab_val:"):
            name = k[len("gtab_val:"):]
            g = full_grads[name]
            val = g.reshape(-1)[torch.from_numpy(ref["gtab_idx:" + name].astype(np.int64))].numpy()
            norms = g.double().reshape(16, -1).norm(dim=1).numpy()
            ref_n = ref["gtab_level_norm:" + name]
            d[f"g:{name}|l2"] = max(rel_l2(val, ref[k]), float(np.abs(norms - ref_n).max() / ref_n.max()))
            d[f"g:{name}|max"] = rel_err(val, ref[k])
    return d


def run(name: str):
    args, kw = FIXTURES[name]
    kw = dict(kw)
    if callable(kw.get("state")):
        kw["state"] = kw["state"]()
    ref = dict(np.load(os.path.join(HERE, name + ".npz")))
    if "params_from" in ref:
        p = dict(np.load(os.path.join(HERE, str(ref["params_from"]) + ".npz")))
        ref.update({k: v for k, v in p.items() if k.startswith("p:")})
    ref = with_fullsize_params(ref)
    if kw.pop("inject", False):
        kw["inject_bins"] = {str(m): torch.from_numpy(ref[f"{m}:bins"]) for m in ref["mods"]}
    captured = {}
    scale = 2.0 ** 16
    best = None
    tried = {}
    while True:
        arrays = capture_run(args, kw, name, scale, captured)
        ok = bool(arrays["amp_finite"])
        tried[scale] = ok
        if ok:
            best = (scale, arrays, dict(captured))
            if scale >= 2.0 ** 24 or (scale * 2) in tried:
                break
            scale *= 2
        else:
            if best is not None:
                break
            scale /= 2
            if scale < 2.0 ** -24:
                raise RuntimeError(f"{name}: no finite loss scale")
    scale, arrays, full = best
    d = deviations(arrays, ref, full)
    d["amp_scale"] = scale
    print(f"{name}: loss scale 2^{int(np.log2(scale))}")
    for k in sorted(d, key=lambda k: -d[k])[:12]:
        print(f"   {k:100s} {d[k]:.3e}")
    return d


def capture_run(args, kw, name, scale, captured):
    """gen_end_to_end at this loss scale; ``captured`` receives the full hash-table gradients of a compact run."""
    captured.clear()
    arrays = mg.gen_end_to_end(*args, name[4:], amp_scale=scale, write=False, keep_table_grads=captured, **kw)
    return {k: (v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)) for k, v in arrays.items()}


def main():
    names = sys.argv[1:] or list(FIXTURES)
    env = dict(np.load(OUT)) if os.path.exists(OUT) else {}
    for n in names:
        d = run(n)
        for k, v in d.items():
            env[f"{n}/{k}"] = np.float64(v)
    np.savez_compressed(OUT, **env)
    print(f"wrote {OUT} ({len(env)} values)")


if __name__ == "__main__":
    main()
