#!/usr/bin/env python
"""Training-trajectory fixture for the PSNR-parity test (SURVEY §8(d) 'PSNR parity').

The CPU restatement (oracle/, pinned bit-exact to the reference by tests/test_oracle_golden.py) trains the
`grid` model on the synthetic scene from a seeded init for K steps, in the benchmark's model state (step
95k: all grid levels active, lr x 0.064).  Every input is reproducible from seeds on any machine: pixel
coordinates from the reference-order host sampler, targets from the analytic scene rendered on the CPU,
and the uniform draws from a CPU generator in fixed-size blocks (independent of the hit count), so the
fixture stores only the configuration, the oracle's per-step losses and its held-out PSNR before and
after training.  tests/test_gpu_train_parity.py replays the same K steps through the HIP path.

    python tests/golden/make_train_parity.py [rgb|raw5] [seed]   (CPU, ~3 / ~2.5 min on 8 threads)

writes train_parity_<name>.npz (seed 0) or train_parity_<name>_s<seed>.npz: seed k > 0 shifts the pixel-sampler and
draw seeds by k (same init), an independent trajectory of the same training problem.  One trajectory's held-out
PSNR scatters by about +-0.1 dB (chaotic float-atomic / AdamW-eps dynamics), so the parity test pairs the HIP run
with the oracle run seed by seed and compares means over seeds.
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

CONFIGS = {
    # BASELINE configs[1] shape: grid, RGB
    "rgb": dict(method="grid", modalities=("rgb",), rays=256, log2T=12, width=160, height=128, n_views=10,
                start_step=95000, steps=300, eval_rays=4096, init_seed=654824, sampler_seed=654824, rng_seed=11,
                eval_seed=5, bg_samples=16),
    # BASELINE configs[2] shape: grid_raw, five mosaicked modalities (each pixel supervises its own band)
    # (a short window at the step-95k learning rate: the first AdamW steps move the hash tables by ~lr per entry and the
    # held-out PSNR by several dB per modality while independent runs of one implementation stay within ~0.05 dB --
    # float-atomic reordering has not yet decorrelated them -- so the 0.1 dB criterion sits well above the noise
    # floor; by step 200 one run's PSNR scatters by 0.1-0.4 dB, scripts/parity_scatter.py)
    "raw5": dict(method="grid_raw", modalities=("rgb", "infrared", "mono", "polarization", "multispectral"),
                 rays=96, log2T=12, width=96, height=80, n_views=10, start_step=95000, steps=50, checkpoints=(25,),
                 eval_rays=2048, init_seed=654824, sampler_seed=654824, rng_seed=11, eval_seed=5, bg_samples=16),
}
# raw5 on the 45-training-view scene (50 views, the benchmark's view count; the 10-view scene above generalises so
# poorly that held-out rgb PSNR falls while the training loss drops): every modality's held-out PSNR rises by
# 1.3-7 dB over the first 50 steps.  Each seed's fixture also records an oracle-prime run (every gradient perturbed by
# 2^-22 relative per step, perturber below): the reference algorithm's own sensitivity, the gate's null scatter.
CONFIGS["raw5v"] = dict(CONFIGS["raw5"], n_views=50, checkpoints=(10, 20, 30, 40), prime=2.0 ** -22, prime_seeds=16)
# BASELINE configs[4] shape: grid_raw_grid_bg_unbalanced (rgb + polarization on 10 of its 45 views, the hash-grid
# background, 3-layer background heads, SO3xR3 pose refinement)
CONFIGS["bg5"] = dict(CONFIGS["raw5v"], method="grid_raw_grid_bg_unbalanced", modalities=("rgb", "polarization"),
                      steps=40, checkpoints=(10, 20, 30))
CFG = CONFIGS["rgb"]
HERE = os.path.dirname(os.path.abspath(__file__))


def method_kind(cfg):
    """(raw mosaicked frames, background kind) of the fixture's method (pipeline.METHODS)."""
    from multimodalstudio_amd.pipeline import METHODS
    raw, bg_kind, _ = METHODS[cfg["method"]]
    return raw, bg_kind


def train_cameras(cfg, mods):
    """The training views: the method's YAML skip list applied (config 5 keeps 10 polarization views of the 45)."""
    from multimodalstudio_amd import scene as ms
    from multimodalstudio_amd.pipeline import skip_views_for
    cams = ms.make_cameras(mods, cfg["n_views"], cfg["width"], cfg["height"], seed=0, train=True)
    for m, skip in (skip_views_for(cfg["method"]) or {}).items():
        if m in cams:
            cams[m] = ms.select_views(cams[m], [v for v in cams[m].view_ids if v not in set(skip)])
    return cams


def load_start_state(cfg, sd: dict, poses: dict = None):
    """The fixture's shared start state (parameters and pose deltas, 'p:' / 'pose:' keys) over the seeded init."""
    if not cfg.get("start_state"):
        return sd, poses
    f = np.load(os.path.join(HERE, cfg["start_state"]))
    sd = {k: torch.from_numpy(f["p:" + k]).clone() if ("p:" + k) in f else v for k, v in sd.items()}
    poses = {k[5:]: torch.from_numpy(f[k]).clone() for k in f.files if k.startswith("pose:")}
    return sd, poses


def param_checksum(sd):
    return float(sum(float(v.double().abs().sum()) for v in sd.values()))


def draws(gen, n, bg_samples):
    """One step's uniform draws in the reference's order as fixed-size blocks: rows
    [0, n_hit) of `uniform` / `pdf` are used, so the stream does not depend on the hit count."""
    uni = torch.rand(n, 1, generator=gen)
    pdf = [torch.rand(n, 1, generator=gen) for _ in range(4)]
    bg = torch.rand(n, bg_samples + 1, generator=gen)
    return uni, pdf, bg


def step_inputs(cfg, sampler, frames, images, mods):
    coords, sel = sampler.sample(frames)
    targets = {m: images[m][sel[m].long(), coords[m][:, 1].long(), coords[m][:, 2].long()] for m in mods}
    return coords, targets


def eval_inputs(cfg, ecams, eimages, m):
    eg = torch.Generator().manual_seed(cfg["eval_seed"])
    n = cfg["eval_rays"]
    c = ecams[m]
    ci = torch.randint(0, c.c2w.shape[0], (n, 1), generator=eg, dtype=torch.int32)
    px = torch.randint(0, cfg["width"], (n, 1), generator=eg, dtype=torch.int32)
    py = torch.randint(0, cfg["height"], (n, 1), generator=eg, dtype=torch.int32)
    coords = torch.cat([ci, py, px], -1)
    tgt = eimages[m][ci[:, 0].long(), py[:, 0].long(), px[:, 0].long()]
    return coords, tgt, draws(eg, n, cfg["bg_samples"])


def seeded(cfg, seed: int):
    """The configuration of seed ``seed`` (sampler and draw streams shifted, init unchanged)."""
    return dict(cfg, sampler_seed=cfg["sampler_seed"] + 1000 * seed, rng_seed=cfg["rng_seed"] + 1000 * seed)


def fixture_name(name: str, seed: int) -> str:
    return f"train_parity_{name}.npz" if seed == 0 else f"train_parity_{name}_s{seed}.npz"


def perturber(rel: float, seed: int):
    """oracle-prime: every gradient entry scaled by (1 + rel * U(-1, 1)) before clipping, each step -- last-bit
    differences of the size float-atomic / GEMM reordering makes (rel ~ 2^-22), so the trajectory's sensitivity to
    them is measured on the reference algorithm itself (the floor under any HIP-vs-oracle comparison)."""
    g = torch.Generator().manual_seed(987654 + seed)

    def hook(params):
        for p in params:
            if p.grad is not None:
                u = torch.rand(p.grad.shape, generator=g, dtype=torch.float64)
                p.grad.mul_((1.0 + rel * (2.0 * u - 1.0)).to(p.grad.dtype))
    return hook


def psnr_of(pred: torch.Tensor, tgt: torch.Tensor, clip: bool) -> float:
    """peak_signal_noise_ratio(data_range=1); clip: of the clipped rendering as compute_metrics takes it
    (/root/reference/src/utils/eval_utils.py:348-357: renderings = output.clip(0., 1.))."""
    pred = pred.clamp(0.0, 1.0) if clip else pred
    return float(-10.0 * np.log10(float(((pred.double() - tgt.double()) ** 2).mean())))


def main(name: str = "rgb", seed: int = 0, perturb: float = 0.0, out_path: str = None, checkpoints=None,
         save: bool = True, save_state: str = None):
    from multimodalstudio_amd import scene as ms
    from multimodalstudio_amd.model import BaseModel, ModelSpec
    from multimodalstudio_amd.pipeline import UniformPixelSampler
    from oracle import model as om
    from oracle import rays as orr
    from oracle.train import OracleTrainer

    torch.set_num_threads(int(os.environ.get("THREADS", min(8, os.cpu_count() or 1))))
    cfg = seeded(CONFIGS[name], seed)
    if checkpoints is not None:
        cfg = dict(cfg, checkpoints=tuple(checkpoints))
    raw, bg_kind = method_kind(cfg)
    mods = list(cfg["modalities"])
    channels = {m: ms.CHANNELS[m] for m in mods}
    torch.manual_seed(cfg["init_seed"])
    model = BaseModel(ModelSpec(channels, log2T=cfg["log2T"], bg_kind=bg_kind))
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    cams = train_cameras(cfg, mods)
    ecams = ms.make_cameras(mods, cfg["n_views"], cfg["width"], cfg["height"], seed=0, train=False)
    cpu = torch.device("cpu")
    images = {m: ms.render_frames(cams[m], channels[m], cpu, m if raw else None) for m in mods}
    eimages = {m: ms.render_frames(ecams[m], channels[m], cpu, m if raw else None) for m in mods}
    masks = {m: ms.mosaick_mask(m, cfg["width"], cfg["height"]) for m in mods}
    frames = {m: {"shape": (cams[m].c2w.shape[0], cfg["height"], cfg["width"]),
                  "indexes": torch.arange(cams[m].c2w.shape[0], dtype=torch.int32)} for m in mods}
    sampler = UniformPixelSampler(cfg["rays"], cfg["sampler_seed"])
    init_ck = param_checksum(sd)
    sd, poses = load_start_state(cfg, sd)
    ot = OracleTrainer(sd, channels, cams, cfg["log2T"], cfg["start_step"], raw=raw, pose=poses, mosaick=masks,
                       bg_kind=bg_kind)
    gen = torch.Generator().manual_seed(cfg["rng_seed"])

    def rng_hook(n_hit, n_rays):
        uni, pdf, bg = {}, {}, {}
        for m in mods:
            u, p, b = draws(gen, n_rays[m], cfg["bg_samples"])
            uni[m], pdf[m], bg[m] = u[:n_hit[m]], [x[:n_hit[m]] for x in p], b
        return om.RNG(uni, pdf, bg)

    ot.rng = rng_hook
    if perturb > 0:
        ot.grad_hook = perturber(perturb, seed)
    out = {"cfg_json": np.frombuffer(repr(cfg).encode(), dtype=np.uint8), "init_checksum": init_ck}

    def evaluate(tag):
        st = om.StepState(step=ot.step)
        rays, rng, tgts, coords_e = {}, om.RNG({}, {}, {}), {}, {}
        for m in mods:
            c = ecams[m]
            coords, tgt, (u, p, b) = eval_inputs(cfg, ecams, eimages, m)
            rays[m] = orr.generate_rays(coords, c.fx, c.fy, c.cx, c.cy, c.c2w, c.distortion, torch.zeros(1, 6), 0.0)
            hit = int(orr.sphere_collider(rays[m].origins, rays[m].directions)[2].sum())
            rng.uniform[m], rng.pdf[m], rng.background[m] = u[:hit], [x[:hit] for x in p], b
            tgts[m], coords_e[m] = tgt, coords
        with torch.no_grad():
            outs = om.model_forward(rays, ot.P, ot.spec, st, rng)
        for m in mods:
            pred = outs[m][m]
            if raw:
                pred = om.select_channel(pred, masks[m], coords_e[m])
            psnr = -10.0 * np.log10(float(((pred - tgts[m]) ** 2).mean()))
            pclip = psnr_of(pred, tgts[m], clip=True)
            print(f"{tag} {m}: PSNR {psnr:.4f} dB (clipped {pclip:.4f})", flush=True)
            out[f"{tag}:{m}:psnr"] = np.float64(psnr)
            out[f"{tag}:{m}:psnr_clip"] = np.float64(pclip)

    evaluate("eval0")
    t0 = time.time()
    for k in range(cfg["steps"]):
        if k in cfg.get("checkpoints", ()):
            evaluate(f"eval{k}")
        coords, targets = step_inputs(cfg, sampler, frames, images, mods)
        out[f"s{k}:loss"] = np.float64(ot.train_step(coords, targets))
        if k % 25 == 0:
            print(f"step {k}: loss {float(out[f's{k}:loss']):.6f} ({time.time() - t0:.1f}s)", flush=True)
    evaluate("eval")
    if cfg.get("prime") and perturb == 0 and seed < cfg.get("prime_seeds", 1 << 30):
        # the oracle-prime companion run of the same seed
        prime = main(name, seed, float(cfg["prime"]), checkpoints=checkpoints, save=False)
        out.update({"prime:" + k: v for k, v in prime.items() if "psnr" in k})
    if save_state:
        st = {"p:" + k: v.detach().numpy() for k, v in ot.P.items()}
        st.update({"pose:" + m: ot.pose[m].detach().numpy() for m in mods})
        st.update({k: v for k, v in out.items() if "psnr" in k or k in ("cfg_json", "init_checksum")})
        np.savez_compressed(save_state, **st)
        return out
    if save:
        path = out_path or os.path.join(os.path.dirname(os.path.abspath(__file__)), fixture_name(name, seed))
        np.savez_compressed(path, **out)
    return out


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("name", nargs="?", default="rgb")
    ap.add_argument("seed", nargs="?", type=int, default=0)
    ap.add_argument("--perturb", type=float, default=0.0, help="oracle-prime: relative gradient perturbation")
    ap.add_argument("--out", default=None)
    ap.add_argument("--checkpoints", type=int, nargs="*", default=None)
    ap.add_argument("--save-state", default=None, help="write the trained parameters + poses (a start state)")
    a = ap.parse_args()
    main(a.name, a.seed, a.perturb, a.out, a.checkpoints, save_state=a.save_state)
