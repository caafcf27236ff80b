"""PSNR / trajectory parity: K training steps of the `grid` model through the HIP path, fed the
exact inputs and uniform draws of the CPU restatement's run (regenerated from the seeds recorded in
tests/golden/make_train_parity.py), then held-out PSNR.

* trajectory: the first steps' losses within 1e-3 relative (fp32 mode).  Later steps are not compared one by
  one: float-atomic gradient sums are not reproducible bit for bit, and AdamW (eps 1e-15) turns last-bit
  differences of near-zero gradients into full-size updates, so per-step losses of two runs of the *same*
  implementation drift apart; the averaged loss over the run and the PSNR are the stable quantities.
* PSNR: |dPSNR| <= 0.1 dB vs the oracle after K steps, for fp32 and for the `fast` preset, on the mean over
  independent seeded trajectories paired HIP / oracle (one run's PSNR scatters by about +-0.07 dB, see _repeated).
"""
from __future__ import annotations

import ast
import os
import sys

import numpy as np
import pytest
import torch

# the benchmarked preset under test (MMS_FAST_PRESET overrides it)
# the throughput presets under the gate: the benchmarked one (fast_h16d: fp16 radiance / head / background forwards,
# row-scaled fp16 backward-data chains, fp16 hidden-layer weight gradients and activation rows -- the reference GPU's
# autocast precision) and the all-split-bf16x3 one (MMS_FAST_PRESET picks one alone)
FAST_PRESETS = [os.environ["MMS_FAST_PRESET"]] if "MMS_FAST_PRESET" in os.environ else ["fast_h16d", "fast"]
FAST = FAST_PRESETS[0]

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden", "train_parity_rgb.npz")
sys.path.insert(0, os.path.join(HERE, "golden"))

TRAJ_STEPS = 5


def run_parity(dev, precision: str, gold: str = GOLD, eps=None, cfg=None, history=None, checkpoints=()):
    """The fixture's training run through the HIP path: (fixture, cfg, per-step losses, held-out PSNR per modality).
    ``cfg`` replaces the fixture (a make_train_parity.CONFIGS entry: run without an oracle to compare against);
    ``history`` (a list) receives (step, PSNR) at each of ``checkpoints`` and at the end."""
    from make_train_parity import draws, eval_inputs, method_kind, step_inputs, train_cameras
    from multimodalstudio_amd.pipeline import skip_views_for
    from multimodalstudio_amd import functions as fx
    from multimodalstudio_amd import model as mm
    from multimodalstudio_amd import pipeline as pl
    from multimodalstudio_amd import scene as ms
    f = np.load(gold) if cfg is None else None
    if cfg is None:
        cfg = ast.literal_eval(f["cfg_json"].tobytes().decode())
    raw, _ = method_kind(cfg)
    mods = list(cfg["modalities"])
    channels = {m: ms.CHANNELS[m] for m in mods}
    fx.set_precision(precision)
    try:
        tc = pl.TrainConfig(method=cfg["method"], modalities=tuple(mods), num_rays_per_modality=cfg["rays"],
                            log2T=cfg["log2T"], width=cfg["width"], height=cfg["height"], n_views=cfg["n_views"],
                            skip_views=skip_views_for(cfg["method"]))
        tr = pl.Trainer(tc, dev)
        ck = float(sum(float(v.detach().double().abs().sum()) for v in tr.model.state_dict().values()))
        if f is not None:
            assert ck == pytest.approx(float(f["init_checksum"]), rel=1e-9), "model init drifted from the fixture"
        if cfg.get("start_state"):
            # the fixture's shared partially trained state (parameters and pose deltas), copied into the flat buffers
            from make_train_parity import load_start_state
            sd, poses = load_start_state(cfg, {k: v.detach().cpu() for k, v in tr.model.state_dict().items()})
            with torch.no_grad():
                for k, v in tr.model.state_dict().items():
                    v.copy_(sd[k].to(dev))
                for m, pz in (poses or {}).items():
                    tr.pose.pose_adjustment[m].copy_(pz.to(dev))
        tr.set_step(cfg["start_step"])
        tr.fields.step_count = 0          # fresh optimizer state, as the oracle run
        # AdamW eps of the fixture's run (the reference's 1e-15 unless the fixture records another)
        tr.fields.eps = float(cfg.get("eps", 1e-15) if eps is None else eps)
        if tr.poses is not None:
            tr.poses.step_count = 0
        # inputs: same host sampler, CPU-rendered targets, same draw stream as the fixture generator
        cpu = torch.device("cpu")
        cams = train_cameras(cfg, mods)
        images = {m: ms.render_frames(cams[m], channels[m], cpu, m if raw else None) for m in mods}
        frames = {m: {"shape": (cams[m].c2w.shape[0], cfg["height"], cfg["width"]),
                      "indexes": torch.arange(cams[m].c2w.shape[0], dtype=torch.int32)} for m in mods}
        sampler = pl.UniformPixelSampler(cfg["rays"], cfg["sampler_seed"])
        gen = torch.Generator().manual_seed(cfg["rng_seed"])
        # eval: held-out views, zero pose delta, no grad, the fixture's eval draws
        ecams = ms.make_cameras(mods, cfg["n_views"], cfg["width"], cfg["height"], seed=0, train=False)
        eimages = {m: ms.render_frames(ecams[m], channels[m], cpu, m if raw else None) for m in mods}
        dcams = {m: pl.DeviceCameras(ecams[m], dev) for m in mods}
        gen_rays = pl.RayGenerator(dcams, pl.CameraOptimizer(mods, {m: dcams[m].num for m in mods}, mode="off"), 0.0)

        def evaluate():
            tr.model.set_step(tr.step, tc.max_iters)
            psnr = {}
            with torch.no_grad():
                rng, ecoords, tgts = mm.RNG({}, {}, {}), {}, {}
                for m in mods:
                    coords, tgt, (u, p, b) = eval_inputs(cfg, ecams, eimages, m)
                    rng.uniform[m], rng.pdf[m], rng.background[m] = u.to(dev), [x.to(dev) for x in p], b.to(dev)
                    ecoords[m], tgts[m] = coords.to(dev), tgt
                outs = tr.model(gen_rays(ecoords), rng)
                for m in mods:
                    pred = outs[m][m]
                    if raw:     # each pixel's own band (RawEvaluator, evaluator.py:721-745)
                        c = ecoords[m]
                        pred = pl.select_right_channel(pred, tr.masks[m][c[:, 1].long(), c[:, 2].long()].long()[:, None])
                    psnr[m] = -10.0 * float(np.log10(float(((pred.float().cpu() - tgts[m]) ** 2).mean())))
            return psnr

        losses = []
        for k in range(cfg["steps"]):
            if history is not None and k in checkpoints:
                history.append((k, evaluate()))
            coords, targets = step_inputs(cfg, sampler, frames, images, mods)
            rng = mm.RNG({}, {}, {})
            for m in mods:
                u, p, b = draws(gen, cfg["rays"], cfg["bg_samples"])
                rng.uniform[m], rng.pdf[m], rng.background[m] = u.to(dev), [x.to(dev) for x in p], b.to(dev)
            _, total, _ = tr.train_step(coords, targets, rng)
            losses.append(float(total))
        psnr = evaluate()
        if history is not None:
            history.append((cfg["steps"], psnr))
        return f, cfg, np.array(losses), psnr
    finally:
        fx.set_precision("fp32")


def _report(tag, f, cfg, losses, psnr):
    ref = np.array([float(f[f"s{k}:loss"]) for k in range(cfg["steps"])])
    rel = np.abs(losses - ref) / np.abs(ref)
    oracle = {m: float(f[f"eval:{m}:psnr"]) for m in cfg["modalities"]}
    start = {m: float(f[f"eval0:{m}:psnr"]) for m in cfg["modalities"]}
    print(f"{tag}: first {TRAJ_STEPS} steps max loss rel err {rel[:TRAJ_STEPS].max():.2e}; mean loss "
          f"{losses.mean():.6f} vs oracle {ref.mean():.6f}; PSNR {psnr} vs oracle {oracle} (start {start})")
    return ref, rel, oracle


REPEATS = 3


def _fixtures(gold: str):
    """The seed-0 fixture and its seeded siblings (make_train_parity.py <name> <seed>: independent trajectories of
    the same training problem)."""
    import glob
    stem = gold[:-len(".npz")]
    return [gold] + sorted(glob.glob(stem + "_s*.npz"), key=lambda p: int(p.rsplit("_s", 1)[1][:-4]))


def _repeated(dev, precision, gold=GOLD):
    """Held-out PSNR differences HIP - oracle, paired seed by seed, at the fixture's checkpoints and at its end.
    Independent trajectories of one implementation drift apart (float-atomic hash-gradient sums are not reproducible
    and AdamW's eps 1e-15 turns last-bit differences of near-zero gradients into full-size updates), so the criterion
    is on the mean difference over independent seeds (each oracle seed run once, the HIP path once per seed; with
    fewer than 4 seeds the HIP path runs REPEATS times per seed).  Returns (cfg, runs, {tag: {mod: mean diff}})."""
    fixtures = _fixtures(gold)
    reps = 1 if len(fixtures) >= 4 else REPEATS
    runs, diffs = [], {}
    for fx_path in fixtures:
        f0 = np.load(fx_path)
        cps = tuple(ast.literal_eval(f0["cfg_json"].tobytes().decode()).get("checkpoints", ()))
        for _ in range(reps):
            hist = []
            f, cfg, losses, psnr = run_parity(dev, precision, fx_path, history=hist, checkpoints=cps)
            ref, rel, oracle = _report(f"{precision}[{os.path.basename(fx_path)}]", f, cfg, losses, psnr)
            runs.append((f, cfg, losses, psnr, ref, rel))
            for step, p in hist:
                tag = "eval" if step == cfg["steps"] else f"eval{step}"
                diffs.setdefault(tag, []).append({m: p[m] - float(f[f"{tag}:{m}:psnr"]) for m in cfg["modalities"]})
    cfg = runs[0][1]
    mods = cfg["modalities"]
    means = {}
    for tag, ds in sorted(diffs.items()):
        mean = {m: float(np.mean([d[m] for d in ds])) for m in mods}
        sd = {m: float(np.std([d[m] for d in ds], ddof=1)) for m in mods}
        print(f"{precision} {tag}: {len(fixtures)} seeds x {reps}: mean dPSNR " +
              " ".join(f"{m} {v:+.4f}" for m, v in mean.items()) + " | sd of one pair " +
              " ".join(f"{m} {v:.4f}" for m, v in sd.items()))
        means[tag] = mean
    return cfg, runs, means


PSNR_TOL = 0.1
# the 0.1 dB bound is applied to a mean over seeds whose null scatter -- the reference algorithm against itself with
# fp32-reordering-size gradient perturbations (oracle' - oracle, recorded in each fixture) -- puts the bound at >= 3.3
# standard errors: a HIP path that IS the reference algorithm up to float reordering fails with probability < 0.1 %
NULL_SE_MAX = PSNR_TOL / 3.3


def null_scatter(gold: str):
    """{tag: {mod: (mean, sd, n)}} of the fixtures' oracle' - oracle held-out PSNR differences (the 'prime:' keys; the
    first seeds carry one), with n = the number of seeded fixtures the gate averages over: the null standard error of
    that mean is sd / sqrt(n)."""
    per = {}
    fixtures = _fixtures(gold)
    for path in fixtures:
        f = np.load(path)
        for k in f.files:
            if k.startswith("prime:") and k.endswith(":psnr"):
                _, tag, m, _ = k.split(":")
                per.setdefault(tag, {}).setdefault(m, []).append(float(f[k]) - float(f[f"{tag}:{m}:psnr"]))
    return {tag: {m: (float(np.mean(v)), float(np.std(v, ddof=1)), len(fixtures)) for m, v in d.items()}
            for tag, d in per.items()}


def _check_psnr(cfg, means, nulls=None):
    """|mean dPSNR| <= 0.1 dB for every modality at every checkpoint (no widening by the seeds' scatter); with the
    fixtures' null scatter, first that the window keeps the seed mean's null standard error <= 0.1 / 3.3 dB."""
    for tag, mean in means.items():
        for m in cfg["modalities"]:
            if nulls:
                mu, sd, n = nulls[tag][m]
                se = sd / np.sqrt(n)
                print(f"{tag} {m}: HIP - oracle {mean[m]:+.4f} dB | oracle' - oracle {mu:+.4f} dB, null SE {se:.4f}")
                assert se <= NULL_SE_MAX, ("the fixture window no longer resolves 0.1 dB", tag, m, se)
            assert abs(mean[m]) <= PSNR_TOL, (tag, m, mean[m])


@pytest.mark.gpu
def test_train_parity_fp32(dev):
    cfg, runs, means = _repeated(dev, "fp32")
    for _, _, losses, _, ref, rel in runs:
        assert rel[:TRAJ_STEPS].max() < 1e-3
        assert abs(losses.mean() - ref.mean()) / ref.mean() < 2e-2
    _check_psnr(cfg, means)


@pytest.mark.gpu
@pytest.mark.parametrize("precision", FAST_PRESETS)
def test_train_parity_fast_preset(dev, precision):
    cfg, runs, means = _repeated(dev, precision)
    for _, _, losses, _, ref, rel in runs:
        assert abs(losses.mean() - ref.mean()) / ref.mean() < 2e-2
    _check_psnr(cfg, means)


GOLD_RAW5V = os.path.join(HERE, "golden", "train_parity_raw5v.npz")
GOLD_BG5 = os.path.join(HERE, "golden", "train_parity_bg5.npz")


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["fp32"] + FAST_PRESETS)
def test_train_parity_grid_raw_5mod(dev, precision):
    """BASELINE configs[2] shape (grid_raw, five mosaicked modalities incl. polarization with saturated highlights, the
    45-training-view scene): mean dPSNR over the 16 seeded fixtures within 0.1 dB per modality at every checkpoint of a
    window in which every modality's held-out PSNR rises by several dB, and in which the reference algorithm's own
    scatter (oracle' - oracle, recorded in the fixtures) keeps the 16-seed mean's standard error <= 0.03 dB; for the
    parity and the benchmarked preset."""
    cfg, runs, means = _repeated(dev, precision, GOLD_RAW5V)
    for _, _, losses, _, ref, rel in runs:
        assert rel[:TRAJ_STEPS].max() < (1e-3 if precision == "fp32" else 1e-2)
        assert abs(losses.mean() - ref.mean()) / ref.mean() < 2e-2
    _check_psnr(cfg, means, null_scatter(GOLD_RAW5V))


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["fp32"] + FAST_PRESETS)
def test_train_parity_config5(dev, precision):
    """BASELINE configs[4] shape (grid_raw_grid_bg_unbalanced: rgb + polarization on 10 of its 45 views, hash-grid
    background with 3-layer heads, SO3xR3 pose refinement): the first steps' losses and the seeds' mean dPSNR as the
    raw5 test, against fixtures of the oracle's config-5 path (pinned to the reference by e2e_grid_raw_gridbg_s95000)."""
    cfg, runs, means = _repeated(dev, precision, GOLD_BG5)
    for _, _, losses, _, ref, rel in runs:
        assert rel[:TRAJ_STEPS].max() < (1e-3 if precision == "fp32" else 1e-2)
        assert abs(losses.mean() - ref.mean()) / ref.mean() < 2e-2
    _check_psnr(cfg, means, null_scatter(GOLD_BG5))
