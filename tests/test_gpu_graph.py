"""Graph-captured steps (multimodalstudio_amd/graphs.py) against the reference and against the eager path.

* Fixed-capacity foreground batches (BaseModel.forward(cap=...): padding rows repeat the first hit ray) on the
  reference's golden end-to-end vectors, checked at exactly the dynamic path's fp32 bounds
  (test_gpu_e2e.assert_e2e_bounds: loss / radiance / accumulation / depth 1e-4, normals and SDF gradients 2e-3,
  hessians 0.15, bins 2e-5, parameter gradients 2e-3 max and 1e-3 relative L2, pose gradients 5e-3) -- the padding
  rows must change nothing.  The 8-ray fixtures run at cap = N (their largest capacity); the benchmark configuration
  at its own size, with the 64-ray granule bucket_capacity picks, is tests/test_gpu_fullsize.py.
* GraphTrainer replays vs eager Trainer.train_step from the same initial state on the same pixel draws, with the
  sampler jitter off (eval-mode sampler, so both paths see identical samples): per-step losses within 1e-3
  relative over 6 steps (the first is eager, then captures and replays).  Not bit-exact: float-atomic gradient
  sums differ between any two runs, and AdamW (eps 1e-15) turns last-bit differences of near-zero gradients into
  full-size updates.
"""
import numpy as np
import pytest
import torch

from test_gpu_e2e import assert_e2e_bounds, e2e_report, load, print_report, run_hip_e2e

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["e2e_grid_rgb_s95000", "e2e_grid_raw_5mod_s95000", "e2e_grid_raw_5mod_sat_s95000",
                                  "e2e_grid_raw_gridbg_s95000"])
def test_e2e_fixed_capacity(dev, name):
    f = load(name)
    N = f[f"{str(f['mods'][0])}:coords"].shape[0]
    mods, model, pose, outs, losses, total = run_hip_e2e(f, dev, cap=N)
    report = e2e_report(f, mods, model, pose, outs, total, cap=N)
    print_report(name + f" cap={N}", report, mods)
    assert_e2e_bounds(name, report, mods)


@pytest.mark.parametrize("precision,max_iters,start", [("fp32", 100000, 95000), ("fast", 100000, 95000),
                                                       ("fast_h16b", 100000, 95000), ("fast_h16c", 100000, 95000),
                                                       ("fast_h16d", 100000, 95000),
                                                       ("fp32", 50000, 45000)])
def test_graph_trainer_matches_eager(dev, precision, max_iters, start):
    """max_iters 50000: the curvature factor (and every other schedule) follow the run's num_iterations in the
    graph key and in the loss alike.  The fp16 presets replay the padding rows of fixed capacity through
    their row-scaled fp16 paths (all-zero dZ rows beside the real ones)."""
    from multimodalstudio_amd import functions as fx
    from multimodalstudio_amd import graphs
    from multimodalstudio_amd import pipeline as pl
    cfg = pl.TrainConfig(method="grid", modalities=("rgb",), num_rays_per_modality=512, log2T=14, n_views=10,
                         width=160, height=128, max_iters=max_iters)

    def make():
        tr = pl.Trainer(cfg, dev)
        tr.set_step(start)
        tr.model.eval()       # no sampler jitter: both paths see identical samples
        return tr

    fx.set_precision(precision)
    try:
        eager, graphed = make(), make()
        runner = graphs.GraphTrainer(graphed, granule=64)
        le, lg = [], []
        for _ in range(6):
            le.append(float(eager.train_step()[1]))
            lg.append(float(runner.step()[1]))
        torch.cuda.synchronize()
    finally:
        fx.set_precision("fp32")
    le, lg = np.array(le), np.array(lg)
    rel = np.abs(le - lg) / np.abs(le)
    print(precision, runner.stats, le, lg, rel)
    assert runner.disabled is None, runner.disabled
    assert runner.stats["replays"] >= 4 and runner.stats["captures"] >= 1, runner.stats
    assert eager.step == graphed.step and eager.fields.step_count == graphed.fields.step_count
    assert rel.max() < 1e-3


@pytest.mark.parametrize("pose", ["shared", "per_camera", "off"])
def test_fused_hit_count_equals_unfused(dev, pose):
    """graphs.GraphTrainer's tail hit count in one launch (mms_count_hits: pose exp map, ray generation, collider and
    count in one block) equals the four-launch count (RaysFunction + ColliderFunction + mms_compact) for shared and
    per-camera pose deltas of growing size, pixels drawn by the trainer's own sampler."""
    from multimodalstudio_amd import graphs
    from multimodalstudio_amd import pipeline as pl
    cfg = pl.TrainConfig(method="grid", modalities=("rgb",), num_rays_per_modality=2048, log2T=14, n_views=10,
                         width=160, height=128)
    tr = pl.Trainer(cfg, dev)
    if pose != "shared":
        n = tr.cams["rgb"].num
        tr.pose = pl.CameraOptimizer(["rgb"], {"rgb": n}, shared=False, mode="off" if pose == "off" else "SO3xR3").to(dev)
        tr.raygen.pose_optimizer = tr.pose
    runner = graphs.GraphTrainer(tr, granule=64)
    g = torch.Generator().manual_seed(7)
    old = graphs.FUSED_COUNT
    try:
        for scale in (0.0, 1e-3, 3e-2, 0.3):
            if pose != "off":
                with torch.no_grad():
                    pa = tr.pose.pose_adjustment["rgb"]
                    pa.copy_((torch.rand(pa.shape, generator=g) * 2 - 1) * scale)
            runner._stage_inputs()
            counts = []
            for fused in (False, True):
                graphs.FUSED_COUNT = fused
                runner.count_dev.fill_(-1)
                counts.append(runner.hit_counts())
            assert counts[0] == counts[1], (scale, counts)
            assert 0 < counts[0][0] <= 2048
    finally:
        graphs.FUSED_COUNT = old


def test_tail_count_after_eager_steps(dev):
    """after an EAGER step the tail's fused hit count must start from zero (a captured step zeroes the
    counter with its gradients; an eager one does not).  Three eager steps with a tail each: every staged count equals
    the unfused count of the same staged pixels (it used to grow by the previous count every step)."""
    from multimodalstudio_amd import graphs
    from multimodalstudio_amd import pipeline as pl
    cfg = pl.TrainConfig(method="grid", modalities=("rgb",), num_rays_per_modality=512, log2T=14, n_views=10,
                         width=160, height=128, gpu_sampler=True)
    tr = pl.Trainer(cfg, dev)
    tr.set_step(95000)
    runner = graphs.GraphTrainer(tr, granule=64)
    assert runner.tail
    old = graphs.FUSED_COUNT
    runner._stage_inputs()
    try:
        for _ in range(3):
            runner._eager_with_tail(runner.coords)
            runner.count_event.synchronize()
            staged = [int(c) for c in runner.count_host.tolist()]
            graphs.FUSED_COUNT = False
            ref = runner.hit_counts()
            graphs.FUSED_COUNT = old
            assert staged == ref, (staged, ref)
            assert 0 < ref[0] <= 512
    finally:
        graphs.FUSED_COUNT = old


@pytest.mark.parametrize("name", ["e2e_grid_raw_5mod_s95000", "e2e_grid_raw_gridbg_s95000"])
@pytest.mark.parametrize("cap", [None, "granule"])
def test_phase_cut_backward(dev, name, cap):
    """The two-phase backward of the graph-replayed data-parallel step (functions.PHASE_CUT, pipeline.backward_batched
    ``cuts``: the rendering side first, then the SDF side from the cut tensors) gives the single backward's results:
    the loss, the outputs and every parameter and pose gradient to float-atomic summation order (1e-4, or 4x the
    spread of two single backwards of the same step where float-atomic order alone moves a cancelling sum -- e.g. a
    bias gradient -- further); phase 1 alone has already finished the radiance (and grid-background) table gradients
    and left the SDF table's untouched."""
    from multimodalstudio_amd import functions as fx
    from multimodalstudio_amd import pipeline as pl
    from test_gpu_e2e import E2ECase, rel_err
    from test_gpu_fullsize import granule_cap
    f = load(name)
    c = None if cap is None else granule_cap(f)
    runs = []
    for split in (False, False, True):
        case = E2ECase(f, dev)
        rays = case.gen(case.coords)
        cuts = None
        if split:
            cuts = fx.PHASE_CUT[0] = []
        try:
            outs = case.model(rays, case.rng, cap=c)
        finally:
            fx.PHASE_CUT[0] = None
        for m, band in case.band.items():
            outs[m][m] = pl.select_right_channel(outs[m][m], band)
        losses, total = pl.compute_loss(outs, case.targets, case.mods, int(f["step"]))
        phase1 = {}

        def mid():
            torch.cuda.synchronize()
            for k, p in case.model.named_parameters():
                if k.endswith("hash_table"):
                    phase1[k] = None if p.grad is None else p.grad.detach().clone()
        pl.backward_batched(total, mid=mid if split else None, cuts=cuts)
        torch.cuda.synchronize()
        if split:
            assert len(cuts) >= 8, len(cuts)
        grads = {k: p.grad.detach().cpu().clone() for k, p in case.model.named_parameters() if p.grad is not None}
        grads.update({f"pose:{k}": p.grad.detach().cpu().clone() for k, p in case.pose.named_parameters()
                      if p.grad is not None})
        runs.append((float(total), {m: outs[m][m].detach().cpu().clone() for m in case.mods}, grads, phase1))
    (l0, o0, g0, _), (_, _, gn, _), (l1, o1, g1, p1) = runs
    assert abs(l0 - l1) <= 1e-6 * abs(l0)
    for m in o0:
        assert rel_err(o1[m], o0[m]) < 1e-6, m
    assert g0.keys() == g1.keys()
    for k in g0:
        noise = rel_err(gn[k], g0[k])          # two single backwards: float-atomic order alone
        assert rel_err(g1[k], g0[k]) < max(1e-4, 4.0 * noise), (k, rel_err(g1[k], g0[k]), noise)
    for k, g in p1.items():
        if k.startswith("surface_model."):
            assert g is None or float(g.abs().max()) == 0.0, k       # the SDF table: phase 2
        else:
            assert g is not None and rel_err(g.cpu(), g0[k]) < 1e-6, k   # final after phase 1
