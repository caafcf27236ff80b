"""Clip + AdamW + LR schedule of the HIP step (pipeline.FlatGroup: mms_sumsq + one fused mms_adamw launch) against
the reference's own optimizer stack, run here on the host CPU as the reference runs it:

  torch.nn.utils.clip_grad_norm_(max_norm=2.0)   fabric.clip_gradients, base_pipeline.py:232-248
  torch.optim.AdamW(lr, weight_decay=0.01, eps=1e-15)   method_configs.py:260-269 (fields 1e-3, camera_poses 1e-4)
  LambdaLR(MultiStepWarmupScheduler.func)       schedulers.py:249-270, stepped after the optimizer (optimizers.py:101-116)

torch.optim / torch.nn.utils are the reference's implementation of this row (no restatement involved).  Gradients
are drawn both small (clip inactive) and large (clip active), over steps that start at 0 (lr factor 0: a no-op
update, Appendix A.9) and mid-warm-up; parameters and both moments within 2e-6 relative after every step, also in
the graph form (mms_adamw_dev with device-resident scalars).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _reference_run(params0, grads, lr, start, max_iters, max_norm=2.0):
    from multimodalstudio_amd.pipeline import lr_factor
    ps = [torch.nn.Parameter(p.clone()) for p in params0]
    opt = torch.optim.AdamW(ps, lr=lr, weight_decay=0.01, eps=1e-15)
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda s: lr_factor(s, max_iters))
    for _ in range(start):     # LambdaLR counts from 0: advance to the run's start step without updates
        sched.step()
    hist = []
    for g in grads:
        for p, gg in zip(ps, g):
            p.grad = gg.clone()
        torch.nn.utils.clip_grad_norm_(ps, max_norm, error_if_nonfinite=False)
        opt.step()
        sched.step()
        st = [opt.state[p] for p in ps]
        hist.append(([p.detach().clone() for p in ps], [s["exp_avg"].clone() for s in st],
                     [s["exp_avg_sq"].clone() for s in st]))
    return hist


@pytest.mark.parametrize("start,scale,captured", [(0, 1e-3, False), (0, 3.0, False), (4000, 1e-3, False),
                                                  (4000, 3.0, False), (4000, 3.0, True)])
def test_flat_adamw_matches_torch(dev, start, scale, captured):
    from multimodalstudio_amd import pipeline as pl
    g = torch.Generator().manual_seed(17 + start)
    shapes = [(1000, 2), (256, 71), (256,), (1,), (3, 5)]
    params0 = [torch.randn(*s, generator=g) * 0.1 for s in shapes]
    grads = [[torch.randn(*s, generator=g) * scale for s in shapes] for _ in range(4)]
    max_iters, lr = 20000, 1e-3
    ref = _reference_run(params0, grads, lr, start, max_iters)
    ps = [torch.nn.Parameter(p.clone().to(dev)) for p in params0]
    grp = pl.FlatGroup(ps, lr=lr, weight_decay=0.01, eps=1e-15)    # fresh AdamW state (step 0), LR at `start`
    for t, gs in enumerate(grads):
        grp.zero_grad()
        for p, gg in zip(ps, gs):
            p.grad.copy_(gg.to(dev))
        f = pl.lr_factor(start + t, max_iters)
        if captured:
            grp.load_hyper(f)
            grp.step_captured()
        else:
            grp.step(f)
        torch.cuda.synchronize()
        rp, rm, rv = ref[t]
        off = 0
        for i, p in enumerate(ps):
            k = p.numel()
            for name, got, want in [("param", p.detach().cpu(), rp[i]),
                                    ("exp_avg", grp.m[off:off + k].view_as(p).cpu(), rm[i]),
                                    ("exp_avg_sq", grp.v[off:off + k].view_as(p).cpu(), rv[i])]:
                scale_ = want.abs().max().item() + 1e-30
                err = (got - want).abs().max().item() / scale_
                assert err < 2e-6, (t, i, name, err)
            off += k


@pytest.mark.parametrize("scale", [1e-3, 3.0])
def test_optim_bank_equals_per_group(dev, scale):
    """pipeline.OptimBank (both groups zeroed, clipped and stepped in one launch each: mms_zero_multi,
    mms_sumsq_multi, mms_adamw_dev_multi, one scalar upload) against each group's own step_captured: the same
    parameters and moments (bit for bit while the clip is inactive; within 2e-6 relative when active, where the sums
    of squares' float-atomic order may differ), and the sum-of-squares accumulators zeroed by zero_grads."""
    from multimodalstudio_amd import pipeline as pl
    g = torch.Generator().manual_seed(5)
    shapes_a, shapes_b = [(4097, 2), (256, 71), (256,)], [(7, 6), (3,)]
    pa0 = [torch.randn(*s, generator=g) * 0.1 for s in shapes_a]
    pb0 = [torch.randn(*s, generator=g) * 0.1 for s in shapes_b]
    grads = [([torch.randn(*s, generator=g) * scale for s in shapes_a],
              [torch.randn(*s, generator=g) * scale for s in shapes_b]) for _ in range(3)]
    runs = []
    for banked in (False, True):
        pa = [torch.nn.Parameter(p.clone().to(dev)) for p in pa0]
        pb = [torch.nn.Parameter(p.clone().to(dev)) for p in pb0]
        ga = pl.FlatGroup(pa, lr=1e-3, weight_decay=0.01, eps=1e-15)
        gb = pl.FlatGroup(pb, lr=1e-4, weight_decay=0.01, eps=1e-15)
        bank = pl.OptimBank([ga, gb]) if banked else None
        for t, (gsa, gsb) in enumerate(grads):
            if banked:
                ga.sumsq.fill_(123.0)     # stale accumulators: zero_grads must clear them
                gb.sumsq.fill_(7.0)
                bank.zero_grads()
            else:
                ga.zero_grad()
                gb.zero_grad()
            for p, gg in zip(pa, gsa):
                p.grad.copy_(gg.to(dev))
            for p, gg in zip(pb, gsb):
                p.grad.copy_(gg.to(dev))
            f = pl.lr_factor(2500 + t, 20000)
            if banked:
                bank.load_hyper(f)
                bank.step_captured()
            else:
                ga.load_hyper(f)
                gb.load_hyper(f)
                ga.step_captured()
                gb.step_captured()
        torch.cuda.synchronize()
        runs.append([x.detach().cpu().clone() for grp in (ga, gb) for x in (grp.flat, grp.m, grp.v, grp.sumsq)])
        assert ga.step_count == gb.step_count == 3
    for i, (a, b) in enumerate(zip(*runs)):
        if i % 4 == 3:     # sums of squares: float atomics in any order
            assert torch.allclose(a, b, rtol=1e-5), (i, a, b)
        elif scale < 1:
            assert torch.equal(a, b), (i, float((a - b).abs().max()))
        else:
            assert float((a - b).abs().max()) <= 2e-6 * float(b.abs().max()), i
