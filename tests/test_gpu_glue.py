"""The step's small fused kernels that replace PyTorch glue, each against the PyTorch expression it replaces:

* mms_pose_exp_fwd/_bwd vs exp_map_SO3xR3 (lie_groups.py:28-63) written in torch ops (fp64), forward and gradient,
  at zero deltas (the clamp branch), small and large rotations;
* mms_hit_gather_fwd/_bwd vs index_select / its autograd (base_model.py:88-93), with repeated indices (padding rows);
* mms_render_stats vs the accumulation / normals / depth renderers (renderers.py:176-242) in torch.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def exp_map_torch(t):
    log_rot = t[:, 3:]
    nrms = (log_rot * log_rot).sum(1)
    ang = torch.clamp(nrms, 1e-4).sqrt()
    inv = 1.0 / ang
    fac1 = inv * ang.sin()
    fac2 = inv * inv * (1.0 - ang.cos())
    B = t.shape[0]
    zero = torch.zeros(B, dtype=t.dtype, device=t.device)
    wx, wy, wz = log_rot[:, 0], log_rot[:, 1], log_rot[:, 2]
    K = torch.stack([zero, -wz, wy, wz, zero, -wx, -wy, wx, zero], -1).view(B, 3, 3)
    R = fac1[:, None, None] * K + fac2[:, None, None] * torch.bmm(K, K) + torch.eye(3, dtype=t.dtype,
                                                                                     device=t.device)[None]
    return torch.cat([R, t[:, :3, None]], dim=-1)


@pytest.mark.parametrize("scale", [0.0, 1e-3, 0.3, 2.0])
def test_pose_exp(dev, scale):
    from multimodalstudio_amd import functions as fx
    g = torch.Generator().manual_seed(3)
    t = (torch.randn(7, 6, generator=g) * scale).to(dev)
    if scale == 0.0:
        t[:, :3] = torch.randn(7, 3, generator=g).to(dev)      # translation only: the clamped-angle branch
    t32 = t.clone().requires_grad_(True)
    m = fx.PoseExpFunction.apply(t32)
    t64 = t.double().requires_grad_(True)
    ref = exp_map_torch(t64)
    assert (m.double() - ref).abs().max().item() < 1e-6
    gm = torch.randn(7, 3, 4, generator=g).to(dev)
    m.backward(gm)
    ref.backward(gm.double())
    err = (t32.grad.double() - t64.grad).abs().max().item()
    assert err < 1e-5 * max(1.0, t64.grad.abs().max().item()), err


def test_hit_gather(dev):
    from multimodalstudio_amd import functions as fx
    g = torch.Generator().manual_seed(5)
    N = 1000
    o, d, u = [torch.randn(N, 3, generator=g).to(dev).requires_grad_(True) for _ in range(3)]
    n, f = [torch.rand(N, generator=g).to(dev).requires_grad_(True) for _ in range(2)]
    idx = torch.randperm(N, generator=g)[:600]
    idx = torch.cat([idx, idx[:1].repeat(40)]).to(dev)           # padding rows repeat the first hit
    outs = fx.HitGatherFunction.apply(idx, o, d, u, n, f)
    refs = [t.index_select(0, idx) for t in (o, d, u, n, f)]
    for a, b in zip(outs, refs):
        assert torch.equal(a, b)
    gs = [torch.randn_like(a) for a in outs]
    got = torch.autograd.grad(outs, (o, d, u, n, f), gs)
    want = torch.autograd.grad(refs, (o, d, u, n, f), gs)
    for a, b in zip(got, want):
        assert (a - b).abs().max().item() < 1e-5


def test_render_stats(dev):
    from multimodalstudio_amd.model import _render_stats
    g = torch.Generator().manual_seed(7)
    R, S, N = 300, 64, 512
    w = torch.rand(R, S, generator=g) / S
    w[:20] *= 1e-3                                                # nearly empty rays: depth below every midpoint
    w = w.to(dev)
    nrm = torch.nn.functional.normalize(torch.randn(R * S, 3, generator=g), dim=-1).to(dev)
    starts = (torch.rand(R * S, generator=g) * 2 + 0.1).to(dev)
    ends = starts + torch.rand(R * S, generator=g).to(dev) * 0.05
    sidx = torch.randperm(N, generator=g)[:R].to(dev)
    stats, _ = _render_stats(w, nrm, starts, ends, R, S, sidx, N, dev)
    acc = torch.zeros(N, 1, device=dev).index_copy_(0, sidx, w.sum(-1, keepdim=True))
    nn_ = torch.zeros(N, 3, device=dev).index_copy_(0, sidx, (w[..., None] * nrm.view(R, S, 3)).sum(1))
    steps = ((starts + ends) / 2).view(R, S)
    dep = torch.zeros(N, 1, device=dev).index_copy_(
        0, sidx, torch.clip((w * steps).sum(-1, keepdim=True), steps.min(), steps.max()))
    assert (stats[:, 0:1] - acc).abs().max().item() < 1e-5
    assert (stats[:, 1:4] - nn_).abs().max().item() < 1e-5
    assert (stats[:, 4:5] - dep).abs().max().item() < 1e-5
    # the lower clip is active for rays with little accumulated weight
    assert (dep[sidx] == steps.min()).any()


def test_weight_prep_batched_matches_single(dev):
    """WeightPrep: after the registering forward, the two batched launches (mms_weight_norm_fwd_batched,
    mms_mlp_pack_batched) reproduce every entry bit for bit against the single-layer mms_weight_norm_fwd /
    mms_mlp_pack, including the backward-orientation images, after a parameter update."""
    from multimodalstudio_amd import functions as fx
    from multimodalstudio_amd.pipeline import TrainConfig, Trainer
    fx.set_precision("fast")
    try:
        t = Trainer(TrainConfig(method="grid", modalities=("rgb",), num_rays_per_modality=256, log2T=12, width=64,
                                height=48, n_views=6), dev)
        t.set_step(95000)
        t.train_step()                        # registers every entry (computed one by one), tables uploaded at its end
        prep = t.model._prep
        assert prep.norm_items and prep.pack_items and not prep.dirty
        assert prep.n_up[0] == len(prep.norm_items) and prep.n_up[2] == len(prep.pack_items)
        t.train_step()                        # batched
        fx.begin_forward(prep, dev)           # one more batched preparation on the updated parameters
        fx.end_forward()
        torch.cuda.synchronize()
        for g, v, W, nrm, idx in prep.norm.values():
            W1, n1 = fx.normed_weight(g, v)   # outside a scope: the single-layer kernel
            assert torch.equal(W, W1) and torch.equal(nrm, n1)
        for key, (W, hi, lo, idx) in prep.pack.items():
            _, _, rows, cols, tr, pm, prec = key
            run = fx.ChainRun([torch.zeros(1)] * 9, [(1, 1.0, 20.0)] * 3, 2 if prec == 3 else prec, chain_prec=prec)
            h1, l1 = run._pack_new(W, rows, cols, tr, pm, prec)
            assert torch.equal(hi, h1) and (lo is None or torch.equal(lo, l1))
    finally:
        fx.set_precision("fp32")


def test_weight_prep_follows_moved_parameters(dev):
    """A forward run BEFORE the trainer's FlatGroup re-points every p.data into its flat buffer: the
    batched preparation must not keep reading the old storage -- the next forward's weights are the current
    parameters' W = g v / ||v||."""
    from multimodalstudio_amd import functions as fx
    from multimodalstudio_amd import model as mm
    from multimodalstudio_amd import pipeline as pl
    fx.set_precision("fast")
    try:
        torch.manual_seed(3)
        model = mm.BaseModel(mm.ModelSpec({"rgb": 3}, log2T=12)).to(dev)
        model.set_step(95000)
        cams = pl.DeviceCameras(mm_cams(), dev)
        gen = pl.RayGenerator({"rgb": cams}, pl.CameraOptimizer(["rgb"], {"rgb": cams.num}, mode="off"), 0.0)
        coords = {"rgb": torch.tensor([[0, 20, 30], [1, 24, 32], [2, 10, 40]], dtype=torch.int32, device=dev)}
        with torch.no_grad():
            model(gen(coords))                 # registers the entries against the original storages
            model(gen(coords))                 # batched tables now in use
        pl.FlatGroup(list(model.parameters()), lr=1e-3, weight_decay=0.01, eps=1e-15)   # moves every p.data
        torch.cuda.empty_cache()
        with torch.no_grad():
            for p in model.parameters():
                p.mul_(1.5)                    # the new storages hold different values than the freed ones
            model(gen(coords))
            model(gen(coords))
            fx.begin_forward(model._prep, dev)
            fx.end_forward()
            torch.cuda.synchronize()
            assert model._prep.norm and all(idx is not None for *_, idx in model._prep.norm.values())
            for g, v, W, nrm, idx in model._prep.norm.values():
                ref = g.reshape(-1, 1) * v / torch.linalg.vector_norm(v, dim=1, keepdim=True)
                assert torch.allclose(W, ref, rtol=1e-5, atol=1e-6)
    finally:
        fx.set_precision("fp32")


def mm_cams():
    from multimodalstudio_amd import scene as ms
    return ms.make_cameras(["rgb"], 6, 64, 48, seed=0)["rgb"]


def test_background_density_only_backward(dev):
    """BackgroundFunction's backward with only the density reaching the loss (the feature gradient
    arrives as None): equals the backward with an explicit zero feature gradient."""
    from multimodalstudio_amd import functions as fx
    from multimodalstudio_amd import model as mm
    torch.manual_seed(5)
    model = mm.BaseModel(mm.ModelSpec({"rgb": 3}, log2T=12)).to(dev)
    pos = (torch.rand(64 * 16, 3, device=dev) - 0.5) * 6
    dirs = torch.nn.functional.normalize(torch.randn(64, 3, device=dev), dim=-1)
    grads = []
    for explicit in (False, True):
        for p in model.parameters():
            p.grad = None
        dens, feat = model.background_model.field(pos, dirs, 16)
        loss = dens.sum() + (0.0 * feat.sum() if explicit else 0.0)
        loss.backward()
        torch.cuda.synchronize()
        grads.append({k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None})
    # the head MLP gets no gradient without the feature's (None there, zeros with the explicit zero gradient)
    assert grads[0] and set(grads[0]) <= set(grads[1])
    for k in grads[1]:
        if k in grads[0]:
            assert torch.allclose(grads[0][k], grads[1][k], rtol=1e-5, atol=1e-7), k
        else:
            assert "head_field" in k and float(grads[1][k].abs().max()) == 0.0, k


def test_weight_norm_bwd_batched_matches_immediate(dev):
    """The training backward's deferred, batched weight-norm gradients (mms_weight_norm_bwd_batched) equal the
    immediate per-layer mms_weight_norm_bwd on the same forward (to float-atomic summation order)."""
    from multimodalstudio_amd import functions as fx
    from multimodalstudio_amd.pipeline import TrainConfig, Trainer
    fx.set_precision("fast")
    try:
        t = Trainer(TrainConfig(method="grid", modalities=("rgb",), num_rays_per_modality=256, log2T=12, width=64,
                                height=48, n_views=6), dev)
        t.set_step(95000)
        coords, sel = t.sampler.sample(t.frames)
        targets = t.targets_for(coords, sel)
        grads = []
        for batched in (True, False):
            t.model.seed_draws(7, dev)
            if batched:
                t.compute_grads(coords, targets)
            else:
                begin, fx.wn_bwd_begin = fx.wn_bwd_begin, lambda: None
                try:
                    t.compute_grads(coords, targets)
                finally:
                    fx.wn_bwd_begin = begin
            torch.cuda.synchronize()
            grads.append(t.fields.grad.clone())
        scale = float(grads[1].abs().max())
        assert float((grads[0] - grads[1]).abs().max()) <= 1e-4 * scale
    finally:
        fx.set_precision("fp32")


def test_inv_variance_equals_torch(dev):
    """mms_inv_variance (the model's reported 1 / inv_variance in one launch) equals SingleVarianceNetwork's torch
    expression 1.0 / exp(10 s).clip(1e-6, 1e6) bit for bit, clip bounds included."""
    from multimodalstudio_amd import _lib
    from multimodalstudio_amd import functions as fx
    for v in (0.3, -0.2, 0.0123, 1.7, -3.0, 2.5, 0.29999):
        s = torch.tensor([v], device=dev)
        out = torch.empty_like(s)
        _lib.call("mms_inv_variance", s.data_ptr(), out.data_ptr(), fx._s())
        ref = 1.0 / torch.exp(s * 10.0).clip(1e-6, 1e6)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), (v, out.item(), ref.item())


@pytest.mark.parametrize("aligned", [True, False])
def test_taps_combine_bwd_geo_columns(dev, aligned):
    """mms_taps_combine_bwd's geo-gradient columns: the centre rows' columns 1..G are the radiance panel gradient's geo
    columns bit for bit, through the float4 path (16-B aligned rows on both sides, columns past G + 1 in the last chunk
    zeroed) and through the element-wise fallback (an unaligned source); column 0 of every row is the sdf gradient of
    the tap formula, the same on both paths."""
    from multimodalstudio_amd import _lib
    from multimodalstudio_amd import functions as fx
    g = torch.Generator().manual_seed(5)
    M, G = 1000, 256
    grads = torch.randn(M, 3, generator=g).to(dev)
    dgrads = torch.randn(M, 3, generator=g).to(dev)
    dhess = torch.randn(M, 3, generator=g).to(dev)
    dsdf = torch.randn(M, 1, generator=g).to(dev)
    panel = torch.randn(M, 320, generator=g).to(dev)   # the radiance panel pitch (16-B rows)
    dgeo = panel[:, 28:28 + G] if aligned else panel[:, 29:29 + G]
    dout = torch.full((5 * M, 260), float("nan"), device=dev)
    _lib.call("mms_taps_combine_bwd", grads.data_ptr(), dgrads.data_ptr(), dhess.data_ptr(), None, M, 4.5e-3, 1.3e-6,
              dout.data_ptr(), dout.stride(0), dsdf.data_ptr(), dsdf.stride(0), dgeo.data_ptr(), dgeo.stride(0), G,
              fx._s())
    torch.cuda.synchronize()
    assert torch.equal(dout[:M, 1:G + 1], dgeo)
    if aligned:
        assert torch.equal(dout[:M, G + 1:], torch.zeros(M, 260 - G - 1, device=dev))
    assert torch.isfinite(dout[:, 0]).all()
    ref = dout[:, 0].clone()
    dout2 = torch.full_like(dout, float("nan"))
    dgeo2 = panel[:, 29:29 + G]     # unaligned: element-wise path
    _lib.call("mms_taps_combine_bwd", grads.data_ptr(), dgrads.data_ptr(), dhess.data_ptr(), None, M, 4.5e-3, 1.3e-6,
              dout2.data_ptr(), dout2.stride(0), dsdf.data_ptr(), dsdf.stride(0), dgeo2.data_ptr(), dgeo2.stride(0), G,
              fx._s())
    torch.cuda.synchronize()
    assert torch.equal(dout2[:, 0], ref)
