"""Generate the golden fixtures in tests/golden/*.npz by RUNNING THE REFERENCE (this container only).

    python tests/golden/make_golden.py

The reference (/root/reference/src, pure PyTorch) is imported through tests/golden/refimport.py
(stubs for absent third-party packages + the two SURVEY §8(c) patches).  Fixtures hold inputs,
the reference's outputs and gradients, and every random draw the reference made (captured by
wrapping torch.rand), so the oracle and the HIP path can replay the identical streams.
Nothing here runs on the GPU box; only the .npz data travels.
"""
from __future__ import annotations

import os
import sys
from contextlib import contextmanager

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

import refimport  # noqa: E402

refimport.patch_sh_and_hash()

from multimodalstudio_amd import scene as mscene  # noqa: E402

OUT = HERE
sys.path.insert(0, os.path.dirname(HERE))
from fullsize_state import FULL_SMOOTH_SCALE, fullsize_state, param_checksum  # noqa: E402  (tests/fullsize_state.py)

RAW5 = ["rgb", "infrared", "mono", "polarization", "multispectral"]


def config5_train_views(n_views=50):
    """The training views of grid_raw_rgb_all_views_pol_10_views.yaml (:39-48): every view except the eval views, and
    for polarization also except skip_image_indices_per_modality -- 45 rgb views, 10 polarization views."""
    import yaml
    with open("/root/reference/confs/grid_raw_rgb_all_views_pol_10_views.yaml") as fh:
        dm = yaml.safe_load(fh)["pipeline"]["datamanager"]
    out = {}
    for m in dm["modalities"]:
        drop = set(dm["eval_image_indices_per_modality"][m]) | set(dm["skip_image_indices_per_modality"].get(m, []))
        out[m] = [v for v in range(n_views) if v not in drop]
    return out


def save(name, **arrays):
    path = os.path.join(OUT, name + ".npz")
    clean = {}
    for k, v in arrays.items():
        if isinstance(v, torch.Tensor):
            v = v.detach().cpu().numpy()
        clean[k] = np.asarray(v)
    np.savez_compressed(path, **clean)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB)")


@contextmanager
def record_rand():
    """Capture every torch.rand draw (shape + values) made by the reference."""
    draws = []
    orig = torch.rand

    def rand(*args, **kwargs):
        t = orig(*args, **kwargs)
        draws.append(t.detach().clone())
        return t

    torch.rand = rand
    try:
        yield draws
    finally:
        torch.rand = orig


# ------------------------------------------------------------------------------------------------
def gen_hashgrid():
    from field_components.encodings import HashEncodingConfig
    from field_components.feature_structures import FeatureGridConfig

    torch.manual_seed(0)
    for log2T, active, radius, stored in [(12, 16, 1.0, True), (12, 9, 1.0, True), (13, 16, 2.0, True),
                                         (19, 16, 1.0, False)]:
        cfg = FeatureGridConfig(encoding=HashEncodingConfig(max_res=1024, log2_hashmap_size=log2T,
                                                            interpolation="Linear", implementation="torch"),
                                radius=radius)
        grid = cfg.setup(input_dim=3)
        enc = grid.encoding
        if stored:
            with torch.no_grad():
                enc.hash_table.mul_(100.0)   # features ~0.1 so interpolation errors are visible
        else:
            from oracle.hashgrid import deterministic_table
            with torch.no_grad():
                enc.hash_table.copy_(deterministic_table(16, log2T) * 100.0)
        grid.update_mask(active)
        g = torch.Generator().manual_seed(log2T * 31 + active)
        M = 1024 if stored else 512
        x = (torch.rand(M, 3, generator=g) * 2.4 - 1.2) * radius
        x[:16] = torch.tensor([0.0, 0.5, -0.5]) * radius          # exact lattice points (ceil == floor)
        x.requires_grad_(True)
        out = grid(x)
        dout = torch.randn(out.shape, generator=g)
        out.backward(dout)
        arrays = dict(x=x.detach(), out=out.detach(), dout=dout, dx=x.grad, scales=enc.scalings,
                      log2T=log2T, active=active, radius=radius)
        if stored:
            arrays.update(table=enc.hash_table.detach(), dtable=enc.hash_table.grad)
        else:
            nz = torch.nonzero(enc.hash_table.grad.abs().sum(-1)).squeeze(-1)
            arrays.update(dtable_idx=nz, dtable_val=enc.hash_table.grad[nz])
        save(f"hashgrid_l{log2T}_a{active}_r{int(radius)}", **arrays)


def gen_mlp():
    from field_components.mlp import MLPConfig
    torch.manual_seed(1)
    cases = {
        "geo": (MLPConfig(num_layers=3, hidden_dim=256, activation="Softplus", activation_params={"beta": 100},
                          out_activation="None", geometric_init=True, weight_norm=True, geometric_init_bias=0.4),
                71, 257),
        "rad": (MLPConfig(num_layers=3, hidden_dim=256, out_activation="ReLU", weight_norm=True), 317, 256),
        "head": (MLPConfig(num_layers=3, hidden_dim=64, out_activation="Sigmoid", weight_norm=True), 256, 3),
        "skip": (MLPConfig(num_layers=8, hidden_dim=64, activation="Softplus", activation_params={"beta": 100},
                           out_activation="None", skip_connections=(4,), geometric_init=True, weight_norm=True),
                 39, 65),
    }
    for name, (cfg, din, dout_dim) in cases.items():
        mlp = cfg.setup(input_dim=din, output_dim=dout_dim)
        g = torch.Generator().manual_seed(7)
        x = torch.randn(128, din, generator=g) * 0.5
        x.requires_grad_(True)
        y = mlp(x)
        dy = torch.randn(y.shape, generator=g)
        y.backward(dy)
        arrays = {"x": x.detach(), "y": y.detach(), "dy": dy, "dx": x.grad}
        for k, v in mlp.state_dict().items():
            arrays["p:" + k] = v
        for k, p in mlp.named_parameters():
            arrays["g:" + k] = p.grad
        save(f"mlp_{name}", **arrays)


# ------------------------------------------------------------------------------------------------
def ref_cameras(cams: mscene.ModalityCameras):
    from cameras.cameras import Cameras
    return Cameras(camera_to_worlds=cams.c2w, fx=cams.fx[:, None], fy=cams.fy[:, None], cx=cams.cx[:, None],
                   cy=cams.cy[:, None], width=cams.width, height=cams.height, distortion_params=cams.distortion)


def gen_raygen():
    from cameras.camera_optimizers import CameraOptimizerConfig
    from model_components.ray_generators import RayGenerator
    mods = ["rgb", "polarization"]
    cams = mscene.make_cameras(mods, n_views=12, width=96, height=80, seed=3)
    data = {m: {"cameras": ref_cameras(cams[m])} for m in mods}
    opt = CameraOptimizerConfig(mode="SO3xR3", shared_optimization=True,
                                modalities_to_optimize={m: True for m in mods}).setup(num_cameras=len(cams["rgb"].view_ids))
    with torch.no_grad():
        opt.pose_adjustment["rgb"].copy_(torch.tensor([[0.01, -0.02, 0.015, 0.02, -0.01, 0.005]]))
        opt.pose_adjustment["polarization"].copy_(torch.tensor([[-0.005, 0.01, 0.0, 0.0, 0.0, 0.0]]))
    gen = RayGenerator(data, opt, pixel_offset=0.0)
    g = torch.Generator().manual_seed(5)
    N = 256
    coords = {}
    for m in mods:
        C = len(cams[m].view_ids)
        coords[m] = torch.stack([torch.randint(0, C, (N,), generator=g), torch.randint(0, 80, (N,), generator=g),
                                 torch.randint(0, 96, (N,), generator=g)], -1).to(torch.int32)
    rb = gen(coords)
    arrays = {}
    loss = 0
    for m in mods:
        r = rb[m]
        w = torch.linspace(0.1, 1.0, N)[:, None]
        loss = loss + (r.origins * w).sum() + (r.directions * w * 2).sum() + (r.up_directions * w).sum() \
            + r.pixel_area.sum() * 1e3
        arrays.update({f"{m}:coords": coords[m], f"{m}:origins": r.origins, f"{m}:directions": r.directions,
                       f"{m}:up": r.up_directions, f"{m}:pixel_area": r.pixel_area,
                       f"{m}:directions_norm": r.directions_norm, f"{m}:c2w": cams[m].c2w,
                       f"{m}:fx": cams[m].fx, f"{m}:fy": cams[m].fy, f"{m}:cx": cams[m].cx, f"{m}:cy": cams[m].cy,
                       f"{m}:distortion": cams[m].distortion,
                       f"{m}:pose": opt.pose_adjustment[m].detach()})
    loss.backward()
    for m in mods:
        arrays[f"{m}:dpose"] = opt.pose_adjustment[m].grad
    save("raygen", **arrays)


def gen_sampler():
    """NeuS sampler with an analytic SDF: bit-exact bins / sorted_index fixture."""
    from cameras.rays import RayBundle
    from model_components.ray_samplers import NeuSSamplerConfig
    from model_components.scene_colliders import SphereCollider
    torch.manual_seed(11)
    R = 512
    g = torch.Generator().manual_seed(11)
    o = torch.nn.functional.normalize(torch.randn(R, 3, generator=g), dim=-1) * 2.5
    tgt = torch.randn(R, 3, generator=g) * 0.3
    d = torch.nn.functional.normalize(tgt - o, dim=-1)
    rb = RayBundle(camera_indices=torch.zeros(R, 1, dtype=torch.long), origins=o, directions=d,
                   up_directions=torch.zeros(R, 3), pixel_area=torch.ones(R, 1) * 1e-4)
    rb, mask = SphereCollider(1.0)(rb)
    hit = rb[mask]
    sampler = NeuSSamplerConfig(num_samples=32, num_samples_importance=32).setup()
    sampler.train()

    def sdf_fn(rs):
        p = rs.frustums.get_start_positions()
        return (torch.linalg.norm(p, dim=-1, keepdim=True) - 0.5)

    orig_merge = None
    import model_components.ray_samplers as rsm
    idx_hist = []
    orig_merge = rsm.merge_ray_samples

    def merge(*a, **k):
        rs, si = orig_merge(*a, **k)
        idx_hist.append(si.clone())
        return rs, si

    rsm.merge_ray_samples = merge
    try:
        with record_rand() as draws:
            out = sampler({"rgb": hit}, sdf_fn=sdf_fn)["ray_samples_per_modality"]["rgb"]
    finally:
        rsm.merge_ray_samples = orig_merge
    bins = torch.cat([out.spacing_starts[..., 0], out.spacing_ends[..., -1:, 0]], -1)
    save("neus_sampler", origins=o, directions=d, mask=mask, nears=hit.nears, fars=hit.fars,
         rand_uniform=draws[0], rand_pdf=torch.stack(draws[1:5]), bins=bins, starts=out.frustums.starts[..., 0],
         ends=out.frustums.ends[..., 0], **{f"sorted_index{i}": si for i, si in enumerate(idx_hist)})


# ------------------------------------------------------------------------------------------------
def set_callbacks(model, step, max_iters=100000):
    """Apply the BEFORE_TRAIN_ITERATION callbacks of the reference for ``step``."""
    import numpy as _np
    spl = min(int(max_iters * 1.0), int(max_iters / 16))
    level = min(max(int(step / spl) + 1, 1), 16)
    if hasattr(model.surface_model.surface_field.field, "feature_grid"):      # grid methods only
        model.surface_model.surface_field.field.feature_grid.update_mask(level)
        model.radiance_model.radiance_field.base_field.feature_grid.update_mask(level)
    gfac = _np.exp((_np.log(1024) - _np.log(16)) / 15)
    delta = max(1.0 / 1024, 1.0 / (16 * gfac ** int(step / spl)))
    model.surface_model.set_numerical_gradients_delta(delta * 2.0)
    model.surface_model.volume_rendering.set_cos_anneal_ratio(min(1.0, step / int(max_iters * 0.05)))
    return level, delta * 2.0


def gen_end_to_end(method, yaml_name, mods, step, tag, n_rays=8, log2T=12, raw=False, grid_bg=False, grids=True,
                   saturate=0.0, W=96, H=80, n_views=12, cam_seed=4, state=None, compact=False, amp_scale=None,
                   write=True, keep_table_grads=None, train_views=None, state_meta=None, inject_bins=None):
    """One reference fwd + loss + bwd.  ``saturate``: that fraction of the polarization frame values is set to 1.0,
    so targets above SkipSaturationLoss's 0.998 threshold (losses.py:152-164) are drawn.  ``state``: load these
    parameters (fullsize_state) instead of the seeded reference init; ``compact``: store no parameters and, of the
    hash-table gradients, per-level norms plus a fixed sample of their nonzero entries (the full-size fixture).
    ``amp_scale``: the reference's own "16-mixed" mode (autocast16.py: the model forward under CUDA's fp16 autocast
    policy, the loss scaled by this power of two before the backward and the gradients unscaled after it, as Fabric's
    GradScaler; arrays["amp_finite"] = its inf / nan check).  ``write``: save the fixture, else only return it.
    ``keep_table_grads``: a dict that receives the full hash-table gradients of a compact run.  ``train_views``: per
    modality, the view ids whose frames the pixel sampler draws from (the datamanager's training split after
    skip_image_indices_per_modality, datasets.py); default every view.  ``state_meta``: extra scalars stored with a
    compact fixture so tests/fullsize_state.py regenerates the same parameters (background kind, table scale).
    ``inject_bins``: per modality, final NeuS spacing bins that replace the up-sampler's (it still runs, so every
    random draw is made as before), built into RaySamples exactly as merge_ray_samples builds them
    (ray_samplers.py:58-66) -- the rest of the step then runs on those samples."""
    from cameras.camera_optimizers import CameraOptimizerConfig
    from cameras.pixel_samplers import UniformPixelSamplerConfig
    from model_components.ray_generators import RayGenerator
    torch.manual_seed(1234)
    modalities = {m: mscene.CHANNELS[m] for m in mods}
    overrides = {"pipeline": {"model": {
        "surface_model": {"surface_field": {"field": {"feature_grid": {"encoding": {"log2_hashmap_size": log2T}}}}},
        "radiance_model": {"radiance_field": {"base_field": {"feature_grid": {"encoding": {"log2_hashmap_size": log2T}}}}},
    }}}
    if grid_bg:
        overrides["pipeline"]["model"]["background_model"] = {"background_field": {"base_field": {
            "feature_grid": {"encoding": {"log2_hashmap_size": log2T}}}}}
    if not grids:
        overrides = None
    cfg, model = refimport.build_model(method, f"/root/reference/confs/{yaml_name}", modalities, overrides)
    model.train()
    if state is not None:
        model.load_state_dict(state, strict=True)
    else:
        with torch.no_grad():
            # widen the tiny init so every stage carries signal
            for n, p in model.named_parameters():
                if n.endswith("hash_table"):
                    p.mul_(50.0)
    level, delta = set_callbacks(model, step)
    cams = mscene.make_cameras(mods, n_views=n_views, width=W, height=H, seed=cam_seed)
    data = {m: {"cameras": ref_cameras(cams[m])} for m in mods}
    opt = CameraOptimizerConfig(mode="SO3xR3", shared_optimization=True,
                                modalities_to_optimize={m: True for m in mods}).setup(num_cameras=len(cams[mods[0]].view_ids))
    with torch.no_grad():
        for i, m in enumerate(mods):
            opt.pose_adjustment[m].copy_(torch.tensor([[0.004 * (i + 1), -0.003, 0.002, 0.003, -0.002 * (i + 1), 0.001]]))
    gen = RayGenerator(data, opt, pixel_offset=0.0)
    # frames + pixel sampler (pixel_samplers.py:71-89)
    frames = {}
    for m in mods:
        C = len(cams[m].view_ids)
        imgs = torch.rand(C, H, W, 1 if raw else modalities[m], generator=torch.Generator().manual_seed(9))
        if saturate > 0 and m == "polarization":
            imgs[imgs > 1.0 - saturate] = 1.0
        idx = torch.arange(C, dtype=torch.int32)
        if train_views is not None and m in train_views:
            # view ids -> positions in the camera list (make_cameras keeps the train split: eval views absent)
            idx = torch.tensor([cams[m].view_ids.index(v) for v in sorted(train_views[m])], dtype=torch.int32)
            imgs = imgs[idx.long()]
        frames[m] = {"images": imgs, "indexes": idx}
    sampler = UniformPixelSamplerConfig(num_rays_per_modality=n_rays).setup(device=None)
    sampler.generator = torch.Generator()
    sampler.generator.manual_seed(654824)
    coords, pixels = sampler.sample(frames)
    rb = gen(coords)
    # record the collider masks and the sampler's final spacing bins per modality (base_model.py:86-95)
    import model_components.scene_colliders as scm
    import model_components.ray_samplers as rsm
    seen = {}
    orig_update = scm.ColliderInstancer.update_ray_bundles
    orig_gen = rsm.NeuSSampler.generate_ray_samples

    def update(self, bundles):
        masks = orig_update(self, bundles)
        seen.setdefault("masks", {k: v.clone() for k, v in masks.items()})
        return masks

    orig_merge = rsm.merge_ray_samples

    def merge(*a, **k):
        out = orig_merge(*a, **k)
        seen.setdefault("sorted_index", []).append(out[1].detach().clone())
        return out

    def generate(self, *a, **k):
        bundles = k.get("ray_bundles", a[0] if a else None)
        seen["hit_rays"] = {m: (b.origins.detach().clone(), b.directions.detach().clone(), b.nears.detach().clone(),
                                b.fars.detach().clone()) for m, b in bundles.items()}
        fn = k["sdf_fn"]

        def sdf_fn(samples):
            v = fn(samples)
            seen.setdefault("sdf_calls", []).append(v.detach().clone())
            return v
        k = dict(k, sdf_fn=sdf_fn)
        out = orig_gen(self, *a, **k)
        if inject_bins is not None:
            rsm_out = out["ray_samples_per_modality"]
            for m, rs in list(rsm_out.items()):
                b = inject_bins[m].to(rs.spacing_starts.dtype)
                eb = rs.spacing_to_euclidean_fn(b, bundles[m])
                rsm_out[m] = bundles[m].get_ray_samples(bin_starts=eb[..., :-1, None], bin_ends=eb[..., 1:, None],
                                                        spacing_starts=b[..., :-1, None], spacing_ends=b[..., 1:, None],
                                                        spacing_to_euclidean_fn=rs.spacing_to_euclidean_fn)
        seen["bins"] = {m: torch.cat([rs.spacing_starts[..., 0], rs.spacing_ends[..., -1:, 0]], -1).detach().clone()
                        for m, rs in out["ray_samples_per_modality"].items()}
        return out

    scm.ColliderInstancer.update_ray_bundles = update
    rsm.NeuSSampler.generate_ray_samples = generate
    rsm.merge_ray_samples = merge
    try:
        with record_rand() as draws:
            if amp_scale is not None:
                import autocast16
                with autocast16.CudaAutocastFp16():
                    outputs = model(rb)
            else:
                outputs = model(rb)
    finally:
        scm.ColliderInstancer.update_ray_bundles = orig_update
        rsm.NeuSSampler.generate_ray_samples = orig_gen
        rsm.merge_ray_samples = orig_merge
    # loss (raw_pipeline.py:112-122 + losses.py)
    lm = cfg.pipeline.loss_manager.setup(modalities=list(mods), num_iterations=100000, model=model)
    if raw:
        for m in mods:
            mm = mscene.mosaick_mask(m, W, H)
            band = mm[coords[m][:, 1].long(), coords[m][:, 2].long()].unsqueeze(1).long()
            outputs[m][m] = torch.gather(outputs[m][m], 1, band)
    losses, total = lm.compute_loss(outputs, pixels, coords, step)
    arrays = {}
    if amp_scale is not None:
        (total * amp_scale).backward()
        params = list(model.parameters()) + list(opt.parameters())
        arrays["amp_finite"] = all(p.grad is None or bool(torch.isfinite(p.grad).all()) for p in params)
        with torch.no_grad():
            for p in params:
                if p.grad is not None:
                    p.grad.mul_(1.0 / amp_scale)
        arrays["amp_scale"] = float(amp_scale)
    else:
        total.backward()
    arrays.update({"step": step, "level": level, "delta": delta, "W": W, "H": H, "raw": raw,
                   "mods": np.array(mods), "loss": total.detach()})
    for k, v in losses.items():
        arrays["loss:" + k] = torch.as_tensor(v).detach()
    if compact:
        arrays["param_checksum"] = param_checksum(model.state_dict())
        arrays["log2T"] = log2T
        for k, v in (state_meta or {}).items():
            arrays["state:" + k] = v
    else:
        for k, v in model.state_dict().items():
            arrays["p:" + k] = v
    gs = torch.Generator().manual_seed(77)
    for k, p in model.named_parameters():
        if p.grad is None:
            continue
        if compact and k.endswith("hash_table"):
            if keep_table_grads is not None:
                keep_table_grads[k] = p.grad.detach().clone()
            g = p.grad.detach().reshape(16, -1).double()
            arrays["gtab_level_norm:" + k] = g.norm(dim=1)
            flat = p.grad.detach().reshape(-1)
            nz = torch.nonzero(flat).reshape(-1)
            pick = nz[torch.randperm(nz.numel(), generator=gs)[:32768]].sort().values
            arrays["gtab_idx:" + k] = pick.to(torch.int32)
            arrays["gtab_val:" + k] = flat[pick]
        else:
            arrays["g:" + k] = p.grad
    for i, d in enumerate(draws):
        arrays[f"rand:{i}"] = d
    for m in mods:
        arrays[f"{m}:coords"] = coords[m]
        arrays[f"{m}:pixels"] = pixels[m]
        arrays[f"{m}:pose"] = opt.pose_adjustment[m].detach()
        arrays[f"{m}:dpose"] = opt.pose_adjustment[m].grad
        for k in ["c2w", "fx", "fy", "cx", "cy", "distortion"]:
            arrays[f"{m}:{k}"] = getattr(cams[m], k)
        arrays[f"{m}:mask"] = seen["masks"][m]
        arrays[f"{m}:bins"] = seen["bins"][m]
        if compact:
            # the up-sampler's inputs and every iteration's SDF values and sorted_index (modalities run one after
            # another, 4 iterations each): the full-size sampler is checked bit-exactly given these
            i = mods.index(m)
            o_h, d_h, n_h, f_h = seen["hit_rays"][m]
            arrays[f"{m}:hit:origins"], arrays[f"{m}:hit:directions"] = o_h, d_h
            arrays[f"{m}:hit:nears"], arrays[f"{m}:hit:fars"] = n_h, f_h
            for it in range(4):
                arrays[f"{m}:sampler:sdf{it}"] = seen["sdf_calls"][4 * i + it].reshape(n_h.shape[0], -1)
                arrays[f"{m}:sampler:sorted_index{it}"] = seen["sorted_index"][4 * i + it].to(torch.uint8)
        o = outputs[m]
        for k in ["normals", "depth", "accumulation", "gradients", "hessians", "inv_s"]:
            if o.get(k) is not None:
                arrays[f"{m}:out:{k}"] = o[k].detach()
        for mm in mods:
            if mm in o:
                arrays[f"{m}:out:{mm}"] = o[mm].detach()
    if write:
        save(f"e2e_{tag}", **arrays)
    return arrays


def gen_eval(method="grid", yaml_name="grid.yaml", mods=("rgb",), step=95000, tag="eval_grid_rgb", raw=False):
    """Evaluation-mode full-view rendering (Evaluator.render_view -> eval_model_query, evaluator.py:100-178,
    eval_utils.py:31-76): every pixel of one small view, model in eval mode under no_grad (no jitter anywhere)."""
    from cameras.camera_optimizers import CameraOptimizerConfig
    from model_components.ray_generators import RayGenerator
    torch.manual_seed(1234)
    modalities = {m: mscene.CHANNELS[m] for m in mods}
    overrides = {"pipeline": {"model": {
        "surface_model": {"surface_field": {"field": {"feature_grid": {"encoding": {"log2_hashmap_size": 12}}}}},
        "radiance_model": {"radiance_field": {"base_field": {"feature_grid": {"encoding": {"log2_hashmap_size": 12}}}}},
    }}}
    cfg, model = refimport.build_model(method, f"/root/reference/confs/{yaml_name}", modalities, overrides)
    with torch.no_grad():
        for n, p in model.named_parameters():
            if n.endswith("hash_table"):
                p.mul_(50.0)
    set_callbacks(model, step)
    model.eval()
    W, H = 24, 20
    cams = mscene.make_cameras(list(mods), n_views=12, width=W, height=H, seed=4)
    data = {m: {"cameras": ref_cameras(cams[m])} for m in mods}
    opt = CameraOptimizerConfig(mode="SO3xR3", shared_optimization=True,
                                modalities_to_optimize={m: True for m in mods}).setup(num_cameras=len(cams[mods[0]].view_ids))
    with torch.no_grad():
        for i, m in enumerate(mods):
            opt.pose_adjustment[m].copy_(torch.tensor([[0.004 * (i + 1), -0.003, 0.002, 0.003, -0.002 * (i + 1), 0.001]]))
    gen = RayGenerator(data, opt, pixel_offset=0.0)
    view = 3
    ys, xs = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
    coords = {m: torch.stack([torch.full((H * W,), view), ys.reshape(-1), xs.reshape(-1)], -1).to(torch.int32)
              for m in mods}
    with torch.no_grad():
        rb = gen(coords)
        outputs = model(rb)
    arrays = {"step": step, "W": W, "H": H, "view": view, "raw": raw, "mods": np.array(mods)}
    for k, v in model.state_dict().items():
        arrays["p:" + k] = v
    gt = torch.rand(H, W, 3, generator=torch.Generator().manual_seed(3))
    arrays["gt"] = gt
    for m in mods:
        arrays[f"{m}:pose"] = opt.pose_adjustment[m].detach()
        for k in ["c2w", "fx", "fy", "cx", "cy", "distortion"]:
            arrays[f"{m}:{k}"] = getattr(cams[m], k)
        o = outputs[m]
        for k in ["normals", "depth", "accumulation", m]:
            arrays[f"{m}:out:{k}"] = o[k].detach().reshape(H, W, -1)
    save(tag, **arrays)


def gen_plugins():
    """Reference-signature modules on their own: SDFField.forward (surface_field.py:99-116), RadianceField.forward
    (radiance_field.py:72-77) and Renderer.render (renderers.py:75-136), forward and backward."""
    from cameras.rays import Frustums
    from model_components.renderers import RadianceRenderer, RendererConfig
    overrides = {"pipeline": {"model": {
        "surface_model": {"surface_field": {"field": {"feature_grid": {"encoding": {"log2_hashmap_size": 12}}}}},
        "radiance_model": {"radiance_field": {"base_field": {"feature_grid": {"encoding": {"log2_hashmap_size": 12}}}}},
    }}}
    torch.manual_seed(21)
    _, model = refimport.build_model("grid", "/root/reference/confs/grid.yaml", {"rgb": 3}, overrides)
    sf = model.surface_model.surface_field
    rf = model.radiance_model.radiance_field
    with torch.no_grad():
        for n, p in list(sf.named_parameters()) + list(rf.named_parameters()):
            if n.endswith("hash_table"):
                p.mul_(50.0)
    sf.field.feature_grid.update_mask(12)
    rf.base_field.feature_grid.update_mask(14)
    g = torch.Generator().manual_seed(22)
    M = 256
    arrays = {"sdf_level": 12, "rad_level": 14}
    # SDFField
    x = (torch.rand(M, 3, generator=g) * 2.2 - 1.1).requires_grad_(True)
    sdf, geo = sf(x)
    dsdf, dgeo = torch.randn(sdf.shape, generator=g), torch.randn(geo.shape, generator=g) * 0.01
    (sdf * dsdf).sum().add_((geo * dgeo).sum()).backward()
    arrays.update({"sdf:x": x.detach(), "sdf:sdf": sdf.detach(), "sdf:geo": geo.detach(), "sdf:dsdf": dsdf,
                   "sdf:dgeo": dgeo, "sdf:dx": x.grad})
    for k, v in sf.state_dict().items():
        arrays["sdf:p:" + k] = v
    for k, p in sf.named_parameters():
        arrays["sdf:g:" + k] = p.grad
    # RadianceField: positions, SH(4) directions (25), additional [geo 256, n.v]
    pos = (torch.rand(M, 3, generator=g) * 2 - 1).requires_grad_(True)
    vd = (torch.rand(M, rf.input_dim - 3 - 257, generator=g) * 2 - 1).requires_grad_(True)
    extra = (torch.randn(M, 257, generator=g) * 0.3).requires_grad_(True)
    feat = rf(pos, vd, extra)
    dfeat = torch.randn(feat.shape, generator=g)
    (feat * dfeat).sum().backward()
    arrays.update({"rad:pos": pos.detach(), "rad:vd": vd.detach(), "rad:extra": extra.detach(),
                   "rad:out": feat.detach(), "rad:dout": dfeat, "rad:dpos": pos.grad, "rad:dvd": vd.grad,
                   "rad:dextra": extra.grad})
    for k, v in rf.state_dict().items():
        arrays["rad:p:" + k] = v
    for k, p in rf.named_parameters():
        arrays["rad:g:" + k] = p.grad
    # Renderer: rgb composited over a background, normals, depth, accumulation
    N, S = 96, 16
    mask = torch.rand(N, generator=g) < 0.7
    R = int(mask.sum())
    w = (torch.rand(R, S, 1, generator=g) * 0.12).requires_grad_(True)
    rgb = torch.rand(R, S, 3, generator=g).requires_grad_(True)
    bg = torch.rand(N, 3, generator=g).requires_grad_(True)
    normals = torch.randn(R, S, 3, generator=g)
    starts = torch.sort(torch.rand(R, S, 1, generator=g) * 2 + 0.5, dim=1)[0]
    ends = starts + 0.05
    fr = Frustums(origins=torch.zeros(R, S, 3), directions=torch.zeros(R, S, 3), starts=starts, ends=ends,
                  pixel_area=torch.ones(R, S, 1))

    class _RS:
        frustums = fr

    renderer = RendererConfig(renderers={"rgb": RadianceRenderer}).setup()
    # render() writes the hit rows into the background tensor it is given (renderers.py:97-105): pass a non-leaf copy
    outs = renderer.render(w, {"rgb": rgb, "background": {"rgb": bg.clone()}, "normals": normals, "depth": _RS()},
                           mask)
    drgb = torch.randn(N, 3, generator=g)
    (outs["rgb"] * drgb).sum().add_(outs["accumulation"].sum()).backward()
    arrays.update({"ren:mask": mask, "ren:w": w.detach(), "ren:rgb": rgb.detach(), "ren:bg": bg.detach(),
                   "ren:normals": normals, "ren:starts": starts, "ren:ends": ends, "ren:drgb": drgb,
                   "ren:dw": w.grad, "ren:dvals": rgb.grad, "ren:dbg": bg.grad})
    for k in ["rgb", "normals", "depth", "accumulation"]:
        arrays["ren:out:" + k] = outs[k].detach()
    save("plugins", **arrays)


LOADER_SCENES = {
    # (raw, modalities, per-modality frame format, excluded frame ids): all-npy scenes (the reference reads npy with
    # np.load; its png path needs OpenCV, absent here), float32 and uint16 frames (normalize_frame)
    "raw": (True, ("rgb", "infrared", "mono", "polarization", "multispectral"),
            {"rgb": "npy", "infrared": "npy_u16", "mono": "npy", "polarization": "npy", "multispectral": "npy_u16"},
            (1, 4)),
    "demosaicked": (False, ("rgb", "mono", "multispectral"), {"rgb": "npy", "mono": "npy_u16", "multispectral": "npy"},
                    (2,)),
}
LOADER_SHAPE = dict(n_views=7, width=40, height=26, seed=3)


def gen_loader():
    """RawMultimodalAlignedDataset / MultimodalAlignedDataset (datasets.py:229-301, 303-360, 444-529, 608-633) loading
    scenes written by data.write_synthetic_scene: frames, cameras, mosaick masks and channel counts."""
    import tempfile
    from data.datasets import (MultimodalAlignedDataset, MultimodalAlignedDatasetConfig, RawMultimodalAlignedDataset,
                               RawMultimodalAlignedDatasetConfig)
    from multimodalstudio_amd import data as md
    out = {}
    for tag, (raw, mods, fmts, excl) in LOADER_SCENES.items():
        with tempfile.TemporaryDirectory() as d:
            md.write_synthetic_scene(d, mods, raw=raw, formats=fmts, **LOADER_SHAPE)
            if raw:
                ds = RawMultimodalAlignedDataset(RawMultimodalAlignedDatasetConfig(), mods, d,
                                                 indexes_to_exclude=list(excl))
            else:
                ds = MultimodalAlignedDataset(MultimodalAlignedDatasetConfig(), mods, d, indexes_to_exclude=list(excl))
            out[f"{tag}:indexes"] = np.array(ds.indexes)
            ch = ds.get_channels_per_modality()
            for m in mods:
                cam = ds.data[m]["cameras"]
                out[f"{tag}:{m}:images"] = ds.data[m]["images"]
                out[f"{tag}:{m}:c2w"] = cam.camera_to_worlds
                for k in ("fx", "fy", "cx", "cy"):
                    out[f"{tag}:{m}:{k}"] = getattr(cam, k)
                out[f"{tag}:{m}:distortion"] = cam.distortion_params
                out[f"{tag}:{m}:channels"] = np.int64(ch[m])
                if raw:
                    out[f"{tag}:{m}:mosaick_mask"] = ds.mosaick_mask_per_modality[m]
            out[f"{tag}:radius"] = np.float64(ds.scene_box.radius)
    save("loader", **out)


def analytic_sdf(p: torch.Tensor) -> torch.Tensor:
    """The mesh fixture's surface: a sphere (r 0.45 about (0.1, -0.05, 0.2)) united with a torus (R 0.6, r 0.12, axis z),
    evaluated in float32 from the (float16) grid points.  tests/test_gpu_mesh.py evaluates the same expression."""
    p = p.float()
    c = torch.tensor([0.1, -0.05, 0.2], dtype=torch.float32)
    sphere = torch.sqrt(((p - c) ** 2).sum(-1)) - 0.45
    q = torch.sqrt(p[:, 0] ** 2 + p[:, 1] ** 2) - 0.6
    torus = torch.sqrt(q ** 2 + p[:, 2] ** 2) - 0.12
    return torch.minimum(sphere, torus)


def gen_mesh(resolution=512, n_sample=65536):
    """get_surface_sliding (/root/reference/src/utils/marching_cubes.py:35-171) on the analytic SDF with its
    skimage.measure.marching_cubes call (:158) intercepted: per crop, the points each pyramid level evaluated (from the
    reference's 100000-point evaluation chunks), and the crop's final volume z (the marching-cubes input) as its sign
    census, float64 sum and a fixed random sample of entries.  skimage / trimesh are absent here: the triangulation
    itself stays unpinned.  The reference moves points to .cuda(); on this CPU-only container that is the identity."""
    import utils.marching_cubes as rmc
    chunks, vols = [], []

    def sdf_fn(pnts):
        chunks.append(int(pnts.shape[0]))
        return analytic_sdf(pnts)

    def fake_mc(volume, level, spacing, mask=None):
        vols.append((len(chunks), np.array(volume, dtype=np.float32, copy=True), tuple(float(x) for x in spacing)))
        return np.zeros((0, 3)), np.zeros((0, 3), dtype=np.int64), np.zeros((0, 3)), np.zeros(0)

    rmc.measure.marching_cubes = fake_mc
    import types
    rmc.trimesh = types.SimpleNamespace(Trimesh=lambda *a, **k: None,
                                        util=types.SimpleNamespace(concatenate=lambda meshes: meshes))
    # the CPU has no float16 avg_pool3d: the GPU kernel's arithmetic (fp32 sum of the 8 halves -- exact --, / 8,
    # rounded to half) restated
    pool = rmc.avg_pool_3d
    rmc.avg_pool_3d = lambda x: pool(x.float()).half() if x.dtype == torch.float16 else pool(x)
    orig_cuda = torch.Tensor.cuda
    torch.Tensor.cuda = lambda self, *a, **k: self
    try:
        rmc.get_surface_sliding(sdf_fn, resolution=resolution, return_mesh=True)
    finally:
        torch.Tensor.cuda = orig_cuda
        rmc.avg_pool_3d = pool
    # evaluation chunks -> per-level counts: a level's chunks are 100000 points each but its last
    levels, acc = [], 0
    for c in chunks:
        acc += c
        if c < 100000:
            levels.append(acc)
            acc = 0
    n_crops = (resolution // 256) ** 3
    assert len(levels) == 4 * n_crops, (len(levels), n_crops)
    out = {"resolution": np.int64(resolution), "level_counts": np.array(levels, dtype=np.int64).reshape(n_crops, 4)}
    g = np.random.default_rng(7)
    idx = g.choice(256 ** 3, n_sample, replace=False).astype(np.int64)
    out["sample_index"] = idx
    crops = []
    for ci, (_, vol, spacing) in enumerate(vols):
        # the crop this call belongs to: the one whose 4 levels the evaluation chunks just completed
        done, acc, lv = 0, 0, 0
        for c in chunks[:_]:
            acc += c
            if c < 100000:
                lv += 1
                acc = 0
        crop = lv // 4 - 1
        crops.append(crop)
        z = vol.reshape(-1)
        out[f"crop{crop}:neg"] = np.int64((z < 0).sum())
        out[f"crop{crop}:sum"] = np.float64(z.astype(np.float64).sum())
        out[f"crop{crop}:sample"] = z[idx]
        out[f"crop{crop}:spacing"] = np.array(spacing)
    out["surface_crops"] = np.array(crops, dtype=np.int64)
    save("mesh_pyramid", **out)


if __name__ == "__main__":
    which = sys.argv[1:] or ["hashgrid", "mlp", "raygen", "sampler", "e2e", "plugins", "eval", "loader", "mesh"]
    if "mesh" in which:
        gen_mesh()
    if "loader" in which:
        gen_loader()
    if "eval" in which:
        gen_eval()
    if "plugins" in which:
        gen_plugins()
    if "hashgrid" in which:
        gen_hashgrid()
    if "mlp" in which:
        gen_mlp()
    if "raygen" in which:
        gen_raygen()
    if "sampler" in which:
        gen_sampler()
    if "e2e" in which:
        gen_end_to_end("grid", "grid.yaml", ["rgb"], 95000, "grid_rgb_s95000")
        gen_end_to_end("grid", "grid.yaml", ["rgb"], 30000, "grid_rgb_s30000")
        # same seed -> same init: keep the parameters only once (s95000 file)
        a = dict(np.load(os.path.join(OUT, "e2e_grid_rgb_s95000.npz")))
        b = dict(np.load(os.path.join(OUT, "e2e_grid_rgb_s30000.npz")))
        assert all(np.array_equal(a[k], b[k]) for k in a if k.startswith("p:"))
        b = {k: v for k, v in b.items() if not k.startswith("p:")}
        b["params_from"] = np.array("e2e_grid_rgb_s95000")
        np.savez_compressed(os.path.join(OUT, "e2e_grid_rgb_s30000.npz"), **b)
        gen_end_to_end("grid_raw", "grid_raw.yaml", ["rgb", "infrared", "mono", "polarization", "multispectral"],
                       95000, "grid_raw_5mod_s95000", raw=True)
    if "e2e_sat" in which or "e2e" in which:
        # the 5-modality step with saturated polarization targets (SkipSaturationLoss active), 16 rays per modality;
        # same seed and modalities -> same init as e2e_grid_raw_5mod_s95000, whose parameters it shares
        gen_end_to_end("grid_raw", "grid_raw.yaml", ["rgb", "infrared", "mono", "polarization", "multispectral"],
                       95000, "grid_raw_5mod_sat_s95000", n_rays=16, raw=True, saturate=0.2)
        a = dict(np.load(os.path.join(OUT, "e2e_grid_raw_5mod_s95000.npz")))
        b = dict(np.load(os.path.join(OUT, "e2e_grid_raw_5mod_sat_s95000.npz")))
        assert all(np.array_equal(a[k], b[k]) for k in a if k.startswith("p:"))
        b = {k: v for k, v in b.items() if not k.startswith("p:")}
        b["params_from"] = np.array("e2e_grid_raw_5mod_s95000")
        np.savez_compressed(os.path.join(OUT, "e2e_grid_raw_5mod_sat_s95000.npz"), **b)
    if "e2e_mlp" in which or "e2e" in which:
        # config 1: mlp_raw, analytic SDF gradients (double backward), skip-connection MLPs, RGB only
        gen_end_to_end("mlp_raw", "mlp_raw.yaml", ["rgb"], 95000, "mlp_raw_rgb_s95000", raw=True, grids=False)
    if "e2e_gridbg" in which or "e2e" in which:
        # config 5: grid background (hash grid r = 2 + MLP), 3-layer background heads, rgb + polarization
        gen_end_to_end("grid_raw_grid_bg_unbalanced", "grid_raw_rgb_all_views_pol_10_views.yaml",
                       ["rgb", "polarization"], 95000, "grid_raw_gridbg_s95000", raw=True, grid_bg=True)
    if "e2e_gridbg30" in which or "e2e" in which:
        # config 5 at step 30000: the surface / radiance grids at 5 active levels while the background grid keeps all 16
        # (BackgroundModel registers no callbacks, background_model.py:120-125); parameters shared with the s95000 file
        gen_end_to_end("grid_raw_grid_bg_unbalanced", "grid_raw_rgb_all_views_pol_10_views.yaml",
                       ["rgb", "polarization"], 30000, "grid_raw_gridbg_s30000", raw=True, grid_bg=True)
        a = dict(np.load(os.path.join(OUT, "e2e_grid_raw_gridbg_s95000.npz")))
        b = dict(np.load(os.path.join(OUT, "e2e_grid_raw_gridbg_s30000.npz")))
        assert all(np.array_equal(a[k], b[k]) for k in a if k.startswith("p:"))
        b = {k: v for k, v in b.items() if not k.startswith("p:")}
        b["params_from"] = np.array("e2e_grid_raw_gridbg_s95000")
        np.savez_compressed(os.path.join(OUT, "e2e_grid_raw_gridbg_s30000.npz"), **b)
    if "e2e_full_raw5" in which:
        # BASELINE configs[2] at its own size: grid_raw.yaml, five mosaicked modalities x 2048 rays
        # (/root/reference/confs/grid_raw.yaml:39-67), log2T 19, step 95000, the 50-view 640 x 512 rig
        gen_end_to_end("grid_raw", "grid_raw.yaml", RAW5, 95000, "full_grid_raw5_l19", n_rays=2048, log2T=19, W=640,
                       H=512, n_views=50, cam_seed=0, raw=True, state=fullsize_state(RAW5, 19), compact=True)
    if "e2e_full_bg" in which:
        # BASELINE configs[4] per GPU at its own size: grid_raw_rgb_all_views_pol_10_views.yaml -- rgb + polarization x
        # 2048 rays, polarization drawn from its 10 training views (skip_image_indices_per_modality and the eval
        # views removed, :39-48), hash-grid background, SO3xR3 poses; log2T 19, step 95000
        bg_mods = ["rgb", "polarization"]
        gen_end_to_end("grid_raw_grid_bg_unbalanced", "grid_raw_rgb_all_views_pol_10_views.yaml", bg_mods, 95000,
                       "full_gridbg_l19", n_rays=2048, log2T=19, W=640, H=512, n_views=50, cam_seed=0, raw=True,
                       grid_bg=True, state=fullsize_state(bg_mods, 19, bg_kind="grid"), compact=True,
                       train_views=config5_train_views(), state_meta={"bg_kind": "grid"})
    if "e2e_full_smooth" in which:
        # the benchmarked configuration with SMOOTH tables (formula tables x FULL_SMOOTH_SCALE instead of x 50): the
        # SDF is smooth on the scale of a sample step, so the free-running HIP sampler must reproduce the reference's
        # bins (tests/test_gpu_fullsize.py::test_fullsize_smooth_free_running)
        gen_end_to_end("grid", "grid.yaml", ["rgb"], 95000, "full_grid_rgb_l19_smooth", n_rays=2048, log2T=19, W=640,
                       H=512, n_views=50, cam_seed=0, state=fullsize_state(["rgb"], 19, table_scale=FULL_SMOOTH_SCALE),
                       compact=True, state_meta={"table_scale": FULL_SMOOTH_SCALE})
    if "e2e_full" in which:
        # BASELINE configs[1] at its own size: grid.yaml, rgb, 2048 rays, log2T 19 (confs/grid.yaml:58-59), step 95000,
        # the benchmark's 50-view 640 x 512 camera rig; parameters regenerated on the box (fullsize_state)
        gen_end_to_end("grid", "grid.yaml", ["rgb"], 95000, "full_grid_rgb_l19", n_rays=2048, log2T=19,
                       W=640, H=512, n_views=50, cam_seed=0, state=fullsize_state(["rgb"], 19), compact=True)
