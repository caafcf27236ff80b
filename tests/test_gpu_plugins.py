"""The reference-signature plugin classes (multimodalstudio_amd/plugins.py) against the reference's own modules.

tests/golden/plugins.npz was produced by running the reference's SDFField, RadianceField and Renderer
(tests/golden/make_golden.py:gen_plugins); the HIP modules are built from mirror configs with the reference's field
names, load the reference's state_dict unchanged (strict) and must reproduce forward outputs and every gradient.
The sampler and ray generator reuse the neus_sampler / raygen fixtures through the plugin signatures.  Tolerances
(fp32 parity preset): outputs 1e-4 of the tensor's scale; gradients 1e-3 (fp32 summation order over 256 rows);
sampler bins exactly.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return dict(np.load(os.path.join(GOLD, name + ".npz")))


def rel_err(actual, ref):
    a = np.asarray(actual, dtype=np.float64)
    r = np.asarray(ref, dtype=np.float64)
    s = np.abs(r).max()
    return np.abs(a - r).max() / s if s > 0 else np.abs(a - r).max()


@pytest.fixture(autouse=True)
def fp32_preset():
    from multimodalstudio_amd import functions as fx
    fx.set_precision("fp32")
    yield


def _grid_cfg(P):
    return P.FeatureGridConfig(encoding=P.HashEncodingConfig(max_res=1024, log2_hashmap_size=12), radius=1.0)


def _state(f, prefix, dev):
    return {k[len(prefix):]: torch.from_numpy(v).to(dev) for k, v in f.items() if k.startswith(prefix)}


def _check_grads(module, f, prefix, tol):
    worst = {}
    for k, p in module.named_parameters():
        ref = f.get(prefix + k)
        if ref is None:
            continue
        worst[k] = rel_err(p.grad.cpu(), ref)
    bad = {k: v for k, v in worst.items() if v > tol}
    assert not bad, bad
    return worst


def test_sdf_field(dev):
    from multimodalstudio_amd import model as mm
    from multimodalstudio_amd import plugins as P
    f = load("plugins")
    cfg = P.SDFFieldConfig(field=P.FeatureGridAndMLPConfig(
        feature_grid=_grid_cfg(P),
        mlp_head=mm.MLPConfig(num_layers=3, hidden_dim=256, activation="Softplus", activation_params={"beta": 100},
                              out_activation="None", geometric_init=True, geometric_init_bias=0.4)))
    sf = cfg.setup().to(dev)
    sf.load_state_dict(_state(f, "sdf:p:", dev), strict=True)
    sf.field.feature_grid.update_mask(int(f["sdf_level"]))
    x = torch.from_numpy(f["sdf:x"]).to(dev).requires_grad_(True)
    sdf, geo = sf(x)
    assert rel_err(sdf.detach().cpu(), f["sdf:sdf"]) < 1e-4
    assert rel_err(geo.detach().cpu(), f["sdf:geo"]) < 1e-4
    assert torch.equal(sf.single_output(x.detach()), sdf.detach())
    ((sdf * torch.from_numpy(f["sdf:dsdf"]).to(dev)).sum() + (geo * torch.from_numpy(f["sdf:dgeo"]).to(dev)).sum()
     ).backward()
    assert rel_err(x.grad.cpu(), f["sdf:dx"]) < 1e-3
    _check_grads(sf, f, "sdf:g:", 1e-3)


def test_radiance_field(dev):
    from multimodalstudio_amd import model as mm
    from multimodalstudio_amd import plugins as P
    f = load("plugins")
    cfg = P.RadianceFieldConfig(base_field=P.FeatureGridAndMLPConfig(
        feature_grid=_grid_cfg(P), mlp_head=mm.MLPConfig(num_layers=3, hidden_dim=256, out_activation="ReLU")))
    vd_dim = f["rad:vd"].shape[1]
    rf = cfg.setup(position_dim=3, view_direction_dim=vd_dim, additional_input_dim=257, output_dim=256).to(dev)
    rf.load_state_dict(_state(f, "rad:p:", dev), strict=True)
    rf.base_field.feature_grid.update_mask(int(f["rad_level"]))
    ins = [torch.from_numpy(f[k]).to(dev).requires_grad_(True) for k in ["rad:pos", "rad:vd", "rad:extra"]]
    out = rf(*ins)
    assert rel_err(out.detach().cpu(), f["rad:out"]) < 1e-4
    (out * torch.from_numpy(f["rad:dout"]).to(dev)).sum().backward()
    for t, k in zip(ins, ["rad:dpos", "rad:dvd", "rad:dextra"]):
        assert rel_err(t.grad.cpu(), f[k]) < 1e-3, k
    _check_grads(rf, f, "rad:g:", 1e-3)


def test_renderer(dev):
    from multimodalstudio_amd import plugins as P
    f = load("plugins")
    mask = torch.from_numpy(f["ren:mask"]).to(dev)
    w = torch.from_numpy(f["ren:w"]).to(dev).requires_grad_(True)
    rgb = torch.from_numpy(f["ren:rgb"]).to(dev).requires_grad_(True)
    bg = torch.from_numpy(f["ren:bg"]).to(dev).requires_grad_(True)
    R, S = w.shape[:2]
    starts, ends = (torch.from_numpy(f[k]).to(dev) for k in ["ren:starts", "ren:ends"])
    rs = P.RaySamples(frustums=P.Frustums(origins=None, directions=None, starts=starts, ends=ends))
    ren = P.RendererConfig(renderers={"rgb": "RadianceRenderer"}).setup()
    outs = ren.render(w, {"rgb": rgb, "background": {"rgb": bg}, "normals": torch.from_numpy(f["ren:normals"]).to(dev),
                          "depth": rs}, mask)
    for k in ["rgb", "normals", "depth", "accumulation"]:
        assert rel_err(outs[k].detach().cpu(), f["ren:out:" + k]) < 1e-5, k
    ((outs["rgb"] * torch.from_numpy(f["ren:drgb"]).to(dev)).sum() + outs["accumulation"].sum()).backward()
    assert rel_err(w.grad.cpu(), f["ren:dw"]) < 1e-5
    assert rel_err(rgb.grad.cpu(), f["ren:dvals"]) < 1e-6
    assert rel_err(bg.grad.cpu(), f["ren:dbg"]) < 1e-6


def test_neus_sampler_plugin_bit_exact(dev):
    """NeuSSampler.generate_ray_samples with the reference's sdf_fn signature (ray_samples -> sdf) on the fixture's
    rays and injected uniforms: final bins and sample starts exactly the reference's."""
    from multimodalstudio_amd import plugins as P
    f = load("neus_sampler")
    o = torch.from_numpy(f["origins"]).to(dev)
    d = torch.from_numpy(f["directions"]).to(dev)
    rb = P.RayBundle(origins=o, directions=d, pixel_area=torch.ones(o.shape[0], 1, device=dev) * 1e-4,
                     camera_indices=torch.zeros(o.shape[0], 1, dtype=torch.long, device=dev),
                     up_directions=torch.zeros_like(o))
    mask = P.collide(rb, 1.0)
    assert np.array_equal(mask.cpu().numpy(), f["mask"])
    hit = rb[mask]
    hit.nears = torch.from_numpy(f["nears"]).to(dev).reshape(-1, 1)    # the reference's MKL-sqrt intervals (1 ulp)
    hit.fars = torch.from_numpy(f["fars"]).to(dev).reshape(-1, 1)
    R = hit.origins.shape[0]

    def sdf_fn(rs):
        p = rs.frustums.get_start_positions().cpu()
        return (torch.linalg.norm(p, dim=-1, keepdim=True) - 0.5).to(dev)

    rand = {"rgb": (torch.from_numpy(f["rand_uniform"]).to(dev),
                    [torch.from_numpy(f["rand_pdf"][i]).to(dev) for i in range(4)])}
    sampler = P.NeuSSamplerConfig(num_samples=32, num_samples_importance=32).setup()
    out = sampler.generate_ray_samples({"rgb": hit}, sdf_fn=sdf_fn, rand=rand)["ray_samples_per_modality"]["rgb"]
    bins = torch.cat([out.spacing_starts[..., 0], out.spacing_ends[..., -1:, 0]], -1)
    assert out.shape == (R, 64)
    assert np.array_equal(bins.cpu().numpy(), f["bins"])
    assert np.array_equal(out.frustums.starts[..., 0].cpu().numpy(), f["starts"])


def test_hash_encoding_plugin_bit_exact(dev):
    """HashEncoding(config).forward(x_hat) (encodings.py:263-304) with x_hat = (x + r) / (2 r) formed as
    FeatureGrid.forward does: bit-exact to the reference fixture (all levels active)."""
    from multimodalstudio_amd import plugins as P
    f = load("hashgrid_l12_a16_r1")
    enc = P.HashEncoding(P.HashEncodingConfig(max_res=1024, log2_hashmap_size=12)).to(dev)
    with torch.no_grad():
        enc.hash_table.copy_(torch.from_numpy(f["table"]))
    x = torch.from_numpy(f["x"]).to(dev)
    xh = (x + 1.0) / (2 * 1.0)
    out = enc(xh)
    assert np.array_equal(out.detach().cpu().numpy(), f["out"])


def test_ray_generator_plugin(dev):
    from multimodalstudio_amd import pipeline as pl
    from multimodalstudio_amd import plugins as P
    from multimodalstudio_amd import scene as ms
    f = load("raygen")
    mods = ["rgb", "polarization"]
    cams = {m: pl.DeviceCameras(ms.ModalityCameras(
        torch.from_numpy(f[f"{m}:c2w"]), torch.from_numpy(f[f"{m}:fx"]), torch.from_numpy(f[f"{m}:fy"]),
        torch.from_numpy(f[f"{m}:cx"]), torch.from_numpy(f[f"{m}:cy"]), torch.from_numpy(f[f"{m}:distortion"]),
        96, 80, []), dev) for m in mods}
    pose = pl.CameraOptimizer(mods, {m: cams[m].num for m in mods}).to(dev)
    with torch.no_grad():
        for m in mods:
            pose.pose_adjustment[m].copy_(torch.from_numpy(f[f"{m}:pose"]))
    gen = P.RayGenerator(cams, pose, 0.0)
    bundles = gen({m: torch.from_numpy(f[f"{m}:coords"]).to(dev) for m in mods})
    for m in mods:
        rb = bundles[m]
        assert isinstance(rb, P.RayBundle)
        for attr, key in [("origins", "origins"), ("directions", "directions"), ("up_directions", "up")]:
            assert rel_err(getattr(rb, attr).detach().cpu(), f[f"{m}:{key}"]) < 1e-5, (m, attr)
