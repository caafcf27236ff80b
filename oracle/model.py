"""ORACLE (test infrastructure only) — model forward, losses and the training step.

Restates (paths under /root/reference/src):
  BaseModel.forward                    models/base_model.py:82-161
  SurfaceModel.forward / gradient      model_components/surface_model.py:66-206 (4-tap and autograd), get_sdf :213-226
  set_delta callback                   model_components/surface_model.py:248-279
  NeuSVolumeRendering                  model_components/volume_rendering.py:171-239
  SingleVarianceNetwork                field_components/single_variance.py:34-36
  RadianceModel.forward                model_components/radiance_model.py:94-151
  BackgroundModel.forward              model_components/background_model.py:73-111
  RaySamples.get_alphas                cameras/rays.py:138-151
  Renderer.render / RadianceRenderer   model_components/renderers.py:75-174 (+ Accumulation/Depth/Normals)
  RawPipeline.select_right_channel     pipelines/raw_pipeline.py:112-122
  LossManager.compute_loss             model_components/losses.py:213-265 (L1, SkipSaturation, Eikonal, Curvature)
  CurvatureLossWarmUpScheduler         engine/schedulers.py:320-343
  MultiStepWarmupScheduler             engine/schedulers.py:249-270
  clip_gradients + AdamW               pipelines/base_pipeline.py:232-248; method_configs.py:260-269
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

from . import fields as of
from . import hashgrid as ohg
from . import rays as orr

TAPS = torch.tensor([[1, -1, -1], [-1, -1, 1], [-1, 1, -1], [1, 1, 1]], dtype=torch.float32)


# ------------------------------------------------------------------------------------------------
# schedule-dependent state (callbacks)
# ------------------------------------------------------------------------------------------------
@dataclass
class StepState:
    """Values the reference's BEFORE_TRAIN_ITERATION callbacks set for a given step."""
    step: int
    max_iters: int = 100000
    num_levels: int = 16
    min_res: int = 16
    max_res: int = 1024
    radius: float = 1.0
    anneal_end_ratio: float = 0.05

    @property
    def steps_per_level(self) -> int:
        spl = int(self.max_iters * 1.0)
        return min(spl, int(self.max_iters / self.num_levels))

    @property
    def active_levels(self) -> int:
        """feature_structures.py:97-108."""
        level = int(self.step / self.steps_per_level) + 1
        return min(max(level, 1), self.num_levels)

    @property
    def delta(self) -> float:
        """surface_model.py:272-278 (before the /sqrt(3) of the 4-tap scheme)."""
        g = ohg.growth_factor(self.min_res, self.max_res, self.num_levels)
        d = 1.0 / (self.min_res * g ** int(self.step / self.steps_per_level))
        d = max(1.0 / self.max_res, d)
        return d * (self.radius * 2.0)

    @property
    def cos_anneal(self) -> float:
        """volume_rendering.py:227-230."""
        end = int(self.max_iters * self.anneal_end_ratio)
        return min(1.0, self.step / end)

    @property
    def curvature_factor(self) -> float:
        """CurvatureLossWarmUpScheduler (schedulers.py:320-343), warm_up_ratio 0.1."""
        warm = int(self.max_iters * 0.1)
        if self.step < warm:
            return self.step / warm
        g = ohg.growth_factor(self.min_res, self.max_res, self.num_levels)
        level = min(max(int(self.step / self.steps_per_level) + 1, 1), self.num_levels)
        return float(np.reciprocal(g ** (level - 1)))


def lr_factor(step: int, max_iters: int = 100000, warm_up_ratio=0.1, milestones=(0.5, 0.75, 0.9), gamma=0.4):
    """MultiStepWarmupScheduler.func (schedulers.py:259-266)."""
    warm = int(max_iters * warm_up_ratio)
    if step < warm:
        return step / warm
    idx = np.searchsorted(milestones, step / max_iters, side="left")
    return gamma ** idx


# ------------------------------------------------------------------------------------------------
# model spec (method_configs.py:59-445 + YAML)
# ------------------------------------------------------------------------------------------------
@dataclass
class ModelSpec:
    modalities: Dict[str, int]                       # name -> channels, config order
    grid: of.GridSpec = field(default_factory=of.GridSpec)
    head_layers: Dict[str, int] = field(default_factory=dict)   # radiance heads (3 layers each)
    bg_head_layers: Dict[str, int] = field(default_factory=dict)
    use_background: bool = True
    num_samples: int = 32
    num_importance: int = 32
    upsample_steps: int = 4
    bg_samples: int = 16
    raw: bool = False
    fields: str = "grid"      # "grid" (hash grid + 3-layer MLPs, 4-tap gradients) | "mlp" (8-layer MLPs, autograd)
    # background base field: None = the NeRF MLP; a GridSpec = config 5's hash grid (r = 2) + 71-128-128-256 MLP
    bg_grid: Optional[of.GridSpec] = None


def spec_grid(modalities: Dict[str, int], log2T: int = 19, raw: bool = False, bg_kind: str = "nerf") -> ModelSpec:
    """Methods grid / grid_raw (bg_kind "nerf"), or grid_raw_grid_bg_unbalanced (bg_kind "grid": the background base
    field a FeatureGridAndMLP with a radius-2 hash grid, head 283-256x3-256, and the radiance model's 3-layer heads,
    method_configs.py:428-445)."""
    s = ModelSpec(modalities=dict(modalities), grid=of.GridSpec(16, 16, 1024, log2T, 1.0), raw=raw)
    s.head_layers = {m: 3 for m in modalities}
    s.bg_head_layers = {m: 1 for m in modalities}
    if bg_kind == "grid":
        s.bg_grid = of.GridSpec(16, 16, 1024, log2T, 2.0)
        s.bg_head_layers = {m: 3 for m in modalities}
    elif bg_kind != "nerf":
        raise ValueError(bg_kind)
    return s


def spec_mlp(modalities: Dict[str, int], raw: bool = False) -> ModelSpec:
    """The mlp / mlp_raw methods (method_configs.py:303-353): MLP fields, analytic SDF gradient, no hessian, the
    grid methods' heads and NeRF background."""
    s = spec_grid(modalities, raw=raw)
    s.fields = "mlp"
    return s


# ------------------------------------------------------------------------------------------------
# surface / volume rendering
# ------------------------------------------------------------------------------------------------
def inv_variance(P) -> torch.Tensor:
    return torch.exp(P["surface_model.volume_rendering.density_fn.variance_network.s"] * 10.0).clip(1e-6, 1e6)


def surface_forward(pos: torch.Tensor, P, spec: ModelSpec, st: StepState):
    """SurfaceModel.forward (surface_model.py:66-127) on flattened start positions [M, 3]."""
    if spec.fields == "mlp":
        # use_numerical_gradients False: d sdf / d x by autograd, kept in the graph (surface_model.py:192-198);
        # compute_hessian False for these methods
        with torch.enable_grad():
            x = pos if pos.requires_grad else pos.detach().requires_grad_(True)
            sdf, geo = of.sdf_field_mlp(x, P)
            grads = torch.autograd.grad(sdf, x, torch.ones_like(sdf), create_graph=True, retain_graph=True)[0]
        return sdf, geo, grads, None
    sdf, geo = of.sdf_field(pos, P, spec.grid, st.active_levels)
    delta = st.delta / np.sqrt(3)
    taps = [of.sdf_field(pos + TAPS[i] * delta, P, spec.grid, st.active_levels)[0] for i in range(4)]
    k = TAPS
    grads = (k[0] * taps[0] + k[1] * taps[1] + k[2] * taps[2] + k[3] * taps[3]) / (4.0 * delta)
    hxx = ((taps[0] + taps[1] + taps[2] + taps[3]) / 2.0 - 2 * sdf) / delta ** 2
    hess = torch.cat([hxx, hxx, hxx], dim=-1) / 3.0
    return sdf, geo, grads, hess


def neus_alpha(sdf, grads, directions, deltas, inv_s, cos_anneal):
    """NeuSVolumeRendering.get_alphas (volume_rendering.py:185-213); sdf [R,S,1], grads [R,S,3]."""
    true_cos = (directions[:, None, :] * grads).sum(-1, keepdim=True)
    iter_cos = -(F.relu(-true_cos * 0.5 + 0.5) * (1.0 - cos_anneal) + F.relu(-true_cos) * cos_anneal)
    nxt = sdf + iter_cos * deltas * 0.5
    prv = sdf - iter_cos * deltas * 0.5
    pc = torch.sigmoid(prv * inv_s)
    nc = torch.sigmoid(nxt * inv_s)
    return ((pc - nc + 1e-5) / (pc + 1e-5)).clip(0.0, 1.0).squeeze(dim=-1)


def neus_weights(alpha):
    """volume_rendering.py:177-183."""
    T = torch.cumprod(torch.cat([torch.ones((alpha.shape[0], 1)), 1.0 - alpha + 1e-7], 1), 1)
    return (alpha * T[:, :-1]).unsqueeze(-1)


# ------------------------------------------------------------------------------------------------
# full forward
# ------------------------------------------------------------------------------------------------
@dataclass
class RNG:
    """Injected uniforms in the reference draw order."""
    uniform: Dict[str, torch.Tensor]          # [N_hit, 1] per modality
    pdf: Dict[str, List[torch.Tensor]]        # 4 x [N_hit, 1] per modality
    background: Dict[str, torch.Tensor]       # [N, bg+1] per modality


def model_forward(rays: Dict[str, orr.Rays], P, spec: ModelSpec, st: StepState, rng: RNG):
    """BaseModel.forward (base_model.py:82-161). Returns per-modality output dicts."""
    outputs = {}
    for mod in spec.modalities:
        r = rays[mod]
        nears, fars, mask = orr.sphere_collider(r.origins, r.directions)
        o_h, d_h, up_h = r.origins[mask], r.directions[mask], r.up[mask]
        n_h, f_h = nears[mask], fars[mask]

        def sdf_fn(pts):
            R, n = pts.shape[:2]
            if spec.fields == "mlp":
                return of.sdf_field_mlp(pts.reshape(-1, 3), P)[0].view(R, n)
            return of.sdf_field(pts.reshape(-1, 3), P, spec.grid, st.active_levels)[0].view(R, n)

        smp, hist = orr.neus_sample(n_h, f_h, o_h, d_h, sdf_fn, rng.uniform[mod], rng.pdf[mod],
                                    spec.num_samples, spec.num_importance, spec.upsample_steps)
        # background
        bg = None
        if spec.use_background:
            bn, bf = orr.background_near_far(r.origins, r.directions)
            bbins = orr.stratified_bins(bn.shape[0], spec.bg_samples, rng.background[mod])
            bsmp = orr.make_samples(bbins, bn, bf, "disparity")
            bg = background_forward(bsmp, r, P, spec, st)
        R, S = smp.starts.shape[:2]
        pos = orr.positions(o_h, d_h, smp.starts).reshape(-1, 3)
        sdf, geo, grads, hess = surface_forward(pos, P, spec, st)
        sdf = sdf.view(R, S, 1)
        grads = grads.view(R, S, 3)
        hess = hess.view(R, S, 3) if hess is not None else None
        normals = F.normalize(grads, p=2, dim=-1)
        s = inv_variance(P)
        alpha = neus_alpha(sdf, grads, d_h, smp.deltas, s, st.cos_anneal)
        weights = neus_weights(alpha)
        rad = radiance_forward(pos, d_h, up_h, normals.detach().reshape(-1, 3), geo, P, spec, st, R, S)
        out = render(weights, rad, normals, smp, bg, mask, spec)
        out["gradients"] = grads
        out["hessians"] = hess
        out["inv_s"] = 1.0 / s
        out["sorted_index"] = hist
        out["bins"] = smp.spacing_bins
        out["weights"] = weights
        out["mask"] = mask
        outputs[mod] = out
    return outputs


def radiance_forward(pos, d_h, up_h, normals, geo, P, spec: ModelSpec, st: StepState, R, S):
    """RadianceModel.forward (radiance_model.py:94-151), use_n_dot_v, SH(4), no reflection (grid.yaml)."""
    dirs = d_h[:, None, :].expand(R, S, 3).reshape(-1, 3)
    ups = up_h[:, None, :].expand(R, S, 3).reshape(-1, 3)
    ndv = torch.sum(normals * -dirs, dim=-1, keepdim=True)
    sh = of.sh_encoding(dirs.clone(), 5)
    if spec.fields == "mlp":
        feat = of.radiance_field_mlp(pos, sh, torch.cat([geo, ndv], -1), P)
    else:
        feat = of.radiance_field(pos, sh, torch.cat([geo, ndv], -1), P, spec.grid, st.active_levels)
    out = {}
    for mod in spec.modalities:
        kind = "polarization" if mod == "polarization" else "plain"
        v = of.modality_head(feat, P, f"radiance_model.modality_heads.{mod}", kind, spec.head_layers[mod], dirs, ups)
        out[mod] = v.view(R, S, -1)
    return out


def background_forward(bsmp: orr.Samples, r: orr.Rays, P, spec: ModelSpec, st: StepState = None):
    """BackgroundModel.forward (background_model.py:73-111) with L-inf contraction."""
    N, S = bsmp.starts.shape[:2]
    pos = orr.positions(r.origins, r.directions, bsmp.starts).reshape(-1, 3)
    dirs = r.directions[:, None, :].expand(N, S, 3).reshape(-1, 3)
    ups = r.up[:, None, :].expand(N, S, 3).reshape(-1, 3)
    pos = of.scene_contraction_linf(pos)
    # the background grid keeps every level at every step: BackgroundModel registers no training callbacks
    # (background_model.py:120-125), so FeatureGrid.set_mask never runs and hash_encoding_mask stays all ones
    density, feat = of.nerf_field(pos, dirs, P, grid=spec.bg_grid,
                                  active_levels=spec.bg_grid.num_levels if spec.bg_grid is not None else 16)
    density = density.view(N, S, -1)
    alphas = 1 - torch.exp(-(bsmp.deltas * density))
    w = orr.weights_from_alphas(alphas)
    out = {}
    for mod in spec.modalities:
        kind = "polarization" if mod == "polarization" else "plain"
        v = of.modality_head(feat, P, f"background_model.modality_heads.{mod}", kind, spec.bg_head_layers[mod],
                             dirs, ups)
        out[mod] = torch.sum(w * v.view(N, S, -1), dim=1)
    return out


def render(weights, rad, normals, smp, bg, mask, spec: ModelSpec):
    """Renderer.render (renderers.py:75-136)."""
    out = {}
    N = mask.shape[0]
    acc = torch.sum(weights, dim=-2)
    for mod in rad:
        C = rad[mod].shape[-1]
        if bg is not None:
            base = bg[mod]
        else:
            base = torch.zeros(N, C)
        comp = torch.sum(weights * rad[mod], dim=-2) + base[mask] * (1.0 - acc)
        full = base.clone()
        full[mask] = comp
        out[mod] = full
    nrm = torch.zeros(N, 3)
    nrm[mask] = torch.sum(weights * normals, dim=-2)
    out["normals"] = nrm
    steps = (smp.starts + smp.ends) / 2
    depth = torch.zeros(N, 1)
    dd = torch.sum(weights * steps, dim=-2)
    depth[mask] = torch.clip(dd, steps.min(), steps.max())
    out["depth"] = depth
    accum = torch.zeros(N, 1)
    accum[mask] = acc
    out["accumulation"] = accum
    return out


# ------------------------------------------------------------------------------------------------
# losses
# ------------------------------------------------------------------------------------------------
def select_channel(rendered: torch.Tensor, mosaick_mask: torch.Tensor, coords: torch.Tensor) -> torch.Tensor:
    """raw_pipeline.py:112-122."""
    band = mosaick_mask[coords[:, 1].long(), coords[:, 2].long()].unsqueeze(dim=1).to(torch.int64)
    return torch.gather(rendered, 1, band)


def compute_loss(outputs, targets: Dict[str, torch.Tensor], spec: ModelSpec, st: StepState,
                 sat_threshold: float = 0.9980):
    """LossManager.compute_loss (losses.py:224-265) for the grid/grid_raw radiance + geometry losses."""
    losses = {}
    total = 0.0
    for mod in spec.modalities:
        out = outputs[mod][mod]
        tgt = targets[mod]
        if mod == "polarization":
            m = tgt > sat_threshold
            if m.any():
                out = out.masked_fill(m, tgt[m].flatten()[0])
        l = F.l1_loss(out, tgt)
        losses[mod] = l
        total = total + l
    grads = torch.cat([outputs[m]["gradients"] for m in spec.modalities], 0)
    gn = torch.norm(grads, 2, dim=-1)
    eik = F.mse_loss(gn, torch.ones_like(gn))
    losses["eikonal_loss"] = eik
    total = total + 0.1 * eik
    if spec.fields == "mlp":
        return losses, total        # geometry losses of the mlp methods: eikonal only (method_configs.py:350-352)
    hess = torch.cat([outputs[m]["hessians"] for m in spec.modalities], 0)
    lap = hess.sum(dim=-1)
    curv = F.l1_loss(lap, torch.zeros_like(lap))
    losses["curvature_loss"] = curv
    total = total + 5e-4 * st.curvature_factor * curv
    return losses, total


# ------------------------------------------------------------------------------------------------
# optimizer step
# ------------------------------------------------------------------------------------------------
def clip_grad_norm(params: List[torch.Tensor], max_norm: float):
    """torch.nn.utils.clip_grad_norm_ semantics (as used by fabric.clip_gradients)."""
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return torch.tensor(0.0)
    total = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(g, 2) for g in grads]), 2)
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    for g in grads:
        g.mul_(coef)
    return total


def adamw_step(params, states, lr, wd=0.01, eps=1e-15, betas=(0.9, 0.999)):
    """torch.optim.AdamW single-tensor semantics (default amsgrad=False)."""
    b1, b2 = betas
    for p in params:
        if p.grad is None:
            continue
        st = states.setdefault(id(p), {"step": 0, "m": torch.zeros_like(p), "v": torch.zeros_like(p)})
        st["step"] += 1
        t = st["step"]
        with torch.no_grad():
            p.mul_(1 - lr * wd)
            st["m"].lerp_(p.grad, 1 - b1)
            st["v"].mul_(b2).addcmul_(p.grad, p.grad, value=1 - b2)
            bc1 = 1 - b1 ** t
            bc2 = 1 - b2 ** t
            step_size = lr / bc1
            denom = (st["v"].sqrt() / math.sqrt(bc2)).add_(eps)
            p.addcdiv_(st["m"], denom, value=-step_size)
