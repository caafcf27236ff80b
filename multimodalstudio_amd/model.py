"""MMS model on the HIP kernels, with the reference's module tree and parameter names.

``BaseModel(...).state_dict()`` has the same keys and shapes as the reference's
``models.base_model.BaseModel`` (/root/reference/src/models/base_model.py:55-80), so reference
checkpoints load unchanged and vice versa.  The orchestration in ``BaseModel.forward`` follows
base_model.py:82-161 stage by stage; every stage runs in libmms_hip.so through functions.py.
"""
from __future__ import annotations

import os

import ctypes
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
from torch import nn

from . import _lib
from . import functions as fx
from .functions import GridCfg


# ------------------------------------------------------------------------------------------------
# field components
# ------------------------------------------------------------------------------------------------
class _WeightParams(nn.Module):
    """Holds original0 (g) / original1 (v) like torch's weight_norm parametrization list."""

    def __init__(self, g: torch.Tensor, v: torch.Tensor):
        super().__init__()
        self.original0 = nn.Parameter(g)
        self.original1 = nn.Parameter(v)


class WeightNormLinear(nn.Module):
    """nn.Linear under parametrizations.weight_norm (mlp.py:206-209): keys bias, parametrizations.weight.original{0,1}."""

    def __init__(self, in_features: int, out_features: int, weight: torch.Tensor, bias: torch.Tensor):
        super().__init__()
        g = torch.linalg.vector_norm(weight, dim=1, keepdim=True).detach().clone()
        self.parametrizations = nn.ModuleDict({"weight": _WeightParams(g, weight.detach().clone())})
        self.bias = nn.Parameter(bias.detach().clone())
        self.in_features, self.out_features = in_features, out_features

    def params(self):
        w = self.parametrizations["weight"]
        return [w.original0, w.original1, self.bias]


@dataclass
class MLPConfig:
    """MLPConfig (mlp.py:36-58)."""
    num_layers: int = 8
    hidden_dim: int = 128
    weight_norm: bool = True
    activation: str = "ReLU"
    activation_params: dict = field(default_factory=dict)
    out_activation: Optional[str] = "Sigmoid"
    skip_connections: Sequence[int] = ()
    geometric_init: bool = False
    geometric_init_bias: float = 0.5


class MLP(nn.Module):
    """Weight-normed MLP (mlp.py:99-209) with the reference's initialisers."""

    def __init__(self, config: MLPConfig, input_dim: int, output_dim: Optional[int] = None):
        super().__init__()
        if not config.weight_norm:
            raise NotImplementedError("the HIP MLP implements the weight-normed layers used by every method config")
        self.config = config
        self.precision_key = "heads"      # functions.PRECISION entry of its GEMMs when run as a plain MLP
        self.input_dim = input_dim
        self.output_dim = output_dim if output_dim is not None else config.hidden_dim
        self.skips = tuple(config.skip_connections or ())
        # mlp.py:115-137: a skip layer i takes cat[h, input] / sqrt(2); the layer before it is narrowed so the
        # concatenation is hidden_dim + input_dim wide
        dims = [input_dim] + [config.hidden_dim + (input_dim if i + 1 in self.skips else 0)
                              for i in range(config.num_layers - 1)] + [self.output_dim]
        shapes = [(dims[i], dims[i + 1] - (dims[0] if i + 1 in self.skips else 0)) for i in range(len(dims) - 1)]
        weights, biases = [], []
        for k, n in shapes:
            lin = nn.Linear(k, n)
            weights.append(lin.weight.data)
            biases.append(lin.bias.data)
        if config.geometric_init:
            self._geometric_init(weights, biases, config.geometric_init_bias, input_dim > 3, self.skips)
        else:
            for w, b in zip(weights, biases):
                nn.init.kaiming_uniform_(w)
                nn.init.zeros_(b)
        self.layers = nn.ModuleList([WeightNormLinear(k, n, weights[i], biases[i])
                                     for i, (k, n) in enumerate(shapes)])
        hidden = fx.ACT[config.activation]
        beta = float(config.activation_params.get("beta", 1.0))
        thr = float(config.activation_params.get("threshold", 20.0))
        out = fx.ACT[config.out_activation if config.out_activation != "None" else None]
        self.acts = tuple([(hidden, beta, thr)] * (len(dims) - 2) + [(out, 1.0, 20.0)])

    @staticmethod
    def _geometric_init(weights, biases, bias, additional_input, skips=()):
        """MLP.geometric_init (mlp.py:173-198)."""
        L = len(weights)
        for l in range(L):
            out_dim, in_dim = weights[l].shape
            if l == L - 1:
                nn.init.normal_(weights[l], mean=np.sqrt(np.pi) / np.sqrt(in_dim), std=0.0001)
                nn.init.constant_(biases[l], -bias)
            elif additional_input and l == 0:
                nn.init.constant_(biases[l], 0.0)
                nn.init.constant_(weights[l][:, 3:], 0.0)
                nn.init.normal_(weights[l][:, :3], 0.0, np.sqrt(2) / np.sqrt(out_dim))
            elif additional_input and l in skips:
                nn.init.constant_(biases[l], 0.0)
                nn.init.normal_(weights[l], 0.0, np.sqrt(2) / np.sqrt(out_dim))
                nn.init.constant_(weights[l][:, -(weights[0].shape[1] - 3):], 0.0)
            else:
                nn.init.constant_(biases[l], 0.0)
                nn.init.normal_(weights[l], 0.0, np.sqrt(2) / np.sqrt(out_dim))

    def params(self) -> List[torch.Tensor]:
        out = []
        for layer in self.layers:
            out += layer.params()
        return out

    def forward(self, x):
        if self.skips:
            return self.forward_diff(x)
        return fx.MLPFunction.apply(x, self.acts, self.precision_key, *self.params())

    def forward_diff(self, x: torch.Tensor) -> torch.Tensor:
        """MLP.forward (mlp.py:152-171) with every product on the twice-differentiable HIP GEMM (autodiff.MatMul) and
        the reference's torch element-wise operators, for fields whose input gradient is differentiated again."""
        from . import autodiff
        c = self.config
        h = x
        L = len(self.layers)
        for i, layer in enumerate(self.layers):
            if i in self.skips:
                h = torch.cat([h, x], -1) / np.sqrt(2)
            w = layer.parametrizations["weight"]
            W = w.original0 * (w.original1 / torch.linalg.vector_norm(w.original1, dim=1, keepdim=True))
            h = autodiff.linear(h, W, layer.bias)
            if i < L - 1:
                h = _act_torch(c.activation, c.activation_params, h)
        if c.out_activation not in (None, "None"):
            h = _act_torch(c.out_activation, {}, h)
        return h


def _act_torch(name: str, params: dict, x: torch.Tensor) -> torch.Tensor:
    if name == "Softplus":
        return torch.nn.functional.softplus(x, beta=float(params.get("beta", 1.0)),
                                            threshold=float(params.get("threshold", 20.0)))
    if name == "ReLU":
        return torch.relu(x)
    if name == "Sigmoid":
        return torch.sigmoid(x)
    raise ValueError(name)


class HashEncoding(nn.Module):
    """HashEncoding (encodings.py:184-310) with implementation 'hip' (parameter hash_table [L*T, F])."""

    def __init__(self, num_levels=16, features_per_level=2, min_res=16, max_res=2048, log2_hashmap_size=19,
                 hash_init_scale=0.001, interpolation: str = "Linear"):
        super().__init__()
        self.num_levels, self.features, self.log2T = num_levels, features_per_level, log2_hashmap_size
        from .hip_ops import INTERP
        if interpolation not in INTERP:
            raise ValueError(f"interpolation '{interpolation}': Linear or Smoothstep (encodings.py:64-67)")
        self.interp = INTERP[interpolation]
        self.growth_factor = float(np.exp((np.log(max_res) - np.log(min_res)) / (num_levels - 1)))
        levels = torch.arange(num_levels)
        self.scalings = torch.floor(min_res * self.growth_factor ** levels)
        T = 2 ** log2_hashmap_size
        table = (torch.rand(size=(T * num_levels, features_per_level)) * 2 - 1) * hash_init_scale
        self.hash_table = nn.Parameter(table)

    def get_out_dim(self):
        return self.num_levels * self.features


class FeatureGrid(nn.Module):
    """FeatureGrid (feature_structures.py:56-127): rescale by radius + coarse-to-fine level mask."""

    def __init__(self, encoding: HashEncoding, radius: float = 1.0):
        super().__init__()
        self.encoding = encoding
        self.radius = float(radius)
        self.active_levels = encoding.num_levels
        self.cfg = GridCfg(encoding.scalings.tolist(), encoding.log2T, self.radius, encoding.features,
                           getattr(encoding, "interp", 0))

    def update_mask(self, level: int):
        """feature_structures.py:85-88 (levels >= `level` contribute zero)."""
        self.active_levels = int(level)

    def forward(self, x):
        return fx.HashGridApply(x, self.encoding.hash_table, self.cfg, self.active_levels)


class FeatureGridAndMLP(nn.Module):
    """FeatureGridAndMLP (feature_structures.py:130-173)."""

    def __init__(self, grid: FeatureGrid, mlp: MLP):
        super().__init__()
        self.feature_grid = grid
        self.mlp_head = mlp


class SingleVarianceNetwork(nn.Module):
    """single_variance.py:19-36."""

    def __init__(self, init_val: float = 0.3):
        super().__init__()
        self.s = nn.Parameter(init_val * torch.ones(1))

    def get_inv_variance(self):
        return torch.exp(self.s * 10.0).clip(1e-6, 1e6)


class _DensityFn(nn.Module):
    def __init__(self):
        super().__init__()
        self.variance_network = SingleVarianceNetwork(0.3)


class NeuSVolumeRendering(nn.Module):
    """NeuSVolumeRendering (volume_rendering.py:161-239)."""

    def __init__(self, anneal_end_ratio: float = 0.05):
        super().__init__()
        self.density_fn = _DensityFn()
        self.anneal_end_ratio = anneal_end_ratio
        self._cos_anneal_ratio = 1.0

    def set_cos_anneal_ratio(self, anneal: float):
        self._cos_anneal_ratio = float(anneal)


class ModalityHead(nn.Module):
    """ModalityHead / PolarizationHead (field_heads.py:55-106)."""

    def __init__(self, kind: str, input_dim: int, output_dim: int, num_layers: int, hidden_dim: int,
                 out_activation: Optional[str]):
        super().__init__()
        self.kind = kind
        cfg = MLPConfig(num_layers=num_layers, hidden_dim=hidden_dim, out_activation=out_activation)
        self.field = MLP(cfg, input_dim, 3 if kind == "polarization" else output_dim)
        if kind == "polarization":
            self.field.precision_key = "pol_head"

    def forward(self, x, directions=None, up_directions=None, S: int = 1):
        y = self.field(x)
        if self.kind == "polarization":
            return fx.PolarizerFunction.apply(y, directions, up_directions, S)
        return y


class SDFField(nn.Module):
    """SDFField (surface_field.py:80-116) around FeatureGridAndMLP (attribute `field`)."""

    def __init__(self, field: FeatureGridAndMLP):
        super().__init__()
        self.field = field


class SurfaceModel(nn.Module):
    """SurfaceModel (surface_model.py:51-285): numerical 4-tap gradients + hessian."""

    def __init__(self, surface_field: SDFField):
        super().__init__()
        self.surface_field = surface_field
        self.volume_rendering = NeuSVolumeRendering()
        self.numerical_gradients_delta = 2.0 / 1024

    def set_numerical_gradients_delta(self, delta: float):
        self.numerical_gradients_delta = float(delta)

    def _grid_and_params(self):
        f = self.surface_field.field
        return f.feature_grid, f.mlp_head.params()

    @property
    def analytic(self) -> bool:
        """mlp methods: a plain MLP field with autograd gradients (use_numerical_gradients False)."""
        return isinstance(self.surface_field.field, MLP)

    def forward(self, pos: torch.Tensor):
        if self.analytic:
            return self._forward_analytic(pos)
        grid, params = self._grid_and_params()
        delta = self.numerical_gradients_delta / np.sqrt(3)
        return fx.SurfaceFunction.apply(pos, grid.encoding.hash_table, grid.cfg, grid.active_levels, float(delta),
                                        *params)

    def _forward_analytic(self, pos: torch.Tensor):
        """SurfaceModel.forward + gradient() of the mlp methods (surface_model.py:66-91, 192-198): sdf, geo from
        SDFField(PE(x)) and the gradient d sdf / dx by autograd with create_graph (so the eikonal loss trains through
        it: the MLP's backward is differentiated again, on the HIP GEMM, autodiff.MatMul); no hessian
        (compute_hessian False)."""
        x = pos if pos.requires_grad else pos.detach().requires_grad_(True)
        with torch.enable_grad():
            out = self.surface_field.field.forward_diff(nerf_encoding(x, 6))
            sdf, geo = out[:, :1], out[:, 1:]
            grads = torch.autograd.grad(sdf, x, torch.ones_like(sdf), create_graph=torch.is_grad_enabled() or
                                        self.training, retain_graph=True)[0]
        normals = torch.nn.functional.normalize(grads, p=2, dim=-1)
        return sdf, geo, grads, None, normals

    def get_sdf(self, pos: torch.Tensor) -> torch.Tensor:
        if self.analytic:
            with torch.no_grad():
                return self.surface_field.field.forward_diff(nerf_encoding(pos, 6))[:, 0].contiguous()
        grid, params = self._grid_and_params()
        with torch.no_grad():
            return fx.sdf_only(pos, grid.encoding.hash_table, grid.cfg, grid.active_levels, params)

    def get_sdf_rays(self, bins, n, f, o, d) -> Optional[torch.Tensor]:
        """get_sdf at the start positions of the samples of spacing bins [R, nb] on rays (n, f, o, d), the positions
        formed inside the panel launch (fx.FUSED_SAMPLER); None where that path does not serve (the caller then
        forms the positions itself)."""
        if self.analytic or not fx.FUSED_SAMPLER:
            return None
        grid, params = self._grid_and_params()
        with torch.no_grad():
            return fx.sdf_only(None, grid.encoding.hash_table, grid.cfg, grid.active_levels, params,
                               rays=(bins, n, f, o, d))


def _render_stats(w, normals, starts, ends, R: int, S: int, sidx, rows: int, dev):
    """[rows, 5] = (accumulation, normals, depth) of the hit rows sidx (zero elsewhere) by mms_render_stats; the depth
    is clipped to the min / max of all sample midpoints as DepthRenderer does (renderers.py:205-214)."""
    buf = torch.zeros(rows * 5 + 2, device=dev)
    stats = buf[:rows * 5].view(rows, 5)
    rng = buf[rows * 5:]       # zeros: the kernels' order-preserving range images start below every value
    with torch.no_grad():
        _lib.call("mms_render_stats", w.data_ptr(), normals.detach().contiguous().data_ptr(), starts.data_ptr(),
                  ends.data_ptr(), R, S, sidx.data_ptr(), stats.data_ptr(), 5, rng.data_ptr(), fx._s())
    return stats, rng


def _render_stats_segments(w, normals, starts, ends, off: List[int], S: int, sidx, rows: int, dev):
    """[n_seg rows, 5] = (accumulation, normals, depth) of every modality segment of a batched hit set: segment m's rays
    [off[m], off[m+1]) scatter to rows m rows + sidx (zero elsewhere), the depth clipped to that segment's own sample
    midpoint range (one DepthRenderer call per modality, renderers.py:205-214)."""
    n = len(off) - 1
    # a captured step carves the (graph-static) outputs from the step's zero arena: no fill launch of their own
    buf = fx._zeroed_views([(n * rows * 5 + 2 * n,)], dev)[0] if fx._capturing(dev) else \
        torch.zeros(n * rows * 5 + 2 * n, device=dev)
    stats = buf[:n * rows * 5].view(n * rows, 5)
    rng = buf[n * rows * 5:]   # zeros: the kernels' order-preserving range images start below every value
    seg = (ctypes.c_int64 * (n + 1))(*off)
    with torch.no_grad():
        _lib.call("mms_render_stats_segments", w.data_ptr(), normals.detach().contiguous().data_ptr(),
                  starts.data_ptr(), ends.data_ptr(), n, ctypes.cast(seg, ctypes.c_void_p), S, sidx.data_ptr(),
                  stats.data_ptr(), 5, rows, rng.data_ptr(), fx._s())
    return stats


def nerf_encoding(x: torch.Tensor, F: int) -> torch.Tensor:
    """NeRFEncoding.forward (encodings.py:161-182), frequencies 2^0 .. 2^(F-1), input included, in torch operators
    (twice differentiable: the analytic-gradient fields differentiate through it again)."""
    freqs = 2.0 ** torch.linspace(0.0, F - 1, F, device=x.device)
    scaled = (x[..., None] * freqs).reshape(*x.shape[:-1], -1)
    return torch.cat([x, torch.sin(torch.cat([scaled, scaled + torch.pi / 2.0], dim=-1))], dim=-1)


class RadianceField(nn.Module):
    def __init__(self, base_field: FeatureGridAndMLP):
        super().__init__()
        self.base_field = base_field


class RadianceModel(nn.Module):
    """RadianceModel (radiance_model.py:57-169) with SH(4) directions and n.v (grid.yaml)."""

    def __init__(self, radiance_field: RadianceField, heads: Dict[str, ModalityHead]):
        super().__init__()
        self.radiance_field = radiance_field
        self.modality_heads = nn.ModuleDict(heads)

    def features(self, pos, dirs, normals, geo, S):
        bf = self.radiance_field.base_field
        if isinstance(bf, MLP):
            # mlp methods: RadianceField(MLP) on [x, SH4(d), geo, n.v] (radiance_model.py:114-141)
            return bf.forward_diff(fx.RadInputFunction.apply(pos, dirs, normals, geo, S))
        g = bf.feature_grid
        return fx.RadianceFunction.apply(pos, dirs, normals, geo, g.encoding.hash_table, g.cfg, g.active_levels, S,
                                         *bf.mlp_head.params())


class NeRFField(nn.Module):
    """NeRFField (nerf_field.py:47-105): base MLP, density head (Softplus), head MLP."""

    def __init__(self, base_field: MLP, head_field: MLP, density_head: ModalityHead):
        super().__init__()
        self.base_field = base_field
        self.head_field = head_field
        self.density_head = density_head


class BackgroundModel(nn.Module):
    """BackgroundModel (background_model.py:46-129) with L-inf scene contraction."""

    def __init__(self, background_field: NeRFField, heads: Dict[str, ModalityHead]):
        super().__init__()
        self.background_field = background_field
        self.modality_heads = nn.ModuleDict(heads)

    def field(self, pos, dirs, S):
        bf = self.background_field
        grid, table, active = None, None, 0
        if isinstance(bf.base_field, FeatureGridAndMLP):
            # config 5: hash grid (r = 2) + MLP base field; its coarse-to-fine callback is never registered
            # (BackgroundModel.get_training_callbacks returns [], background_model.py:118-123): all levels active
            g = bf.base_field.feature_grid
            grid, table, active = g.cfg, g.encoding.hash_table, g.active_levels
            base = bf.base_field.mlp_head.params()
        else:
            base = bf.base_field.params()
        dens = bf.density_head.field.params()
        head = bf.head_field.params()
        return fx.BackgroundFunction.apply(pos, dirs, table, S, len(base) // 3, len(dens) // 3, grid, active, *base,
                                           *dens, *head)


# ------------------------------------------------------------------------------------------------
# model
# ------------------------------------------------------------------------------------------------
@dataclass
class ModelSpec:
    """The fields of method_configs 'grid' / 'grid_raw' that shape the hot path (method_configs.py:59-260)."""
    modalities: Dict[str, int]
    log2T: int = 19
    num_levels: int = 16
    min_res: int = 16
    max_res: int = 1024
    radius: float = 1.0
    num_samples: int = 32
    num_importance: int = 32
    upsample_steps: int = 4
    base_variance: float = 64.0
    bg_samples: int = 16
    # field kind: "grid" (hash grid + 3-layer MLPs, 4-tap numerical gradients: methods grid / grid_raw) or "mlp"
    # (8-layer skip MLPs on PE(x), autograd SDF gradients, no hessian: methods mlp / mlp_raw, method_configs.py:303-353)
    fields: str = "grid"
    # background field: "nerf" (PE -> 39-256x4 MLP, head 283-256x3-128, 1-layer heads; method 'grid' / 'grid_raw') or
    # "grid" (config 5 'grid_raw_grid_bg_unbalanced', method_configs.py:428-444: hash grid r = 2 + 71-128-128-256 MLP,
    # head 283-256x3-256, the radiance model's 3-layer heads)
    bg_kind: str = "nerf"
    # HashEncodingConfig.interpolation of every grid: "Linear" (the reference torch path; parity-pinned) or
    # "Smoothstep" (the reference config default, which only its tcnn backend implements; parity-unpinned)
    interpolation: str = "Linear"


@dataclass
class RNG:
    """Uniform draws in the reference's order; None entries are drawn on the device."""
    uniform: Dict[str, torch.Tensor] = field(default_factory=dict)
    pdf: Dict[str, List[torch.Tensor]] = field(default_factory=dict)
    background: Dict[str, torch.Tensor] = field(default_factory=dict)
    # final NeuS spacing bins per modality ([N_hit, S + 1]): given for EVERY modality of a batch, they replace the
    # up-sampler's output (the parity tests pin the rest of the step on the reference's own samples; the sampler is
    # pinned on its own, bit-exact given the reference's SDFs)
    bins: Dict[str, torch.Tensor] = field(default_factory=dict)


_BG_STREAMS: Dict[int, "torch.cuda.Stream"] = {}
# issue point of the background branch in the foreground sampler's launch sequence: after sampler iteration
# MMS_BG_AT (0..upsample_steps-1), after the whole sampler (-1; a captured graph then dispatches the critical branch
# first: 591k -> 602k rays/s, round 4) or before it (-2)
BG_AT = int(os.environ.get("MMS_BG_AT", "-1"))


def background_stream(dev) -> "torch.cuda.Stream":
    """The per-device HIP stream the background branch runs on (BaseModel.concurrent_background)."""
    i = torch.device(dev).index or 0
    if i not in _BG_STREAMS:
        _BG_STREAMS[i] = torch.cuda.Stream(device=i)
    return _BG_STREAMS[i]


def join_background(dev) -> None:
    """Order the current stream after everything queued on the background stream (its backward included)."""
    i = torch.device(dev).index or 0
    if i in _BG_STREAMS:
        torch.cuda.current_stream(i).wait_stream(_BG_STREAMS[i])


class _JoinBackground(torch.autograd.Function):
    """Identity on a background output, applied on the main stream after the join.  Its backward queues a final
    callback that joins the background stream into the caller's stream, so whatever reads the gradients after
    ``backward()`` returns (the weight-norm flush, the optimizer, a test) is ordered after the background's
    backward kernels -- which accumulate the parameter gradients in place, outside autograd's own stream sync."""

    @staticmethod
    def forward(ctx, x, dev_index: int):
        ctx.dev_index = dev_index
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        i = ctx.dev_index
        torch.autograd.Variable._execution_engine.queue_callback(lambda: join_background(i))
        return g, None


def _pad_rows(t: Optional[torch.Tensor], R: int) -> Optional[torch.Tensor]:
    """Injected per-hit-ray uniforms padded with zeros to a fixed-capacity batch of R rows (padding rows' samples are
    discarded)."""
    if t is None or t.shape[0] >= R:
        return t
    return torch.cat([t, t.new_zeros(R - t.shape[0], *t.shape[1:])])


def _linspace(n: int, lo: float = 0.0, hi: float = 1.0) -> torch.Tensor:
    """torch.linspace on the host (the reference's CPU values), for upload."""
    return torch.linspace(lo, hi, n)


def sample_start_positions(bins, n, f, o, d) -> torch.Tensor:
    """Start positions o + d * start of the uniform-spacing samples of ``bins`` [R, S+1] (rays.py:69-81), [R*S, 3]."""
    R, nb = bins.shape
    pos = torch.empty(R * (nb - 1), 3, device=bins.device)
    _lib.call("mms_samples_fwd", bins.data_ptr(), nb, nb, n.data_ptr(), f.data_ptr(), o.data_ptr(), d.data_ptr(),
              0, R, None, None, None, pos.data_ptr(), fx._s())
    return pos


@torch.no_grad()
def neus_sample(n_h, f_h, o_h, d_h, t_rand, pdf_rands, sdf_fn, num_samples: int = 32, num_importance: int = 32,
                upsample_steps: int = 4, base_variance: float = 64.0, lin=None, history: Optional[list] = None,
                after_iter=None, sdf_rays_fn=None):
    """NeuSSampler.generate_ray_samples (ray_samplers.py:448-514) for one modality's hit rays on the HIP kernels.

    n_h / f_h [R] nears / fars, o_h / d_h [R, 3]; t_rand [R, 1] single-jitter uniforms of the uniform sampler (or
    None: evaluation, no jitter), pdf_rands: ``upsample_steps`` [R, 1] PDF-sampler uniforms (or None).
    ``sdf_fn(positions [R*S, 3]) -> sdf [R*S]`` is evaluated at sample starts (the reference's sdf_fn(ray_samples)).
    Returns the final spacing bins [R, num_samples + num_importance + 1]; ``history`` (a list) receives each
    iteration's ``sorted_index`` [R, S + n_new] (merge_ray_samples :38-68) -- bit-exact to the reference's.
    ``after_iter(it)``, if given, is called after iteration ``it``'s launches (an issue point for other work);
    ``sdf_rays_fn(bins, n, f, o, d)``, if given and not returning None, evaluates sdf_fn at the bins' sample starts
    without the positions' own launch."""
    R = n_h.shape[0]
    dev = n_h.device
    if lin is None:
        lin = lambda n, hi, device: _linspace(n, 0.0, hi).to(device)  # noqa: E731
    S = num_samples
    bins = torch.empty(R, S + 1, device=dev)
    _lib.call("mms_stratified_bins", lin(S + 1, 1.0, dev).data_ptr(), S + 1, fx._p(t_rand), 1, R, bins.data_ptr(),
              fx._s())
    n_new = num_importance // upsample_steps
    u_lin = lin(n_new + 1, 1.0 - 1.0 / (n_new + 1), dev)
    sdf_prev, prev_idx, s_prev, n_prev_new = None, None, 0, S
    new_bins = bins
    for it in range(upsample_steps):
        sdf_new = sdf_rays_fn(new_bins, n_h, f_h, o_h, d_h) if sdf_rays_fn is not None else None
        if sdf_new is None:
            sdf_new = sdf_fn(sample_start_positions(new_bins, n_h, f_h, o_h, d_h))
        sdf_new = sdf_new.reshape(-1).contiguous()
        sdf_out = torch.empty(R, S, device=dev)
        new_bins = torch.empty(R, n_new + 1, device=dev)
        merged = torch.empty(R, S + n_new + 1, device=dev)
        sidx = torch.empty(R, S + n_new, dtype=torch.int32, device=dev)
        rnd = pdf_rands[it] if pdf_rands is not None else None
        if rnd is not None:
            rnd = rnd.contiguous()
        _lib.call("mms_neus_step", R, S, bins.data_ptr(), fx._p(sdf_prev), s_prev, sdf_new.data_ptr(), n_prev_new,
                  fx._p(prev_idx), n_h.data_ptr(), f_h.data_ptr(), float(base_variance * 2 ** it), fx._p(rnd),
                  u_lin.data_ptr(), n_new, sdf_out.data_ptr(), new_bins.data_ptr(), merged.data_ptr(),
                  sidx.data_ptr(), fx._s())
        if history is not None:
            history.append(sidx)
        if after_iter is not None:
            after_iter(it)
        sdf_prev, prev_idx, s_prev, n_prev_new = sdf_out, sidx, S, n_new
        bins = merged
        S += n_new
    return bins


class BaseModel(nn.Module):
    """BaseModel (base_model.py:38-199) — collider -> NeuS sampler -> background -> surface -> radiance -> render."""

    def __init__(self, spec: ModelSpec):
        super().__init__()
        self.spec = spec
        mods = spec.modalities

        def grid(radius=1.0):
            enc = HashEncoding(spec.num_levels, 2, spec.min_res, spec.max_res, spec.log2T,
                               interpolation=spec.interpolation)
            return FeatureGrid(enc, radius)

        if spec.fields == "mlp":
            sdf_mlp = MLP(MLPConfig(num_layers=8, hidden_dim=256, activation="Softplus",
                                    activation_params={"beta": 100}, out_activation="None", skip_connections=(4,),
                                    geometric_init=True, geometric_init_bias=0.4), 3 + 36, 257)
            self.surface_model = SurfaceModel(SDFField(sdf_mlp))
            rad_mlp = MLP(MLPConfig(num_layers=8, hidden_dim=256, out_activation="ReLU", skip_connections=(4,)),
                          3 + 25 + 257, 256)
        else:
            sdf_mlp = MLP(MLPConfig(num_layers=3, hidden_dim=256, activation="Softplus",
                                    activation_params={"beta": 100}, out_activation="None", geometric_init=True,
                                    geometric_init_bias=0.4), 3 + 36 + 32, 257)
            self.surface_model = SurfaceModel(SDFField(FeatureGridAndMLP(grid(), sdf_mlp)))
            rad_mlp = MLP(MLPConfig(num_layers=3, hidden_dim=256, out_activation="ReLU"), 3 + 25 + 257 + 32, 256)
        heads = {}
        for m, c in mods.items():
            if m == "polarization":
                heads[m] = ModalityHead("polarization", 256, c, 3, 256, "None")
            else:
                heads[m] = ModalityHead("plain", 256, c, 3, 64, "Sigmoid")
        # construction order = the parameter-initialisation RNG order: radiance MLP, heads, then the radiance grid
        rad_field = rad_mlp if spec.fields == "mlp" else FeatureGridAndMLP(grid(), rad_mlp)
        self.radiance_model = RadianceModel(RadianceField(rad_field), heads)
        # construction order = parameter-initialisation RNG order (base, head, density head, modality heads)
        bg_heads = {}
        if spec.bg_kind == "grid":
            bg_base = FeatureGridAndMLP(grid(2.0), MLP(MLPConfig(num_layers=3, hidden_dim=128, out_activation="ReLU"),
                                                       3 + 36 + 32, 256))
            bg_head = MLP(MLPConfig(num_layers=4, hidden_dim=256, out_activation="ReLU"), 256 + 27, 256)
            dens = ModalityHead("plain", 256, 1, 1, 64, "Softplus")
            for m, c in mods.items():
                if m == "polarization":
                    bg_heads[m] = ModalityHead("polarization", 256, c, 3, 256, "None")
                else:
                    bg_heads[m] = ModalityHead("plain", 256, c, 3, 64, "Sigmoid")
        else:
            bg_base = MLP(MLPConfig(num_layers=4, hidden_dim=256, out_activation="ReLU"), 39, 256)
            bg_head = MLP(MLPConfig(num_layers=4, hidden_dim=256, out_activation="ReLU"), 256 + 27, 128)
            dens = ModalityHead("plain", 256, 1, 1, 64, "Softplus")
            for m, c in mods.items():
                if m == "polarization":
                    bg_heads[m] = ModalityHead("polarization", 128, c, 1, 64, "None")
                else:
                    bg_heads[m] = ModalityHead("plain", 128, c, 1, 64, "Sigmoid")
        self.background_model = BackgroundModel(NeRFField(bg_base, bg_head, dens), bg_heads)
        self._lin = {}
        # training shortcut (SURVEY §8(d) MLP FLOPs note): heads of other modalities only feed outputs no loss reads
        self.own_heads_only = False
        # the background branch on its own HIP stream (overlaps the foreground; same results)
        self.concurrent_background = True

    # -- callbacks (BEFORE_TRAIN_ITERATION), restated from the reference schedules --------------------
    def set_step(self, step: int, max_iters: int = 100000):
        spl = min(int(max_iters * 1.0), int(max_iters / self.spec.num_levels))
        level = min(max(int(step / spl) + 1, 1), self.spec.num_levels)
        if self.spec.fields == "grid":
            self.surface_model.surface_field.field.feature_grid.update_mask(level)
            self.radiance_model.radiance_field.base_field.feature_grid.update_mask(level)
        g = float(np.exp((np.log(self.spec.max_res) - np.log(self.spec.min_res)) / (self.spec.num_levels - 1)))
        delta = max(1.0 / self.spec.max_res, 1.0 / (self.spec.min_res * g ** int(step / spl)))
        self.surface_model.set_numerical_gradients_delta(delta * (self.spec.radius * 2.0))
        self.surface_model.volume_rendering.set_cos_anneal_ratio(min(1.0, step / int(max_iters * 0.05)))

    def _lin_dev(self, n: int, hi: float, device) -> torch.Tensor:
        key = (n, hi, str(device))
        if key not in self._lin:
            self._lin[key] = _linspace(n, 0.0, hi).to(device)
        return self._lin[key]

    # -- NeuS sampler (ray_samplers.py:448-514), no autograd ------------------------------------------
    @torch.no_grad()
    def neus_bins(self, n_h, f_h, o_h, d_h, t_rand, pdf_rands, after_iter=None):
        sp = self.spec
        return neus_sample(n_h, f_h, o_h, d_h, t_rand, pdf_rands, self.surface_model.get_sdf, sp.num_samples,
                           sp.num_importance, sp.upsample_steps, sp.base_variance, lin=self._lin_dev,
                           after_iter=after_iter, sdf_rays_fn=getattr(self.surface_model, "get_sdf_rays", None))

    # -- forward ----------------------------------------------------------------------------------------
    def forward(self, rays: Dict[str, Dict[str, torch.Tensor]], rng: Optional[RNG] = None, cap: Optional[int] = None):
        if getattr(self, "_prep", None) is None:
            self._prep = fx.WeightPrep()    # not a module attribute: the state_dict stays the reference's
        dev = next(iter(rays.values()))["origins"].device
        fx.begin_forward(self._prep, dev)   # every layer's W and MMA images prepared in one batch, looked up below
        try:
            return self._forward(rays, rng, cap)
        finally:
            fx.end_forward()

    def _forward(self, rays, rng, cap):
        """rays[mod] = {"origins", "directions", "up_directions"} ([N,3] device); returns per-modality outputs.

        The reference loops over modalities (base_model.py:102-159), each with its own sampler and field calls; the
        surface, radiance and background fields are shared, so here every modality's rays go through them as ONE
        batch (one collider / compaction / sampler / field / hash-grid / weight-gradient launch per stage for all
        modalities) and only the heads and the compositing stay per modality (HeadsCompositeFunction).  Each
        modality's hit rays are a contiguous segment of the batch, in the reference's per-modality ray order, so every
        per-ray result is the one the modality loop computes.  Modalities with different ray counts (an evaluation
        chunk tail) form separate batches.

        ``cap``: fixed-capacity foreground batch for graph capture (graphs.py).  Each modality's hit rays are
        compacted into ``cap`` rows without reading the hit count on the host; rows past the count repeat the first
        hit ray, composite into a dummy output row N that is cut off, and are skipped by the geometric losses
        (outputs[mod]["count"] is the device hit count), so every gradient they produce is exactly zero and the
        results equal the dynamic path's.  Per-ray outputs ("gradients", "weights", ...) then have ``cap`` rows."""
        rng = rng or RNG()
        groups: Dict[int, List[str]] = {}
        for m in self.spec.modalities:
            groups.setdefault(int(rays[m]["origins"].shape[0]), []).append(m)
        outputs, drew = {}, False
        for gi, (N, mods) in enumerate(groups.items()):
            out, d = self._forward_batch(mods, rays, rng, cap, N, gi)
            outputs.update(out)
            drew = drew or d
        if drew:
            dev = next(iter(rays.values()))["origins"].device
            _lib.call("mms_counter_advance", self._draw_counter(dev).data_ptr(), 1 << 32, fx._s())
        return {m: outputs[m] for m in self.spec.modalities}

    def _draws_for(self, mods, get, rows, shape_tail, dev):
        """Injected per-modality draws concatenated in modality order (per-hit-ray draws cut / zero-padded to
        ``rows[i]``); None when no modality has any and the model is not training (evaluation: no jitter); missing
        ones drawn fresh."""
        parts = [get(m) for m in mods]
        if all(p is None for p in parts) and not self.training:
            return None
        out = []
        for i, p in enumerate(parts):
            if p is None:
                p = torch.rand(rows[i], *shape_tail, device=dev)
            elif tuple(shape_tail) == (1,):
                p = _pad_rows(p[:rows[i]], rows[i])
            out.append(p)
        return out[0] if len(out) == 1 else torch.cat(out, 0)

    def _forward_batch(self, mods, rays, rng, cap, N: int, gi: int):
        sp = self.spec
        nm = len(mods)
        dev = rays[mods[0]]["origins"].device
        s_param = self.surface_model.volume_rendering.density_fn.variance_network.s
        cat = (lambda ts: ts[0]) if nm == 1 else (lambda ts: torch.cat(ts, 0))
        o = cat([rays[m]["origins"] for m in mods])
        d = cat([rays[m]["directions"] for m in mods])
        up = cat([rays[m]["up_directions"] for m in mods])
        nears, fars, bnears, bfars, mask = fx.ColliderFunction.apply(o, d, 1.0)
        seg = N if cap is None else min(int(cap), N)
        gidx, sidx_all, counts = fx.compact_segments(mask, nm, N, seg)
        if cap is None:
            # dynamic shapes: the hit counts on the host (one read for every modality)
            Rm = [int(c) for c in counts.tolist()]
            sidx_m = [sidx_all[i * N:i * N + Rm[i]] for i in range(nm)]
            idx = cat([gidx[i * N:i * N + Rm[i]] for i in range(nm)])
            sidx_cat = cat(sidx_m)
            count_of = [None] * nm
        else:
            Rm = [seg] * nm
            sidx_m = [sidx_all[i * seg:(i + 1) * seg] for i in range(nm)]
            idx, sidx_cat = gidx, sidx_all
            count_of = [counts[i:i + 1] for i in range(nm)]
        off = [0]
        for r in Rm:
            off.append(off[-1] + r)
        R = off[-1]
        o_h, d_h, up_h, n_h, f_h = fx.HitGatherFunction.apply(idx, o, d, up, nears, fars)
        drew = False
        if self.training and not any(m in rng.uniform or m in rng.pdf or m in rng.background for m in mods):
            # every modality's jitter, PDF and background draws in one device launch (mms_uniform)
            t_rand, pdf, bt = self._device_draws(gi, R, nm * N, dev)
            drew = True
        else:
            t_rand = self._draws_for(mods, rng.uniform.get, Rm, (1,), dev)
            pdf = None
            if any(m in rng.pdf for m in mods) or self.training:
                pdf = [self._draws_for(mods, lambda m, j=j: (rng.pdf[m][j] if m in rng.pdf else None), Rm, (1,), dev)
                       for j in range(sp.upsample_steps)]
            bt = self._draws_for(mods, rng.background.get, [N] * nm, (sp.bg_samples + 1,), dev)
        # background (background_model.py:73-111) on all rays.  It depends on the foreground only through the final
        # composite, so it runs on a second HIP stream (forward here, and -- autograd runs each node's backward on its
        # forward's stream -- its backward too), overlapping the NeuS sampler and the surface / radiance work; the
        # main stream joins it right before the composite, and every backward through it ends with a join
        cur = torch.cuda.current_stream(dev)
        bgs = background_stream(dev) if self.concurrent_background else cur
        if bgs is not cur:
            bgs.wait_stream(cur)
        # every head on every modality's rays (radiance_model.py:143-149) -- or, with own_heads_only (training: only
        # the ray's own modality's output reaches the loss, raw_pipeline.py:112-122), just its own
        own = self.own_heads_only and torch.is_grad_enabled()

        # (two-phase backward, functions.PHASE_CUT: the background reads the rays through leaf copies, so phase 1 stops
        # there and the rays' backward runs once, in phase 2)
        o_c, d_c, up_c, bn_c, bf_c = fx.cut(o), fx.cut(d), fx.cut(up), fx.cut(bnears), fx.cut(bfars)

        def background():
            with torch.cuda.stream(bgs):
                # the reported 1 / s (an output only, no loss term reads it: compute_metrics' inv_s) off the main stream
                with torch.no_grad():
                    vn = self.surface_model.volume_rendering.density_fn.variance_network
                    if vn.s.device.type == "cuda":
                        inv_s = torch.empty_like(vn.s)     # one launch (mms_inv_variance) for the four torch ops
                        _lib.call("mms_inv_variance", vn.s.data_ptr(), inv_s.data_ptr(), fx._s())
                    else:
                        inv_s = 1.0 / vn.get_inv_variance()
                nb = sp.bg_samples + 1
                blin = self._lin_dev(nb, 1.0, dev)
                bbins = torch.empty(nm * N, nb, device=dev)
                _lib.call("mms_stratified_bins", blin.data_ptr(), nb, fx._p(bt), nb, nm * N, bbins.data_ptr(), fx._s())
                bpos, bdeltas, _, _ = fx.SamplesFunction.apply(bbins, bn_c, bf_c, o_c, d_c, 1)
                density, bfeat = self.background_model.field(bpos, d_c, sp.bg_samples)
                bw = fx.DensityWeightsFunction.apply(density, bdeltas, sp.bg_samples)
                bg_out = self._heads_composite(self.background_model.modality_heads, mods, own, bfeat, bw, d_c, up_c,
                                               sp.bg_samples, [i * N for i in range(nm)], [N] * nm)
            return inv_s, bg_out
        # NeuS sampling (ray_samplers.py:448-514) -- latency-bound launches the background work overlaps; the
        # background branch is issued at BG_AT in the sampler's launch sequence (a captured graph dispatches in issue
        # order, so the critical foreground branch goes first)
        bg_res = []
        grad_on = torch.is_grad_enabled()
        at = BG_AT if BG_AT < sp.upsample_steps else -1

        def issue_bg(it=None):
            if not bg_res:
                with torch.set_grad_enabled(grad_on):
                    bg_res.append(background())
        if at == -2:
            issue_bg()
        if rng.bins and not all(m in rng.bins for m in mods):
            raise ValueError(f"injected NeuS bins cover {sorted(rng.bins)} but the batch has modalities {list(mods)}: "
                             "give every modality's bins or none")
        if rng.bins:
            # injected samples: each modality's bins, fixed-capacity segments padded with their first ray's bins (the
            # padding rows repeat the first hit ray)
            parts = []
            for i, m in enumerate(mods):
                b = rng.bins[m][:Rm[i]]
                if b.shape[0] < Rm[i]:
                    b = torch.cat([b, b[:1].expand(Rm[i] - b.shape[0], -1)])
                parts.append(b)
            bins = cat(parts).contiguous()
        else:
            bins = self.neus_bins(n_h.detach(), f_h.detach(), o_h.detach(), d_h.detach(), t_rand, pdf,
                                  after_iter=(lambda it: issue_bg() if it == at else None) if at >= 0 else None)
        issue_bg()
        inv_s, bg_out = bg_res[0]
        S = bins.shape[1] - 1
        pos, deltas, starts, ends = fx.SamplesFunction.apply(bins, n_h, f_h, o_h, d_h, 0)
        # surface + radiance
        sdf, geo, grads, hess, normals = self.surface_model(pos)
        vr = self.surface_model.volume_rendering
        # the SDF side's tensors as the rendering side reads them (leaf copies under functions.PHASE_CUT)
        sdf, geo, grads, hess = fx.cut(sdf), fx.cut(geo), fx.cut(grads), fx.cut(hess)
        pos_c, d_hc, up_hc, deltas = fx.cut(pos), fx.cut(d_h), fx.cut(up_h), fx.cut(deltas)
        w = fx.NeusWeightsFunction.apply(sdf, grads, d_hc, deltas, s_param, vr._cos_anneal_ratio, S)
        feat = self.radiance_model.features(pos_c, d_hc, normals.detach(), geo, S)
        # padded batches: the statistics scatter their padding rays into a dummy row N (cut off below); the composite
        # discards them (mms_composite nout = N), so its outputs need no cut -- no slice in the autograd graph, no
        # padded copy of the background
        rows = N if cap is None else N + 1
        if bgs is not cur:
            cur.wait_stream(bgs)
            inv_s.record_stream(cur)
            for k in list(bg_out):
                bg_out[k].record_stream(cur)    # made on the background stream, read (and freed) on this one
                if torch.is_grad_enabled() and bg_out[k].requires_grad:
                    bg_out[k] = _JoinBackground.apply(bg_out[k], torch.device(dev).index or 0)
        fg = self._heads_composite(self.radiance_model.modality_heads, mods, own, feat, w, d_hc, up_hc, S, off[:-1], Rm,
                                   sidx=sidx_m, bgs=bg_out, rows=N, hits=[mask[i * N:(i + 1) * N] for i in range(nm)])
        # accumulation / normals / depth renderers (renderers.py:176-242, no grad): one launch pair for all modalities
        stats = _render_stats_segments(w, normals, starts, ends, off, S, sidx_cat, rows, dev)
        geo_batch = {"grads": grads, "hess": hess, "counts": None if cap is None else counts, "seg_rays": seg, "S": S,
                     "mods": tuple(mods)}
        outputs = {}
        for i, mod in enumerate(mods):
            a, b = off[i], off[i + 1]
            out = {h: v for (k, h), v in fg.items() if k == i}
            st = stats[i * rows:i * rows + N]
            out["normals"] = st[:, 1:4]
            out["depth"] = st[:, 4:5]
            out["accumulation"] = st[:, 0:1]
            out["count"] = count_of[i]
            out["gradients"] = grads[a * S:b * S].view(b - a, S, 3)
            out["hessians"] = hess[a * S:b * S].view(b - a, S, 3) if hess is not None else None
            out["inv_s"] = inv_s
            out["weights"] = w[a:b]
            out["bins"] = bins[a:b]
            out["mask"] = mask[i * N:(i + 1) * N]
            out["_geo"] = geo_batch
            outputs[mod] = out
        return outputs, drew

    def _heads_composite(self, heads: nn.ModuleDict, mods, own: bool, feat, w, dirs, ups, S: int, seg_off, seg_rays,
                         sidx=None, bgs=None, rows=None, hits=None):
        """Every (modality segment, head) output of one branch through HeadsCompositeFunction: {(segment, head name):
        [rows, C]}.  With gradients each pair is a job of its own (its head's backward covers exactly its rows);
        without (evaluation) each head runs once over the whole batch and the pairs composite slices of it."""
        names = list(heads)
        specs, params = [], []
        for h in names:
            mod = heads[h]
            ps = mod.field.params()
            specs.append(fx.HeadSpec(mod.kind, mod.field.acts, mod.field.precision_key, len(ps)))
            params += ps
        pairs = [(i, mods[i]) for i in range(len(mods)) if mods[i] in heads] if own else \
            [(i, h) for i in range(len(mods)) for h in names]
        grad = torch.is_grad_enabled()
        jobs, items, bg_list, keys, out = [], [], [], [], {}
        job_of_head = {}
        for i, h in pairs:
            bg = None if bgs is None else bgs[(i, h)]
            if seg_rays[i] == 0:
                out[(i, h)] = bg        # no hit ray: the modality's output is its background
                continue
            hid = names.index(h)
            if grad:
                jobs.append((hid, seg_off[i], seg_rays[i]))
                j, sub = len(jobs) - 1, 0
            else:
                if hid not in job_of_head:
                    jobs.append((hid, 0, sum(seg_rays)))
                    job_of_head[hid] = len(jobs) - 1
                j, sub = job_of_head[hid], seg_off[i]
            items.append((j, sub, seg_rays[i], seg_off[i], None if sidx is None else sidx[i], rows,
                          None if hits is None else hits[i]))
            bg_list.append(bg)
            keys.append((i, h))
        if items:
            res = fx.HeadsCompositeFunction.apply(feat, w, dirs, ups, S, specs, jobs, items, *bg_list, *params)
            if not isinstance(res, tuple):
                res = (res,)
            out.update(zip(keys, res))
        return out

    # -- training-mode uniform draws on the device ----------------------------------------------------
    def seed_draws(self, seed: int, dev) -> None:
        """Restart the forward's device draw stream at (seed, counter 0): two forwards after the same seed_draws draw
        the same values (torch.cuda.manual_seed's role for the reference's torch.rand draws)."""
        self.draw_seed = int(seed)
        self._draw_counter(dev).zero_()

    def _draw_counter(self, dev) -> torch.Tensor:
        """Device Philox counter of the forward's draws (not a registered buffer: the state_dict stays the
        reference's); advanced once per forward on the device, so captured graphs draw fresh values every replay."""
        c = getattr(self, "_draw_ctr", None)
        if c is None or c.device != dev:
            c = torch.zeros(1, dtype=torch.int64, device=dev)
            self._draw_ctr = c
        return c

    def _device_draws(self, gi: int, R: int, N: int, dev):
        """(jitter [R,1], PDF draws 4 x [R,1], background [N, bg+1]) ~ U[0,1) of a whole modality batch from one
        mms_uniform launch, the stream keyed by (draw_seed, batch index); the reference draws these with torch.rand in
        the same shapes per modality (SURVEY §8(d) 'RNG')."""
        sp = self.spec
        nb = sp.bg_samples + 1
        k = sp.upsample_steps
        buf = torch.empty(R * (1 + k) + N * nb, device=dev)
        _lib.call("mms_uniform", int(getattr(self, "draw_seed", 0)) & ((1 << 64) - 1), gi,
                  self._draw_counter(dev).data_ptr(), 0, buf.numel(), buf.data_ptr(), fx._s())
        t_rand = buf[:R].view(R, 1)
        pdf = [buf[R * (1 + j):R * (2 + j)].view(R, 1) for j in range(k)]
        bt = buf[R * (1 + k):].view(N, nb)
        return t_rand, pdf, bt
