"""Reference-signature plugin classes: the drop-in surface for MMS-FW's config-driven modules.

MMS-FW instantiates every module as ``config._target(config, **kw)`` (/root/reference/src/configs/configs.py:55-63).
The classes here take the reference's own config objects (duck-typed: the same field names; the mirror dataclasses
below exist for callers without the reference) and keep the reference's forward signatures and parameter names, so
a maintainer switches a method config over by pointing ``_target`` at them.  Every forward runs
on the HIP kernels of libmms_hip.so (functions.py); nothing here has a CPU path.

  HashEncoding(config, in_dim)                    encodings.py:184-310   forward(x_hat [...,3]) -> [..., L F]
  NeRFEncoding(config, in_dim)                    encodings.py:131-182   forward(x [...,3])
  FeatureGrid(config, input_dim, output_dim)      feature_structures.py:56-127
  FeatureGridAndMLP(config, input_dim, output_dim) feature_structures.py:130-173
  SDFField(config)                                surface_field.py:80-116  forward(x) -> (sdf, geo), single_output
  RadianceField(config, position_dim, view_direction_dim, additional_input_dim, output_dim)
                                                  radiance_field.py:50-80  forward(positions, view_directions, extra)
  NeuSSampler(config)                             ray_samplers.py:425-551  generate_ray_samples(ray_bundles, sdf_fn=)
  Renderer(config)                                renderers.py:40-136      render(weights, data_fields, mask)
  RayGenerator(cameras, pose_optimizer, offset)   ray_generators.py:30-81  forward(coords) -> Dict[str, RayBundle]
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Callable, Dict, Optional

import numpy as np
import torch
from torch import nn

from . import _lib
from . import functions as fx
from . import model as mm
from . import pipeline as pl
from .hip_ops import HashGridFunction


# ------------------------------------------------------------------------------------------------
# config mirrors (same field names and defaults as the reference dataclasses)
# ------------------------------------------------------------------------------------------------
class _Setup:
    def setup(self, **kwargs):
        """InstantiateConfig.setup (configs.py:55-63)."""
        return self._target(self, **kwargs)


@dataclass
class HashEncodingConfig(_Setup):
    """encodings.py:48-67 (implementation 'hip' added; interpolation "Linear" is the parity-pinned torch mode,
    "Smoothstep" -- the reference default, tcnn's -- runs too, parity-unpinned)."""
    num_levels: int = 16
    features_per_level: int = 2
    min_res: int = 16
    max_res: int = 2048
    log2_hashmap_size: int = 19
    hash_init_scale: float = 0.001
    interpolation: Optional[str] = "Linear"
    implementation: str = "hip"

    @property
    def _target(self):
        return HashEncoding


@dataclass
class NeRFEncodingConfig(_Setup):
    """encodings.py:80-91."""
    num_frequencies: int = 6
    min_freq_exp: float = 0.0
    max_freq_exp: int = 5
    include_input: bool = True

    @property
    def _target(self):
        return NeRFEncoding


@dataclass
class FeatureGridConfig(_Setup):
    """feature_structures.py:28-42."""
    encoding: Any = field(default_factory=HashEncodingConfig)
    coarse_to_fine: bool = True
    steps_per_level_ratio: float = 1.0
    level_init: int = 1
    radius: float = 1

    @property
    def _target(self):
        return FeatureGrid


@dataclass
class FeatureGridAndMLPConfig(_Setup):
    """feature_structures.py:44-53."""
    feature_grid: Any = field(default_factory=FeatureGridConfig)
    mlp_head: Any = field(default_factory=mm.MLPConfig)
    return_features: bool = False
    output_dim: Optional[int] = None

    @property
    def _target(self):
        return FeatureGridAndMLP


@dataclass
class SDFFieldConfig(_Setup):
    """surface_field.py:26-46."""
    use_position_encoding: bool = True
    position_encoding: Any = field(default_factory=NeRFEncodingConfig)
    geo_feature_dim: int = 256
    field: Any = field(default_factory=FeatureGridAndMLPConfig)
    inside_outside: bool = False

    @property
    def _target(self):
        return SDFField


@dataclass
class RadianceFieldConfig(_Setup):
    """radiance_field.py:30-35."""
    base_field: Any = field(default_factory=FeatureGridAndMLPConfig)

    @property
    def _target(self):
        return RadianceField


@dataclass
class NeuSSamplerConfig(_Setup):
    """ray_samplers.py:108-120 (SamplerConfig fields used by the NeuS path)."""
    num_samples: int = 64
    num_samples_importance: int = 64
    num_upsample_steps: int = 4
    base_variance: float = 64
    single_jitter: bool = True
    train_stratified: bool = True

    @property
    def _target(self):
        return NeuSSampler


@dataclass
class RendererConfig(_Setup):
    """renderers.py:28-40: which fields composite as radiance (every other key: semantic / normals / depth)."""
    renderers: Dict[str, Any] = field(default_factory=dict)
    background_color: str = "None"

    @property
    def _target(self):
        return Renderer


# ------------------------------------------------------------------------------------------------
# tensor dataclasses (cameras/rays.py)
# ------------------------------------------------------------------------------------------------
@dataclass
class RayBundle:
    """rays.py:220-300 (the fields the hot path reads)."""
    origins: torch.Tensor
    directions: torch.Tensor
    pixel_area: torch.Tensor
    camera_indices: Optional[torch.Tensor] = None
    up_directions: Optional[torch.Tensor] = None
    directions_norm: Optional[torch.Tensor] = None
    nears: Optional[torch.Tensor] = None
    fars: Optional[torch.Tensor] = None

    @property
    def shape(self):
        return self.origins.shape[:-1]

    def __getitem__(self, idx) -> "RayBundle":
        """TensorDataclass.__getitem__ (tensor_dataclass.py:149-162): index every field."""
        kw = {k: (getattr(self, k)[idx] if getattr(self, k) is not None else None)
              for k in self.__dataclass_fields__}
        return RayBundle(**kw)


@dataclass
class Frustums:
    """rays.py:36-100: per-sample views (rays broadcast over the sample axis, no copies)."""
    origins: torch.Tensor
    directions: torch.Tensor
    starts: torch.Tensor
    ends: torch.Tensor
    pixel_area: Optional[torch.Tensor] = None
    up_directions: Optional[torch.Tensor] = None
    positions: Optional[torch.Tensor] = None   # start positions from the samples kernel [R, S, 3]

    def get_start_positions(self) -> torch.Tensor:
        if self.positions is not None:
            return self.positions
        return self.origins + self.directions * self.starts

    def get_positions(self) -> torch.Tensor:
        return self.origins + self.directions * (self.starts + self.ends) / 2


@dataclass
class RaySamples:
    """rays.py:118-217 (the fields the NeuS path produces)."""
    frustums: Frustums
    camera_indices: Optional[torch.Tensor] = None
    deltas: Optional[torch.Tensor] = None
    spacing_starts: Optional[torch.Tensor] = None
    spacing_ends: Optional[torch.Tensor] = None

    @property
    def shape(self):
        return self.frustums.starts.shape[:-1]


# ------------------------------------------------------------------------------------------------
# field components
# ------------------------------------------------------------------------------------------------
def _check_interp(cfg) -> str:
    """HashEncodingConfig.interpolation (encodings.py:64-67): "Linear" (the torch backend's only mode, :235-238; the
    parity-pinned one) or "Smoothstep" (tcnn's, parity-unpinned: tcnn is not available to pin it)."""
    interp = getattr(cfg, "interpolation", None)
    if interp not in (None, "Linear", "Smoothstep"):
        raise ValueError(f"interpolation '{interp}' is not supported by the hip hash grid (Linear or Smoothstep)")
    return interp or "Linear"


class HashEncoding(mm.HashEncoding):
    """HashEncoding(config, in_dim) (encodings.py:184-233); forward takes x_hat in [0, 1] like pytorch_fwd
    (:263-304).  Parameter ``hash_table`` [L 2^log2T, F], initialised U(-1, 1) * hash_init_scale (:230-233)."""

    def __init__(self, config, in_dim: int = 3):
        if in_dim != 3:
            raise ValueError("HashEncoding takes 3-D inputs")
        interp = _check_interp(config)
        super().__init__(config.num_levels, config.features_per_level, config.min_res, config.max_res,
                         config.log2_hashmap_size, config.hash_init_scale, interpolation=interp)
        self.config = config
        self.input_dim = in_dim

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        shp = x.shape[:-1]
        out = HashGridFunction.apply(x.reshape(-1, 3), self.hash_table, self.scalings.tolist(), self.log2T, 0.0,
                                     self.num_levels, self.interp)
        return out.reshape(*shp, self.get_out_dim())


class _NeRFEncodingFunction(torch.autograd.Function):
    """[x, sin(x_i 2^k) (i-major), sin(x_i 2^k + pi/2)] on the panel kernel (mms_geo_input_fwd, no taps)."""

    @staticmethod
    def forward(ctx, x, F: int):
        M = x.shape[0]
        X = fx._alloc(M, 3 + 6 * F, x.device)
        x = x.contiguous()
        _lib.call("mms_geo_input_fwd", x.data_ptr(), 3, M, 0, 0.0, F, X.data_ptr(), X.stride(0), fx._s())
        ctx.X, ctx.F = X, F
        return X

    @staticmethod
    def backward(ctx, dX):
        X, F = ctx.X, ctx.F
        M = X.shape[0]
        dX = dX if dX.stride(1) == 1 else dX.contiguous()
        dpos = torch.zeros(M, 3, device=X.device)
        _lib.call("mms_geo_input_bwd", X.data_ptr(), X.stride(0), dX.data_ptr(), dX.stride(0), None, 0, M, 0, F,
                  dpos.data_ptr(), 3, fx._s())
        ctx.X = None
        return dpos, None


class NeRFEncoding(nn.Module):
    """NeRFEncoding(config, in_dim) (encodings.py:131-182) for the configs' frequency ladders 2^0 .. 2^(F-1) with
    the input included (every method config's position / direction encodings)."""

    def __init__(self, config, in_dim: int = 3):
        super().__init__()
        F = int(config.num_frequencies)
        if in_dim != 3 or not config.include_input or float(config.min_freq_exp) != 0.0 or \
                float(config.max_freq_exp) != F - 1:
            raise NotImplementedError("hip NeRFEncoding: 3-D input, include_input, frequencies 2^0 .. 2^(F-1)")
        self.config, self.input_dim, self.F = config, in_dim, F

    def get_out_dim(self) -> int:
        return self.input_dim * (2 * self.F + 1)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        shp = x.shape[:-1]
        return _NeRFEncodingFunction.apply(x.reshape(-1, 3), self.F).reshape(*shp, self.get_out_dim())


class FeatureGrid(mm.FeatureGrid):
    """FeatureGrid(config, input_dim, output_dim) (feature_structures.py:56-127)."""

    def __init__(self, config, input_dim: Optional[int] = None, output_dim: Optional[int] = None):
        super().__init__(HashEncoding(config.encoding, 3), float(config.radius))
        self.config = config
        self.output_dim = self.encoding.get_out_dim()
        self.active_levels = self.encoding.num_levels   # hash_encoding_mask starts all ones (:70-73)

    @property
    def hash_encoding_mask(self) -> torch.Tensor:
        F = self.encoding.features
        m = torch.ones(self.encoding.num_levels * F)
        m[self.active_levels * F:] = 0
        return m

    def level_for_step(self, step: int, max_num_iterations: int) -> int:
        """The BEFORE_TRAIN_ITERATION callback's level (feature_structures.py:97-108)."""
        c = self.config
        spl = min(int(max_num_iterations * c.steps_per_level_ratio), int(max_num_iterations / c.encoding.num_levels))
        return min(max(int(step / spl) + 1, c.level_init), c.encoding.num_levels)

    def get_out_dim(self) -> int:
        return self.output_dim


def _acts_of(mlp: mm.MLP):
    return mlp.acts


class FeatureGridAndMLP(nn.Module):
    """FeatureGridAndMLP(config, input_dim, output_dim) (feature_structures.py:130-173): MLP on
    [x, auxiliary columns, grid(x)].  ``family`` picks the precision preset entry (functions.PRECISION)."""

    def __init__(self, config, input_dim: int = 3, output_dim: Optional[int] = None, family: str = "radiance"):
        super().__init__()
        self.config = config
        self.feature_grid = FeatureGrid(config.feature_grid, input_dim=3)
        self.input_dim = input_dim
        self.mlp_head = mm.MLP(config.mlp_head, input_dim + self.feature_grid.get_out_dim(), output_dim)
        self.output_dim = self.mlp_head.output_dim
        self.family = family

    def get_out_dim(self) -> int:
        return self.output_dim

    def forward(self, input_tensor: torch.Tensor):
        shp = input_tensor.shape[:-1]
        x = input_tensor.reshape(-1, input_tensor.shape[-1])
        g = self.feature_grid
        out, feats = fx.FeatureGridMLPFunction.apply(x, g.encoding.hash_table, g.cfg, g.active_levels,
                                                     _acts_of(self.mlp_head), fx.PRECISION[self.family],
                                                     *self.mlp_head.params())
        out = out.reshape(*shp, out.shape[-1])
        if getattr(self.config, "return_features", False):
            return out, feats.reshape(*shp, feats.shape[-1])
        return out


# ------------------------------------------------------------------------------------------------
# fields
# ------------------------------------------------------------------------------------------------
class SDFField(nn.Module):
    """SDFField(config) (surface_field.py:80-116): forward(x [...,3]) -> (sdf [...,1], geo [...,G])."""

    def __init__(self, config):
        super().__init__()
        self.config = config
        self.position_encoding = NeRFEncoding(config.position_encoding, in_dim=3)
        self.input_dim = self.position_encoding.get_out_dim() if config.use_position_encoding else 3
        self.output_dim = 1 + config.geo_feature_dim if config.geo_feature_dim is not None else 1
        self.field = FeatureGridAndMLP(config.field, input_dim=self.input_dim, output_dim=self.output_dim,
                                       family="sdf")
        self._fused = (config.use_position_encoding and self.position_encoding.F == 6 and self.input_dim == 39
                       and self.field.feature_grid.get_out_dim() == 32 and config.geo_feature_dim is not None)

    def forward(self, x: torch.Tensor):
        shp = x.shape[:-1]
        xf = x.reshape(-1, 3)
        if self._fused:
            g = self.field.feature_grid
            sdf, geo = fx.SDFFieldFunction.apply(xf, g.encoding.hash_table, g.cfg, g.active_levels,
                                                 *self.field.mlp_head.params())
        else:
            h = self.position_encoding(xf) if self.config.use_position_encoding else xf
            out = self.field(h)
            if self.config.geo_feature_dim is None:
                return out.reshape(*shp, 1), None
            sdf, geo = out[:, :1], out[:, 1:]
        return sdf.reshape(*shp, 1), geo.reshape(*shp, geo.shape[-1])

    def single_output(self, x: torch.Tensor) -> torch.Tensor:
        """surface_field.py:70-72."""
        return self.forward(x)[0]


class RadianceField(nn.Module):
    """RadianceField(config, position_dim, view_direction_dim, additional_input_dim, output_dim)
    (radiance_field.py:50-80)."""

    def __init__(self, config, position_dim: int = 3, view_direction_dim: int = 3, additional_input_dim: int = 0,
                 output_dim: int = 3):
        super().__init__()
        self.config = config
        self.input_dim = position_dim + view_direction_dim + additional_input_dim
        self.output_dim = output_dim
        self.base_field = FeatureGridAndMLP(config.base_field, input_dim=self.input_dim, output_dim=output_dim,
                                            family="radiance")

    def forward(self, positions, view_directions, additional_inputs):
        inputs = torch.cat([positions, view_directions, additional_inputs], dim=-1)
        return self.base_field(inputs)


# ------------------------------------------------------------------------------------------------
# sampler / renderer / ray generator
# ------------------------------------------------------------------------------------------------
class _SampleView:
    """What a reference sdf_fn reads from the sampler's intermediate RaySamples: the start positions."""

    def __init__(self, positions: torch.Tensor):
        self.frustums = Frustums(origins=None, directions=None, starts=None, ends=None, positions=positions)


def ray_samples_from_bins(bins: torch.Tensor, bundle: RayBundle, kind: int = 0) -> RaySamples:
    """RayBundle.get_ray_samples (rays.py:304-349) of spacing bins [R, S+1] on the samples kernel."""
    R, nb = bins.shape
    S = nb - 1
    n, f = bundle.nears.reshape(-1).contiguous(), bundle.fars.reshape(-1).contiguous()
    o, d = bundle.origins.contiguous(), bundle.directions.contiguous()
    pos, deltas, starts, ends = fx.SamplesFunction.apply(bins, n, f, o, d, kind)
    fr = Frustums(origins=o[:, None, :].expand(R, S, 3), directions=d[:, None, :].expand(R, S, 3),
                  starts=starts.view(R, S, 1), ends=ends.view(R, S, 1),
                  pixel_area=bundle.pixel_area[:, None, :].expand(R, S, 1) if bundle.pixel_area is not None else None,
                  up_directions=(bundle.up_directions[:, None, :].expand(R, S, 3)
                                 if bundle.up_directions is not None else None),
                  positions=pos.view(R, S, 3))
    cam = bundle.camera_indices[:, None, :].expand(R, S, 1) if bundle.camera_indices is not None else None
    return RaySamples(frustums=fr, camera_indices=cam, deltas=deltas.view(R, S, 1),
                      spacing_starts=bins[:, :-1, None], spacing_ends=bins[:, 1:, None])


class NeuSSampler(nn.Module):
    """NeuSSampler(config).generate_ray_samples(ray_bundles, sdf_fn=...) (ray_samplers.py:448-514): uniform
    single-jitter bins, ``num_upsample_steps`` NeuS up-sampling iterations on the HIP kernels (bit-exact bins and
    merge order, tests/test_gpu_sampler.py).  ``sdf_fn(ray_samples)`` is the reference's callback: it reads
    ``ray_samples.frustums.get_start_positions()``.  Uniform draws: torch.rand on the device in training mode, none
    in eval mode; ``rand`` = {mod: (t_rand [R,1], [pdf_rand [R,1]] * steps)} injects them (parity tests)."""

    def __init__(self, config, **kwargs):
        super().__init__()
        self.config = config

    def generate_ray_samples(self, ray_bundles: Dict[str, RayBundle] = None, **kwargs):
        sdf_fn: Callable = kwargs.get("sdf_fn")
        rand = kwargs.get("rand") or {}
        assert ray_bundles is not None and sdf_fn is not None
        c = self.config
        out = {}
        for mod, rb in ray_bundles.items():
            if rb is None:
                out[mod] = None
                continue
            R = rb.origins.shape[0]
            if R == 0:
                out[mod] = torch.tensor([])
                continue
            dev = rb.origins.device
            t_rand, pdf = rand.get(mod, (None, None))
            if t_rand is None and self.training:
                t_rand = torch.rand(R, 1, device=dev)
            if pdf is None and self.training:
                pdf = [torch.rand(R, 1, device=dev) for _ in range(c.num_upsample_steps)]
            n, f = rb.nears.reshape(-1).contiguous(), rb.fars.reshape(-1).contiguous()

            def positions_sdf(p, _fn=sdf_fn, _R=R):
                s = _fn(_SampleView(p.view(_R, -1, 3)))
                return s.reshape(-1)

            bins = mm.neus_sample(n.detach(), f.detach(), rb.origins.detach().contiguous(),
                                  rb.directions.detach().contiguous(), t_rand, pdf, positions_sdf, c.num_samples,
                                  c.num_samples_importance, c.num_upsample_steps, float(c.base_variance))
            out[mod] = ray_samples_from_bins(bins, rb)
        return {"ray_samples_per_modality": out}


class Renderer(nn.Module):
    """Renderer(config).render(weights [R,S,1], data_fields, mask [N] bool) (renderers.py:75-136).  Radiance keys
    composite with the background on the composite kernel; 'normals' / 'depth' / other keys as the reference's
    Normals / Depth / Semantic renderers; 'accumulation' always."""

    def __init__(self, config, **kwargs):
        super().__init__()
        self.config = config

    def _background(self, bg, mask, C):
        colour = getattr(self.config, "background_color", "None")
        N, dev = mask.shape[0], mask.device
        if colour == "None" and bg is not None:
            return bg
        if colour == "white":
            return torch.ones(N, C, device=dev)
        if colour == "black":
            return torch.zeros(N, C, device=dev)
        if colour == "random":
            return torch.rand(N, C, device=dev)
        raise ValueError(f"Background color {colour} not supported.")

    def render(self, weights: torch.Tensor, data_fields: Dict[str, Any], mask: torch.Tensor):
        R, S = weights.shape[0], weights.shape[1]
        w = weights.reshape(R, S)
        idx = torch.nonzero(mask.reshape(-1)).reshape(-1)
        N = mask.shape[0]
        bgs = data_fields.get("background")
        outputs = {}
        for mod, val in data_fields.items():
            if mod == "background":
                continue
            if mod in self.config.renderers:
                C = val.shape[-1]
                bg = self._background(bgs[mod] if bgs is not None else None, mask, C)
                outputs[mod] = fx.CompositeFunction.apply(w, val.reshape(R * S, C), bg.reshape(N, C), idx, S)
            elif mod == "depth":
                steps = ((val.frustums.starts + val.frustums.ends) / 2).reshape(R, S)
                d = (w * steps).sum(-1, keepdim=True)
                d = torch.clip(d, steps.min(), steps.max())
                outputs[mod] = torch.zeros(N, 1, device=w.device, dtype=d.dtype).index_copy(0, idx, d)
            else:
                C = val.shape[-1]
                v = fx.CompositeFunction.apply(w, val.reshape(R * S, C), None, None, S)
                outputs[mod] = torch.zeros(N, C, device=w.device, dtype=v.dtype).index_copy(0, idx, v)
        acc = w.sum(-1, keepdim=True)
        outputs["accumulation"] = torch.zeros(N, 1, device=w.device, dtype=acc.dtype).index_copy(0, idx, acc)
        return outputs


class RayGenerator(nn.Module):
    """RayGenerator(cameras, pose_optimizer, pixel_offset).forward(coords) -> Dict[str, RayBundle]
    (ray_generators.py:54-81) on the raygen kernel with SO3xR3 pose refinement."""

    def __init__(self, cameras: Dict[str, pl.DeviceCameras], pose_optimizer: pl.CameraOptimizer,
                 pixel_offset: float = 0.0):
        super().__init__()
        self.inner = pl.RayGenerator(cameras, pose_optimizer, pixel_offset)

    def forward(self, ray_indices: Dict[str, torch.Tensor]) -> Dict[str, RayBundle]:
        rays = self.inner(ray_indices)
        return {m: RayBundle(origins=r["origins"], directions=r["directions"], pixel_area=r["pixel_area"],
                             camera_indices=r["camera_indices"].long(), up_directions=r["up_directions"],
                             directions_norm=r["directions_norm"]) for m, r in rays.items()}


def collide(bundle: RayBundle, radius: float = 1.0):
    """SphereCollider.forward (scene_colliders.py:60-80) on a RayBundle: sets nears / fars, returns the hit mask."""
    n, f, _, _, mask = fx.ColliderFunction.apply(bundle.origins.contiguous(), bundle.directions.contiguous(), radius)
    bundle.nears, bundle.fars = n[:, None], f[:, None]
    return mask.bool()
