"""Training step around the hot path: pixel sampling, ray generation with pose refinement, the model,
losses and the optimizer step — the MI355X counterpart of RawPipeline/BasePipeline.train_step
(/root/reference/src/pipelines/raw_pipeline.py:67-82, base_pipeline.py:138-153).

Parameters of each optimizer group live in ONE flat fp32 buffer (params are views into it) and so do
their gradients, so grad-norm clipping is one reduction, AdamW is one launch, and the data-parallel
gradient all-reduce (ddp.py) is a handful of large RCCL calls instead of one per tensor.
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
from torch import nn

from . import _lib
from . import functions as fx
from . import scene as mscene
from .model import RNG, BaseModel, ModelSpec


def _s():
    return torch.cuda.current_stream().cuda_stream


# ------------------------------------------------------------------------------------------------
# cameras / rays
# ------------------------------------------------------------------------------------------------
class DeviceCameras:
    """Per-modality camera tensors on the device (Cameras fields used by cameras.py:460-703)."""

    def __init__(self, cams: mscene.ModalityCameras, device):
        self.c2w = cams.c2w.reshape(-1, 12).contiguous().to(device)
        self.fx = cams.fx.contiguous().to(device)
        self.fy = cams.fy.contiguous().to(device)
        self.cx = cams.cx.contiguous().to(device)
        self.cy = cams.cy.contiguous().to(device)
        self.distortion = cams.distortion.contiguous().to(device) if cams.distortion is not None else None
        self.num = cams.c2w.shape[0]


def exp_map_so3xr3(tangent: torch.Tensor) -> torch.Tensor:
    """lie_groups.py:28-63 on the (1 x 6) / (C x 6) pose deltas: one mms_pose_exp_fwd launch (and one backward)."""
    return fx.PoseExpFunction.apply(tangent)


class CameraOptimizer(nn.Module):
    """CameraOptimizer (camera_optimizers.py:34-133), SO3xR3, shared (1 x 6) or per-camera deltas."""

    def __init__(self, modalities: List[str], num_cameras: Dict[str, int], mode: str = "SO3xR3",
                 shared: bool = True, optimize: Optional[Dict[str, bool]] = None):
        super().__init__()
        self.mode = mode
        self.shared = shared
        self.optimize = optimize or {m: True for m in modalities}
        self.pose_adjustment = nn.ParameterDict()
        if mode != "off":
            for m in modalities:
                n = 1 if shared else num_cameras[m]
                self.pose_adjustment[m] = nn.Parameter(torch.zeros(n, 6))

    def matrices(self, mod: str, device) -> torch.Tensor:
        if self.mode == "off" or mod not in self.pose_adjustment:
            return torch.eye(4, device=device)[None, :3, :4]
        mat = exp_map_so3xr3(self.pose_adjustment[mod])
        return mat if self.optimize.get(mod, True) else mat.detach()


class RayGenerator(nn.Module):
    """RayGenerator.forward (ray_generators.py:54-81) on the raygen kernel."""

    def __init__(self, cameras: Dict[str, DeviceCameras], pose_optimizer: CameraOptimizer, pixel_offset: float):
        super().__init__()
        self.cameras = cameras
        self.pose_optimizer = pose_optimizer
        self.pixel_offset = float(pixel_offset)

    def forward(self, coords: Dict[str, torch.Tensor]):
        out = {}
        for mod, c in coords.items():
            cams = self.cameras[mod]
            mats = self.pose_optimizer.matrices(mod, c.device)
            o, d, u, a, dn = fx.RaysFunction.apply(mats, c, cams, self.pixel_offset)
            out[mod] = {"origins": o, "directions": d, "up_directions": u, "pixel_area": a, "directions_norm": dn,
                        "camera_indices": c[:, :1]}
        return out


class UniformPixelSampler:
    """UniformPixelSampler.sample (pixel_samplers.py:71-89): host CPU generator, draw order frame, x, y."""

    def __init__(self, num_rays_per_modality: int, seed: int):
        self.n = num_rays_per_modality
        self.generator = torch.Generator()
        self.generator.manual_seed(seed)

    def sample(self, frames: Dict[str, dict]):
        coords, sel = {}, {}
        for mod, data in frames.items():
            n_frames, height, width = data["shape"]
            ri = torch.randint(0, n_frames, (self.n, 1), dtype=torch.int32, generator=self.generator)
            fi = data["indexes"][ri]
            px = torch.randint(0, width, (self.n, 1), dtype=torch.int32, generator=self.generator)
            py = torch.randint(0, height, (self.n, 1), dtype=torch.int32, generator=self.generator)
            coords[mod] = torch.cat([fi, py, px], dim=-1)
            sel[mod] = ri.squeeze(-1)
        return coords, sel


# ------------------------------------------------------------------------------------------------
# flat-buffer fused AdamW
# ------------------------------------------------------------------------------------------------
class FlatGroup:
    """One optimizer param group with params and grads viewed into flat device buffers."""

    def __init__(self, params: List[nn.Parameter], lr: float, weight_decay: float, eps: float,
                 betas=(0.9, 0.999)):
        self.params = [p for p in params]
        n = sum(p.numel() for p in self.params)
        pad = (-n) % 4
        dev = self.params[0].device
        self.flat = torch.zeros(n + pad, device=dev)
        self.grad = torch.zeros(n + pad, device=dev)
        self.m = torch.zeros(n + pad, device=dev)
        self.v = torch.zeros(n + pad, device=dev)
        self.sumsq = torch.zeros(1, device=dev)
        # this step's AdamW scalars for graph replays (mms_adamw_dev; layout of mms_adamw_scalars)
        self.hyper = torch.zeros(8, device=dev)
        # two pinned staging buffers, alternated: a step's scalars can be queued behind the previous replay while
        # the copy queued before it may still be pending
        self._hyper_host = [torch.zeros(8).pin_memory() if dev.type == "cuda" else torch.zeros(8) for _ in range(2)]
        self._hyper_slot = 0
        off = 0
        for p in self.params:
            k = p.numel()
            self.flat[off:off + k].copy_(p.data.reshape(-1))
            p.data = self.flat[off:off + k].view_as(p)
            p.grad = self.grad[off:off + k].view_as(p)
            off += k
        self.n = n
        self.lr, self.wd, self.eps, self.betas = lr, weight_decay, eps, betas
        self.step_count = 0

    def zero_grad(self):
        self.grad.zero_()
        for p in self.params:   # re-attach in case autograd replaced a grad tensor
            pass

    def check_grads_attached(self):
        off = 0
        for p in self.params:
            k = p.numel()
            if p.grad is None or p.grad.data_ptr() != self.grad[off:off + k].data_ptr():
                g = p.grad
                view = self.grad[off:off + k].view_as(p)
                if g is not None:
                    view.copy_(g)
                p.grad = view
            off += k

    def _advance(self, lr_factor: float):
        """Advance the optimizer's step counter (torch AdamW's state['step'], 1 on the first update); this step's
        base-scheduled learning rate."""
        self.step_count += 1
        return self.lr * lr_factor

    def step(self, lr_factor: float, max_norm: float = 2.0):
        """clip_grad_norm_(max_norm) then torch AdamW math (single launch each; scalars stay on device)."""
        self.check_grads_attached()
        lr = self._advance(lr_factor)
        self.sumsq.zero_()
        _lib.call("mms_sumsq", self.grad.data_ptr(), self.n, self.sumsq.data_ptr(), _s())
        _lib.call("mms_adamw", self.flat.data_ptr(), self.grad.data_ptr(), self.m.data_ptr(), self.v.data_ptr(), self.n,
                  self.sumsq.data_ptr(), float(max_norm), float(lr), float(self.wd), float(self.betas[0]),
                  float(self.betas[1]), float(self.eps), int(self.step_count), _s())

    def load_hyper(self, lr_factor: float):
        """Graph mode, before a replay: advance the step and upload its scalars (read by the captured launch)."""
        lr = self._advance(lr_factor)
        host = self._hyper_host[self._hyper_slot]
        self._hyper_slot ^= 1
        _lib.call("mms_adamw_scalars", float(lr), float(self.wd), float(self.betas[0]), float(self.betas[1]),
                  float(self.eps), int(self.step_count), host.data_ptr())
        self.hyper.copy_(host, non_blocking=True)

    def step_captured(self, max_norm: float = 2.0):
        """The clip + AdamW launches with device-resident scalars (captured into the step graph)."""
        self.check_grads_attached()
        self.sumsq.zero_()
        _lib.call("mms_sumsq", self.grad.data_ptr(), self.n, self.sumsq.data_ptr(), _s())
        _lib.call("mms_adamw_dev", self.flat.data_ptr(), self.grad.data_ptr(), self.m.data_ptr(), self.v.data_ptr(),
                  self.n, self.sumsq.data_ptr(), float(max_norm), self.hyper.data_ptr(), _s())


ZERO_MULTI_MAX = 8      # buffers per mms_zero_multi launch (kMaxSeg, csrc/loss_optim.hip)


class OptimBank:
    """The trainer's optimizer groups (FlatGroup) stepped together in graph-replayed steps: the gradients and sum-of-
    squares accumulators zeroed in one launch, the groups' clip norms in one, their AdamW updates in one
    (mms_*_multi), and every group's per-step scalars in one device buffer filled by one upload.  The same
    arithmetic as each group's step_captured; the eager path keeps the per-group calls."""

    def __init__(self, groups: List[Optional[FlatGroup]]):
        self.groups = [g for g in groups if g is not None]
        G = len(self.groups)
        if not 1 <= G <= 4:
            raise ValueError("OptimBank holds 1 to 4 groups")
        dev = self.groups[0].flat.device
        self.hyper = torch.zeros(G * 8, device=dev)
        for i, g in enumerate(self.groups):
            g.hyper = self.hyper[8 * i:8 * i + 8]
        self._hyper_host = [torch.zeros(G * 8).pin_memory() if dev.type == "cuda" else torch.zeros(G * 8)
                            for _ in range(2)]
        self._hyper_slot = 0
        I64, VP, F32 = ctypes.c_int64 * G, ctypes.c_void_p * G, ctypes.c_float * G
        gs = self.groups
        self._sum = (G, VP(*[g.grad.data_ptr() for g in gs]), I64(*[g.n for g in gs]),
                     VP(*[g.sumsq.data_ptr() for g in gs]))
        self._args = [G, VP(*[g.flat.data_ptr() for g in gs]), VP(*[g.grad.data_ptr() for g in gs]),
                      VP(*[g.m.data_ptr() for g in gs]), VP(*[g.v.data_ptr() for g in gs]), I64(*[g.n for g in gs]),
                      VP(*[g.sumsq.data_ptr() for g in gs]), None, VP(*[g.hyper.data_ptr() for g in gs])]
        self._F32 = F32

    def zero_grads(self, extra: Sequence[torch.Tensor] = ()):
        """Every group's gradient buffer and sum-of-squares accumulator = 0, and the ``extra`` f32 buffers (the step's
        zero arena), in one launch."""
        for g in self.groups:
            g.check_grads_attached()
        bufs = [g.grad for g in self.groups] + [g.sumsq for g in self.groups] + list(extra)
        # one launch per ZERO_MULTI_MAX buffers (mms_zero_multi's segment table): one launch for the trainer's two
        # groups + hit counter + arena, more only for larger banks
        for i in range(0, len(bufs), ZERO_MULTI_MAX):
            part = bufs[i:i + ZERO_MULTI_MAX]
            n = len(part)
            _lib.call("mms_zero_multi", n, (ctypes.c_void_p * n)(*[b.data_ptr() for b in part]),
                      (ctypes.c_int64 * n)(*[b.numel() for b in part]), _s())

    def load_hyper(self, lr_factor: float):
        """Graph mode, before a replay: advance every group's step and upload their scalars in one copy."""
        host = self._hyper_host[self._hyper_slot]
        self._hyper_slot ^= 1
        for i, g in enumerate(self.groups):
            lr = g._advance(lr_factor)
            _lib.call("mms_adamw_scalars", float(lr), float(g.wd), float(g.betas[0]), float(g.betas[1]),
                      float(g.eps), int(g.step_count), host.data_ptr() + 32 * i)
        self.hyper.copy_(host, non_blocking=True)

    def step_captured(self, max_norm: float = 2.0):
        """clip_grad_norm_(max_norm) + AdamW of every group with device-resident scalars (two launches), the
        accumulators zeroed by zero_grads at the step's start."""
        for g in self.groups:
            g.check_grads_attached()
        _lib.call("mms_sumsq_multi", *self._sum, _s())
        args = list(self._args)
        args[7] = self._F32(*[float(max_norm)] * len(self.groups))
        _lib.call("mms_adamw_dev_multi", *args, _s())


def lr_factor(step: int, max_iters: int = 100000, warm_up_ratio=0.1, milestones=(0.5, 0.75, 0.9), gamma=0.4):
    """MultiStepWarmupScheduler.func (schedulers.py:259-266) as LambdaLR evaluates it."""
    warm = int(max_iters * warm_up_ratio)
    if step < warm:
        return step / warm
    idx = int(np.searchsorted(milestones, step / max_iters, side="left"))
    return gamma ** idx


def curvature_factor(step: int, max_iters: int = 100000, num_levels=16, min_res=16, max_res=1024):
    """CurvatureLossWarmUpScheduler (schedulers.py:320-343), warm_up_ratio 0.1."""
    warm = int(max_iters * 0.1)
    if step < warm:
        return step / warm
    spl = min(int(max_iters * 1.0), int(max_iters / num_levels))
    g = float(np.exp((np.log(max_res) - np.log(min_res)) / (num_levels - 1)))
    level = min(max(int(step / spl) + 1, 1), num_levels)
    return float(np.reciprocal(g ** (level - 1)))


# ------------------------------------------------------------------------------------------------
# losses
# ------------------------------------------------------------------------------------------------
# one autograd node for the whole loss of the batched model (MMS_FUSED_LOSS=0: per-term nodes + Python arithmetic)
FUSED_LOSS = os.environ.get("MMS_FUSED_LOSS", "1") != "0"


def compute_loss(outputs, targets: Dict[str, torch.Tensor], modalities: List[str], step: int,
                 sat_threshold: float = 0.9980, max_iters: int = 100000):
    """LossManager.compute_loss (losses.py:224-265) for the grid / grid_raw configs.  ``max_iters`` is the run's
    num_iterations: the curvature weight's warm-up / level schedule follows it (schedulers.py:320-343)."""
    geo = outputs[modalities[0]].get("_geo")
    analytic = outputs[modalities[0]]["hessians"] is None
    if FUSED_LOSS and geo is not None and tuple(geo["mods"]) == tuple(modalities) and \
            all(outputs[m].get("_geo") is geo for m in modalities):
        # the model's batched geometry: every term and the total in one autograd node (functions.StepLossFunction)
        n = len(modalities)
        sat = [sat_threshold if m == "polarization" else None for m in modalities]
        w_curv = 0.0 if analytic else 5e-4 * curvature_factor(step, max_iters)
        total, terms = fx.StepLossFunction.apply(n, sat, w_curv, geo["S"], geo["counts"], geo["seg_rays"],
                                                 geo["grads"], None if analytic else geo["hess"],
                                                 *[outputs[m][m] for m in modalities],
                                                 *[targets[m] for m in modalities])
        losses = {m: terms[i] for i, m in enumerate(modalities)}
        losses["eikonal_loss"] = terms[n]
        if not analytic:
            losses["curvature_loss"] = terms[n + 1]
        return losses, total
    losses = {}
    total = None
    for mod in modalities:
        thr = sat_threshold if mod == "polarization" else None
        l = fx.L1LossFunction.apply(outputs[mod][mod], targets[mod], thr)
        losses[mod] = l
        total = l if total is None else total + l
    # mlp methods: no hessian and no curvature loss (method_configs.py:350-352: geometry losses = eikonal only)
    analytic = outputs[modalities[0]]["hessians"] is None
    geo = outputs[modalities[0]].get("_geo")
    if geo is not None and tuple(geo["mods"]) == tuple(modalities) and \
            all(outputs[m].get("_geo") is geo for m in modalities):
        # the model's batched geometry (every modality's rows of one tensor): the concatenation the reference
        # builds (losses.py:235-248), read in place
        eik, curv = fx.GeoLossSegFunction.apply(geo["S"], geo["counts"], geo["seg_rays"], geo["grads"], geo["hess"])
        return _finish_loss(losses, total, eik, curv, analytic, step, max_iters)
    grads = [outputs[m]["gradients"].reshape(-1, 3) for m in modalities]
    hess = [torch.zeros_like(g) if analytic else outputs[m]["hessians"].reshape(-1, 3)
            for m, g in zip(modalities, grads)]
    counts = [outputs[m].get("count") for m in modalities]
    if any(c is not None for c in counts):
        # fixed-capacity batches (graph-captured steps): padding rows carry no geometric loss
        S = outputs[modalities[0]]["weights"].shape[1]
        eik, curv = fx.GeoLossMaskedFunction.apply(S, counts, *grads, *hess)
    else:
        eik, curv = fx.GeoLossFunction.apply(*grads, *hess)
    return _finish_loss(losses, total, eik, curv, analytic, step, max_iters)


def _finish_loss(losses, total, eik, curv, analytic: bool, step: int, max_iters: int):
    """Weighted eikonal (0.1) and curvature (5e-4 x warm-up / level factor) terms (method_configs.py:252-253)."""
    losses["eikonal_loss"] = eik
    total = total + 0.1 * eik
    if not analytic:
        cf = curvature_factor(step, max_iters)
        losses["curvature_loss"] = curv
        total = total + (5e-4 * cf) * curv
    return losses, total


def select_right_channel(rendered: torch.Tensor, band: torch.Tensor) -> torch.Tensor:
    """RawPipeline.select_right_channel_per_pixel (raw_pipeline.py:112-122): gather at the mosaick band."""
    return torch.gather(rendered, 1, band)


# ------------------------------------------------------------------------------------------------
# trainer
# ------------------------------------------------------------------------------------------------
CONFS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "confs")
# the BASELINE configurations' YAML per method (confs/: the reference files' keys read here, same schema)
METHOD_CONF = {"grid": "grid.yaml", "grid_raw": "grid_raw.yaml", "mlp_raw": "mlp_raw.yaml",
               "grid_raw_grid_bg_unbalanced": "grid_raw_rgb_all_views_pol_10_views.yaml"}


def read_conf(path: str) -> dict:
    """The training-step keys of an MMS-FW experiment YAML (the reference's confs/*.yaml schema, applied over the method
    registry by Config.update_config, /root/reference/src/configs/configs.py:214-242): method, max_num_iterations and
    pipeline.datamanager's modalities, eval views (eval_image_indices or eval_image_indices_per_modality), skipped
    training views (skip_image_indices_per_modality, datamanager.py) and pixel_sampler.num_rays_per_modality."""
    import yaml
    with open(path) as f:
        y = yaml.safe_load(f)
    dm = (y.get("pipeline") or {}).get("datamanager") or {}
    mods = list(dm.get("modalities") or [])
    ev = dm.get("eval_image_indices_per_modality")
    if ev is None and dm.get("eval_image_indices") is not None:
        ev = {m: list(dm["eval_image_indices"]) for m in mods}
    return {"method": y.get("method"), "max_num_iterations": y.get("max_num_iterations"), "modalities": mods,
            "eval_views": {m: list(v) for m, v in (ev or {}).items()},
            "skip_views": {m: list(v) for m, v in (dm.get("skip_image_indices_per_modality") or {}).items()},
            "num_rays_per_modality": (dm.get("pixel_sampler") or {}).get("num_rays_per_modality")}


def skip_views_for(method: str) -> Optional[Dict[str, List[int]]]:
    """skip_image_indices_per_modality of the method's BASELINE YAML (config 5 keeps 10 polarization training views:
    confs/grid_raw_rgb_all_views_pol_10_views.yaml:47-48 in the reference), None when it skips nothing."""
    name = METHOD_CONF.get(method)
    if name is None:
        return None
    return read_conf(os.path.join(CONFS, name))["skip_views"] or None


METHODS = {
    # method name: (raw mosaicked frames, background field kind, field kind)
    "grid": (False, "nerf", "grid"),
    "grid_raw": (True, "nerf", "grid"),
    "grid_raw_grid_bg_unbalanced": (True, "grid", "grid"),
    "mlp": (False, "nerf", "mlp"),
    "mlp_raw": (True, "nerf", "mlp"),
}


@dataclass
class TrainConfig:
    method: str = "grid"                 # a METHODS key
    modalities: tuple = ("rgb",)
    num_rays_per_modality: int = 2048
    log2T: int = 19
    width: int = 640
    height: int = 512
    n_views: int = 50
    max_iters: int = 100000
    pose_mode: str = "SO3xR3"
    seed: int = 654824
    skip_views: Optional[Dict[str, List[int]]] = None   # skip_image_indices_per_modality (datamanager config)
    data_dir: Optional[str] = None      # an on-disk MMS-DATA scene (data.MMSDataset) instead of the analytic one
    gpu_sampler: bool = False           # draw pixels on the device (data.GPUPixelSampler) instead of the host
    own_heads_only: bool = True         # training renders each modality's rays through its own head only


_SEEDS: Dict[tuple, torch.Tensor] = {}


def _seed(total: torch.Tensor) -> torch.Tensor:
    """d total / d total = 1 as a persistent tensor (made outside any capture, on the first eager step): a captured
    backward reads it instead of filling a fresh ones_like each replay."""
    key = (total.device, total.dtype, tuple(total.shape))
    one = _SEEDS.get(key)
    if one is None:
        if total.device.type == "cuda" and torch.cuda.is_current_stream_capturing():
            return torch.ones_like(total)
        one = _SEEDS[key] = torch.ones_like(total)
    return one


def backward_batched(total: torch.Tensor, between=None, mid=None, cuts=None) -> None:
    """total.backward() with the layers' weight-norm gradients applied in one batched launch at its end.

    ``between`` (data-parallel graph steps): the MLPs' weight-gradient GEMMs are deferred, ``between()`` runs once the
    backward has queued everything else -- the hash-table gradients are final there -- and the deferred launches and
    the weight-norm flush follow it (graphs.GraphTrainer ends one captured graph and begins the next there).
    ``cuts`` (the forward ran under functions.PHASE_CUT): the backward runs in two caller-thread phases, the rendering
    side first, then ``mid()`` -- the radiance table gradient is final there --, then the SDF side from the cut
    tensors (functions.phase_two)."""
    fx.wn_bwd_begin()
    try:
        def run():
            total.backward(_seed(total))
            if cuts is not None:
                if mid is not None:
                    mid()
                fx.phase_two(cuts)
        if between is not None:
            fx.wgrad_defer_begin()
            try:
                run()
            finally:
                between()
            fx.wgrad_flush()
        else:
            run()
    finally:
        fx._WGRAD_DEFER[0] = None
        fx._WGRAD_DEFER_STREAM[0] = None
        fx.wn_bwd_flush()


class Trainer:
    """Synthetic-scene trainer: frames resident in HBM, host pixel sampler, full train step on the HIP path."""

    def __init__(self, cfg: TrainConfig, device, rank: int = 0, frames_on_device: bool = True):
        self.cfg = cfg
        self.device = device
        self.raw, bg_kind, fields = METHODS[cfg.method]
        mods = list(cfg.modalities)
        self.modalities = mods
        channels = {m: mscene.CHANNELS[m] for m in mods}
        torch.manual_seed(654824)
        self.model = BaseModel(ModelSpec(channels, log2T=cfg.log2T, bg_kind=bg_kind, fields=fields)).to(device)
        self.model.draw_seed = (cfg.seed << 8) + 1000003 * rank + 17   # per-rank stream of the forward's draws
        # training renders each modality's rays through its own head only (the loss reads nothing else; gradients are
        # identical); evaluation (no grad) renders every head as the reference does
        self.model.own_heads_only = cfg.own_heads_only
        self.dataset = None
        if cfg.data_dir is not None:
            # the train split of an on-disk scene: every frame but the eval views and the skipped ones
            from .data import MMSDataset
            excl = {m: list(mscene.EVAL_VIEWS) + list((cfg.skip_views or {}).get(m, [])) for m in mods}
            self.dataset = MMSDataset(cfg.data_dir, mods, indexes_to_exclude=excl)
            if self.dataset.raw != self.raw:
                raise ValueError(f"method {cfg.method} needs {'raw' if self.raw else 'demosaicked'} frames")
            cams = dict(self.dataset.cameras)
        else:
            cams = mscene.make_cameras(mods, cfg.n_views, cfg.width, cfg.height, seed=0, train=True)
            for m, skip in (cfg.skip_views or {}).items():
                if m in cams:
                    cams[m] = mscene.select_views(cams[m], [v for v in cams[m].view_ids if v not in set(skip)])
        self.cams = {m: DeviceCameras(cams[m], device) for m in mods}
        self.pose = CameraOptimizer(mods, {m: self.cams[m].num for m in mods}, mode=cfg.pose_mode).to(device)
        self.raygen = RayGenerator(self.cams, self.pose, 0.0)
        self.sampler = UniformPixelSampler(cfg.num_rays_per_modality, cfg.seed + rank)
        # frames cached in HBM (the reference caches all training frames in RAM, dataloaders.py:135-162)
        if self.dataset is not None:
            self.images = {m: self.dataset.images[m].to(device) for m in mods}
        else:
            self.images = {m: mscene.render_frames(cams[m], channels[m], device, m if self.raw else None) for m in mods}
        self.host_cams = cams
        self.frames = {m: {"shape": tuple(self.images[m].shape[:3]),
                           "indexes": torch.arange(cams[m].c2w.shape[0], dtype=torch.int32)} for m in mods}
        if self.dataset is not None:
            self.masks = {m: k.to(device) for m, k in self.dataset.mosaick_masks.items()} if self.raw else {}
        else:
            self.masks = {m: mscene.mosaick_mask(m, cfg.width, cfg.height).to(device) for m in mods} if self.raw else {}
        self.gpu_sampler = None
        if cfg.gpu_sampler:
            from .data import GPUPixelSampler
            self.gpu_sampler = GPUPixelSampler(self.images, cfg.num_rays_per_modality, cfg.seed, rank)
        self.fields = FlatGroup(list(self.model.parameters()), lr=1e-3, weight_decay=0.01, eps=1e-15)
        pose_params = list(self.pose.parameters())
        self.poses = FlatGroup(pose_params, lr=1e-4, weight_decay=0.01, eps=1e-15) if pose_params else None
        self.optim = OptimBank([self.fields, self.poses]) if self.fields.flat.device.type == "cuda" else None
        self.step = 0

    def targets_for(self, coords: Dict[str, torch.Tensor], sel: Dict[str, torch.Tensor]):
        """Pixel values at the sampled pixels (pixel_samplers.py:86: images[frame, y, x])."""
        out = {}
        for m, c in coords.items():
            img = self.images[m]
            ri = sel[m].to(img.device).long()
            cd = c.to(img.device).long()
            out[m] = img[ri, cd[:, 1], cd[:, 2]]
        return out

    def set_step(self, step: int):
        """Position the schedules (LR, callbacks) at ``step``.  The optimizers keep their own update counts: a
        trainer positioned at step 95000 with fresh moments is a fresh torch AdamW (state['step'] starts at 0)
        under a LambdaLR at 95000."""
        self.step = step
        self.model.set_step(step, self.cfg.max_iters)

    def train_step(self, coords=None, targets=None, rng: Optional[RNG] = None, ddp=None):
        """One training iteration (raw_pipeline.py:67-82); the BEFORE_TRAIN_ITERATION callbacks (coarse-to-fine
        mask, tap delta, cos anneal: feature_structures.py:97-108, surface_model.py:254-271,
        volume_rendering.py:227-230) are applied for the current step first, as the reference's trainer does."""
        losses, total, outputs = self.compute_grads(coords, targets, rng, ddp)
        f = lr_factor(self.step, self.cfg.max_iters)
        self.fields.step(f)
        if self.poses is not None:
            self.poses.step(f)
        self.step += 1
        return losses, total, outputs

    def compute_grads(self, coords=None, targets=None, rng: Optional[RNG] = None, ddp=None):
        """Forward, losses, backward and (data parallel) the averaged gradient exchange: the train step up to the
        optimizer (fabric.backward, raw_pipeline.py:67-77)."""
        self.model.set_step(self.step, self.cfg.max_iters)
        if coords is None and self.gpu_sampler is not None:
            coords, _, targets = self.gpu_sampler.sample()
        elif coords is None:
            coords, sel = self.sampler.sample(self.frames)
            targets = self.targets_for(coords, sel)
        dev = self.device
        coords_d = {m: c.to(dev, non_blocking=True) for m, c in coords.items()}
        targets_d = {m: t.to(dev, non_blocking=True) for m, t in targets.items()}
        fx.zero_arena_begin(dev)
        try:
            return self._compute_grads(coords_d, targets_d, rng, ddp)
        finally:
            fx.zero_arena_end()

    def _compute_grads(self, coords_d, targets_d, rng, ddp):
        dev = self.device
        rays = self.raygen(coords_d)
        fx.reset_grad_uses()
        outputs = self.model(rays, rng)
        if self.raw:
            for m in self.modalities:
                band = self.masks[m][coords_d[m][:, 1].long(), coords_d[m][:, 2].long()].long()[:, None]
                outputs[m][m] = select_right_channel(outputs[m][m], band)
        losses, total = compute_loss(outputs, targets_d, self.modalities, self.step, max_iters=self.cfg.max_iters)
        self.fields.zero_grad()
        if self.poses is not None:
            self.poses.zero_grad()
        groups = [self.fields] + ([self.poses] if self.poses is not None else [])
        if ddp is not None and ddp.world > 1:
            # hash-table gradients are all-reduced as soon as their backward kernels are queued (overlapping the rest
            # of the backward), everything else after it
            ddp.begin_step()
            hook = lambda g: ddp.grad_ready(g, groups)  # noqa: E731
            fx.GRAD_READY_HOOKS.append(hook)
            try:
                backward_batched(total)
            finally:
                fx.GRAD_READY_HOOKS.remove(hook)
            ddp.finish_step(groups)
        else:
            backward_batched(total)
        return losses, total, outputs
