"""Fused autograd stages of the hot path, each a small chain of libmms_hip.so kernels.

Every Function restates one stage of the reference's per-ray computation with an explicit backward
(paths under /root/reference/src):

  SurfaceFunction     SDFField + 4-tap numerical gradient (surface_model.py:66-153; surface_field.py:99-116)
  RadianceFunction    RadianceModel input assembly + RadianceField (radiance_model.py:94-141; radiance_field.py:72-77)
  BackgroundFunction  BackgroundModel NeRF field (background_model.py:73-99; nerf_field.py:92-105)
  NeusWeightsFunction NeuSVolumeRendering (volume_rendering.py:171-213)
  DensityWeightsFunction RaySamples.get_alphas + get_weights_from_alphas (rays.py:138-217)
  CompositeFunction   RadianceRenderer / background sum (renderers.py:152-174; background_model.py:101-109)
  SamplesFunction     spacing bins -> euclidean samples (ray_samplers.py:178-181; rays.py:69-81, 304-349)
  RaysFunction        Cameras.generate_rays with pose refinement (cameras.py:460-703)
  ColliderFunction    SphereCollider + background near/far (scene_colliders.py:60-113)
  PolarizerFunction   PolarizationHead Stokes alignment (field_heads.py:90-106; polarizer.py:54-101)
  L1LossFunction / GeoLossFunction   losses.py:68-164

There is no CPU path: every function requires HIP device tensors.
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import List, Optional, Sequence, Tuple

import torch

from . import _lib
from .hip_ops import (NN, NT, TN, _splits_for, act_bwd, gemm, gemm_tn_grouped, gemm_tn_wide16, weight_norm_bwd,
                      weight_norm_fwd)

ACT = {None: 0, "None": 0, "ReLU": 1, "Softplus": 2, "Sigmoid": 3}

# GEMM operand precision per MLP family: 0 exact fp32 MFMA (parity mode), 1 bf16, 2 split bf16x3.
PRESETS = {
    "fp32": {"sdf": 0, "radiance": 0, "heads": 0, "pol_head": 0, "background": 0, "mlp": 0},
    # throughput mode: every MLP of the grid methods on split-bf16x3 MFMA (x = hi + lo on both operands, ~17
    # significant bits, fp32 accumulation), the analytic-gradient MLP fields (mlp methods, differentiated twice) on
    # the exact fp32 MFMA.  The SDF needs the extra mantissa for its 4-tap finite differences (sdf differences over
    # 4 delta ~ 4.5e-3, hessians over delta^2 ~ 1.3e-6); the radiance, head and background MLPs need it for converged
    # quality: with their operands in plain bf16 the held-out PSNR of grid_raw5 after 3000 steps from scratch was
    # 0.56 dB below fp32 (paired over 3 seeds), 0.27 dB with bf16 only in their backward (mode 4), and -0.12 +- 0.16 dB
    # with split-bf16x3 throughout (profiles/round3_converged_psnr.json)
    "fast": {"sdf": 2, "radiance": 2, "heads": 2, "pol_head": 2, "background": 2, "mlp": 0},
    # NOT parity presets, kept to price the precision: "fast_bf16" = round 2's fast (bf16 radiance / heads /
    # background), "fast_m4" = their forward split-bf16x3 and backward bf16 (PRECISION value 4)
    "fast_bf16": {"sdf": 2, "radiance": 1, "heads": 1, "pol_head": 2, "background": 1, "mlp": 0},
    "fast_m4": {"sdf": 2, "radiance": 4, "heads": 4, "pol_head": 2, "background": 4, "mlp": 0},
    "bf16x3": {"sdf": 2, "radiance": 2, "heads": 2, "pol_head": 2, "background": 2, "mlp": 2},
}
# weight gradients dW += dZ^T X of every chain-run MLP on bf16 operands (fp32 accumulation over the ~280k rows), the
# forward and backward-data chains unchanged: the reference GPU's fp16 autocast runs these GEMMs on 16-bit operands too
# (trainer.py:51); the data gradients that propagate to the SDF geometry, the hash tables and the poses keep split-bf16x3
PRESETS["fast_w16"] = dict(PRESETS["fast"], wgrad=1)
# the reference GPU's own forward precision for the radiance, head and background MLPs: their forward chains on fp16
# operands (one fp16 MFMA per product, fp32 accumulation -- autocast "16-mixed", trainer.py:51), their backward-data
# chains and weight gradients split-bf16x3 (wider than the reference's fp16 backward: no loss scaling needed); the SDF
# chain stays split-bf16x3 throughout (its 4-tap hessians)
PRESETS["fast_h16"] = dict(PRESETS["fast"], radiance=5, heads=5, pol_head=5, background=5)
# ... and the reference's fp16 backward-data chains too (mms_mlp_chain prec 6): every chain's backward on fp16 operands
# after its first layer (that one's input, dY from memory, stays split-bf16x3), each row scaled by a power of two to
# its largest |dZ| (no global loss scale, no underflow), fp32 accumulation and fp32 dZ stores; the weight gradients
# and every forward unchanged
PRESETS["fast_h16b"] = dict(PRESETS["fast_h16"], bwd16=1)
# NOT the benchmarked preset (its weight gradients have bf16's 8 significant bits, the reference's autocast keeps 11):
# fast_h16b with bf16 weight gradients, priced in converged PSNR (+0.007 +- 0.085 dB vs fp32, 9 seeds) and rays/s
PRESETS["fast_h16bw"] = dict(PRESETS["fast_h16b"], wgrad=1)
# ... and the reference's fp16 weight gradients too: the prec-6 backward chains store each hidden layer's dZ as the
# fp16 row-scaled values their next layer already multiplies (half the bytes of the fp32 panels), and the weight
# gradients of those layers run one fp16 MFMA per product on them and on X rounded to fp16 in a common per-launch scale
# (mms_gemm_tn_wide16: the autocast nn.Linear backward's operand precision, fp32 accumulation); the layers whose dZ is
# the chain's input (the SDF / background output layers, the radiance field's last layer) stay split-bf16x3
PRESETS["fast_h16c"] = dict(PRESETS["fast_h16b"], wgrad16=1)
# ... and the reference's fp16 activations: those chains' hidden-layer outputs stored as fp16 rows (the backward's act'
# source and the weight gradients' X: half the bytes written by the forward, read by the backward and the weight
# gradients); the forward itself still feeds each layer from its fp32 accumulators
PRESETS["fast_h16d"] = dict(PRESETS["fast_h16c"], y16=1)
for _p in PRESETS.values():
    _p.setdefault("sdf_chain", 0)      # 0: the chain runs on the "sdf" GEMM precision
    _p.setdefault("wgrad", 0)          # 0: the weight gradients on the family's backward operand mode
    _p.setdefault("bwd16", 0)          # 1: split-bf16x3 backward-data chains run prec 6
    _p.setdefault("wgrad16", 0)        # 1: prec-6 chains' hidden-layer weight gradients on fp16 dZ (gemm_tn_wide16)
    _p.setdefault("y16", 0)            # 1 (with wgrad16): those chains' hidden activations stored as fp16 rows
# NOT a parity preset: the SDF chain on bf16 weights x split activations (mms_mlp_chain prec 3, two MFMAs per product;
# with bf16-ROUNDED weights the SDF is a different, rippled function: 56x the reference's hessian scale off on the
# e2e fixtures and a 24x larger curvature loss over the rgb training trajectory), kept to measure what the curvature
# parity costs
PRESETS["fast_x2"] = dict(PRESETS["fast_bf16"], sdf_chain=3)
PRECISION = dict(PRESETS["fp32"])


def fwd_prec(p: int) -> int:
    """GEMM / chain operand mode of a family's forward: PRECISION value 4 = split-bf16x3 forward, bf16 backward; 5 =
    fp16 forward (the fused chain), split-bf16x3 backward."""
    return 2 if p == 4 else p


def bwd_prec(p: int) -> int:
    """... and of its backward (data and weight gradients)."""
    return 1 if p == 4 else (2 if p == 5 else p)


def set_precision(mode: str) -> None:
    """Select the MLP GEMM precision preset ('fp32' parity | 'fast' | 'bf16x3' | 'fast_bf16' | 'fast_m4' | 'fast_x2')."""
    PRECISION.update(PRESETS[mode])


def _alloc(rows: int, cols: int, dev, zero: bool = False) -> torch.Tensor:
    """[rows, cols] view of a [rows, cols rounded up to 4] buffer: 16-byte aligned rows keep the GEMM and
    panel kernels on their float4 paths for odd widths (71, 257, 317, ...)."""
    ld = (cols + 3) // 4 * 4
    buf = torch.zeros(rows, ld, device=dev) if zero else torch.empty(rows, ld, device=dev)
    return buf[:, :cols]


# Weight-normalised weights (and their packed MFMA images) computed once per model forward, all layers in one launch:
# the SDF MLP alone is evaluated 5 times per modality and step (4 sampler iterations + the training pass) and every
# modality reuses the same fields.  BaseModel.forward opens a scope (begin_forward) at its start; a captured graph
# holds the two batched launches, so replays recompute every entry from the current parameters.
class _NormItem(ctypes.Structure):
    """MmsNormItem (include/mms_hip.h)."""
    _fields_ = [("g", ctypes.c_void_p), ("v", ctypes.c_void_p), ("N", ctypes.c_int64), ("K", ctypes.c_int64),
                ("W", ctypes.c_void_p), ("ldw", ctypes.c_int64), ("norms", ctypes.c_void_p), ("row0", ctypes.c_int64)]


class _PackItem(ctypes.Structure):
    """MmsPackItem (include/mms_hip.h)."""
    _fields_ = [("W", ctypes.c_void_p), ("N", ctypes.c_int64), ("K", ctypes.c_int64), ("ldw", ctypes.c_int64),
                ("transpose", ctypes.c_int64), ("permute", ctypes.c_int64), ("rows", ctypes.c_int64),
                ("cols", ctypes.c_int64), ("hi", ctypes.c_void_p), ("lo", ctypes.c_void_p), ("elem0", ctypes.c_int64)]


class WeightPrep:
    """A model's weight preparation, batched: every weight-normed layer's W = g v / ||v|| (mlp.py:206-209) and every
    bf16 MMA image the chain kernels read (forward and backward orientation) are recomputed at the start of each
    model forward by two launches (mms_weight_norm_fwd_batched, mms_mlp_pack_batched) instead of one per layer and
    image.  Entries register themselves on first use (computed individually that once) into persistent buffers; the
    item tables live in device memory, append-only with a fixed capacity, so a captured graph's launches keep reading
    a valid table.  Outside a model forward nothing is cached (parameters are read afresh)."""

    MAX_NORM, MAX_PACK = 64, 128

    def __init__(self):
        self.norm = {}      # key -> [g, v, W, nrm, index]
        self.pack = {}      # key -> [W, hi, lo, index, args]
        self.norm_items: List[_NormItem] = []
        self.pack_items: List[_PackItem] = []
        self.rows = 0
        self.elems = 0
        self.dirty = False
        self.fresh = False
        self.table_n = None
        self.table_p = None
        self.n_up = (0, 0, 0, 0)   # (norm items, rows, pack items, elems) in the device tables
        self.done = set()          # entries computed individually in the current forward
        self.dev = None

    def _stale(self) -> bool:
        """True when a registered parameter's storage moved since it was registered (e.g. FlatGroup re-pointing
        p.data into its flat buffer after a first forward): the device tables would read freed memory."""
        for g, v, W, nrm, idx in self.norm.values():
            if idx is not None and (self.norm_items[idx].g != g.data_ptr() or self.norm_items[idx].v != v.data_ptr()):
                return True
        return False

    def reset(self) -> None:
        """Forget every entry (they re-register on their next use)."""
        self.__init__()

    def run(self, dev) -> None:
        """Recompute every registered entry (start of a model forward)."""
        if self.norm_items and self._stale():
            if torch.cuda.is_current_stream_capturing():
                # a captured graph would keep reading the device tables' freed g / v storage on every replay;
                # GraphTrainer always runs an eager step (which resets here) before it captures
                raise RuntimeError("WeightPrep: parameters moved since registration and a stream capture is active; "
                                   "run one eager forward before capturing")
            self.reset()
        self.fresh = False
        self.done.clear()
        self.dev = dev
        if not self.norm_items:
            return
        if self.dirty:
            if torch.cuda.is_current_stream_capturing():
                return                      # no table upload inside a capture: lookups compute individually
            self._upload(dev)
        nn_, rows, np_, elems = self.n_up
        _lib.call("mms_weight_norm_fwd_batched", self.table_n.data_ptr(), nn_, rows, _s())
        if np_:
            _lib.call("mms_mlp_pack_batched", self.table_p.data_ptr(), np_, elems, _s())
        self.fresh = True

    def close(self) -> None:
        """End of a model forward: entries registered in it go into the device tables now (outside any capture), so
        the next forward -- possibly a captured one -- prepares them in the batch."""
        self.fresh = False
        if self.dirty and self.dev is not None and not torch.cuda.is_current_stream_capturing():
            self._upload(self.dev)

    def _upload(self, dev) -> None:
        if self.table_n is None:
            self.table_n = torch.zeros(self.MAX_NORM * ctypes.sizeof(_NormItem), dtype=torch.uint8, device=dev)
            self.table_p = torch.zeros(self.MAX_PACK * ctypes.sizeof(_PackItem), dtype=torch.uint8, device=dev)
        for items, table, T in ((self.norm_items, self.table_n, _NormItem), (self.pack_items, self.table_p, _PackItem)):
            if items:
                arr = (T * len(items))(*items)
                table[:ctypes.sizeof(arr)].copy_(torch.frombuffer(bytearray(arr), dtype=torch.uint8))
        self.n_up = (len(self.norm_items), self.rows, len(self.pack_items), self.elems)
        self.dirty = False

    def normed(self, g: torch.Tensor, v: torch.Tensor):
        key = (v.data_ptr(), g.data_ptr(), tuple(v.shape))
        e = self.norm.get(key)
        if e is None:
            N, K = v.shape
            W, nrm = _alloc(N, K, v.device), torch.empty(N, device=v.device)
            idx = None
            if len(self.norm_items) < self.MAX_NORM:
                idx = len(self.norm_items)
                self.norm_items.append(_NormItem(g.data_ptr(), v.data_ptr(), N, K, W.data_ptr(),
                                                 W.stride(0), nrm.data_ptr(), self.rows))
                self.rows += N
                self.dirty = True
            e = self.norm[key] = [g, v, W, nrm, idx]
        g, v, W, nrm, idx = e
        if not (self.fresh and idx is not None and idx < self.n_up[0]) and key not in self.done:
            weight_norm_fwd(g.reshape(-1), v, W, nrm)
            self.done.add(key)
        return W, nrm

    def packed(self, W: torch.Tensor, rows: int, cols: int, transpose: bool, permute: bool, prec: int):
        key = (W.data_ptr(), tuple(W.shape), rows, cols, bool(transpose), int(permute), int(prec))
        e = self.pack.get(key)
        N, K = W.shape
        if e is None:
            hi = torch.empty(rows, cols, dtype=torch.bfloat16, device=W.device)
            lo = torch.empty_like(hi) if prec == 2 else None
            idx = None
            if len(self.pack_items) < self.MAX_PACK:
                idx = len(self.pack_items)
                self.pack_items.append(_PackItem(W.data_ptr(), N, K, W.stride(0), int(transpose), int(permute), rows,
                                                 cols, hi.data_ptr(), _p(lo), self.elems))
                self.elems += rows * cols
                self.dirty = True
            e = self.pack[key] = [W, hi, lo, idx]
        W, hi, lo, idx = e
        if not (self.fresh and idx is not None and idx < self.n_up[2]) and key not in self.done:
            _lib.call("mms_mlp_pack", W.data_ptr(), N, K, W.stride(0), int(transpose), int(permute), rows, cols,
                      hi.data_ptr(), _p(lo), _s())
            self.done.add(key)
        return hi, lo


_ACTIVE_PREP: List[Optional[WeightPrep]] = [None]


def begin_forward(prep: Optional[WeightPrep] = None, dev=None) -> None:
    """Open a model-forward scope: the model's weights are prepared in one batch and looked up from it."""
    _ACTIVE_PREP[0] = prep
    if prep is not None:
        prep.run(dev)


def end_forward() -> None:
    """Close the scope: outside a model forward (plugin modules, backward passes) nothing is cached, so parameters
    updated in place are always read afresh."""
    if _ACTIVE_PREP[0] is not None:
        _ACTIVE_PREP[0].close()
    _ACTIVE_PREP[0] = None


def normed_weight(g: torch.Tensor, v: torch.Tensor):
    """(W = g v / ||v||_row in a 16-B aligned [N, K] view, row norms) of one weight-normed layer (mlp.py:206-209)."""
    prep = _ACTIVE_PREP[0]
    if prep is not None:
        return prep.normed(g, v)
    N, K = v.shape
    W = _alloc(N, K, v.device)
    nrm = torch.empty(N, device=v.device)
    weight_norm_fwd(g.reshape(-1), v, W, nrm)
    return W, nrm


def grad_target(p: torch.Tensor) -> Optional[torch.Tensor]:
    """The buffer a parameter's gradient is accumulated into directly by the backward kernels.

    Parameter gradients are written in place into ``p.grad`` (for the trainer: views into the flat
    gradient buffer of pipeline.FlatGroup) and the autograd Functions return ``None`` for them: no
    per-parameter zero-fill, temporary and AccumulateGrad add per step (AccumulateGrad's semantics --
    sum into .grad -- are kept: every kernel here accumulates)."""
    if not p.requires_grad:
        return None
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    return p.grad


def _s() -> int:
    return torch.cuda.current_stream().cuda_stream


# Called with a parameter's gradient buffer as soon as the backward kernels have finished writing it (queued on the
# current stream): the data-parallel trainer starts that gradient's all-reduce there (ddp.DDP.grad_ready).
GRAD_READY_HOOKS: List = []
_PENDING_USES = {}   # parameter data_ptr -> backward contributions still to come this step


def reset_grad_uses() -> None:
    _PENDING_USES.clear()


def _grad_use(p: torch.Tensor) -> None:
    """A differentiable forward use of parameter ``p`` (its backward will add one gradient contribution)."""
    _PENDING_USES[p.data_ptr()] = _PENDING_USES.get(p.data_ptr(), 0) + 1


def _grad_ready(p: torch.Tensor, g: Optional[torch.Tensor]) -> None:
    """One backward contribution to ``p``'s gradient ``g`` is queued; the last one of the step fires the hooks (a
    table used by several modalities' fields is final only after every modality's backward)."""
    if g is None:
        return
    k = p.data_ptr()
    left = _PENDING_USES.get(k, 1) - 1
    _PENDING_USES[k] = left
    if left <= 0:
        _PENDING_USES.pop(k, None)
        for h in GRAD_READY_HOOKS:
            h(g)


def _p(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _f32arr(vals):
    return ctypes.cast((ctypes.c_float * len(vals))(*[float(v) for v in vals]), ctypes.c_void_p)


class GridCfg:
    """Static description of one FeatureGrid(HashEncoding) (encodings.py:48-67, feature_structures.py:28-45)."""

    def __init__(self, scales: Sequence[float], log2T: int, radius: float, features: int = 2, interp: int = 0):
        self.scales = [float(s) for s in scales]
        self.L = len(self.scales)
        self.log2T = int(log2T)
        self.radius = float(radius)
        self.F = int(features)
        self.interp = int(interp)     # 0 "Linear" (the parity mode), 1 "Smoothstep" (tcnn's default, unpinned)
        self._arr = (ctypes.c_float * self.L)(*self.scales)

    @property
    def scales_ptr(self):
        return ctypes.cast(self._arr, ctypes.c_void_p)

    @property
    def out_dim(self):
        return self.L * self.F


def grid_fwd(g: GridCfg, pos: torch.Tensor, ldx: int, M: int, table, active: int, out: torch.Tensor, col: int,
             group: int = 1):
    """Hash-grid features of M rows into out[:, col:col + 2L]; group=5 for the [centre | 4 taps] SDF batch (gathered
    in (sample, tap) order, same values)."""
    Mg = M // group
    _lib.call("mms_hashgrid_fwd_grouped", pos.data_ptr(), Mg, group, Mg, ldx, table.data_ptr(), g.L, g.log2T, g.F,
              g.interp, g.scales_ptr, g.radius, active, out.data_ptr() + 4 * col, out.stride(0), _s())


# the SDF / radiance input panels in one launch each (mms_sdf_panel_fwd, mms_rad_panel_fwd); MMS_FUSED_PANEL=0: the
# input-column kernel + the hash-grid gather as two launches
FUSED_PANEL = os.environ.get("MMS_FUSED_PANEL", "1") != "0"
FUSED_RAD_PANEL = FUSED_PANEL and os.environ.get("MMS_FUSED_RAD", "1") != "0"


def sdf_panel(pos: torch.Tensor, ldp: int, M: int, ntaps: int, delta: float, g: GridCfg, table, active: int,
              X: torch.Tensor) -> None:
    """Rows [x(3), PE(36), grid(32)] of the SDF MLP input for M positions (+ ntaps = 4 tap blocks of M rows)."""
    if FUSED_PANEL:
        _lib.call("mms_sdf_panel_fwd", pos.data_ptr(), ldp, M, ntaps, delta, 6, table.data_ptr(), g.L, g.log2T, g.F,
                  g.interp, g.scales_ptr, g.radius, active, X.data_ptr(), X.stride(0), _s())
        return
    _lib.call("mms_geo_input_fwd", pos.data_ptr(), ldp, M, ntaps, delta, 6, X.data_ptr(), X.stride(0), _s())
    grid_fwd(g, X, X.stride(0), (1 + ntaps) * M, table, active, X, 39, group=1 + ntaps)


# hash-grid backward with both gradients: the table walk computes both (scripts/hash_bench.py: the walk without
# position gradients + the gather-style mms_hashgrid_dpos_grouped cost the same as the walk computing both).
# HASH_SPLIT = True (tests only) routes the position gradient through the gather kernel.
HASH_SPLIT = False


def grid_bwd(g: GridCfg, pos, ldx, M, table, active, dout: torch.Tensor, col: int, dtable, dpos, group: int = 1):
    """Table / position gradients; group=5 for the [centre | 4 taps] SDF batch (M = 5 x centres)."""
    Mg = M // group
    split = HASH_SPLIT and dtable is not None and dpos is not None
    wpos = None if split else dpos
    _lib.call("mms_hashgrid_bwd_grouped", pos.data_ptr(), Mg, group, Mg, ldx, table.data_ptr(), g.L, g.log2T, g.F,
              g.interp, g.scales_ptr, g.radius, active, dout.data_ptr() + 4 * col, dout.stride(0), _p(dtable), _p(wpos),
              0 if wpos is None else wpos.stride(0), _s())
    if split:
        _lib.call("mms_hashgrid_dpos_grouped", pos.data_ptr(), Mg, group, Mg, ldx, table.data_ptr(), g.L, g.log2T,
                  g.F, g.interp, g.scales_ptr, g.radius, active, dout.data_ptr() + 4 * col, dout.stride(0),
                  dpos.data_ptr(), dpos.stride(0), _s())


# ------------------------------------------------------------------------------------------------
# MLP core (shared by the fused field functions)
# ------------------------------------------------------------------------------------------------
class MLPRun:
    """Forward activations of a weight-normed MLP kept for the explicit backward."""

    def __init__(self, params: Sequence[torch.Tensor], acts: Sequence[Tuple[int, float, float]], prec: int = 0):
        self.prec = int(prec)
        self.fprec, self.bprec = fwd_prec(self.prec), bwd_prec(self.prec)   # forward / backward GEMM modes
        self.params = list(params)
        self.acts = list(acts)
        self.L = len(self.params) // 3
        self.Ws: List[torch.Tensor] = []
        self.norms: List[torch.Tensor] = []
        self.Zs: List[Optional[torch.Tensor]] = []
        self.Ys: List[torch.Tensor] = []
        self.x = None

    def forward(self, x: torch.Tensor, keep: bool, last_out: Optional[torch.Tensor] = None) -> torch.Tensor:
        M = x.shape[0]
        self.x = x
        h = x
        dev = x.device
        for l in range(self.L):
            g, v, b = self.params[3 * l: 3 * l + 3]
            N, K = v.shape
            W, nrm = normed_weight(g, v)
            act, beta, thr = self.acts[l]
            if l == self.L - 1 and last_out is not None:
                Y = last_out
            elif l == self.L - 1:
                Y = torch.empty(M, N, device=dev)   # leaves the MLP: consumers expect a contiguous tensor
            else:
                Y = _alloc(M, N, dev)
            # the backward takes ReLU' / Sigmoid' from the output: only Softplus keeps its pre-activation
            Z = _alloc(M, N, dev) if (keep and act == 2) else None
            gemm(NT, M, N, K, h, h.stride(0), W, W.stride(0), Y, Y.stride(0), bias=b, Z=Z,
                 ldz=0 if Z is None else Z.stride(0), act=act, beta=beta, thr=thr, prec=self.fprec)
            if keep:
                self.Ws.append(W)
                self.norms.append(nrm)
                self.Zs.append(Z)
                self.Ys.append(Y)
            h = Y
        return h

    def _grad_src(self, l: int):
        """(tensor, derivative id) layer l's activation derivative is taken from: the stored pre-activation for
        Softplus, else the layer output (ReLU: the same test; Sigmoid: id 4, y (1 - y))."""
        act = self.acts[l][0]
        if act == 2 or self.Zs[l] is not None:
            return self.Zs[l], act
        return self.Ys[l], (4 if act == 3 else act)

    def backward(self, dy: torch.Tensor, need_dx: bool, pre_activated: bool = False,
                 dx_out: Optional[torch.Tensor] = None) -> Tuple[Optional[torch.Tensor], List[torch.Tensor]]:
        """dy = gradient of the last layer's output, or (pre_activated) already of its pre-activation; dx is written
        into ``dx_out`` (a [M, K] view with unit column stride) when given."""
        x = self.x
        M = x.shape[0]
        dev = x.device
        grads: List[Optional[torch.Tensor]] = [None] * len(self.params)   # accumulated in place (grad_target)
        act, beta, thr = self.acts[self.L - 1]
        if act != 0 and not pre_activated:
            dZ = _alloc(M, dy.shape[1], dev)
            aux, did = self._grad_src(self.L - 1)
            act_bwd(dy, aux, did, beta, thr, dZ)
        else:
            dZ = dy
        dx = None
        dWs = _dw_views([self.params[3 * l + 1] for l in range(self.L)], dev)
        for l in range(self.L - 1, -1, -1):
            g, v, b = self.params[3 * l: 3 * l + 3]
            N, K = v.shape
            Xin = x if l == 0 else self.Ys[l - 1]
            gt, vt, bt = grad_target(g), grad_target(v), grad_target(b)
            if gt is not None or vt is not None or bt is not None:
                dW = dWs[l]
                db = bt if bt is not None else torch.zeros(N, device=dev)
                tiles = ((N + 127) // 128) * ((K + 127) // 128)
                _wgrad(lambda N=N, K=K, dZ=dZ, Xin=Xin, dW=dW, db=db, tiles=tiles: gemm(
                    TN, N, K, M, dZ, dZ.stride(0), Xin, Xin.stride(0), dW, K, accumulate=True,
                    splits=_splits_for(M, tiles, self.bprec), prec=self.bprec, colsum=db))
                dg = gt.reshape(-1) if gt is not None else torch.zeros(N, device=dev)
                dv = vt if vt is not None else torch.zeros(N, K, device=dev)
                _wn_bwd(g.reshape(-1), v, self.norms[l], dW, dg, dv)
            if l > 0:
                pa, pbeta, pthr = self.acts[l - 1]
                dprev = _alloc(M, K, dev)
                zaux, did = self._grad_src(l - 1) if pa != 0 else (None, 0)
                gemm(NN, M, K, N, dZ, dZ.stride(0), self.Ws[l], self.Ws[l].stride(0), dprev, dprev.stride(0),
                     aux=zaux, ldaux=0 if zaux is None else zaux.stride(0), dact=did, beta=pbeta, thr=pthr,
                     prec=self.bprec)
                dZ = dprev
            elif need_dx:
                dx = dx_out if dx_out is not None else _alloc(M, K, dev)
                gemm(NN, M, K, N, dZ, dZ.stride(0), self.Ws[0], self.Ws[0].stride(0), dx, dx.stride(0),
                     prec=self.bprec)
        return dx, grads


class SmallRun:
    """A single weight-normed linear layer with C <= 16 outputs on the narrow-layer kernels (mms_small_linear_fwd/bwd,
    fp32 VALU): the background density head (256 -> 1) and the 1-layer background modality heads (128 -> C).  Same
    interface as MLPRun; the bf16 precision modes only (the fp32 parity mode keeps the f32-MFMA GEMMs)."""

    def __init__(self, params: Sequence[torch.Tensor], acts: Sequence[Tuple[int, float, float]], prec: int = 1):
        self.params = list(params)
        self.acts = list(acts)
        self.prec = int(prec)
        self.x = self.W = self.norm = self.Y = None

    @staticmethod
    def serves(params, acts, prec: int) -> bool:
        if prec == 0 or len(params) != 3:
            return False
        N, K = params[1].shape
        return acts[0][0] in (0, 1, 2, 3) and SmallRun.shape_ok(N, K)

    @staticmethod
    def shape_ok(N: int, K: int) -> bool:
        """The narrower of the two kernels' limits (mms_small_linear_bwd: K 128 up to 16 outputs, K 256 up to 8, K 512
        up to 4), so a layer whose forward runs here always has a backward."""
        return 1 <= N <= 16 and (K == 128 or (K in (256, 512) and N <= 2048 // K))

    def forward(self, x: torch.Tensor, keep: bool, last_out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """x [M, K] with unit column stride and 16-B aligned rows (a column view of a wider panel is fine)."""
        M = x.shape[0]
        g, v, b = self.params
        N, K = v.shape
        W, nrm = normed_weight(g, v)
        act, beta, thr = self.acts[0]
        Y = last_out if last_out is not None else torch.empty(M, N, device=x.device)
        _lib.call("mms_small_linear_fwd", x.data_ptr(), x.stride(0), M, K, W.data_ptr(), _p(b), N, act, beta, thr,
                  Y.data_ptr(), Y.stride(0), _s())
        if keep:
            self.x, self.W, self.norm, self.Y = x, W, nrm, Y
        return Y

    def backward(self, dy: torch.Tensor, need_dx: bool, pre_activated: bool = False,
                 dx_out: Optional[torch.Tensor] = None, accumulate: bool = False):
        """dx written into (or, accumulate, added to) ``dx_out`` when given; parameter gradients accumulated in place."""
        x, Y = self.x, self.Y
        M = x.shape[0]
        dev = x.device
        g, v, b = self.params
        N, K = v.shape
        act, beta, thr = self.acts[0]
        gt, vt, bt = grad_target(g), grad_target(v), grad_target(b)
        need_w = gt is not None or vt is not None or bt is not None
        dW = _dw_views([v], dev)[0] if need_w else None
        db = (bt if bt is not None else torch.zeros(N, device=dev)) if need_w else None
        dx = None
        if need_dx:
            dx = dx_out if dx_out is not None else _alloc(M, K, dev)
        dy = dy if dy.stride(1) == 1 else dy.contiguous()
        _lib.call("mms_small_linear_bwd", x.data_ptr(), x.stride(0), M, K, self.W.data_ptr(), N,
                  0 if pre_activated else act, beta, thr, Y.data_ptr(), Y.stride(0), dy.data_ptr(), dy.stride(0),
                  _p(dx), 0 if dx is None else dx.stride(0), int(accumulate and dx_out is not None), _p(dW), _p(db),
                  _s())
        if need_w:
            _wn_bwd(g.reshape(-1), v, self.norm, dW, gt.reshape(-1) if gt is not None else
                    torch.zeros(N, device=dev), vt if vt is not None else torch.zeros(N, K, device=dev))
        self.x = self.Y = None
        return dx, [None, None, None]


# the SDF taps' weight-gradient row inside the backward chain (MMS_TAP_WGRAD=0: a grouped weight-gradient item)
TAP_WGRAD_IN_CHAIN = os.environ.get("MMS_TAP_WGRAD", "1") != "0"

class ChainRun:
    """A weight-normed 3- or 4-layer MLP on the fused chain kernel (mms_mlp_chain: all layers in one launch, bf16 or
    split-bf16x3 operands) plus the weight-gradient GEMMs.  Serves the SDF (71-256-256-257), radiance
    (317-256-256-256) and background NeRF (39-256-256-256-256, 283-256-256-256-128) MLPs in the bf16 precision modes;
    the fp32 parity mode keeps MLPRun.

    ``rows_full``: rows >= rows_full only need output column 0 (the SDF's tap rows, surface_model.py:137-153)."""

    def __init__(self, params: Sequence[torch.Tensor], acts: Sequence[Tuple[int, float, float]], prec: int,
                 chain_prec: int = 0):
        if prec not in (1, 2, 4, 5):
            raise ValueError("the fused chain runs the bf16 (1), split-bf16x3 (2), x3-forward (4) and fp16-forward (5) "
                             "modes")
        self.params, self.acts = list(params), list(acts)
        # the forward chain's operand mode (or chain_prec 3: split activations x bf16 weights); the backward chain and
        # the weight gradients run bwd_prec (mode 4: split-bf16x3 forward, bf16 backward)
        self.prec = bwd_prec(int(prec))
        self.cprec = int(chain_prec) or fwd_prec(int(prec))
        self.bcprec = self.prec if int(prec) in (4, 5) else self.cprec
        if PRECISION.get("bwd16", 0) and self.bcprec == 2:
            self.bcprec = 6
        self.L = len(self.params) // 3
        if self.L not in (3, 4):
            raise ValueError("chains of 3 or 4 layers")
        self.beta, self.thr = float(acts[0][1]), float(acts[0][2])

    def _pack(self, W, rows: int, cols: int, transpose: bool, permute: int, prec: Optional[int] = None):
        prec = self.cprec if prec is None else prec
        if prec == 5:
            permute = int(permute) | 4      # fp16 image (mms_mlp_pack permute bit 2), hi only
        prep = _ACTIVE_PREP[0]
        if prep is not None:
            return prep.packed(W, rows, cols, transpose, permute, prec)
        return self._pack_new(W, rows, cols, transpose, permute, prec)

    def _pack_new(self, W, rows: int, cols: int, transpose: bool, permute: bool, prec: int):
        hi = torch.empty(rows, cols, dtype=torch.bfloat16, device=W.device)
        lo = torch.empty_like(hi) if prec == 2 else None
        N, K = W.shape
        _lib.call("mms_mlp_pack", W.data_ptr(), N, K, W.stride(0), int(transpose), int(permute), rows, cols,
                  hi.data_ptr(), _p(lo), _s())
        return hi, lo

    def _chain(self, backward: bool, X, K0: int, rows_full: int, packs, bias, aux, outs, Ns, acts,
               xaux=None, xact: int = 0, xout=None, w2row0=None, tap_part=None, rinv=None, emax=None, f16=None):
        prec = self.bcprec if backward else self.cprec
        n = self.L
        VP = ctypes.c_void_p * n
        his = VP(*[p[0].data_ptr() for p in packs])
        los = VP(*[(p[1].data_ptr() if p[1] is not None else None) for p in packs])
        bs = VP(*[(b.data_ptr() if b is not None else None) for b in bias])
        auxs = VP(*[(a.data_ptr() if a is not None else None) for a in aux])
        ldaux = (ctypes.c_int64 * n)(*[(a.stride(0) if a is not None else 0) for a in aux])
        os_ = VP(*[(o.data_ptr() if o is not None else None) for o in outs])
        ldo = (ctypes.c_int64 * n)(*[(o.stride(0) if o is not None else 0) for o in outs])
        ns = (ctypes.c_int * n)(*Ns)
        ac = (ctypes.c_int * n)(*acts)
        cast = lambda a: ctypes.cast(a, ctypes.c_void_p)
        _lib.call("mms_mlp_chain", prec, int(backward), n, X.data_ptr(), X.stride(0), K0,
                  X.shape[0], rows_full,
                  _p(xaux), 0 if xaux is None else xaux.stride(0), int(xact), _p(xout),
                  0 if xout is None else xout.stride(0), cast(his), cast(los), cast(bs), cast(auxs), cast(ldaux),
                  cast(os_), cast(ldo), cast(ns), cast(ac), self.beta, self.thr, _p(w2row0), _p(tap_part),
                  0 if tap_part is None else tap_part.stride(0),
                  None if rinv is None else cast(VP(*[_p(r) for r in rinv])), _p(emax),
                  None if f16 is None else cast((ctypes.c_int * n)(*[int(bool(f)) for f in f16])), _s())

    def forward(self, x: torch.Tensor, keep: bool, rows_full: Optional[int] = None,
                dense_col0: bool = False, last_out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """x [M, K0] (16-B aligned rows); returns the last layer's output [M, N_last] (row stride rounded to 4; or
        ``last_out``, a 16-B aligned [M, N_last] view the caller owns), or with dense_col0 (rows_full = 0) its column 0
        as a dense [M] vector."""
        M, K0 = x.shape
        dev = x.device
        L = self.L
        self.x = x
        self.Ws, self.norms = [], []
        for l in range(L):
            g, v, _ = self.params[3 * l: 3 * l + 3]
            W, nrm = normed_weight(g, v)
            self.Ws.append(W)
            self.norms.append(nrm)
        Ns = [W.shape[0] for W in self.Ws]
        nt = [(n + 31) // 32 for n in Ns]
        packs = [self._pack(self.Ws[0], 32 * nt[0], 16 * ((K0 + 15) // 16), False, False)] + \
                [self._pack(self.Ws[l], 32 * nt[l], 32 * nt[l - 1], False, True) for l in range(1, L)]
        self.rows_full = M if rows_full is None else int(rows_full)
        if dense_col0 and self.rows_full != 0:
            raise ValueError("dense_col0 needs rows_full = 0")
        if dense_col0:
            last = torch.empty(M, device=dev).view(M, 1)
        else:
            last = last_out if last_out is not None else _alloc(M, Ns[-1], dev)
        y16 = keep and self._fp16_panels(Ns) and bool(PRECISION.get("y16", 0))
        if y16:   # (whole 32-column tiles per row)
            Y = [torch.empty(M, 32 * ((Ns[l] + 31) // 32), dtype=torch.float16, device=dev)[:, :Ns[l]]
                 for l in range(L - 1)] + [last]
        else:
            Y = [_alloc(M, Ns[l], dev) if keep else None for l in range(L - 1)] + [last]
        self._chain(False, x, K0, self.rows_full, packs, [self.params[3 * l + 2] for l in range(L)], [None] * L, Y,
                    Ns, [a[0] for a in self.acts], w2row0=self.Ws[-1],
                    f16=[y16] * (L - 1) + [False] if y16 else None)
        self.Y = Y
        # a training forward fetches the backward's transposed images too, so a model forward prepares them in the
        # same batched launch (WeightPrep) instead of one pack launch each in the backward
        self.bwd_packs = self._bwd_packs(K0) if keep else None
        return Y[-1].view(M) if dense_col0 else Y[-1]

    def _fp16_panels(self, Ns) -> bool:
        """Presets fast_h16c / d: this MLP's hidden-layer weight gradients take fp16 panels (a prec-6 backward chain
        whose hidden layers feed the wide weight-gradient engine)."""
        return bool(PRECISION.get("wgrad16", 0)) and self.bcprec == 6 and min(Ns[:self.L - 1]) >= 128

    def _bwd_packs(self, K0: int):
        """Backward chain images: W_last^T (natural: B = dy from memory), then the earlier layers' W^T (register-fed,
        permuted)."""
        L = self.L
        Ns = [W.shape[0] for W in self.Ws]
        up = lambda n, k: k * ((n + k - 1) // k)  # noqa: E731
        p = self.bcprec
        p0, pr = (2, 5) if p == 6 else (p, p)     # prec 6: the first layer split-bf16x3, the rest fp16
        return [self._pack(self.Ws[L - 1], up(Ns[L - 2], 32), up(Ns[L - 1], 16), True, False, p0)] + \
               [self._pack(self.Ws[l], up(Ns[l - 1] if l > 0 else K0, 32), up(Ns[l], 32), True, True, pr)
                for l in range(L - 2, -1, -1)]

    def backward(self, dy: torch.Tensor, dx_out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """dy [M, N_last] (rows >= rows_full: column 0 only); accumulates the parameter gradients (grad_target) and
        returns dx [M, K0] (written into ``dx_out``, a [M, K0] view with unit column stride, when given)."""
        x, Y = self.x, self.Y
        M, K0 = x.shape
        dev = x.device
        L = self.L
        Ns = [W.shape[0] for W in self.Ws]
        acts = [a[0] for a in self.acts]
        packs = self.bwd_packs if self.bwd_packs is not None else self._bwd_packs(K0)
        # the scaled input's store writes 16 ceil(N/16) columns per row (zeros past N)
        dZl = _alloc(M, 32 * ((Ns[L - 1] + 31) // 32), dev)[:, :Ns[L - 1]] if acts[L - 1] != 0 else None
        order = list(range(L - 2, -1, -1))           # hidden layers, last first
        # preset wgrad16: the hidden layers' dZ as the chain's fp16 row-scaled values (whole 32-column tiles per row),
        # their inverse row scales and per-layer largest exponents (chain slot order), for gemm_tn_wide16
        w16 = self._fp16_panels(Ns)
        rinv = emax = None
        if w16:
            dZ = [torch.empty(M, 32 * ((Ns[l] + 31) // 32), dtype=torch.float16, device=dev)[:, :Ns[l]]
                  for l in range(L - 1)]
            rinv = [torch.empty(M, device=dev) for _ in range(L - 1)]
            emax = torch.zeros(L, dtype=torch.int32, device=dev)
        else:
            dZ = [_alloc(M, Ns[l], dev) for l in range(L - 1)]
        dx = dx_out if dx_out is not None else _alloc(M, K0, dev)
        dy = dy if dy.stride(1) == 1 and dy.stride(0) % 4 == 0 else _copy_aligned(dy)
        rf = self.rows_full
        dWs = _dw_views([self.params[3 * l + 1] for l in range(L)], dev)
        dbs = []
        for l in range(L):
            N = self.params[3 * l + 1].shape[0]
            bt = grad_target(self.params[3 * l + 2])
            dbs.append(bt if bt is not None else torch.zeros(N, device=dev))
        needs = [any(grad_target(p) is not None for p in self.params[3 * l: 3 * l + 3]) for l in range(L)]
        # the SDF chain: the taps' (rows >= rows_full: sdf column only) share of the last layer's weight-gradient row 0
        # is summed inside the backward chain from the Y rows it loads anyway (per-block partial rows, mms_mlp_chain
        # tap_part), then reduced into dW[0] / db[0] (mms_rowsum_add)
        tapw = TAP_WGRAD_IN_CHAIN and rf < M and needs[L - 1] and L == 3 and acts[0] == 2 and acts[L - 1] == 0
        tap_part = None
        if tapw:
            n0 = Ns[L - 2]
            B = _lib.lib().mms_mlp_chain_block_rows()
            tap_part = torch.empty(-(-M // B) - rf // B, n0 + 4, device=dev)
        self._chain(True, dy, Ns[L - 1], rf, packs, [None] * L, [Y[l] for l in order] + [None],
                    [dZ[l] for l in order] + [dx], [Ns[l] for l in order] + [K0], [acts[l] for l in order] + [0],
                    xaux=Y[L - 1] if acts[L - 1] != 0 else None, xact=acts[L - 1], xout=dZl, tap_part=tap_part,
                    rinv=None if rinv is None else [rinv[l] for l in order] + [None], emax=emax,
                    f16=[Y[l].dtype == torch.float16 for l in order] + [False])
        if tapw:
            _lib.call("mms_rowsum_add", tap_part.data_ptr(), tap_part.shape[0], n0 + 1, tap_part.stride(0),
                      dWs[L - 1].data_ptr(), n0, dbs[L - 1].data_ptr(), _s())
        dZ = dZ + [dZl if dZl is not None else dy]
        Xin = [x] + Y[:L - 1]
        # every layer's weight gradient dW_l += dZ_l^T X_l (+ bias column sums) in ONE grouped launch
        items, items16, wn = [], [], []
        for l in range(L):
            g, v, b = self.params[3 * l: 3 * l + 3]
            N, K = v.shape
            gt, vt = grad_target(g), grad_target(v)
            if not needs[l]:
                continue
            dW = dWs[l]
            db = dbs[l]
            A, B = dZ[l], Xin[l]
            if w16:
                # one mixed launch: the hidden layers' fp16 dZ (chain slot c's rinv / emax), the output layer's fp32 dY
                B = B if _aligned16(B) else _copy_aligned(B)
                if l < L - 1:
                    c = order.index(l)
                    items16.append((N, K, M, A, rinv[l], emax[c:c + 1], B, dW, db))
                else:
                    A = A if _aligned16(A) else _copy_aligned(A)
                    items16.append((N, K, rf if rf < M else M, A, None, None, B, dW, db))
                    if rf < M and not tapw:
                        items16.append((1, K, M - rf, A[rf:], None, None, B[rf:], dW, db))
            elif l == L - 1 and rf < M:
                # rows past rows_full carry only the output column 0 (summed by the chain above when tapw)
                items.append((N, K, rf, A, B, dW, db))
                if not tapw:
                    items.append((1, K, M - rf, A[rf:], B[rf:], dW, db))
            else:
                items.append((N, K, M, A, B, dW, db))
            wn.append((g, v, l, dW, gt, vt, N, K))
        if items or items16:
            wp = PRECISION.get("wgrad", 0) or self.prec     # the weight gradients' operand mode (preset "wgrad")

            def launch(items=items, items16=items16, prec=wp):
                if items16:
                    gemm_tn_wide16(items16)
                if items:
                    gemm_tn_grouped(items, prec)
            if _WGRAD_DEFER[0] is not None:
                _wgrad(launch)
            elif ASYNC_WGRAD and _WN_BWD[0] is not None:
                _wgrad_async(launch, [t for it in items + items16 for t in it[3:] if isinstance(t, torch.Tensor)], dev)
            else:
                launch()
        for g, v, l, dW, gt, vt, N, K in wn:
            _wn_bwd(g.reshape(-1), v, self.norms[l], dW, gt.reshape(-1) if gt is not None else
                    torch.zeros(N, device=dev), vt if vt is not None else torch.zeros(N, K, device=dev))
        self.Y = self.x = self.bwd_packs = None
        return dx


# Deferred weight gradients (wgrad_defer_begin / wgrad_flush): the data-parallel graph step ends its first captured
# graph when the backward has queued the hash-table gradients (97 % of the all-reduce payload), starts
# their all-reduce, and replays the MLPs' weight-gradient GEMMs -- queued here instead of launched -- as a second graph
# while the exchange runs (graphs.GraphTrainer).  Everything a deferred launch reads stays referenced by its closure.
_WGRAD_DEFER: List[Optional[list]] = [None]


_WGRAD_DEFER_STREAM: List[Optional[int]] = [None]


def wgrad_defer_begin(this_stream_only: bool = False) -> None:
    """Queue the MLPs' weight-gradient launches until wgrad_flush; ``this_stream_only``: only those issued on the
    calling stream (the background stream's stay inline, beside the main stream's work)."""
    if _WN_BWD[0] is None:
        raise RuntimeError("weight gradients are deferred only inside a batched training backward (wn_bwd_begin)")
    _WGRAD_DEFER[0] = []
    _WGRAD_DEFER_STREAM[0] = _s() if this_stream_only else None


def wgrad_flush() -> None:
    """Launch the deferred weight-gradient GEMMs in backward order (before the deferred weight-norm flush, which
    reads their dW)."""
    q, _WGRAD_DEFER[0] = _WGRAD_DEFER[0], None
    _WGRAD_DEFER_STREAM[0] = None
    for fn in q or []:
        fn()


def _wgrad(fn) -> None:
    """Run a weight-gradient launch now, or queue it while the weight gradients are deferred."""
    if _WGRAD_DEFER[0] is not None and (_WGRAD_DEFER_STREAM[0] is None or _WGRAD_DEFER_STREAM[0] == _s()):
        _WGRAD_DEFER[0].append(fn)
    else:
        fn()


# Weight gradients on a side stream (MMS_SYNC_WGRAD=0).  Inside a training backward (deferred weight norm: nothing
# reads dW before the flush) an MLP's grouped weight-gradient launch can go to a side stream forked from the caller's,
# beside the hash-grid backward (the grid needs only the chain's dx); a final autograd callback joins the side stream
# back into the caller's stream, so the weight-norm flush and the optimizer see every gradient.  With the 128 x 128
# tiled engine that overlap paid (521k -> 545-556k rays/s in round 2); the wide engine's 8-wave, 152 KB-LDS blocks
# fill whole CUs, so beside the hash walk they only contend: inline, wide 540.6k vs side stream, tiled 514-522k,
# wide 506.8k (round-3 A/B, profiles/round3b_wgrad_ab.txt).  Inline by default.
ASYNC_WGRAD = os.environ.get("MMS_SYNC_WGRAD", "1") != "1"
_WGRAD_STREAMS: dict = {}


def wgrad_stream(dev) -> "torch.cuda.Stream":
    i = torch.device(dev).index or 0
    if i not in _WGRAD_STREAMS:
        _WGRAD_STREAMS[i] = torch.cuda.Stream(device=i)
    return _WGRAD_STREAMS[i]


def join_wgrad(i: int) -> None:
    if i in _WGRAD_STREAMS:
        torch.cuda.current_stream(i).wait_stream(_WGRAD_STREAMS[i])


def _wgrad_async(launch, tensors, dev) -> None:
    """launch() (an MLP's weight-gradient launch) on the side stream, forked from the caller's; ``tensors``: what it
    reads or writes (made or freed on the caller's stream)."""
    cur = torch.cuda.current_stream(dev)
    side = wgrad_stream(dev)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        launch()
    seen = set()
    for t in tensors:
        if t.data_ptr() not in seen:
            seen.add(t.data_ptr())
            t.record_stream(side)
    i = torch.device(dev).index or 0
    torch.autograd.Variable._execution_engine.queue_callback(lambda: join_wgrad(i))


# Weight-norm backward of the layers, deferred inside a training backward (wn_bwd_begin / wn_bwd_flush, Trainer and
# GraphTrainer) and then applied in one batched launch; immediate everywhere else (a bare loss.backward()).
class _WnBwdItem(ctypes.Structure):
    """MmsWnBwdItem (include/mms_hip.h)."""
    _fields_ = [("g", ctypes.c_void_p), ("v", ctypes.c_void_p), ("norms", ctypes.c_void_p), ("N", ctypes.c_int64),
                ("K", ctypes.c_int64), ("dW", ctypes.c_void_p), ("lddw", ctypes.c_int64), ("dg", ctypes.c_void_p),
                ("dv", ctypes.c_void_p), ("row0", ctypes.c_int64)]


_WN_BWD: List[Optional[dict]] = [None]     # v.data_ptr() -> (g, v, norms, dW, dg, dv), one entry per layer
_WN_DW: List[Optional[dict]] = [None]      # v.data_ptr() -> the layer's dW accumulation buffer of this backward
_WN_BWD_MAX = 32


def wn_bwd_begin() -> None:
    """Defer the weight-norm backward: every use of a layer in this backward (the SDF and radiance MLPs serve every
    modality) accumulates its weight gradient into ONE dW buffer, and the flush applies the (linear) weight-norm
    backward once per layer -- no two blocks of the batched launch update the same parameter."""
    _WN_BWD[0] = {}
    _WN_DW[0] = {}


def _dw_views(vs, dev) -> List[torch.Tensor]:
    """Zeroed dW accumulation buffers of layers (their v tensors): fresh per call, or shared per layer while the
    weight-norm backward is deferred."""
    st = _WN_DW[0]
    if st is None:
        return _zeroed_views([tuple(v.shape) for v in vs], dev)
    missing = [v for v in vs if v.data_ptr() not in st]
    if missing:
        for v, buf in zip(missing, _zeroed_views([tuple(v.shape) for v in missing], dev)):
            st[v.data_ptr()] = buf
    return [st[v.data_ptr()] for v in vs]


def wn_bwd_flush() -> None:
    """Apply the deferred weight-norm gradients (batches of up to 32 layers per launch)."""
    items = list((_WN_BWD[0] or {}).values())
    _WN_BWD[0] = _WN_DW[0] = None
    for i in range(0, len(items or []), _WN_BWD_MAX):
        chunk = items[i:i + _WN_BWD_MAX]
        arr, row0 = (_WnBwdItem * len(chunk))(), 0
        for j, (g, v, nrm, dW, dg, dv) in enumerate(chunk):
            N, K = v.shape
            arr[j] = _WnBwdItem(g.data_ptr(), v.data_ptr(), nrm.data_ptr(), N, K, dW.data_ptr(), dW.stride(0),
                                dg.data_ptr(), dv.data_ptr(), row0)
            row0 += N
        _lib.call("mms_weight_norm_bwd_batched", ctypes.cast(arr, ctypes.c_void_p), len(chunk), row0, _s())


def _wn_bwd(g, v, norms, dW, dg, dv) -> None:
    st = _WN_BWD[0]
    if st is not None:
        # once per layer (dW is the layer's shared accumulation buffer); the tensors stay referenced until the flush
        if v.data_ptr() not in st:
            st[v.data_ptr()] = (g, v, norms, dW, dg, dv)
    else:
        weight_norm_bwd(g, v, norms, dW, dg, dv)


class _ZeroArena:
    """One zero-filled f32 buffer per training step that the step's scratch gradients are carved from (zero_arena_begin
    / zero_arena_end around forward + loss + backward): ONE fill launch per step instead of one per backward function
    (~30 fills, each a graph node of ~5 us).  Sized from the previous step's demand; a step that needs more takes
    fresh zeroed buffers for the rest.  Buffers a captured graph may reference are never freed."""

    def __init__(self):
        self.buf: Optional[torch.Tensor] = None
        self.keep: List[torch.Tensor] = []
        self.off = 0
        self.need = 0
        self.dev = None
        self.in_step = False   # between begin / end: demand is counted even before the buffer exists
        self.active = False


_ARENA = _ZeroArena()
_ARENA_OFF = os.environ.get("MMS_NO_ZERO_ARENA", "0") == "1"   # debugging: per-function zero fills
_ALIGN = 64          # floats: every carved buffer starts on a 256-B boundary (vector / GEMM paths)
# debugging (scripts/fullsize_graph_probe.py): a zero gap of this many floats after every carved buffer, checked by
# arena_guard_report() -- a kernel that writes past its zeroed buffer shows up as a nonzero gap, named by its carve site
_ARENA_GUARD = int(os.environ.get("MMS_ARENA_GUARD", "0"))
_ARENA_SITES: List = []


def arena_guard_report() -> List[str]:
    """Carve sites whose guard gap was written (MMS_ARENA_GUARD builds only); call after a synchronize."""
    a = _ARENA
    bad = []
    for off, n, site in _ARENA_SITES:
        if a.buf is not None and off + n + _ARENA_GUARD <= a.buf.numel():
            gap = a.buf[off + n: off + n + _ARENA_GUARD]
            nz = int((gap != 0).sum())
            if nz:
                bad.append(f"{site}: {nz} gap floats written past a {n}-float buffer")
    return bad


def _arena_grow(dev) -> None:
    # outside a capture only (a buffer allocated while capturing would live in that graph's private pool)
    a = _ARENA
    size = a.buf.numel() if a.buf is not None else 0
    capturing = torch.device(dev).type == "cuda" and torch.cuda.is_current_stream_capturing()
    if a.need > size and not capturing:
        if a.buf is not None:
            a.keep.append(a.buf)
        a.buf = torch.empty(int(a.need * 1.25) + 4 * _ALIGN, device=dev)


def zero_arena_prepare(dev) -> Optional[torch.Tensor]:
    """The buffer the next zero_arena_begin(dev, zeroed=...) will carve from (grown first if the last step needed
    more), for a caller that zeroes it together with other buffers in one launch; None when there is none."""
    _arena_grow(dev)
    a = _ARENA
    return a.buf if a.buf is not None and a.buf.device == torch.device(dev) else None


def zero_arena_begin(dev, zeroed: Optional[torch.Tensor] = None) -> None:
    """Start a step's arena; ``zeroed``: the zero_arena_prepare buffer the caller has already zeroed."""
    a = _ARENA
    if zeroed is None or zeroed is not a.buf:
        _arena_grow(dev)
        zeroed = None
    a.dev = dev
    a.need, a.off = 0, 0
    _ARENA_SITES.clear()
    a.in_step = not _ARENA_OFF
    a.active = a.buf is not None and a.buf.device == torch.device(dev)
    if a.active and zeroed is None:
        a.buf.zero_()


def zero_arena_end() -> None:
    a = _ARENA
    if a.in_step:
        # sized right after the step that measured the demand, so the graphs captured next (GraphTrainer captures
        # straight after one eager step, every later begin runs inside a capture) already carve from it
        _arena_grow(a.dev)
    a.active = False
    a.in_step = False


def _zeroed_views(shapes, dev) -> List[Optional[torch.Tensor]]:
    """Zero-filled f32 accumulation buffers (None for a None shape) carved from the step's zero arena, or from one
    fresh zeroed allocation outside a training step / past the arena."""
    if all(sh is None for sh in shapes):
        return [None] * len(shapes)        # nothing carved: the arena offset keeps its 256-B alignment
    sizes = [0 if sh is None else math.prod(sh) for sh in shapes]
    padded = [(n + _ALIGN - 1) // _ALIGN * _ALIGN for n in sizes]
    total = max(sum(padded), 1)
    a = _ARENA
    if a.in_step:
        a.need += total + _ARENA_GUARD     # (counted from the first step on: the buffer is sized at the next begin)
    if a.active and a.off + total + _ARENA_GUARD <= a.buf.numel():
        buf = a.buf[a.off:a.off + total]
        if _ARENA_GUARD:
            import traceback
            site = " <- ".join(f"{fr.name}:{fr.lineno}" for fr in traceback.extract_stack(limit=6)[-6:-1][::-1])
            _ARENA_SITES.append((a.off, total, f"{shapes} @ {site}"))
        a.off += total + _ARENA_GUARD
    else:
        buf = torch.zeros(total, device=dev)
    out, off = [], 0
    for sh, n, pn in zip(shapes, sizes, padded):
        out.append(None if sh is None else buf[off:off + n].view(tuple(sh)))
        off += pn
    return out


# Gradient accumulators shared by a tensor's consumers.  A tensor read by k autograd Functions (the rays' directions:
# five consumers; the hit rays' directions: four; the sample positions and the SDF gradients: two) otherwise costs
# k - 1 ATen adds per step (autograd sums the parts; each add a ~4-5 us graph node).  Its producer attaches a GradAcc
# in the forward; every consumer on the producer's stream whose backward kernel accumulates (+=) into a zeroed buffer
# accumulates into the accumulator's ONE buffer instead and returns None for that input; the producer -- whose
# backward runs after all of its outputs' consumers, on the same stream -- takes the buffer (plus the parts the other
# consumers returned) as the output's gradient.  Consumers on the background stream keep returning their parts:
# autograd orders them with the main stream and adds them (a shared buffer across the two streams raced on the first
# step, round 4).  MMS_GRAD_ACC=0: per-consumer buffers everywhere.
GRAD_ACC = os.environ.get("MMS_GRAD_ACC", "1") != "0"

# Two-phase backward (graph-replayed data-parallel steps, graphs.GraphTrainer): while PHASE_CUT is a list, the model's
# forward hands every tensor that the SDF side (the surface field, the NeuS samples, the hit rays, the rays) passes to
# the radiance / rendering / background / loss side through cut(): the consumers get a detached leaf copy and the pair
# is recorded.  The training backward then runs in two caller-thread phases (pipeline.backward_batched ``mid``):
# phase 1 from the loss down to the cut leaves -- the radiance field and its hash table, the heads, the composite, the
# NeuS weights and the background, so the radiance (and grid-background) table gradients are final when it returns --
# and phase 2 from the cut tensors with the leaves' gradients -- the SDF field, its table, the sampler, the rays and the
# poses.  Between the two the graph capture ends and restarts on the caller's thread, so the radiance table's
# all-reduce goes out while the SDF backward replays.  The arithmetic is unchanged: phase 2 delivers each
# leaf's gradient to its producer as the single backward would (test_gpu_graph.py::test_phase_cut_backward).
PHASE_CUT: List = [None]


def cut(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    """Forward: the phase-1 consumers' view of SDF-side tensor ``t`` (a detached leaf while PHASE_CUT is active)."""
    rec = PHASE_CUT[0]
    if rec is None or t is None or not t.requires_grad:
        return t
    d = t.detach().requires_grad_(True)
    rec.append((t, d))
    return d


def phase_two(cuts) -> None:
    """Backward phase 2: the cut tensors' gradients (accumulated on their leaf copies by phase 1) into the SDF side."""
    ts, gs = [], []
    for t, d in cuts:
        if d.grad is not None:
            ts.append(t)
            gs.append(d.grad)
    if ts:
        torch.autograd.backward(ts, gs)


class GradAcc:
    __slots__ = ("shape", "dev", "_buf", "_home")

    def __init__(self, t: torch.Tensor):
        # made in the producer's forward, on the stream its backward will run on (autograd's stream semantics)
        self.shape, self.dev, self._buf = tuple(t.shape), t.device, None
        self._home = self._key()

    def _key(self):
        return torch.cuda.current_stream(self.dev).cuda_stream if self.dev.type == "cuda" else 0

    def buf(self) -> torch.Tensor:
        """The zeroed accumulation buffer (carved from the step's zero arena on first use)."""
        if self._buf is None:
            self._buf = _zeroed_views([self.shape], self.dev)[0]
        return self._buf

    def total(self, incoming: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        """The producer's view: the accumulated gradient (+ the parts autograd delivered)."""
        b, self._buf = self._buf, None
        if b is None:
            return incoming
        return b if incoming is None else b + incoming


def attach_acc(t: torch.Tensor) -> torch.Tensor:
    """Producer forward: give output ``t`` a shared gradient accumulator (GRAD_ACC)."""
    if GRAD_ACC:
        t._mms_acc = GradAcc(t)
    return t


def acc_of(t) -> Optional[GradAcc]:
    """Consumer forward: the accumulator of input ``t`` -- None when none is attached or when this consumer runs on
    another stream than the producer (its backward then returns its part as usual: autograd orders and adds it)."""
    a = getattr(t, "_mms_acc", None) if t is not None else None
    return a if a is not None and a._key() == a._home else None


def acc_or_zeroed(acc: Optional[GradAcc], shape, dev, need: bool = True) -> Optional[torch.Tensor]:
    """Consumer backward: the buffer its kernel accumulates into -- the shared one, or a zeroed one of its own."""
    if not need:
        return None
    return acc.buf() if acc is not None else _zeroed_views([tuple(shape)], dev)[0]


def acc_ret(acc: Optional[GradAcc], g):
    """Consumer backward: the gradient it returns for that input (None when it went into the shared buffer)."""
    return None if acc is not None else g


def _capturing(dev) -> bool:
    return torch.device(dev).type == "cuda" and torch.cuda.is_current_stream_capturing()


def _aligned16(t: torch.Tensor) -> bool:
    """16-B aligned rows of unit column stride (the wide weight-gradient engine's fp32 operands)."""
    return t.data_ptr() % 16 == 0 and t.stride(1) == 1 and t.stride(0) % 4 == 0


def _copy_aligned(t: torch.Tensor) -> torch.Tensor:
    out = _alloc(t.shape[0], t.shape[1], t.device)
    out.copy_(t)
    return out


# ------------------------------------------------------------------------------------------------
# surface field (SDF + taps)
# ------------------------------------------------------------------------------------------------
SDF_ACTS = ((2, 100.0, 20.0), (2, 100.0, 20.0), (0, 1.0, 20.0))


class SurfaceFunction(torch.autograd.Function):
    """pos [M,3] -> (sdf [M,1], geo [M,G], grads [M,3], hess [M,3], normals [M,3]).

    Rows of the MLP batch: [centre M | 4 x taps M]; panel columns [x(3), PE-tail(36), grid(32)].
    `delta` is the tap offset numerical_gradients_delta / sqrt(3) (surface_model.py:138).
    """

    @staticmethod
    def forward(ctx, pos, table, grid: GridCfg, active: int, delta: float, *params):
        ctx.set_materialize_grads(False)   # unused outputs' gradients arrive as None (no zero fills)
        ctx.acc_pos = acc_of(pos)
        M = pos.shape[0]
        dev = pos.device
        pos = pos.contiguous()
        K0 = 3 + 36 + grid.out_dim
        X = _alloc(5 * M, K0, dev)
        d32 = float(torch.tensor(delta, dtype=torch.float32))
        sdf_panel(pos, 3, M, 4, d32, grid, table, active, X)
        prec = PRECISION["sdf"]
        ctx.chain = None
        if prec != 0:
            # bf16 modes: the whole 3-layer chain in one kernel; tap rows keep only the sdf column
            chain = ChainRun(params, SDF_ACTS, prec, PRECISION["sdf_chain"])
            out = chain.forward(X, keep=True, rows_full=M)
            ctx.chain = chain
        else:
            out = _sdf_mlp_unfused(ctx, X, M, params, dev)
        G = out.shape[1] - 1
        four_delta = float(torch.tensor(4.0 * delta, dtype=torch.float32))
        delta_sq = float(torch.tensor(delta ** 2, dtype=torch.float32))
        grads = torch.empty(M, 3, device=dev)
        hess = torch.empty(M, 3, device=dev)
        normals = torch.empty(M, 3, device=dev)
        _lib.call("mms_taps_combine_fwd", out.data_ptr(), out.stride(0), M, four_delta, delta_sq, grads.data_ptr(),
                  hess.data_ptr(), normals.data_ptr(), _s())
        # views of the MLP output rows (row stride = the panel pitch): the consumers take strides, no copies
        sdf = out[:M, 0:1]
        geo = out[:M, 1:]
        ctx.grid, ctx.active, ctx.M, ctx.G = grid, active, M, G
        ctx.table = ctx.table_p = table          # the Parameter itself: its .grad is accumulated in place
        if ctx.needs_input_grad[1]:
            _grad_use(table)
        ctx.four_delta, ctx.delta_sq = four_delta, delta_sq
        ctx.X = X
        ctx.save_for_backward(pos, table, grads, *params)
        ctx.acc_grads = GradAcc(grads) if GRAD_ACC else None
        if ctx.acc_grads is not None:
            grads._mms_acc = ctx.acc_grads
        return sdf, geo, grads, hess, normals

    @staticmethod
    def backward(ctx, dsdf, dgeo, dgrads, dhess, dnormals):
        pos, table, grads, *params = ctx.saved_tensors
        if ctx.acc_grads is not None:
            dgrads = ctx.acc_grads.total(dgrads)
        M, G = ctx.M, ctx.G
        dev = pos.device
        # dout: centre rows all 257 columns, tap rows only the sdf column (everything read is written here)
        dout = _alloc(5 * M, G + 1, dev)
        c = lambda t: None if t is None else (t if t.stride(-1) == 1 else t.contiguous())
        dsdf, dgeo = c(dsdf), c(dgeo)
        # taps_combine_bwd reads these [M, 3] with a fixed row stride of 3: dense copies unless already dense
        cc = lambda t: None if t is None else t.contiguous()
        _lib.call("mms_taps_combine_bwd", grads.data_ptr(), _p(cc(dgrads)), _p(cc(dhess)), _p(cc(dnormals)), M,
                  ctx.four_delta, ctx.delta_sq, dout.data_ptr(), dout.stride(0), _p(dsdf),
                  0 if dsdf is None else dsdf.stride(0), _p(dgeo), 0 if dgeo is None else dgeo.stride(0), G, _s())
        need_table = ctx.needs_input_grad[1]
        need_pos = ctx.needs_input_grad[0]
        if ctx.chain is not None:
            dX = ctx.chain.backward(dout)
            pgrads = [None] * len(params)
        else:
            dX, pgrads = _sdf_mlp_unfused_bwd(ctx, dout, params, dev)
        X = ctx.X
        K0 = X.stride(0)
        dtable = grad_target(ctx.table) if need_table else None
        dP = _zeroed_views([(5 * M, 3)], dev)[0] if need_pos else None
        dpos = acc_or_zeroed(ctx.acc_pos, (M, 3), dev, need_pos)
        grid_bwd(ctx.grid, X, K0, 5 * M, table, ctx.active, dX, 39, dtable, dP, group=5)
        _grad_ready(ctx.table_p, dtable)
        if need_pos:
            _lib.call("mms_geo_input_bwd", X.data_ptr(), K0, dX.data_ptr(), dX.stride(0), dP.data_ptr(), 3, M, 4, 6,
                      dpos.data_ptr(), 3, _s())
        ctx.run = ctx.H = ctx.W3 = ctx.X = ctx.table = ctx.chain = None
        return (acc_ret(ctx.acc_pos, dpos), None, None, None, None, *pgrads)


def _sdf_mlp_unfused(ctx, X, M, params, dev):
    """fp32 parity mode: hidden layers over all 5M rows; the output layer (257 wide: sdf + geo feature) only
    needs the sdf column on the 4M tap rows (surface_model.py:137-153 uses the taps' sdf alone)."""
    run = MLPRun(params[:-3], SDF_ACTS[:-1], PRECISION["sdf"])
    H = run.forward(X, keep=True)
    g3, v3, b3 = params[-3:]
    N3, K3 = v3.shape
    W3, n3 = normed_weight(g3, v3)
    out = _alloc(5 * M, N3, dev)
    prec = PRECISION["sdf"]
    gemm(NT, M, N3, K3, H, H.stride(0), W3, W3.stride(0), out, out.stride(0), bias=b3, prec=prec)
    gemm(NT, 4 * M, 1, K3, H[M:], H.stride(0), W3, W3.stride(0), out[M:], out.stride(0), bias=b3, prec=prec)
    ctx.run, ctx.H, ctx.W3, ctx.n3, ctx.prec = run, H, W3, n3, prec
    return out


def _sdf_mlp_unfused_bwd(ctx, dout, params, dev):
    M = ctx.M
    # output layer: centre rows (257 columns) and tap rows (sdf column) as two GEMM pairs
    H, W3, prec = ctx.H, ctx.W3, ctx.prec
    g3, v3, b3 = params[-3:]
    N3, K3 = v3.shape
    gt, vt, bt = grad_target(g3), grad_target(v3), grad_target(b3)
    if gt is not None or vt is not None or bt is not None:
        dW3 = _dw_views([v3], dev)[0]
        db3 = bt if bt is not None else torch.zeros(N3, device=dev)
        def wg(dout=dout, H=H, dW3=dW3, db3=db3):
            gemm(TN, N3, K3, M, dout, dout.stride(0), H, H.stride(0), dW3, K3, accumulate=True,
                 splits=_splits_for(M, 6, prec), prec=prec, colsum=db3)
            gemm(TN, 1, K3, 4 * M, dout[M:], dout.stride(0), H[M:], H.stride(0), dW3, K3, accumulate=True,
                 splits=_splits_for(4 * M, 2, prec), prec=prec, colsum=db3)
        _wgrad(wg)
        _wn_bwd(g3.reshape(-1), v3, ctx.n3, dW3, gt.reshape(-1) if gt is not None else
                        torch.zeros(N3, device=dev), vt if vt is not None else torch.zeros(N3, K3, device=dev))
    # dZ of the last hidden layer = (dout W3) * softplus'(Z) -- the activation gradient fused as aux
    run = ctx.run
    pa, pbeta, pthr = SDF_ACTS[-2]
    Zl = run.Zs[-1]
    dZ = _alloc(5 * M, K3, dev)
    gemm(NN, M, K3, N3, dout, dout.stride(0), W3, W3.stride(0), dZ, dZ.stride(0), aux=Zl, ldaux=Zl.stride(0),
         dact=pa, beta=pbeta, thr=pthr, prec=prec)
    gemm(NN, 4 * M, K3, 1, dout[M:], dout.stride(0), W3, W3.stride(0), dZ[M:], dZ.stride(0), aux=Zl[M:],
         ldaux=Zl.stride(0), dact=pa, beta=pbeta, thr=pthr, prec=prec)
    dX, pgrads = run.backward(dZ, need_dx=True, pre_activated=True)
    return dX, list(pgrads) + [None, None, None]


# the NeuS sampler's inference panels straight from the spacing bins (mms_sdf_panel_rays_fwd); MMS_FUSED_SAMPLER=0:
# the sample positions first (mms_samples_fwd), then the panel
FUSED_SAMPLER = FUSED_PANEL and os.environ.get("MMS_FUSED_SAMPLER", "1") != "0"


def sdf_only(pos: torch.Tensor, table, grid: GridCfg, active: int, params, rays=None) -> torch.Tensor:
    """Inference SDF (SurfaceModel.get_sdf, surface_model.py:213-226; evaluated under no_grad by the sampler).
    ``rays`` = (bins [R, nb], nears, fars, origins [R, 3], dirs [R, 3]) instead of ``pos``: the start positions of
    the bins' samples (sample_start_positions), formed inside the panel launch."""
    if rays is not None:
        bins, n, f, o, d = rays
        R, nb = bins.shape
        M = R * (nb - 1)
        dev = bins.device
        X = _alloc(M, 3 + 36 + grid.out_dim, dev)
        _lib.call("mms_sdf_panel_rays_fwd", bins.data_ptr(), bins.stride(0), nb, n.data_ptr(), f.data_ptr(),
                  o.data_ptr(), d.data_ptr(), R, 6, table.data_ptr(), grid.L, grid.log2T, grid.F, grid.interp,
                  grid.scales_ptr, grid.radius, active, X.data_ptr(), X.stride(0), _s())
    else:
        M = pos.shape[0]
        dev = pos.device
        X = _alloc(M, 3 + 36 + grid.out_dim, dev)
        sdf_panel(pos, pos.stride(0), M, 0, 0.0, grid, table, active, X)
    if PRECISION["sdf"] != 0:
        # fused chain, no hidden-layer stores, only the sdf column of the output layer (rows_full = 0), written as
        # the dense [M] vector the sampler kernel reads
        return ChainRun(params, SDF_ACTS, PRECISION["sdf"], PRECISION["sdf_chain"]).forward(X, keep=False, rows_full=0,
                                                                                         dense_col0=True)
    # only the sdf column of the last layer is needed
    last = list(params[-3:])
    g, v, b = last
    p2 = list(params[:-3]) + [g[:1], v[:1].contiguous(), b[:1]]
    run = MLPRun(p2, SDF_ACTS, PRECISION["sdf"])
    out = run.forward(X, keep=False)
    return out[:, 0]


def _chain_shape(params, acts, prec: int = 2) -> bool:
    """True when the fused chain kernel serves this MLP (mms_mlp_chain's dispatch table): the SDF (71-256-256-257,
    Softplus, Softplus, none) and radiance (317-256-256-256, ReLU x 3) chains, the background NeRF's 4-layer ReLU
    MLPs (base 39-256-256-256-256, head 283-256-256-256-128 / -256) and the plain heads 256-64-64-C."""
    dims = [params[1].shape[1]] + [params[3 * l + 1].shape[0] for l in range(len(params) // 3)]
    a = tuple(x[0] for x in acts)
    if len(params) == 9:
        if (dims == [71, 256, 256, 257] and a == (2, 2, 0)) or (dims == [317, 256, 256, 256] and a == (1, 1, 1)):
            return True
        # the modality heads 256-64-64-C, C <= 32: plain (Sigmoid out) and polarization (Stokes, no out activation)
        return prec in (1, 2, 4, 5) and dims[:3] == [256, 64, 64] and dims[3] <= 32 and a in ((1, 1, 3), (1, 1, 0))
    if len(params) == 12 and prec in (1, 2, 4, 5) and a == (1, 1, 1, 1):
        return dims in ([39, 256, 256, 256, 256], [283, 256, 256, 256, 128], [283, 256, 256, 256, 256])
    return False


def mlp_runner(params, acts, prec: int):
    """The MLP engine for a weight-normed MLP: the fused 3-layer chain kernel in the bf16 modes where its shape is
    served, the narrow-layer kernels for a single layer of <= 16 outputs, else the per-layer GEMM engine (every shape,
    every precision)."""
    if prec != 0 and _chain_shape(params, acts, prec):
        return ChainRun(params, acts, prec)
    if prec == 5:
        prec = 2        # fp16 forwards are a fused-chain mode: other shapes keep split-bf16x3
    if SmallRun.serves(params, acts, prec):
        return SmallRun(params, acts, prec)
    return MLPRun(params, acts, prec)


def _run_forward(run, X, keep: bool):
    return run.forward(X, keep=keep)


def _run_backward(run, dy):
    """dX of an MLP runner; parameter gradients are accumulated in place (grad_target)."""
    if isinstance(run, ChainRun):
        return run.backward(dy if dy.stride(1) == 1 and dy.stride(0) % 4 == 0 else _copy_aligned(dy))
    dx, _ = run.backward(dy.contiguous(), need_dx=True)
    return dx


class SDFFieldFunction(torch.autograd.Function):
    """SDFField.forward (surface_field.py:99-116) for the grid methods: PE(x) (encodings.py:161-182, 6 frequencies,
    input included) -> FeatureGridAndMLP (feature_structures.py:153-169) -> (sdf [M,1], geo [M,G]).  No taps: the
    plain field evaluation the reference's SDFField / single_output perform; autograd to x, the table and the MLP."""

    @staticmethod
    def forward(ctx, pos, table, grid: GridCfg, active: int, *params):
        ctx.set_materialize_grads(False)   # unused outputs' gradients arrive as None (no zero fills)
        M = pos.shape[0]
        dev = pos.device
        pos = pos.contiguous()
        K0 = 3 + 36 + grid.out_dim
        X = _alloc(M, K0, dev)
        sdf_panel(pos, 3, M, 0, 0.0, grid, table, active, X)
        run = mlp_runner(params, SDF_ACTS, PRECISION["sdf"])
        out = _run_forward(run, X, keep=True)
        ctx.run, ctx.X, ctx.grid, ctx.active, ctx.table = run, X, grid, active, table
        ctx.save_for_backward(pos, table)
        G = out.shape[1] - 1
        return out[:, :1].contiguous(), out[:, 1:].contiguous() if G > 0 else out[:, :0]

    @staticmethod
    def backward(ctx, dsdf, dgeo):
        pos, table = ctx.saved_tensors
        M = pos.shape[0]
        dev = pos.device
        G = dgeo.shape[1] if dgeo is not None else ctx.run.params[-2].shape[0] - 1
        dout = _alloc(M, G + 1, dev)
        dout[:, :1] = dsdf if dsdf is not None else 0.0
        dout[:, 1:] = dgeo if dgeo is not None else 0.0
        dX = _run_backward(ctx.run, dout)
        X = ctx.X
        need_pos = ctx.needs_input_grad[0]
        dP, dpos = _zeroed_views([(M, 3), (M, 3)] if need_pos else [None, None], dev)
        dtable = grad_target(ctx.table) if ctx.needs_input_grad[1] else None
        grid_bwd(ctx.grid, X, X.stride(0), M, table, ctx.active, dX, 39, dtable, dP)
        if need_pos:
            _lib.call("mms_geo_input_bwd", X.data_ptr(), X.stride(0), dX.data_ptr(), dX.stride(0), dP.data_ptr(), 3, M,
                      0, 6, dpos.data_ptr(), 3, _s())
        n = len(ctx.run.params)
        ctx.run = ctx.X = ctx.table = None
        return (dpos, None, None, None, *([None] * n))


class FeatureGridMLPFunction(torch.autograd.Function):
    """FeatureGridAndMLP.forward (feature_structures.py:153-169) for any input width: the MLP panel is
    [input (x = columns 0..2, then the auxiliary columns), grid(x)], the grid written straight into the panel by the
    hash kernel; MLP on the chain kernel or the GEMM engine (mlp_runner).  Returns the MLP output (and, with
    return_features, the grid features)."""

    @staticmethod
    def forward(ctx, inp, table, grid: GridCfg, active: int, acts, prec: int, *params):
        ctx.set_materialize_grads(False)   # unused outputs' gradients arrive as None (no zero fills)
        M, K_in = inp.shape
        dev = inp.device
        X = _alloc(M, K_in + grid.out_dim, dev)
        X[:, :K_in] = inp
        grid_fwd(grid, X, X.stride(0), M, table, active, X, K_in)
        run = mlp_runner(params, acts, prec)
        out = _run_forward(run, X, keep=True)
        ctx.run, ctx.X, ctx.grid, ctx.active, ctx.table, ctx.K_in = run, X, grid, active, table, K_in
        ctx.save_for_backward(table)
        feats = X[:, K_in:].clone()
        ctx.mark_non_differentiable(feats)
        return out, feats

    @staticmethod
    def backward(ctx, dout, dfeats):
        (table,) = ctx.saved_tensors
        X, K_in = ctx.X, ctx.K_in
        M = X.shape[0]
        dev = X.device
        dX = _run_backward(ctx.run, dout)
        need_in = ctx.needs_input_grad[0]
        dP = torch.zeros(M, 3, device=dev) if need_in else None
        dtable = grad_target(ctx.table) if ctx.needs_input_grad[1] else None
        grid_bwd(ctx.grid, X, X.stride(0), M, table, ctx.active, dX, K_in, dtable, dP)
        dinp = None
        if need_in:
            dinp = dX[:, :K_in].clone()
            dinp[:, :3] += dP
        n = len(ctx.run.params)
        ctx.run = ctx.X = ctx.table = None
        return (dinp, None, None, None, None, None, *([None] * n))


# ------------------------------------------------------------------------------------------------
# radiance field
# ------------------------------------------------------------------------------------------------
RAD_ACTS = ((1, 1.0, 20.0), (1, 1.0, 20.0), (1, 1.0, 20.0))


class RadianceFunction(torch.autograd.Function):
    """(pos [M,3], dirs [R,3], normals [M,3] (detached), geo [M,G], table) -> feature [M,256]."""

    @staticmethod
    def forward(ctx, pos, dirs, normals, geo, table, grid: GridCfg, active: int, S: int, *params):
        ctx.acc_pos, ctx.acc_dirs = acc_of(pos), acc_of(dirs)
        M = pos.shape[0]
        G = geo.shape[1]
        dev = pos.device
        K0 = 3 + 25 + G + 1 + grid.out_dim
        X = _alloc(M, K0, dev)
        pos = pos.contiguous()
        dirs = dirs.contiguous()
        normals = normals.contiguous()
        geo = geo if geo.stride(1) == 1 else geo.contiguous()    # row-strided views are read in place
        if FUSED_RAD_PANEL:
            g = grid
            _lib.call("mms_rad_panel_fwd", pos.data_ptr(), 3, dirs.data_ptr(), normals.data_ptr(), geo.data_ptr(),
                      geo.stride(0), M, S, G, table.data_ptr(), g.L, g.log2T, g.F, g.interp, g.scales_ptr, g.radius,
                      active, X.data_ptr(), X.stride(0), _s())
        else:
            _lib.call("mms_rad_input_fwd", pos.data_ptr(), 3, dirs.data_ptr(), normals.data_ptr(), geo.data_ptr(),
                      geo.stride(0), M, S, G, X.data_ptr(), X.stride(0), _s())
            grid_fwd(grid, X, X.stride(0), M, table, active, X, 29 + G)
        prec = PRECISION["radiance"]
        run = ChainRun(params, RAD_ACTS, prec) if prec != 0 else MLPRun(params, RAD_ACTS, prec)
        feat = run.forward(X, keep=True)
        ctx.run, ctx.X, ctx.grid, ctx.active, ctx.S, ctx.G = run, X, grid, active, S, G
        ctx.table = ctx.table_p = table
        if ctx.needs_input_grad[4]:
            _grad_use(table)
        ctx.save_for_backward(pos, dirs, normals, table, *params)
        return feat

    @staticmethod
    def backward(ctx, dfeat):
        pos, dirs, normals, table, *params = ctx.saved_tensors
        M, S, G = pos.shape[0], ctx.S, ctx.G
        R = M // S
        dev = pos.device
        if isinstance(ctx.run, ChainRun):
            dX = ctx.run.backward(dfeat.contiguous())
            pgrads = [None] * len(params)
        else:
            dX, pgrads = ctx.run.backward(dfeat.contiguous(), need_dx=True)
        X = ctx.X
        K0 = X.stride(0)
        dtable = grad_target(ctx.table) if ctx.needs_input_grad[4] else None
        need_pos = ctx.needs_input_grad[0]
        dP = _zeroed_views([(M, 3)], dev)[0] if need_pos else None
        dpos = acc_or_zeroed(ctx.acc_pos, (M, 3), dev, need_pos)
        ddirs = acc_or_zeroed(ctx.acc_dirs, (R, 3), dev, ctx.needs_input_grad[1])
        grid_bwd(ctx.grid, X, K0, M, table, ctx.active, dX, 29 + G, dtable, dP)
        _grad_ready(ctx.table_p, dtable)   # the radiance table's last contribution: its all-reduce overlaps the rest
        # d geo = the panel gradient's geo columns, handed on as a view (no copy)
        dgeo = dX[:, 28:28 + G] if ctx.needs_input_grad[3] else None
        _lib.call("mms_rad_input_bwd", dX.data_ptr(), dX.stride(0), _p(dP), 3, dirs.data_ptr(), normals.data_ptr(), R,
                  S, G, _p(dpos), 3, None, G, _p(ddirs), _s())
        ctx.run = None
        ctx.X = None
        ctx.table = None
        return (acc_ret(ctx.acc_pos, dpos), acc_ret(ctx.acc_dirs, ddirs), None, dgeo, None, None, None, None, *pgrads)


class RadInputFunction(torch.autograd.Function):
    """The radiance MLP input [x, SH4(d), geo, n.v] (radiance_model.py:114-132) without grid columns, for the mlp
    methods' RadianceField(MLP): mms_rad_input_fwd / _bwd (normals detached, base_model.py:129)."""

    @staticmethod
    def forward(ctx, pos, dirs, normals, geo, S: int):
        M, G = geo.shape
        dev = pos.device
        X = _alloc(M, 3 + 25 + G + 1, dev)
        pos, dirs, normals = pos.contiguous(), dirs.contiguous(), normals.contiguous()
        geo = geo if geo.stride(1) == 1 else geo.contiguous()
        _lib.call("mms_rad_input_fwd", pos.data_ptr(), 3, dirs.data_ptr(), normals.data_ptr(), geo.data_ptr(),
                  geo.stride(0), M, S, G, X.data_ptr(), X.stride(0), _s())
        ctx.save_for_backward(dirs, normals)
        ctx.S, ctx.G, ctx.M = S, G, M
        return X

    @staticmethod
    def backward(ctx, dX):
        dirs, normals = ctx.saved_tensors
        M, S, G = ctx.M, ctx.S, ctx.G
        dev = dX.device
        dX = dX if dX.stride(1) == 1 else dX.contiguous()
        dpos, ddirs = _zeroed_views([(M, 3) if ctx.needs_input_grad[0] else None,
                                     (M // S, 3) if ctx.needs_input_grad[1] else None], dev)
        dgeo = dX[:, 28:28 + G] if ctx.needs_input_grad[3] else None      # a view of the panel gradient
        _lib.call("mms_rad_input_bwd", dX.data_ptr(), dX.stride(0), None, 3, dirs.data_ptr(), normals.data_ptr(), M // S,
                  S, G, _p(dpos), 3, None, G, _p(ddirs), _s())
        return dpos, ddirs, None, dgeo, None


# ------------------------------------------------------------------------------------------------
# plain MLP (heads)
# ------------------------------------------------------------------------------------------------
class MLPFunction(torch.autograd.Function):
    """A plain weight-normed MLP (modality heads) on the GEMM engine; ``key`` names its PRECISION entry."""

    @staticmethod
    def forward(ctx, x, acts, key, *params):
        run = mlp_runner(params, acts, PRECISION[key])
        # grad mode is off inside Function.forward: decide from what the graph will need
        x = x if (x.stride(-1) == 1 and x.stride(0) % 4 == 0 and x.data_ptr() % 16 == 0) else _copy_aligned(x)
        y = _run_forward(run, x, keep=any(ctx.needs_input_grad))
        ctx.run = run
        ctx.save_for_backward(*params)
        return y

    @staticmethod
    def backward(ctx, dy):
        if isinstance(ctx.run, ChainRun):
            dx = _run_backward(ctx.run, dy)
            grads = [None] * len(ctx.run.params)
        else:
            dx, grads = ctx.run.backward(dy.contiguous(), need_dx=ctx.needs_input_grad[0])
        ctx.run = None
        return (dx, None, None, *grads)


# ------------------------------------------------------------------------------------------------
# background NeRF field: contraction + PE -> base MLP -> density head ; [feat, PE(d)] -> head MLP
# ------------------------------------------------------------------------------------------------
BG_BASE_ACTS = ((1, 1.0, 20.0),) * 4      # ReLU hidden + ReLU out (NeRF MLP and the config-5 grid MLP alike)
BG_DENS_ACTS = ((2, 1.0, 20.0),)
BG_HEAD_ACTS = ((1, 1.0, 20.0),) * 4


class BackgroundFunction(torch.autograd.Function):
    """pos [M,3] (raw sample starts), dirs [R,3] -> density [M,1], feature [M,F].  ``grid``/``table``: the config-5
    background base field is a FeatureGridAndMLP (hash grid r = 2 on the contracted x, method_configs.py:428-444);
    None for the NeRF MLP base field."""

    @staticmethod
    def forward(ctx, pos, dirs, table, S: int, nb: int, nd: int, grid: Optional[GridCfg], active: int, *params):
        ctx.set_materialize_grads(False)   # unused outputs' gradients arrive as None (no zero fills)
        ctx.acc_dirs = acc_of(dirs)
        M = pos.shape[0]
        dev = pos.device
        base_p, dens_p, head_p = params[:3 * nb], params[3 * nb:3 * (nb + nd)], params[3 * (nb + nd):]
        # base input panel [contracted x, PE tail (36)] (+ the grid features of the contracted x for the config-5
        # FeatureGridAndMLP base field, feature_structures.py:153-169, written straight into columns 39..70)
        X = _alloc(M, 39 + (grid.out_dim if grid is not None else 0), dev)
        Fb = base_p[-2].shape[0]
        H = _alloc(M, Fb + 27, dev)
        pos = pos.contiguous()
        dirs = dirs.contiguous()
        _lib.call("mms_bg_input_fwd", pos.data_ptr(), M, dirs.data_ptr(), S, X.data_ptr(), X.stride(0), H.data_ptr(),
                  H.stride(0), Fb, _s())
        if grid is not None:
            grid_fwd(grid, X, X.stride(0), M, table, active, X, 39)
        ctx.grid, ctx.active, ctx.table = grid, active, table
        if grid is not None and ctx.needs_input_grad[2]:
            _grad_use(table)
        # base and head MLPs: 4-layer chain kernels in bf16 (mlp_runner), per-layer GEMMs otherwise
        base = mlp_runner(base_p, BG_BASE_ACTS[:nb], PRECISION["background"])
        base.forward(X, keep=True, last_out=H[:, :Fb])  # writes cols [0, Fb) of the head panel
        dens = mlp_runner(dens_p, BG_DENS_ACTS, PRECISION["background"])
        density = _mlp_strided(dens, H, Fb)             # density head reads the base features in place
        head = mlp_runner(head_p, BG_HEAD_ACTS[:len(head_p) // 3], PRECISION["background"])
        feat = head.forward(H, keep=True)
        ctx.base, ctx.dens, ctx.head, ctx.X, ctx.H = base, dens, head, X, H
        ctx.S, ctx.nb, ctx.nd, ctx.Fb = S, nb, nd, Fb
        ctx.save_for_backward(pos, dirs, *params)
        return density, feat

    @staticmethod
    def backward(ctx, ddensity, dfeat):
        pos, dirs, *params = ctx.saved_tensors
        M, S, Fb = pos.shape[0], ctx.S, ctx.Fb
        R = M // S
        dev = pos.device
        if dfeat is not None:
            dH = _run_backward(ctx.head, dfeat)                                      # [M, Fb+27]
        else:
            # only the density reached the loss: the head panel's gradient is the density head's alone
            dH = _zeroed_views([(M, ctx.H.stride(0))], dev)[0][:, :Fb + 27]
        if ddensity is None:
            ddensity = torch.zeros(M, 1, device=dev)
        # the density head's input gradient accumulates straight into the head panel's base columns
        _mlp_strided_bwd(ctx.dens, ddensity.contiguous(), ctx.H, Fb, dx_into=dH[:, :Fb])
        dbase_out = dH[:, :Fb]
        dX = _run_backward(ctx.base, dbase_out)
        if ctx.grid is not None:
            # grid features of the contracted x: table gradients, and d(contracted x) into the panel's x columns
            dtable = grad_target(ctx.table) if ctx.needs_input_grad[2] else None
            dP = torch.zeros(M, 3, device=dev)
            grid_bwd(ctx.grid, ctx.X, ctx.X.stride(0), M, ctx.table, ctx.active, dX, 39, dtable, dP)
            _grad_ready(ctx.table, dtable)
            dX[:, :3] += dP
        dpos = torch.empty(M, 3, device=dev) if ctx.needs_input_grad[0] else None
        ddirs = acc_or_zeroed(ctx.acc_dirs, (R, 3), dev, ctx.needs_input_grad[1])
        _lib.call("mms_bg_input_bwd", pos.data_ptr(), ctx.X.data_ptr(), ctx.X.stride(0), dX.data_ptr(), dX.stride(0),
                  dirs.data_ptr(), dH.data_ptr(), dH.stride(0), Fb, R, S, _p(dpos), _p(ddirs), _s())
        ctx.base = ctx.dens = ctx.head = ctx.X = ctx.H = ctx.table = None
        return (dpos, acc_ret(ctx.acc_dirs, ddirs), None, None, None, None, None, None, *([None] * len(params)))


def _mlp_strided(run, H: torch.Tensor, Fb: int) -> torch.Tensor:
    """Run a 1-layer MLP on the first Fb columns of panel H (row stride H.stride(0))."""
    if isinstance(run, SmallRun):
        return run.forward(H[:, :Fb], keep=True)
    g, v, b = run.params
    N, K = v.shape
    M = H.shape[0]
    dev = H.device
    W, nrm = normed_weight(g, v)
    act, beta, thr = run.acts[0]
    Y = torch.empty(M, N, device=dev)
    Z = _alloc(M, N, dev)
    gemm(NT, M, N, K, H, H.stride(0), W, W.stride(0), Y, Y.stride(0), bias=b, Z=Z, ldz=Z.stride(0), act=act,
         beta=beta, thr=thr, prec=run.fprec)
    run.Ws, run.norms, run.Zs, run.Ys = [W], [nrm], [Z], [Y]
    return Y


def _mlp_strided_bwd(run, dy: torch.Tensor, H: torch.Tensor, Fb: int, dx_into: Optional[torch.Tensor] = None):
    """Backward of _mlp_strided; the input gradient is returned, or (dx_into) added into that [M, K] view."""
    if isinstance(run, SmallRun):
        dx, _ = run.backward(dy, need_dx=True, dx_out=dx_into, accumulate=dx_into is not None)
        return dx, [None, None, None]
    g, v, b = run.params
    N, K = v.shape
    M = H.shape[0]
    dev = H.device
    act, beta, thr = run.acts[0]
    dZ = _alloc(M, N, dev)
    act_bwd(dy, run.Zs[0], act, beta, thr, dZ)
    gt, vt, bt = grad_target(g), grad_target(v), grad_target(b)
    if gt is not None or vt is not None or bt is not None:
        dW = _dw_views([v], dev)[0]
        db = bt if bt is not None else torch.zeros(N, device=dev)
        _wgrad(lambda dZ=dZ, H=H, dW=dW, db=db: gemm(
            TN, N, K, M, dZ, dZ.stride(0), H, H.stride(0), dW, K, accumulate=True,
            splits=_splits_for(M, 1, run.bprec), prec=run.bprec, colsum=db))
        dg = gt.reshape(-1) if gt is not None else torch.zeros(N, device=dev)
        dv = vt if vt is not None else torch.zeros(N, K, device=dev)
        _wn_bwd(g.reshape(-1), v, run.norms[0], dW, dg, dv)
    if dx_into is not None:
        gemm(NN, M, K, N, dZ, dZ.stride(0), run.Ws[0], run.Ws[0].stride(0), dx_into, dx_into.stride(0),
             accumulate=True, prec=run.bprec)
        return dx_into, [None, None, None]
    dxin = _alloc(M, K, dev)
    gemm(NN, M, K, N, dZ, dZ.stride(0), run.Ws[0], run.Ws[0].stride(0), dxin, dxin.stride(0), prec=run.bprec)
    return dxin, [None, None, None]


# ------------------------------------------------------------------------------------------------
# volume rendering
# ------------------------------------------------------------------------------------------------
class NeusWeightsFunction(torch.autograd.Function):
    """(sdf [R*S,1], grads [R*S,3], dirs [R,3], deltas [R*S], s_param [1]) -> weights [R, S]."""

    @staticmethod
    def forward(ctx, sdf, grads, dirs, deltas, s_param, cos_anneal: float, S: int):
        ctx.acc_grads, ctx.acc_dirs = acc_of(grads), acc_of(dirs)
        ctx.s_leaf = s_param.is_leaf
        M = sdf.shape[0]
        R = M // S
        dev = sdf.device
        if sdf.dim() != 2 or sdf.shape[1] != 1:
            sdf = sdf.reshape(M, 1)
        lds = sdf.stride(0)                 # sdf may be a column view of the SDF MLP output
        grads, dirs, deltas = grads.contiguous(), dirs.contiguous(), deltas.contiguous()
        alpha = torch.empty(R, S, device=dev)
        w = torch.empty(R, S, device=dev)
        _lib.call("mms_neus_weights_fwd", sdf.data_ptr(), lds, grads.data_ptr(), dirs.data_ptr(), deltas.data_ptr(),
                  s_param.data_ptr(), float(cos_anneal), R, S, alpha.data_ptr(), w.data_ptr(), _s())
        ctx.save_for_backward(sdf, grads, dirs, deltas, s_param, alpha)
        ctx.cos_anneal, ctx.S = float(cos_anneal), S
        return w

    @staticmethod
    def backward(ctx, dw):
        sdf, grads, dirs, deltas, s_param, alpha = ctx.saved_tensors
        S = ctx.S
        R = sdf.shape[0] // S
        dev = sdf.device
        dsdf = torch.empty(sdf.shape[0], 1, device=dev)
        ddeltas = _zeroed_views([deltas.shape], dev)[0]
        # the variance parameter's gradient: atomics straight into its .grad (grad_target: no AccumulateGrad add)
        s_direct = ctx.s_leaf and s_param.requires_grad
        ds = grad_target(s_param) if s_direct else _zeroed_views([s_param.shape], dev)[0]
        dgrads = acc_or_zeroed(ctx.acc_grads, grads.shape, dev)
        ddirs = acc_or_zeroed(ctx.acc_dirs, dirs.shape, dev)
        _lib.call("mms_neus_weights_bwd", sdf.data_ptr(), sdf.stride(0), grads.data_ptr(), dirs.data_ptr(), deltas.data_ptr(),
                  s_param.data_ptr(), ctx.cos_anneal, R, S, alpha.data_ptr(), dw.contiguous().data_ptr(),
                  dsdf.data_ptr(), 1, dgrads.data_ptr(), ddirs.data_ptr(), ddeltas.data_ptr(), ds.data_ptr(), _s())
        return (dsdf, acc_ret(ctx.acc_grads, dgrads), acc_ret(ctx.acc_dirs, ddirs), ddeltas, None if s_direct else ds,
                None, None)


class DensityWeightsFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, density, deltas, S: int):
        M = density.shape[0]
        R = M // S
        density, deltas = density.contiguous(), deltas.contiguous()
        alpha = torch.empty(R, S, device=density.device)
        w = torch.empty(R, S, device=density.device)
        _lib.call("mms_density_weights_fwd", density.data_ptr(), 1, deltas.data_ptr(), R, S, alpha.data_ptr(),
                  w.data_ptr(), _s())
        ctx.save_for_backward(density, deltas, alpha)
        ctx.S = S
        return w

    @staticmethod
    def backward(ctx, dw):
        density, deltas, alpha = ctx.saved_tensors
        S = ctx.S
        R = density.shape[0] // S
        dden = torch.empty_like(density)
        ddel = _zeroed_views([tuple(deltas.shape)], deltas.device)[0]
        _lib.call("mms_density_weights_bwd", density.data_ptr(), 1, deltas.data_ptr(), R, S, alpha.data_ptr(),
                  dw.contiguous().data_ptr(), dden.data_ptr(), 1, ddel.data_ptr(), _s())
        return dden, ddel, None


class CompositeFunction(torch.autograd.Function):
    """weights [R,S], vals [R*S, C] -> out [N, C] = bg with hit rows idx[r] replaced by sum w c + bg (1 - sum w).

    With bg None the output has R rows (no scatter).  Renderer.render (renderers.py:94-106) semantics.
    """

    @staticmethod
    def forward(ctx, w, vals, bg, idx, S: int):
        R = w.shape[0]
        C = vals.shape[1]
        w, vals = w.contiguous(), vals.contiguous()
        if bg is not None:
            out = bg.detach().clone().contiguous()
            bgc = bg.contiguous()
        else:
            out = torch.empty(R, C, device=w.device)
            bgc = None
        _lib.call("mms_composite_fwd", w.data_ptr(), vals.data_ptr(), C, C, _p(bgc), R, S, _p(idx), out.shape[0],
                  None, out.data_ptr(), _s())
        ctx.save_for_backward(w, vals, bgc, idx)
        ctx.S = S
        ctx.has_bg = bg is not None
        return out

    @staticmethod
    def backward(ctx, dout):
        w, vals, bgc, idx = ctx.saved_tensors
        S = ctx.S
        R, C = w.shape[0], vals.shape[1]
        dout = dout.contiguous()
        dvals = torch.empty_like(vals) if ctx.needs_input_grad[1] else None
        dw = torch.empty_like(w)                 # every weight written by the kernel
        dbg = dout.clone() if ctx.has_bg else None
        _lib.call("mms_composite_bwd", w.data_ptr(), vals.data_ptr(), C, C, _p(bgc), R, S, _p(idx), dout.shape[0],
                  None, dout.data_ptr(), _p(dvals), C, dw.data_ptr(), _p(dbg), _s())
        return dw, dvals, dbg, None, None


# ------------------------------------------------------------------------------------------------
# samples, rays, collider
# ------------------------------------------------------------------------------------------------
class SamplesFunction(torch.autograd.Function):
    """bins [R, S+1] (detached) + nears/fars [R] + origins/dirs [R,3] -> positions [R*S,3], deltas [R*S],
    starts [R*S], ends [R*S]."""

    @staticmethod
    def forward(ctx, bins, nears, fars, origins, dirs, kind: int):
        ctx.set_materialize_grads(False)   # unused outputs' gradients arrive as None (no zero fills)
        ctx.acc_o, ctx.acc_d = acc_of(origins), acc_of(dirs)
        R, nb = bins.shape
        S = nb - 1
        dev = bins.device
        bins, nears, fars = bins.contiguous(), nears.contiguous(), fars.contiguous()
        origins, dirs = origins.contiguous(), dirs.contiguous()
        starts = torch.empty(R * S, device=dev)
        ends = torch.empty(R * S, device=dev)
        deltas = torch.empty(R * S, device=dev)
        pos = torch.empty(R * S, 3, device=dev)
        _lib.call("mms_samples_fwd", bins.data_ptr(), nb, nb, nears.data_ptr(), fars.data_ptr(), origins.data_ptr(),
                  dirs.data_ptr(), kind, R, starts.data_ptr(), ends.data_ptr(), deltas.data_ptr(), pos.data_ptr(),
                  _s())
        ctx.save_for_backward(bins, nears, fars, dirs)
        ctx.kind = kind
        ctx.mark_non_differentiable(ends)
        ctx.acc_pos = GradAcc(pos) if GRAD_ACC else None
        if ctx.acc_pos is not None:
            pos._mms_acc = ctx.acc_pos
        return pos, deltas, starts, ends

    @staticmethod
    def backward(ctx, dpos, ddeltas, dstarts, dends):
        bins, nears, fars, dirs = ctx.saved_tensors
        if ctx.acc_pos is not None:
            dpos = ctx.acc_pos.total(dpos)
        R, nb = bins.shape
        dn, df = _zeroed_views([nears.shape, fars.shape], bins.device)
        do = acc_or_zeroed(ctx.acc_o, (R, 3), bins.device)
        dd = acc_or_zeroed(ctx.acc_d, (R, 3), bins.device)
        _lib.call("mms_samples_bwd", bins.data_ptr(), nb, nb, nears.data_ptr(), fars.data_ptr(), dirs.data_ptr(),
                  ctx.kind, R, _p(None if dpos is None else dpos.contiguous()),
                  _p(None if ddeltas is None else ddeltas.contiguous()),
                  _p(None if dstarts is None else dstarts.contiguous()), dn.data_ptr(), df.data_ptr(), do.data_ptr(),
                  dd.data_ptr(), _s())
        return None, dn, df, acc_ret(ctx.acc_o, do), acc_ret(ctx.acc_d, dd), None


class HitGatherFunction(torch.autograd.Function):
    """The hit rays' origins, directions, up directions, nears and fars (base_model.py:88-93: the bundle indexed with
    the collider mask) in one gather launch; the backward scatters all five gradients in one launch."""

    @staticmethod
    def forward(ctx, idx, o, d, up, nears, fars):
        ctx.set_materialize_grads(False)   # unused outputs' gradients arrive as None (no zero fills)
        ctx.acc_in = (acc_of(o), acc_of(d), acc_of(up))
        R, N = idx.shape[0], o.shape[0]
        dev = o.device
        o, d, up, nears, fars = o.contiguous(), d.contiguous(), up.contiguous(), nears.contiguous(), fars.contiguous()
        oh, dh, uh = [torch.empty(R, 3, device=dev) for _ in range(3)]
        nh, fh = torch.empty(R, device=dev), torch.empty(R, device=dev)
        _lib.call("mms_hit_gather_fwd", idx.data_ptr(), R, o.data_ptr(), d.data_ptr(), up.data_ptr(), nears.data_ptr(),
                  fars.data_ptr(), oh.data_ptr(), dh.data_ptr(), uh.data_ptr(), nh.data_ptr(), fh.data_ptr(), _s())
        ctx.save_for_backward(idx)
        ctx.N = N
        ctx.acc_dh = GradAcc(dh) if GRAD_ACC else None
        if ctx.acc_dh is not None:
            dh._mms_acc = ctx.acc_dh
        return oh, dh, uh, nh, fh

    @staticmethod
    def backward(ctx, doh, ddh, duh, dnh, dfh):
        (idx,) = ctx.saved_tensors
        if ctx.acc_dh is not None:
            ddh = ctx.acc_dh.total(ddh)
        N = ctx.N
        gn, gf = _zeroed_views([(N,), (N,)], idx.device)
        ao, ad, au = ctx.acc_in
        go, gd, gu = [acc_or_zeroed(a, (N, 3), idx.device) for a in (ao, ad, au)]
        c = lambda t: None if t is None else t.contiguous()
        _lib.call("mms_hit_gather_bwd", idx.data_ptr(), idx.shape[0], _p(c(doh)), _p(c(ddh)), _p(c(duh)), _p(c(dnh)),
                  _p(c(dfh)), go.data_ptr(), gd.data_ptr(), gu.data_ptr(), gn.data_ptr(), gf.data_ptr(), _s())
        return None, acc_ret(ao, go), acc_ret(ad, gd), acc_ret(au, gu), gn, gf


class PoseExpFunction(torch.autograd.Function):
    """exp_map_SO3xR3 (lie_groups.py:28-63): pose deltas [B, 6] = (t, w) -> [R(w) | t] [B, 3, 4], one launch each
    way (the reference's ~20 tensor ops forward and their autograd backward)."""

    @staticmethod
    def forward(ctx, tangent):
        ctx.leaf = tangent.is_leaf and tangent.is_contiguous()
        tangent = tangent.contiguous()
        B = tangent.shape[0]
        mats = torch.empty(B, 3, 4, device=tangent.device)
        _lib.call("mms_pose_exp_fwd", tangent.data_ptr(), B, mats.data_ptr(), _s())
        ctx.save_for_backward(tangent)
        return mats

    @staticmethod
    def backward(ctx, dmats):
        (tangent,) = ctx.saved_tensors
        # a leaf parameter's gradient is accumulated in place (grad_target: no AccumulateGrad add per step)
        direct = ctx.leaf and tangent.requires_grad
        dt = grad_target(tangent) if direct else _zeroed_views([tuple(tangent.shape)], tangent.device)[0]
        _lib.call("mms_pose_exp_bwd", tangent.data_ptr(), dmats.contiguous().data_ptr(), tangent.shape[0],
                  dt.data_ptr(), _s())
        return None if direct else dt


class RaysFunction(torch.autograd.Function):
    """camera_opt_to_camera mats [C|1, 3, 4] -> origins, dirs, ups (+ pixel_area, directions_norm)."""

    @staticmethod
    def forward(ctx, mats, coords, cams, pixel_offset: float):
        ctx.set_materialize_grads(False)   # unused outputs' gradients arrive as None (no zero fills)
        N = coords.shape[0]
        dev = coords.device
        mats = mats.contiguous()
        o = torch.empty(N, 3, device=dev)
        d = torch.empty(N, 3, device=dev)
        u = torch.empty(N, 3, device=dev)
        a = torch.empty(N, 1, device=dev)
        dn = torch.empty(N, 1, device=dev)
        per_cam = 1 if mats.shape[0] > 1 else 0
        _lib.call("mms_raygen_fwd", coords.data_ptr(), N, cams.fx.data_ptr(), cams.fy.data_ptr(), cams.cx.data_ptr(),
                  cams.cy.data_ptr(), cams.c2w.data_ptr(), _p(cams.distortion), mats.data_ptr(), per_cam,
                  float(pixel_offset), o.data_ptr(), d.data_ptr(), u.data_ptr(), a.data_ptr(), dn.data_ptr(), _s())
        ctx.save_for_backward(mats, coords)
        ctx.cams, ctx.off, ctx.per_cam = cams, float(pixel_offset), per_cam
        ctx.mark_non_differentiable(a, dn)
        ctx.accs = None
        if GRAD_ACC and ctx.needs_input_grad[0]:
            ctx.accs = (GradAcc(o), GradAcc(d), GradAcc(u))
            o._mms_acc, d._mms_acc, u._mms_acc = ctx.accs
        return o, d, u, a, dn

    @staticmethod
    def backward(ctx, do, dd, du, da, ddn):
        mats, coords = ctx.saved_tensors
        if ctx.accs is not None:
            do, dd, du = [a.total(g) for a, g in zip(ctx.accs, (do, dd, du))]
        cams = ctx.cams
        N = coords.shape[0]
        dm = _zeroed_views([tuple(mats.shape)], mats.device)[0]
        _lib.call("mms_raygen_bwd", coords.data_ptr(), N, cams.fx.data_ptr(), cams.fy.data_ptr(), cams.cx.data_ptr(),
                  cams.cy.data_ptr(), cams.c2w.data_ptr(), _p(cams.distortion), mats.data_ptr(), ctx.per_cam,
                  ctx.off, _p(None if do is None else do.contiguous()), _p(None if dd is None else dd.contiguous()),
                  _p(None if du is None else du.contiguous()), dm.data_ptr(), _s())
        return dm, None, None, None


class ColliderFunction(torch.autograd.Function):
    """origins/dirs [N,3] -> nears, fars, bg_nears, bg_fars [N] (+ uint8 mask)."""

    @staticmethod
    def forward(ctx, origins, dirs, radius: float):
        ctx.set_materialize_grads(False)   # unused outputs' gradients arrive as None (no zero fills)
        ctx.acc_o, ctx.acc_d = acc_of(origins), acc_of(dirs)
        N = origins.shape[0]
        dev = origins.device
        origins, dirs = origins.contiguous(), dirs.contiguous()
        n = torch.empty(N, device=dev)
        f = torch.empty(N, device=dev)
        bn = torch.empty(N, device=dev)
        bf = torch.empty(N, device=dev)
        mask = torch.empty(N, dtype=torch.uint8, device=dev)
        _lib.call("mms_collider_fwd", origins.data_ptr(), dirs.data_ptr(), N, float(radius), n.data_ptr(),
                  f.data_ptr(), mask.data_ptr(), bn.data_ptr(), bf.data_ptr(), _s())
        ctx.save_for_backward(origins, dirs)
        ctx.radius = float(radius)
        ctx.mark_non_differentiable(mask)
        return n, f, bn, bf, mask

    @staticmethod
    def backward(ctx, dn, df, dbn, dbf, dmask):
        origins, dirs = ctx.saved_tensors
        N = origins.shape[0]
        do = acc_or_zeroed(ctx.acc_o, origins.shape, origins.device)
        dd = acc_or_zeroed(ctx.acc_d, dirs.shape, origins.device)
        c = lambda t: None if t is None else t.contiguous()
        _lib.call("mms_collider_bwd", origins.data_ptr(), dirs.data_ptr(), N, ctx.radius, _p(c(dn)), _p(c(df)),
                  _p(c(dbn)), _p(c(dbf)), do.data_ptr(), dd.data_ptr(), _s())
        return acc_ret(ctx.acc_o, do), acc_ret(ctx.acc_d, dd), None


def compact_padded(mask: torch.Tensor, cap: int):
    """Fixed-capacity compaction for static-shape (graph-captured) steps, no host read: (gather index [cap] -- rows
    past the hit count repeat the first hit ray --, scatter index [cap] -- N for those padding rows --, device hit
    count [1])."""
    N = mask.shape[0]
    idx = torch.empty(N, dtype=torch.int64, device=mask.device)
    sidx = torch.empty(cap, dtype=torch.int64, device=mask.device)
    cnt = torch.empty(1, dtype=torch.int64, device=mask.device)
    _lib.call("mms_compact_padded", mask.data_ptr(), N, cap, idx.data_ptr(), sidx.data_ptr(), cnt.data_ptr(), _s())
    return idx[:cap], sidx, cnt


def compact(mask: torch.Tensor) -> torch.Tensor:
    """Order-preserving indices of mask != 0 (int64); one device->host read of the count."""
    N = mask.shape[0]
    idx = torch.empty(N, dtype=torch.int64, device=mask.device)
    cnt = torch.empty(1, dtype=torch.int64, device=mask.device)
    _lib.call("mms_compact", mask.data_ptr(), N, idx.data_ptr(), cnt.data_ptr(), _s())
    return idx[: int(cnt.item())]


# ------------------------------------------------------------------------------------------------
# losses
# ------------------------------------------------------------------------------------------------
class L1LossFunction(torch.autograd.Function):
    """nn.L1Loss(mean) with optional SkipSaturation fill (losses.py:152-164)."""

    @staticmethod
    def forward(ctx, out, target, sat_thr: Optional[float]):
        N, C = target.shape
        out_c = out.contiguous()
        target = target.contiguous()
        loss = torch.zeros((), device=out.device)
        scratch = torch.empty(1, dtype=torch.int64, device=out.device) if sat_thr is not None else None
        thr = float(sat_thr) if sat_thr is not None else 0.0
        _lib.call("mms_l1_loss_fwd", out_c.data_ptr(), C, target.data_ptr(), N, C, thr, _p(scratch),
                  loss.data_ptr(), _s())
        ctx.save_for_backward(out_c, target, scratch)
        ctx.thr = thr
        return loss

    @staticmethod
    def backward(ctx, dl):
        out, target, scratch = ctx.saved_tensors
        N, C = target.shape
        dout = _zeroed_views([tuple(out.shape)], out.device)[0]
        _lib.call("mms_l1_loss_bwd", out.data_ptr(), C, target.data_ptr(), N, C, ctx.thr, _p(scratch),
                  dl.contiguous().data_ptr(), 1.0, dout.data_ptr(), C, _s())
        return dout, None, None


class GeoLossFunction(torch.autograd.Function):
    """Eikonal MSE(||g||, 1) and curvature L1(sum h, 0) over the concatenated modalities (losses.py:107-150)."""

    @staticmethod
    def forward(ctx, *tensors):
        ctx.set_materialize_grads(False)   # unused outputs' gradients arrive as None (no zero fills)
        n = len(tensors) // 2
        grads, hess = tensors[:n], tensors[n:]
        total = sum(g.shape[0] for g in grads)
        inv = 1.0 / float(total)
        eik, curv = torch.zeros(2, device=grads[0].device).unbind(0)   # outputs: not from the step arena
        for g, h in zip(grads, hess):
            _lib.call("mms_geo_loss_fwd", g.contiguous().data_ptr(), h.contiguous().data_ptr(), g.shape[0], inv,
                      eik.data_ptr(), curv.data_ptr(), _s())
        ctx.save_for_backward(*[t.contiguous() for t in tensors])
        ctx.inv, ctx.n = inv, n
        return eik, curv

    @staticmethod
    def backward(ctx, deik, dcurv):
        ts = ctx.saved_tensors
        n = ctx.n
        outs = []
        dg_list, dh_list = [], []
        for g, h in zip(ts[:n], ts[n:]):
            dg, dh = _zeroed_views([g.shape, h.shape], g.device)
            _lib.call("mms_geo_loss_bwd", g.data_ptr(), h.data_ptr(), g.shape[0], ctx.inv,
                      _p(None if deik is None else deik.contiguous()), 1.0,
                      _p(None if dcurv is None else dcurv.contiguous()), 1.0, dg.data_ptr(), dh.data_ptr(), _s())
            dg_list.append(dg)
            dh_list.append(dh)
        return (*dg_list, *dh_list)


class GeoLossMaskedFunction(torch.autograd.Function):
    """GeoLossFunction over fixed-capacity batches: modality m's rows >= counts[m] * S are padding and carry no loss,
    and the mean runs over the true rows (1 / total formed on the device from the hit counts)."""

    @staticmethod
    def forward(ctx, S: int, counts, *tensors):
        ctx.set_materialize_grads(False)   # unused outputs' gradients arrive as None (no zero fills)
        n = len(tensors) // 2
        grads, hess = tensors[:n], tensors[n:]
        dev = grads[0].device
        call = torch.cat([c.reshape(1) for c in counts]) if len(counts) > 1 else counts[0].reshape(1)
        eik, curv = torch.zeros(2, device=dev).unbind(0)   # outputs: not from the step arena
        ts = [t.contiguous() for t in tensors]
        for g, h, c in zip(ts[:n], ts[n:], counts):
            _lib.call("mms_geo_loss_fwd_masked", g.data_ptr(), h.data_ptr(), g.shape[0], S, c.data_ptr(),
                      call.data_ptr(), call.shape[0], eik.data_ptr(), curv.data_ptr(), _s())
        ctx.save_for_backward(call, *ts)
        ctx.counts, ctx.S, ctx.n = list(counts), S, n
        return eik, curv

    @staticmethod
    def backward(ctx, deik, dcurv):
        call, *ts = ctx.saved_tensors
        n, S = ctx.n, ctx.S
        dg_list, dh_list = [], []
        for g, h, c in zip(ts[:n], ts[n:], ctx.counts):
            dg, dh = _zeroed_views([g.shape, h.shape], g.device)
            _lib.call("mms_geo_loss_bwd_masked", g.data_ptr(), h.data_ptr(), g.shape[0], S, c.data_ptr(),
                      call.data_ptr(), call.shape[0], _p(None if deik is None else deik.contiguous()), 1.0,
                      _p(None if dcurv is None else dcurv.contiguous()), 1.0, dg.data_ptr(), dh.data_ptr(), _s())
            dg_list.append(dg)
            dh_list.append(dh)
        return (None, None, *dg_list, *dh_list)


class PolarizerFunction(torch.autograd.Function):
    """Stokes [M,3] -> 4 polarised intensities [M,4] (field_heads.py:90-106, polarizer.py:54-101)."""

    @staticmethod
    def forward(ctx, stokes, dirs, ups, S: int):
        M = stokes.shape[0]
        stokes, dirs, ups = stokes.contiguous(), dirs.contiguous(), ups.contiguous()
        out = torch.empty(M, 4, device=stokes.device)
        _lib.call("mms_polarizer_fwd", stokes.data_ptr(), dirs.data_ptr(), ups.data_ptr(), M, S, out.data_ptr(), _s())
        ctx.save_for_backward(stokes, dirs, ups)
        ctx.S = S
        return out

    @staticmethod
    def backward(ctx, dout):
        stokes, dirs, ups = ctx.saved_tensors
        S = ctx.S
        R = stokes.shape[0] // S
        ds = torch.empty_like(stokes)
        dd, du = _zeroed_views([dirs.shape, ups.shape], dirs.device)
        _lib.call("mms_polarizer_bwd", stokes.data_ptr(), dirs.data_ptr(), ups.data_ptr(), R, S,
                  dout.contiguous().data_ptr(), ds.data_ptr(), dd.data_ptr(), du.data_ptr(), _s())
        return ds, dd, du, None


# ------------------------------------------------------------------------------------------------
# modalities batched through the shared fields
# ------------------------------------------------------------------------------------------------
def compact_segments(mask: torch.Tensor, n_seg: int, N: int, cap: int):
    """Every modality's hit-ray compaction in one launch (mms_compact_segments): (gather index [n_seg cap] of global
    ray indices, index within the modality [n_seg cap] -- N for padding rows --, device hit counts [n_seg])."""
    dev = mask.device
    scratch = torch.empty(n_seg * N, dtype=torch.int64, device=dev)
    gidx = torch.empty(n_seg * cap, dtype=torch.int64, device=dev)
    sidx = torch.empty(n_seg * cap, dtype=torch.int64, device=dev)
    cnt = torch.empty(n_seg, dtype=torch.int64, device=dev)
    _lib.call("mms_compact_segments", mask.data_ptr(), n_seg, N, cap, scratch.data_ptr(), gidx.data_ptr(),
              sidx.data_ptr(), cnt.data_ptr(), _s())
    return gidx, sidx, cnt


class HeadSpec:
    """One modality head for HeadsCompositeFunction: 'plain' (MLP + out activation) or 'polarization' (MLP to Stokes +
    PolarizerFunction), its activations, its PRECISION key and its parameter count."""

    def __init__(self, kind: str, acts, key: str, n_params: int):
        self.kind, self.acts, self.key, self.n_params = kind, tuple(acts), key, int(n_params)


class HeadsCompositeFunction(torch.autograd.Function):
    """Modality heads + compositing of a batched ray set in ONE autograd node (RadianceModel heads
    radiance_model.py:143-149 / field_heads.py:71-106, Renderer.render renderers.py:75-136; the background's heads and
    sum background_model.py:101-109).  All modalities' rays share the field evaluation; each modality's rays are a
    contiguous segment of the batch, and only heads and compositing are per modality.

    ``jobs``: (head id, first ray, rays) -- a head evaluated on the feature rows of those rays (S rows per ray);
    ``items``: (job id, first ray within the job, rays, first ray in ``w``, scatter index or None, output rows) -- one
    composited output each, over the job's values, scattered into a copy of its background (``bgs[i]``, or None: a
    plain [rays, C] sum).  The backward writes the feature, weight and direction gradients of every segment into one
    buffer each (no per-modality zero fill + slice-add), and accumulates the head parameters' gradients in place."""

    @staticmethod
    def forward(ctx, feat, w, dirs, ups, S: int, heads, jobs, items, *rest):
        ctx.set_materialize_grads(False)
        ctx.acc_d, ctx.acc_u = acc_of(dirs), acc_of(ups)
        n_items = len(items)
        bgs, params = rest[:n_items], rest[n_items:]
        offs, o = [], 0
        for h in heads:
            offs.append(o)
            o += h.n_params
        keep = any(ctx.needs_input_grad)
        dirs_c, ups_c = dirs.contiguous(), ups.contiguous()
        runs, vals = [], []
        for h_id, r0, rays in jobs:
            h = heads[h_id]
            ps = params[offs[h_id]:offs[h_id] + h.n_params]
            x = feat[r0 * S:(r0 + rays) * S]
            run = mlp_runner(ps, h.acts, PRECISION[h.key])
            y = _run_forward(run, x, keep=keep)
            if h.kind == "polarization":
                st = y if y.is_contiguous() else y.contiguous()
                v = torch.empty(rays * S, 4, device=feat.device)
                _lib.call("mms_polarizer_fwd", st.data_ptr(), dirs_c[r0:].data_ptr(), ups_c[r0:].data_ptr(), rays * S,
                          S, v.data_ptr(), _s())
                y = st
            else:
                v = y
            runs.append((run, y))
            vals.append(v)
        w_c = w.contiguous()
        outs = []
        for (j, sub, rays, w0, sidx, rows, hit), bg in zip(items, bgs):
            v = vals[j]
            C = v.shape[1]
            hit = hit if bg is not None and sidx is not None else None
            if bg is not None:
                # with the hit mask the launch itself keeps the background on the rows no ray lands on
                out = torch.empty(bg.shape, device=bg.device) if hit is not None else bg.detach().clone().contiguous()
            else:
                out = torch.empty(rays if sidx is None else rows, C, device=feat.device)
            if _lib.SYNC_CALLS:
                _composite_extents("fwd", w_c[w0:], v[sub * S:], v.stride(0), C, bg, rays, S, sidx, out.shape[0],
                                   hit, None, None, 0, None, out)
            _lib.call("mms_composite_fwd", w_c[w0:].data_ptr(), v[sub * S:].data_ptr(), v.stride(0), C,
                      _p(None if bg is None else bg.contiguous()), rays, S, _p(sidx), out.shape[0], _p(hit),
                      out.data_ptr(), _s())
            outs.append(out)
        ctx.heads, ctx.jobs, ctx.items, ctx.S, ctx.runs, ctx.vals = heads, jobs, items, S, runs, vals
        ctx.n_params = len(params)
        ctx.save_for_backward(w_c, dirs_c, ups_c, *[None if b is None else b.contiguous() for b in bgs])
        ctx.feat_shape = tuple(feat.shape)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *douts):
        w, dirs, ups, *bgs = ctx.saved_tensors
        heads, jobs, items, S = ctx.heads, ctx.jobs, ctx.items, ctx.S
        dev = w.device
        R = w.shape[0]
        live = [d is not None for d in douts]
        # weight gradient: one buffer; written directly when the items with gradients partition its rows
        w_ranges = [(it[3], it[2]) for it, on in zip(items, live) if on]
        dw = torch.empty_like(w) if _partitions(w_ranges, R) else _zeroed_views([tuple(w.shape)], dev)[0]
        dw_direct = _partitions(w_ranges, R)
        dvals = [None] * len(jobs)
        dbgs = [None] * len(items)
        for i, ((j, sub, rays, w0, sidx, rows, hit), dout) in enumerate(zip(items, douts)):
            if dout is None:
                continue
            v = ctx.vals[j]
            C = v.shape[1]
            if dvals[j] is None:
                dvals[j] = _alloc(v.shape[0], C, dev) if _job_covered(j, items, live) else \
                    _zeroed_views([(v.shape[0], (C + 3) // 4 * 4)], dev)[0][:, :C]
            bg = bgs[i]
            hit = hit if bg is not None and sidx is not None else None
            dout = dout.contiguous()
            dbg = None if bg is None else (torch.empty(dout.shape, device=dev) if hit is not None else dout.clone())
            dwi = dw[w0:] if dw_direct else torch.empty(rays, S, device=dev)
            if _lib.SYNC_CALLS:
                _composite_extents("bwd", w[w0:], v[sub * S:], v.stride(0), C, bg, rays, S, sidx, dout.shape[0], hit,
                                   dout, dvals[j][sub * S:], dvals[j].stride(0), dwi, dbg)
            _lib.call("mms_composite_bwd", w[w0:].data_ptr(), v[sub * S:].data_ptr(), v.stride(0), C, _p(bg), rays, S,
                      _p(sidx), dout.shape[0], _p(hit), dout.data_ptr(), dvals[j][sub * S:].data_ptr(),
                      dvals[j].stride(0), dwi.data_ptr(), _p(dbg), _s())
            if not dw_direct:
                dw[w0:w0 + rays] += dwi
            dbgs[i] = dbg
        need_feat = ctx.needs_input_grad[0]
        f_ranges = [(jobs[j][1], jobs[j][2]) for j in range(len(jobs)) if dvals[j] is not None]
        f_direct = _partitions(f_ranges, ctx.feat_shape[0] // S)
        dfeat = None
        if need_feat:
            dfeat = torch.empty(ctx.feat_shape, device=dev) if f_direct else \
                _zeroed_views([ctx.feat_shape], dev)[0]
        need_dir = ctx.needs_input_grad[2] or ctx.needs_input_grad[3]
        ddirs = dups = None
        if need_dir and any(heads[jobs[j][0]].kind == "polarization" and dvals[j] is not None
                            for j in range(len(jobs))):
            ddirs = acc_or_zeroed(ctx.acc_d, dirs.shape, dev)
            dups = acc_or_zeroed(ctx.acc_u, ups.shape, dev)
        for j, (h_id, r0, rays) in enumerate(jobs):
            if dvals[j] is None:
                continue
            run, y = ctx.runs[j]
            dy = dvals[j]
            if heads[h_id].kind == "polarization":
                # Stokes gradient of the intensities' (PolarizerFunction), direction / up gradients accumulated
                dd = ddirs[r0:] if ddirs is not None else torch.zeros(rays, 3, device=dev)
                du = dups[r0:] if dups is not None else torch.zeros(rays, 3, device=dev)
                dyc = dy.contiguous()
                dsc = torch.empty(rays * S, 3, device=dev)
                _lib.call("mms_polarizer_bwd", y.data_ptr(), dirs[r0:].data_ptr(), ups[r0:].data_ptr(), rays, S,
                          dyc.data_ptr(), dsc.data_ptr(), dd.data_ptr(), du.data_ptr(), _s())
                dy = dsc
            if not need_feat:
                _mlp_backward(run, dy, None)
                continue
            rows = dfeat[r0 * S:(r0 + rays) * S]
            if f_direct:
                _mlp_backward(run, dy, rows)
            else:
                rows += _mlp_backward(run, dy, None)
        ctx.runs = ctx.vals = None
        return (dfeat, dw if ctx.needs_input_grad[1] else None,
                acc_ret(ctx.acc_d, ddirs) if ctx.needs_input_grad[2] else None,
                acc_ret(ctx.acc_u, dups) if ctx.needs_input_grad[3] else None, None, None, None, None, *dbgs,
                *([None] * ctx.n_params))


def _composite_extents(tag, w, v, ldv, C, bg, R, S, idx, nout, hit, dout, dv, lddv, dw, dbg) -> None:
    """Debugging (MMS_SYNC_CALLS=1): the elements mms_composite_fwd / _bwd will touch lie inside every operand."""
    def need(name, t, n):
        # elements reachable from the view's first one in its storage (a strided view may reach past its numel)
        avail = None if t is None else t.untyped_storage().nbytes() // t.element_size() - t.storage_offset()
        if t is not None and avail < n:
            raise RuntimeError(f"composite {tag}: {name} reaches {avail} elements, the launch touches {n} "
                               f"(R {R}, S {S}, C {C}, nout {nout}, ldv {ldv}, lddv {lddv}, shapes "
                               f"{None if t is None else tuple(t.shape)})")
    need("w", w, R * S)
    need("vals", v, (R * S - 1) * ldv + C)
    need("dvals", dv, (R * S - 1) * lddv + C)
    need("dw", dw, R * S)
    need("dout", dout, nout * C)
    need("bg", bg, nout * C)
    need("dbg", dbg, nout * C)
    need("hit", hit, nout)
    if idx is not None:
        need("idx", idx, R)
        mx = int(idx[:R].max())
        if mx > nout:
            raise RuntimeError(f"composite {tag}: scatter index {mx} > nout {nout}")


def _partitions(ranges, total: int) -> bool:
    """True when the (start, length) ranges tile [0, total) exactly once."""
    pos = 0
    for a, n in sorted(ranges):
        if a != pos:
            return False
        pos += n
    return pos == total


def _job_covered(j: int, items, live) -> bool:
    """True when job j's items with gradients write every value row of the job exactly once."""
    rng = [(it[1], it[2]) for it, on in zip(items, live) if on and it[0] == j]
    total = max([a + n for a, n in rng] + [0])
    return _partitions(rng, total) and total > 0


def _mlp_backward(run, dy: torch.Tensor, dx_out: Optional[torch.Tensor]) -> torch.Tensor:
    """dX of an MLP runner (written into dx_out when given); parameter gradients accumulated in place."""
    if isinstance(run, ChainRun):
        dy = dy if dy.stride(1) == 1 and dy.stride(0) % 4 == 0 and dy.data_ptr() % 16 == 0 else _copy_aligned(dy)
        return run.backward(dy, dx_out=dx_out)
    dx, _ = run.backward(dy.contiguous(), need_dx=True, dx_out=dx_out)
    return dx


class GeoLossSegFunction(torch.autograd.Function):
    """Eikonal MSE(||g||, 1) and curvature L1(sum h, 0) over every modality's rows of a batched hit set
    (LossManager.compute_loss concatenates the modalities' gradients / hessians, losses.py:235-260).  ``counts``
    (fixed-capacity batches): device hit counts [n_seg]; segment m owns rows [m rows_per_seg S, (m+1) rows_per_seg S)
    of which the first counts[m] S are real.  None: every row is real."""

    @staticmethod
    def forward(ctx, S: int, counts, seg_rays: int, grads, hess):
        ctx.set_materialize_grads(False)
        dev = grads.device
        g = grads.reshape(-1, 3).contiguous()
        h = hess.reshape(-1, 3).contiguous() if hess is not None else None
        M = g.shape[0]
        eik, curv = torch.zeros(2, device=dev).unbind(0)   # outputs: not from the step arena
        if counts is None:
            _lib.call("mms_geo_loss_fwd", g.data_ptr(), _p(h), M, 1.0 / float(max(M, 1)), eik.data_ptr(),
                      curv.data_ptr(), _s())
        else:
            n = counts.shape[0]
            rows = seg_rays * S
            for m in range(n):
                _lib.call("mms_geo_loss_fwd_masked", g[m * rows:].data_ptr(),
                          _p(None if h is None else h[m * rows:]), rows, S, counts[m:].data_ptr(), counts.data_ptr(),
                          n, eik.data_ptr(), curv.data_ptr(), _s())
        ctx.save_for_backward(g, h, counts)
        ctx.S, ctx.seg_rays, ctx.shape = S, seg_rays, (tuple(grads.shape), None if hess is None else tuple(hess.shape))
        return eik, curv

    @staticmethod
    def backward(ctx, deik, dcurv):
        g, h, counts = ctx.saved_tensors
        S = ctx.S
        M = g.shape[0]
        dg, dh = _zeroed_views([(M, 3), (M, 3) if h is not None else None], g.device)
        de = _p(None if deik is None else deik.contiguous())
        dc = _p(None if dcurv is None else dcurv.contiguous())
        if counts is None:
            _lib.call("mms_geo_loss_bwd", g.data_ptr(), _p(h), M, 1.0 / float(max(M, 1)), de, 1.0, dc, 1.0,
                      dg.data_ptr(), _p(dh), _s())
        else:
            n = counts.shape[0]
            rows = ctx.seg_rays * S
            for m in range(n):
                _lib.call("mms_geo_loss_bwd_masked", g[m * rows:].data_ptr(), _p(None if h is None else h[m * rows:]),
                          rows, S, counts[m:].data_ptr(), counts.data_ptr(), n, de, 1.0, dc, 1.0,
                          dg[m * rows:].data_ptr(), _p(None if dh is None else dh[m * rows:]), _s())
        gs, hs = ctx.shape
        return None, None, None, dg.view(gs), (dh.view(hs) if dh is not None else None)


class StepLossFunction(torch.autograd.Function):
    """The whole training loss of a batched hit set in one autograd node (LossManager.compute_loss, losses.py:213-265):
    per modality nn.L1Loss(mean) with the polarization SkipSaturation fill (:152-164), the eikonal MSE and curvature L1
    over every modality's rows (:107-150, GeoLossSegFunction's kernels), total = sum of L1 terms + 0.1 eik + w_curv
    curv (method_configs.py:252-253) -- the terms land in one device buffer and one launch forms the total; the
    backward hands each term's kernel the total's gradient with its weight as the scale, so none of the scalar
    add / mul nodes (and their backward launches) exist.  Returns (total, terms [n_mod + 2], not differentiable)."""

    @staticmethod
    def forward(ctx, n_mod: int, sat_thrs, w_curv: float, S: int, counts, seg_rays: int, grads, hess, *outs_targets):
        ctx.set_materialize_grads(False)
        ctx.acc_g = acc_of(grads)
        outs, targets = outs_targets[:n_mod], outs_targets[n_mod:]
        dev = grads.device
        # carved from the step's zero arena in a captured step (its outputs are the graph's static buffers anyway,
        # valid until the next replay); eager steps return buffers of their own
        terms = _zeroed_views([(n_mod + 2,)], dev)[0] if _capturing(dev) else torch.zeros(n_mod + 2, device=dev)
        ctx.fused = FUSED_STEP_LOSS and all(t is None for t in sat_thrs) and n_mod <= 8
        if ctx.fused:
            return StepLossFunction._forward_fused(ctx, n_mod, w_curv, S, counts, seg_rays, grads, hess, outs,
                                                   targets, terms, dev)
        saved, scr = [], []
        for i in range(n_mod):
            o, t = outs[i], targets[i].contiguous()
            o = o if o.stride(1) == 1 else o.contiguous()
            N, C = t.shape
            thr = sat_thrs[i]
            sc = torch.empty(1, dtype=torch.int64, device=dev) if thr is not None else None
            _lib.call("mms_l1_loss_fwd", o.data_ptr(), o.stride(0), t.data_ptr(), N, C, 0.0 if thr is None else thr,
                      _p(sc), terms[i:].data_ptr(), _s())
            saved += [o, t]
            scr.append(sc)
        g = grads.reshape(-1, 3).contiguous()
        h = hess.reshape(-1, 3).contiguous() if hess is not None else None
        M = g.shape[0]
        eik, curv = terms[n_mod:], terms[n_mod + 1:]
        if counts is None:
            _lib.call("mms_geo_loss_fwd", g.data_ptr(), _p(h), M, 1.0 / float(max(M, 1)), eik.data_ptr(),
                      curv.data_ptr(), _s())
        else:
            n = counts.shape[0]
            rows = seg_rays * S
            for m in range(n):
                _lib.call("mms_geo_loss_fwd_masked", g[m * rows:].data_ptr(),
                          _p(None if h is None else h[m * rows:]), rows, S, counts[m:].data_ptr(), counts.data_ptr(),
                          n, eik.data_ptr(), curv.data_ptr(), _s())
        w = [1.0] * n_mod + [0.1] + ([float(w_curv)] if h is not None else [])
        total = torch.empty((), device=dev)
        _lib.call("mms_weighted_sum", terms.data_ptr(), len(w), _f32arr(w), total.data_ptr(), _s())
        ctx.mark_non_differentiable(terms)
        ctx.save_for_backward(g, h, counts, *saved)
        ctx.n_mod, ctx.sat, ctx.scr, ctx.w_curv, ctx.S, ctx.seg_rays = n_mod, sat_thrs, scr, float(w_curv), S, seg_rays
        ctx.shape = (tuple(grads.shape), None if hess is None else tuple(hess.shape))
        ctx.out_shapes = [tuple(o.shape) for o in outs]
        return total, terms

    @staticmethod
    def _geo_segs(g, h, counts, seg_rays: int, S: int):
        """(grads, hess, rows, count) per geometric segment, counts_all, n_counts, inv_total."""
        M = g.shape[0]
        if counts is None:
            return [(g, h, M, None)], None, 0, 1.0 / float(max(M, 1))
        n = counts.shape[0]
        rows = seg_rays * S
        return [(g[m * rows:], None if h is None else h[m * rows:], rows, counts[m:]) for m in range(n)], counts, n, 0.0

    @staticmethod
    def _forward_fused(ctx, n_mod, w_curv, S, counts, seg_rays, grads, hess, outs, targets, terms, dev):
        """forward's terms by mms_step_loss_fwd (one launch for every L1 and geometric segment; no SkipSaturation)."""
        ol = [o if o.stride(1) == 1 else o.contiguous() for o in outs]
        tl = [t.contiguous() for t in targets]
        g = grads.reshape(-1, 3).contiguous()
        h = hess.reshape(-1, 3).contiguous() if hess is not None else None
        segs, call, nc, inv = StepLossFunction._geo_segs(g, h, counts, seg_rays, S)
        n, ng = n_mod, len(segs)
        VP, I64 = ctypes.c_void_p, ctypes.c_int64
        _lib.call("mms_step_loss_fwd", n, (VP * n)(*[o.data_ptr() for o in ol]), (I64 * n)(*[o.stride(0) for o in ol]),
                  (VP * n)(*[t.data_ptr() for t in tl]), (I64 * n)(*[t.shape[0] for t in tl]),
                  (ctypes.c_int * n)(*[t.shape[1] for t in tl]), (ctypes.c_float * n)(*([0.0] * n)),
                  (VP * n)(*([None] * n)), (VP * n)(*[terms[i:].data_ptr() for i in range(n)]), ng,
                  (VP * ng)(*[sg[0].data_ptr() for sg in segs]), (VP * ng)(*[_p(sg[1]) for sg in segs]),
                  (I64 * ng)(*[sg[2] for sg in segs]), S, (VP * ng)(*[_p(sg[3]) for sg in segs]), _p(call), nc, inv,
                  terms[n_mod:].data_ptr(), terms[n_mod + 1:].data_ptr(), _s())
        w = [1.0] * n_mod + [0.1] + ([float(w_curv)] if h is not None else [])
        total = torch.empty((), device=dev)
        _lib.call("mms_weighted_sum", terms.data_ptr(), len(w), _f32arr(w), total.data_ptr(), _s())
        ctx.mark_non_differentiable(terms)
        ctx.save_for_backward(g, h, counts, *[x for pair in zip(ol, tl) for x in pair])
        ctx.n_mod, ctx.scr, ctx.w_curv, ctx.S, ctx.seg_rays = n_mod, None, float(w_curv), S, seg_rays
        ctx.shape = (tuple(grads.shape), None if hess is None else tuple(hess.shape))
        ctx.out_shapes = [tuple(o.shape) for o in outs]
        return total, terms

    @staticmethod
    def _backward_fused(ctx, dl, g, h, counts, saved):
        n_mod, dev, S = ctx.n_mod, g.device, ctx.S
        douts = [_zeroed_views([ctx.out_shapes[i]], dev)[0] for i in range(n_mod)]
        M = g.shape[0]
        dh = _zeroed_views([(M, 3)], dev)[0] if h is not None else None
        dg = acc_or_zeroed(ctx.acc_g, (M, 3), dev).view(M, 3)
        segs, call, nc, inv = StepLossFunction._geo_segs(g, h, counts, ctx.seg_rays, S)
        rows = [sg[2] for sg in segs]
        offs = [0]
        for r in rows[:-1]:
            offs.append(offs[-1] + r)
        ol, tl = saved[0::2], saved[1::2]
        n, ng = n_mod, len(segs)
        VP, I64 = ctypes.c_void_p, ctypes.c_int64
        _lib.call("mms_step_loss_bwd", n, (VP * n)(*[o.data_ptr() for o in ol]), (I64 * n)(*[o.stride(0) for o in ol]),
                  (VP * n)(*[t.data_ptr() for t in tl]), (I64 * n)(*[t.shape[0] for t in tl]),
                  (ctypes.c_int * n)(*[t.shape[1] for t in tl]), (ctypes.c_float * n)(*([0.0] * n)),
                  (VP * n)(*([None] * n)), (VP * n)(*[d.data_ptr() for d in douts]),
                  (I64 * n)(*[d.stride(0) for d in douts]), ng, (VP * ng)(*[sg[0].data_ptr() for sg in segs]),
                  (VP * ng)(*[_p(sg[1]) for sg in segs]), (I64 * ng)(*rows), S, (VP * ng)(*[_p(sg[3]) for sg in segs]),
                  _p(call), nc, inv, dl.data_ptr(), 0.1, ctx.w_curv, (VP * ng)(*[dg[o:].data_ptr() for o in offs]),
                  (VP * ng)(*[(None if dh is None else dh[o:].data_ptr()) for o in offs]), _s())
        gs, hs = ctx.shape
        return (None, None, None, None, None, None, acc_ret(ctx.acc_g, dg.view(gs)),
                (dh.view(hs) if dh is not None else None), *douts, *([None] * n_mod))

    @staticmethod
    def backward(ctx, dtotal, dterms):
        g, h, counts, *saved = ctx.saved_tensors
        n_mod = ctx.n_mod
        dev = g.device
        if dtotal is None:
            return (None,) * (8 + 2 * n_mod)
        dl = dtotal.contiguous()
        if ctx.fused:
            return StepLossFunction._backward_fused(ctx, dl, g, h, counts, saved)
        douts = []
        for i in range(n_mod):
            o, t = saved[2 * i], saved[2 * i + 1]
            N, C = t.shape
            thr = ctx.sat[i]
            d = _zeroed_views([ctx.out_shapes[i]], dev)[0]
            _lib.call("mms_l1_loss_bwd", o.data_ptr(), o.stride(0), t.data_ptr(), N, C, 0.0 if thr is None else thr,
                      _p(ctx.scr[i]), dl.data_ptr(), 1.0, d.data_ptr(), d.stride(0), _s())
            douts.append(d)
        M = g.shape[0]
        dh = _zeroed_views([(M, 3)], dev)[0] if h is not None else None
        dg = acc_or_zeroed(ctx.acc_g, (M, 3), dev).view(M, 3)
        S = ctx.S
        if counts is None:
            _lib.call("mms_geo_loss_bwd", g.data_ptr(), _p(h), M, 1.0 / float(max(M, 1)), dl.data_ptr(), 0.1,
                      dl.data_ptr(), ctx.w_curv, dg.data_ptr(), _p(dh), _s())
        else:
            n = counts.shape[0]
            rows = ctx.seg_rays * S
            for m in range(n):
                _lib.call("mms_geo_loss_bwd_masked", g[m * rows:].data_ptr(), _p(None if h is None else h[m * rows:]),
                          rows, S, counts[m:].data_ptr(), counts.data_ptr(), n, dl.data_ptr(), 0.1, dl.data_ptr(),
                          ctx.w_curv, dg[m * rows:].data_ptr(), _p(None if dh is None else dh[m * rows:]), _s())
        gs, hs = ctx.shape
        ctx.scr = None
        return (None, None, None, None, None, None, acc_ret(ctx.acc_g, dg.view(gs)),
                (dh.view(hs) if dh is not None else None), *douts, *([None] * n_mod))


# the step loss's L1 and geometric terms in one launch each way (mms_step_loss_fwd / _bwd) when no modality uses the
# SkipSaturation fill; MMS_FUSED_STEP_LOSS=0: one launch per term and segment
FUSED_STEP_LOSS = os.environ.get("MMS_FUSED_STEP_LOSS", "1") != "0"


def HashGridApply(x, table, cfg: GridCfg, active: int):
    """Standalone FeatureGrid forward (feature_structures.py:78-83) with autograd to x and table."""
    from .hip_ops import HashGridFunction
    return HashGridFunction.apply(x, table, cfg.scales, cfg.log2T, cfg.radius, active, cfg.interp)
