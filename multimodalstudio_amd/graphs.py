"""Graph-captured training step: the whole of ``Trainer.train_step`` replayed as hipGraphs.

The eager step issues ~470 kernel launches from Python (autograd nodes, ctypes calls, allocator work); on
MI355X the GPU sat idle for about half of every step waiting for them (profiles/round1_fast_trace_summary.txt:
busy 9.7 of 20.6 ms per step).  Here the step body -- pixel-value gather, ray generation with pose refinement,
the model, losses, backward, grad-norm clip and AdamW -- is captured once with ``torch.cuda.graph``
(hipStreamBeginCapture under ROCm) and replayed; per step the host only samples pixels (the reference's CPU
generator, pixel_samplers.py:71-89), uploads them into static buffers and launches the graph.

Static shapes.  The foreground batch is the set of rays that hit the unit sphere (scene_colliders.py:60-80,
base_model.py:88-93); its size N_hit changes every step.  A replayable graph needs fixed sizes, so each
modality's hit rays are compacted into a fixed-capacity batch of ``cap`` rows (BaseModel.forward(cap=...),
``mms_compact_padded``): rows past the true count repeat the first hit ray (valid, finite inputs), scatter
their composite into a dummy output row N that the loss never reads, and are skipped by the eikonal /
curvature terms (``GeoLossMaskedFunction``), so every gradient they produce is exactly zero.  ``cap`` is the
largest N_hit over the modalities rounded up to a granule (64 rays); one graph is kept per capacity, and the
neighbouring capacities are captured together with the first one.  Choosing ``cap`` needs N_hit on the host:
a collider pass on the step's rays (raygen + collider + compaction count, no autograd) and one small
device->host read per step -- the step's only synchronisation.

Scalars.  Values the kernels take by value are baked into a graph: the coarse-to-fine level, the tap delta,
the cos-anneal ratio and the curvature-loss factor (feature_structures.py:97-108, surface_model.py:254-271,
volume_rendering.py:227-230, schedulers.py:320-343).  They are part of the graph key; a step whose values
differ from the previous step's runs eagerly (early in a 100k-step run some of them change every step), and a
graph is captured once they hold still.  The AdamW scalars (learning-rate schedule, bias corrections) change
every step and are read from a device buffer instead (``mms_adamw_dev``).

Multi-GPU: the RCCL gradient all-reduce stays outside the graphs, so each rank may replay a different capacity
and no collective is ever captured.  The data-parallel step is four graphs: (1a) the forward and the backward's first
phase (the rendering side, functions.PHASE_CUT) with the MLPs' weight-gradient GEMMs deferred
(functions.wgrad_defer_begin) -- when it ends the radiance table's gradient (and a grid background's) is final, so its
bucketed all-reduce is launched right after the replay; (1m) the backward's second phase (the SDF field, its table, the
sampler, the rays and the poses), replayed while that all-reduce runs -- when it ends the SDF table's gradient is final
and its all-reduce goes out; (1b) the deferred weight-gradient GEMMs + weight-norm flush, replayed while those run; (2)
the rest of the all-reduce, then clip + AdamW (+ the next step's draws).  The three backward graphs are one capture
split on the caller's thread where pipeline.backward_batched calls ``mid`` and ``between``.
"""
from __future__ import annotations

import os
import sys
from typing import Dict, Optional, Tuple

import torch

from . import _lib
from . import functions as fx
from .pipeline import Trainer, backward_batched, compute_loss, curvature_factor, lr_factor, select_right_channel


CAPTURE_MODE = None   # override of the capture_error_mode (probes)
# the optimizer groups zeroed / clipped / stepped together (pipeline.OptimBank: 3 launches and 1 scalar upload per
# step instead of 8 and 2); MMS_BANKED_OPTIM=0: per group
BANKED_OPTIM = os.environ.get("MMS_BANKED_OPTIM", "1") != "0"
# the tail's next-step hit count in one launch (mms_count_hits; 618.7k -> 620.5k rays/s, 2 x 2 A/B);
# MMS_FUSED_COUNT=0: pose exp + raygen + collider + compact
FUSED_COUNT = os.environ.get("MMS_FUSED_COUNT", "1") != "0"


def bucket_capacity(counts, granule: int, n: int) -> int:
    """Fixed foreground capacity for hit counts ``counts``: the largest, rounded up to ``granule``, at most n.

    Invariant: a replayed step's own compaction count is <= the capacity chosen here.  The counts come from the
    previous step's tail (mms_count_hits with the poses that step's optimizer wrote), which is the same ray
    generation and collider arithmetic as the step's own RaysFunction + ColliderFunction + compaction
    (test_gpu_graph.py::test_fused_hit_count_equals_unfused pins the equality).  The composite relies on it: hit rows
    are written only by a composited ray (mms_composite_fwd's padding blocks fill the non-hit rows), so a hit ray past
    the capacity would leave its output row unwritten."""
    c = max(counts)
    return min(n, -(-c // granule) * granule)


class GraphTrainer:
    """Drive a ``pipeline.Trainer`` with graph-captured steps (see the module docstring)."""

    def __init__(self, trainer: Trainer, granule: int = 64, neighbours: int = 2, ddp=None):
        self.t = trainer
        self.ddp = ddp
        self.granule = int(granule)
        self.neighbours = int(neighbours)
        dev = trainer.device
        n = trainer.cfg.num_rays_per_modality
        self.n = n
        mods = trainer.modalities
        if trainer.gpu_sampler is not None:
            # device-drawn pixels: the sampler's persistent buffers are the graphs' static inputs
            self.coords, self.sel = trainer.gpu_sampler.coords, trainer.gpu_sampler.sel
        else:
            self.coords = {m: torch.zeros(n, 3, dtype=torch.int32, device=dev) for m in mods}
            self.sel = {m: torch.zeros(n, dtype=torch.int64, device=dev) for m in mods}
        self.h_coords = {m: torch.zeros(n, 3, dtype=torch.int32).pin_memory() for m in mods}
        self.h_sel = {m: torch.zeros(n, dtype=torch.int64).pin_memory() for m in mods}
        self.count_dev = torch.zeros(len(mods), dtype=torch.int64, device=dev)
        self.count_host = torch.zeros(len(mods), dtype=torch.int64).pin_memory()
        self.idx_scratch = torch.empty(n, dtype=torch.int64, device=dev)
        # identity pose matrices (pose refinement off) for the fused hit count, made here: outside any capture
        self._eye = {dev: torch.eye(4, device=dev)[None, :3, :4].contiguous()}
        self.side = torch.cuda.Stream(device=dev)
        self.graphs: Dict[tuple, Tuple[torch.cuda.CUDAGraph, Optional[torch.cuda.CUDAGraph], tuple]] = {}
        self.pool = None
        self.last_sig = None
        self.ran_eager = False
        self.disabled: Optional[str] = None
        # device sampler: every step (graph or eager) ends by staging the next step's pixels and hit counts
        self.tail = trainer.gpu_sampler is not None
        self.staged = False
        self.hyper_step = None      # the step whose AdamW scalars are already queued (behind the last replay)
        self.count_event = torch.cuda.Event() if torch.cuda.is_available() else None
        self.stats = {"replays": 0, "eager": 0, "captures": 0}

    # -- host side ---------------------------------------------------------------------------------
    def scalar_signature(self) -> tuple:
        """The by-value kernel scalars of the current step (the callbacks applied for t.step)."""
        t = self.t
        t.model.set_step(t.step, t.cfg.max_iters)
        sm = t.model.surface_model
        rg = t.model.radiance_model.radiance_field.base_field.feature_grid
        return (sm.surface_field.field.feature_grid.active_levels, rg.active_levels,
                float(sm.numerical_gradients_delta), float(sm.volume_rendering._cos_anneal_ratio),
                float(curvature_factor(t.step, t.cfg.max_iters)))

    def _stage_inputs(self):
        """Host pixel sampling (reference RNG order) into pinned buffers, then async upload to the static ones."""
        t = self.t
        if t.gpu_sampler is not None:
            coords, _, _ = t.gpu_sampler.sample()
            return coords
        coords, sel = t.sampler.sample(t.frames)
        for m in t.modalities:
            self.h_coords[m].copy_(coords[m])
            self.h_sel[m].copy_(sel[m].to(torch.int64))
            self.coords[m].copy_(self.h_coords[m], non_blocking=True)
            self.sel[m].copy_(self.h_sel[m], non_blocking=True)
        return coords

    @torch.no_grad()
    def _count_hits(self, zeroed: bool = False):
        """Enqueue ray generation (current pose deltas) + collider + compaction count for the staged rays and the
        count's copy into pinned host memory (no synchronisation)."""
        t = self.t
        dev = t.device
        if FUSED_COUNT and not zeroed:
            self.count_dev.zero_()    # (a captured step zeroes it at its start, with the gradients: zeroed=True)
        for i, m in enumerate(t.modalities):
            if FUSED_COUNT:
                # pose exp map, ray generation, collider and count in one launch (mms_count_hits)
                pa = t.pose.pose_adjustment
                tangent = pa[m].detach() if (t.pose.mode != "off" and m in pa) else None
                if tangent is None:
                    mats, B = self._eye[dev], 1
                else:
                    tangent = tangent.contiguous()
                    mats, B = None, tangent.shape[0]
                cams = t.cams[m]
                _lib.call("mms_count_hits", self.coords[m].data_ptr(), self.n, cams.fx.data_ptr(), cams.fy.data_ptr(),
                          cams.cx.data_ptr(), cams.cy.data_ptr(), cams.c2w.data_ptr(), fx._p(cams.distortion),
                          fx._p(tangent), fx._p(mats), B, 1 if B > 1 else 0, float(t.raygen.pixel_offset), 1.0,
                          self.count_dev[i:i + 1].data_ptr(), fx._s())
                continue
            mats = t.pose.matrices(m, dev)
            o, d, _, _, _ = fx.RaysFunction.apply(mats, self.coords[m], t.cams[m], t.raygen.pixel_offset)
            mask = fx.ColliderFunction.apply(o, d, 1.0)[4]
            _lib.call("mms_compact", mask.data_ptr(), self.n, self.idx_scratch.data_ptr(),
                      self.count_dev[i:i + 1].data_ptr(), fx._s())
        self.count_host.copy_(self.count_dev, non_blocking=True)

    def hit_counts(self):
        """N_hit per modality for the staged rays, read on the host (the step's only synchronisation)."""
        self._count_hits()
        torch.cuda.current_stream().synchronize()
        return [int(c) for c in self.count_host.tolist()]

    def _tail(self, captured: bool = False):
        """Device-sampler steps end by drawing the NEXT step's pixels and counting its hits (with the poses this step's
        optimizer just updated), so the host only waits for that count -- no eager ray generation, collider or
        synchronisation between two replays.  Captured at the end of each graph (``captured``: the step zeroed the
        hit counter with its gradients, OptimBank.zero_grads); after an eager step the counter is zeroed here."""
        self.t.gpu_sampler.sample()
        self._count_hits(zeroed=captured and BANKED_OPTIM)

    # -- the captured work ---------------------------------------------------------------------------
    def _targets(self):
        t = self.t
        if t.gpu_sampler is not None:
            return t.gpu_sampler.values      # gathered by the sampler kernel with the coordinates
        return {m: t.images[m][self.sel[m], self.coords[m][:, 1].long(), self.coords[m][:, 2].long()]
                for m in t.modalities}

    def _forward_backward(self, cap: int, between=None, mid=None):
        t = self.t
        targets = self._targets()
        if BANKED_OPTIM:
            # the gradients, the clip accumulators and the step's zero arena in one launch
            arena = fx.zero_arena_prepare(t.device)
            # (+ the hit counter the tail's mms_count_hits adds into; the host has read it before this replay)
            extra = ((self.count_dev.view(torch.float32),) if FUSED_COUNT else ()) + (() if arena is None else (arena,))
            t.optim.zero_grads(extra)
            fx.zero_arena_begin(t.device, zeroed=arena)
        else:
            t.fields.zero_grad()
            if t.poses is not None:
                t.poses.zero_grad()
            fx.zero_arena_begin(t.device)
        try:
            return self._forward_backward_body(t, targets, cap, between, mid)
        finally:
            fx.zero_arena_end()

    def _forward_backward_body(self, t, targets, cap: int, between=None, mid=None):
        rays = t.raygen(self.coords)
        fx.reset_grad_uses()
        cuts = None
        if mid is not None:
            # the two-phase backward (functions.PHASE_CUT): the forward records where the SDF side hands over
            cuts = fx.PHASE_CUT[0] = []
        try:
            outputs = t.model(rays, None, cap=cap)
        finally:
            fx.PHASE_CUT[0] = None
        if t.raw:
            for m in t.modalities:
                c = self.coords[m]
                band = t.masks[m][c[:, 1].long(), c[:, 2].long()].long()[:, None]
                outputs[m][m] = select_right_channel(outputs[m][m], band)
        losses, total = compute_loss(outputs, targets, t.modalities, t.step, max_iters=t.cfg.max_iters)
        backward_batched(total, between, mid, cuts)
        return losses, total

    def table_grads(self, phase: Optional[int] = None):
        """Flat-buffer views of the hash-table gradients.  ``phase`` 1: those final when the backward's first phase
        ends (the radiance field's and a grid background's table: functions.PHASE_CUT); 2: the SDF field's, final
        when the second phase ends; None: all."""
        out = []
        for name, p in self.t.model.named_parameters():
            if not name.endswith("hash_table"):
                continue
            sdf = name.startswith("surface_model.")
            if phase is None or (phase == 2) == sdf:
                out.append(p.grad.view(-1))
        return out

    @staticmethod
    def _capture_stream():
        """The stream the step graphs are captured on (torch's default capture stream; a high-priority capture stream
        measured 16 % slower steps, round 4: 499k vs 591k rays/s)."""
        if torch.cuda.graph.default_capture_stream is None:
            torch.cuda.graph.default_capture_stream = torch.cuda.Stream()
        return torch.cuda.graph.default_capture_stream

    def _capture_split(self, cap: int, mode: str):
        """Data-parallel capture: the forward/backward split into three graphs -- (a) the forward and the backward's
        first phase (the rendering side: the radiance and grid-background table gradients are final when it ends), (m)
        the second phase (the SDF side: the SDF table gradient is final when it ends), (b) the deferred weight
        gradients and the weight-norm flush -- at the two caller-thread points of pipeline.backward_batched (``mid``,
        ``between``)."""
        gs = [torch.cuda.CUDAGraph() for _ in range(3)]
        pool = () if self.pool is None else (self.pool,)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        live = [0]

        def cut_here():
            gs[live[0]].capture_end()
            live[0] += 1
            gs[live[0]].capture_begin(gs[0].pool(), capture_error_mode=mode)

        with torch.cuda.stream(self._capture_stream()):
            gs[0].capture_begin(*pool, capture_error_mode=mode)
            try:
                out = self._forward_backward(cap, cut_here, cut_here)
            except BaseException:
                try:
                    gs[live[0]].capture_end()
                except Exception:
                    pass
                raise
            gs[live[0]].capture_end()
        if live[0] != 2:
            raise RuntimeError(f"the backward reached {live[0]} of its 2 split points")
        return gs, out

    def _optimizer(self):
        t = self.t
        if BANKED_OPTIM:
            t.optim.step_captured()
            return
        t.fields.step_captured()
        if t.poses is not None:
            t.poses.step_captured()

    def capture(self, key: tuple) -> None:
        cap = key[0]
        # thread-local capture mode when a process group is up: RCCL's watchdog thread queries events meanwhile
        mode = CAPTURE_MODE or ("thread_local" if self.ddp is not None else "global")
        torch.cuda.synchronize()
        if self.ddp is None:
            g1 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g1, pool=self.pool, stream=self._capture_stream(), capture_error_mode=mode):
                out = self._forward_backward(cap)
                self._optimizer()
                if self.tail:
                    self._tail(captured=True)
            pool = g1.pool()
        else:
            g1, out = self._capture_split(cap, mode)
            pool = g1[0].pool()
        if self.pool is None:
            self.pool = pool
        g2 = None
        if self.ddp is not None:
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2, pool=self.pool, stream=self._capture_stream(), capture_error_mode=mode):
                self._optimizer()
                if self.tail:
                    self._tail(captured=True)
        self.graphs[key] = (g1, g2, out)
        self.stats["captures"] += 1

    # -- one training iteration ------------------------------------------------------------------
    def _queue_hyper(self):
        """Queue this step's AdamW scalars (advances the optimizers' step counts)."""
        t = self.t
        f = lr_factor(t.step, t.cfg.max_iters)
        if BANKED_OPTIM:
            t.optim.load_hyper(f)
        else:
            t.fields.load_hyper(f)
            if t.poses is not None:
                t.poses.load_hyper(f)
        self.hyper_step = t.step

    def _drop_queued_hyper(self):
        """An eager step follows a queued scalar upload: undo its step-count advance (the eager optimizer advances)."""
        if self.hyper_step is not None:
            self.t.fields.step_count -= 1
            if self.t.poses is not None:
                self.t.poses.step_count -= 1
            self.hyper_step = None

    def eager_step(self, coords):
        """Trainer.train_step on the already-staged inputs (dynamic shapes, no graph), on the side stream the
        captures run on (lazy per-stream state is initialised before the first capture)."""
        self._drop_queued_hyper()
        self.stats["eager"] += 1
        self.ran_eager = True
        cur = torch.cuda.current_stream()
        self.side.wait_stream(cur)
        with torch.cuda.stream(self.side):
            losses, total, _ = self.t.train_step(coords, self._targets(), ddp=self.ddp)
        cur.wait_stream(self.side)
        return losses, total

    def step(self):
        """One training iteration; returns (losses, total) -- when replayed, the graph's output tensors (valid until
        the next replay)."""
        t = self.t
        sig = self.scalar_signature()
        if self.disabled is not None:
            return self.eager_step(self._stage_inputs())
        if self.staged:
            # pixels drawn and hits counted by the previous step's tail: wait for that count only
            self.count_event.synchronize()
            counts = [int(c) for c in self.count_host.tolist()]
            coords = self.coords
        else:
            coords = self._stage_inputs()
            counts = self.hit_counts()
        self.staged = False
        stable = sig == self.last_sig
        self.last_sig = sig
        if min(counts) == 0 or not (stable and self.ran_eager):
            # a modality without hits, scalars that changed this step, or nothing run yet: one eager step
            return self._eager_with_tail(coords)
        cap = bucket_capacity(counts, self.granule, self.n)
        key = (cap,) + sig
        if key not in self.graphs:
            try:
                for k in [0] + [d for j in range(1, self.neighbours + 1) for d in (j, -j)]:
                    c = min(cap + k * self.granule, self.n)
                    if c >= self.granule or c == cap:
                        kk = (c,) + sig
                        if kk not in self.graphs:
                            self.capture(kk)
            except Exception as e:  # capture unsupported here: keep training eagerly
                self.disabled = f"{type(e).__name__}: {e}"
                print(f"[graphs] capture failed, eager steps from now on: {self.disabled}", file=sys.stderr)
                torch.cuda.synchronize()
                return self.eager_step(coords)
        if self.hyper_step != t.step:
            self._drop_queued_hyper()
            self._queue_hyper()
        self.hyper_step = None
        g1, g2, out = self.graphs[key]
        if self.ddp is None:
            g1.replay()
        else:
            # the radiance (+ grid background) table's all-reduce, launched after the first graph, runs while the
            # second replays the SDF backward; the SDF table's while the third replays the deferred weight gradients;
            # the rest follows, then the optimizer graph
            g1[0].replay()
            self.ddp.overlap_exchange([(self.table_grads(1), g1[1].replay), (self.table_grads(2), g1[2].replay)],
                                      [t.fields] + ([t.poses] if t.poses is not None else []))
            g2.replay()
        if self.tail:
            self.count_event.record()
            self.staged = True
        t.step += 1
        self.stats["replays"] += 1
        if self.tail:
            # the next step's scalars, queued behind this replay: the host's next step only waits for the hit count
            self._queue_hyper()
        return out

    def _eager_with_tail(self, coords):
        out = self.eager_step(coords)
        if self.tail:
            self._tail()
            self.count_event.record()
            self.staged = True
        return out
