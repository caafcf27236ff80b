"""ORACLE (test infrastructure only) — one CPU training step of the restated reference path.

Used as bench.py's ``cpu_baseline`` leg (the reference's own pure-PyTorch CPU field path, restated and
pinned bit-exact to it by tests/test_oracle_golden.py) and by PSNR-parity tests.  Restates
RawPipeline/BasePipeline.train_step (/root/reference/src/pipelines/raw_pipeline.py:67-82,
base_pipeline.py:138-153): rays -> model -> losses -> backward -> clip(2.0) -> AdamW -> scheduler.
"""
from __future__ import annotations

from typing import Dict, List

import torch

from . import model as om
from . import rays as orr


class OracleTrainer:
    def __init__(self, state_dict: Dict[str, torch.Tensor], modalities: Dict[str, int], cams: dict, log2T: int,
                 step: int, raw: bool = False, pose: Dict[str, torch.Tensor] = None,
                 mosaick: Dict[str, torch.Tensor] = None, fields: str = "grid", bg_kind: str = "nerf"):
        self.P = {k: v.detach().clone().float().cpu().requires_grad_(True) for k, v in state_dict.items()}
        self.spec = om.spec_mlp(modalities, raw=raw) if fields == "mlp" else om.spec_grid(modalities, log2T=log2T,
                                                                                              raw=raw, bg_kind=bg_kind)
        self.cams = cams
        self.mods = list(modalities)
        self.pose = {m: (pose[m].detach().clone() if pose else torch.zeros(1, 6)).requires_grad_(True)
                     for m in self.mods}
        self.step = step
        self.mosaick = mosaick or {}      # raw methods: per-modality band masks (select_right_channel)
        self.field_state: dict = {}
        self.pose_state: dict = {}
        # optional callable(params) run between backward and clipping: perturbation studies of the trajectory's
        # sensitivity to last-bit gradient differences (tests/golden/make_train_parity.py --perturb)
        self.grad_hook = None

    def rng(self, n_hit: Dict[str, int], n_rays: Dict[str, int]) -> om.RNG:
        """Uniform draws in the reference's order."""
        uni = {m: torch.rand(n_hit[m], 1) for m in self.mods}
        pdf = {m: [torch.rand(n_hit[m], 1) for _ in range(4)] for m in self.mods}
        bg = {m: torch.rand(n_rays[m], self.spec.bg_samples + 1) for m in self.mods}
        return om.RNG(uni, pdf, bg)

    def train_step(self, coords: Dict[str, torch.Tensor], targets: Dict[str, torch.Tensor]):
        st = om.StepState(step=self.step)
        rays = {}
        for m in self.mods:
            c = self.cams[m]
            rays[m] = orr.generate_rays(coords[m], c.fx, c.fy, c.cx, c.cy, c.c2w, c.distortion, self.pose[m], 0.0)
        with torch.no_grad():
            hits = {m: int(orr.sphere_collider(rays[m].origins, rays[m].directions)[2].sum()) for m in self.mods}
        rng = self.rng(hits, {m: coords[m].shape[0] for m in self.mods})
        outs = om.model_forward(rays, self.P, self.spec, st, rng)
        if self.spec.raw:
            # RawPipeline.train_step: each pixel's own band (raw_pipeline.py:74-76, 112-122)
            for m in self.mods:
                outs[m][m] = om.select_channel(outs[m][m], self.mosaick[m], coords[m])
        losses, total = om.compute_loss(outs, targets, self.spec, st)
        for p in list(self.P.values()) + list(self.pose.values()):
            p.grad = None
        total.backward()
        f = om.lr_factor(self.step)
        fields: List[torch.Tensor] = list(self.P.values())
        poses: List[torch.Tensor] = list(self.pose.values())
        if self.grad_hook is not None:
            self.grad_hook(fields + poses)
        om.clip_grad_norm(fields, 2.0)
        om.clip_grad_norm(poses, 2.0)
        om.adamw_step(fields, self.field_state, 1e-3 * f)
        om.adamw_step(poses, self.pose_state, 1e-4 * f)
        self.step += 1
        return float(total)
