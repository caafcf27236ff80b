"""Evaluation render path: chunked full-view rendering under no_grad, PSNR and TEST_RAYS_PER_SEC.

Mirrors Evaluator.render_view / eval_model_query / compute_metrics (/root/reference/src/engine/evaluator.py:100-178,
431-440; utils/eval_utils.py:31-76, 325-360): every pixel of a view becomes a ray (the full-image dataloader's
[frame, y, x] coordinates), rays are queried in chunks of ``eval_num_rays_per_chunk`` with the model in eval mode
(no jitter in any sampler, ray_samplers.py:212 / :365), chunk outputs are concatenated back into H x W images, and
PSNR = 10 log10(1 / MSE) of the [0, 1]-clipped rendering against the frame (torchmetrics peak_signal_noise_ratio,
data_range 1).  Raw modalities are compared mosaicked: each pixel's own band of the rendering (RawEvaluator
select_right_channel_per_rendered_pixel, evaluator.py:721-745).  Everything runs on the forward HIP kernels.
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional

import numpy as np
import torch

from . import scene as mscene
from .pipeline import DeviceCameras, RayGenerator, select_right_channel

PER_RAY_KEYS = ("depth", "accumulation", "normals")


def psnr(rendering: torch.Tensor, gt: torch.Tensor) -> float:
    """peak_signal_noise_ratio(clip(rendering, 0, 1), gt, data_range=1.0) (eval_utils.py:348-357)."""
    r = rendering.clip(0.0, 1.0).to(torch.float64)
    mse = torch.mean((r - gt.to(torch.float64)) ** 2)
    return float(10.0 * torch.log10(1.0 / mse))


def ssim(rendering: torch.Tensor, gt: torch.Tensor, data_range: float = 1.0, kernel_size: int = 11,
         sigma: float = 1.5, k1: float = 0.01, k2: float = 0.03) -> float:
    """structural_similarity_index_measure(clip(rendering, 0, 1), gt, data_range=1.0) on [H, W, C] images, as
    compute_metrics calls it for full views (eval_utils.py:325-394): an 11 x 11 Gaussian window (sigma 1.5) over
    reflect-padded images, c1 = (k1 L)^2, c2 = (k2 L)^2, the map cropped to the unpadded interior and averaged.
    torchmetrics' published formula restated (torchmetrics is absent here: parity unpinned)."""
    x = rendering.clip(0.0, 1.0).to(torch.float64).permute(2, 0, 1)[None]
    y = gt.to(torch.float64).permute(2, 0, 1)[None]
    C = x.shape[1]
    d = torch.arange((1 - kernel_size) / 2, (1 + kernel_size) / 2, 1.0, dtype=torch.float64, device=x.device)
    g = torch.exp(-((d / sigma) ** 2) / 2)
    g = g / g.sum()
    kern = (g[:, None] * g[None, :]).expand(C, 1, kernel_size, kernel_size)
    pad = (kernel_size - 1) // 2
    xp = torch.nn.functional.pad(x, (pad, pad, pad, pad), mode="reflect")
    yp = torch.nn.functional.pad(y, (pad, pad, pad, pad), mode="reflect")
    stats = torch.nn.functional.conv2d(torch.cat([xp, yp, xp * xp, yp * yp, xp * yp]), kern, groups=C)
    mx, my, xx, yy, xy = stats.split(1)
    c1, c2 = (k1 * data_range) ** 2, (k2 * data_range) ** 2
    vx, vy, cxy = xx - mx * mx, yy - my * my, xy - mx * my
    full = ((2 * mx * my + c1) * (2 * cxy + c2)) / ((mx * mx + my * my + c1) * (vx + vy + c2))
    return float(full[..., pad:-pad, pad:-pad].mean())


def degree_of_polarization(data: torch.Tensor) -> torch.Tensor:
    """to_dop (polarizer.py:103-116): Stokes (0.5 sum I, I0 - I90, I45 - I135) of the 4 intensities [..., 4], then
    ||(s1, s2)|| / s0."""
    s0 = 0.5 * data.sum(-1)
    s1, s2 = data[..., 0] - data[..., 2], data[..., 1] - data[..., 3]
    return torch.sqrt(s1 * s1 + s2 * s2) / s0


def angle_of_polarization(data: torch.Tensor) -> torch.Tensor:
    """to_aop (polarizer.py:118-134): 0.5 atan2(s2, s1 + 1e-7) wrapped into [0, pi]."""
    s1, s2 = data[..., 0] - data[..., 2], data[..., 1] - data[..., 3]
    aop = 0.5 * torch.atan2(s2, s1 + 1e-7)
    aop = torch.where(aop < 0, aop + np.pi, aop)
    return torch.clamp(aop, 0, np.pi)


def full_view_coords(frame: int, H: int, W: int, device) -> torch.Tensor:
    """Every pixel of one frame as [frame, y, x] int32 rows, row-major (the full-image dataloader's order)."""
    ys, xs = torch.meshgrid(torch.arange(H, device=device), torch.arange(W, device=device), indexing="ij")
    f = torch.full((H * W,), int(frame), device=device)
    return torch.stack([f, ys.reshape(-1), xs.reshape(-1)], -1).to(torch.int32)


class FullViewEvaluator:
    """Render full views of a BaseModel in chunks and score them.

    ``cameras``: per-modality DeviceCameras of the split being rendered; ``ray_generator``: a pipeline.RayGenerator
    (pose refinement applied as in training); ``mosaick``: per-modality [H, W] band masks for raw methods, or None."""

    def __init__(self, model, ray_generator: RayGenerator, height: int, width: int,
                 eval_num_rays_per_chunk: int = 2048, mosaick: Optional[Dict[str, torch.Tensor]] = None):
        self.model = model
        self.raygen = ray_generator
        self.H, self.W = int(height), int(width)
        self.chunk = int(eval_num_rays_per_chunk)
        self.mosaick = mosaick
        self.last_rays_per_sec = None

    @torch.no_grad()
    def query(self, coords: Dict[str, torch.Tensor]) -> Dict[str, Dict[str, torch.Tensor]]:
        """eval_model_query (eval_utils.py:31-76): chunked model calls, outputs concatenated per modality.  Sets
        ``last_rays_per_sec`` (EventName.TEST_RAYS_PER_SEC: all modalities' rays / wall time, device-synchronised)."""
        was_training = self.model.training
        self.model.eval()
        n = max(c.shape[0] for c in coords.values())
        parts: Dict[str, Dict[str, List[torch.Tensor]]] = {m: {} for m in coords}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        try:
            for i in range(0, n, self.chunk):
                chunk = {m: c[i:i + self.chunk] for m, c in coords.items() if c.shape[0] > i}
                rays = self.raygen(chunk)
                out = self.model(rays)
                for m in chunk:
                    o = out[m]
                    for k, v in o.items():
                        if isinstance(v, torch.Tensor) and v.dim() >= 1 and v.shape[0] == chunk[m].shape[0] and \
                                (k in PER_RAY_KEYS or k in self.model.spec.modalities):
                            parts[m].setdefault(k, []).append(v)
        finally:
            self.model.train(was_training)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        self.last_rays_per_sec = sum(c.shape[0] for c in coords.values()) / dt
        return {m: {k: torch.cat(v, 0) for k, v in p.items()} for m, p in parts.items()}

    @torch.no_grad()
    def render_view(self, frames: Dict[str, int]) -> Dict[str, Dict[str, torch.Tensor]]:
        """Evaluator.render_view (evaluator.py:100-178) for one frame per modality: images [H, W, C] per head plus
        depth / accumulation / normals; raw methods add 'mosaicked' [H, W, 1] (the modality's own band per pixel).
        RawEvaluator.generate_eval_renderings' extras (evaluator.py:621-700, eval_utils.py:77-160) under the key
        '_aligned': every head on the FIRST modality's view ('aligned' renderings), each raw head mosaicked with its
        modality's pattern over that view ('<head>:mosaicked'), and for polarization the degree / angle of
        polarization of the aligned rendering (polarizer.to_dop / to_aop, the angle divided by pi)."""
        dev = next(self.model.parameters()).device
        coords = {m: full_view_coords(f, self.H, self.W, dev) for m, f in frames.items()}
        flat = self.query(coords)
        out = {}
        for m, o in flat.items():
            img = {k: v.reshape(self.H, self.W, -1) for k, v in o.items()}
            if self.mosaick is not None:
                c = coords[m]
                band = self.mosaick[m][c[:, 1].long(), c[:, 2].long()].long()[:, None]
                img["mosaicked"] = select_right_channel(o[m], band).reshape(self.H, self.W, 1)
            out[m] = img
        first = next(iter(flat))
        heads = [h for h in self.model.spec.modalities if h in flat[first]]
        aligned = {h: out[first][h] for h in heads}
        if self.mosaick is not None:
            c = coords[first]
            for h in heads:
                band = self.mosaick[h][c[:, 1].long(), c[:, 2].long()].long()[:, None]
                aligned[f"{h}:mosaicked"] = select_right_channel(flat[first][h], band).reshape(self.H, self.W, 1)
        if "polarization" in aligned:
            aligned["degree_of_polarization"] = degree_of_polarization(aligned["polarization"])
            aligned["angle_of_polarization"] = angle_of_polarization(aligned["polarization"]) / np.pi
        out["_aligned"] = aligned
        return out

    def compute_metrics(self, renderings: Dict[str, Dict[str, torch.Tensor]], gt: Dict[str, torch.Tensor]):
        """Evaluator.compute_metrics (evaluator.py:431-440, eval_utils.py:325-394): PSNR and SSIM per modality (raw:
        mosaicked vs the raw frame)."""
        metrics = {}
        for m, r in renderings.items():
            if m.startswith("_"):
                continue
            img = r["mosaicked"] if "mosaicked" in r else r[m]
            metrics[m] = {"PSNR": psnr(img, gt[m]), "SSIM": ssim(img, gt[m])}
        return metrics


def eval_split(trainer, n_views: Optional[int] = None, eval_num_rays_per_chunk: int = 2048):
    """Render the synthetic scene's held-out views (scene.EVAL_VIEWS) with a trainer's model and pose refinement;
    returns ({mod: mean PSNR}, TEST_RAYS_PER_SEC averaged over views).  GT frames are rendered analytically like the
    training frames (scene.render_frames)."""
    cfg = trainer.cfg
    mods = trainer.modalities
    dev = trainer.device
    cams = mscene.make_cameras(mods, cfg.n_views, cfg.width, cfg.height, seed=0, train=False)
    dcams = {m: DeviceCameras(cams[m], dev) for m in mods}
    raygen = RayGenerator(dcams, trainer.pose, 0.0)
    ev = FullViewEvaluator(trainer.model, raygen, cfg.height, cfg.width, eval_num_rays_per_chunk,
                           trainer.masks if trainer.raw else None)
    C = cams[mods[0]].c2w.shape[0] if n_views is None else min(n_views, cams[mods[0]].c2w.shape[0])
    scores = {m: [] for m in mods}
    rates = []
    for v in range(C):
        gt = {m: mscene.render_frames(_one_view(cams[m], v), mscene.CHANNELS[m], dev,
                                      m if trainer.raw else None)[0] for m in mods}
        rend = ev.render_view({m: v for m in mods})
        for m, s in ev.compute_metrics(rend, gt).items():
            scores[m].append(s["PSNR"])
        rates.append(ev.last_rays_per_sec)
    return {m: sum(v) / len(v) for m, v in scores.items()}, sum(rates) / len(rates)


def _one_view(cams: mscene.ModalityCameras, v: int) -> mscene.ModalityCameras:
    return mscene.ModalityCameras(cams.c2w[v:v + 1], cams.fx[v:v + 1], cams.fy[v:v + 1], cams.cx[v:v + 1],
                                  cams.cy[v:v + 1], cams.distortion[v:v + 1], cams.width, cams.height,
                                  cams.view_ids[v:v + 1])
