"""ORACLE (test infrastructure only) — ray generation, collider, samplers.

Restates (paths under /root/reference/src):
  exp_map_SO3xR3                      cameras/lie_groups.py:28-63
  CameraOptimizer.forward (shared)    cameras/camera_optimizers.py:86-119
  pose_utils.multiply                 utils/poses.py:53-67
  Cameras._generate_rays_from_coords  cameras/cameras.py:460-703 (perspective only)
  radial_and_tangential_undistort     cameras/camera_utils.py:280-383 (params read [k1,k2,k3,k4,p1,p2])
  SphereCollider.forward              model_components/scene_colliders.py:60-80
  update_ray_bundles_for_background   model_components/scene_colliders.py:107-113
  SpacedSampler.generate_ray_samples  model_components/ray_samplers.py:183-233 (uniform / disparity)
  PDFSampler.generate_ray_samples     model_components/ray_samplers.py:316-422
  merge_ray_samples                   model_components/ray_samplers.py:38-68
  NeuSSampler.generate_ray_samples    model_components/ray_samplers.py:448-514
  rendering_sdf_with_fixed_inv_s      model_components/ray_samplers.py:516-551
  RaySamples.get_weights_from_alphas  cameras/rays.py:201-217

Random draws are injected: every sampler takes its uniforms as an argument.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Dict, List, Optional

import torch
import torch.nn.functional as F


# ------------------------------------------------------------------------------------------------
# ray generation
# ------------------------------------------------------------------------------------------------
def exp_map_so3xr3(tangent: torch.Tensor) -> torch.Tensor:
    """lie_groups.py:28-63: tangent [B, 6] (t, omega) -> [B, 3, 4]."""
    log_rot = tangent[:, 3:]
    nrms = (log_rot * log_rot).sum(1)
    ang = torch.clamp(nrms, 1e-4).sqrt()
    inv = 1.0 / ang
    fac1 = inv * ang.sin()
    fac2 = inv * inv * (1.0 - ang.cos())
    B = tangent.shape[0]
    zero = torch.zeros(B, dtype=tangent.dtype)
    wx, wy, wz = log_rot[:, 0], log_rot[:, 1], log_rot[:, 2]
    skew = torch.stack([zero, -wz, wy, wz, zero, -wx, -wy, wx, zero], -1).view(B, 3, 3)
    skew2 = torch.bmm(skew, skew)
    R = fac1[:, None, None] * skew + fac2[:, None, None] * skew2 + torch.eye(3, dtype=tangent.dtype)[None]
    return torch.cat([R, tangent[:, :3, None]], dim=-1)


def pose_multiply(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """poses.py:53-67: A @ B for [.., 3, 4] poses."""
    R1, t1 = a[..., :3, :3], a[..., :3, 3:]
    R2, t2 = b[..., :3, :3], b[..., :3, 3:]
    return torch.cat([R1.matmul(R2), t1 + R1.matmul(t2)], dim=-1)


def _residual_and_jacobian(x, y, xd, yd, dp):
    """camera_utils.py:280-343."""
    k1, k2, k3, k4, p1, p2 = (dp[..., i] for i in range(6))
    r = x * x + y * y
    d = 1.0 + r * (k1 + r * (k2 + r * (k3 + r * k4)))
    fx = d * x + 2 * p1 * x * y + p2 * (r + 2 * x * x) - xd
    fy = d * y + 2 * p2 * x * y + p1 * (r + 2 * y * y) - yd
    d_r = k1 + r * (2.0 * k2 + r * (3.0 * k3 + r * 4.0 * k4))
    d_x = 2.0 * x * d_r
    d_y = 2.0 * y * d_r
    fx_x = d + d_x * x + 2.0 * p1 * y + 6.0 * p2 * x
    fx_y = d_y * x + 2.0 * p1 * x + 2.0 * p2 * y
    fy_x = d_x * y + 2.0 * p2 * y + 2.0 * p1 * x
    fy_y = d + d_y * y + 2.0 * p2 * x + 6.0 * p1 * y
    return fx, fy, fx_x, fx_y, fy_x, fy_y


def undistort(coords: torch.Tensor, dp: torch.Tensor, eps: float = 1e-3, iters: int = 10) -> torch.Tensor:
    """camera_utils.py:346-383 (Newton iterations on the distorted coords)."""
    x, y = coords[..., 0], coords[..., 1]
    for _ in range(iters):
        fx, fy, fx_x, fx_y, fy_x, fy_y = _residual_and_jacobian(x, y, coords[..., 0], coords[..., 1], dp)
        den = fy_x * fx_y - fx_x * fy_y
        xn = fx * fy_y - fy * fx_y
        yn = fy * fx_x - fx * fy_x
        ok = torch.abs(den) > eps
        x = x + torch.where(ok, xn / den, torch.zeros_like(den))
        y = y + torch.where(ok, yn / den, torch.zeros_like(den))
    return torch.stack([x, y], dim=-1)


@dataclass
class Rays:
    origins: torch.Tensor
    directions: torch.Tensor
    up: torch.Tensor
    pixel_area: torch.Tensor
    directions_norm: torch.Tensor
    camera_indices: torch.Tensor


def generate_rays(coords_fyx: torch.Tensor, fx, fy, cx, cy, c2w, distortion: Optional[torch.Tensor],
                  pose_adjustment: Optional[torch.Tensor], pixel_offset: float = 0.0) -> Rays:
    """RayGenerator.forward + Cameras.generate_rays (ray_generators.py:54-81; cameras.py:460-703).

    coords_fyx: int [N, 3] = (frame index, y, x); fx.. per-camera [C]; c2w [C, 3, 4]; distortion [C, 6] or None;
    pose_adjustment: [1, 6] shared SO3xR3 delta (camera_optimizers.py:108-112) or None (mode off).
    """
    c = coords_fyx[:, 0].long()
    yy = coords_fyx[:, 1].long().to(torch.float32) + pixel_offset
    xx = coords_fyx[:, 2].long().to(torch.float32) + pixel_offset
    N = c.shape[0]
    if pose_adjustment is not None:
        params = pose_adjustment.expand((c2w.shape[0], 6))[c]
        mat = exp_map_so3xr3(params)
    else:
        mat = torch.eye(4)[None, :3, :4].tile(N, 1, 1)
    fxr, fyr, cxr, cyr = fx[c], fy[c], cx[c], cy[c]
    coord = torch.stack([(xx - cxr) / fxr, -(yy - cyr) / fyr], -1)
    cxo = torch.stack([(xx - cxr + 1) / fxr, -(yy - cyr) / fyr], -1)
    cyo = torch.stack([(xx - cxr) / fxr, -(yy - cyr + 1) / fyr], -1)
    stack = torch.stack([coord, cxo, cyo], dim=0)
    if distortion is not None:
        stack = undistort(stack.reshape(3, -1, 2), distortion[c]).reshape(3, N, 2)
    dirs = torch.empty(3, N, 3)
    dirs[..., 0] = stack[..., 0]
    dirs[..., 1] = stack[..., 1]
    dirs[..., 2] = -1.0
    pose = pose_multiply(c2w[c], mat)
    R = pose[..., :3, :3]
    dirs = torch.sum(dirs[..., None, :] * R, dim=-1)
    dnorm = torch.norm(dirs, dim=-1, keepdim=True)[0]
    dirs = F.normalize(dirs, dim=-1)
    origins = pose[..., :3, 3]
    d = dirs[0]
    up = (pose[..., :3] @ torch.tensor([0.0, 1.0, 0.0]).expand_as(d)[..., None]).squeeze(-1)
    dx = torch.sqrt(torch.sum((d - dirs[1]) ** 2, dim=-1))
    dy = torch.sqrt(torch.sum((d - dirs[2]) ** 2, dim=-1))
    return Rays(origins, d, up, (dx * dy)[..., None], dnorm, c[:, None])


# ------------------------------------------------------------------------------------------------
# collider
# ------------------------------------------------------------------------------------------------
def sphere_collider(origins, directions, radius: float = 1.0):
    """scene_colliders.py:60-80 -> nears [N,1], fars [N,1], mask [N]."""
    dot = (directions * origins).sum(dim=-1, keepdims=True)
    under = dot ** 2 - (origins.norm(p=2, dim=-1, keepdim=True) ** 2 - radius ** 2)
    mask = (under > 0.01).squeeze(dim=-1)
    under = under.clamp_min(0.01)
    inter = torch.sqrt(under) * torch.tensor([-1.0, 1.0]) - dot
    inter = inter.clamp_min(0.01)
    return inter[:, 0:1], inter[:, 1:2], mask


def background_near_far(origins, directions, radius: float = 1.0):
    """scene_colliders.py:107-113: hit rays start at the far intersection; far += 3 for all rays."""
    nears, fars, mask = sphere_collider(origins, directions, radius)
    nears = nears.clone()
    nears[mask] = fars[mask]
    fars = torch.ones_like(fars) * fars + 3.0
    return nears, fars


# ------------------------------------------------------------------------------------------------
# samples
# ------------------------------------------------------------------------------------------------
@dataclass
class Samples:
    """RaySamples subset used by the hot path (rays.py:94-122, 304-349)."""
    spacing_bins: torch.Tensor        # [R, S+1] in [0,1] (detached)
    starts: torch.Tensor              # [R, S, 1] euclidean
    ends: torch.Tensor                # [R, S, 1]
    kind: str                         # "uniform" | "disparity"

    @property
    def deltas(self):
        return self.ends - self.starts


def spacing_to_euclidean(bins, nears, fars, kind: str):
    """SpacedSampler.spacing_to_euclidean_fn (ray_samplers.py:178-181)."""
    if kind == "uniform":
        return fars * bins + nears * (1 - bins)
    s_near, s_far = 1 / nears, 1 / fars
    return 1 / (s_far * bins + s_near * (1 - bins))


def make_samples(bins, nears, fars, kind) -> Samples:
    bins = bins.detach()
    e = spacing_to_euclidean(bins, nears, fars, kind)
    return Samples(bins, e[..., :-1, None], e[..., 1:, None], kind)


def stratified_bins(num_rays: int, num_samples: int, t_rand: Optional[torch.Tensor]):
    """ray_samplers.py:209-221: jittered linspace; t_rand [R,1] (single jitter) or [R,S+1]."""
    bins = torch.linspace(0.0, 1.0, num_samples + 1)[None, ...]
    if t_rand is None:
        return bins.expand(num_rays, -1)
    centers = (bins[..., 1:] + bins[..., :-1]) / 2.0
    upper = torch.cat([centers, bins[..., -1:]], -1)
    lower = torch.cat([bins[..., :1], centers], -1)
    return lower + (upper - lower) * t_rand


def positions(origins, directions, starts):
    """Frustums.get_start_positions (rays.py:69-81): o + d * start."""
    return origins[:, None, :] + directions[:, None, :] * starts


def weights_from_alphas(alphas: torch.Tensor) -> torch.Tensor:
    """rays.py:201-217: alphas [R,S,1] -> weights [R,S,1]."""
    T = torch.cumprod(torch.cat([torch.ones((*alphas.shape[:1], 1, 1)), 1.0 - alphas + 1e-7], 1), 1)
    return alphas * T[:, :-1, :]


def fixed_inv_s_alpha(sdf: torch.Tensor, deltas: torch.Tensor, inv_s: float) -> torch.Tensor:
    """rendering_sdf_with_fixed_inv_s (ray_samplers.py:516-551): sdf [R,S], deltas [R,S] -> alpha [R,S-1]."""
    R = sdf.shape[0]
    prev, nxt = sdf[:, :-1], sdf[:, 1:]
    dl = deltas[:, :-1]
    mid = (prev + nxt) * 0.5
    cos = (nxt - prev) / (dl + 1e-5)
    prev_cos = torch.cat([torch.zeros([R, 1]), cos[:, :-1]], dim=-1)
    cos = torch.stack([prev_cos, cos], dim=-1)
    cos, _ = torch.min(cos, dim=-1, keepdim=False)
    cos = cos.clip(-1e3, 0.0)
    pe = mid - cos * dl * 0.5
    ne = mid + cos * dl * 0.5
    pc = torch.sigmoid(pe * inv_s)
    nc = torch.sigmoid(ne * inv_s)
    return (pc - nc + 1e-5) / (pc + 1e-5)


def pdf_bins(existing_bins: torch.Tensor, weights: torch.Tensor, num_samples: int, rand: Optional[torch.Tensor],
             padding: float = 1e-5, eps: float = 1e-5) -> torch.Tensor:
    """PDFSampler.generate_ray_samples (ray_samplers.py:357-403), include_original=False, single jitter.

    existing_bins [R, S+1]; weights [R, S] ; rand [R, 1] in [0,1) or None (eval midpoints) -> bins [R, num_samples+1].
    """
    num_bins = num_samples + 1
    w = weights + padding
    wsum = torch.sum(w, dim=-1, keepdim=True)
    pad = torch.relu(eps - wsum)
    w = w + pad / w.shape[-1]
    wsum = wsum + pad
    pdf = w / wsum
    cdf = torch.min(torch.ones_like(pdf), torch.cumsum(pdf, dim=-1))
    cdf = torch.cat([torch.zeros_like(cdf[..., :1]), cdf], dim=-1)
    if rand is not None:
        u = torch.linspace(0.0, 1.0 - (1.0 / num_bins), steps=num_bins)
        u = u.expand(size=(*cdf.shape[:-1], num_bins))
        u = u + rand / num_bins
    else:
        u = torch.linspace(0.0, 1.0 - (1.0 / num_bins), steps=num_bins) + 1.0 / (2 * num_bins)
        u = u.expand(size=(*cdf.shape[:-1], num_bins))
    u = u.contiguous()
    inds = torch.searchsorted(cdf, u, side="right")
    below = torch.clamp(inds - 1, 0, existing_bins.shape[-1] - 1)
    above = torch.clamp(inds, 0, existing_bins.shape[-1] - 1)
    cdf_g0 = torch.gather(cdf, -1, below)
    bins_g0 = torch.gather(existing_bins, -1, below)
    cdf_g1 = torch.gather(cdf, -1, above)
    bins_g1 = torch.gather(existing_bins, -1, above)
    t = torch.clip(torch.nan_to_num((u - cdf_g0) / (cdf_g1 - cdf_g0), 0), 0, 1)
    return bins_g0 + t * (bins_g1 - bins_g0)


def merge_bins(bins1: torch.Tensor, bins2: torch.Tensor):
    """merge_ray_samples (ray_samplers.py:38-68) on spacing bins: returns merged bins and sorted_index."""
    starts1, starts2 = bins1[..., :-1], bins2[..., :-1]
    ends = torch.maximum(bins1[..., -1:], bins2[..., -1:])
    merged, sorted_index = torch.sort(torch.cat([starts1, starts2], -1), dim=-1, stable=True)
    return torch.cat([merged, ends], dim=-1).detach(), sorted_index


def neus_sample(nears, fars, origins, directions, sdf_fn: Callable, t_rand: Optional[torch.Tensor],
                pdf_rands: Optional[List[torch.Tensor]], num_samples=32, num_importance=32, upsample_steps=4,
                base_variance=64.0):
    """NeuSSampler.generate_ray_samples for one modality's hit rays (ray_samplers.py:464-514).

    sdf_fn(points [R, n, 3]) -> sdf [R, n] evaluated under no_grad.  Returns final spacing bins [R, S+1]
    plus the per-iteration sorted indices (for bit-exact checks).
    """
    R = nears.shape[0]
    bins = stratified_bins(R, num_samples, t_rand).detach()
    smp = make_samples(bins, nears, fars, "uniform")
    new_smp = smp
    sdf = None
    sorted_index = None
    history = []
    n_new = num_importance // upsample_steps
    for it in range(upsample_steps):
        with torch.no_grad():
            new_sdf = sdf_fn(positions(origins, directions, new_smp.starts).detach())
        if sorted_index is not None:
            sdf = torch.gather(torch.cat([sdf, new_sdf], -1), 1, sorted_index)
        else:
            sdf = new_sdf
        with torch.no_grad():
            alphas = fixed_inv_s_alpha(sdf, smp.deltas[..., 0], base_variance * 2 ** it)
            w = weights_from_alphas(alphas[..., None])
            w = torch.cat((w, torch.zeros_like(w[:, :1])), dim=1)
        nb = pdf_bins(smp.spacing_bins, w[..., 0], n_new, None if pdf_rands is None else pdf_rands[it])
        new_smp = make_samples(nb, nears, fars, "uniform")
        merged, sorted_index = merge_bins(smp.spacing_bins, nb)
        history.append(sorted_index)
        smp = make_samples(merged, nears, fars, "uniform")
    return smp, history
