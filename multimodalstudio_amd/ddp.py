"""Ray-batch data parallelism: one process per GPU, gradient all-reduce over RCCL (torch.distributed 'nccl').

Reference: Lightning Fabric DDP (/root/reference/src/engine/trainer.py:57-63) averages every model
gradient inside fabric.backward (raw_pipeline.py:77).  Here each optimizer group's gradients already sit
in one flat buffer (pipeline.FlatGroup), so the exchange is a few large all-reduces — sized for xGMI ring
bandwidth instead of per-tensor buckets — and the camera-pose gradients are averaged too (documented
deviation: the reference's pose grads stay rank-local).
"""
from __future__ import annotations

import os
from typing import List

import torch
import torch.distributed as dist


def init_from_env(backend: str = "nccl"):
    """Initialise from torchrun's RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* environment."""
    if not dist.is_available() or "WORLD_SIZE" not in os.environ or int(os.environ["WORLD_SIZE"]) <= 1:
        return None
    if not dist.is_initialized():
        dist.init_process_group(backend=backend)
    return DDP(dist.get_world_size())


class DDP:
    def __init__(self, world_size: int, bucket_bytes: int = 256 << 20):
        self.world = world_size
        self.bucket = bucket_bytes // 4

    def allreduce_grads(self, groups: List) -> None:
        """Average flat gradient buffers across ranks (in place), in buckets of <= bucket_bytes."""
        if self.world <= 1:
            return
        for g in groups:
            buf = g.grad
            n = buf.numel()
            for off in range(0, n, self.bucket):
                chunk = buf[off: off + self.bucket]
                dist.all_reduce(chunk, op=dist.ReduceOp.SUM)
            buf.mul_(1.0 / self.world)

    def max_over_ranks(self, value: float, device) -> float:
        t = torch.tensor([value], dtype=torch.float64, device=device)
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def barrier(self):
        if self.world > 1:
            dist.barrier()
