"""Probe: GraphTrainer capture in 2 concurrent processes on one GPU, with / without a gloo group and collectives."""
import faulthandler
import os
import sys

import torch
import torch.distributed as dist

faulthandler.enable()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodalstudio_amd import ddp as mddp  # noqa: E402
from multimodalstudio_amd import graphs  # noqa: E402
from multimodalstudio_amd.pipeline import TrainConfig, Trainer  # noqa: E402

variant = sys.argv[1]
rank = int(os.environ["RANK"])
dev = torch.device("cuda", 0)
ddp = None
if variant != "nopg":
    dist.init_process_group("gloo")
    ddp = mddp.DDP(2)
if variant == "cudacoll":
    x = torch.ones(1000, device=dev)
    dist.all_reduce(x)
    torch.cuda.synchronize()
if variant == "cpucoll":
    x = torch.ones(1000)
    dist.all_reduce(x)
t = Trainer(TrainConfig(method="grid_raw", modalities=("rgb", "polarization"), num_rays_per_modality=256, log2T=14,
                        width=64, height=48), dev, rank=rank)
t.set_step(95000)
g = graphs.GraphTrainer(t, ddp=ddp if variant != "nopg" else None)
for i in range(4):
    g.step()
torch.cuda.synchronize()
print("OK", variant, rank, g.stats, flush=True)
