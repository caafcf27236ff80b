"""Autograd fan-in of one training step's graph (diagnostics): every node that receives gradients from two or more
consumers costs an ATen add launch per step; list them with their consumers."""
import collections
import sys

import torch

sys.path.insert(0, ".")
from multimodalstudio_amd import functions as fx  # noqa: E402
from multimodalstudio_amd.pipeline import TrainConfig, Trainer, compute_loss  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    fx.set_precision("fast")
    tr = Trainer(TrainConfig(method="grid", modalities=("rgb",), num_rays_per_modality=2048, log2T=19,
                             gpu_sampler=True), dev)
    tr.set_step(95000)
    from multimodalstudio_amd.graphs import GraphTrainer, bucket_capacity
    g = GraphTrainer(tr)
    for _ in range(3):
        tr.train_step()
    torch.cuda.synchronize()
    g._stage_inputs()
    counts = g.hit_counts()
    cap = bucket_capacity(counts, g.granule, g.n)
    targets = g._targets()
    fx.zero_arena_begin(dev)
    rays = tr.raygen(g.coords)
    fx.reset_grad_uses()
    outputs = tr.model(rays, None, cap=cap)
    losses, total = compute_loss(outputs, targets, tr.modalities, tr.step, max_iters=tr.cfg.max_iters)
    fanin = collections.defaultdict(list)
    seen, stack = set(), [total.grad_fn]
    while stack:
        n = stack.pop()
        if n is None or n in seen:
            continue
        seen.add(n)
        for nxt, nr in n.next_functions:
            if nxt is not None:
                fanin[(nxt, nr)].append(n.name())
                stack.append(nxt)
    print(f"{len(seen)} autograd nodes")
    for (n, nr), srcs in sorted(fanin.items(), key=lambda kv: -len(kv[1])):
        if len(srcs) > 1:
            extra = ""
            if n.name() == "torch::autograd::AccumulateGrad":
                extra = f" param {tuple(n.variable.shape)}"
            else:
                try:
                    extra = f" shape {n._input_metadata[nr].shape}"
                except Exception:
                    pass
            print(f"{len(srcs) - 1} add(s): {n.name()} output {nr}{extra}  from {collections.Counter(srcs).most_common()}")
    fx.zero_arena_end()


if __name__ == "__main__":
    main()
