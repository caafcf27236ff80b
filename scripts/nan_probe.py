"""Eager training steps of the bench workload under a precision preset, checking every parameter and gradient for
non-finite values after each step (the first step and tensor that go bad, and the largest |grad| per tensor).

    python scripts/nan_probe.py fast_h16c [steps] [graph]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from multimodalstudio_amd import functions as fx
    from multimodalstudio_amd.pipeline import Trainer, TrainConfig, skip_views_for
    prec = sys.argv[1] if len(sys.argv) > 1 else "fast_h16c"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    fx.set_precision(prec)
    dev = torch.device("cuda", 0)
    cfg = TrainConfig(method="grid", modalities=["rgb"], num_rays_per_modality=2048, log2T=19,
                      skip_views=skip_views_for("grid"), gpu_sampler=True)
    t = Trainer(cfg, dev, rank=0)
    t.set_step(95000)
    params = [(n, p) for n, p in t.model.named_parameters()]
    if getattr(t, "poses", None) is not None:
        params += [(f"pose{i}", p) for i, p in enumerate(t.poses.params)]
    runner = None
    if len(sys.argv) > 3 and sys.argv[3] == "graph":
        from multimodalstudio_amd.graphs import GraphTrainer
        runner = GraphTrainer(t)
    for s in range(steps):
        if runner is not None:
            losses, total = runner.step()
        else:
            losses, total, _ = t.train_step()
        torch.cuda.synchronize()
        if runner is not None:
            print(f"  graph stats {runner.stats}", flush=True)
        bad = [n for n, p in params if not bool(torch.isfinite(p).all())]
        badg = [n for n, p in params if p.grad is not None and not bool(torch.isfinite(p.grad).all())]
        gmax = max((float(p.grad.abs().max()) for n, p in params if p.grad is not None and p.grad.numel()), default=0.0)
        print(f"step {s}: loss {float(total):.6g} max|grad| {gmax:.3e} bad params {bad[:4]} bad grads {badg[:4]}",
              flush=True)
        if bad or badg or not bool(torch.isfinite(total)):
            break


if __name__ == "__main__":
    main()
