"""Two-rank check of the real data-parallel training paths, run by tests/test_gpu_ddp.py as
``python -m torch.distributed.run --nproc-per-node 2 tests/ddp_check.py <out.json> [precision]`` (both ranks on
cuda:0, gloo collectives: RCCL needs one GPU per rank; precision: a functions.PRESETS name, fp32 by default).  Not a
pytest module.

0. GraphTrainer(ddp) x 5 (graph replays: the radiance and background tables' all-reduce launched after the backward's
   first phase, overlapping the SDF backward graph, the SDF table's after the second, overlapping the deferred weight
   gradients, the rest after them): averaged gradients, parameters identical on both ranks, the regions launched in
   that order, and the steps were replayed.
1. Trainer.compute_grads(ddp) -- hash-table gradients all-reduced while the backward still runs, the rest after --
   equals the average of the two ranks' local gradients (local pass = same batch, same device RNG seed, no ddp).
2. Trainer.train_step(ddp) x 2: parameters identical on both ranks.
"""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def gather(t):
    parts = [torch.empty_like(t.cpu()) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t.detach().cpu().contiguous())
    return parts


def log(msg):
    print(f"[rank {os.environ.get('RANK')}] {msg}", flush=True)


def main():
    import faulthandler
    faulthandler.enable()
    out_path = sys.argv[1]
    precision = sys.argv[2] if len(sys.argv) > 2 else "fp32"
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from multimodalstudio_amd import ddp as mddp
    from multimodalstudio_amd import functions as fx
    from multimodalstudio_amd.graphs import GraphTrainer
    from multimodalstudio_amd.pipeline import TrainConfig, Trainer
    fx.set_precision(precision)
    # config 5's method: three hash tables (surface, radiance, grid background) -- the radiance and background tables'
    # all-reduce goes out after the backward's first phase, the surface table's after its second
    cfg = TrainConfig(method="grid_raw_grid_bg_unbalanced", modalities=("rgb", "polarization"),
                      num_rays_per_modality=256, log2T=14, width=64, height=48)
    ddp = mddp.DDP(world, bucket_bytes=1 << 20)
    res = {"world": world}
    # graph-replayed data-parallel steps on a fresh trainer (as bench.py drives it: no eager default-stream steps
    # before the captures)
    tg = Trainer(cfg, dev, rank=rank)
    tg.set_step(95000)
    g = GraphTrainer(tg, ddp=ddp)
    # the graph path's exchange: the local gradients the replayed forward/backward graph left, and what the
    # all-reduce between the two graphs made of them
    # (split path: the hash-table regions are launched while the second backward graph replays, so their local values
    # are snapshotted at launch -- ordered before the collective on the stream -- and the rest when the exchange
    # finishes the step)
    seen = {"local": [], "reduced": [], "early": [], "overlapped": 0, "stage_ok": True}
    orig_ready, orig_finish = ddp.grad_ready, ddp.finish_step

    in_graph = [False]
    orig_ox = ddp.overlap_exchange

    def spy_ox(stages, groups):
        in_graph[0] = True
        try:
            orig_ox(stages, groups)
        finally:
            in_graph[0] = False
    ddp.overlap_exchange = spy_ox

    def spy_ready(grad, groups):
        # replayed steps: the surface table goes out second (after the backward's second phase), the others first
        names = [n for n, p in tg.model.named_parameters() if p.grad is not None and p.grad.data_ptr() == grad.data_ptr()]
        second = bool(names) and names[0].startswith("surface_model.")
        early_second = [e for e in seen["early"] if e[2]]
        if in_graph[0] and not second and early_second:
            seen["stage_ok"] = False
        seen["early"].append((grad.data_ptr(), grad.detach().reshape(-1).clone(), second))
        orig_ready(grad, groups)

    def spy_finish(groups):
        local = [gr.grad.clone() for gr in groups]
        for ptr, early, _ in seen["early"]:
            for gr, lg in zip(groups, local):
                off = (ptr - gr.grad.data_ptr()) // 4
                if 0 <= off < gr.grad.numel():
                    lg[off:off + early.numel()] = early
        seen["overlapped"] += len(seen["early"])
        seen["early"] = []
        seen["local"].append(local)
        orig_finish(groups)
        seen["reduced"].append([gr.grad.clone() for gr in groups])

    ddp.grad_ready, ddp.finish_step = spy_ready, spy_finish
    for _ in range(5):
        g.step()
    torch.cuda.synchronize()
    ddp.grad_ready, ddp.finish_step = orig_ready, orig_finish
    ddp.overlap_exchange = orig_ox
    if seen["local"]:
        errs = []
        for local, red in zip(seen["local"], seen["reduced"]):
            for lg, rg in zip(local, red):
                mean = sum(gather(lg)) / world
                errs.append(float((rg.cpu() - mean).abs().max()) / max(float(mean.abs().max()), 1e-30))
        res["graph_grad_err"] = max(errs)
        res["graph_allreduces"] = len(seen["local"])
        res["graph_overlapped_regions"] = seen["overlapped"]
        res["graph_stage_order_ok"] = seen["stage_ok"]
    p = gather(tg.fields.flat)
    q = gather(tg.poses.flat)
    res["graph_params_equal"] = bool(torch.equal(p[0], p[1]) and torch.equal(q[0], q[1]))
    res["graph_stats"] = g.stats
    res["graph_disabled"] = g.disabled
    log("graph steps")
    del g, tg
    # 1. averaged gradients
    t = Trainer(cfg, dev, rank=rank)
    t.set_step(95000)
    coords, sel = t.sampler.sample(t.frames)
    targets = t.targets_for(coords, sel)
    t.model.seed_draws(100 + rank, dev)
    t.compute_grads(coords, targets)
    local = t.fields.grad.clone()
    local_pose = t.poses.grad.clone()
    log("local grads")
    t.model.seed_draws(100 + rank, dev)
    t.compute_grads(coords, targets, ddp=ddp)
    torch.cuda.synchronize()
    log("reduced grads")
    mean = sum(gather(local)) / world
    mean_pose = sum(gather(local_pose)) / world
    red = t.fields.grad.cpu()
    scale = float(mean.abs().max())
    res["grad_err"] = float((red - mean).abs().max()) / scale
    res["pose_grad_err"] = float((t.poses.grad.cpu() - mean_pose).abs().max()) / max(float(mean_pose.abs().max()), 1e-30)
    res["grads_differ_across_ranks"] = float((gather(local)[0] - gather(local)[1]).abs().max()) / scale
    res["reduced_equal_across_ranks"] = bool(torch.equal(*gather(t.fields.grad)))
    # 2. eager data-parallel steps
    for _ in range(2):
        t.train_step(ddp=ddp)
    torch.cuda.synchronize()
    p = gather(t.fields.flat)
    res["eager_params_equal"] = bool(torch.equal(p[0], p[1]))
    log("eager steps")
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
