#!/usr/bin/env python
"""Train-rays/s benchmark of the MMS hot path on MI355X (BASELINE.json metric, configs[1] by default).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config grid_rgb|grid_raw5] [--rays R]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = one full training iteration of RawPipeline/BasePipeline.train_step on synthetic data of the
MMS-DATA shape: host pixel sampling (reference RNG), ray generation with SO3xR3 pose refinement, the
collider, the 4-iteration NeuS sampler, hash grids, SDF MLP with 4 numerical-gradient taps, radiance
MLP, heads, background NeRF, NeuS compositing, losses, backward, grad clipping, AdamW.  Random-init
weights; model state at step 95000 (all 16 grid levels active).  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (method, modalities, workload description)
    "grid_rgb": ("grid", ("rgb",), "confs/grid.yaml, RGB-only (modalities: [rgb]), hash grid + MLPs, 1 GPU"),
    "grid_raw5": ("grid_raw", ("rgb", "infrared", "mono", "polarization", "multispectral"),
                  "confs/grid_raw.yaml, 5-modality mosaicked, per-modality heads"),
}

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
F32_MFMA_PEAK_TF = 157.3   # dense f32-input MFMA (v_mfma_f32_32x32x2_f32) peak, MI355X_MICROARCH.md
BF16_MFMA_PEAK_TF = 2500.0  # dense bf16 MFMA peak (no sparsity), MI355X_MICROARCH.md
# split-bf16x3 runs 3 bf16 MFMAs per f32 product: its ceiling for the algorithmic 2MNK flops is a third
MFMA_PEAK_TF = {"fp32": F32_MFMA_PEAK_TF, "bf16": BF16_MFMA_PEAK_TF, "bf16x3": BF16_MFMA_PEAK_TF / 3}
PREC_NAMES = {0: "fp32", 1: "bf16", 2: "bf16x3"}
DTYPES = {"fp32": "fp32", "fast": "bf16 MFMA (fp32 accumulate; SDF MLP split-bf16x3), fp32 elsewhere",
          "bf16x3": "split-bf16x3 MFMA (fp32-accurate), fp32 elsewhere"}
HASH_FWD_B = 16 * 8 * 2 * 4 + 12 + 128          # bytes per lookup, forward
HASH_BWD_B = 128 + 12 + 16 * 8 * 2 * (4 + 4)    # bytes per lookup, backward (table grads)


def gemm_work(a):
    """(precision label, (algorithmic flops, algorithmic HBM bytes)) of one mms_gemm launch (argument order of
    include/mms_hip.h): 2MNK flops; bytes = operands once + C written (+ Z, aux, read-modify-write)."""
    prec, M, N, K = a[0], a[3], a[4], a[5]
    Z, aux, accumulate, splits = a[13], a[15], a[21], a[22]
    mn = float(M) * N
    nbytes = 4.0 * (float(M) * K + float(N) * K + mn * (1 + (Z is not None) + (aux is not None) +
                                                         (bool(accumulate) and splits <= 1)))
    mode = {(0, 0): "NT", (0, 1): "NN", (1, 1): "TN"}.get((a[1], a[2]), "??")
    return f"{PREC_NAMES[prec]}:{mode}", (2.0 * M * N * K, nbytes)


def chain_work(a):
    """(precision label, (algorithmic flops, algorithmic HBM bytes)) of one mms_mlp_chain launch (include/mms_hip.h
    argument order): the three layers' 2MNK, narrowed on the SDF tap rows (rows >= rows_full: one output column of
    the last forward layer, one input column of the first backward layer); bytes = input rows + the stores each
    layer makes (+ the forward outputs the backward reads for its activation derivatives)."""
    import ctypes
    prec, bwd, K0, M, rf = a[0], a[1], a[4], a[5], a[6]
    rf = M if rf < 0 else min(rf, M)
    N = ctypes.cast(a[19], ctypes.POINTER(ctypes.c_int))
    outs = ctypes.cast(a[17], ctypes.POINTER(ctypes.c_void_p))
    n0, n1, n2 = N[0], N[1], N[2]
    st = [outs[i] is not None for i in range(3)]
    if bwd:
        flops = 2.0 * (rf * K0 + (M - rf)) * n0 + 2.0 * M * (n0 * n1 + n1 * n2)
        nbytes = 4.0 * ((rf * K0 + (M - rf)) + M * (n0 * st[0] + n1 * st[1] + n2 * st[2]) + M * (n0 + n1))
    else:
        flops = 2.0 * M * (K0 * n0 + n0 * n1) + 2.0 * (rf * n2 + (M - rf)) * n1
        nbytes = 4.0 * (M * K0 + M * (n0 * st[0] + n1 * st[1]) + (rf * n2 + (M - rf)) * st[2])
    return f"{PREC_NAMES[prec]}:chain{'_bwd' if bwd else '_fwd'}", (flops, nbytes)


def work_fns():
    return {
        "mms_gemm": gemm_work,
        "mms_mlp_chain": chain_work,
        "mms_hashgrid_fwd": lambda a: float(a[1]) * HASH_FWD_B,
        "mms_hashgrid_bwd_grouped": lambda a: float(a[1]) * a[2] * HASH_BWD_B,
    }


def cpu_baseline(trainer, cfg, seconds: float):
    """The fixture-pinned CPU restatement (oracle/) of the same workload, bounded sample, on host cores."""
    from oracle.train import OracleTrainer
    from multimodalstudio_amd import scene as ms
    mods = list(cfg.modalities)
    channels = {m: ms.CHANNELS[m] for m in mods}
    sd = {k: v.detach().cpu() for k, v in trainer.model.state_dict().items()}
    ot = OracleTrainer(sd, channels, trainer.host_cams, cfg.log2T, trainer.step, raw=False)
    n_rays = 256
    g = torch.Generator().manual_seed(1)

    def batch():
        coords, targets = {}, {}
        for m in mods:
            cams = trainer.host_cams[m]
            C = cams.c2w.shape[0]
            c = torch.stack([torch.randint(0, C, (n_rays,), generator=g), torch.randint(0, cfg.height, (n_rays,),
                            generator=g), torch.randint(0, cfg.width, (n_rays,), generator=g)], -1).to(torch.int32)
            coords[m] = c
            targets[m] = torch.rand(n_rays, channels[m], generator=g)
        return coords, targets

    ot.train_step(*batch())   # warmup
    times = []
    t_start = time.perf_counter()
    while (time.perf_counter() - t_start < seconds and len(times) < 50) or len(times) < 3:
        c, t = batch()
        t0 = time.perf_counter()
        ot.train_step(c, t)
        times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    return {
        "value": round(n_rays * len(mods) / med, 2),
        "unit": "rays/s",
        "cores": torch.get_num_threads(),
        "kind": "port",
        "sample": f"{len(times)} timed steps (median) of the CPU restatement (oracle/, bit-exact to the reference "
                  f"torch path) at {n_rays} rays/modality, same config, log2T={cfg.log2T}, fwd+bwd+AdamW; "
                  f"host {platform.processor() or platform.machine()}",
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="grid_rgb", choices=list(CONFIGS))
    ap.add_argument("--rays", type=int, default=2048, help="num_rays_per_modality (grid.yaml: 2048)")
    ap.add_argument("--log2T", type=int, default=19)
    ap.add_argument("--start-step", type=int, default=95000)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--precision", default="fast", choices=list(DTYPES),
                    help="MLP GEMM precision preset (functions.PRESETS); fp32 = reference-parity mode")
    ap.add_argument("--mode", default="graph", choices=["graph", "eager"],
                    help="graph: hipGraph-captured steps (multimodalstudio_amd/graphs.py); eager: Python-launched")
    ap.add_argument("--timing-steps", type=int, default=5,
                    help="eager steps after the timed region whose watched launches are timed with HIP events")
    args = ap.parse_args()

    from multimodalstudio_amd import _lib
    from multimodalstudio_amd import ddp as mddp
    from multimodalstudio_amd.pipeline import Trainer, TrainConfig
    from multimodalstudio_amd import functions as mfn
    mfn.set_precision(args.precision)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    ddp = mddp.init_from_env("nccl") if world > 1 else None

    method, mods, desc = CONFIGS[args.config]
    cfg = TrainConfig(method=method, modalities=mods, num_rays_per_modality=args.rays, log2T=args.log2T)
    trainer = Trainer(cfg, dev, rank=rank)
    trainer.set_step(args.start_step)
    runner = None
    if args.mode == "graph":
        from multimodalstudio_amd.graphs import GraphTrainer
        runner = GraphTrainer(trainer, ddp=ddp)
        step = runner.step
    else:
        step = lambda: trainer.train_step(ddp=ddp)  # noqa: E731

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if ddp:
        ddp.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if ddp:
        ddp.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if ddp:
        elapsed = ddp.max_over_ranks(elapsed, dev)
    if runner is not None:
        print(f"[bench] graph steps: {runner.stats}, {len(runner.graphs)} graphs"
              + (f", capture disabled: {runner.disabled}" if runner.disabled else ""), file=sys.stderr)
    # per-kernel durations: eager steps of the same workload right after the timed region, every watched launch
    # bracketed by HIP events on the stream it is launched on (a graph replay cannot bracket single kernels)
    timing_steps = max(1, args.timing_steps)
    if not args.no_kernel_timing:
        _lib.TIMER.start(work_fns())
        for _ in range(timing_steps):
            trainer.train_step(ddp=ddp)
        torch.cuda.synchronize()
        _lib.TIMER.stop()

    rays_per_step = args.rays * len(mods) * world
    value = rays_per_step * args.steps / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps

    roof = None
    kernels = []
    if not args.no_kernel_timing:
        summ = _lib.TIMER.summary()
        for name, (n, ms, work) in summ.items():
            launches_per_step = n / timing_steps
            if name.startswith("mms_gemm") or name.startswith("mms_mlp_chain"):
                # roofline = the slower of the MFMA and the HBM bound for this launch mix
                flops, nbytes = work
                peak = MFMA_PEAK_TF[name.split(":")[1]]       # "mms_gemm:<precision>:<NT|NN|TN>", "mms_mlp_chain:..."
                t_mfma = flops / (peak * 1e12)
                t_hbm = nbytes / (HBM_PEAK_GBS * 1e9)
                if t_mfma >= t_hbm:
                    ach = flops / (ms * 1e-3) / 1e12
                    rec = {"bound": "mfma", "achieved": round(ach, 3), "peak": peak, "unit": "TFLOP/s",
                           "frac": round(ach / peak, 4)}
                else:
                    ach = nbytes / (ms * 1e-3) / 1e9
                    rec = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": round(ach / HBM_PEAK_GBS, 4)}
                rec.update({"kernel": name, "avg_ms": round(ms, 5), "launches_per_step": launches_per_step,
                            "ms_per_step": round(ms * launches_per_step, 4), "traffic": None,
                            "tflops": round(flops / (ms * 1e-3) / 1e12, 3),
                            "gbs": round(nbytes / (ms * 1e-3) / 1e9, 1)})
                kernels.append(rec)
            else:
                ach = work / (ms * 1e-3) / 1e9
                kernels.append({"kernel": name, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                                "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "avg_ms": round(ms, 5),
                                "launches_per_step": launches_per_step,
                                "ms_per_step": round(ms * launches_per_step, 4), "traffic": None})
        # HBM traffic per launch from the committed rocprofv3 PMC passes of this workload (scripts/gpu_pmc.sh ->
        # scripts/pmc_traffic.py -> profiles/pmc_traffic_<precision>.json); null when not collected
        pmc_path = os.path.join(ROOT, "profiles", f"pmc_traffic_{args.precision}.json")
        pmc = json.load(open(pmc_path))["kernels"] if os.path.exists(pmc_path) else {}
        for rec in kernels:
            if rec["kernel"] in pmc:
                rec["traffic"] = pmc[rec["kernel"]]["hbm_bytes_per_launch"]
                rec["traffic_unit"] = "bytes/launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)"
        kernels.sort(key=lambda k: -k["ms_per_step"])
        if kernels:
            top = kernels[0]
            roof = {k: top[k] for k in ["bound", "achieved", "peak", "unit", "frac", "traffic"]}
            if "traffic_unit" in top:
                roof["traffic_unit"] = top["traffic_unit"]
            roof["kernel"] = top["kernel"]
            roof["avg_ms"] = top["avg_ms"]

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(trainer, cfg, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "train rays/sec (grid.yaml MMS-DATA-shaped synthetic scene)",
            "value": round(value, 1),
            "unit": "rays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": DTYPES[args.precision],
            "data": "synthetic (analytic MMS-DATA-shaped scene, 45 train views 640x512, random-init weights)",
            "config": {"workload": desc, "num_rays_per_modality": args.rays, "modalities": list(mods),
                       "rays_per_step": rays_per_step, "log2_hashmap_size": args.log2T,
                       "model_step": args.start_step, "precision": args.precision, "parallelism": f"dp{world}",
                       "step_mode": ("hipgraph replay (fixed-capacity foreground batches)" if runner is not None and
                                     runner.disabled is None else "eager")},
            "kernel_timing": (f"{timing_steps} eager steps of the same workload after the timed region, HIP events "
                              "around every watched launch on its stream" if not args.no_kernel_timing else None),
            "roofline": roof,
            "roofline_kernels": kernels,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if ddp:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
