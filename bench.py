#!/usr/bin/env python
"""Train-rays/s benchmark of the MMS hot path on MI355X (BASELINE.json metric, configs[1] by default).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config grid_rgb|grid_raw5] [--rays R]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = one full training iteration of RawPipeline/BasePipeline.train_step on synthetic data of the
MMS-DATA shape: pixel sampling (device Philox draws over HBM-resident frames; --sampler host: the
reference-order host sampler), ray generation with SO3xR3 pose refinement, the
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
    "grid_bg5": ("grid_raw_grid_bg_unbalanced", ("rgb", "polarization"),
                 "confs/grid_raw_rgb_all_views_pol_10_views.yaml, rgb + polarization (10 pol views), hash-grid "
                 "background, pose refinement"),
}

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
F32_MFMA_PEAK_TF = 157.3   # dense f32-input MFMA (v_mfma_f32_32x32x2_f32) peak, MI355X_MICROARCH.md
BF16_MFMA_PEAK_TF = 2500.0  # dense bf16 MFMA peak (no sparsity), MI355X_MICROARCH.md
# split-bf16x3 runs 3 bf16 MFMAs per f32 product: its ceiling for the algorithmic 2MNK flops is a third
# (bf16x2: the SDF chain's split activations x bf16 weights, 2 bf16 MFMAs per product)
MFMA_PEAK_TF = {"fp32": F32_MFMA_PEAK_TF, "bf16": BF16_MFMA_PEAK_TF, "bf16x3": BF16_MFMA_PEAK_TF / 3,
                "bf16x2": BF16_MFMA_PEAK_TF / 2, "fp16": BF16_MFMA_PEAK_TF}
PREC_NAMES = {0: "fp32", 1: "bf16", 2: "bf16x3", 3: "bf16x2", 5: "fp16", 6: "fp16-rowscaled"}
DTYPES = {"fp32": "fp32",
          "fast": "split-bf16x3 MFMA (bf16 hi + lo operands, fp32 accumulate) for every MLP, fp32 elsewhere",
          "fast_bf16": "bf16 MFMA (fp32 accumulate; SDF MLP and polarization heads split-bf16x3) -- not a parity "
                       "preset: -0.56 dB converged PSNR, fp32 elsewhere",
          "fast_m4": "split-bf16x3 forward / bf16 backward for the radiance, head and background MLPs -- not a parity "
                     "preset, fp32 elsewhere",
          "fast_x2": "bf16 MFMA (fp32 accumulate; SDF MLP chain bf16 weights x split-bf16 activations -- not a parity "
                     "preset: hessians off), fp32 elsewhere",
          "bf16x3": "split-bf16x3 MFMA (fp32-accurate), fp32 elsewhere",
          "fast_w16": "split-bf16x3 MFMA (bf16 hi + lo operands, fp32 accumulate) for every MLP forward and data "
                      "gradient, bf16 MFMA (fp32 accumulate) for the MLP weight gradients, fp32 elsewhere",
          "fast_h16": "fp16 MFMA (fp32 accumulate: the reference's autocast) for the radiance / head / background MLP "
                      "forwards, split-bf16x3 for their backward and for the SDF MLP, fp32 elsewhere",
          "fast_h16b": "fp16 MFMA (fp32 accumulate: the reference's autocast) for the radiance / head / background MLP "
                       "forwards and for every MLP's backward-data chain after its first layer (per-row power-of-two "
                       "scaled), split-bf16x3 for the SDF MLP forward, the chains' first backward layer and the weight "
                       "gradients, fp32 elsewhere",
          "fast_h16bw": "as fast_h16b with bf16 MFMA (fp32 accumulate) for the MLP weight gradients -- not the "
                        "benchmarked preset, fp32 elsewhere",
          "fast_h16c": "fp16 MFMA (fp32 accumulate: the reference's autocast) for the radiance / head / background MLP "
                       "forwards, for every MLP's backward-data chain after its first layer (per-row power-of-two "
                       "scaled) and for the hidden layers' weight gradients (fp16 dZ rows in their row scale, fp16 X in "
                       "a per-launch scale); split-bf16x3 for the SDF MLP forward, the chains' first backward layer and "
                       "the output layers' weight gradients, fp32 elsewhere",
          "fast_h16d": "fp16 MFMA (fp32 accumulate: the reference's autocast) for the radiance / head / background MLP "
                       "forwards, for every MLP's backward-data chain after its first layer (per-row power-of-two "
                       "scaled) and for the hidden layers' weight gradients; fp16 storage of those MLPs' hidden "
                       "activations and dZ rows (the reference autocast's fp16 activations); split-bf16x3 for the SDF "
                       "MLP forward, the chains' first backward layer and the output layers' weight gradients, fp32 "
                       "elsewhere"}
# the benchmarked preset (tests/test_cpu_host.py::test_benchmarked_preset_* guard its numerics)
DEFAULT_PRECISION = "fast_h16d"
HASH_FWD_B = 16 * 8 * 2 * 4 + 12 + 128          # bytes per lookup, forward
HASH_BWD_B = 128 + 12 + 16 * 8 * 2 * (4 + 4)    # bytes per lookup, backward (table grads)
HASH_BWD_ATOMIC_B = 16 * 8 * 2 * 4              # the float-atomic bytes one backward lookup adds into the table
ATOMIC_PEAK_GBS = 1300.0                        # MI355X_MICROARCH.md "Global float atomics": chip-wide added bytes


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


def gemm_grouped_work(a):
    """(precision label, (flops, bytes)) of one mms_gemm_tn_grouped launch: the weight gradients of one MLP's layers
    (sum over items of 2 M N K flops; bytes = both operands once + dW read and written)."""
    prec, n, M, N, K = a[0], a[1], a[2], a[3], a[4]
    flops = sum(2.0 * M[i] * N[i] * K[i] for i in range(n))
    nbytes = sum(4.0 * (float(K[i]) * (M[i] + N[i]) + 2.0 * M[i] * N[i]) for i in range(n))
    return f"{PREC_NAMES[prec]}:TN_grouped", (flops, nbytes)


def gemm_wide16_work(a):
    """(label, (flops, bytes)) of one mms_gemm_tn_wide16 launch (one MLP's weight gradients, items of mixed operand
    modes): 2 M N K flops per item; bytes = the dZ rows (fp16: 2 B per element + the row's 4-B inverse scale; fp32: 4 B),
    the X rows (2 or 4 B per element) once, dW read and written."""
    import ctypes
    n, M, N, K = a[0], a[1], a[2], a[3]
    ainv = ctypes.cast(a[6], ctypes.POINTER(ctypes.c_void_p)) if a[6] else None
    b16 = ctypes.cast(a[10], ctypes.POINTER(ctypes.c_int)) if a[10] else None
    flops = sum(2.0 * M[i] * N[i] * K[i] for i in range(n))
    nbytes = 0.0
    for i in range(n):
        a16 = ainv is not None and bool(ainv[i])
        nbytes += (2.0 * M[i] + 4.0 if a16 else 4.0 * M[i]) * K[i] + (2.0 if (b16 is not None and b16[i]) else 4.0) * \
            K[i] * N[i] + 8.0 * M[i] * N[i]
    return "fp16:TN_grouped", (flops, nbytes)


def chain_work(a):
    """(precision label, (algorithmic flops, algorithmic HBM bytes)) of one mms_mlp_chain launch (include/mms_hip.h
    argument order): every layer's 2MNK, narrowed on the SDF tap rows (rows >= rows_full: one output column of the
    last forward layer, one input column of the first backward layer); bytes = input rows + the stores each layer
    makes (+ the forward outputs the backward reads for its activation derivatives)."""
    import ctypes
    prec, bwd, nl, K0, M, rf = a[0], a[1], a[2], a[5], a[6], a[7]
    rf = M if rf < 0 else min(rf, M)
    Np = ctypes.cast(a[20], ctypes.POINTER(ctypes.c_int))
    outs = ctypes.cast(a[18], ctypes.POINTER(ctypes.c_void_p))
    n = [Np[i] for i in range(nl)]
    # bytes per stored element: 4 (fp32), or 2 + 4 / n (a prec-6 hidden layer's fp16 dZ rows and their inverse scale),
    # or 2 (fp16 hidden activations, f16); the backward's activation rows (aux) 2 B per element when f16
    rinv = ctypes.cast(a[27], ctypes.POINTER(ctypes.c_void_p)) if len(a) > 27 and a[27] else None
    f16 = ctypes.cast(a[29], ctypes.POINTER(ctypes.c_int)) if len(a) > 29 and a[29] else None
    h = [bool(f16 is not None and f16[i]) for i in range(nl)]
    st = [0.0 if outs[i] is None else (0.5 + 1.0 / n[i] if (rinv is not None and rinv[i]) else
                                       (0.5 if (h[i] and not bwd) else 1.0)) for i in range(nl)]
    ya = [0.5 if h[i] else 1.0 for i in range(nl)]      # backward: bytes factor of layer i's activation rows
    mid = sum(n[l - 1] * n[l] for l in range(1, nl - 1))
    if bwd:
        f0 = 2.0 * (rf * K0 + (M - rf)) * n[0]       # the first backward layer (B = dY from memory)
        flops = f0 + 2.0 * M * (mid + n[nl - 2] * n[nl - 1])
        nbytes = 4.0 * ((rf * K0 + (M - rf)) + M * sum(n[l] * st[l] for l in range(nl)) +
                        M * sum(n[l] * ya[l] for l in range(nl - 1)))
    else:
        flops = 2.0 * M * (K0 * n[0] + mid) + 2.0 * (rf * n[nl - 1] + (M - rf)) * n[nl - 2]
        nbytes = 4.0 * (M * K0 + M * sum(n[l] * st[l] for l in range(nl - 1)) + (rf * n[nl - 1] + (M - rf)) * st[nl - 1])
    # which MLP: the SDF field (71 input columns; its backward's last layer has 71 outputs), the radiance field, or
    # the background NeRF's base / head (4 layers); rows_full = 0 marks the sampler's inference-only SDF evaluations
    width = n[nl - 1] if bwd else K0
    if nl == 4:
        role = "bg_base" if width < 64 else "bg_head"
    elif n[0] == 64:
        role = "head"                      # the modality heads 256-64-64-C (bwd: 64-64-256 from C)
    else:
        role = ("sdf" if width < 128 else "radiance") + ("_infer" if (not bwd and rf == 0) else "")
    label = f"{PREC_NAMES[prec]}:{role}{'_bwd' if bwd else '_fwd'}"
    if prec == 6 and bwd:
        # fp16-rowscaled: the first backward layer runs split-bf16x3 (3 MFMAs per product), the register-fed layers
        # one fp16 MFMA: the third element is the launch's work in single-MFMA-equivalent flops (its mode ceiling)
        return label, (flops, nbytes, flops + 2.0 * f0)
    return label, (flops, nbytes)


def hash_fwd_work(a):
    """(role, SURVEY §8(d) bytes) of one mms_hashgrid_fwd(_grouped) launch: the SDF batch [centre | 4 taps] (the dominant
    launch), the sampler's / background's smaller 72-column panels, or the radiance panel."""
    Mg, group, ldx = int(a[1]), int(a[2]), int(a[4])     # mms_hashgrid_fwd_grouped(pos, Mg, group, gstride, ldx, ...)
    M = Mg * group
    role = "sdf_taps" if (ldx == 72 and M > 200000) else ("radiance" if ldx >= 300 else "sampler_or_bg")
    return role, float(M) * HASH_FWD_B


def sdf_panel_work(a):
    """(role, bytes) of one mms_sdf_panel_fwd launch (include/mms_hip.h argument order): the SURVEY §8(d) bytes of its
    hash-grid lookups plus the x / PE columns it writes (3 + 6 pe_freqs floats per row)."""
    M, ntaps, F = int(a[2]), int(a[3]), int(a[5])
    rows = M * (ntaps + 1)
    role = "sdf_taps" if ntaps == 4 else "sampler"
    return role, float(rows) * (HASH_FWD_B + 4 * (3 + 6 * F))


def sdf_panel_rays_work(a):
    """(role, bytes) of one mms_sdf_panel_rays_fwd launch (the sampler's panels formed from the spacing bins): as
    sdf_panel_work for its R (nb - 1) rows."""
    nb, R, F = int(a[2]), int(a[7]), int(a[8])
    return "sampler", float(R * (nb - 1)) * (HASH_FWD_B + 4 * (3 + 6 * F))


def rad_panel_work(a):
    """(role, bytes) of one mms_rad_panel_fwd launch: the hash-grid lookups' SURVEY §8(d) bytes plus the x / SH / n.v
    columns written and the geo feature read and written (4 B each way per column)."""
    M, G = int(a[6]), int(a[8])
    return "radiance", float(M) * (HASH_FWD_B + 4 * 29 + 8 * G)


def work_fns():
    return {
        "mms_gemm": gemm_work,
        "mms_gemm_tn_grouped": gemm_grouped_work,
        "mms_gemm_tn_wide": gemm_grouped_work,
        "mms_gemm_tn_wide16": gemm_wide16_work,
        "mms_mlp_chain": chain_work,
        "mms_hashgrid_fwd_grouped": hash_fwd_work,
        "mms_sdf_panel_fwd": sdf_panel_work,
        "mms_sdf_panel_rays_fwd": sdf_panel_rays_work,
        "mms_rad_panel_fwd": rad_panel_work,
        "mms_hashgrid_bwd_grouped": lambda a: ("sdf_taps" if a[2] == 5 else "radiance_or_bg",
                                               (float(a[1]) * a[2] * HASH_BWD_B, float(a[1]) * a[2] * HASH_BWD_ATOMIC_B)),
    }


def kernel_records(summ, timing_steps: int, precision: str):
    """One record per watched launch kind: MLP launches (GEMMs, chains) rated by their algorithmic 2MNK flops against
    the dense bf16 MFMA peak (split-bf16x3 also against its own third-rate ceiling, fp32 against the f32 MFMA peak),
    hash-grid launches by their SURVEY §8(d) bytes against HBM.  ``traffic`` = HBM bytes per launch from the
    committed rocprofv3 PMC passes of this workload (profiles/pmc_traffic_<precision>.json), null if not collected."""
    kernels = []
    for name, (n, ms, work) in summ.items():
        launches_per_step = n / timing_steps
        rec = {"kernel": name, "avg_ms": round(ms, 5), "launches_per_step": launches_per_step,
               "ms_per_step": round(ms * launches_per_step, 4), "traffic": None}
        if name.startswith("mms_gemm") or name.startswith("mms_mlp_chain"):   # (incl. the grouped weight gradients)
            flops, nbytes = work[:2]
            mode = name.split(":")[1]      # "mms_gemm:<precision>:<NT|NN|TN>", "mms_mlp_chain:<precision>:<role>"
            peak = F32_MFMA_PEAK_TF if mode == "fp32" else BF16_MFMA_PEAK_TF
            ach = flops / (ms * 1e-3) / 1e12
            rec.update({"bound": "mfma", "achieved": round(ach, 3), "peak": peak, "unit": "TFLOP/s",
                        "frac": round(ach / peak, 4), "gbs": round(nbytes / (ms * 1e-3) / 1e9, 1)})
            if mode in ("bf16x3", "bf16x2"):
                rec.update({"mode_peak": round(MFMA_PEAK_TF[mode], 1),
                            "frac_of_mode_peak": round(ach / MFMA_PEAK_TF[mode], 4)})
            elif mode == "fp16-rowscaled" and len(work) > 2 and work[2] > 0:
                # priced per layer: the split-bf16x3 first layer at a third of the peak, the fp16 layers at the peak
                mp = BF16_MFMA_PEAK_TF * flops / work[2]
                rec.update({"mode_peak": round(mp, 1), "frac_of_mode_peak": round(ach / mp, 4)})
        else:
            atomic = None
            if isinstance(work, tuple):
                work, atomic = work
            ach = work / (ms * 1e-3) / 1e9
            rec.update({"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(ach / HBM_PEAK_GBS, 4)})
            if atomic is not None:
                # the backward's binding ceiling: float atomics execute at the memory side at ~1.3 TB/s of added bytes
                aa = atomic / (ms * 1e-3) / 1e9
                rec["atomic_ceiling"] = {"achieved": round(aa, 1), "peak": ATOMIC_PEAK_GBS, "unit": "GB/s added",
                                         "frac": round(aa / ATOMIC_PEAK_GBS, 4)}
        kernels.append(rec)
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_traffic_{precision}.json")
    pmc = json.load(open(pmc_path))["kernels"] if os.path.exists(pmc_path) else {}
    for rec in kernels:
        if rec["kernel"] in pmc:
            rec["traffic"] = pmc[rec["kernel"]]["hbm_bytes_per_launch"]
            rec["traffic_unit"] = "bytes/launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)"
    kernels.sort(key=lambda k: -k["ms_per_step"])
    return kernels


CPU_CONFIGS = {
    # BASELINE.md §2 configurations the CPU restatement is timed on: (method, modalities)
    "grid_rgb": ("grid", ("rgb",)),
    "grid_raw5": ("grid_raw", ("rgb", "infrared", "mono", "polarization", "multispectral")),
    "mlp_raw": ("mlp_raw", ("rgb",)),
    "grid_bg5": ("grid_raw_grid_bg_unbalanced", ("rgb", "polarization")),
}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def cpu_threads() -> tuple:
    """(threads used, CPUs in this process's affinity mask): BASELINE.md §2 asks for len(os.sched_getaffinity(0));
    on a shared GPU box the job's CPU share is OMP_NUM_THREADS (set by the pool), so the smaller of the two."""
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    return (min(aff, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else aff), aff


def cpu_baseline(config: str, log2T: int, step: int, seconds: float, n_rays: int = 256):
    """The fixture-pinned CPU restatement (oracle/) of one BASELINE configuration, bounded sample, on host cores:
    the reference's own pure-PyTorch path restated (tests/test_oracle_golden.py pins it to the reference's outputs),
    random-init weights of that method, model state at ``step``."""
    from oracle.train import OracleTrainer
    from multimodalstudio_amd import scene as ms
    from multimodalstudio_amd.model import BaseModel, ModelSpec
    from multimodalstudio_amd.pipeline import METHODS
    from multimodalstudio_amd.pipeline import skip_views_for
    method, mods = CPU_CONFIGS[config]
    raw, bg_kind, fields = METHODS[method]
    mods = list(mods)
    channels = {m: ms.CHANNELS[m] for m in mods}
    threads, affinity = cpu_threads()
    torch.set_num_threads(threads)
    torch.manual_seed(654824)
    model = BaseModel(ModelSpec(channels, log2T=log2T, bg_kind=bg_kind, fields=fields))
    sd = {k: v.detach() for k, v in model.state_dict().items()}
    del model
    W, H = 640, 512
    cams = ms.make_cameras(mods, 50, W, H, seed=0, train=True)
    for m, skip in (skip_views_for(method) or {}).items():
        if m in cams:
            cams[m] = ms.select_views(cams[m], [v for v in cams[m].view_ids if v not in set(skip)])
    masks = {m: ms.mosaick_mask(m, W, H) for m in mods} if raw else None
    ot = OracleTrainer(sd, channels, cams, log2T, step, raw=raw, mosaick=masks, fields=fields, bg_kind=bg_kind)
    g = torch.Generator().manual_seed(1)

    def batch():
        coords, targets = {}, {}
        for m in mods:
            C = cams[m].c2w.shape[0]
            c = torch.stack([torch.randint(0, C, (n_rays,), generator=g), torch.randint(0, H, (n_rays,), generator=g),
                             torch.randint(0, W, (n_rays,), generator=g)], -1).to(torch.int32)
            coords[m] = c
            targets[m] = torch.rand(n_rays, 1 if raw else channels[m], generator=g)
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
        "affinity_cpus": affinity,
        "cpu_model": cpu_model(),
        "kind": "port",
        "sample": f"{len(times)} timed steps (median) of the CPU restatement (oracle/, pinned to the reference torch "
                  f"path) of {config} ({method}, {len(mods)} modalit{'y' if len(mods) == 1 else 'ies'}) at {n_rays} "
                  f"rays/modality, log2T={log2T}, model step {step}, fwd+bwd+AdamW; {torch.get_num_threads()} threads "
                  f"on {cpu_model()} ({affinity} CPUs in the affinity mask)",
    }


def timed_run(config: str, args, dev, rank: int, ddp, steps: int, warmup: int) -> dict:
    """Build the trainer for ``config``, run ``warmup`` untimed steps, then time exactly ``steps`` steps bracketed by a
    barrier + device synchronise on both sides; the time is the max over ranks."""
    from multimodalstudio_amd.pipeline import Trainer, TrainConfig
    method, mods, _ = CONFIGS[config]
    world = ddp.world if ddp is not None else 1
    from multimodalstudio_amd.pipeline import skip_views_for
    cfg = TrainConfig(method=method, modalities=mods, num_rays_per_modality=args.rays, log2T=args.log2T,
                      skip_views=skip_views_for(method), gpu_sampler=args.sampler == "device")
    trainer = Trainer(cfg, dev, rank=rank)
    trainer.model.concurrent_background = not args.serial_background
    trainer.set_step(args.start_step)
    runner = None
    if args.mode == "graph":
        from multimodalstudio_amd.graphs import GraphTrainer
        runner = GraphTrainer(trainer, ddp=ddp)
        step = runner.step
    else:
        step = lambda: trainer.train_step(ddp=ddp)  # noqa: E731
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if ddp:
        ddp.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if ddp:
        ddp.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if ddp:
        elapsed = ddp.max_over_ranks(elapsed, dev)
    if runner is not None:
        print(f"[bench] {config}: graph steps: {runner.stats}, {len(runner.graphs)} graphs"
              + (f", capture disabled: {runner.disabled}" if runner.disabled else ""), file=sys.stderr)
    rays_per_step = args.rays * len(mods) * world
    mode = ("hipgraph replay (fixed-capacity foreground batches)" if runner is not None and runner.disabled is None
            else "eager")
    return {"trainer": trainer, "runner": runner, "elapsed": elapsed, "cfg": cfg, "rays_per_step": rays_per_step,
            "value": rays_per_step * steps / elapsed, "ms_per_step": 1000.0 * elapsed / steps, "step_mode": mode,
            "steps": steps, "warmup": warmup}


def spawn_ranks(n: int) -> int:
    """``python bench.py --gpus N`` without a torch.distributed environment: one process per GPU, as the reference's
    Fabric launch does (/root/reference/src/engine/trainer.py:57-63), through torch.distributed.run with the same
    arguments; this process touches no GPU and exits with the launcher's status (rank 0 prints the JSON line)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


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
    ap.add_argument("--precision", default=DEFAULT_PRECISION, choices=list(DTYPES),
                    help="MLP GEMM precision preset (functions.PRESETS); fp32 = reference-parity mode")
    ap.add_argument("--sampler", default="device", choices=["device", "host"],
                    help="pixel sampler: HBM-resident frames + device Philox draws (default), or the reference-order "
                         "host sampler with a per-step upload")
    ap.add_argument("--serial-background", action="store_true",
                    help="run the background branch on the main stream (default: its own stream, overlapped)")
    ap.add_argument("--mode", default="graph", choices=["graph", "eager"],
                    help="graph: hipGraph-captured steps (multimodalstudio_amd/graphs.py); eager: Python-launched")
    ap.add_argument("--secondary", default="grid_raw5,grid_bg5",
                    help="also time these configs (comma-separated; nested records: the first as 'secondary', BASELINE "
                         "configs[4] as 'config5'); '' to skip")
    ap.add_argument("--timing-steps", type=int, default=5,
                    help="eager steps after the timed region whose watched launches are timed with HIP events")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))

    from multimodalstudio_amd import _lib
    from multimodalstudio_amd import ddp as mddp
    from multimodalstudio_amd.pipeline import Trainer, TrainConfig
    from multimodalstudio_amd import functions as mfn
    mfn.set_precision(args.precision)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE {world}: measuring {world} rank(s)", file=sys.stderr)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    ddp = mddp.init_from_env("nccl") if world > 1 else None

    method, mods, desc = CONFIGS[args.config]
    run = timed_run(args.config, args, dev, rank, ddp, args.steps, args.warmup)
    trainer, runner, elapsed, cfg = run["trainer"], run["runner"], run["elapsed"], run["cfg"]
    # per-kernel durations: eager steps of the same workload right after the timed region, every watched launch
    # bracketed by HIP events on the stream it is launched on (a graph replay cannot bracket single kernels)
    timing_steps = max(1, args.timing_steps)
    if not args.no_kernel_timing:
        # the background branch on the main stream here: a launch's events then bracket that kernel alone, not the
        # time it shares the chip with the overlapped background stream
        # (and the weight-gradient launches inline, not on their side stream beside the hash-grid backward)
        trainer.model.concurrent_background = False
        async_wgrad, mfn.ASYNC_WGRAD = mfn.ASYNC_WGRAD, False
        _lib.TIMER.start(work_fns())
        for _ in range(timing_steps):
            trainer.train_step(ddp=ddp)
        torch.cuda.synchronize()
        _lib.TIMER.stop()
        trainer.model.concurrent_background = not args.serial_background
        mfn.ASYNC_WGRAD = async_wgrad

    rays_per_step, value, ms_per_step, run_mode = run["rays_per_step"], run["value"], run["ms_per_step"], run["step_mode"]

    roof, hash_roof, kernels = None, None, []
    if not args.no_kernel_timing:
        kernels = kernel_records(_lib.TIMER.summary(), timing_steps, args.precision)
        # headline (north_star / SURVEY §8(d)): MFMA utilisation of the fused geometry-MLP chain, forward, rated by
        # its algorithmic 2MNK flops against the dense bf16 MFMA peak; the hash-grid lookups against HBM beside it
        by_name = {k["kernel"]: k for k in kernels}
        sdf = [k for k in kernels if k["kernel"].startswith("mms_mlp_chain:")
               and k["kernel"].endswith(":sdf_fwd")]
        top = sdf[0] if sdf else (kernels[0] if kernels else None)
        if top is not None:
            roof = {k: top[k] for k in ["bound", "achieved", "peak", "unit", "frac", "traffic"] if k in top}
            for k in ["kernel", "avg_ms", "frac_of_mode_peak", "mode_peak", "traffic_unit"]:
                if k in top:
                    roof[k] = top[k]
        keys = ["kernel", "achieved", "peak", "unit", "frac", "avg_ms", "traffic", "atomic_ceiling"]
        hash_roof = {d: {k: by_name[n][k] for k in keys if k in by_name[n]}
                     for d, n in [("fwd", "mms_hashgrid_fwd_grouped:sdf_taps"), ("fwd_radiance", "mms_hashgrid_fwd_grouped:radiance"),
                                  ("fwd", "mms_sdf_panel_fwd:sdf_taps"), ("fwd_radiance", "mms_rad_panel_fwd:radiance"),
                                  ("bwd", "mms_hashgrid_bwd_grouped:sdf_taps"),
                                  ("bwd_radiance", "mms_hashgrid_bwd_grouped:radiance_or_bg")] if n in by_name}

    cpu, cpu_all = None, None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the headline config's CPU baseline, then the other BASELINE.md §2 configurations beside it
        cpu = cpu_baseline(args.config, args.log2T, args.start_step, args.cpu_seconds) if args.config in CPU_CONFIGS \
            else None
        cpu_all = {c: cpu_baseline(c, args.log2T, args.start_step, args.cpu_seconds / 2)
                   for c in CPU_CONFIGS if c != args.config}

    extra = {}
    names = [c for c in (args.secondary or "").split(",") if c and c != args.config]
    if names:
        del trainer, runner, run
    for name in names:
        # further driver-timed lines in the same process: the 5-modality workload (BASELINE configs[2] per GPU) and
        # config 5 (configs[4] per GPU: rgb + 10-view polarization, hash-grid background, pose refinement)
        torch.cuda.empty_cache()
        r2 = timed_run(name, args, dev, rank, ddp, max(1, min(args.steps, 20)), max(1, min(args.warmup, 5)))
        extra[name] = {"config": {"workload": CONFIGS[name][2], "modalities": list(CONFIGS[name][1]),
                                  "num_rays_per_modality": args.rays, "rays_per_step": r2["rays_per_step"],
                                  "parallelism": f"dp{world}"},
                       "value": round(r2["value"], 1), "per_rank_value": round(r2["value"] / world, 1),
                       "unit": "rays/s", "steps": r2["steps"], "warmup": r2["warmup"],
                       "ms_per_step": round(r2["ms_per_step"], 3), "step_mode": r2["step_mode"],
                       "cpu_baseline": (cpu_all or {}).get(name)}
        del r2
    secondary = extra.pop(names[0]) if names else None

    if rank == 0:
        line = {
            "metric": "train rays/sec (grid.yaml MMS-DATA-shaped synthetic scene)",
            "value": round(value, 1),
            "unit": "rays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            # the reference's own TRAIN_RAYS_PER_SEC is per rank (trainer.py:107-114); value is the whole job's
            "per_rank_value": round(value / world, 1),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": DTYPES[args.precision],
            "data": "synthetic (analytic MMS-DATA-shaped scene, 45 train views 640x512, random-init weights)",
            "config": {"workload": desc, "num_rays_per_modality": args.rays, "modalities": list(mods),
                       "rays_per_step": rays_per_step, "log2_hashmap_size": args.log2T,
                       "model_step": args.start_step, "precision": args.precision,
                       "pixel_sampler": args.sampler, "parallelism": f"dp{world}",
                       "step_mode": run_mode},
            "kernel_timing": (f"{timing_steps} eager steps of the same workload after the timed region, HIP events "
                              "around every watched launch on its stream (background branch on the main stream for these "
                              "steps, so each launch is timed alone)" if not args.no_kernel_timing else None),
            "roofline": roof,
            "roofline_hash_grid": hash_roof,
            "roofline_kernels": kernels,
            "cpu_baseline": cpu,
            "cpu_baseline_configs": cpu_all,
            "secondary": secondary,
            "config5": extra.get("grid_bg5"),
        }
        print(json.dumps(line))
    if ddp:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
