"""Diagnostic: the HIP step on the full-size fixture, per-ray outputs dumped for analysis on the CPU.

    python scripts/fullsize_diag.py [precision]   -> gpurun_out/fullsize_diag_<precision>.npz
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from test_gpu_e2e import E2ECase, load  # noqa: E402


def main(prec="fp32", name="e2e_full_grid_rgb_l19"):
    from multimodalstudio_amd import functions as fx
    fx.set_precision(prec)
    f = load(name)
    dev = torch.device("cuda:0")
    case = E2ECase(f, dev)
    outs, losses, total = case.run_step(None)
    torch.cuda.synchronize()
    o = outs["rgb"]
    out = {"loss": total.item()}
    for k in ("rgb", "normals", "accumulation", "depth", "gradients", "hessians", "bins", "weights"):
        out[k] = o[k].detach().cpu().numpy()
    for k, p in case.model.named_parameters():
        if p.grad is not None and not k.endswith("hash_table"):
            out["g:" + k] = p.grad.cpu().numpy()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"fullsize_diag_{prec}.npz"), **out)
    print("saved", total.item())


if __name__ == "__main__":
    main(*sys.argv[1:])
