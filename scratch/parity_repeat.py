"""Run-to-run spread of the training-parity PSNR (tests/test_gpu_train_parity.py:run_parity), per preset."""
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, ".."))
import test_gpu_train_parity as T  # noqa: E402

dev = torch.device("cuda", 0)
for prec in sys.argv[1:]:
    for rep in range(3):
        f, cfg, losses, psnr = T.run_parity(dev, prec)
        oracle = {m: float(f[f"eval:{m}:psnr"]) for m in cfg["modalities"]}
        print(prec, rep, psnr, oracle, {m: psnr[m] - oracle[m] for m in psnr}, flush=True)
