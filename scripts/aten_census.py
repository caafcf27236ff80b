"""Census of the ATen ops one training step issues on the device, by op and by the package line that issued it."""
import collections
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, ".")
from multimodalstudio_amd import functions as fx  # noqa: E402
from multimodalstudio_amd.pipeline import TrainConfig, Trainer  # noqa: E402

SKIP = {"aten.view.default", "aten.detach.default", "aten._unsafe_view.default", "aten.t.default",
        "aten.as_strided.default", "aten.slice.Tensor", "aten.select.int", "aten.unsqueeze.default",
        "aten.squeeze.dim", "aten.expand.default", "aten.reshape.default", "aten.alias.default",
        "aten.empty.memory_format", "aten.empty_strided.default", "aten.transpose.int", "aten.split.Tensor",
        "aten.permute.default", "aten.unbind.int", "aten.lift_fresh.default", "aten._to_copy.default"}


class Census(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.ops = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func)
        if name not in SKIP:
            site = "?"
            for fr in reversed(traceback.extract_stack()[:-1]):
                if "multimodalstudio_amd" in fr.filename:
                    site = f"{fr.filename.split('multimodalstudio_amd/')[-1]}:{fr.lineno} {fr.line.strip()[:70]}"
                    break
            if name.startswith("aten.add"):
                shapes = [tuple(a.shape) + (a.stride(),) for a in args if isinstance(a, torch.Tensor)]
                site = f"{site} {shapes}"
            self.ops[(name, site)] += 1
        return func(*args, **(kwargs or {}))


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
    for label, fn in [("host: stage + hit counts", lambda: (g._stage_inputs(), g.hit_counts())),
                      ("captured body: forward + backward + optimizer", None)]:
        c = Census()
        with c:
            if fn is not None:
                out = fn()
                counts = out[1]
            else:
                cap = bucket_capacity(counts, g.granule, g.n)
                g._forward_backward(cap)
                g._optimizer()
        torch.cuda.synchronize()
        tot = sum(c.ops.values())
        print(f"== {label}: {tot} ATen ops")
        for (name, site), n in sorted(c.ops.items(), key=lambda kv: -kv[1]):
            print(f"{n:4d}  {name:45s} {site}")


if __name__ == "__main__":
    main()
