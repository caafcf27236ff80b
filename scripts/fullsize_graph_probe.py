#!/usr/bin/env python
"""Diagnostic: the full-size graph-replay step of one fixture under a variant (GPU box), the parity test
tests/test_gpu_fullsize.py::test_fullsize_graph_replay without its truth check.

    python scripts/fullsize_graph_probe.py <fixture> [serial_bg|default|guard]

guard: MMS_ARENA_GUARD must be set (e.g. 4096): two eager steps with a zero gap after every carved zero-arena buffer,
then the gaps that were written are reported (a kernel writing past its buffer), before any capture.
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    name = sys.argv[1]
    variant = sys.argv[2] if len(sys.argv) > 2 else "default"
    from multimodalstudio_amd import functions as fx
    from test_gpu_e2e import E2ECase, load
    from test_gpu_fullsize import granule_cap
    dev = torch.device("cuda", 0)
    f = load(name)
    cap = granule_cap(f)
    case = E2ECase(f, dev, concurrent_background=variant not in ("serial_bg", "guard"), inject_bins=True)
    params = case.params()

    def step():
        fx.zero_arena_begin(dev)
        try:
            fx.reset_grad_uses()
            return case.run_step(cap, batched=True)
        finally:
            fx.zero_arena_end()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        step()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    print(f"{name} {variant}: eager warm-up ok (cap {cap})", flush=True)
    if variant == "guard":
        for it in range(2):     # the second step carves from the arena the first one sized
            with torch.cuda.stream(side):
                step()
            torch.cuda.synchronize()
            bad = fx.arena_guard_report()
            print(f"{name} guard step {it}: {len(fx._ARENA_SITES)} carved buffers, {len(bad)} overruns", flush=True)
            for b in bad:
                print("   OVERRUN", b, flush=True)
        return
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for p in params:
            p.grad.zero_()
        outs, losses, total = step()
    torch.cuda.synchronize()
    print(f"{name} {variant}: captured", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print(f"{name} {variant}: replay ok, loss {float(total):.6f} (fixture {float(f['loss']):.6f})", flush=True)


if __name__ == "__main__":
    main()
