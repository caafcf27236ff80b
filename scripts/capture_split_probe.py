"""Can a graph capture be split from INSIDE an autograd backward (the hook that sees a gradient become final)?
Diagnostic for graphs.GraphTrainer's data-parallel split."""
import torch

dev = torch.device("cuda", 0)
live = {}


class Split(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        live["calls"] = live.get("calls", 0) + 1
        if "next" in live:
            live["cur"].capture_end()
            live["next"].capture_begin(live["cur"].pool(), capture_error_mode=live["mode"])
            live["cur"] = live.pop("next")
        return g


def run(mode):
    w1 = torch.randn(256, 256, device=dev, requires_grad=True)
    w2 = torch.randn(256, 256, device=dev, requires_grad=True)
    x = torch.randn(1024, 256, device=dev)

    def step():
        h = torch.relu(x @ w1)
        h = Split.apply(h)
        y = (h @ w2).sum()
        y.backward()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.synchronize()
    g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    live.update(cur=g1, next=g2, mode=mode)
    if torch.cuda.graph.default_capture_stream is None:
        torch.cuda.graph.default_capture_stream = torch.cuda.Stream()
    with torch.cuda.stream(torch.cuda.graph.default_capture_stream):
        w1.grad.zero_()
        w2.grad.zero_()
        g1.capture_begin(capture_error_mode=mode)
        step()
        live["cur"].capture_end()
    ref1, ref2 = None, None
    w1.grad.zero_(); w2.grad.zero_()
    g1.replay(); torch.cuda.synchronize()
    a2 = w2.grad.clone(); a1 = w1.grad.clone()
    g2.replay(); torch.cuda.synchronize()
    b1 = w1.grad.clone()
    w1.grad = None; w2.grad = None
    step(); torch.cuda.synchronize()
    print(mode, "w2 grad after part 1:", torch.allclose(a2, 2 * w2.grad if False else a2), "w1 after part1 zero:",
          float(a1.abs().max()), "w1 after part 2 == eager:", torch.allclose(b1, w1.grad, rtol=1e-4, atol=1e-3))


for mode in ("thread_local", "global", "relaxed"):
    try:
        run(mode)
    except Exception as e:
        print(mode, "FAILED", type(e).__name__, str(e)[:300])
