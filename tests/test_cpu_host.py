"""CPU-only tests: the C-ABI boundary (load + exports + argument validation, no device compute), the
host-side schedules against the oracle, and the multi-process (gloo, world_size 2) gradient exchange."""
from __future__ import annotations

import os
import sys

import pytest
import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.fixture(scope="module")
def L():
    from multimodalstudio_amd import _lib, build
    if not _lib.LIB_PATH.exists():
        build.build()
    return _lib.lib()


def test_header_parses_and_library_exports_every_symbol(L):
    from multimodalstudio_amd import _lib
    names = _lib.exported_symbols()
    assert len(names) >= 40
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, f"libmms_hip.so misses symbols declared in include/mms_hip.h: {missing}"
    for core in ("mms_hashgrid_fwd", "mms_hashgrid_bwd", "mms_hashgrid_bwd_grouped", "mms_gemm", "mms_neus_step",
                 "mms_raygen_fwd", "mms_composite_fwd", "mms_adamw", "mms_last_error", "mms_version"):
        assert core in names


def test_version_string(L):
    v = L.mms_version().decode()
    assert v and "gfx950" in v


def _err(L):
    return L.mms_last_error().decode()


def test_gemm_rejects_bad_arguments_before_touching_the_device(L):
    # prec out of range
    rc = L.mms_gemm(7, 0, 0, 4, 4, 4, 1, 4, 1, 4, 1, 4, None, None, 0, None, 0, 0, 0, 1.0, 20.0, 0, 1, -1, None, None)
    assert rc != 0 and "prec" in _err(L)
    # split-K with a non-accumulating epilogue
    rc = L.mms_gemm(0, 1, 1, 4, 4, 4096, 1, 4, 1, 4, 1, 4, None, None, 0, None, 0, 1, 0, 1.0, 20.0, 0, 4, -1, None, None)
    assert rc != 0 and "split-K" in _err(L)
    # fused column sum needs a T-source A
    rc = L.mms_gemm(0, 0, 0, 4, 4, 4, 1, 4, 1, 4, 1, 4, None, None, 0, None, 0, 0, 0, 1.0, 20.0, 0, 1, -1, 8, None)
    assert rc != 0 and "column sum" in _err(L)
    # empty problems are a no-op success
    assert L.mms_gemm(0, 0, 0, 0, 4, 4, None, 4, None, 4, None, 4, None, None, 0, None, 0, 0, 0, 1.0, 20.0, 0, 1, -1,
                      None, None) == 0


def test_hashgrid_rejects_bad_config(L):
    import ctypes
    sc = (ctypes.c_float * 16)(*([16.0] * 16))
    rc = L.mms_hashgrid_fwd(1, 10, 3, 1, 16, 19, 3, 0, ctypes.cast(sc, ctypes.c_void_p), 1.0, 16, 1, 32, None)
    assert rc != 0 and "features_per_level" in _err(L)
    rc = L.mms_hashgrid_fwd(1, 10, 3, 1, 17, 19, 2, 0, ctypes.cast(sc, ctypes.c_void_p), 1.0, 16, 1, 40, None)
    assert rc != 0 and "num_levels" in _err(L)
    rc = L.mms_hashgrid_fwd(1, 10, 3, 1, 16, 19, 2, 2, ctypes.cast(sc, ctypes.c_void_p), 1.0, 16, 1, 40, None)
    assert rc != 0 and "interp" in _err(L)
    rc = L.mms_hashgrid_bwd_grouped(1, 10, 3, 10, 3, 1, 16, 19, 2, 0, ctypes.cast(sc, ctypes.c_void_p), 1.0, 16, 1,
                                    32, 1, None, 0, None)
    assert rc != 0 and "group" in _err(L)


def test_ops_fail_loudly_on_cpu_tensors():
    from multimodalstudio_amd import hip_ops
    x = torch.zeros(4, 3)
    t = torch.zeros(16 << 12, 2)
    with pytest.raises(RuntimeError):
        hip_ops.hashgrid_forward(x, t, [16.0] * 16, 12, 1.0, 16)


def test_lr_and_curvature_schedules_match_oracle():
    from multimodalstudio_amd import pipeline
    from oracle import model as om
    for max_iters in (100000, 50000, 20000):
        for step in (0, 1, 999, 4999, 10000, 10001, 19999, 49999, 50000, 75000, 90000, 99999):
            if step >= max_iters:
                continue
            assert pipeline.lr_factor(step, max_iters) == om.lr_factor(step, max_iters)
            st = om.StepState(step=step, max_iters=max_iters)
            assert pipeline.curvature_factor(step, max_iters) == st.curvature_factor, (step, max_iters)


def test_compute_loss_uses_the_runs_max_iters():
    """The curvature weight follows num_iterations (schedulers.py:320-343): compute_loss must not fall back to the
    100k default.  Checked on the host through the factor compute_loss passes to the weight."""
    import inspect
    from multimodalstudio_amd import pipeline
    assert "curvature_factor(step, max_iters)" in inspect.getsource(pipeline._finish_loss)
    # the fused step-loss node and both per-term geometry-loss paths
    assert inspect.getsource(pipeline.compute_loss).count("step, max_iters)") == 3
    assert "max_iters=self.cfg.max_iters" in inspect.getsource(pipeline.Trainer._compute_grads)
    from multimodalstudio_amd import graphs
    assert "max_iters=t.cfg.max_iters" in inspect.getsource(graphs.GraphTrainer._forward_backward_body)
    assert pipeline.curvature_factor(45000, 50000) != pipeline.curvature_factor(45000, 100000)


def _ddp_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from multimodalstudio_amd.ddp import DDP

    class G:
        pass
    g = G()
    n = 1000003
    g.grad = torch.arange(n, dtype=torch.float32) * (rank + 1)
    ddp = DDP(world, bucket_bytes=1 << 20)   # several buckets
    ddp.allreduce_grads([g])
    mx = ddp.max_over_ranks(float(rank) + 0.5, torch.device("cpu"))
    expect = torch.arange(n, dtype=torch.float32) * (sum(range(1, world + 1)) / world)
    q.put((rank, bool(torch.allclose(g.grad, expect)), mx))
    dist.destroy_process_group()


def test_ddp_gradient_average_gloo_world2():
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res
    assert all(mx == 1.5 for _, _, mx in res), res


def test_every_called_entry_point_is_declared():
    """Each _lib.call("mms_...") in the package names a header declaration (an undeclared one would be called with
    ctypes' default 32-bit argument conversion; _lib.call refuses it at run time, this catches it statically)."""
    import re
    from multimodalstudio_amd import _lib
    pkg = os.path.join(ROOT, "multimodalstudio_amd")
    called = set()
    for fn in os.listdir(pkg):
        if fn.endswith(".py"):
            called |= set(re.findall(r'call\(\s*"(mms_\w+)"', open(os.path.join(pkg, fn)).read()))
    assert called, "no entry-point calls found"
    missing = sorted(c for c in called if c not in _lib.SIGNATURES)
    assert not missing, f"called but not declared in include/mms_hip.h: {missing}"


def test_graph_capacity_buckets():
    from multimodalstudio_amd.graphs import bucket_capacity
    assert bucket_capacity([850], 64, 2048) == 896
    assert bucket_capacity([850, 900, 12], 64, 2048) == 960
    assert bucket_capacity([896], 64, 2048) == 896
    assert bucket_capacity([2040], 64, 2048) == 2048
    assert bucket_capacity([1], 64, 2048) == 64


def test_model_init_matches_train_parity_fixture():
    """BaseModel parameter initialisation consumes the RNG in the fixture's order (construction order of the module
    tree): the same seed gives the init the training-parity fixture recorded (caught on the host, before the GPU)."""
    import ast
    import numpy as np
    from multimodalstudio_amd import model as mm
    from multimodalstudio_amd import scene as ms
    f = np.load(os.path.join(os.path.dirname(__file__), "golden", "train_parity_rgb.npz"))
    cfg = ast.literal_eval(f["cfg_json"].tobytes().decode())
    torch.manual_seed(654824)
    model = mm.BaseModel(mm.ModelSpec({m: ms.CHANNELS[m] for m in cfg["modalities"]}, log2T=cfg["log2T"]))
    ck = float(sum(float(v.detach().double().abs().sum()) for v in model.state_dict().values()))
    assert ck == pytest.approx(float(f["init_checksum"]), rel=1e-9)


def test_zero_arena_is_sized_by_the_first_step_and_carved_after():
    """functions._ZeroArena (host logic, on CPU tensors): the first step only measures its demand (fresh zeroed
    buffers), the arena is allocated at that step's end -- before the graphs captured next -- and later steps carve
    zeroed, 256-B aligned, non-overlapping views from it (round-2 fix: the demand used to be counted only once the
    buffer existed, so the arena never engaged)."""
    from multimodalstudio_amd import functions as fx
    a, dev = fx._ARENA, torch.device("cpu")
    saved = (a.buf, list(a.keep), a.need, a.off, a.in_step, a.active, a.dev)
    try:
        a.buf, a.keep, a.need = None, [], 0
        fx.zero_arena_begin(dev)
        first = fx._zeroed_views([(5, 3), None, (7,)], dev)
        assert first[1] is None and a.buf is None and a.need > 0
        fx.zero_arena_end()
        assert a.buf is not None and a.buf.numel() >= a.need
        fx.zero_arena_begin(dev)
        v1, v2 = fx._zeroed_views([(5, 3), (7,)], dev)
        base, end = a.buf.data_ptr(), a.buf.data_ptr() + 4 * a.buf.numel()
        for v in (v1, v2):
            assert base <= v.data_ptr() < end and (v.data_ptr() - base) % 256 == 0 and float(v.abs().sum()) == 0.0
        assert v2.data_ptr() >= v1.data_ptr() + 4 * v1.numel()
        v1.fill_(3.0)
        fx.zero_arena_end()
        fx.zero_arena_begin(dev)           # the next step's fill zeroes what the last one wrote
        w1, = fx._zeroed_views([(5, 3)], dev)
        assert w1.data_ptr() == v1.data_ptr() and float(w1.abs().sum()) == 0.0
        # an all-None request carves nothing (it used to advance the offset by one float, misaligning
        # every later view of the step)
        off = a.off
        assert fx._zeroed_views([None, None], dev) == [None, None] and a.off == off
        w2, = fx._zeroed_views([(3,)], dev)
        assert (w2.data_ptr() - a.buf.data_ptr()) % 256 == 0
        fx.zero_arena_end()
    finally:
        a.buf, a.keep, a.need, a.off, a.in_step, a.active, a.dev = saved


def test_benchmarked_preset_keeps_the_sdf_forward_split_bf16x3():
    """The preset bench.py benchmarks by default (bench.DEFAULT_PRECISION, VERDICT r5: this guard used to check `fast`
    while the bench ran `fast_h16b`) keeps the SDF MLP forward on split-bf16x3 -- the bf16-weight SDF chain (prec 3,
    preset fast_x2) moved the hessians 56x the reference's hessian scale (tests/test_gpu_e2e.py) --, its weight
    gradients on split-bf16x3 or, for the hidden layers, fp16 (wgrad16, with fp16 activation rows y16 only beside
    it: the reference GPU's autocast precision), the radiance / head / background forwards on split-bf16x3 or fp16
    (bf16 there cost 0.56 dB of converged PSNR, profiles/round3_converged_psnr.json), and the mlp methods'
    analytic-gradient fields on fp32."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from multimodalstudio_amd import functions as fx
    p = fx.PRESETS[bench.DEFAULT_PRECISION]
    assert p["sdf"] == 2 and p["sdf_chain"] in (0, 2) and p["mlp"] == 0 and p["wgrad"] == 0
    assert p["wgrad16"] in (0, 1) and (p["y16"] == 0 or (p["wgrad16"] == 1 and p["bwd16"] == 1))
    assert all(p[k] in (2, 5) for k in ("radiance", "heads", "pol_head", "background"))
    assert fx.PRESETS["fast_x2"]["sdf_chain"] == 3
    assert fx.fwd_prec(4) == 2 and fx.bwd_prec(4) == 1 and fx.fwd_prec(2) == fx.bwd_prec(2) == 2
    assert fx.fwd_prec(5) == 5 and fx.bwd_prec(5) == 2


def test_ssim_matches_direct_window_sums():
    """evaluate.ssim (torchmetrics' SSIM restated: 11x11 Gaussian, sigma 1.5, reflect padding, interior mean) against
    direct per-window sums in numpy; identical images score 1, noise lowers it."""
    from multimodalstudio_amd import evaluate as ev
    g = torch.Generator().manual_seed(0)
    x = torch.rand(21, 18, 2, generator=g)
    y = (x + 0.1 * torch.randn(21, 18, 2, generator=g)).clip(0, 1)
    assert abs(ev.ssim(x, x) - 1.0) < 1e-12
    k, sig = 11, 1.5
    d = np.arange(k) - (k - 1) / 2
    w1 = np.exp(-(d / sig) ** 2 / 2)
    w1 /= w1.sum()
    w = np.outer(w1, w1)
    p = (k - 1) // 2
    xs = np.pad(x.numpy().astype(np.float64), ((p, p), (p, p), (0, 0)), mode="reflect")
    ys = np.pad(y.numpy().astype(np.float64), ((p, p), (p, p), (0, 0)), mode="reflect")
    H, W = xs.shape[0] - 2 * p, xs.shape[1] - 2 * p
    c1, c2 = 0.01 ** 2, 0.03 ** 2
    vals = []
    for c in range(2):
        for i in range(p, H - p):        # the map is cropped to the interior of the unpadded image
            for j in range(p, W - p):
                a = xs[i:i + k, j:j + k, c]
                b = ys[i:i + k, j:j + k, c]
                mx, my = (w * a).sum(), (w * b).sum()
                vx = (w * a * a).sum() - mx * mx
                vy = (w * b * b).sum() - my * my
                cxy = (w * a * b).sum() - mx * my
                vals.append(((2 * mx * my + c1) * (2 * cxy + c2)) / ((mx * mx + my * my + c1) * (vx + vy + c2)))
    assert abs(ev.ssim(y, x) - float(np.mean(vals))) < 1e-10
    assert ev.ssim(y, x) < 0.99


def test_polarization_extras():
    """evaluate.degree_of_polarization / angle_of_polarization (polarizer.py:103-134) on intensities of known Stokes
    vectors: I = 0.5 [s0 + s1, s0 + s2, s0 - s1, s0 - s2]."""
    from multimodalstudio_amd import evaluate as ev
    s0, p, psi = 0.8, 0.3, 0.4
    s1, s2 = s0 * p * np.cos(2 * psi), s0 * p * np.sin(2 * psi)
    I = 0.5 * torch.tensor([[s0 + s1, s0 + s2, s0 - s1, s0 - s2]], dtype=torch.float64)
    assert abs(float(ev.degree_of_polarization(I)[0]) - p) < 1e-12
    assert abs(float(ev.angle_of_polarization(I)[0]) - psi) < 1e-6


def test_small_linear_serves_only_shapes_with_a_backward(L):
    """functions.SmallRun accepts a layer for the narrow-layer kernels only where mms_small_linear_bwd accepts it too
    (checked through the C-ABI's argument validation: M = 0 returns after the shape checks, no device work)."""
    from multimodalstudio_amd.functions import SmallRun
    for K in (64, 128, 256, 512):
        for N in range(1, 18):
            rc_b = L.mms_small_linear_bwd(None, K, 0, K, None, N, 0, 1.0, 20.0, None, N, None, N, None, K, 0, None,
                                          None, None)
            rc_f = L.mms_small_linear_fwd(None, K, 0, K, None, None, N, 0, 1.0, 20.0, None, N, None)
            ok = SmallRun.shape_ok(N, K)
            assert ok == (rc_b == 0 and rc_f == 0), (N, K, rc_b, rc_f, _err(L))
