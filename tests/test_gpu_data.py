"""GPU input stage: the device pixel sampler (mms_pixel_sample) and training from an on-disk MMS-DATA scene.

The device sampler draws from Philox, not torch.Generator, so it is checked for its distribution (uniform frames,
columns and rows within 5 % over 262144 draws), for gathering exactly images[frame, y, x], for advancing its device
counter (inside a captured graph too), and end to end: graph-replayed training steps from a scene written to disk.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_pixel_sampler_distribution_and_values(dev):
    from multimodalstudio_amd.data import GPUPixelSampler
    g = torch.Generator().manual_seed(0)
    frames = {"rgb": torch.rand(7, 13, 17, 3, generator=g).to(dev), "polarization": torch.rand(5, 9, 11, 1, generator=g).to(dev)}
    n = 1 << 18
    s = GPUPixelSampler(frames, n, seed=1234)
    coords, sel, vals = s.sample()
    torch.cuda.synchronize()
    for m, img in frames.items():
        F, H, W, C = img.shape
        c = coords[m].long()
        assert int(c[:, 0].min()) >= 0 and int(c[:, 0].max()) < F
        assert torch.equal(c[:, 0], sel[m])
        for col, k in [(0, F), (1, H), (2, W)]:
            cnt = torch.bincount(c[:, col], minlength=k).double()
            assert cnt.numel() == k
            assert float((cnt / (n / k) - 1).abs().max()) < 0.05, (m, col)
        assert torch.equal(vals[m], img[sel[m], c[:, 1], c[:, 2]])
    first = coords["rgb"].clone()
    assert int(s.counters["rgb"].item()) == n
    s.sample()
    torch.cuda.synchronize()
    assert not torch.equal(first, coords["rgb"])
    assert int(s.counters["rgb"].item()) == 2 * n
    # the draw counter advances on the device: a captured graph replays fresh draws
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            s.sample()
    torch.cuda.current_stream().wait_stream(side)
    graph.replay()
    torch.cuda.synchronize()
    a = coords["rgb"].clone()
    graph.replay()
    torch.cuda.synchronize()
    assert not torch.equal(a, coords["rgb"])


def test_training_from_disk_with_device_sampler(dev, tmp_path):
    from multimodalstudio_amd import data as md
    from multimodalstudio_amd import functions as fx
    from multimodalstudio_amd.graphs import GraphTrainer
    from multimodalstudio_amd.pipeline import TrainConfig, Trainer
    path = md.write_synthetic_scene(str(tmp_path / "scene"), ["rgb", "polarization"], n_views=12, width=64,
                                    height=48, raw=True)
    fx.set_precision("fast")
    try:
        t = Trainer(TrainConfig(method="grid_raw", modalities=("rgb", "polarization"), num_rays_per_modality=512,
                                log2T=14, data_dir=path, gpu_sampler=True), dev)
        assert t.images["rgb"].shape == (11, 48, 64, 1)      # 12 views minus eval view 9
        t.set_step(95000)
        g = GraphTrainer(t)
        losses = [float(g.step()[1]) for _ in range(6)]
    finally:
        fx.set_precision("fp32")
    assert all(np.isfinite(losses)), losses
    assert g.disabled is None and g.stats["replays"] >= 1, g.stats
