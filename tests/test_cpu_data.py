"""On-disk MMS-DATA format (data.py) on the host: the writer's scene reads back as the analytic frames, cameras,
splits and mosaick masks (datasets.py:229-254, 444-529 semantics), and the frame I/O keeps cv2's channel order."""
import json
import os

import numpy as np
import pytest
import torch

from multimodalstudio_amd import data as md
from multimodalstudio_amd import scene as ms


@pytest.fixture(scope="module")
def scenes(tmp_path_factory):
    root = tmp_path_factory.mktemp("mmsdata")
    mods = ["rgb", "infrared", "polarization", "multispectral"]
    raw = md.write_synthetic_scene(str(root / "raw"), mods, n_views=12, width=40, height=30, raw=True)
    dem = md.write_synthetic_scene(str(root / "dem"), mods, n_views=12, width=40, height=30, raw=False)
    return mods, raw, dem


def test_metadata_schema(scenes):
    mods, raw, _ = scenes
    meta = json.load(open(os.path.join(raw, "meta_data.json")))
    assert meta["raw"] is True and meta["undistorted"] is False and meta["pixel_offset"] == 0.0
    assert meta["scene_box"]["collider_type"] == "sphere"
    for m in mods:
        e = meta["modalities"][m]
        assert len(e["distortion_params"]) == 6 and e["mosaick_pattern"] == ms.MOSAICK[m]
        assert [f["frame_id"] for f in e["frames"]] == list(range(12))
        assert np.asarray(e["frames"][0]["camtoworld"]).shape == (3, 4)


@pytest.mark.parametrize("raw", [True, False])
def test_dataset_reads_back_the_scene(scenes, raw):
    mods, raw_dir, dem_dir = scenes
    path = raw_dir if raw else dem_dir
    excl = {m: list(ms.EVAL_VIEWS) for m in mods}
    ds = md.MMSDataset(path, mods, indexes_to_exclude=excl)
    ref_cams = ms.make_cameras(mods, 12, 40, 30, seed=0, train=True)
    assert ds.raw == raw
    for m in mods:
        c = ds.cameras[m]
        assert c.view_ids == [v for v in range(12) if v not in ms.EVAL_VIEWS]
        assert torch.allclose(c.c2w, ref_cams[m].c2w)
        assert torch.allclose(c.distortion, ref_cams[m].distortion)
        ref = ms.render_frames(ref_cams[m], ms.CHANNELS[m], torch.device("cpu"), m if raw else None)
        got = ds.images[m]
        assert got.shape == ref.shape, (m, got.shape, ref.shape)
        nc = got.shape[-1]
        tol = 0.5 / 65535 + 1e-7 if nc == 1 else (0.5 / 255 + 1e-7 if nc == 3 else 0.0)
        assert float((got - ref).abs().max()) <= tol, m
        if raw:
            assert torch.equal(ds.mosaick_masks[m], ms.mosaick_mask(m, 40, 30))
    assert ds.get_channels_per_modality() == {m: ms.CHANNELS[m] for m in mods}
    ev = md.MMSDataset(path, ["rgb"], indexes_to_choose={"rgb": [9]})
    assert ev.cameras["rgb"].view_ids == [9] and len(ev) == 1


def test_frame_io_channel_order(tmp_path):
    bgr = (np.arange(5 * 4 * 3) % 256).astype(np.uint8).reshape(5, 4, 3)
    p = str(tmp_path / "f.png")
    md.write_frame(p, bgr)
    assert np.array_equal(md.read_frame(p), bgr)        # cv2 semantics: what is written BGR reads back BGR
    g16 = (np.arange(20) * 3000).astype(np.uint16).reshape(5, 4, 1)
    md.write_frame(str(tmp_path / "g.png"), g16)
    assert np.array_equal(md.read_frame(str(tmp_path / "g.png")), g16)
    assert md.normalize_frame(g16).max() == pytest.approx(57000 / 65535)


@pytest.mark.parametrize("tag", ["raw", "demosaicked"])
def test_loader_matches_reference_dataset(tmp_path, tag):
    """MMSDataset against the reference's own loader (tests/golden/loader.npz: RawMultimodalAlignedDataset /
    MultimodalAlignedDataset, datasets.py:229-301, 303-360, 444-529, 608-633, run by tests/golden/make_golden.py
    loader on the same writer's all-npy scenes, float32 and uint16 frames): frames, cameras, split, mosaick masks and
    channel counts exactly equal."""
    gold = np.load(os.path.join(os.path.dirname(__file__), "golden", "loader.npz"))
    # the scene table of the fixture generator, restated (make_golden imports the reference at module level)
    scenes = {
        "raw": (True, ("rgb", "infrared", "mono", "polarization", "multispectral"),
                {"rgb": "npy", "infrared": "npy_u16", "mono": "npy", "polarization": "npy", "multispectral": "npy_u16"},
                (1, 4)),
        "demosaicked": (False, ("rgb", "mono", "multispectral"),
                        {"rgb": "npy", "mono": "npy_u16", "multispectral": "npy"}, (2,)),
    }
    raw, mods, fmts, excl = scenes[tag]
    d = md.write_synthetic_scene(str(tmp_path / tag), mods, raw=raw, formats=fmts, n_views=7, width=40, height=26,
                                 seed=3)
    ds = md.MMSDataset(d, mods, indexes_to_exclude={m: list(excl) for m in mods})
    chans = ds.get_channels_per_modality()
    for m in mods:
        cam = ds.cameras[m]
        assert cam.view_ids == [int(i) for i in gold[f"{tag}:indexes"]], m
        np.testing.assert_array_equal(ds.images[m].numpy(), gold[f"{tag}:{m}:images"], err_msg=m)
        np.testing.assert_array_equal(cam.c2w.numpy(), gold[f"{tag}:{m}:c2w"], err_msg=m)
        for k in ("fx", "fy", "cx", "cy"):
            np.testing.assert_array_equal(getattr(cam, k).numpy(), gold[f"{tag}:{m}:{k}"].reshape(-1), err_msg=k)
        np.testing.assert_array_equal(cam.distortion.numpy(), gold[f"{tag}:{m}:distortion"], err_msg=m)
        assert chans[m] == int(gold[f"{tag}:{m}:channels"]), m
        if raw:
            np.testing.assert_array_equal(ds.mosaick_masks[m].numpy(), gold[f"{tag}:{m}:mosaick_mask"], err_msg=m)
    assert float(ds.scene_box["radius"]) == float(gold[f"{tag}:radius"])


REF_CONFS = "/root/reference/confs"


@pytest.mark.parametrize("name", ["grid.yaml", "grid_raw.yaml", "mlp_raw.yaml", "grid_raw_rgb_all_views_pol_10_views.yaml"])
def test_conf_extracts_match_reference(name):
    """confs/*.yaml (the training-step keys the bench and trainer read, e.g. config 5's skipped polarization views)
    parse to the same values as the reference's own YAML file (checked where the reference is present)."""
    from multimodalstudio_amd.pipeline import CONFS, read_conf
    mine = read_conf(os.path.join(CONFS, name))
    if os.path.isdir(REF_CONFS):
        assert mine == read_conf(os.path.join(REF_CONFS, name))
    assert mine["num_rays_per_modality"] == 2048 and mine["max_num_iterations"] == 100000


def test_config5_skip_views():
    """Config 5 (grid_raw_grid_bg_unbalanced) trains polarization on 10 of the 45 non-eval views."""
    from multimodalstudio_amd import scene as ms
    from multimodalstudio_amd.pipeline import skip_views_for
    skip = skip_views_for("grid_raw_grid_bg_unbalanced")
    assert set(skip) == {"polarization"}
    train = [v for v in range(50) if v not in ms.EVAL_VIEWS and v not in skip["polarization"]]
    assert len(train) == 10
    assert skip_views_for("grid_raw") is None
