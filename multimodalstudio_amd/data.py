"""On-disk MMS-DATA scenes and the GPU-resident input stage.

* Format: ``<scene>/meta_data.json`` + ``<scene>/modalities/<mod>/<frame>.png|.npy``, the schema
  preprocessing/utils.py:469-571 writes (/root/reference/src): per modality the camera model, width / height,
  fx / fy / cx / cy, ``distortion_params`` (6 values, read in the reader's order [k1, k2, k3, k4, p1, p2],
  camera_utils.py:302-307 -- SURVEY Appendix A item 1), the raw ``mosaick_pattern`` and per frame ``frame_id``,
  ``file_name`` and the 3x4 ``camtoworld``; top level ``raw``, ``undistorted``, ``pixel_offset``, ``scene_box``,
  ``worldtogt``.
* ``MMSDataset`` loads a split like MultimodalAlignedDataset / RawMultimodalAlignedDataset (datasets.py:303-360,
  444-529, 608-633): frames filtered by frame id, sorted, normalised to [0, 1] when stored as integers
  (utils/misc.py:150-157), BGR -> RGB for demosaicked rgb (:477-483), mosaick masks for raw scenes (:229-254), and
  per-modality channel counts (:171-176, :296-301).  Frames go to HBM once (CacheDataloader caches them in
  memory, dataloaders.py:107-167).
* ``GPUPixelSampler`` draws every step's pixels on the device (``mms_pixel_sample``): coordinates, frame
  selection and target values without host work or a host-to-device copy.
* ``write_synthetic_scene`` writes the analytic scene of scene.py in this format (tests, benchmarks).
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from . import scene as mscene

CHANNEL_FORMAT = {1: ".png", 3: ".png"}     # preprocessing/utils.py:548-555: png for 1 / 3 channels, else npy


# ------------------------------------------------------------------------------------------------
# frame I/O (utils/io.py:42-63, utils/misc.py:150-157)
# ------------------------------------------------------------------------------------------------
def read_frame(path: str) -> np.ndarray:
    """read_frame: png -> [H, W, C] in the file's integer type (3-channel pngs in BGR order, as cv2.imread
    returns them), npy -> the stored array."""
    if path.lower().endswith(".npy"):
        return np.load(path, allow_pickle=False)
    from PIL import Image
    with Image.open(path) as im:
        a = np.array(im)
    if a.ndim == 2:
        return a[..., None]
    if a.shape[-1] == 3:
        return a[..., ::-1].copy()          # PIL gives RGB; cv2.imread gives BGR
    return a


def write_frame(path: str, frame: np.ndarray) -> None:
    """write_frame: png for uint8 / uint16 frames with 1 or 3 channels (3 channels given in BGR order), npy else."""
    if path.lower().endswith(".npy"):
        np.save(path, frame)
        return
    from PIL import Image
    if frame.shape[-1] == 1:
        Image.fromarray(frame[..., 0]).save(path)
    else:
        Image.fromarray(np.ascontiguousarray(frame[..., ::-1])).save(path)


def normalize_frame(frame: np.ndarray) -> np.ndarray:
    if frame.dtype == np.uint8:
        return frame / 255.0
    if frame.dtype == np.uint16:
        return frame / 65535.0
    raise NotImplementedError(f"Normalization for {frame.dtype} not implemented.")


# ------------------------------------------------------------------------------------------------
# dataset
# ------------------------------------------------------------------------------------------------
class MMSDataset:
    """One split of an MMS-DATA scene for ``modalities``.

    ``indexes_to_choose`` / ``indexes_to_exclude``: frame ids per modality (None = every frame), the datamanager's
    eval_image_indices_per_modality / skip_image_indices_per_modality split."""

    def __init__(self, data_dir: str, modalities: Sequence[str],
                 indexes_to_choose: Optional[Dict[str, Sequence[int]]] = None,
                 indexes_to_exclude: Optional[Dict[str, Sequence[int]]] = None):
        self.data_dir = data_dir
        self.modalities = list(modalities)
        with open(os.path.join(data_dir, "meta_data.json")) as f:
            self.metadata = json.load(f)
        md = self.metadata
        self.raw = bool(md.get("raw", False))
        self.pixel_offset = float(md.get("pixel_offset", 0.0))
        self.scene_box = md["scene_box"]
        self.images: Dict[str, torch.Tensor] = {}
        self.cameras: Dict[str, mscene.ModalityCameras] = {}
        self.mosaick_masks: Dict[str, torch.Tensor] = {}
        for mod in self.modalities:
            m = md["modalities"][mod]
            choose = set(indexes_to_choose[mod]) if indexes_to_choose and mod in indexes_to_choose else None
            exclude = set(indexes_to_exclude[mod]) if indexes_to_exclude and mod in indexes_to_exclude else set()
            frames = [fr for fr in m["frames"] if (choose is None or fr["frame_id"] in choose)
                      and fr["frame_id"] not in exclude]
            frames.sort(key=lambda fr: fr["frame_id"])
            imgs = []
            for fr in frames:
                a = read_frame(os.path.join(data_dir, "modalities", mod, fr["file_name"]))
                if a.max() > 1:
                    a = normalize_frame(a)
                imgs.append(torch.tensor(np.asarray(a, dtype=np.float32)))
            images = torch.stack(imgs)
            if mod == "rgb" and not self.raw and images.shape[-1] == 3:
                images = images[..., [2, 1, 0]]      # MultimodalAlignedDataset.load_data: BGR -> RGB
            self.images[mod] = images
            C = len(frames)
            dist = None
            if not md.get("undistorted", False):
                dist = torch.tensor(m["distortion_params"], dtype=torch.float32).expand(C, 6).contiguous()
            self.cameras[mod] = mscene.ModalityCameras(
                c2w=torch.tensor([fr["camtoworld"] for fr in frames], dtype=torch.float32),
                fx=torch.full((C,), float(m["fx"])), fy=torch.full((C,), float(m["fy"])),
                cx=torch.full((C,), float(m["cx"])), cy=torch.full((C,), float(m["cy"])),
                distortion=dist, width=int(m["width"]), height=int(m["height"]),
                view_ids=[fr["frame_id"] for fr in frames])
            if self.raw:
                self.mosaick_masks[mod] = build_mosaick_mask(torch.tensor(m["mosaick_pattern"]), int(m["width"]),
                                                             int(m["height"]))

    def get_channels_per_modality(self) -> Dict[str, int]:
        if self.raw:
            return {m: int(len(torch.unique(torch.tensor(self.metadata["modalities"][m]["mosaick_pattern"]))))
                    for m in self.modalities}
        return {m: int(self.images[m].shape[-1]) for m in self.modalities}

    def __len__(self) -> int:
        return int(self.images[self.modalities[0]].shape[0])


def build_mosaick_mask(pattern: torch.Tensor, width: int, height: int) -> torch.Tensor:
    """RawDataset.build_mosaick_mask (datasets.py:229-250): the pattern tiled over H x W, int8."""
    nw, nh = -(-width // pattern.shape[1]), -(-height // pattern.shape[0])
    return pattern.repeat((nh, nw))[:height, :width].to(torch.int8)


# ------------------------------------------------------------------------------------------------
# synthetic scene writer
# ------------------------------------------------------------------------------------------------
def write_synthetic_scene(path: str, modalities: Sequence[str], n_views: int = 50, width: int = 640,
                          height: int = 512, raw: bool = True, seed: int = 0,
                          formats: Optional[Dict[str, str]] = None) -> str:
    """scene.py's analytic scene in the MMS-DATA on-disk format: 1- and 3-channel frames as 16- / 8-bit pngs,
    others as npy (float32); raw scenes store the mosaicked single-band frames and each modality's pattern.
    ``formats[mod]``: 'png' / 'npy' (float32) / 'npy_u16' (uint16 counts, normalised by the loader) overrides the
    default per modality (an all-npy scene is what the reference's loader reads without OpenCV)."""
    os.makedirs(os.path.join(path, "modalities"), exist_ok=True)
    cams = mscene.make_cameras(list(modalities), n_views, width, height, seed=seed, train=None)
    md = {"undistorted": False, "raw": bool(raw), "pixel_offset": 0.0,
          "scene_box": {"aabb": [[-1, -1, -1], [1, 1, 1]], "collider_type": "sphere", "radius": 1.0},
          "worldtogt": np.eye(4).tolist(), "modalities": {}}
    for mod in modalities:
        c = cams[mod]
        ch = mscene.CHANNELS[mod]
        frames = mscene.render_frames(c, ch, torch.device("cpu"), mod if raw else None).numpy()
        os.makedirs(os.path.join(path, "modalities", mod), exist_ok=True)
        entries = []
        nc = frames.shape[-1]
        fmt = (formats or {}).get(mod, "png" if nc in CHANNEL_FORMAT else "npy")
        for i, v in enumerate(c.view_ids):
            ext = ".png" if fmt == "png" else ".npy"
            name = f"{v:04}{ext}"
            f = frames[i]
            if fmt == "npy_u16":
                f = np.round(f * 65535.0).astype(np.uint16)
            if ext == ".png":
                f = np.round(f * (65535.0 if nc == 1 else 255.0)).astype(np.uint16 if nc == 1 else np.uint8)
                if nc == 3:
                    f = f[..., ::-1]                 # stored BGR, as cv2.imwrite would
            write_frame(os.path.join(path, "modalities", mod, name), f)
            entries.append({"frame_id": int(v), "file_name": name, "camtoworld": c.c2w[i].tolist()})
        m = {"camera_model": "OPENCV", "width": width, "height": height, "fx": float(c.fx[0]), "fy": float(c.fy[0]),
             "cx": float(c.cx[0]), "cy": float(c.cy[0]), "distortion_params": c.distortion[0].tolist(),
             "frames": entries}
        if raw:
            m["mosaick_pattern"] = mscene.MOSAICK[mod]
        md["modalities"][mod] = m
    with open(os.path.join(path, "meta_data.json"), "w") as f:
        json.dump(md, f, indent=2)
    return path


# ------------------------------------------------------------------------------------------------
# GPU pixel sampler
# ------------------------------------------------------------------------------------------------
class GPUPixelSampler:
    """UniformPixelSampler over HBM-resident frames, drawn on the device (mms_pixel_sample).

    ``frames[mod]``: [n_frames, H, W, C] device tensor; every ``sample`` call writes coordinates [n, 3] int32,
    frame selections [n] int64 and target values [n, C] into persistent device buffers (graph-capturable: the draw
    counters advance on the device).  Each modality has its own Philox stream (seed, stream id = modality
    position + 16 * rank)."""

    def __init__(self, frames: Dict[str, torch.Tensor], num_rays_per_modality: int, seed: int, rank: int = 0):
        self.frames = frames
        self.n = int(num_rays_per_modality)
        self.seed = int(seed)
        dev = next(iter(frames.values())).device
        self.counters = {m: torch.zeros(1, dtype=torch.int64, device=dev) for m in frames}
        self.stream_ids = {m: i + 16 * rank for i, m in enumerate(frames)}
        self.coords = {m: torch.empty(self.n, 3, dtype=torch.int32, device=dev) for m in frames}
        self.sel = {m: torch.empty(self.n, dtype=torch.int64, device=dev) for m in frames}
        self.values = {m: torch.empty(self.n, f.shape[-1], device=dev) for m, f in frames.items()}
        self.frame_ids = {m: torch.arange(f.shape[0], dtype=torch.int32, device=dev) for m, f in frames.items()}

    def sample(self):
        """(coords, sel, values) per modality, all on the device (views of persistent buffers)."""
        for m, img in self.frames.items():
            Fn, H, W, C = img.shape
            _lib.call("mms_pixel_sample", self.seed, self.stream_ids[m], self.counters[m].data_ptr(), self.n, Fn, H,
                      W, self.frame_ids[m].data_ptr(), img.data_ptr(), C, self.coords[m].data_ptr(),
                      self.sel[m].data_ptr(), self.values[m].data_ptr(), torch.cuda.current_stream().cuda_stream)
        return self.coords, self.sel, self.values
