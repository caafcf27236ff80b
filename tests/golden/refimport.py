"""Import helper for the read-only reference (THIS CONTAINER ONLY; never on the GPU box).

Used solely by ``make_golden.py`` to generate the committed golden fixtures.  It installs
permissive stub modules for third-party packages that are absent from this image
(tyro, lightning, cv2, ...) so the reference's pure-PyTorch hot path can be imported and
executed, and applies the two patches documented in SURVEY.md §8(c):

* hash grids use ``interpolation="Linear"`` (the torch fallback asserts on anything else,
  /root/reference/src/field_components/encodings.py:235-238);
* ``SHEncoding`` is routed to the reference's own torch SH helper
  (/root/reference/src/utils/math.py:21-83) because encodings.py:377 calls tcnn unconditionally.
"""
import importlib.abc
import importlib.machinery
import os
import sys
import types

REF_SRC = "/root/reference/src"
_STUB_TOP = {
    "torchtyping", "tyro", "cv2", "torchvision", "lightning", "torchmetrics", "trimesh",
    "skimage", "h5py", "polanalyser", "wandb", "mcubes", "pymeshlab", "lpips", "tensorboard",
}


class _Stub:
    def __init__(self, *a, **k):
        pass

    def __call__(self, *a, **k):
        return _Stub()

    def __getattr__(self, name):
        if name.startswith("__") and name.endswith("__"):
            raise AttributeError(name)
        return _Stub()

    def __getitem__(self, item):
        return _Stub()

    def __class_getitem__(cls, item):
        return cls

    def __mro_entries__(self, bases):
        return (object,)

    def __iter__(self):
        return iter(())

    def __bool__(self):
        return False


class _StubModule(types.ModuleType):
    def __getattr__(self, name):
        if name.startswith("__") and name.endswith("__"):
            raise AttributeError(name)
        return _Stub


class _Finder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    def find_spec(self, fullname, path=None, target=None):
        top = fullname.split(".")[0]
        if top in _STUB_TOP or fullname == "torch.utils.tensorboard" or fullname.startswith("torch.utils.tensorboard."):
            return importlib.machinery.ModuleSpec(fullname, self, is_package=True)
        return None

    def create_module(self, spec):
        m = _StubModule(spec.name)
        m.__path__ = []
        return m

    def exec_module(self, module):
        pass


_installed = False


def install():
    """Install stubs + sys.path entry; import configs first (circular-import order)."""
    global _installed
    if _installed:
        return
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    sys.meta_path.insert(0, _Finder())
    sys.path.insert(0, REF_SRC)
    import configs.configs  # noqa: F401  (must be first)
    _installed = True


def patch_sh_and_hash():
    """Apply the two SURVEY §8(c) patches (see module docstring)."""
    install()
    import field_components.encodings as enc
    from utils.math import components_from_spherical_harmonics

    if getattr(enc.SHEncoding, "_mms_patched", False):
        return

    def sh_init(self, config, in_dim=3):
        enc.Encoding.__init__(self, config, in_dim=in_dim)

    def sh_forward(self, x):
        return components_from_spherical_harmonics(self.config.degree + 1, x)

    enc.SHEncoding.__init__ = sh_init
    enc.SHEncoding.forward = sh_forward
    enc.SHEncoding._mms_patched = True

    orig_init = enc.HashEncoding.__init__

    def hash_init(self, config, in_dim=3):
        config.interpolation = "Linear"
        config.implementation = "torch"
        orig_init(self, config, in_dim=in_dim)

    enc.HashEncoding.__init__ = hash_init


def build_model(method, yaml_path=None, modalities=None, overrides=None):
    """Build the reference BaseModel for ``method`` (+ YAML merge), CPU, train mode."""
    import copy
    import yaml as _yaml
    patch_sh_and_hash()
    from configs.method_configs import method_configs
    from configs.configs import Config
    from data.scene_box import SceneBox

    cfg = copy.deepcopy(method_configs[method])
    if yaml_path is not None:
        with open(yaml_path) as f:
            upd = _yaml.safe_load(f)
        upd = {k: v for k, v in upd.items() if k in cfg.__dict__}
        Config.update_config(cfg, upd)
    if overrides:
        Config.update_config(cfg, overrides)
    mods = modalities if modalities is not None else {"rgb": 3}
    model = cfg.pipeline.model.setup(scene_box=SceneBox(radius=1.0, collider_type="sphere"), modalities=mods)
    return cfg, model
