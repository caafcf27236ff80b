"""Parameters of the full-size golden fixture (tests/golden/e2e_full_grid_rgb_l19.npz), regenerated instead of stored.

BASELINE configs[1] at its own size has two 64 MiB hash tables; the fixture keeps none of its parameters.  They are the
product's BaseModel initialised under torch.manual_seed(FULL_SEED) on the CPU (deterministic for one torch build: the
same image runs here and on the GPU box) with every hash table replaced by oracle.hashgrid.deterministic_table x
FULL_TABLE_SCALE, and the SDF MLP's grid-feature input columns given deterministic weights.  The fixture stores ``param_checksum`` of the non-table parameters, so an init that drifted is caught
before any comparison.  Test infrastructure: imported by tests/golden/make_golden.py and the tests only.
"""
from __future__ import annotations

FULL_SEED = 1234
FULL_TABLE_SCALE = 50.0
# the smooth full-size fixture (e2e_full_grid_rgb_l19_smooth): formula tables at 1/500 of the rough fixtures' amplitude
FULL_SMOOTH_SCALE = 0.1


def fullsize_state(mods, log2T: int, seed: int = FULL_SEED, table_scale: float = FULL_TABLE_SCALE, bg_kind="nerf"):
    import torch

    from multimodalstudio_amd import scene as ms
    from multimodalstudio_amd.model import BaseModel, ModelSpec
    from oracle.hashgrid import deterministic_table
    rng = torch.random.get_rng_state()
    try:
        torch.manual_seed(seed)
        m = BaseModel(ModelSpec({k: ms.CHANNELS[k] for k in mods}, log2T=log2T, bg_kind=bg_kind))
    finally:
        torch.random.set_rng_state(rng)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    for k in sd:
        if k.endswith("hash_table"):
            sd[k] = deterministic_table(16, log2T) * table_scale
    # the geometric init zeroes the SDF MLP's layer-0 columns past x (mlp.py:188-191), so at init the SDF hash table
    # gets an all-zero gradient and its backward would go unpinned: give the grid-feature columns (39..70) a
    # deterministic weight of the x columns' scale
    k = "surface_model.surface_field.field.mlp_head.layers.0.parametrizations.weight.original1"
    v = sd[k]
    i = torch.arange(v.shape[0], dtype=torch.float64)[:, None]
    j = torch.arange(39, v.shape[1], dtype=torch.float64)[None, :]
    v[:, 39:] = (0.05 * torch.sin(0.7 * i + 1.1 * j + 0.3)).float()
    return sd


def param_checksum(sd) -> float:
    """float64 sum of |p| over the non-table parameters."""
    return float(sum(float(v.double().abs().sum()) for k, v in sd.items() if not k.endswith("hash_table")))


def with_fullsize_params(f: dict) -> dict:
    """Fixture dict ``f`` with its regenerated parameters as 'p:' keys (checksum-checked); unchanged otherwise."""
    if "param_checksum" not in f:
        return f
    mods = [str(m) for m in f["mods"]]
    sd = fullsize_state(mods, int(f["log2T"]), table_scale=float(f.get("state:table_scale", FULL_TABLE_SCALE)),
                        bg_kind=str(f.get("state:bg_kind", "nerf")))
    ck = param_checksum(sd)
    want = float(f["param_checksum"])
    if abs(ck - want) > 1e-9 * abs(want):
        raise RuntimeError(f"regenerated full-size parameters differ from the fixture's (checksum {ck!r} vs {want!r})")
    f = dict(f)
    f.update({"p:" + k: v.numpy() for k, v in sd.items()})
    return f


def sorted_index_equal_up_to_ties(got, ref, final_bins=None) -> bool:
    """An up-sampler iteration's sorted_index against the reference's, up to the order of TIED keys: torch.sort is not
    stable, so where a new sample lands exactly on an existing bin the reference's own CPU runs order the two indices
    either way (measured on the full-size fixtures: a few swapped pairs per modality, at bins equal to the last bit).
    Every maximal run of differing columns in a row must hold the same indices in both; with ``final_bins`` (the last
    iteration's sorted bins) the run's bins must also be equal."""
    import numpy as np
    got, ref = np.asarray(got, np.int64), np.asarray(ref, np.int64)
    if got.shape != ref.shape:
        return False
    for r in np.nonzero((got != ref).any(1))[0]:
        cols = np.nonzero(got[r] != ref[r])[0]
        runs = np.split(cols, np.nonzero(np.diff(cols) > 1)[0] + 1)
        for run in runs:
            if sorted(got[r, run]) != sorted(ref[r, run]):
                return False
            if final_bins is not None and not np.all(final_bins[r, run] == final_bins[r, run[0]]):
                return False
    return True
