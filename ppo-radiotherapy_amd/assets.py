"""Voxel assets: the lung mask and the tumour library.

Reference counterpart: environment.py:28-30 (class-level LUNGS_ARRAY /
TUMOUR_DIRS loaded from ./data) and environment.py:86-97 (reset_tumour loads
one 67x43x70 f32 {0,1} volume from disk per episode).

Here a library is held once, in compact form, and copied to HBM once per
process: the lung mask (u8[V]) plus every tumour as its sorted C-order voxel
list (int32, the order np.where returns) -- a 67x43x70 tumour is 16-586
voxels, so the 1000-tumour reference library is ~0.4 MB instead of 807 MB of
dense volumes.

Two sources:
* `reference_library()`  -- data/lungs.npy + data/tumours_ref.npz (the
  reference's own assets, tumour names in the survey container's
  os.listdir order so np.random.choice indices carry over).
* `synthetic_library(shape, ...)` -- BASELINE configs at 64^3 / 128^3: lungs
  nearest-resampled from the reference mask, spherical tumours inside the lung
  mask with radii drawn so voxel counts span the reference's 16-586 range.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA_DIR = os.path.join(_REPO, "data")


@dataclass
class TumourLibrary:
    shape: tuple            # (D, H, W)
    lungs: np.ndarray       # u8 [D,H,W] in {0,1}
    names: list             # per-tumour names "x_y_z_radius"
    voxels: np.ndarray      # int32 concat of sorted flat indices
    offsets: np.ndarray     # int64 [K+1]
    _cache: dict = field(default_factory=dict, repr=False)

    @property
    def n_tumours(self) -> int:
        return len(self.offsets) - 1

    @property
    def V(self) -> int:
        return int(np.prod(self.shape))

    def tumour_voxels(self, k: int) -> np.ndarray:
        return self.voxels[self.offsets[k]:self.offsets[k + 1]]

    def tumour_dense(self, k: int) -> np.ndarray:
        vol = np.zeros(self.V, np.float32)
        vol[self.tumour_voxels(k)] = 1.0
        return vol.reshape(self.shape)

    def tumour_coords(self, k: int) -> np.ndarray:
        """int64 [n,3] in np.where order (environment.py:146,151)."""
        return np.stack(np.unravel_index(self.tumour_voxels(k).astype(np.int64), self.shape), axis=-1)

    def centroid(self, k: int) -> np.ndarray:
        """environment.py:145-148: mean of integer coords, f64 (exact sums)."""
        return self.tumour_coords(k).mean(axis=0)

    def max_tumour_voxels(self) -> int:
        return int(np.max(np.diff(self.offsets))) if self.n_tumours else 0

    def index_of(self, name: str) -> int:
        return self.names.index(name)


def reference_library(data_dir: str = DATA_DIR) -> TumourLibrary:
    lungs = np.load(os.path.join(data_dir, "lungs.npy"))
    z = np.load(os.path.join(data_dir, "tumours_ref.npz"))
    shape = tuple(int(x) for x in z["shape"])
    assert shape == lungs.shape
    return TumourLibrary(shape=shape, lungs=lungs.astype(np.uint8), names=[str(x) for x in z["names"]],
                         voxels=z["voxels"].astype(np.int32), offsets=z["offsets"].astype(np.int64))


def resample_nearest(mask: np.ndarray, shape) -> np.ndarray:
    """Nearest-neighbour resample with cell-centre alignment."""
    idx = [np.minimum(((np.arange(n) + 0.5) * s / n).astype(np.int64), s - 1)
           for n, s in zip(shape, mask.shape)]
    return mask[np.ix_(*idx)]


def synthetic_library(shape=(64, 64, 64), n_tumours: int = 1000, seed: int = 0,
                      data_dir: str = DATA_DIR) -> TumourLibrary:
    """Synthetic library on an arbitrary grid (BASELINE configs 64^3/128^3).

    Radii scale with the grid so a tumour covers a similar fraction of the lung
    as in the reference (16-586 voxels at 67x43x70).  Deterministic in `seed`.
    """
    ref = np.load(os.path.join(data_dir, "lungs.npy"))
    lungs = resample_nearest(ref, shape).astype(np.uint8)
    rng = np.random.default_rng(seed)
    scale = (np.prod(shape) / np.prod(ref.shape)) ** (1.0 / 3.0)
    lung_idx = np.flatnonzero(lungs.ravel())
    D, H, W = shape
    zz, yy, xx = np.meshgrid(np.arange(D), np.arange(H), np.arange(W), indexing="ij")
    names, parts, offsets = [], [], [0]
    while len(names) < n_tumours:
        c = np.array(np.unravel_index(lung_idx[rng.integers(lung_idx.size)], shape), np.float64)
        c = c + rng.uniform(-0.5, 0.5, 3)
        r = rng.uniform(1.6, 5.2) * scale
        lo = np.maximum(np.floor(c - r).astype(int), 0)
        hi = np.minimum(np.ceil(c + r).astype(int) + 1, shape)
        sl = tuple(slice(a, b) for a, b in zip(lo, hi))
        d2 = (zz[sl] - c[0]) ** 2 + (yy[sl] - c[1]) ** 2 + (xx[sl] - c[2]) ** 2
        inside = d2 <= r * r
        if inside.sum() < 8:
            continue
        flat = np.ravel_multi_index(tuple(g[sl][inside] for g in (zz, yy, xx)), shape)
        flat = np.sort(flat).astype(np.int32)
        parts.append(flat)
        offsets.append(offsets[-1] + flat.size)
        names.append(f"{c[0]:.2f}_{c[1]:.2f}_{c[2]:.2f}_{r:.2f}.npy")
    return TumourLibrary(shape=tuple(shape), lungs=lungs, names=names,
                         voxels=np.concatenate(parts), offsets=np.asarray(offsets, np.int64))


def library_for(grid) -> TumourLibrary:
    """The reference grid uses the reference assets; any other grid the
    synthetic generator (cached per process)."""
    grid = tuple(int(x) for x in grid)
    lib = _LIB_CACHE.get(grid)
    if lib is None:
        ref_shape = tuple(np.load(os.path.join(DATA_DIR, "lungs.npy"), mmap_mode="r").shape)
        lib = reference_library() if grid == ref_shape else synthetic_library(grid)
        _LIB_CACHE[grid] = lib
    return lib


_LIB_CACHE: dict = {}
