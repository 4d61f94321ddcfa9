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
* `reference_style_library(n, seed, shape)` -- graphics.py's own generator
  (graphics.py:110-208) restated in voxel space (no trimesh): position and
  radius draws, the 20-point inside-the-lungs acceptance, sphere voxelization
  at pitch 0.05 mesh units, reference filename format.
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


# graphics.py:190-208 voxelizes the lung mesh at pitch 0.05; the mesh->voxel
# origin of the reference grid, fitted from the 1000 reference tumours
# (filename position vs voxel centroid, per-axis std 0.02 mesh units)
REF_PITCH = 0.05
REF_ORIGIN = (-17.5098, -1.3827, -1.8291)
# sphere voxelization slack (voxels): trimesh's subdivide + fill of an
# icosphere(subdivisions=2) marks every voxel its surface touches; d <= r/p +
# 0.65 matches the reference voxel counts (median ratio 1.0) with a mean Jaccard
# of ~0.64 per tumour -- the residual is the reference's astype(int) truncation
# of the tumour bounds (alignment noise 0.4-0.5 voxel, uncorrelated with the
# sub-voxel position), which no voxel-space restatement can reproduce
REF_VOXEL_SLACK = 0.65


def _sphere_voxels(center_mesh, radius, shape, origin, pitch):
    """Sorted flat indices of the voxels whose centres lie within
    radius/pitch + REF_VOXEL_SLACK of the sphere centre (per-axis pitch)."""
    pitch = np.broadcast_to(np.asarray(pitch, np.float64), (3,))
    c = (np.asarray(center_mesh, np.float64) - np.asarray(origin)) / pitch
    R = radius / pitch + REF_VOXEL_SLACK
    lo = np.maximum(np.floor(c - R).astype(int), 0)
    hi = np.minimum(np.ceil(c + R).astype(int) + 1, np.asarray(shape))
    if np.any(hi <= lo):
        return np.zeros(0, np.int32)
    zz, yy, xx = np.meshgrid(*[np.arange(a, b) for a, b in zip(lo, hi)], indexing="ij")
    inside = ((zz - c[0]) / R[0]) ** 2 + ((yy - c[1]) / R[1]) ** 2 + ((xx - c[2]) / R[2]) ** 2 <= 1.0
    return np.sort(np.ravel_multi_index((zz[inside], yy[inside], xx[inside]), shape)).astype(np.int32)


def reference_style_library(n_tumours: int = 1000, seed: int = 0, shape=None, data_dir: str = DATA_DIR,
                            mean_radius: float = 0.1, std_radius: float = 0.05, resolution: int = 20,
                            min_size: float = 0.05) -> TumourLibrary:
    """graphics.py:133-208 (generate_tumour / get_random_sphere_bounded /
    is_inside / pregenerate_voxel_data) in voxel space:

    * position = round(U(lung bounds), 2) mesh units, radius =
      round(|N(0.1, 0.05)|, 2), redrawn while radius < 0.05 (graphics.py:158-163);
    * accepted when `resolution` random points of the sphere surface lie in
      the lungs (graphics.py:110-122) -- here: in a lung voxel of the mask;
    * voxelized at pitch 0.05 (graphics.py:166-188), see REF_VOXEL_SLACK;
    * named f"{x}_{y}_{z}_{r}.npy" (graphics.py:204).

    `shape` other than the reference 67x43x70 resamples the lungs and scales
    the pitch per axis.  Deterministic in `seed` (numpy Generator, not the
    reference's global np.random stream)."""
    ref = np.load(os.path.join(data_dir, "lungs.npy"))
    shape = tuple(ref.shape) if shape is None else tuple(int(x) for x in shape)
    lungs = (ref if shape == tuple(ref.shape) else resample_nearest(ref, shape)).astype(np.uint8)
    pitch = REF_PITCH * np.asarray(ref.shape, np.float64) / np.asarray(shape, np.float64)
    origin = np.asarray(REF_ORIGIN)
    lo_b = origin
    hi_b = origin + pitch * (np.asarray(shape) - 1)
    rng = np.random.default_rng(seed)
    names, parts, offsets = [], [], [0]
    while len(names) < n_tumours:
        position = np.round(rng.uniform(lo_b, hi_b), 2)
        radius = float(np.round(abs(rng.normal(mean_radius, std_radius)), 2))
        if radius < min_size:
            continue
        d = rng.normal(size=(resolution, 3))
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        pts = np.rint((position + d * radius - origin) / pitch).astype(np.int64)
        ok = np.all((pts >= 0) & (pts < np.asarray(shape)), axis=1)
        if not ok.all() or not lungs[pts[:, 0], pts[:, 1], pts[:, 2]].all():
            continue
        flat = _sphere_voxels(position, radius, shape, origin, pitch)
        if flat.size == 0:
            continue
        parts.append(flat)
        offsets.append(offsets[-1] + flat.size)
        names.append(f"{position[0]}_{position[1]}_{position[2]}_{radius}.npy")
    return TumourLibrary(shape=shape, lungs=lungs, names=names, voxels=np.concatenate(parts),
                         offsets=np.asarray(offsets, np.int64))


def resampled_reference_library(shape=(64, 64, 64), data_dir: str = DATA_DIR) -> TumourLibrary:
    """The reference's own lungs and 1000 tumours on another grid: every
    volume nearest-resampled with the lung mask's cell-centre mapping
    (`resample_nearest`), so an agent trained on the reference grid
    (saves/*.model, whose observations are grid-normalised, environment.py:
    259-268) sees the same normalised geometry.  Tumours that vanish under
    the resampling keep their nearest voxel."""
    ref = reference_library(data_dir)
    lungs = resample_nearest(ref.lungs, shape).astype(np.uint8)
    idx = [np.minimum(((np.arange(n) + 0.5) * s / n).astype(np.int64), s - 1) for n, s in zip(shape, ref.shape)]
    parts, offsets = [], [0]
    for k in range(ref.n_tumours):
        src = ref.tumour_dense(k) > 0
        vol = src[np.ix_(*idx)]
        flat = np.flatnonzero(vol.ravel())
        if flat.size == 0:  # thinner than a target cell: the cell nearest its centroid
            c = ref.centroid(k)
            cell = [int(np.argmin(np.abs((np.arange(n) + 0.5) * s / n - (ci + 0.5))))
                    for n, s, ci in zip(shape, ref.shape, c)]
            flat = np.array([np.ravel_multi_index(tuple(cell), shape)])
        flat = np.sort(flat).astype(np.int32)
        parts.append(flat)
        offsets.append(offsets[-1] + flat.size)
    return TumourLibrary(shape=tuple(shape), lungs=lungs, names=list(ref.names),
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
