"""
Trajectory output of the engine (reference: espresso.py:1054-1159).

The reference writes chunked, resizable, gzip HDF5 datasets
``Times (T,1,1)``, ``Ids/Types (T,N,1)``, ``Unwrapped_Positions /
Velocities / Directors (T,N,3)`` under group ``h5_group_tag``.  When h5py is
importable the same layout is written; otherwise (this image has no h5py)
each chunk is written as ``<file>.chunkNNNNNN.npz`` with the same keys and
shapes, and ``read_trajectory`` concatenates them.
"""

from __future__ import annotations

import pathlib

import numpy as np

_KEYS = ["Times", "Ids", "Types", "Unwrapped_Positions", "Velocities", "Directors"]


class _H5Writer:
    def __init__(self, path: pathlib.Path, group: str, n_colloids: int, chunk: int):
        import h5py

        self._h5py = h5py
        self.path = path
        self.group = group
        with h5py.File(path.as_posix(), "a") as f:
            g = f.require_group(group)
            kw = dict(compression="gzip")
            g.require_dataset("Times", shape=(chunk, 1, 1), maxshape=(None, 1, 1), dtype=float, **kw)
            for name in ["Ids", "Types"]:
                g.require_dataset(
                    name, shape=(chunk, n_colloids, 1), maxshape=(None, n_colloids, 1),
                    dtype=int, **kw,
                )
            for name in ["Unwrapped_Positions", "Velocities", "Directors"]:
                g.require_dataset(
                    name, shape=(chunk, n_colloids, 3), maxshape=(None, n_colloids, 3),
                    dtype=float, **kw,
                )

    def write(self, values: dict, offset: int):
        n_new = len(values["Times"])
        with self._h5py.File(self.path.as_posix(), "a") as f:
            g = f[self.group]
            for key in _KEYS:
                ds = g[key]
                ds.resize(offset + n_new, axis=0)
                ds[offset : offset + n_new, ...] = values[key]


class _NpzWriter:
    def __init__(self, path: pathlib.Path, group: str, n_colloids: int, chunk: int):
        self.path = path
        self.group = group
        self._count = 0

    def write(self, values: dict, offset: int):
        out = self.path.with_name(f"{self.path.name}.chunk{self._count:06d}.npz")
        np.savez(out, group=np.array(self.group), offset=np.array(offset), **values)
        self._count += 1


def make_writer(path, group: str, n_colloids: int, chunk: int):
    path = pathlib.Path(path)
    try:
        import h5py  # noqa: F401

        return _H5Writer(path, group, n_colloids, chunk)
    except ImportError:
        return _NpzWriter(path, group, n_colloids, chunk)


def read_trajectory(path) -> dict:
    """Read back what make_writer wrote (either format)."""
    path = pathlib.Path(path)
    try:
        import h5py

        if path.exists():
            with h5py.File(path.as_posix(), "r") as f:
                g = f[list(f.keys())[0]]
                return {k: np.asarray(g[k]) for k in _KEYS}
    except ImportError:
        pass
    chunks = sorted(path.parent.glob(path.name + ".chunk*.npz"))
    parts = {k: [] for k in _KEYS}
    for c in chunks:
        with np.load(c, allow_pickle=False) as z:
            for k in _KEYS:
                parts[k].append(z[k])
    return {k: (np.concatenate(v, axis=0) if v else np.zeros((0,))) for k, v in parts.items()}
