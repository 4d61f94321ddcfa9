"""Minimal `gymnasium.spaces.Box` stand-in (gymnasium is not a dependency of
the hot path; if it is importable its Box is used instead)."""
from __future__ import annotations

import numpy as np

try:  # pragma: no cover - gymnasium is absent in this image
    from gymnasium.spaces import Box  # type: ignore
except Exception:  # noqa: BLE001

    class Box:
        """Box(low, high, shape, dtype) with the attributes train.py reads
        (environment.py:59-65, train.py:96-100)."""

        def __init__(self, low, high, shape, dtype=np.float32, seed=None):
            self.shape = tuple(int(s) for s in shape)
            self.dtype = np.dtype(dtype)
            self.low = np.full(self.shape, low, dtype=self.dtype)
            self.high = np.full(self.shape, high, dtype=self.dtype)
            self._rng = np.random.default_rng(seed)

        def sample(self):
            return self._rng.uniform(self.low, self.high).astype(self.dtype)

        def contains(self, x) -> bool:
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

        def seed(self, seed=None):
            self._rng = np.random.default_rng(seed)

        def __repr__(self):
            return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"
