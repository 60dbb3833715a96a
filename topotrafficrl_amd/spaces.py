"""Minimal gymnasium-compatible space descriptors (gymnasium is optional; when it is
installed, ``to_gymnasium()`` returns the real space)."""
from __future__ import annotations

import numpy as np


class Box:
    def __init__(self, low, high, shape, dtype="float32"):
        self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), np.dtype(dtype)

    def __repr__(self):
        return f"Box({self.low}, {self.high}, {self.shape}, {self.dtype})"

    def to_gymnasium(self):
        from gymnasium import spaces
        return spaces.Box(low=self.low, high=self.high, shape=self.shape, dtype=self.dtype)


class Discrete:
    def __init__(self, n: int):
        self.n = int(n)
        self.shape = ()
        self.dtype = np.dtype(np.int64)

    def __repr__(self):
        return f"Discrete({self.n})"

    def sample(self, rng: np.random.Generator | None = None, size=None):
        rng = rng or np.random.default_rng()
        return rng.integers(0, self.n, size=size)

    def to_gymnasium(self):
        from gymnasium import spaces
        return spaces.Discrete(self.n)
