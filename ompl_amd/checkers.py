"""Device validity checkers (the closed set the GPU can evaluate).

Arbitrary user ``StateValidityChecker::isValid`` code stays on the CPU; these
are the predicates of the reference workloads, restated on device:

  HypercubeChecker       demos/HypercubeBenchmark.cpp:57-72
  Circles2DChecker       tests/resources/circles2D.h:139-150 (Circles2D::noOverlap)
  SpheresChecker         the 3-D form of Circles2D::noOverlap on the first three reals
  KinematicChainChecker  demos/KinematicChain.h:193-277
  AllValidChecker        base/StateValidityChecker.h:165-183
"""
from __future__ import annotations

import numpy as np

from . import abi


class Checker:
    kind = abi.CHECK_ALL_VALID

    def __init__(self):
        self._data = np.zeros(0, dtype=np.float64)
        self.ndim = 0
        self.edge_width = 0.0
        self.count = 0

    def to_abi(self) -> abi.CheckerStruct:
        c = abi.CheckerStruct()
        c.kind = self.kind
        c.ndim = self.ndim
        c.edge_width = self.edge_width
        c.count = self.count
        c.reserved = 0
        c.data = self._data.ctypes.data_as(abi._D) if self._data.size else None
        return c


class AllValidChecker(Checker):
    kind = abi.CHECK_ALL_VALID


class HypercubeChecker(Checker):
    kind = abi.CHECK_HYPERCUBE

    def __init__(self, ndim: int, edge_width: float = 0.1):
        super().__init__()
        self.ndim = int(ndim)
        self.edge_width = float(edge_width)


class SpheresChecker(Checker):
    """Invalid iff (c-p).(c-p) < r^2 for some sphere (strict, as noOverlap)."""

    kind = abi.CHECK_SPHERES

    def __init__(self, centers, radii):
        super().__init__()
        c = np.asarray(centers, dtype=np.float64).reshape(-1, 3)
        r = np.broadcast_to(np.asarray(radii, dtype=np.float64), (c.shape[0],))
        self._data = np.ascontiguousarray(np.column_stack([c, r * r]))
        self.count = c.shape[0]


class Circles2DChecker(Checker):
    kind = abi.CHECK_CIRCLES2D

    def __init__(self, circles):
        """circles: rows (x, y, r); r^2 is precomputed like Circle::r2_."""
        super().__init__()
        c = np.asarray(circles, dtype=np.float64).reshape(-1, 3)
        self._data = np.ascontiguousarray(np.column_stack([c[:, 0], c[:, 1], c[:, 2] * c[:, 2]]))
        self.count = c.shape[0]


class KinematicChainChecker(Checker):
    kind = abi.CHECK_KCHAIN

    def __init__(self, env_segments):
        """env_segments: rows (x0, y0, x1, y1) (the demo's Environment)."""
        super().__init__()
        self._data = np.ascontiguousarray(np.asarray(env_segments, dtype=np.float64).reshape(-1, 4))
        self.count = self._data.shape[0]
