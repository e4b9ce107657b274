"""State-space descriptors mirroring the reference's StateSpace classes.

Only what the device path needs: the metric kind, the state width, component
weights and the motion-validation resolution (longestValidSegment_), computed
exactly as the reference does at setup():

  longestValidSegment_ = getMaximumExtent() * longestValidSegmentFraction_
                                                     (StateSpace.cpp:237-249)
  RealVector extent = sqrt(sum (high-low)^2)         (RealVectorStateSpace.cpp:167-176)
  SO3 extent = pi/2                                  (SO3StateSpace.cpp:166-169)
  fraction default 0.01, factor default 1            (StateSpace.cpp:92-94)
  SpaceInformation::setStateValidityCheckingResolution(r) sets the fraction on
  the space and (compound) its components            (SpaceInformation.h:192-196,
                                                      StateSpace.cpp:1078-1083)
"""
from __future__ import annotations

import math

from . import abi


def _rv_extent(low, high) -> float:
    e = 0.0
    for lo, hi in zip(low, high):
        d = float(hi) - float(lo)
        e += d * d
    return math.sqrt(e)


def _rv_measure(low, high) -> float:
    # RealVectorStateSpace::getMeasure — RealVectorStateSpace.cpp:178-186
    m = 1.0
    for lo, hi in zip(low, high):
        m *= hi - lo
    return m


class StateSpace:
    kind = -1
    dim = 0

    def __init__(self):
        self.fraction = 0.01
        self.factor = 1

    # reference API names
    def setLongestValidSegmentFraction(self, f: float):
        if f < 2.220446049250313e-16 or f > 1.0 - 2.220446049250313e-16:
            raise ValueError("The fraction of the extent must be larger than 0 and less than 1")
        self.fraction = float(f)

    def setValidSegmentCountFactor(self, factor: int):
        if factor < 1:
            raise ValueError("The multiplicative factor for the valid segment count between two states must be "
                             "strictly positive")
        self.factor = int(factor)

    def getMeasure(self) -> float:
        raise NotImplementedError(type(self).__name__)

    def getMaximumExtent(self) -> float:
        raise NotImplementedError

    def getDimension(self) -> int:
        """Manifold dimension (StateSpace::getDimension); `dim` is the stored doubles per state."""
        return self.dim

    def lvs(self):
        return (self.getMaximumExtent() * self.fraction, 0.0)

    def to_abi(self) -> abi.SpaceStruct:
        s = abi.SpaceStruct()
        s.kind = self.kind
        s.dim = self.dim
        s.weight[0], s.weight[1] = 1.0, 1.0
        l0, l1 = self.lvs()
        s.lvs[0], s.lvs[1] = l0, l1
        s.factor[0], s.factor[1] = self.factor, self.factor
        s.link_length = 0.0
        return s


class RealVectorStateSpace(StateSpace):
    kind = abi.SPACE_REALVECTOR

    def __init__(self, dim: int, low=0.0, high=1.0):
        super().__init__()
        self.dim = int(dim)
        self.low = [float(low)] * self.dim if not hasattr(low, "__len__") else [float(v) for v in low]
        self.high = [float(high)] * self.dim if not hasattr(high, "__len__") else [float(v) for v in high]

    def getMaximumExtent(self):
        return _rv_extent(self.low, self.high)

    def getMeasure(self):
        return _rv_measure(self.low, self.high)


class SO3StateSpace(StateSpace):
    kind = abi.SPACE_SO3
    dim = 4

    def getDimension(self):
        return 3  # SO3StateSpace.cpp:246

    def getMaximumExtent(self):
        return 0.5 * math.pi

    def getMeasure(self):
        return math.pi * math.pi  # SO3StateSpace.cpp:171-175


class SE3StateSpace(StateSpace):
    """SE3 = R^3 (weight 1) + SO3 (weight 1) (SE3StateSpace.h:114-121).  The
    resolution fraction is applied to both components; validSegmentCount is the
    max of the component counts (StateSpace.cpp:1085-1097)."""

    kind = abi.SPACE_SE3
    dim = 7

    def getDimension(self):
        return 6  # R^3 + SO(3), CompoundStateSpace::getDimension

    def __init__(self, low=0.0, high=1.0):
        super().__init__()
        self.low = [float(low)] * 3 if not hasattr(low, "__len__") else [float(v) for v in low]
        self.high = [float(high)] * 3 if not hasattr(high, "__len__") else [float(v) for v in high]
        self.weights = (1.0, 1.0)

    def getMaximumExtent(self):
        # CompoundStateSpace::getMaximumExtent — StateSpace.cpp:996-1003
        return self.weights[0] * _rv_extent(self.low, self.high) + self.weights[1] * (0.5 * math.pi)

    def getMeasure(self):
        # CompoundStateSpace::getMeasure (StateSpace.cpp:1005-1012): product of weighted components
        return (self.weights[0] * _rv_measure(self.low, self.high)) * (self.weights[1] * (math.pi * math.pi))

    def lvs(self):
        return (_rv_extent(self.low, self.high) * self.fraction, (0.5 * math.pi) * self.fraction)

    def to_abi(self):
        s = super().to_abi()
        s.weight[0], s.weight[1] = self.weights
        return s


class KinematicChainSpace(StateSpace):
    """demos/KinematicChain.h:87-175: RealVectorStateSpace(n) in [-pi, pi]^n with the
    chain metric; extent stays the RealVector extent (not overridden)."""

    kind = abi.SPACE_KCHAIN

    def __init__(self, num_links: int, link_length: float):
        super().__init__()
        self.dim = int(num_links)
        self.link_length = float(link_length)
        self.low = [-math.pi] * self.dim
        self.high = [math.pi] * self.dim

    def getMaximumExtent(self):
        return _rv_extent(self.low, self.high)

    def to_abi(self):
        s = super().to_abi()
        s.link_length = self.link_length
        return s
