"""ompl_amd — MI355X (gfx950) backend for OMPL's nearest-neighbour queries and
discrete motion validation.

The product is the C ABI library ``ompl_amd/lib/libompl_gpu.so`` (include/ompl_gpu.h)
and the C++ plugin headers in ``include/ompl_amd/``; this package is the Python
mirror of the same interfaces (ctypes) used by the tests and the benchmark.
"""
from . import abi
from .checkers import (AllValidChecker, Circles2DChecker, HypercubeChecker, KinematicChainChecker,
                       SpheresChecker)
from .motion import DiscreteMotionValidatorGPU
from .nn import NearestNeighborsGPU
from .spaces import KinematicChainSpace, RealVectorStateSpace, SE3StateSpace, SO3StateSpace

__all__ = [
    "abi", "NearestNeighborsGPU", "DiscreteMotionValidatorGPU", "RealVectorStateSpace", "SO3StateSpace",
    "SE3StateSpace", "KinematicChainSpace", "AllValidChecker", "HypercubeChecker", "SpheresChecker",
    "Circles2DChecker", "KinematicChainChecker",
]
