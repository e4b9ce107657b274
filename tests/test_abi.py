"""CPU tests of the C-ABI boundary: the library loads, exports every symbol that
include/ompl_gpu.h declares, and rejects bad arguments without a device."""
import ctypes as C
import math
import os
import re

import pytest

from ompl_amd import abi
from ompl_amd.spaces import KinematicChainSpace, RealVectorStateSpace, SE3StateSpace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ompl_gpu_[a-z0-9_]+)\s*\(", src)))


def test_every_declared_symbol_is_exported():
    names = _declared("ompl_gpu.h")
    assert len(names) >= 25
    lib = C.CDLL(abi.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(abi.SIGNATURES), set(names) ^ set(abi.SIGNATURES)


def test_abi_version():
    assert abi.lib.ompl_gpu_abi_version() == 1


def test_struct_layout_matches_header():
    # ompl_gpu_space: 2*int32 + 2*double + 2*double + 2*uint32 + double = 56 bytes
    assert C.sizeof(abi.SpaceStruct) == 56
    assert C.sizeof(abi.CheckerStruct) == 32


def test_null_arguments_are_rejected():
    assert abi.lib.ompl_gpu_nn_create(None, None, 0) == abi.ERR_INVALID_ARG
    h = C.c_void_p()
    sp = SE3StateSpace().to_abi()
    st = abi.lib.ompl_gpu_nn_create(C.byref(h), C.byref(sp), 0)
    if abi.device_count() == 0:
        assert st == abi.ERR_DEVICE
        assert b"device" in abi.lib.ompl_gpu_last_error()
    bad = RealVectorStateSpace(40).to_abi()  # above the compiled feature buckets
    assert abi.lib.ompl_gpu_nn_create(C.byref(h), C.byref(bad), 0) == abi.ERR_UNSUPPORTED
    assert abi.lib.ompl_gpu_nn_knn(None, None, 0, 1, None, None, None) == abi.ERR_INVALID_ARG
    assert abi.lib.ompl_gpu_mv_check(None, None, None, 0, None, None, None) == abi.ERR_INVALID_ARG


def test_space_resolution_matches_reference_setup():
    """longestValidSegment_ = extent * fraction (StateSpace.cpp:237-249)."""
    se3 = SE3StateSpace().to_abi()
    assert se3.lvs[0] == math.sqrt(3.0) * 0.01 and se3.lvs[1] == (0.5 * math.pi) * 0.01
    assert se3.weight[0] == 1.0 and se3.weight[1] == 1.0 and se3.dim == 7
    ch = KinematicChainSpace(12, 1 / 12).to_abi()
    e = 0.0
    for _ in range(12):
        e += (2 * math.pi) * (2 * math.pi)
    assert ch.lvs[0] == math.sqrt(e) * 0.01 and ch.link_length == 1 / 12
    r6 = RealVectorStateSpace(6)
    r6.setLongestValidSegmentFraction(0.001)
    assert r6.to_abi().lvs[0] == math.sqrt(6.0) * 0.001
    with pytest.raises(ValueError):
        r6.setLongestValidSegmentFraction(0.0)
