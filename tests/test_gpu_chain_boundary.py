"""KinematicChain decisions at their knife edges: states built to sit as close as fp64 allows to
(a) an integer of d / longestValidSegment (validSegmentCount = ceil(d / lvs), StateSpace.cpp:851-854,
the chain metric KinematicChain.h:105-124) and (b) the validity boundary of the self / environment
segment tests (intersectionTest's DBL_EPSILON / FLT_EPSILON thresholds, KinematicChain.h:243-275).
The device evaluates cos / sin with its own math library; the reference (and the oracle) with
glibc's.  Each edge state is found by bisection on the host with the oracle (glibc), to adjacent
doubles of the path parameter, and the device must agree on both sides of every edge."""
import math

import numpy as np
import pytest

import pyoracle as O
from ompl_amd import DiscreteMotionValidatorGPU
from ompl_amd import workloads as W
from ompl_amd.checkers import AllValidChecker, KinematicChainChecker
from ompl_amd.spaces import KinematicChainSpace

pytestmark = pytest.mark.gpu

N_EDGES = 300


def _bisect(f, lo, hi, a, b):
    """f(state(lo)) != f(state(hi)), state(t) = a + (b - a) t; shrink to adjacent t doubles"""
    flo = f(a + (b - a) * lo)
    for _ in range(200):
        mid = 0.5 * (lo + hi)
        if mid <= lo or mid >= hi:
            break
        if f(a + (b - a) * mid) == flo:
            lo = mid
        else:
            hi = mid
    return a + (b - a) * lo, a + (b - a) * hi


def test_chain_segment_count_edges(gpu):
    """validSegmentCount on both sides of nd = ceil(d / lvs) steps, device against glibc"""
    sp = KinematicChainSpace(12, 1.0 / 12)
    mv = DiscreteMotionValidatorGPU(sp, AllValidChecker(), gpu)
    rng = np.random.default_rng(17)
    base = W.uniform_chain(rng, N_EDGES, 12)
    dirs = W.uniform_chain(rng, N_EDGES, 12) * 0.2
    s1, s2 = [], []
    for a, dv in zip(base, dirs):
        b = a + dv
        na, nb = O.valid_segment_count(sp, a, a + dv * 0.3), O.valid_segment_count(sp, a, b)
        if na == nb:
            continue
        lo, hi = _bisect(lambda s: O.valid_segment_count(sp, a, s), 0.3, 1.0, a, b)
        s1 += [a, a]
        s2 += [lo, hi]
    s1, s2 = np.array(s1), np.array(s2)
    assert len(s1) > N_EDGES
    _, nd = mv.checkMotions(s1, s2, want_nd=True)
    ond = np.array([O.valid_segment_count(sp, a, b) for a, b in zip(s1, s2)])
    flips = int((nd != ond).sum())
    assert np.all(ond[1::2] == ond[0::2] + 1)  # each pair straddles an integer
    assert flips == 0, f"{flips} of {len(s1)} segment counts differ from glibc's at the ceil boundary"
    mv.close()


def test_chain_validity_edges(gpu):
    """isValid on both sides of the horn environment's / the self-intersection boundary"""
    sp = KinematicChainSpace(12, 1.0 / 12)
    ck = KinematicChainChecker(W.horn_environment(12, math.log(12.0) / 12.0))
    mv = DiscreteMotionValidatorGPU(sp, ck, gpu)
    rng = np.random.default_rng(23)
    x = W.uniform_chain(rng, 40 * N_EDGES, 12) * 0.5
    v = O.is_valid(sp, ck, x)
    good, bad = x[v], x[~v]
    assert len(good) > N_EDGES and len(bad) > N_EDGES
    edge = []
    for a, b in zip(good[:N_EDGES], bad[:N_EDGES]):
        lo, hi = _bisect(lambda s: bool(O.is_valid(sp, ck, s)[0]), 0.0, 1.0, a, b)
        edge += [lo, hi]
    edge = np.array(edge)
    ov = O.is_valid(sp, ck, edge)
    assert np.all(ov[0::2] != ov[1::2])
    gv = mv.isValid(edge)
    flips = int((gv != ov).sum())
    # and the same states as the endpoints of motions: checkMotion tests s2 (the edge state)
    gm = mv.checkMotions(edge, edge)  # nd = 0: the motion is valid iff isValid(s2)
    assert flips == 0 and np.array_equal(gm, ov), f"{flips} of {len(edge)} edge states differ from glibc's"
    mv.close()
