"""BASELINE configs[0]: the RigidBodyPlanning demo (demos/RigidBodyPlanning.cpp:66-129) with
og::RRT — SE(3) with R^3 bounds [-1, 1], an always-valid checker, a random start and goal —
planned with the device RRT loop (ompl_amd/rrt.py) on the reference's random streams, and
compared iteration by iteration with the oracle's sequential RRT loop (RRT.cpp:128-192) fed
the same samples.

Seed order after RNG::setSeed(s), as in the demo's plan(): start.random() and goal.random()
(a state sampler each, 3 seeds each), og::RRT (rng_, 1), planner->setup() (the NN structure's
RNG, 1), si->printSettings() (allocValidStateSampler: a UniformValidStateSampler's state
sampler, 3), solve() (sampler_, 3)."""
import numpy as np
import pytest

import pyoracle as O
from ompl_amd import sampling as S
from ompl_amd.checkers import AllValidChecker
from ompl_amd.rrt import DBL_EPSILON, RRT
from ompl_amd.spaces import SE3StateSpace

pytestmark = pytest.mark.gpu


def _demo(seed, gpu):
    S.set_seed(seed)
    sp = SE3StateSpace(-1.0, 1.0)                     # RigidBodyPlanning.cpp:69-76
    start = S.StateSampler(sp).sample_uniform(1)[0]   # start.random()   :84-85
    goal = S.StateSampler(sp).sample_uniform(1)[0]    # goal.random()    :88-89
    planner = RRT(sp, AllValidChecker(), gpu)         # og::RRT(si)      (the demo uses RRTConnect)
    planner.setup()                                   # planner->setup() :101
    S.StateSampler(sp)                                # si->printSettings(): valid state sampler :105
    return sp, start, goal, planner


def _oracle_rrt(sp, start, goal, samples, maxd):
    """RRT.cpp:128-192 with the goal test, on the oracle's metric / interpolation / validator."""
    ck = AllValidChecker()
    tree = [np.asarray(start, dtype=np.float64)]
    parent = {}
    for i, s in enumerate(samples):
        ids, d, _ = O.knn(sp, np.array(tree), s[None], 1)
        j, dj = int(ids[0, 0]), float(d[0, 0])
        to = O.interpolate(sp, tree[j], s, maxd / dj) if dj > maxd else s.copy()
        v, _, _, _ = O.check_motions(sp, ck, np.array(tree[j])[None], to[None])
        if v[0]:
            tree.append(to)
            parent[len(tree) - 1] = j
            if O.distance(sp, to, goal) < DBL_EPSILON:
                return i, np.array(tree), parent
    return None, np.array(tree), parent


@pytest.mark.parametrize("seed", [42, 7])
def test_rigid_body_planning_rrt_matches_oracle(gpu, seed):
    sp, start, goal, planner = _demo(seed, gpu)
    assert planner.getRange() == pytest.approx(0.2 * sp.getMaximumExtent())  # SelfConfig.cpp:98
    solved, iters, path = planner.solve(start, goal, 20000, batch=64)
    assert solved
    # the same samples, drawn again from a fresh run of the same construction order
    _, _, _, again = _demo(seed, gpu)
    again.sampler = S.StateSampler(sp)                # solve()'s sampler_
    samples = again.next_samples(iters, goal)
    sol_i, tree, parent = _oracle_rrt(sp, start, goal, samples, planner.getRange())
    assert sol_i == iters - 1                         # solved at the same iteration
    assert planner.nn.size() == len(tree)
    np.testing.assert_array_equal(planner.nn.states(), tree)
    assert planner.parent == parent
    assert path[0] == 0 and path[-1] == len(tree) - 1
    assert np.allclose(planner.nn.states()[path[-1]], goal, atol=0)


def test_rrt_solve_reports_approximate_solution(gpu):
    """Too few iterations to reach the goal: not solved, the closest added state is reported."""
    sp, start, goal, planner = _demo(3, gpu)
    solved, iters, path = planner.solve(start, goal, 3, batch=3)
    assert not solved and iters == 3
    st = planner.nn.states()
    if len(st) > 1:
        d = [O.distance(sp, x, goal) for x in st[1:]]
        assert path[-1] == 1 + int(np.argmin(d))
        assert path[0] == 0
