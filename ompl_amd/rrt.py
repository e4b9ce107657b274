"""ompl::geometric::RRT with its loop on the device (geometric/planners/rrt/src/RRT.cpp).

The planner's per-iteration work — nearest (RRT.cpp:137), steer to the range (:141-146),
checkMotion (:148), add (:170-173), the goal test (:175-187) — runs in one device call per batch
of iterations (ompl_gpu_rrt_solve_device); this class supplies what the reference computes
around it, in the reference's order, from the reference's random streams:

  RRT(si)                 rng_ takes the next seed (RRT.h:192)
  setup()                 range = 0.2 x maximum extent (SelfConfig::configurePlannerRange,
                          SelfConfig.cpp:98) when unset; the nearest-neighbour structure takes
                          one seed (GNAT's pivot selector, GreedyKCenters.h:127)
  solve()                 the start states join the tree (:104-109); the state sampler is
                          allocated on the first call (:117, 3 seeds for SE3); iteration i draws
                          rng_.uniform01() and samples the goal when it is below the goal bias
                          (GoalState::sampleGoal), else sampler_->sampleUniform (:130-134)

so a program that mirrors the reference's construction order after RNG::setSeed(s) sees the
same samples, the same tree and the same solution.
"""
from __future__ import annotations

import numpy as np

from . import sampling as S
from .motion import DiscreteMotionValidatorGPU
from .nn import NearestNeighborsGPU

DBL_EPSILON = 2.220446049250313e-16


class RRT:
    def __init__(self, space, checker, device: int = 0):
        self.space, self.checker, self.device = space, checker, device
        self.rng_seed = S.next_seed()            # RRT::rng_
        self.goal_bias = 0.05                    # RRT.h:183
        self.max_distance = 0.0
        self.nn = None
        self.mv = None
        self.sampler = None
        self._u = np.empty(0)                    # rng_.uniform01() stream, drawn ahead
        self._used = 0
        self._pending = None                     # samples drawn but not run (after a solution)
        self.parent: dict[int, int] = {}

    # reference parameter names
    def setGoalBias(self, b: float):
        self.goal_bias = float(b)

    def setRange(self, d: float):
        self.max_distance = float(d)

    def getRange(self) -> float:
        return self.max_distance

    def setup(self):
        if self.max_distance < 1e-12:
            self.max_distance = 0.2 * self.space.getMaximumExtent()
        if self.nn is None:
            S.next_seed()                        # the structure's own RNG (one per instance)
            self.nn = NearestNeighborsGPU(self.space, self.device)
            self.mv = DiscreteMotionValidatorGPU(self.space, self.checker, self.device)

    def _uniform01(self, n: int) -> np.ndarray:
        need = self._used + n
        if need > len(self._u):                  # regrow the prefix of the same stream
            self._u = S.rng_uniform(self.rng_seed, max(need, 2 * len(self._u)))
        out = self._u[self._used:need]
        self._used = need
        return out

    def next_samples(self, n: int, goal) -> np.ndarray:
        """The samples of the next n iterations (RRT.cpp:130-134)."""
        if self._pending is not None and len(self._pending):
            take = self._pending[:n]
            self._pending = self._pending[n:]
            if len(take) == n:
                return take
            return np.concatenate([take, self.next_samples(n - len(take), goal)])
        if self.sampler is None:
            self.sampler = S.StateSampler(self.space)
        u = self._uniform01(n)
        out = np.empty((n, self.space.dim))
        biased = u < self.goal_bias
        out[biased] = goal
        k = int((~biased).sum())
        if k:
            out[~biased] = self.sampler.sample_uniform(k)
        return out

    def solve(self, start, goal, max_iterations: int, threshold: float = DBL_EPSILON, batch: int = 256):
        """Returns (solved, iterations run, path as a list of state ids from start to the solution
        or the approximate solution)."""
        import torch

        self.setup()
        if self.nn.size() == 0:
            self.start_id = int(self.nn.add(np.asarray(start, dtype=np.float64)[None])[0])
        dev = torch.device("cuda", self.device)
        near = torch.empty(batch, dtype=torch.int32, device=dev)
        added = torch.empty(batch, dtype=torch.int32, device=dev)
        best_d, best_id, it = np.inf, None, 0
        solved_id = None
        while it < max_iterations:
            n = min(batch, max_iterations - it)
            smp = torch.from_numpy(self.next_samples(n, goal)).to(dev)
            sol, aid, ad = self.nn.rrt_solve_device(self.mv, smp.data_ptr(), n, self.max_distance, goal, threshold,
                                                   near.data_ptr(), added.data_ptr())
            na = near[:n].cpu().numpy().view(np.uint32)
            aa = added[:n].cpu().numpy().view(np.uint32)
            last = n if sol is None else sol + 1
            for j in range(last):
                if aa[j] != 0xFFFFFFFF:
                    self.parent[int(aa[j])] = int(na[j])
            if aid is not None and ad < best_d:
                best_d, best_id = ad, aid
            it += last
            if sol is not None:
                solved_id = int(aa[sol])
                # the reference stops drawing at the solution: the samples drawn past it are
                # kept, in order, for a later solve() on the same planner
                rest = smp[last:n].cpu().numpy()
                self._pending = rest if self._pending is None or not len(self._pending) else \
                    np.concatenate([rest, self._pending])
                break
        end = solved_id if solved_id is not None else best_id
        path = []
        while end is not None:
            path.append(end)
            end = self.parent.get(end)
        return solved_id is not None, it, path[::-1]
