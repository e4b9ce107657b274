"""Offline estimate: how many k-d tiles must a block of B adjacent queries scan, against the
per-query tile counts of the group walk?  (SE3 10^6 states, k2 = 13, 64-state tiles.)

A tile is needed by query q iff its box lower bound is below q's final k2-th distance; the union
over a block of B consecutive queries (k-d home order) is what a lane-per-query block walk scans.
usage: python tools/sim_block_union.py [n_states] [n_queries] [n_blocks_sampled]
"""
import sys

import numpy as np

sys.path.insert(0, ".")
from ompl_amd import workloads as W  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
NQ = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
NB = int(sys.argv[3]) if len(sys.argv) > 3 else 12
K2 = 13
TILE = 64
rng = np.random.default_rng(1)
X = W.uniform_se3(rng, N)
Q = W.uniform_se3(rng, NQ)


def build(idx, out):
    """k-d median split along the widest coordinate until 64 states; appends leaves in order."""
    stack = [idx]
    while stack:
        ids = stack.pop()
        if len(ids) <= TILE:
            out.append(ids)
            continue
        P = X[ids]
        c = int(np.argmax(P.max(0) - P.min(0)))
        # left child takes a multiple of 64 states (tiles stay full)
        half = ((len(ids) + 1) // 2 + TILE - 1) // TILE * TILE
        half = min(half, len(ids) - 1)
        part = np.argpartition(P[:, c], half)
        stack.append(ids[part[half:]])
        stack.append(ids[part[:half]])


leaves = []
build(np.arange(N), leaves)
nt = len(leaves)
lo = np.stack([X[l].min(0) for l in leaves])
hi = np.stack([X[l].max(0) for l in leaves])
cen = np.stack([X[l].mean(0) for l in leaves])
print("tiles", nt)

# home tile of a query: the tile whose box contains it, else nearest box centre (approximation)
def dist(P, q):
    t = np.sqrt(((P[:, :3] - q[:3]) ** 2).sum(1))
    dq = np.abs(P[:, 3:] @ q[3:])
    return t + np.arccos(np.minimum(dq, 1.0))


def box_lb(q):
    g = np.maximum(np.maximum(lo[:, :3] - q[:3], q[:3] - hi[:, :3]), 0)
    tg = np.sqrt((g * g).sum(1))
    v = q[3:]
    gp = np.maximum(np.maximum(lo[:, 3:] - v, v - hi[:, 3:]), 0)
    gm = np.maximum(np.maximum(lo[:, 3:] + v, -v - hi[:, 3:]), 0)
    r = np.sqrt(np.minimum((gp * gp).sum(1), (gm * gm).sum(1)))
    return tg + r


home = np.array([int(np.argmin(((cen - q) ** 2).sum(1))) for q in Q[: min(NQ, 20000)]]) if NQ <= 20000 else None
if home is None:
    # cheap: home by nearest centre on translation + quaternion
    from scipy.spatial import cKDTree

    home = cKDTree(cen).query(Q)[1]
order = np.argsort(home, kind="stable")
Qs = Q[order]
for B in (2, 16, 32, 64, 128, 256):
    tot_union = tot_per = 0
    nq_done = 0
    brng = np.random.default_rng(5)
    starts = brng.choice(NQ // B, size=NB, replace=False) * B
    for s in starts:
        need = np.zeros(nt, bool)
        for q in Qs[s: s + B]:
            d = dist(X, q)
            tau = np.partition(d, K2 - 1)[K2 - 1]
            m = box_lb(q) < tau
            need |= m
            tot_per += m.sum()
        tot_union += need.sum()
        nq_done += B
    print(f"B={B:4d}: per-query needed tiles {tot_per / nq_done:7.1f}, block union {tot_union / (nq_done / B):8.1f} "
          f"tiles = {tot_union / nq_done:7.2f} tile scans per query (lane-per-query: {64 * tot_union / nq_done:8.0f} pairs/query)")
