"""BIT*'s batch sample pipeline on the device: updateSamples draws states from
the base sampler on the reference RNG streams, checks each with the StateValidityChecker, keeps
the valid ones until the batch is full or the tries run out (ImplicitGraph.cpp:924-1000), appends
them to the sample store (addToSamples, :682-692), and nearestSamples answers nearestR(v, r_) /
nearestK(v, k_) for vertices (:303-321).  The device pipeline checks validity in batches; it must
keep exactly the states, the try count and the stream position of the sequential loop, which
the oracle replays with its own restatement of the RNG streams (oracle/rng.cpp)."""
import math

import numpy as np
import pytest

import pyoracle as O
from ompl_amd import sampling
from ompl_amd import workloads as W
from ompl_amd.bitstar import ImplicitGraphSamples
from ompl_amd.checkers import SpheresChecker
from ompl_amd.spaces import RealVectorStateSpace, SE3StateSpace

pytestmark = pytest.mark.gpu


def _sequential(sp, ck, seeds, batches, stream_len):
    """The reference loop over one long stream: per batch (new, ) -> kept states, tries."""
    stream = O.sample_uniform(sp, seeds, stream_len)
    valid = O.is_valid(sp, ck, stream).astype(bool)
    at, have, kept, tries = 0, 0, [], []
    for new in batches:
        required = have + new
        max_tries = 2 * required
        t = 0
        while t < max_tries and have < required:
            assert at < stream_len, "oracle stream too short"
            if valid[at]:
                kept.append(stream[at])
                have += 1
            at += 1
            t += 1
        tries.append(t)
    return np.array(kept).reshape(-1, sp.dim), tries, stream[at:at + 4]


@pytest.mark.parametrize("radius,batches", [(0.1, [3000, 2000]), (0.2, [3000, 2000])])
def test_update_samples_matches_sequential_loop(gpu, radius, batches):
    sp = SE3StateSpace()
    centres, radii = W.sphere_field(32, radius, 7)
    ck = SpheresChecker(centres, radii)
    sampling.set_seed(42)
    g = ImplicitGraphSamples(sp, ck, gpu)
    seeds = g.sampler.local_seeds()
    want, want_tries, next_states = _sequential(sp, ck, seeds, batches, 4 * sum(batches) + 64)
    got_tries = []
    for new in batches:
        g.add_new_samples(new)
        before = g.num_state_collision_checks
        ids = g.update_samples()
        got_tries.append(g.num_state_collision_checks - before)
        assert len(ids) == 0 or ids[0] == g.samples.total() - len(ids)
    assert got_tries == want_tries
    assert g.samples.size() == len(want)
    np.testing.assert_array_equal(g.samples.states(), want)
    # the streams stand exactly where the sequential loop left them
    np.testing.assert_array_equal(g.sampler.sample_uniform(4), next_states)


def test_update_samples_stops_at_max_tries(gpu):
    """A field that rejects most states: the loop ends on averageNumOfAllowedFailedAttempts *
    numRequiredSamples tries with fewer samples than requested."""
    sp = RealVectorStateSpace(3)
    centres, radii = W.sphere_field(32, 0.3, 7, low=0.0, high=1.0)
    ck = SpheresChecker(centres, radii)
    sampling.set_seed(7)
    g = ImplicitGraphSamples(sp, ck, gpu)
    seeds = g.sampler.local_seeds()
    want, want_tries, next_states = _sequential(sp, ck, seeds, [2000], 4064)
    g.add_new_samples(2000)
    g.update_samples()
    assert want_tries == [4000] and g.num_state_collision_checks == 4000
    assert 0 < g.num_samples < 2000 and g.num_samples == len(want)
    np.testing.assert_array_equal(g.samples.states(), want)
    np.testing.assert_array_equal(g.sampler.sample_uniform(4), next_states)


@pytest.mark.parametrize("use_k", [False, True])
def test_nearest_samples(gpu, use_k):
    sp = SE3StateSpace()
    centres, radii = W.sphere_field(32, 0.1, 7)
    ck = SpheresChecker(centres, radii)
    sampling.set_seed(3)
    g = ImplicitGraphSamples(sp, ck, gpu, use_k_nearest=use_k)
    g.add_new_samples(20000)
    if use_k:
        assert g.k == math.ceil(1.1 * (math.e + math.e / 6) * math.log(20000))
    else:  # 1.1 * r_RGG,min * (ln n / n)^(1/6), SURVEY Appendix B: r_RGG,min = 1.2828 for [0,1]^3 x SO3
        assert abs(g.calculate_minimum_rgg_r() - 1.2828) < 1e-4
    vertices = sampling.StateSampler(sp).sample_uniform(300)
    res = g.nearest_samples(vertices)  # updateSamples runs first
    data = g.samples.states()
    assert len(data) == 20000
    if use_k:
        ids, d, cnt = res
        oi, od, oc = O.knn(sp, data, vertices, g.k)
        np.testing.assert_array_equal(cnt, oc)
        np.testing.assert_array_equal(ids.astype(np.int64), oi.astype(np.int64))
        np.testing.assert_array_equal(d, od)
    else:
        off, ids, d = res
        oo, oi, od = O.radius(sp, data, vertices, g.r)
        np.testing.assert_array_equal(off, oo)
        np.testing.assert_array_equal(ids.astype(np.int64), oi.astype(np.int64))
        np.testing.assert_array_equal(d, od)
        assert int(off[-1]) > 0
