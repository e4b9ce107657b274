// plugin_test.cpp — exercises ompl_amd::NearestNeighborsGPU<_T> through the OMPL
// NearestNeighbors<_T> interface the way the planners use it (element = pointer to a
// Motion-like struct with a `state` member, default construction, add / nearest /
// nearestK / nearestR / remove / list / clear) and checks every answer against the oracle's
// brute force (linked from oracle/liboracle.so — test infrastructure).
//
// Built by tests/test_cpp_plugin.py (standalone surface or the reference's own
// NearestNeighbors.h with -DOMPL_AMD_WITH_OMPL).  Prints "PLUGIN OK" on success.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <random>
#include <vector>

#include "ompl_amd/NearestNeighborsGPU.h"
#include "../../oracle/oracle.h"

struct State {
    double v[7];
};
struct Motion {  // like RRT::Motion (RRT.h:147-165): the NN sees only `state`
    State *state;
};

#define CHECK(c)                                                                 \
    do {                                                                         \
        if (!(c)) {                                                              \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            return 1;                                                            \
        }                                                                        \
    } while (0)

int main(int argc, char **argv) {
    const bool run = argc > 1 && std::string(argv[1]) == "run";
    ompl_gpu_space sp{};
    sp.kind = OMPL_GPU_SPACE_SE3;
    sp.dim = 7;
    sp.weight[0] = sp.weight[1] = 1.0;
    sp.lvs[0] = std::sqrt(3.0) * 0.01;
    sp.lvs[1] = (0.5 * M_PI) * 0.01;
    sp.factor[0] = sp.factor[1] = 1;
    ompl_amd::setDefaultGpuSpace(sp, 0);
    ompl_amd::setDefaultStatePacker([](const void *s, double *out) {
        const State *st = static_cast<const State *>(s);
        for (int i = 0; i < 7; ++i) out[i] = st->v[i];
    });
    if (!run) {  // compile-only mode: the interface type-checks
        std::printf("PLUGIN COMPILED\n");
        return 0;
    }
    std::mt19937_64 rng(3);
    std::uniform_real_distribution<double> u(0.0, 1.0);
    const int n = 5000, nq = 40;
    std::vector<State> states(n + nq);
    for (auto &s : states) {
        for (int i = 0; i < 3; ++i) s.v[i] = u(rng);
        double x0 = u(rng), r1 = std::sqrt(1 - x0), r2 = std::sqrt(x0), t1 = 2 * M_PI * u(rng), t2 = 2 * M_PI * u(rng);
        s.v[3] = std::sin(t1) * r1; s.v[4] = std::cos(t1) * r1; s.v[5] = std::sin(t2) * r2; s.v[6] = std::cos(t2) * r2;
    }
    std::vector<Motion> motions(n + nq);
    for (int i = 0; i < n + nq; ++i) motions[i].state = &states[i];

    // what planners do: std::make_shared<NN<Motion*>>() then setDistanceFunction
    std::shared_ptr<ompl::NearestNeighbors<Motion *>> nn = std::make_shared<ompl_amd::NearestNeighborsGPU<Motion *>>();
    nn->setDistanceFunction([&](const Motion *a, const Motion *b) { return oracle_distance(&sp, a->state->v, b->state->v); });
    CHECK(nn->reportsSortedResults());
    bool threw = false;
    try {
        nn->nearest(&motions[0]);
    } catch (const ompl::Exception &e) {
        threw = std::string(e.what()) == "No elements found in nearest neighbors data structure";
    }
    CHECK(threw);
    for (int i = 0; i < 1000; ++i) nn->add(&motions[i]);  // incremental, like RRT.cpp:173
    std::vector<Motion *> bulk;
    for (int i = 1000; i < n; ++i) bulk.push_back(&motions[i]);
    nn->add(bulk);                                          // vector add, like BIT* batches
    CHECK(nn->size() == (std::size_t)n);

    std::vector<double> data(n * 7);
    for (int i = 0; i < n; ++i)
        for (int c = 0; c < 7; ++c) data[i * 7 + c] = states[i].v[c];
    const uint32_t k = 10;
    std::vector<uint32_t> ids(k);
    std::vector<double> ds(k);
    uint32_t cnt;
    std::vector<Motion *> nbh;
    for (int j = 0; j < nq; ++j) {
        Motion *q = &motions[n + j];
        oracle_knn(&sp, data.data(), n, q->state->v, 1, k, ids.data(), ds.data(), &cnt);
        CHECK(nn->nearest(q) == &motions[ids[0]]);
        nn->nearestK(q, k, nbh);
        CHECK(nbh.size() == k);
        for (uint32_t r = 0; r < k; ++r) CHECK(nbh[r] == &motions[ids[r]]);
        const double rad = ds[5];
        nn->nearestR(q, rad, nbh);
        CHECK(nbh.size() == 6);  // inclusive <= (NearestNeighborsLinear.h:139)
        for (uint32_t r = 0; r < 6; ++r) CHECK(nbh[r] == &motions[ids[r]]);
    }
    nn->nearestK(&motions[7], 0, nbh);
    CHECK(nbh.empty());
    CHECK(nn->nearest(&motions[7]) == &motions[7]);  // a stored element is its own nearest
    // remove (GNAT.h:190-207) then queries never return it
    CHECK(nn->remove(&motions[7]));
    CHECK(!nn->remove(&motions[7]));
    CHECK(nn->size() == (std::size_t)n - 1);
    CHECK(nn->nearest(&motions[7]) != &motions[7]);
    std::vector<Motion *> all;
    nn->list(all);
    CHECK(all.size() == (std::size_t)n - 1);
    nn->clear();
    CHECK(nn->size() == 0);
    std::printf("PLUGIN OK\n");
    return 0;
}
