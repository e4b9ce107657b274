// mv_plugin_test.cpp — ompl_amd::MotionValidatorGPU through the ompl::base::MotionValidator
// interface (both checkMotion overloads, the batched extension and the counters,
// MotionValidator.h:79-139), checked edge by edge against the oracle's restatement of
// DiscreteMotionValidator (oracle/liboracle.so — test infrastructure).
// Built by tests/test_cpp_plugin.py.  Prints "MV PLUGIN OK" on success.
#include <cmath>
#include <cstdio>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "ompl_amd/MotionValidatorGPU.h"
#include "../../oracle/oracle.h"

struct SE3State : ompl::base::State {
    double v[7];
};

#define CHECK(c)                                                                      \
    do {                                                                              \
        if (!(c)) {                                                                   \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            return 1;                                                                 \
        }                                                                             \
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
    std::mt19937_64 rng(11);
    std::uniform_real_distribution<double> u(0.0, 1.0);
    std::vector<double> spheres;  // 32 spheres of radius 0.1: (cx, cy, cz, r^2)
    for (int i = 0; i < 32; ++i) {
        for (int c = 0; c < 3; ++c) spheres.push_back(u(rng));
        spheres.push_back(0.01);
    }
    ompl_gpu_checker ck{};
    ck.kind = OMPL_GPU_CHECK_SPHERES;
    ck.count = 32;
    ck.data = spheres.data();
    auto pack = [](const ompl::base::State *s, double *out) {
        const auto *st = static_cast<const SE3State *>(s);
        for (int i = 0; i < 7; ++i) out[i] = st->v[i];
    };
    auto interp = [&sp](const ompl::base::State *a, const ompl::base::State *b, double t, ompl::base::State *o) {
        oracle_interpolate(&sp, static_cast<const SE3State *>(a)->v, static_cast<const SE3State *>(b)->v, t,
                           static_cast<SE3State *>(o)->v);
    };
    if (!run) {  // compile-only mode: the interface type-checks
        std::printf("MV PLUGIN COMPILED\n");
        return 0;
    }
    // what SpaceInformation::setMotionValidator stores (SpaceInformation.h:168-172)
    std::shared_ptr<ompl::base::MotionValidator> mv =
        std::make_shared<ompl_amd::MotionValidatorGPU>(nullptr, sp, ck, 0, pack, interp);
    const int m = 1500;
    std::vector<SE3State> a(m), b(m);
    for (int i = 0; i < m; ++i) {
        for (SE3State *s : {&a[i], &b[i]}) {
            for (int c = 0; c < 3; ++c) s->v[c] = u(rng);
            const double x0 = u(rng), r1 = std::sqrt(1 - x0), r2 = std::sqrt(x0), t1 = 2 * M_PI * u(rng),
                         t2 = 2 * M_PI * u(rng);
            s->v[3] = std::sin(t1) * r1;
            s->v[4] = std::cos(t1) * r1;
            s->v[5] = std::sin(t2) * r2;
            s->v[6] = std::cos(t2) * r2;
        }
    }
    unsigned nvalid = 0, nlast = 0;
    for (int i = 0; i < m; ++i) {
        uint8_t ov = 0;
        int32_t nd = 0, fi = 0;
        oracle_check_motions(&sp, &ck, a[i].v, b[i].v, 1, &ov, &nd, &fi);
        const bool v = mv->checkMotion(&a[i], &b[i]);
        CHECK(v == (ov != 0));
        nvalid += v;
        SE3State lv;
        std::pair<ompl::base::State *, double> last(&lv, -7.0);
        const bool v2 = mv->checkMotion(&a[i], &b[i], last);
        CHECK(v2 == v);
        if (v2) {
            CHECK(last.second == -7.0);  // untouched on success
        } else if (nd > 0) {
            ++nlast;
            CHECK(last.second == (double)(fi - 1) / (double)nd);
            SE3State e;
            oracle_interpolate(&sp, a[i].v, b[i].v, last.second, e.v);
            for (int c = 0; c < 7; ++c) CHECK(lv.v[c] == e.v[c]);
        }
    }
    CHECK(nvalid > 0 && nvalid < (unsigned)m && nlast > 0);
    CHECK(mv->getValidMotionCount() == 2 * nvalid);
    CHECK(mv->getCheckedMotionCount() == 2u * m);
    std::vector<std::pair<const ompl::base::State *, const ompl::base::State *>> edges;
    for (int i = 0; i < m; ++i) edges.emplace_back(&a[i], &b[i]);
    std::vector<uint8_t> valid;
    static_cast<ompl_amd::MotionValidatorGPU *>(mv.get())->checkMotions(edges, valid);
    unsigned nv2 = 0;
    for (int i = 0; i < m; ++i) nv2 += valid[i];
    CHECK(nv2 == nvalid);
    CHECK(mv->getValidMotionCount() == 3 * nvalid);
    mv->resetMotionCounter();
    CHECK(mv->getValidMotionCount() == 0 && mv->getInvalidMotionCount() == 0);
    std::printf("MV PLUGIN OK\n");
    return 0;
}
