// ref_linear.cpp — TEST INFRASTRUCTURE ONLY.
//
// Harness that compiles the reference's own brute-force nearest-neighbour
// structure, src/ompl/datastructures/NearestNeighborsLinear.h (header-only,
// standard library + ompl/util/Exception.h only), UNMODIFIED from
// /root/reference, and exposes it through a tiny C ABI for the tests and the
// golden-fixture generator.  Build: oracle/Makefile -> oracle/_ref/libref_linear.so.
//
// The element type is an integer id; the distance function is the oracle's
// restatement of the reference state-space metric (oracle.cpp).  This pins the
// selection / ordering / k>n / empty-structure semantics of our kNN and
// radius results to the reference's code (the reference test suite uses
// exactly this class as ground truth, tests/datastructures/nearestneighbors.cpp:122-184).
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "ompl/datastructures/NearestNeighborsLinear.h"
#include "oracle.h"

namespace {
struct Ctx {
    const ompl_gpu_space *sp;
    const double *data;  // n AoS states, ids 0..n-1
    const double *q;     // the current query, id = UINT32_MAX
};
}  // namespace

extern "C" {

// nearestK for nq queries; returns per query the ids/dists in the order the
// reference returns them (std::partial_sort, NearestNeighborsLinear.h:119-131).
int ref_linear_knn(const ompl_gpu_space *sp, const double *data, size_t n, const double *q, size_t nq, uint32_t k,
                   uint32_t *ids, double *dists, uint32_t *counts) {
    Ctx ctx{sp, data, nullptr};
    const uint32_t QID = 0xFFFFFFFFu;
    ompl::NearestNeighborsLinear<uint32_t> nn;
    nn.setDistanceFunction([&ctx, QID](const uint32_t &a, const uint32_t &b) {
        const double *pa = a == QID ? ctx.q : ctx.data + (size_t)a * ctx.sp->dim;
        const double *pb = b == QID ? ctx.q : ctx.data + (size_t)b * ctx.sp->dim;
        return oracle_distance(ctx.sp, pa, pb);
    });
    std::vector<uint32_t> all(n);
    for (size_t i = 0; i < n; ++i) all[i] = (uint32_t)i;
    nn.add(all);
    std::vector<uint32_t> out;
    for (size_t i = 0; i < nq; ++i) {
        ctx.q = q + i * sp->dim;
        nn.nearestK(QID, k, out);
        counts[i] = (uint32_t)out.size();
        for (size_t j = 0; j < k; ++j) {
            ids[i * k + j] = j < out.size() ? out[j] : 0xFFFFFFFFu;
            dists[i * k + j] = j < out.size() ? oracle_distance(sp, data + (size_t)out[j] * sp->dim, ctx.q) : -1.0;
        }
    }
    return 0;
}

// nearest(): first minimum (NearestNeighborsLinear.h:98-116); returns -1 and the
// exception text in err (if non-NULL, 128 bytes) when the structure is empty.
int ref_linear_nearest(const ompl_gpu_space *sp, const double *data, size_t n, const double *q, size_t nq,
                       uint32_t *ids, char *err) {
    Ctx ctx{sp, data, nullptr};
    const uint32_t QID = 0xFFFFFFFFu;
    ompl::NearestNeighborsLinear<uint32_t> nn;
    nn.setDistanceFunction([&ctx, QID](const uint32_t &a, const uint32_t &b) {
        const double *pa = a == QID ? ctx.q : ctx.data + (size_t)a * ctx.sp->dim;
        const double *pb = b == QID ? ctx.q : ctx.data + (size_t)b * ctx.sp->dim;
        return oracle_distance(ctx.sp, pa, pb);
    });
    for (size_t i = 0; i < n; ++i) nn.add((uint32_t)i);
    try {
        for (size_t i = 0; i < nq; ++i) {
            ctx.q = q + i * sp->dim;
            ids[i] = nn.nearest(QID);
        }
    } catch (const std::exception &e) {
        if (err) {
            std::strncpy(err, e.what(), 127);
            err[127] = 0;
        }
        return -1;
    }
    return 0;
}

// nearestR (NearestNeighborsLinear.h:135-142): pass ids == NULL to get counts only.
int ref_linear_radius(const ompl_gpu_space *sp, const double *data, size_t n, const double *q, size_t nq, double r,
                      const uint64_t *offsets, uint32_t *ids, uint64_t *counts) {
    Ctx ctx{sp, data, nullptr};
    const uint32_t QID = 0xFFFFFFFFu;
    ompl::NearestNeighborsLinear<uint32_t> nn;
    nn.setDistanceFunction([&ctx, QID](const uint32_t &a, const uint32_t &b) {
        const double *pa = a == QID ? ctx.q : ctx.data + (size_t)a * ctx.sp->dim;
        const double *pb = b == QID ? ctx.q : ctx.data + (size_t)b * ctx.sp->dim;
        return oracle_distance(ctx.sp, pa, pb);
    });
    std::vector<uint32_t> all(n);
    for (size_t i = 0; i < n; ++i) all[i] = (uint32_t)i;
    nn.add(all);
    std::vector<uint32_t> out;
    for (size_t i = 0; i < nq; ++i) {
        ctx.q = q + i * sp->dim;
        nn.nearestR(QID, r, out);
        counts[i] = out.size();
        if (ids)
            for (size_t j = 0; j < out.size(); ++j) ids[offsets[i] + j] = out[j];
    }
    return 0;
}

}  // extern "C"
