// oracle.cpp — TEST INFRASTRUCTURE ONLY (see oracle.h header comment).
//
// CPU restatement of the reference's hot-path leaves in IEEE double with the
// reference's operation order.  Compiled with -O2 -ffp-contract=off so that no
// multiply-add is fused (the reference x86-64 build has no FMA:
// CMakeModules/CompilerSettings.cmake:8 sets no -march).
#include "oracle.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <thread>
#include <vector>

namespace {

constexpr double kPi = 3.141592653589793238462643383279502884;   // boost pi<double>()
constexpr double kQuatNormErr = 1e-9;                              // SO3StateSpace.cpp:47
const double kDblEps = std::numeric_limits<double>::epsilon();
const double kFltEps = (double)std::numeric_limits<float>::epsilon();

// RealVectorStateSpace::distance — RealVectorStateSpace.cpp:230-242
double l2(const double *a, const double *b, int n) {
    double acc = 0.0;
    for (int i = 0; i < n; ++i) {
        double diff = a[i] - b[i];
        acc += diff * diff;
    }
    return std::sqrt(acc);
}

// SO3 arcLength — SO3StateSpace.cpp:254-262 (q = x,y,z,w)
double arc(const double *p, const double *q) {
    double dq = std::fabs(p[0] * q[0] + p[1] * q[1] + p[2] * q[2] + p[3] * q[3]);
    if (dq > 1.0 - kQuatNormErr) return 0.0;
    return std::acos(dq);
}

// KinematicChainSpace::distance — demos/KinematicChain.h:105-124
double chain_dist(const double *a, const double *b, int n, double link) {
    double th1 = 0., th2 = 0., dx = 0., dy = 0., dist = 0.;
    for (int i = 0; i < n; ++i) {
        th1 += a[i];
        th2 += b[i];
        dx += std::cos(th1) - std::cos(th2);
        dy += std::sin(th1) - std::sin(th2);
        dist += std::sqrt(dx * dx + dy * dy);
    }
    return dist * link;
}

// RealVectorStateSpace::interpolate — RealVectorStateSpace.cpp:257-265
void lerp(const double *f, const double *t_, double t, double *o, int n) {
    for (int i = 0; i < n; ++i) o[i] = f[i] + (t_[i] - f[i]) * t;
}

// SO3StateSpace::interpolate (slerp) — SO3StateSpace.cpp:289-318
void slerp(const double *f, const double *to, double t, double *o) {
    double theta = arc(f, to);
    if (theta > kDblEps) {
        double d = 1.0 / std::sin(theta);
        double s0 = std::sin((1.0 - t) * theta);
        double s1 = std::sin(t * theta);
        double dq = f[0] * to[0] + f[1] * to[1] + f[2] * to[2] + f[3] * to[3];
        if (dq < 0) s1 = -s1;
        o[0] = (f[0] * s0 + to[0] * s1) * d;
        o[1] = (f[1] * s0 + to[1] * s1) * d;
        o[2] = (f[2] * s0 + to[2] * s1) * d;
        o[3] = (f[3] * s0 + to[3] * s1) * d;
    } else {
        if (o != f) std::memcpy(o, f, 4 * sizeof(double));
    }
}

// KinematicChainSpace::interpolate (±pi wrap) — demos/KinematicChain.h:150-175
void chain_interp(const double *f, const double *to, double t, double *o, int n) {
    for (int i = 0; i < n; ++i) {
        double diff = to[i] - f[i];
        if (std::fabs(diff) <= kPi) {
            o[i] = f[i] + diff * t;
        } else {
            if (diff > 0.0)
                diff = 2.0 * kPi - diff;
            else
                diff = -2.0 * kPi - diff;
            o[i] = f[i] - diff * t;
            if (o[i] > kPi)
                o[i] -= 2.0 * kPi;
            else if (o[i] < -kPi)
                o[i] += 2.0 * kPi;
        }
    }
}

// StateSpace::validSegmentCount — StateSpace.cpp:851-854
uint32_t seg_count(double d, double lvs, uint32_t factor) {
    return factor * (uint32_t)std::ceil(d / lvs);
}

// ---- validity checkers ------------------------------------------------------

// demos/HypercubeBenchmark.cpp:57-72
bool hypercube_valid(const double *s, int ndim, double edge) {
    bool found = false;
    for (int i = ndim - 1; i >= 0; i--) {
        if (!found) {
            if (s[i] > edge) found = true;
        } else if (s[i] < (1. - edge)) {
            return false;
        }
    }
    return true;
}

// tests/resources/circles2D.h:139-150 (and its 3-D extension for SPHERES)
bool circles_valid(const double *s, const double *c, int count) {
    for (int i = 0; i < count; ++i) {
        double dx = c[3 * i + 0] - s[0];
        double dy = c[3 * i + 1] - s[1];
        if (dx * dx + dy * dy < c[3 * i + 2]) return false;
    }
    return true;
}
bool spheres_valid(const double *s, const double *c, int count) {
    for (int i = 0; i < count; ++i) {
        double dx = c[4 * i + 0] - s[0];
        double dy = c[4 * i + 1] - s[1];
        double dz = c[4 * i + 2] - s[2];
        if (dx * dx + dy * dy + dz * dz < c[4 * i + 3]) return false;
    }
    return true;
}

// KinematicChainValidityChecker::intersectionTest — demos/KinematicChain.h:243-276
bool seg_intersect(const double *s0, const double *s1) {
    double s10_x = s0[2] - s0[0];
    double s10_y = s0[3] - s0[1];
    double s32_x = s1[2] - s1[0];
    double s32_y = s1[3] - s1[1];
    double denom = s10_x * s32_y - s32_x * s10_y;
    if (std::fabs(denom) < kDblEps) return false;
    bool denomPositive = denom > 0;
    double s02_x = s0[0] - s1[0];
    double s02_y = s0[1] - s1[1];
    double s_numer = s10_x * s02_y - s10_y * s02_x;
    if ((s_numer < kFltEps) == denomPositive) return false;
    double t_numer = s32_x * s02_y - s32_y * s02_x;
    if ((t_numer < kFltEps) == denomPositive) return false;
    if (((s_numer - denom > -kFltEps) == denomPositive) || ((t_numer - denom > kFltEps) == denomPositive))
        return false;
    return true;
}

// KinematicChainValidityChecker::isValidImpl — demos/KinematicChain.h:200-241
bool chain_valid(const double *s, int n, double link, const double *env, int nenv) {
    std::vector<double> seg(4 * (n + 1));
    double theta = 0., x = 0., y = 0., xN, yN;
    for (int i = 0; i < n; ++i) {
        theta += s[i];
        xN = x + std::cos(theta) * link;
        yN = y + std::sin(theta) * link;
        seg[4 * i + 0] = x; seg[4 * i + 1] = y; seg[4 * i + 2] = xN; seg[4 * i + 3] = yN;
        x = xN;
        y = yN;
    }
    xN = x + std::cos(theta) * 0.001;
    yN = y + std::sin(theta) * 0.001;
    seg[4 * n + 0] = x; seg[4 * n + 1] = y; seg[4 * n + 2] = xN; seg[4 * n + 3] = yN;
    const int ns = n + 1;
    for (int i = 0; i < ns; ++i)           // selfIntersectionTest :214-221
        for (int j = i + 1; j < ns; ++j)
            if (seg_intersect(&seg[4 * i], &seg[4 * j])) return false;
    for (int i = 0; i < ns; ++i)           // environmentIntersectionTest :223-230
        for (int j = 0; j < nenv; ++j)
            if (seg_intersect(&seg[4 * i], &env[4 * j])) return false;
    return true;
}

}  // namespace

extern "C" {

// CompoundStateSpace::distance — StateSpace.cpp:1068-1076 (SE3 = R3 + SO3)
double oracle_distance(const ompl_gpu_space *sp, const double *a, const double *b) {
    switch (sp->kind) {
    case OMPL_GPU_SPACE_REALVECTOR:
        return l2(a, b, sp->dim);
    case OMPL_GPU_SPACE_SO3:
        return arc(a, b);
    case OMPL_GPU_SPACE_SE3: {
        double dist = 0.0;
        dist += sp->weight[0] * l2(a, b, 3);
        dist += sp->weight[1] * arc(a + 3, b + 3);
        return dist;
    }
    case OMPL_GPU_SPACE_KCHAIN:
        return chain_dist(a, b, sp->dim, sp->link_length);
    }
    return std::numeric_limits<double>::quiet_NaN();
}

// SpaceInformation::getMotionStates with alloc = true — SpaceInformation.cpp:201-275: count
// is raised by one to the number of segments; fewer than 2 segments yield only the
// endpoints (when asked for); otherwise [s1], interpolate(j / segments) for j in
// [1, segments - 1], [s2]
uint32_t oracle_motion_states(const ompl_gpu_space *sp, const double *s1, const double *s2, size_t m,
                              uint32_t count, int endpoints, double *out) {
    const uint32_t segs = count + 1;
    const uint32_t per = segs < 2 ? (endpoints ? 2u : 0u) : segs + (endpoints ? 1u : 0u) - (endpoints ? 0u : 1u);
    const int dim = sp->dim;
    for (size_t e = 0; e < m; ++e) {
        const double *a = s1 + e * dim, *b = s2 + e * dim;
        double *o = out + e * per * dim;
        uint32_t added = 0;
        if (endpoints && per > 0) {
            std::copy(a, a + dim, o);
            ++added;
        }
        if (segs >= 2)
            for (uint32_t j = 1; j < segs && added < per; ++j) {
                oracle_interpolate(sp, a, b, (double)j / (double)segs, o + (size_t)added * dim);
                ++added;
            }
        if (added < per && endpoints) {
            std::copy(b, b + dim, o + (size_t)added * dim);
            ++added;
        }
    }
    return per;
}

// CompoundStateSpace::interpolate — StateSpace.cpp:1109-1116
void oracle_interpolate(const ompl_gpu_space *sp, const double *from, const double *to, double t, double *out) {
    switch (sp->kind) {
    case OMPL_GPU_SPACE_REALVECTOR: lerp(from, to, t, out, sp->dim); break;
    case OMPL_GPU_SPACE_SO3: slerp(from, to, t, out); break;
    case OMPL_GPU_SPACE_SE3:
        lerp(from, to, t, out, 3);
        slerp(from + 3, to + 3, t, out + 3);
        break;
    case OMPL_GPU_SPACE_KCHAIN: chain_interp(from, to, t, out, sp->dim); break;
    }
}

// CompoundStateSpace::validSegmentCount (max over components) — StateSpace.cpp:1085-1097
uint32_t oracle_valid_segment_count(const ompl_gpu_space *sp, const double *a, const double *b) {
    switch (sp->kind) {
    case OMPL_GPU_SPACE_REALVECTOR: return seg_count(l2(a, b, sp->dim), sp->lvs[0], sp->factor[0]);
    case OMPL_GPU_SPACE_SO3: return seg_count(arc(a, b), sp->lvs[0], sp->factor[0]);
    case OMPL_GPU_SPACE_SE3: {
        uint32_t sc = 0;
        uint32_t s0 = seg_count(l2(a, b, 3), sp->lvs[0], sp->factor[0]);
        if (s0 > sc) sc = s0;
        uint32_t s1 = seg_count(arc(a + 3, b + 3), sp->lvs[1], sp->factor[1]);
        if (s1 > sc) sc = s1;
        return sc;
    }
    case OMPL_GPU_SPACE_KCHAIN:
        return seg_count(chain_dist(a, b, sp->dim, sp->link_length), sp->lvs[0], sp->factor[0]);
    }
    return 0;
}

int oracle_is_valid(const ompl_gpu_space *sp, const ompl_gpu_checker *ck, const double *s) {
    switch (ck->kind) {
    case OMPL_GPU_CHECK_ALL_VALID: return 1;
    case OMPL_GPU_CHECK_HYPERCUBE: return hypercube_valid(s, ck->ndim, ck->edge_width);
    case OMPL_GPU_CHECK_SPHERES: return spheres_valid(s, ck->data, ck->count);
    case OMPL_GPU_CHECK_CIRCLES2D: return circles_valid(s, ck->data, ck->count);
    case OMPL_GPU_CHECK_KCHAIN: return chain_valid(s, sp->dim, sp->link_length, ck->data, ck->count);
    }
    return 0;
}

// DiscreteMotionValidator::checkMotion(s1,s2) — DiscreteMotionValidator.cpp:93-145 (bisection FIFO)
// and checkMotion(s1,s2,lastValid) — :48-91 (linear sweep, for first_invalid).
uint64_t oracle_check_motions(const ompl_gpu_space *sp, const ompl_gpu_checker *ck, const double *s1,
                              const double *s2, size_t m, uint8_t *valid, int32_t *nd_out,
                              int32_t *first_invalid) {
    const int dim = sp->dim;
    std::vector<double> test(dim);
    std::vector<std::pair<int, int>> fifo;
    uint64_t checks = 0;
    for (size_t e = 0; e < m; ++e) {
        const double *a = s1 + e * dim, *b = s2 + e * dim;
        int nd = (int)oracle_valid_segment_count(sp, a, b);
        if (nd_out) nd_out[e] = nd;
        // --- bisection variant (the default planners call) ---
        bool result = true;
        ++checks;
        if (!oracle_is_valid(sp, ck, b)) {
            result = false;
        } else if (nd >= 2) {
            fifo.clear();
            size_t head = 0;
            fifo.emplace_back(1, nd - 1);
            while (head < fifo.size()) {
                std::pair<int, int> x = fifo[head];
                int mid = (x.first + x.second) / 2;
                oracle_interpolate(sp, a, b, (double)mid / (double)nd, test.data());
                ++checks;
                if (!oracle_is_valid(sp, ck, test.data())) {
                    result = false;
                    break;
                }
                ++head;
                if (x.first < mid) fifo.emplace_back(x.first, mid - 1);
                if (x.second > mid) fifo.emplace_back(mid + 1, x.second);
            }
        }
        if (valid) valid[e] = result ? 1 : 0;
        // --- linear variant: first invalid sample ---
        if (first_invalid) {
            int fi = -1;
            if (nd > 1) {
                for (int j = 1; j < nd; ++j) {
                    oracle_interpolate(sp, a, b, (double)j / (double)nd, test.data());
                    if (!oracle_is_valid(sp, ck, test.data())) { fi = j; break; }
                }
            }
            if (fi < 0 && !oracle_is_valid(sp, ck, b)) fi = nd;
            first_invalid[e] = fi;
        }
    }
    return checks;
}

uint64_t oracle_check_motions_mt(const ompl_gpu_space *sp, const ompl_gpu_checker *ck, const double *s1,
                                 const double *s2, size_t m, uint8_t *valid, int nthreads) {
    if (nthreads <= 1) return oracle_check_motions(sp, ck, s1, s2, m, valid, nullptr, nullptr);
    std::vector<std::thread> th;
    std::vector<uint64_t> cnt(nthreads, 0);
    const size_t per = (m + nthreads - 1) / nthreads;
    for (int t = 0; t < nthreads; ++t) {
        size_t b = t * per, e = std::min(m, b + per);
        if (b >= e) break;
        th.emplace_back([=, &cnt] {
            cnt[t] = oracle_check_motions(sp, ck, s1 + b * sp->dim, s2 + b * sp->dim, e - b,
                                          valid ? valid + b : nullptr, nullptr, nullptr);
        });
    }
    uint64_t tot = 0;
    for (size_t t = 0; t < th.size(); ++t) { th[t].join(); tot += cnt[t]; }
    return tot;
}

// Brute force kNN with NearestNeighborsLinear semantics (NearestNeighborsLinear.h:119-131):
// results sorted ascending; ties resolved by insertion index (Linear's partial_sort leaves
// tie order unspecified; the tests accept any order inside a tie class).
void oracle_knn(const ompl_gpu_space *sp, const double *data, size_t n, const double *q, size_t nq,
                uint32_t k, uint32_t *ids, double *dists, uint32_t *counts) {
    const int dim = sp->dim;
    std::vector<std::pair<double, uint32_t>> all(n);
    for (size_t qi = 0; qi < nq; ++qi) {
        for (size_t i = 0; i < n; ++i)
            all[i] = {oracle_distance(sp, data + i * dim, q + qi * dim), (uint32_t)i};
        size_t kk = std::min<size_t>(k, n);
        std::partial_sort(all.begin(), all.begin() + kk, all.end());
        for (size_t j = 0; j < kk; ++j) {
            ids[qi * k + j] = all[j].second;
            dists[qi * k + j] = all[j].first;
        }
        for (size_t j = kk; j < k; ++j) {
            ids[qi * k + j] = 0xFFFFFFFFu;
            dists[qi * k + j] = std::numeric_limits<double>::infinity();
        }
        if (counts) counts[qi] = (uint32_t)kk;
    }
}

// nearestR with Linear semantics (NearestNeighborsLinear.h:135-142): d <= r inclusive, sorted.
void oracle_radius(const ompl_gpu_space *sp, const double *data, size_t n, const double *q, size_t nq,
                   double r, const uint64_t *offsets, uint32_t *ids, double *dists, uint64_t *counts) {
    const int dim = sp->dim;
    std::vector<std::pair<double, uint32_t>> hit;
    for (size_t qi = 0; qi < nq; ++qi) {
        hit.clear();
        for (size_t i = 0; i < n; ++i) {
            double d = oracle_distance(sp, data + i * dim, q + qi * dim);
            if (d <= r) hit.emplace_back(d, (uint32_t)i);
        }
        if (counts) counts[qi] = hit.size();
        if (ids) {
            std::sort(hit.begin(), hit.end());
            for (size_t j = 0; j < hit.size(); ++j) {
                ids[offsets[qi] + j] = hit[j].second;
                dists[offsets[qi] + j] = hit[j].first;
            }
        }
    }
}

}  // extern "C"

/* PRM* roadmap construction, the reference's sequential loop: PRM::addMilestone
 * (geometric/planners/prm/src/PRM.cpp:562-596) with KStarStrategy (ConnectionStrategy.h:145-149):
 * vertex i asks the nearest-neighbour structure (which holds vertices 0..i-1) for its
 * k_i = ceil(k_const * log(i + 1)) nearest, checks checkMotion(state[n], state[i]) for each, then
 * is added.  Neighbours in (distance, index) order (NearestNeighborsLinear semantics). */
extern "C" void oracle_prm_causal(const ompl_gpu_space *sp, const ompl_gpu_checker *ck, const double *states, size_t n,
                                  double k_const, uint32_t k_cap, uint32_t *nbr, uint32_t *cnt, uint8_t *valid) {
    const int dim = sp->dim;
    std::vector<uint32_t> ids(k_cap);
    std::vector<double> ds(k_cap), s1(k_cap * dim), s2(k_cap * dim);
    std::vector<uint8_t> v(k_cap);
    for (size_t i = 0; i < n; ++i) {
        const double kk = std::ceil(k_const * std::log((double)(i + 1)));
        uint32_t k = kk > 0 ? (uint32_t)kk : 0u;
        if (k > k_cap) k = k_cap;
        uint32_t c = 0;
        if (k > 0 && i > 0) oracle_knn(sp, states, i, states + i * dim, 1, k, ids.data(), ds.data(), &c);
        cnt[i] = c;
        for (uint32_t r = 0; r < k_cap; ++r) {
            nbr[i * k_cap + r] = r < c ? ids[r] : 0xFFFFFFFFu;
            valid[i * k_cap + r] = 0;
        }
        for (uint32_t r = 0; r < c; ++r)
            for (int d = 0; d < dim; ++d) {
                s1[r * dim + d] = states[(size_t)ids[r] * dim + d];
                s2[r * dim + d] = states[i * dim + d];
            }
        if (c) {
            oracle_check_motions(sp, ck, s1.data(), s2.data(), c, v.data(), nullptr, nullptr);
            for (uint32_t r = 0; r < c; ++r) valid[i * k_cap + r] = v[r];
        }
    }
}
