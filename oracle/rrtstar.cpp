// rrtstar.cpp — TEST INFRASTRUCTURE ONLY: the reference's RRT* iteration, sequential, as the
// checker of the device batch (ompl_gpu_rrtstar_batch_device + ompl_amd/rrtstar.py) and as the
// CPU baseline of the bench's RRT* workload.
//
// RRTstar::solve (src/ompl/geometric/planners/rrt/src/RRTstar.cpp:247-542) with its defaults:
// k-nearest neighbourhoods (useKNearest_, RRTstar.h:445), delayed collision checking (delayCC_,
// :458), rewire factor 1.1 (:449), no new-state rejection (:393-406 else branch), no tree
// pruning, no goal test (samples are given; the goal handling of :459-537 is planner logic), the
// path-length objective (motionCost = distance, combineCosts = +, isCostBetterThan = <,
// PathLengthOptimizationObjective / OptimizationObjective.cpp), per sample s:
//   nmotion = nearest(s)                                                   :266
//   d = distance(nmotion, s); x = s, or interpolate(nmotion, s, maxd / d) when d > maxd   :271-279
//   if checkMotion(nmotion, x):                                            :282
//     motion.incCost = distance(nmotion, x), cost = cost(nmotion) + incCost   :287-289
//     nbh = nearestK(x, ceil(k_rrt ln(size + 1)))                          :292, :603-611
//     delayCC: costs[i] = cost(nbh_i) + distance(nbh_i, x), neighbours in cost order, the first with
//       nbh_i == nmotion or (distance(nbh_i, x) < maxd and checkMotion(nbh_i, x)) is the parent,
//       the ones before it are marked invalid                              :319-357
//     add x                                                                :410-411
//     for each nbh_i != parent: new = cost(x) + incCost_i; if new < cost(nbh_i) and the motion is
//       valid (cached mark, else distance < maxd and checkMotion(x, nbh_i)): rewire nbh_i to x,
//       updateChildCosts(nbh_i)                                            :414-457, :620-643
// The neighbour structure is the brute force with (distance, id) order (NearestNeighborsLinear
// semantics) or the GNAT restatement (gnat.cpp).  The cost sort is std::stable_sort, so equal
// costs keep neighbour order (the reference's std::sort leaves ties unspecified; exact cost ties
// between distinct states do not occur with continuous samples).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <limits>
#include <numeric>
#include <vector>

#include "oracle.h"

namespace {

struct Tree {
    const ompl_gpu_space *sp;
    int dim;
    std::vector<double> states;
    std::vector<int64_t> parent;
    std::vector<double> inc, cost;
    std::vector<std::vector<uint32_t>> children;
    oracle_gnat *gnat = nullptr;

    size_t size() const { return parent.size(); }
    const double *st(uint64_t i) const { return states.data() + i * dim; }

    void add(const double *x, int64_t par, double ic, double c) {
        states.insert(states.end(), x, x + dim);
        parent.push_back(par);
        inc.push_back(ic);
        cost.push_back(c);
        children.emplace_back();
        if (par >= 0) children[par].push_back((uint32_t)(size() - 1));
        if (gnat) oracle_gnat_add(gnat, x, 1);
    }

    // nearestK in (distance, id) order
    void knn(const double *q, uint32_t k, std::vector<uint32_t> &ids, std::vector<double> &ds) const {
        const size_t n = size();
        const uint32_t kk = (uint32_t)std::min<size_t>(k, n);
        ids.resize(kk);
        ds.resize(kk);
        if (gnat) {
            std::vector<uint32_t> gi(k), cnt(1);
            std::vector<double> gd(k);
            oracle_gnat_knn(gnat, q, 1, k, gi.data(), gd.data(), cnt.data(), 1);
            for (uint32_t r = 0; r < kk; ++r) {
                ids[r] = gi[r];
                ds[r] = gd[r];
            }
            return;
        }
        std::vector<std::pair<double, uint32_t>> all(n);
        for (size_t i = 0; i < n; ++i) all[i] = {oracle_distance(sp, st(i), q), (uint32_t)i};
        std::partial_sort(all.begin(), all.begin() + kk, all.end());
        for (uint32_t r = 0; r < kk; ++r) {
            ids[r] = all[r].second;
            ds[r] = all[r].first;
        }
    }

    void remove_from_parent(uint32_t m) {  // RRTstar.cpp:620-631
        auto &ch = children[parent[m]];
        for (auto it = ch.begin(); it != ch.end(); ++it)
            if (*it == m) {
                ch.erase(it);
                break;
            }
    }

    void update_child_costs(uint32_t m) {  // RRTstar.cpp:633-643
        for (uint32_t c : children[m]) {
            cost[c] = cost[m] + inc[c];
            update_child_costs(c);
        }
    }
};

bool check_motion(const ompl_gpu_space *sp, const ompl_gpu_checker *ck, const double *a, const double *b, uint64_t &calls) {
    uint8_t v = 0;
    oracle_check_motions(sp, ck, a, b, 1, &v, nullptr, nullptr);
    ++calls;
    return v != 0;
}

}  // namespace

extern "C" uint64_t oracle_rrtstar(const ompl_gpu_space *sp, const ompl_gpu_checker *ck, const double *states0,
                                   size_t n0, const int64_t *parent0, const double *inc0, const double *cost0,
                                   const double *samples, size_t ns, double maxd, double k_rrt, int use_gnat,
                                   double time_budget_s, uint32_t *nearest_out, uint32_t *added_out,
                                   int64_t *parent_choice, int64_t *parent_out, double *inc_out, double *cost_out,
                                   uint64_t *stats) {
    Tree t;
    t.sp = sp;
    t.dim = sp->dim;
    const int dim = sp->dim;
    if (use_gnat) t.gnat = oracle_gnat_create(sp, 8, 4, 12, 50, 1);
    t.states.assign(states0, states0 + n0 * dim);
    t.parent.assign(parent0, parent0 + n0);
    t.inc.assign(inc0, inc0 + n0);
    t.cost.assign(cost0, cost0 + n0);
    t.children.assign(n0, {});
    for (size_t i = 0; i < n0; ++i)
        if (parent0[i] >= 0) t.children[parent0[i]].push_back((uint32_t)i);
    if (t.gnat) oracle_gnat_add_bulk(t.gnat, states0, n0);
    uint64_t added = 0, rewires = 0, calls = 0, processed = 0;
    std::vector<uint32_t> ids;
    std::vector<double> ds, costs, x(dim);
    std::vector<int8_t> valid;
    std::vector<size_t> order;
    const auto t0 = std::chrono::steady_clock::now();
    for (size_t i = 0; i < ns; ++i) {
        if (time_budget_s > 0 &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > time_budget_s)
            break;
        ++processed;
        const double *s = samples + i * dim;
        t.knn(s, 1, ids, ds);
        const uint32_t nm = ids[0];
        nearest_out[i] = nm;
        added_out[i] = 0xFFFFFFFFu;
        parent_choice[i] = -1;
        const double d = oracle_distance(sp, t.st(nm), s);
        if (d > maxd)
            oracle_interpolate(sp, t.st(nm), s, maxd / d, x.data());
        else
            std::copy(s, s + dim, x.begin());
        if (!check_motion(sp, ck, t.st(nm), x.data(), calls)) continue;
        double m_inc = oracle_distance(sp, t.st(nm), x.data());
        double m_cost = t.cost[nm] + m_inc;
        int64_t m_parent = nm;
        const double card = (double)(t.size() + 1);
        const uint32_t k = (uint32_t)std::ceil(k_rrt * std::log(card));
        t.knn(x.data(), k, ids, ds);
        const size_t nb = ids.size();
        costs.resize(nb);
        valid.assign(nb, 0);
        for (size_t r = 0; r < nb; ++r) costs[r] = t.cost[ids[r]] + ds[r];
        order.resize(nb);
        std::iota(order.begin(), order.end(), 0);
        std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return costs[a] < costs[b]; });
        for (size_t o = 0; o < nb; ++o) {
            const size_t r = order[o];
            if (ids[r] == nm || (ds[r] < maxd && check_motion(sp, ck, t.st(ids[r]), x.data(), calls))) {
                m_inc = ds[r];
                m_cost = costs[r];
                m_parent = ids[r];
                valid[r] = 1;
                break;
            }
            valid[r] = -1;
        }
        t.add(x.data(), m_parent, m_inc, m_cost);
        const uint32_t xi = (uint32_t)(t.size() - 1);
        added_out[i] = xi;
        parent_choice[i] = m_parent;
        ++added;
        for (size_t r = 0; r < nb; ++r) {
            const uint32_t v = ids[r];
            if ((int64_t)v == m_parent) continue;
            const double nc = t.cost[xi] + ds[r];
            if (nc < t.cost[v]) {
                bool ok;
                if (valid[r] == 0)
                    ok = ds[r] < maxd && check_motion(sp, ck, x.data(), t.st(v), calls);
                else
                    ok = valid[r] == 1;
                if (ok) {
                    t.remove_from_parent(v);
                    t.parent[v] = xi;
                    t.inc[v] = ds[r];
                    t.cost[v] = nc;
                    t.children[xi].push_back(v);
                    t.update_child_costs(v);
                    ++rewires;
                }
            }
        }
    }
    if (parent_out) std::copy(t.parent.begin(), t.parent.end(), parent_out);
    if (inc_out) std::copy(t.inc.begin(), t.inc.end(), inc_out);
    if (cost_out) std::copy(t.cost.begin(), t.cost.end(), cost_out);
    if (stats) {
        stats[0] = processed;
        stats[1] = added;
        stats[2] = rewires;
        stats[3] = calls;
        stats[4] = (uint64_t)(1e9 * std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    }
    if (t.gnat) oracle_gnat_destroy(t.gnat);
    return processed;
}
