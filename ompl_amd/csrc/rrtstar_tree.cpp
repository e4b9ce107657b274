// rrtstar_tree.cpp — RRT*'s cost logic over a staged device batch (host C++; see rrtstar_tree.h).
//
// For every sample of the batch whose state x joined the tree, in sample order, exactly as
// RRTstar::solve with delayCC (RRTstar.cpp:285-457, the path-length objective: motionCost =
// distance, combineCosts = +, isCostBetterThan = <):
//   the motion as created: parent nmotion, incCost = distance(nmotion, x), cost = cost(nmotion) +
//     incCost (:285-289);
//   the neighbours in order of cost(nbh) + distance(nbh, x) (a stable sort: equal costs keep the
//     (distance, id) order; the reference's std::sort leaves such ties unspecified), the first with
//     nbh == nmotion or (distance < maxDistance and checkMotion(nbh, x)) becomes the parent, the
//     ones before it are marked invalid (:319-357);
//   x joins its parent's children (:410-411);
//   rewiring, in neighbourhood order (:414-457): for each nbh != parent with cost(x) + distance <
//     cost(nbh) and a valid motion (the cached mark, else distance < maxDistance and
//     checkMotion(x, nbh)), nbh leaves its parent's children (removeFromParent :620-631), takes x
//     as parent, and its subtree's costs follow (updateChildCosts :633-643).
// The checkMotion results are the device's bits; none of the device work depends on costs.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <system_error>
#include <thread>
#include <memory>
#include <cstring>
#include <new>
#include <numeric>

#include "../../include/ompl_gpu.h"
#include "rrtstar_tree.h"

namespace ompl_amd {
void set_last_error(const char *msg);  // capi.hip
}

using ompl_amd::RrtStarStaged;

namespace {

ompl_gpu_status bad(ompl_gpu_status s, const char *msg) {
    ompl_amd::set_last_error(msg);
    return s;
}

// the states whose cost changed during one sample's rewiring (a rewired neighbour and its
// subtree): an open-addressing set tagged by the sample's epoch, so that the rewiring loop reads
// each neighbour's cost from the contiguous copy taken before it (cv) unless the state is in the
// set — one random read of the tree's costs per neighbour instead of two
struct Touched {
    static constexpr uint32_t kSlots = 4096, kMax = 2048;
    std::vector<uint64_t> slot = std::vector<uint64_t>(kSlots, 0);
    uint32_t epoch = 0, count = 0;
    bool all = false;  // too many: every read goes to the tree
    void reset() {
        ++epoch;
        count = 0;
        all = false;
    }
    static uint32_t hash(uint32_t v) { return (v * 0x9E3779B1u) >> 20; }
    void add(uint32_t v) {
        if (all) return;
        if (++count > kMax) {
            all = true;
            return;
        }
        const uint64_t tag = ((uint64_t)epoch << 32) | v;
        for (uint32_t h = hash(v);; h = (h + 1) & (kSlots - 1)) {
            if ((uint32_t)(slot[h] >> 32) != epoch) {
                slot[h] = tag;
                return;
            }
            if (slot[h] == tag) return;
        }
    }
    bool has(uint32_t v) const {
        if (all) return true;
        const uint64_t tag = ((uint64_t)epoch << 32) | v;
        for (uint32_t h = hash(v);; h = (h + 1) & (kSlots - 1)) {
            if ((uint32_t)(slot[h] >> 32) != epoch) return false;
            if (slot[h] == tag) return true;
        }
    }
};

// A few host threads for the per-neighbour pass (the costs are read by neighbour id, random over
// the tree: ~7 ns each on one core, so a batch's 1.8 M neighbourhood entries cost ~14 ms on one
// thread).  Workers spin while a commit is active and sleep on a condition variable otherwise.
class Pool {
public:
    explicit Pool(int nthreads) {
        try {
            for (int k = 1; k < nthreads; ++k) th_.emplace_back([this, k] { work(k); });
        } catch (const std::system_error &) {  // fewer threads than asked: the caller does the rest
        }
        n_ = 1 + (int)th_.size();
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            quit_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    int size() const { return n_; }
    void begin() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            active_.store(true);
        }
        cv_.notify_all();
    }
    void end() { active_.store(false); }
    // f(k) on every thread k in [0, size()), the caller being thread 0; returns when all are done
    void run(const std::function<void(int)> &f) {
        if (n_ == 1) {
            f(0);
            return;
        }
        job_ = &f;
        pending_.store(n_ - 1, std::memory_order_relaxed);
        gen_.fetch_add(1, std::memory_order_seq_cst);
        if (sleepers_.load(std::memory_order_seq_cst) > 0) {  // wake the workers that stopped spinning
            { std::lock_guard<std::mutex> lk(mu_); }
            cv_.notify_all();
        }
        f(0);
        while (pending_.load(std::memory_order_acquire)) __builtin_ia32_pause();
    }

private:
    // a worker spins for the next job while the pool is active, at most kSpin pauses after its last
    // one (the two pool phases of a sample are microseconds apart), then sleeps until a job or the
    // end: a sequential stretch of the commit (the rewiring loop) or the time between commits does
    // not keep the host cores busy
    static constexpr int kSpin = 1 << 14;
    void work(int k) {
        uint64_t seen = 0;
        for (;;) {
            int spins = 0;
            while (gen_.load(std::memory_order_acquire) == seen) {
                if (active_.load(std::memory_order_relaxed) && spins < kSpin) {
                    ++spins;
                    __builtin_ia32_pause();
                    continue;
                }
                sleepers_.fetch_add(1, std::memory_order_seq_cst);
                {
                    std::unique_lock<std::mutex> lk(mu_);
                    cv_.wait(lk, [&] { return quit_ || gen_.load(std::memory_order_seq_cst) != seen; });
                }
                sleepers_.fetch_sub(1, std::memory_order_seq_cst);
                {
                    std::lock_guard<std::mutex> lk(mu_);
                    if (quit_) return;
                }
                spins = 0;
            }
            seen = gen_.load(std::memory_order_acquire);
            (*job_)(k);
            pending_.fetch_sub(1, std::memory_order_release);
        }
    }
    std::vector<std::thread> th_;
    int n_ = 1;
    std::mutex mu_;
    std::condition_variable cv_;
    bool quit_ = false;
    std::atomic<bool> active_{false};
    std::atomic<int> sleepers_{0};
    std::atomic<uint64_t> gen_{0};
    std::atomic<int> pending_{0};
    const std::function<void(int)> *job_ = nullptr;
};

template <class Mark>
uint64_t update_child_costs(ompl_gpu_rrtstar_tree *t, uint32_t m, Mark &&mark) {  // RRTstar.cpp:633-643, iterative
    auto &st = t->stack;
    st.clear();
    st.push_back(m);
    uint64_t visits = 0;
    while (!st.empty()) {
        const uint32_t u = st.back();
        st.pop_back();
        const double cu = t->cost[u];
        visits += t->children[u].size();
        for (uint32_t c : t->children[u]) {
            t->cost[c] = cu + t->inc[c];
            mark(c);
            if (!t->children[c].empty()) st.push_back(c);
        }
    }
    return visits;
}

// removeFromParent (RRTstar.cpp:620-631) in O(1): every state knows its slot in its parent's
// children list, and the last child moves into the freed slot.  The order of a children list
// changes nothing: updateChildCosts sets each child's cost from its parent's, in any order.
void remove_from_parent(ompl_gpu_rrtstar_tree *t, uint32_t m) {
    auto &ch = t->children[(size_t)t->parent[m]];
    const uint32_t i = t->slot[m], last = ch.back();
    ch[i] = last;
    t->slot[last] = i;
    ch.pop_back();
}

void add_child(ompl_gpu_rrtstar_tree *t, uint32_t p, uint32_t c) {
    t->slot[c] = (uint32_t)t->children[p].size();
    t->children[p].push_back(c);
}

void grow(ompl_gpu_rrtstar_tree *t, size_t n) {
    if (t->parent.size() >= n) return;
    t->parent.resize(n, -1);
    t->inc.resize(n, 0.0);
    t->cost.resize(n, 0.0);
    t->children.resize(n);
    t->slot.resize(n, 0);
}

}  // namespace

extern "C" {

ompl_gpu_status ompl_gpu_rrtstar_tree_create(ompl_gpu_rrtstar_tree **out) {
    if (!out) return bad(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    *out = new (std::nothrow) ompl_gpu_rrtstar_tree();
    return *out ? OMPL_GPU_OK : bad(OMPL_GPU_ERR_OOM, "out of host memory");
}

void ompl_gpu_rrtstar_tree_destroy(ompl_gpu_rrtstar_tree *t) { delete t; }

ompl_gpu_status ompl_gpu_rrtstar_tree_add(ompl_gpu_rrtstar_tree *t, size_t m, const int64_t *parent,
                                          const double *inc, const double *cost) {
    if (!t) return bad(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    const size_t first = t->parent.size();
    for (size_t j = 0; j < m; ++j) {
        const int64_t p = parent ? parent[j] : -1;
        if (p < -1 || p >= (int64_t)(first + j)) return bad(OMPL_GPU_ERR_INVALID_ARG, "parent must be -1 or an earlier id");
        // a start state's cost is the objective's identity (RRTstar.cpp:208-213): with any other
        // cost a rewire could reach a root, which has no parent to leave (:620-631)
        if (p == -1 && cost && !(cost[j] == 0.0))
            return bad(OMPL_GPU_ERR_INVALID_ARG, "a start state (parent -1) must have cost 0");
    }
    try {
        grow(t, first + m);
    } catch (const std::bad_alloc &) {
        return bad(OMPL_GPU_ERR_OOM, "out of host memory");
    }
    for (size_t j = 0; j < m; ++j) {
        const size_t v = first + j;
        t->parent[v] = parent ? parent[j] : -1;
        t->inc[v] = inc ? inc[j] : 0.0;
        t->cost[v] = cost ? cost[j] : 0.0;  // a start state's cost: the identity (RRTstar.cpp:208-213)
        if (t->parent[v] >= 0) {
            add_child(t, (uint32_t)t->parent[v], (uint32_t)v);
            // a cost that is not its parent's + incCost can rise under updateChildCosts
            if (!(t->cost[v] == t->cost[(size_t)t->parent[v]] + t->inc[v])) t->consistent = false;
        }
    }
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_rrtstar_tree_size(const ompl_gpu_rrtstar_tree *t, size_t *n) {
    if (!t || !n) return bad(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    *n = t->parent.size();
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_rrtstar_tree_read(const ompl_gpu_rrtstar_tree *t, size_t first, size_t m, int64_t *parent,
                                           double *inc, double *cost) {
    if (!t) return bad(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    if (first > t->parent.size() || m > t->parent.size() - first) return bad(OMPL_GPU_ERR_INVALID_ARG, "range past the tree");
    if (parent) std::memcpy(parent, t->parent.data() + first, sizeof(int64_t) * m);
    if (inc) std::memcpy(inc, t->inc.data() + first, sizeof(double) * m);
    if (cost) std::memcpy(cost, t->cost.data() + first, sizeof(double) * m);
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_rrtstar_tree_totals(const ompl_gpu_rrtstar_tree *t, uint64_t totals[6]) {
    if (!t || !totals) return bad(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    std::memcpy(totals, t->totals, sizeof(t->totals));
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_rrtstar_stage_host(ompl_gpu_rrtstar_tree *t, size_t ns, const uint32_t *nearest,
                                            const uint32_t *added, const double *inc, const uint64_t *offsets,
                                            const uint32_t *ids, const double *dist, const uint8_t *bits) {
    if (!t || (ns && (!nearest || !added || !inc || !offsets))) return bad(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    const size_t E = ns ? (size_t)offsets[ns] : 0;
    if (E && (!ids || !dist || !bits)) return bad(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    for (size_t i = 0; i < ns; ++i)
        if (offsets[i] > offsets[i + 1]) return bad(OMPL_GPU_ERR_INVALID_ARG, "offsets must not decrease");
    RrtStarStaged b;
    try {
        b.ns = ns;
        b.nearest.assign(nearest, nearest + ns);
        b.added.assign(added, added + ns);
        b.inc.assign(inc, inc + ns);
        b.off.assign(offsets, offsets + ns + 1);
        if (!ns) b.off.assign(1, 0);
        b.ids.assign(ids, ids + E);
        b.dist.assign(dist, dist + E);
        b.bits.assign(bits, bits + E);
    } catch (const std::bad_alloc &) {
        return bad(OMPL_GPU_ERR_OOM, "out of host memory");
    }
    std::lock_guard<std::mutex> lk(t->mu);
    t->staged.push_back(std::move(b));
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_rrtstar_commit(ompl_gpu_rrtstar_tree *t, double max_distance, size_t ns_cap,
                                        int64_t *nearest, int64_t *added, int64_t *chosen, size_t *ns_out) {
    if (!t) return bad(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    RrtStarStaged b;
    {
        std::lock_guard<std::mutex> lk(t->mu);
        if (t->staged.empty()) return bad(OMPL_GPU_ERR_INVALID_ARG, "no staged batch");
        if ((nearest || added || chosen) && t->staged.front().ns > ns_cap)
            return bad(OMPL_GPU_ERR_INVALID_ARG, "output arrays shorter than the staged batch");
        b = std::move(t->staged.front());
        t->staged.pop_front();
    }
    const size_t ns = b.ns;
    if (ns_out) *ns_out = ns;
    const double maxd = max_distance;
    uint64_t rewires = 0, checks = 0, nadd = 0, visits = 0;
    if (!t->touched) t->touched = std::make_shared<Touched>();
    Touched &touched = *std::static_pointer_cast<Touched>(t->touched);
    if (!t->pool) {
        try {
            t->pool = std::make_shared<Pool>((int)std::max(1u, std::min(8u, std::thread::hardware_concurrency())));
        } catch (const std::exception &) {
            return bad(OMPL_GPU_ERR_OOM, "no host threads");
        }
    }
    Pool &pool = *std::static_pointer_cast<Pool>(t->pool);
    struct Active {  // the workers spin for the length of the commit
        Pool &p;
        explicit Active(Pool &q) : p(q) { p.begin(); }
        ~Active() { p.end(); }
    } active(pool);
    struct Best {
        size_t r;
        double c;
    };
    std::vector<Best> bests((size_t)pool.size());
    try {
        uint32_t top = 0;
        for (size_t i = 0; i < ns; ++i)
            if (b.added[i] != 0xFFFFFFFFu) top = std::max(top, b.added[i] + 1);
        const size_t n = std::max(t->parent.size(), (size_t)top);  // every id the batch names is a state
        bool ok = b.off.size() == ns + 1 && b.off[ns] == b.ids.size();
        for (size_t i = 0; ok && i < ns; ++i) ok = b.nearest[i] < n && b.off[i] <= b.off[i + 1];
        for (size_t j = 0; ok && j < b.ids.size(); ++j) ok = b.ids[j] < n;
        if (!ok) return bad(OMPL_GPU_ERR_INVALID_ARG, "staged batch names ids outside the tree");
        // the added ids are new (>= the tree's size), strictly increasing, and each added state's
        // nearest state and neighbours are earlier states
        uint64_t next = t->parent.size();
        for (size_t i = 0; ok && i < ns; ++i) {
            const uint32_t x = b.added[i];
            if (x == 0xFFFFFFFFu) continue;
            ok = x >= next && b.nearest[i] < x;
            next = (uint64_t)x + 1;
            for (uint64_t j = b.off[i]; ok && j < b.off[i + 1]; ++j) ok = b.ids[j] < x;
        }
        if (!ok) return bad(OMPL_GPU_ERR_INVALID_ARG, "staged batch: added ids not new and increasing, or neighbours not earlier");
        grow(t, top);
        for (size_t i = 0; i < ns; ++i) {
            const uint32_t nm = b.nearest[i], x = b.added[i];
            if (nearest) nearest[i] = nm;
            if (added) added[i] = x == 0xFFFFFFFFu ? -1 : (int64_t)x;
            if (chosen) chosen[i] = -1;
            ++checks;  // checkMotion(nmotion, x) (:282)
            if (x == 0xFFFFFFFFu) continue;
            const uint64_t a = b.off[i], e = b.off[i + 1];
            const size_t nb = (size_t)(e - a);
            const uint32_t *ids = b.ids.data() + a;
            const double *d = b.dist.data() + a;
            const uint8_t *bt = b.bits.data() + a;
            double m_inc = b.inc[i], m_cost = t->cost[nm] + m_inc;
            int64_t m_parent = nm;
            // delayCC: neighbours in cost order, the first with a valid connection (:319-357).  The
            // stable sort's order is the (cost, index) order, so the first valid neighbour is the
            // valid one of least (cost, index), and the ones the loop marks invalid before it are
            // exactly those of smaller (cost, index): two scans, no sort
            t->costs.resize(nb);
            t->cv.resize(nb);
            // each thread a contiguous part: the neighbours' costs (cv), cost + distance (costs) and
            // its part's valid candidate of least (cost, index)
            const int T = nb >= 1024 ? pool.size() : 1;
            auto part = [&](int k) {
                const size_t r0 = nb * (size_t)k / (size_t)T, r1 = nb * (size_t)(k + 1) / (size_t)T;
                size_t bi = nb;
                double bcost = 0.0;
                for (size_t r = r0; r < r1; ++r) {
                    const double cr = t->cost[ids[r]];
                    const double c = cr + d[r];
                    t->cv[r] = cr;
                    t->costs[r] = c;
                    if ((bi == nb || c < bcost) && (ids[r] == nm || (d[r] < maxd && (bt[r] & 1)))) {
                        bi = r;
                        bcost = c;
                    }
                }
                bests[(size_t)k] = Best{bi, bcost};
            };
            if (T > 1)
                pool.run(part);
            else
                part(0);
            size_t best = nb;
            double bc = 0.0;
            for (int k = 0; k < T; ++k)  // parts in index order: a strict < keeps the lower index on ties
                if (bests[(size_t)k].r < nb && (best == nb || bests[(size_t)k].c < bc)) {
                    best = bests[(size_t)k].r;
                    bc = bests[(size_t)k].c;
                }
            if (best < nb) {
                m_inc = d[best];
                m_cost = bc;
                m_parent = ids[best];
            }
            // the motion joins the tree (:410-411)
            t->parent[x] = m_parent;
            t->inc[x] = m_inc;
            t->cost[x] = m_cost;
            add_child(t, (uint32_t)m_parent, x);
            if (chosen) chosen[i] = m_parent;
            ++nadd;
            // rewiring (:414-457), with the parent choice's marks: the neighbours before the parent in
            // (cost, index) order were found invalid (-1), the parent valid (1), the rest unchecked (0)
            touched.reset();
            const double cx = t->cost[x];  // x is no neighbour's descendant: its cost stays
            if (t->consistent) {
                // costs only fall in a consistent tree, so a neighbour whose cost as read before the loop
                // (cv) x cannot lower never becomes a candidate later: the pool collects, in index
                // order, the neighbours x can lower (and counts the parent choice's checkMotion calls);
                // the sequential loop visits only those, with the tree bookkeeping of the candidates a
                // few ahead prefetched (the rewires' random reads were the cost of this loop)
                auto scan = [&](int k) {
                    const size_t r0 = nb * (size_t)k / (size_t)T, r1 = nb * (size_t)(k + 1) / (size_t)T;
                    auto &cl = t->cand[(size_t)k];
                    cl.clear();
                    uint64_t ck = 0;
                    for (size_t r = r0; r < r1; ++r) {
                        const bool before = best == nb || t->costs[r] < bc || (t->costs[r] == bc && r < best);
                        if ((before || r == best) && ids[r] != nm && d[r] < maxd) ++ck;  // checkMotion(nbh, x)
                        if ((int64_t)ids[r] == m_parent) continue;
                        if (cx + d[r] < t->cv[r]) cl.push_back((uint32_t)r);
                    }
                    t->cand_checks[(size_t)k] = ck;
                };
                t->cand.resize((size_t)pool.size());
                t->cand_checks.resize((size_t)pool.size());
                if (T > 1)
                    pool.run(scan);
                else
                    scan(0);
                for (int k = 0; k < T; ++k) {
                    checks += t->cand_checks[(size_t)k];
                    const auto &cl = t->cand[(size_t)k];
                    const size_t nc_ = cl.size();
                    for (size_t q = 0; q < nc_; ++q) {
                        // (hints only: a rewire may move what they point at)
                        if (q + 12 < nc_) {
                            const uint32_t v = ids[cl[q + 12]];
                            __builtin_prefetch(&t->parent[v]);
                            __builtin_prefetch(&t->slot[v]);
                            __builtin_prefetch(&t->children[v]);
                            __builtin_prefetch(&t->cost[v], 1);
                            __builtin_prefetch(&t->inc[v], 1);
                        }
                        if (q + 6 < nc_) {
                            const uint32_t v = ids[cl[q + 6]];
                            const int64_t p = t->parent[v];
                            if (p >= 0) __builtin_prefetch(&t->children[(size_t)p]);
                        }
                        if (q + 3 < nc_) {
                            const uint32_t v = ids[cl[q + 3]];
                            const int64_t p = t->parent[v];
                            if (p >= 0) {
                                const auto &ch = t->children[(size_t)p];
                                if (!ch.empty()) {
                                    __builtin_prefetch(ch.data() + t->slot[v], 1);
                                    __builtin_prefetch(ch.data() + ch.size() - 1);
                                    __builtin_prefetch(&t->slot[ch.back()], 1);
                                }
                            }
                        }
                        const size_t r = cl[q];
                        const bool before = best == nb || t->costs[r] < bc || (t->costs[r] == bc && r < best);
                        const int8_t mark = r == best ? 1 : (before ? -1 : 0);
                        const uint32_t v = ids[r];
                        if (t->parent[v] < 0) continue;  // a start state keeps no parent (cost 0: never lowered)
                        const double nc = cx + d[r];
                        if (touched.has(v) && !(nc < t->cost[v])) continue;
                        bool ok;
                        if (mark == 0) {
                            ok = d[r] < maxd && (bt[r] & 2);
                            if (d[r] < maxd) ++checks;
                        } else {
                            ok = mark == 1;
                        }
                        if (!ok) continue;
                        remove_from_parent(t, v);
                        t->parent[v] = x;
                        t->inc[v] = d[r];
                        t->cost[v] = nc;
                        add_child(t, x, v);
                        touched.add(v);
                        visits += update_child_costs(t, v, [&](uint32_t c) { touched.add(c); });
                        ++rewires;
                    }
                }
                continue;
            }
            for (size_t r = 0; r < nb; ++r) {
                const bool before = best == nb || t->costs[r] < bc || (t->costs[r] == bc && r < best);
                const int8_t mark = r == best ? 1 : (before ? -1 : 0);
                if ((before || r == best) && ids[r] != nm && d[r] < maxd) ++checks;  // checkMotion(nbh, x) calls
                const uint32_t v = ids[r];
                if ((int64_t)v == m_parent || t->parent[v] < 0) continue;  // a start state keeps no parent
                const double nc = cx + d[r];
                // the cost as this loop found it, or as an earlier rewire of this loop left it.  In a
                // consistent tree (every cost = parent's cost + incCost, as RRT* keeps it) costs only
                // fall, so nc >= the cost found means no rewire either way
                if (t->consistent) {
                    if (!(nc < t->cv[r])) continue;
                    if (touched.has(v) && !(nc < t->cost[v])) continue;
                } else {
                    const double cur = touched.has(v) ? t->cost[v] : t->cv[r];
                    if (!(nc < cur)) continue;
                }
                bool ok;
                if (mark == 0) {
                    ok = d[r] < maxd && (bt[r] & 2);
                    if (d[r] < maxd) ++checks;
                } else {
                    ok = mark == 1;
                }
                if (!ok) continue;
                remove_from_parent(t, v);
                t->parent[v] = x;
                t->inc[v] = d[r];
                t->cost[v] = nc;
                add_child(t, x, v);
                touched.add(v);
                visits += update_child_costs(t, v, [&](uint32_t c) { touched.add(c); });
                ++rewires;
            }
        }
    } catch (const std::bad_alloc &) {
        return bad(OMPL_GPU_ERR_OOM, "out of host memory");
    }
    t->totals[0] += rewires;
    t->totals[1] += checks;
    t->totals[2] += nadd;
    t->totals[3] += b.ids.size();
    t->totals[4] += ns;
    t->totals[5] += visits;
    {
        std::lock_guard<std::mutex> lk(t->mu);
        if (t->spare.size() < 2) t->spare.push_back(std::move(b));  // its buffers serve a later stage
    }
    return OMPL_GPU_OK;
}

}  // extern "C"
