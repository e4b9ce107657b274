// gnat.cpp — TEST INFRASTRUCTURE ONLY: CPU restatement of the reference's default
// nearest-neighbour structure, the Geometric Near-neighbor Access Tree (Brin '95) as
// OMPL implements it in src/ompl/datastructures/NearestNeighborsGNAT.h.  Used as
// (a) an exactness cross-check (GNAT kNN == brute force, as the reference test
// tests/datastructures/nearestneighbors.cpp:147-184 requires) and (b) the timed CPU
// baseline on the GPU box, where the reference itself cannot travel.
//
// What is restated (file:line in NearestNeighborsGNAT.h):
//   defaults degree 8 / min 4 / max 12 / 50 points per leaf     :95-114
//   add (descend to nearest child pivot, update ranges)          :147-159, :444-476
//   bulk add (everything in the root, then split)                :160-176
//   split with greedy k-centers (GreedyKCenters.h:82-121)        :493-541
//   nearestK: result max-heap, node min-heap keyed dist-maxRadius,
//             sibling pruning with min/maxRange, queue pruning   :335-356, :565-612, :84-91
//   nearestR: same with fixed radius, inclusive                  :358-376, :622-662
// Differences that do not change results: states are stored contiguously (no
// per-state heap objects, no std::function) which makes this restatement FASTER
// than the reference — a conservative CPU baseline.  Removal is not restated
// (the baselines never remove).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>
#include <queue>
#include <random>
#include <thread>
#include <vector>

#include "oracle.h"

namespace {

struct Node {
    uint32_t degree;
    uint32_t pivot;
    double minRadius = std::numeric_limits<double>::infinity();
    double maxRadius = -std::numeric_limits<double>::infinity();
    std::vector<double> minRange, maxRange;
    std::vector<uint32_t> data;
    std::vector<Node *> kids;

    Node(uint32_t deg, uint32_t cap, uint32_t piv)
        : degree(deg), pivot(piv), minRange(deg, std::numeric_limits<double>::infinity()),
          maxRange(deg, -std::numeric_limits<double>::infinity()) {
        data.reserve(cap + 1);
    }
    ~Node() {
        for (Node *k : kids) delete k;
    }
    void radius(double d) {
        if (minRadius > d) minRadius = d;
        if (maxRadius < d) maxRadius = d;
    }
    void range(unsigned i, double d) {
        if (minRange[i] > d) minRange[i] = d;
        if (maxRange[i] < d) maxRange[i] = d;
    }
};

using Cand = std::pair<double, uint32_t>;  // (distance, id), max-heap by distance
struct NodeEntry {
    Node *node;
    double dist;
};
struct NodeOrder {  // smaller (dist - maxRadius) first — NearestNeighborsGNAT.h:84-91
    bool operator()(const NodeEntry &a, const NodeEntry &b) const {
        return (a.dist - a.node->maxRadius) > (b.dist - b.node->maxRadius);
    }
};

}  // namespace

struct oracle_gnat {
    ompl_gpu_space sp;
    uint32_t degree, minDegree, maxDegree, leafCap;
    std::vector<double> states;  // AoS, id = row
    Node *root = nullptr;
    size_t count = 0;
    std::mt19937_64 rng;

    const double *st(uint32_t id) const { return states.data() + (size_t)id * sp.dim; }
    double dist(uint32_t a, uint32_t b) const { return oracle_distance(&sp, st(a), st(b)); }
    double dist(const double *q, uint32_t b) const { return oracle_distance(&sp, q, st(b)); }

    bool needSplit(const Node *n) const { return n->data.size() > leafCap && n->data.size() > n->degree; }

    // GreedyKCenters::kcenters — GreedyKCenters.h:82-121 (dists is n x k row-major)
    void kcenters(const std::vector<uint32_t> &pts, unsigned k, std::vector<unsigned> &centers,
                  std::vector<double> &dists) {
        const size_t n = pts.size();
        std::vector<double> minDist(n, std::numeric_limits<double>::infinity());
        dists.assign(n * k, 0.0);
        centers.clear();
        centers.push_back((unsigned)std::uniform_int_distribution<size_t>(0, n - 1)(rng));
        for (unsigned i = 1; i < k; ++i) {
            unsigned ind = 0;
            const uint32_t c = pts[centers[i - 1]];
            double maxDist = -std::numeric_limits<double>::infinity();
            for (size_t j = 0; j < n; ++j) {
                double d = dists[j * k + i - 1] = dist(pts[j], c);
                if (d < minDist[j]) minDist[j] = d;
                if (minDist[j] > maxDist) {
                    ind = (unsigned)j;
                    maxDist = minDist[j];
                }
            }
            if (maxDist < std::numeric_limits<double>::epsilon()) break;
            centers.push_back(ind);
        }
        const uint32_t c = pts[centers.back()];
        const unsigned last = (unsigned)centers.size() - 1;
        for (size_t j = 0; j < n; ++j) dists[j * k + last] = dist(pts[j], c);
    }

    // Node::split — NearestNeighborsGNAT.h:493-541
    void split(Node *nd) {
        std::vector<unsigned> piv;
        std::vector<double> dm;
        const unsigned k = nd->degree;
        kcenters(nd->data, k, piv, dm);
        nd->kids.reserve(piv.size());
        for (unsigned p : piv) nd->kids.push_back(new Node(k, leafCap, nd->data[p]));
        nd->degree = (uint32_t)piv.size();
        const unsigned deg = nd->degree;
        for (size_t j = 0; j < nd->data.size(); ++j) {
            unsigned best = 0;
            for (unsigned i = 1; i < deg; ++i)
                if (dm[j * k + i] < dm[j * k + best]) best = i;
            Node *child = nd->kids[best];
            if (j != piv[best]) {
                child->data.push_back(nd->data[j]);
                child->radius(dm[j * k + best]);
            }
            for (unsigned i = 0; i < deg; ++i) nd->kids[i]->range(best, dm[j * k + i]);
        }
        for (Node *c : nd->kids) {
            unsigned d = (unsigned)((deg * c->data.size()) / nd->data.size());
            c->degree = std::min(std::max(d, minDegree), maxDegree);
            if (c->minRadius >= std::numeric_limits<double>::infinity()) c->minRadius = c->maxRadius = 0.;
        }
        std::vector<uint32_t>().swap(nd->data);
        for (Node *c : nd->kids)
            if (needSplit(c)) split(c);
    }

    // Node::add — NearestNeighborsGNAT.h:444-476
    void insert(Node *nd, uint32_t id) {
        while (!nd->kids.empty()) {
            const size_t sz = nd->kids.size();
            double ds[64];
            std::vector<double> big;
            double *d = ds;
            if (sz > 64) { big.resize(sz); d = big.data(); }
            d[0] = dist(id, nd->kids[0]->pivot);
            double mind = d[0];
            unsigned mi = 0;
            for (unsigned i = 1; i < sz; ++i)
                if ((d[i] = dist(id, nd->kids[i]->pivot)) < mind) { mind = d[i]; mi = i; }
            for (unsigned i = 0; i < sz; ++i) nd->kids[i]->range(mi, d[i]);
            nd->kids[mi]->radius(mind);
            nd = nd->kids[mi];
        }
        nd->data.push_back(id);
        ++count;
        if (needSplit(nd)) split(nd);
    }

    static bool pushK(std::vector<Cand> &heap, size_t k, double d, uint32_t id) {  // insertNeighborK :544-558
        if (heap.size() < k) {
            heap.emplace_back(d, id);
            std::push_heap(heap.begin(), heap.end());
            return true;
        }
        if (d < heap.front().first) {
            std::pop_heap(heap.begin(), heap.end());
            heap.back() = {d, id};
            std::push_heap(heap.begin(), heap.end());
            return true;
        }
        return false;
    }

    // Node::nearestK — :565-612
    void visitK(const Node *nd, const double *q, size_t k, std::vector<Cand> &heap,
                std::priority_queue<NodeEntry, std::vector<NodeEntry>, NodeOrder> &nq, size_t &offset) const {
        for (uint32_t id : nd->data) pushK(heap, k, dist(q, id), id);
        if (nd->kids.empty()) return;
        const size_t sz = nd->kids.size(), off = offset++;
        double dp[64];
        int perm[64];
        for (size_t i = 0; i < sz; ++i) perm[i] = (int)((i + off) % sz);
        for (size_t i = 0; i < sz; ++i) {
            if (perm[i] < 0) continue;
            const Node *c = nd->kids[perm[i]];
            dp[perm[i]] = dist(q, c->pivot);
            pushK(heap, k, dp[perm[i]], c->pivot);
            if (heap.size() == k) {
                const double r = heap.front().first;
                for (size_t j = 0; j < sz; ++j)
                    if (perm[j] >= 0 && i != j &&
                        (dp[perm[i]] - r > c->maxRange[perm[j]] || dp[perm[i]] + r < c->minRange[perm[j]]))
                        perm[j] = -1;
            }
        }
        const double r = heap.front().first;
        for (size_t i = 0; i < sz; ++i) {
            int p = perm[i];
            if (p < 0) continue;
            Node *c = nd->kids[p];
            if (heap.size() < k || (dp[p] - r <= c->maxRadius && dp[p] + r >= c->minRadius))
                nq.push({c, dp[p]});
        }
    }

    // nearestKInternal — :335-356 ; postprocessNearest — :379-384
    void knn(const double *q, size_t k, uint32_t *ids, double *ds, uint32_t *cnt, size_t &offset) const {
        std::vector<Cand> heap;
        heap.reserve(k + 1);
        std::priority_queue<NodeEntry, std::vector<NodeEntry>, NodeOrder> nq;
        if (root && k > 0) {
            pushK(heap, k, dist(q, root->pivot), root->pivot);
            visitK(root, q, k, heap, nq, offset);
            while (!nq.empty()) {
                const double r = heap.front().first;
                NodeEntry e = nq.top();
                nq.pop();
                if (heap.size() == k && (e.dist > e.node->maxRadius + r || e.dist < e.node->minRadius - r)) continue;
                visitK(e.node, q, k, heap, nq, offset);
            }
        }
        std::sort_heap(heap.begin(), heap.end());
        for (size_t j = 0; j < heap.size(); ++j) { ids[j] = heap[j].second; ds[j] = heap[j].first; }
        for (size_t j = heap.size(); j < k; ++j) { ids[j] = 0xFFFFFFFFu; ds[j] = std::numeric_limits<double>::infinity(); }
        *cnt = (uint32_t)heap.size();
    }

    // Node::nearestR — :622-662 ; nearestRInternal — :358-376.  hit(d, id) is called for every
    // element with d <= r (inclusive), in traversal order.
    template <class Hit>
    void radiusVisit(const double *q, double r, size_t &offset, Hit &&hit) const {
        if (!root) return;
        std::priority_queue<NodeEntry, std::vector<NodeEntry>, NodeOrder> nq;
        const double d0 = dist(q, root->pivot);
        if (d0 <= r) hit(d0, root->pivot);
        auto visit = [&](const Node *nd) {
            for (uint32_t id : nd->data) {
                const double d = dist(q, id);
                if (d <= r) hit(d, id);
            }
            if (nd->kids.empty()) return;
            const size_t sz = nd->kids.size(), off = offset++;
            double dp[64];
            int perm[64];
            for (size_t i = 0; i < sz; ++i) perm[i] = (int)((i + off) % sz);
            for (size_t i = 0; i < sz; ++i) {
                if (perm[i] < 0) continue;
                const Node *c = nd->kids[perm[i]];
                dp[perm[i]] = dist(q, c->pivot);
                if (dp[perm[i]] <= r) hit(dp[perm[i]], c->pivot);
                for (size_t j = 0; j < sz; ++j)
                    if (perm[j] >= 0 && i != j &&
                        (dp[perm[i]] - r > c->maxRange[perm[j]] || dp[perm[i]] + r < c->minRange[perm[j]]))
                        perm[j] = -1;
            }
            for (size_t i = 0; i < sz; ++i) {
                int p = perm[i];
                if (p < 0) continue;
                Node *c = nd->kids[p];
                if (dp[p] - r <= c->maxRadius && dp[p] + r >= c->minRadius) nq.push({c, dp[p]});
            }
        };
        visit(root);
        while (!nq.empty()) {
            NodeEntry e = nq.top();
            nq.pop();
            if (e.dist > e.node->maxRadius + r || e.dist < e.node->minRadius - r) continue;
            visit(e.node);
        }
    }

    uint64_t radiusCount(const double *q, double r, size_t &offset) const {
        uint64_t hits = 0;
        radiusVisit(q, r, offset, [&](double, uint32_t) { ++hits; });
        return hits;
    }

    // nearestR's result list: sorted ascending (postprocessNearest, :379-384), ties by id
    void radius(const double *q, double r, size_t &offset, std::vector<Cand> &out) const {
        out.clear();
        radiusVisit(q, r, offset, [&](double d, uint32_t id) { out.emplace_back(d, id); });
        std::sort(out.begin(), out.end());
    }

    std::vector<std::vector<Cand>> radiusResults;  // oracle_gnat_radius -> oracle_gnat_radius_fetch
};

extern "C" {

oracle_gnat *oracle_gnat_create(const ompl_gpu_space *sp, uint32_t degree, uint32_t min_degree,
                                uint32_t max_degree, uint32_t max_pts_per_leaf, uint64_t seed) {
    auto *g = new oracle_gnat();
    g->sp = *sp;
    g->degree = degree;
    g->minDegree = std::min(degree, min_degree);
    g->maxDegree = std::max(max_degree, degree);
    g->leafCap = max_pts_per_leaf;
    g->rng.seed(seed);
    return g;
}

void oracle_gnat_destroy(oracle_gnat *g) {
    delete g->root;
    delete g;
}

size_t oracle_gnat_size(const oracle_gnat *g) { return g->count; }

// add(data) one at a time — NearestNeighborsGNAT.h:147-159
void oracle_gnat_add(oracle_gnat *g, const double *s, size_t n) {
    const size_t base = g->states.size() / g->sp.dim;
    g->states.insert(g->states.end(), s, s + n * g->sp.dim);
    for (size_t i = 0; i < n; ++i) {
        uint32_t id = (uint32_t)(base + i);
        if (!g->root) {
            g->root = new Node(g->degree, g->leafCap, id);
            g->count = 1;
        } else {
            g->insert(g->root, id);
        }
    }
}

// add(vector) into an empty tree — NearestNeighborsGNAT.h:160-176
void oracle_gnat_add_bulk(oracle_gnat *g, const double *s, size_t n) {
    if (g->root || n == 0) {
        oracle_gnat_add(g, s, n);
        return;
    }
    g->states.insert(g->states.end(), s, s + n * g->sp.dim);
    g->root = new Node(g->degree, g->leafCap, 0);
    g->root->data.reserve(n);
    for (size_t i = 1; i < n; ++i) g->root->data.push_back((uint32_t)i);
    g->count = n;
    if (g->needSplit(g->root)) g->split(g->root);
}

void oracle_gnat_knn(const oracle_gnat *g, const double *q, size_t nq, uint32_t k, uint32_t *ids, double *dists,
                     uint32_t *counts, int nthreads) {
    auto work = [=](size_t b, size_t e) {
        size_t offset = 0;
        for (size_t i = b; i < e; ++i)
            g->knn(q + i * g->sp.dim, k, ids + i * k, dists + i * k, counts + i, offset);
    };
    if (nthreads <= 1) {
        work(0, nq);
        return;
    }
    std::vector<std::thread> th;
    const size_t per = (nq + nthreads - 1) / nthreads;
    for (int t = 0; t < nthreads; ++t) {
        size_t b = t * per, e = std::min(nq, b + per);
        if (b < e) th.emplace_back(work, b, e);
    }
    for (auto &t : th) t.join();
}

uint64_t oracle_gnat_radius_count(const oracle_gnat *g, const double *q, size_t nq, double r, uint64_t *counts,
                                  int nthreads) {
    std::vector<uint64_t> part(std::max(1, nthreads), 0);
    auto work = [=, &part](int t, size_t b, size_t e) {
        size_t offset = 0;
        for (size_t i = b; i < e; ++i) {
            uint64_t c = g->radiusCount(q + i * g->sp.dim, r, offset);
            if (counts) counts[i] = c;
            part[t] += c;
        }
    };
    if (nthreads <= 1) {
        work(0, 0, nq);
    } else {
        std::vector<std::thread> th;
        const size_t per = (nq + nthreads - 1) / nthreads;
        for (int t = 0; t < nthreads; ++t) {
            size_t b = t * per, e = std::min(nq, b + per);
            if (b < e) th.emplace_back(work, t, b, e);
        }
        for (auto &t : th) t.join();
    }
    uint64_t tot = 0;
    for (uint64_t v : part) tot += v;
    return tot;
}

// nearestR with the results: offsets[nq + 1] (CSR), returns the total; the ids / distances are
// kept in the handle until oracle_gnat_radius_fetch copies them out (sorted by (distance, id))
uint64_t oracle_gnat_radius(oracle_gnat *g, const double *q, size_t nq, double r, uint64_t *offsets, int nthreads) {
    g->radiusResults.assign(nq, {});
    auto work = [=](size_t b, size_t e) {
        size_t offset = 0;
        for (size_t i = b; i < e; ++i) g->radius(q + i * g->sp.dim, r, offset, g->radiusResults[i]);
    };
    if (nthreads <= 1) {
        work(0, nq);
    } else {
        std::vector<std::thread> th;
        const size_t per = (nq + nthreads - 1) / nthreads;
        for (int t = 0; t < nthreads; ++t) {
            size_t b = t * per, e = std::min(nq, b + per);
            if (b < e) th.emplace_back(work, b, e);
        }
        for (auto &t : th) t.join();
    }
    offsets[0] = 0;
    for (size_t i = 0; i < nq; ++i) offsets[i + 1] = offsets[i] + g->radiusResults[i].size();
    return offsets[nq];
}

void oracle_gnat_radius_fetch(oracle_gnat *g, uint32_t *ids, double *dists) {
    size_t at = 0;
    for (auto &v : g->radiusResults) {
        for (const Cand &c : v) {
            ids[at] = c.second;
            dists[at] = c.first;
            ++at;
        }
    }
    std::vector<std::vector<Cand>>().swap(g->radiusResults);
}

}  // extern "C"
