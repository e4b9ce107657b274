// NearestNeighborsGPU.h — drop-in MI355X replacement for the reference's default
// nearest-neighbour structure (NearestNeighborsGNAT / GNATNoThreadSafety, selected in
// tools/config/SelfConfig.h:106-117) behind the unchanged ompl::NearestNeighbors<_T>
// interface (datastructures/NearestNeighbors.h:46-115).
//
// Planners default-construct their structure (RRT.h:130-138, RRTstar.h:142-149,
// PRM.h:255-266, informedtrees/bitstar/ImplicitGraph.cpp:1690-1703):
//
//     ompl_amd::setDefaultGpuSpace(space_descriptor);                 // once
//     ompl_amd::setDefaultStatePacker([&](const void *s, double *out) {
//         si->getStateSpace()->copyToReals(v, static_cast<const ompl::base::State *>(s)); ...});
//     planner->setNearestNeighbors<ompl_amd::NearestNeighborsGPU>();
//
// (or, with the one-line SelfConfig patch of INTEGRATION.md, OMPL_AMD_NN=gpu makes it the
// default: SelfConfigGPU.h).
//
// Element -> coordinates: an explicit ElementPacker<_T>, else (SFINAE) `elem->state`
// (RRT/RRT* Motion, RRT.h:160) or `elem->state()` (BIT* Vertex) fed to the default state
// packer.  The metric is the bound space's; no CPU fallback exists — a missing device or packer
// throws.
//
// Semantics kept:
//   * results sorted ascending (ties by insertion order), nearestR inclusive, k == 0 -> empty,
//     k > size -> size results, nearest() on an empty structure throws
//     ompl::Exception("No elements found in nearest neighbors data structure")
//     (NearestNeighborsGNAT.h:218); copies of _T are stored and states are never freed;
//   * one ompl::RNG per instance, constructed with the structure, as the reference GNAT owns
//     one through GreedyKCenters::rng_ (GreedyKCenters.h:127): every RNG() draws a seed from
//     the process-wide generator (RandomNumbers.cpp:218-223), so planners that build their
//     samplers after the NN get the same streams as with the reference structure;
//   * setDistanceFunction (NearestNeighbors.h:58-61) is honoured by verification: the device
//     ranks with the bound space's metric, so after each add() a few (new element, stored
//     element) pairs are measured with the caller's function and with the library's metric
//     (ompl_gpu_nn_distance_host, the reference's formulas on the host) and a disagreement
//     beyond 1e-9 relative throws ompl::Exception instead of silently ranking by another metric.
#pragma once

#include <cmath>
#include <cstdint>
#include <functional>
#include <mutex>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../ompl_gpu.h"
#include "ompl_surface.h"

namespace ompl_amd {

template <typename _T>
using ElementPacker = std::function<void(const _T &, double *)>;
using StatePacker = std::function<void(const void *state, double *out)>;

struct GpuNNDefaults {
    ompl_gpu_space space{};
    int device = 0;
    bool configured = false;
    StatePacker statePacker;
};

inline GpuNNDefaults &gpuDefaults() {
    static GpuNNDefaults d;
    return d;
}
inline void setDefaultGpuSpace(const ompl_gpu_space &s, int device = 0) {
    gpuDefaults().space = s;
    gpuDefaults().device = device;
    gpuDefaults().configured = true;
}
inline void setDefaultStatePacker(StatePacker p) { gpuDefaults().statePacker = std::move(p); }

namespace detail {
template <typename T, typename = void>
struct HasStateMember : std::false_type {};
template <typename T>
struct HasStateMember<T, std::void_t<decltype(std::declval<const T &>()->state)>> : std::true_type {};
template <typename T, typename = void>
struct HasStateCall : std::false_type {};
template <typename T>
struct HasStateCall<T, std::void_t<decltype(std::declval<const T &>()->state())>> : std::true_type {};
template <typename T, typename = void>
struct Hashable : std::false_type {};
template <typename T>
struct Hashable<T, std::void_t<decltype(std::hash<T>{}(std::declval<const T &>()))>> : std::true_type {};

[[noreturn]] inline void raise(ompl_gpu_status st, const char *what) {
    throw ompl::Exception(std::string("NearestNeighborsGPU: ") + what + " failed (status " + std::to_string((int)st) +
                          "): " + ompl_gpu_last_error());
}
inline void check(ompl_gpu_status st, const char *what) {
    if (st != OMPL_GPU_OK) raise(st, what);
}

// id lookup for remove(): hashed when _T is hashable (pointers, integer vertices,
// shared_ptr), else a reverse scan — both pick the latest live insertion of an equal element,
// as NearestNeighborsLinear::remove does (NearestNeighborsLinear.h:90-96)
template <typename _T, bool H = Hashable<_T>::value>
struct IdIndex {
    std::unordered_map<_T, std::vector<std::size_t>> ids;
    void clear() { ids.clear(); }
    void add(const _T &e, std::size_t id) { ids[e].push_back(id); }
    template <class Live>
    bool take(const _T &e, std::size_t &id, const std::vector<_T> &, Live live) {
        auto it = ids.find(e);
        if (it == ids.end()) return false;
        auto &v = it->second;
        while (!v.empty()) {
            const std::size_t i = v.back();
            v.pop_back();
            if (live(i)) {
                id = i;
                if (v.empty()) ids.erase(it);
                return true;
            }
        }
        ids.erase(it);
        return false;
    }
};
template <typename _T>
struct IdIndex<_T, false> {
    void clear() {}
    void add(const _T &, std::size_t) {}
    template <class Live>
    bool take(const _T &e, std::size_t &id, const std::vector<_T> &elems, Live live) {
        for (std::size_t i = elems.size(); i-- > 0;)
            if (live(i) && elems[i] == e) {
                id = i;
                return true;
            }
        return false;
    }
};
}  // namespace detail

template <typename _T>
class NearestNeighborsGPU : public ompl::NearestNeighbors<_T> {
public:
    using typename ompl::NearestNeighbors<_T>::DistanceFunction;

    NearestNeighborsGPU() {
        const GpuNNDefaults &d = gpuDefaults();
        if (!d.configured)
            throw ompl::Exception("NearestNeighborsGPU: call ompl_amd::setDefaultGpuSpace() before planner setup");
        init(d.space, d.device);
    }
    NearestNeighborsGPU(const ompl_gpu_space &space, int device, ElementPacker<_T> packer = nullptr)
      : packer_(std::move(packer)) {
        init(space, device);
    }
    ~NearestNeighborsGPU() override {
        if (h_) ompl_gpu_nn_destroy(h_);
    }
    NearestNeighborsGPU(const NearestNeighborsGPU &) = delete;
    NearestNeighborsGPU &operator=(const NearestNeighborsGPU &) = delete;

    void setElementPacker(ElementPacker<_T> p) { packer_ = std::move(p); }

    // NearestNeighbors.h:58-61: keep the function (getDistanceFunction returns it) and verify
    // it against the device metric on the elements as they arrive
    void setDistanceFunction(const DistanceFunction &distFun) override {
        ompl::NearestNeighbors<_T>::setDistanceFunction(distFun);
        verify_ = static_cast<bool>(distFun);
        if (verify_ && elems_.size() >= 2) verifyPairs(0, elems_.size());
    }
    // verification on / off (on by default once a distance function is set)
    void setVerifyDistance(bool on) { verify_ = on && static_cast<bool>(this->distFun_); }
    std::size_t verifiedPairs() const { return verified_; }

    bool reportsSortedResults() const override { return true; }

    void clear() override {
        detail::check(ompl_gpu_nn_clear(h_), "clear");
        elems_.clear();
        removed_.clear();
        index_.clear();
        live_ = 0;
    }

    void add(const _T &data) override { add(std::vector<_T>(1, data)); }

    void add(const std::vector<_T> &data) override {
        if (data.empty()) return;
        std::vector<double> buf(data.size() * dim_);
        for (std::size_t i = 0; i < data.size(); ++i) pack(data[i], buf.data() + i * dim_);
        detail::check(ompl_gpu_nn_add(h_, buf.data(), data.size(), nullptr), "add");
        const std::size_t first = elems_.size();
        elems_.insert(elems_.end(), data.begin(), data.end());
        removed_.resize(elems_.size(), 0);
        for (std::size_t i = first; i < elems_.size(); ++i) index_.add(elems_[i], i);
        live_ += data.size();
        if (verify_) verifyPairs(first, elems_.size());
    }

    // By value equality of _T, latest insertion first (NearestNeighborsLinear.h:90-96).
    bool remove(const _T &data) override {
        std::size_t i = 0;
        if (!index_.take(data, i, elems_, [this](std::size_t j) { return !removed_[j]; })) return false;
        detail::check(ompl_gpu_nn_remove(h_, i), "remove");
        removed_[i] = 1;
        --live_;
        return true;
    }

    _T nearest(const _T &data) const override {
        if (live_ == 0) throw ompl::Exception("No elements found in nearest neighbors data structure");
        std::vector<double> q(dim_);
        pack(data, q.data());
        uint64_t id = 0;
        double d = 0;
        detail::check(ompl_gpu_nn_nearest(h_, q.data(), 1, &id, &d), "nearest");
        return elems_[id];
    }

    void nearestK(const _T &data, std::size_t k, std::vector<_T> &nbh) const override {
        std::vector<std::vector<_T>> out;
        nearestKBatch(std::vector<_T>(1, data), k, out);
        nbh.swap(out[0]);
    }

    void nearestR(const _T &data, double radius, std::vector<_T> &nbh) const override {
        nbh.clear();
        if (live_ == 0) return;
        std::vector<double> q(dim_);
        pack(data, q.data());
        uint64_t *ids = nullptr;
        double *ds = nullptr;
        uint64_t off[2] = {0, 0};
        detail::check(ompl_gpu_nn_radius(h_, q.data(), 1, radius, &ids, &ds, off), "nearestR");
        nbh.reserve(off[1]);
        for (uint64_t j = off[0]; j < off[1]; ++j) nbh.push_back(elems_[ids[j]]);
        ompl_gpu_free(ids);
        ompl_gpu_free(ds);
    }

    std::size_t size() const override { return live_; }

    void list(std::vector<_T> &data) const override {
        data.clear();
        data.reserve(live_);
        for (std::size_t i = 0; i < elems_.size(); ++i)
            if (!removed_[i]) data.push_back(elems_[i]);
    }

    // Batched extension: one device launch for many queries (what PRM* / BIT* batches use).
    void nearestKBatch(const std::vector<_T> &queries, std::size_t k, std::vector<std::vector<_T>> &out) const {
        out.assign(queries.size(), std::vector<_T>());
        if (k == 0 || live_ == 0 || queries.empty()) return;  // NearestNeighborsGNAT.h:224-232
        const std::size_t nq = queries.size();
        std::vector<double> q(nq * dim_);
        for (std::size_t i = 0; i < nq; ++i) pack(queries[i], q.data() + i * dim_);
        const uint32_t kk = (uint32_t)std::min<std::size_t>(k, live_);
        std::vector<uint64_t> ids(nq * kk);
        std::vector<double> ds(nq * kk);
        std::vector<uint32_t> cnt(nq);
        detail::check(ompl_gpu_nn_knn(h_, q.data(), nq, kk, ids.data(), ds.data(), cnt.data()), "nearestK");
        for (std::size_t i = 0; i < nq; ++i) {
            out[i].reserve(cnt[i]);
            for (uint32_t j = 0; j < cnt[i]; ++j) out[i].push_back(elems_[ids[i * kk + j]]);
        }
    }

    // the instance's RNG (seed-stream alignment with the reference; also picks verify pairs)
    ompl::RNG &rng() { return rng_; }
    ompl_gpu_nn *handle() const { return h_; }

private:
    static constexpr std::size_t kVerifyPerAdd = 4;     // pairs measured per verified add() call
    static constexpr std::size_t kVerifyDense = 4096;   // then only one add() in kVerifyStride
    static constexpr std::size_t kVerifyStride = 256;

    void init(const ompl_gpu_space &space, int device) {
        dim_ = space.dim;
        detail::check(ompl_gpu_nn_create(&h_, &space, device), "create");
    }

    void pack(const _T &e, double *out) const {
        if (packer_) return packer_(e, out);
        const StatePacker &sp = gpuDefaults().statePacker;
        if constexpr (detail::HasStateMember<_T>::value) {
            if (sp) return sp(static_cast<const void *>(e->state), out);
        } else if constexpr (detail::HasStateCall<_T>::value) {
            if (sp) return sp(static_cast<const void *>(e->state()), out);  // bitstar/Vertex.h:89-92
        }
        throw ompl::Exception("NearestNeighborsGPU: no element packer / state packer for this element type");
    }

    // compare the caller's distance function with the device metric on pairs (e, x): e among
    // the elements [first, end) just added, x a random stored element
    void verifyPairs(std::size_t first, std::size_t end) {
        const std::size_t n = elems_.size();
        if (n < 2 || !this->distFun_) return;
        // every add() until kVerifyDense pairs agreed, then one add() in kVerifyStride
        if (verified_ >= kVerifyDense && (++adds_since_ % kVerifyStride) != 0) return;
        const std::size_t m = std::min<std::size_t>(kVerifyPerAdd, end - first);
        std::vector<double> a(m * dim_), b(m * dim_), dev(m);
        std::vector<std::size_t> ia(m), ib(m);
        for (std::size_t j = 0; j < m; ++j) {
            ia[j] = first + (std::size_t)rng_.uniformInt(0, (int)(end - first - 1));
            ib[j] = (std::size_t)rng_.uniformInt(0, (int)(n - 2));  // any other element
            if (ib[j] >= ia[j]) ++ib[j];
            pack(elems_[ia[j]], a.data() + j * dim_);
            pack(elems_[ib[j]], b.data() + j * dim_);
        }
        detail::check(ompl_gpu_nn_distance_host(h_, a.data(), b.data(), m, dev.data()), "distance");
        for (std::size_t j = 0; j < m; ++j) {
            const double user = this->distFun_(elems_[ia[j]], elems_[ib[j]]);
            const double tol = 1e-9 * std::max(1.0, std::fabs(user));
            if (!(std::fabs(user - dev[j]) <= tol))
                throw ompl::Exception("NearestNeighborsGPU: the distance function set with setDistanceFunction gives " +
                                      std::to_string(user) + " where the device metric of the bound state space "
                                      "gives " + std::to_string(dev[j]) +
                                      "; the GPU structure can only rank by the space's own metric");
            ++verified_;
        }
    }

    ompl::RNG rng_;  // one seed drawn per instance (GNAT: GreedyKCenters::rng_)
    ompl_gpu_nn *h_ = nullptr;
    int dim_ = 0;
    ElementPacker<_T> packer_;
    std::vector<_T> elems_;   // id -> element (the reference also stores copies of _T)
    std::vector<char> removed_;
    detail::IdIndex<_T> index_;
    std::size_t live_ = 0;
    bool verify_ = false;
    std::size_t verified_ = 0, adds_since_ = 0;
};

}  // namespace ompl_amd
