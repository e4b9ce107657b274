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
// Element -> coordinates: an explicit ElementPacker<_T>, else (SFINAE) `elem->state`
// (RRT/RRT* Motion, RRT.h:160) or `elem->state()` (BIT* Vertex) fed to the default state
// packer.  The metric is the bound space's (the planners' distance function is always
// si_->distance, RRT.cpp:79); no CPU fallback exists — a missing device or packer throws.
//
// Semantics kept: results sorted ascending (ties by insertion order), nearestR inclusive,
// k == 0 -> empty, k > size -> size results, nearest() on an empty structure throws
// ompl::Exception("No elements found in nearest neighbors data structure")
// (NearestNeighborsGNAT.h:218).  Like the reference, the structure stores copies of _T and
// never frees states.
#pragma once

#include <cstdint>
#include <functional>
#include <mutex>
#include <string>
#include <type_traits>
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

[[noreturn]] inline void raise(ompl_gpu_status st, const char *what) {
    throw ompl::Exception(std::string("NearestNeighborsGPU: ") + what + " failed (status " + std::to_string((int)st) +
                          "): " + ompl_gpu_last_error());
}
inline void check(ompl_gpu_status st, const char *what) {
    if (st != OMPL_GPU_OK) raise(st, what);
}
}  // namespace detail

template <typename _T>
class NearestNeighborsGPU : public ompl::NearestNeighbors<_T> {
public:
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

    bool reportsSortedResults() const override { return true; }

    void clear() override {
        detail::check(ompl_gpu_nn_clear(h_), "clear");
        elems_.clear();
        removed_.clear();
        live_ = 0;
    }

    void add(const _T &data) override { add(std::vector<_T>(1, data)); }

    void add(const std::vector<_T> &data) override {
        if (data.empty()) return;
        std::vector<double> buf(data.size() * dim_);
        for (std::size_t i = 0; i < data.size(); ++i) pack(data[i], buf.data() + i * dim_);
        detail::check(ompl_gpu_nn_add(h_, buf.data(), data.size(), nullptr), "add");
        elems_.insert(elems_.end(), data.begin(), data.end());
        removed_.resize(elems_.size(), 0);
        live_ += data.size();
    }

    // By value equality of _T, latest insertion first (NearestNeighborsLinear.h:90-96).
    bool remove(const _T &data) override {
        for (std::size_t i = elems_.size(); i-- > 0;)
            if (!removed_[i] && elems_[i] == data) {
                detail::check(ompl_gpu_nn_remove(h_, i), "remove");
                removed_[i] = 1;
                --live_;
                return true;
            }
        return false;
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

private:
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

    ompl_gpu_nn *h_ = nullptr;
    int dim_ = 0;
    ElementPacker<_T> packer_;
    std::vector<_T> elems_;   // id -> element (the reference also stores copies of _T)
    std::vector<char> removed_;
    std::size_t live_ = 0;
};

}  // namespace ompl_amd
