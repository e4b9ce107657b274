// capi.hip — implementation of the C ABI declared in include/ompl_gpu.h.
//
// Device data layout (HBM):
//   feat : SoA [F][cap] fp64 feature rows of the stored states (kernels.h FeatGeom),
//          cap a multiple of kTile; unused / removed slots hold NaN so the kernels
//          never need bounds or liveness checks (a NaN distance is never selected).
//   raw  : SoA [dim][cap] raw states for KCHAIN (for the other spaces raw == feat).
// Ids are insertion indices, as the reference NN stores copies of _T in insertion
// order (NearestNeighborsLinear.h:78-88); the C++ wrapper maps id <-> _T.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "../../include/ompl_gpu.h"
#include "kernels.h"
#include "rrtstar_tree.h"
#include "sampler_impl.h"
#include "topk.h"

using namespace ompl_amd;

namespace {

thread_local std::string g_last_error;

ompl_gpu_status fail(ompl_gpu_status s, const std::string &msg) {
    g_last_error = msg;
    return s;
}

#define HIP_OR_FAIL(expr)                                                                              \
    do {                                                                                               \
        hipError_t _e = (expr);                                                                        \
        if (_e != hipSuccess) {                                                                        \
            return fail(_e == hipErrorOutOfMemory ? OMPL_GPU_ERR_OOM : OMPL_GPU_ERR_DEVICE,            \
                        std::string(#expr) + ": " + hipGetErrorString(_e));                            \
        }                                                                                              \
    } while (0)

bool space_ok(const ompl_gpu_space *s, DevSpace *d, FeatGeom *g) {
    if (!s) return false;
    d->kind = s->kind;
    d->dim = s->dim;
    d->w0 = s->weight[0];
    d->w1 = s->weight[1];
    d->lvs0 = s->lvs[0];
    d->lvs1 = s->lvs[1];
    d->f0 = s->factor[0] ? s->factor[0] : 1;
    d->f1 = s->factor[1] ? s->factor[1] : 1;
    d->link = s->link_length;
    if (d->dim > kChainMaxLinks) return false;
    return feature_geometry(*d, g);
}

// grow-only device buffer
struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t b) {
        if (b <= bytes) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        size_t nb = std::max(b, (size_t)4096);
        hipError_t e = hipMalloc(&p, nb);
        if (e == hipSuccess) bytes = nb;
        return e;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

int cu_count(int device) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return 256;
    return prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
}

}  // namespace

struct ompl_gpu_nn {
    int device = 0;
    int num_cus = 256;
    hipStream_t own = nullptr, stream = nullptr;
    DevSpace sp{};
    FeatGeom g{};
    double *feat = nullptr;  // [F][cap]
    double *raw = nullptr;   // [dim][cap] (KCHAIN) or == feat
    float *feat32 = nullptr; // [rows32][cap] fp32 copy for the screening scan (knn_fast.hip)
    uint8_t *live = nullptr; // [cap] 1 = stored and not removed (the device k-d build's input)
    int rows32 = 0;
    uint64_t cap = 0, n_total = 0, n_live = 0;
    std::vector<uint8_t> removed;
    std::mutex mu;
    DevBuf q, out_d, out_i, ws, ws2, stage, counts, offsets, qoff, ids, dists, sorted_ids, sorted_d, tmp, fb_q, fb_d,
        fb_i, fb_c, fb_cd, fb_ci, slab_i, slab_d;
    uint32_t radius_slab = 64;      // per-query slab of the one-pass radius walk (adapts upward)
    uint64_t radius_one_pass = 0;   // radius calls answered by the one-pass walk
    uint64_t radius_two_pass = 0;   // radius calls whose longest segment overflowed the slab
    DevBuf rrt_n, rrt_pd, rrt_pi;  // device RRT growth: live size + barrier words, per-block partial minima
    int rrt_coop = -1;             // persistent RRT grid size (0: two-launch form), found on first use
    int rrt_abort_streak = 0;      // consecutive aborted persistent grids (a device kept busy by others)
    int rrt_latched = 0;           // two-launch batches since the streak latched (retry after kRrtRetryAfter)
    bool rrt_spin_read = false;    // OMPL_GPU_RRT_SPIN_LIMIT read (tests)
    uint64_t rrt_spin_override = 0;
    void *rrt_sync = nullptr;      // its uncached synchronisation record
    DevBuf rrt_goal;               // goal record + goal reals of ompl_gpu_rrt_solve_device
    DevBuf rrt_save;               // motion-validator counters before a persistent run (restored on abort)
    uint64_t rrt_aborts = 0;       // persistent runs that aborted and re-ran in the two-launch form
    DevBuf prm_bf, prm_raw, prm_kj, prm_sd, prm_si, prm_len, prm_off, prm_eoff, prm_cnt64;  // PRM* batches
    DevBuf prm_p32;                                                                         // chain positions
    struct {  // RRT* iteration batches (ompl_gpu_rrtstar_batch_device)
        DevBuf near_i, near_d, src, xa, xb, from, inc, va, vb, rank, list, chg, xc, bf, kj, sd, si, len, off, cd, ci,
            scnt, ocnt, ooff, oi, od, oseg, fwd, bwd, bits, soff, scan, p32, sorti, sortd, ovf;
    } rs;
    std::vector<double> hfeat;
    // screening bounds: box of the first three coordinates and max |coordinate|
    double lo[kKeyDims] = {0}, hi[kKeyDims] = {0}, absmax = 0.0;
    double qeta = 0.0;  // SE3: largest |norm^2 - 1| of the stored quaternions (fp32 screen error bound)
    // k-d sorted fp32 copy for the culled walks: built on the device, states added later go to
    // its Morton-ordered tail, removals are tombstoned in place (kernels.h SortedStore)
    SortedStore sorted;
    DevBuf raw_aos;         // [n_total][da] fp64 raw states by id (edge endpoints), appended lazily
    DevBuf large_counter;   // large-k select: queries that spilled to the pool, queries re-run exactly
    DevBuf edge_q;          // per-edge CSR segment (query) of ompl_gpu_nn_edges_device
    uint64_t aos_n = 0;     // ids [0, aos_n) converted
    uint64_t sorted_builds = 0, sorted_appends = 0;  // device k-d builds / tail appends
    bool cull = true;         // ompl_gpu_nn_set_exact(h, 2) disables the culled screen
    DevBuf cull_counter;      // SortedStore::counters: kNN walk [tiles fetched, tiles of a brute-force
                              // walk, (tile, query) pairs scanned], radius walk [tiles, pairs] (device)
    bool fast = true;        // OMPL_GPU_EXACT_ONLY=1 forces the exact fp64 scan
    uint64_t fast_queries = 0;
    DevBuf stats_dev;         // device counters: [0] queries re-run exactly, [1] of those, full scans
    bool stats_init = false;
    // profiling of the dominant scan kernel (HIP events on the launch stream)
    bool profile = false;
    std::vector<KernelTimer> pending;
    double prof_ms = 0.0;
    uint64_t prof_launches = 0;
    std::string prof_name;
};

namespace ompl_amd {
thread_local KernelTimer *g_kernel_timer = nullptr;
void set_last_error(const char *msg) { g_last_error = msg; }  // sampler.cpp
}

namespace {
// coordinates whose running box the handle tracks: SE3 translation, R^n first <= 6
int tracked_dims(const DevSpace &sp) {
    if (sp.kind == OMPL_GPU_SPACE_SE3) return 3;
    if (sp.kind == OMPL_GPU_SPACE_REALVECTOR) return std::min(sp.dim, kKeyDims);
    return 0;
}

// Morton key box: the tracked coordinates, plus for SE3 the vector part of the
// sign-canonical quaternion, which lies in [-1, 1]
FastBounds current_bounds(const ompl_gpu_nn *h) {
    FastBounds b{};
    const int nt = tracked_dims(h->sp);
    b.nkey = h->sp.kind == OMPL_GPU_SPACE_SE3 ? 6 : nt;
    for (int c = 0; c < nt; ++c) {
        b.lo[c] = (float)h->lo[c];
        const double ext = h->hi[c] - h->lo[c];
        b.inv[c] = ext > 0 ? (float)(1.0 / ext) : 0.f;
    }
    for (int c = nt; c < b.nkey; ++c) {
        b.lo[c] = -1.f;
        b.inv[c] = 0.5f;
    }
    b.absmax = (float)h->absmax;
    b.qeta = (float)h->qeta * 1.01f;
    return b;
}
// arms g_kernel_timer for the scope of one query call when the handle profiles
struct ProfileScope {
    ompl_gpu_nn *h;
    KernelTimer t;
    bool armed = false;
    explicit ProfileScope(ompl_gpu_nn *hh) : h(hh) {
        if (!h->profile) return;
        if (hipEventCreate(&t.begin) != hipSuccess) return;
        if (hipEventCreate(&t.end) != hipSuccess) {
            (void)hipEventDestroy(t.begin);
            return;
        }
        armed = true;
        g_kernel_timer = &t;
    }
    ~ProfileScope() {
        if (!armed) return;
        g_kernel_timer = nullptr;
        h->pending.push_back(t);
    }
};
}  // namespace

struct ompl_gpu_mv {
    int device = 0;
    hipStream_t own = nullptr, stream = nullptr;
    DevSpace sp{};
    FeatGeom g{};
    DevChecker ck{};
    double *ck_data = nullptr;
    std::vector<double> ck_host;  // host copy of the checker data (ompl_gpu_svc_check_host)
    unsigned long long *counters = nullptr;  // valid, invalid, isValid calls
    std::mutex mu;
    DevBuf s1, s2, valid, nd, fi, ms;
    DevBuf edge_q;  // per-edge CSR segment (query) of ompl_gpu_mv_check_edges_device, written on this stream
};

extern "C" {

int ompl_gpu_abi_version(void) { return OMPL_GPU_ABI_VERSION; }

const char *ompl_gpu_last_error(void) { return g_last_error.c_str(); }

ompl_gpu_status ompl_gpu_device_count(int *count) {
    if (!count) return fail(OMPL_GPU_ERR_INVALID_ARG, "count is NULL");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    *count = e == hipSuccess ? c : 0;
    return e == hipSuccess ? OMPL_GPU_OK : fail(OMPL_GPU_ERR_DEVICE, hipGetErrorString(e));
}

void ompl_gpu_free(void *p) { std::free(p); }

// ------------------------------------------------------------------------------ NN

ompl_gpu_status ompl_gpu_nn_create(ompl_gpu_nn **out, const ompl_gpu_space *space, int device) {
    if (!out) return fail(OMPL_GPU_ERR_INVALID_ARG, "out is NULL");
    *out = nullptr;
    DevSpace sp;
    FeatGeom g;
    if (!space_ok(space, &sp, &g)) return fail(OMPL_GPU_ERR_UNSUPPORTED, "unsupported state space");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
        return fail(OMPL_GPU_ERR_DEVICE, "no such HIP device");
    HIP_OR_FAIL(hipSetDevice(device));
    auto *h = new ompl_gpu_nn();
    h->device = device;
    h->num_cus = cu_count(device);
    h->sp = sp;
    h->g = g;
    h->rows32 = fp32_rows(sp, g);
    h->fast = true;  // ompl_gpu_nn_set_exact_only(h, 1): the fp64 kernels only
    hipError_t e = hipStreamCreateWithFlags(&h->own, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete h;
        return fail(OMPL_GPU_ERR_DEVICE, hipGetErrorString(e));
    }
    h->stream = h->own;
    *out = h;
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_nn_destroy(ompl_gpu_nn *h) {
    if (!h) return OMPL_GPU_OK;
    (void)hipSetDevice(h->device);
    (void)hipStreamSynchronize(h->stream);
    if (h->raw && h->raw != h->feat) (void)hipFree(h->raw);
    if (h->feat) (void)hipFree(h->feat);
    if (h->feat32) (void)hipFree(h->feat32);
    if (h->live) (void)hipFree(h->live);
    if (h->rrt_sync) (void)hipFree(h->rrt_sync);
    free_sorted_store(&h->sorted);
    if (h->own) (void)hipStreamDestroy(h->own);
    delete h;
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_nn_set_stream(ompl_gpu_nn *h, void *s) {
    if (!h) return fail(OMPL_GPU_ERR_INVALID_ARG, "handle is NULL");
    std::lock_guard<std::mutex> lk(h->mu);
    h->stream = s ? (hipStream_t)s : h->own;
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_nn_sync(ompl_gpu_nn *h) {
    if (!h) return fail(OMPL_GPU_ERR_INVALID_ARG, "handle is NULL");
    HIP_OR_FAIL(hipSetDevice(h->device));
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    return OMPL_GPU_OK;
}

static ompl_gpu_status grow(ompl_gpu_nn *h, uint64_t need) {
    if (need <= h->cap) return OMPL_GPU_OK;
    uint64_t nc = std::max<uint64_t>(h->cap * 2, need);
    nc = std::max<uint64_t>(nc, 4096);
    nc = (nc + kTile - 1) / kTile * kTile;
    const int F = h->g.F;
    const bool sep_raw = h->sp.kind == OMPL_GPU_SPACE_KCHAIN;
    double *nf = nullptr, *nr = nullptr;
    float *n32 = nullptr;
    if (h->rows32) {
        HIP_OR_FAIL(hipMalloc(&n32, sizeof(float) * h->rows32 * nc));
        HIP_OR_FAIL(hipMemsetAsync(n32, 0xFF, sizeof(float) * h->rows32 * nc, h->stream));  // NaN
        if (h->n_total)
            HIP_OR_FAIL(hipMemcpy2DAsync(n32, nc * sizeof(float), h->feat32, h->cap * sizeof(float),
                                         h->n_total * sizeof(float), h->rows32, hipMemcpyDeviceToDevice, h->stream));
    }
    uint8_t *nl = nullptr;
    HIP_OR_FAIL(hipMalloc(&nl, nc));
    HIP_OR_FAIL(hipMemsetAsync(nl, 0, nc, h->stream));
    if (h->n_total) HIP_OR_FAIL(hipMemcpyAsync(nl, h->live, h->n_total, hipMemcpyDeviceToDevice, h->stream));
    HIP_OR_FAIL(hipMalloc(&nf, sizeof(double) * F * nc));
    HIP_OR_FAIL(hipMemsetAsync(nf, 0xFF, sizeof(double) * F * nc, h->stream));  // all-ones = NaN
    if (sep_raw) {
        HIP_OR_FAIL(hipMalloc(&nr, sizeof(double) * h->sp.dim * nc));
        HIP_OR_FAIL(hipMemsetAsync(nr, 0xFF, sizeof(double) * h->sp.dim * nc, h->stream));
    }
    if (h->n_total) {
        HIP_OR_FAIL(hipMemcpy2DAsync(nf, nc * sizeof(double), h->feat, h->cap * sizeof(double),
                                     h->n_total * sizeof(double), F, hipMemcpyDeviceToDevice, h->stream));
        if (sep_raw)
            HIP_OR_FAIL(hipMemcpy2DAsync(nr, nc * sizeof(double), h->raw, h->cap * sizeof(double),
                                         h->n_total * sizeof(double), h->sp.dim, hipMemcpyDeviceToDevice,
                                         h->stream));
    }
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    if (h->raw && h->raw != h->feat) (void)hipFree(h->raw);
    if (h->feat) (void)hipFree(h->feat);
    if (h->feat32) (void)hipFree(h->feat32);
    if (h->live) (void)hipFree(h->live);
    h->live = nl;
    h->feat = nf;
    h->feat32 = n32;
    h->raw = sep_raw ? nr : nf;
    h->cap = nc;
    return OMPL_GPU_OK;
}

static ompl_gpu_status add_locked(ompl_gpu_nn *h, const double *states, size_t n, uint64_t *first_id,
                                  const double *d_feat = nullptr, const double *d_raw = nullptr);

// feature rows of n AoS states (host_features: glibc libm, bit-identical to the reference),
// split over host threads for large batches: 8,192 chain states cost ~3 ms on one core, all of
// it GPU idle time at the head of a PRM* batch
static void host_features_batch(const DevSpace &sp, const FeatGeom &g, const double *states, size_t n, double *out) {
    const size_t per_thread = 512;
    const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const size_t T = std::min<size_t>(hw, (n + per_thread - 1) / per_thread);
    auto work = [&](size_t a, size_t b) {
        for (size_t i = a; i < b; ++i) host_features(sp, g, states + i * sp.dim, out + i * g.F);
    };
    if (T <= 1) {
        work(0, n);
        return;
    }
    std::vector<std::thread> pool;
    pool.reserve(T - 1);
    const size_t chunk = (n + T - 1) / T;
    size_t done = chunk;  // rows [0, done) are covered by this thread and the started ones
    try {
        for (size_t t = 1; t < T; ++t) {
            pool.emplace_back(work, std::min(n, t * chunk), std::min(n, (t + 1) * chunk));
            done = std::min(n, (t + 1) * chunk);
        }
    } catch (const std::system_error &) {  // no thread to be had: this one does the rest
    }
    work(0, std::min(n, chunk));
    work(done, n);
    for (std::thread &th : pool) th.join();
}

ompl_gpu_status ompl_gpu_nn_add(ompl_gpu_nn *h, const double *states, size_t n, uint64_t *first_id) {
    if (!h || (n && !states)) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    std::lock_guard<std::mutex> lk(h->mu);
    return add_locked(h, states, n, first_id);
}

// append n AoS states (caller holds the lock); d_feat / d_raw: the states' feature rows and raw
// rows already on the device (AoS, a PRM* batch's), else computed and uploaded here
static ompl_gpu_status add_locked(ompl_gpu_nn *h, const double *states, size_t n, uint64_t *first_id,
                                  const double *d_feat, const double *d_raw) {
    HIP_OR_FAIL(hipSetDevice(h->device));
    if (first_id) *first_id = h->n_total;
    if (n == 0) return OMPL_GPU_OK;
    if (h->n_total + n > 0xFFFFFFF0ull) return fail(OMPL_GPU_ERR_UNSUPPORTED, "more than 2^32-16 states");
    ompl_gpu_status s = grow(h, h->n_total + n);
    if (s != OMPL_GPU_OK) return s;
    const int F = h->g.F, dim = h->sp.dim;
    const bool sep_raw = h->raw != h->feat;
    if (!d_feat || (sep_raw && !d_raw)) {
        h->hfeat.resize((size_t)n * F);
        host_features_batch(h->sp, h->g, states, n, h->hfeat.data());
        const size_t stage_bytes = sizeof(double) * n * (F + (sep_raw ? dim : 0));
        HIP_OR_FAIL(h->stage.ensure(stage_bytes));
        double *sf = (double *)h->stage.p;
        HIP_OR_FAIL(hipMemcpyAsync(sf, h->hfeat.data(), sizeof(double) * n * F, hipMemcpyHostToDevice, h->stream));
        d_feat = sf;
        if (sep_raw) {
            double *sr = sf + n * F;
            HIP_OR_FAIL(hipMemcpyAsync(sr, states, sizeof(double) * n * dim, hipMemcpyHostToDevice, h->stream));
            d_raw = sr;
        }
    }
    HIP_OR_FAIL(launch_store_soa(d_feat, (uint32_t)n, F, h->feat, h->cap, h->n_total, h->stream));
    if (sep_raw) HIP_OR_FAIL(launch_store_soa(d_raw, (uint32_t)n, dim, h->raw, h->cap, h->n_total, h->stream));
    if (h->rows32) HIP_OR_FAIL(launch_rows32(h->sp, h->g, h->feat, h->cap, h->n_total, n, h->feat32, h->stream));
    HIP_OR_FAIL(hipMemsetAsync(h->live + h->n_total, 1, n, h->stream));
    // screening bounds (knn_fast.hip): key box of the first <= 6 coordinates, max |coordinate|;
    // the sorted copy picks the new ids up in its tail at the next query (ensure_sorted)
    const int nb = tracked_dims(h->sp);
    const int na = h->sp.kind == OMPL_GPU_SPACE_SE3 ? 3 : (h->sp.kind == OMPL_GPU_SPACE_SO3 ? 0 : dim);
    for (size_t i = 0; i < n; ++i) {
        const double *s = states + i * dim;
        for (int c = 0; c < nb; ++c) {
            if (h->n_total == 0 && i == 0) h->lo[c] = h->hi[c] = s[c];
            h->lo[c] = std::min(h->lo[c], s[c]);
            h->hi[c] = std::max(h->hi[c], s[c]);
        }
        for (int c = 0; c < na; ++c) h->absmax = std::max(h->absmax, std::fabs(s[c]));
        if (h->sp.kind == OMPL_GPU_SPACE_SE3) {
            const double n2 = s[3] * s[3] + s[4] * s[4] + s[5] * s[5] + s[6] * s[6];
            const double eta = std::fabs(n2 - 1.0);
            h->qeta = (eta == eta) ? std::max(h->qeta, eta) : 1.0;  // NaN: no fp32 screen
        }
    }
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));  // host staging buffers are reused
    h->n_total += n;
    h->n_live += n;
    h->removed.resize(h->n_total, 0);
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_nn_remove(ompl_gpu_nn *h, uint64_t id) {
    if (!h) return fail(OMPL_GPU_ERR_INVALID_ARG, "handle is NULL");
    std::lock_guard<std::mutex> lk(h->mu);
    if (id >= h->n_total || h->removed[id]) return fail(OMPL_GPU_ERR_NOT_FOUND, "id not stored");
    HIP_OR_FAIL(hipSetDevice(h->device));
    // tombstone: a NaN in feature row 0 makes every distance to this state NaN
    const double nan = __builtin_nan("");
    HIP_OR_FAIL(hipMemcpyAsync(h->feat + id, &nan, sizeof(double), hipMemcpyHostToDevice, h->stream));
    const float nanf = __builtin_nanf("");
    if (h->rows32)
        HIP_OR_FAIL(hipMemcpyAsync(h->feat32 + id, &nanf, sizeof(float), hipMemcpyHostToDevice, h->stream));
    HIP_OR_FAIL(hipMemsetAsync(h->live + id, 0, 1, h->stream));
    HIP_OR_FAIL(tombstone_sorted_store(&h->sorted, id, h->stream));  // the sorted copy, in place
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));                     // the host NaNs are stack values
    h->removed[id] = 1;
    h->n_live--;
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_nn_clear(ompl_gpu_nn *h) {
    if (!h) return fail(OMPL_GPU_ERR_INVALID_ARG, "handle is NULL");
    std::lock_guard<std::mutex> lk(h->mu);
    HIP_OR_FAIL(hipSetDevice(h->device));
    if (h->cap) {
        HIP_OR_FAIL(hipMemsetAsync(h->feat, 0xFF, sizeof(double) * h->g.F * h->cap, h->stream));
        if (h->raw != h->feat)
            HIP_OR_FAIL(hipMemsetAsync(h->raw, 0xFF, sizeof(double) * h->sp.dim * h->cap, h->stream));
        if (h->rows32) HIP_OR_FAIL(hipMemsetAsync(h->feat32, 0xFF, sizeof(float) * h->rows32 * h->cap, h->stream));
        HIP_OR_FAIL(hipMemsetAsync(h->live, 0, h->cap, h->stream));
        HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    }
    h->n_total = h->n_live = 0;
    h->absmax = 0.0;
    h->qeta = 0.0;
    h->sorted.built = false;  // keeps its allocations
    h->aos_n = 0;
    h->removed.clear();
    h->rrt_abort_streak = h->rrt_latched = 0;
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_nn_size(const ompl_gpu_nn *h, size_t *live, size_t *total) {
    if (!h) return fail(OMPL_GPU_ERR_INVALID_ARG, "handle is NULL");
    if (live) *live = h->n_live;
    if (total) *total = h->n_total;
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_nn_distance_host(const ompl_gpu_nn *h, const double *a, const double *b, size_t m,
                                          double *out) {
    if (!h || (m && (!a || !b || !out))) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    const int dim = h->sp.dim;
    for (size_t i = 0; i < m; ++i) out[i] = raw_distance(h->sp, a + i * dim, b + i * dim);
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_nn_get_states(ompl_gpu_nn *h, uint64_t first, size_t n, double *out) {
    if (!h || (n && !out)) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    std::lock_guard<std::mutex> lk(h->mu);
    if (first + n > h->n_total) return fail(OMPL_GPU_ERR_INVALID_ARG, "range beyond stored states");
    if (n == 0) return OMPL_GPU_OK;
    HIP_OR_FAIL(hipSetDevice(h->device));
    const int dim = h->sp.dim;
    std::vector<double> soa((size_t)dim * n);
    HIP_OR_FAIL(hipMemcpy2DAsync(soa.data(), n * sizeof(double), h->raw + first, h->cap * sizeof(double),
                                 n * sizeof(double), dim, hipMemcpyDeviceToHost, h->stream));
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    for (size_t i = 0; i < n; ++i)
        for (int c = 0; c < dim; ++c) out[i * dim + c] = soa[(size_t)c * n + i];
    return OMPL_GPU_OK;
}

static uint64_t n_end_of(const ompl_gpu_nn *h) { return (h->n_total + kTile - 1) / kTile * kTile; }

// the fp32 screens need coordinates far from fp32 overflow (kernels.h kScreenMaxAbs); NaN fails
static bool screen_safe(const ompl_gpu_nn *h) {
    // SE3 quaternions far from unit norm would make the chord screen's error bound useless
    return h->absmax < kScreenMaxAbs && !(h->qeta > 1e-4);
}

#ifdef OMPL_AMD_PROBE
constexpr int kCullCounters = 23;  // + walk event counters and timers of the probe build (tools/walk_probe.py)
#else
constexpr int kCullCounters = 5;
#endif

// bring the sorted copy the culled walks read up to date, on the handle's stream with no host
// round trip: a full device build when there is none (or too many tombstones / a full tail),
// else the states added since the last call go to its tail
static ompl_gpu_status ensure_sorted(ompl_gpu_nn *h) {
    SortedStore &s = h->sorted;
    bool rebuild = !s.built || s.removed * 4 > (uint64_t)s.main_live + 256;
    if (!rebuild && h->n_total > s.covered) {
        bool fits = false;
        HIP_OR_FAIL(append_sorted_store(h->sp, h->g, h->feat32, h->feat, h->cap, h->n_total, current_bounds(h), &s,
                                        h->stream, &fits));
        rebuild = !fits;
        if (fits) h->sorted_appends++;
    }
    if (rebuild) {
        HIP_OR_FAIL(build_sorted_store(h->sp, h->g, h->feat32, h->feat, h->cap, h->n_total, (uint32_t)h->n_live, h->live,
                                       &s, h->stream));
        h->sorted_builds++;
    }
    if (!h->cull_counter.p) {
        const size_t bytes = sizeof(unsigned long long) * kCounterSlots * kCounterStride;
        HIP_OR_FAIL(h->cull_counter.ensure(bytes));
        HIP_OR_FAIL(hipMemsetAsync(h->cull_counter.p, 0, bytes, h->stream));
    }
    s.counters = (unsigned long long *)h->cull_counter.p;
    return OMPL_GPU_OK;
}

static int aos_width(const ompl_gpu_nn *h);
static ompl_gpu_status ensure_aos(ompl_gpu_nn *h);

// knn on device-resident features (queries already converted); caller holds the lock
static ompl_gpu_status knn_features_locked(ompl_gpu_nn *h, const double *d_qf, size_t nq, uint32_t k, uint32_t *d_ids,
                                           double *d_dist) {
    // large-k path: every k above the register buckets; from 33 on where it beats them (not the
    // chain, whose wave scan serves PRM*'s k <= 64 itself)
    // (the culled group walk serves k <= 61 on SE3 / R^n: fast_k2)
    const bool walk_k = h->fast && h->cull && cull_supported(h->sp) && screen_safe(h) &&
                        fast_k2(h->sp, k, (uint32_t)nq, true) > 0;
    const bool mid_k = k > 32 && h->fast && h->sp.kind != OMPL_GPU_SPACE_KCHAIN && !walk_k;
    const bool large = (k > (uint32_t)kMaxK || mid_k) && large_k_supported(h->sp) && screen_safe(h);
    if (k > (uint32_t)kMaxK && !large)
        return fail(OMPL_GPU_ERR_UNSUPPORTED, screen_safe(h) ? "k above 64 is not supported for this state space"
                                                             : "k above 64 needs stored coordinates below 1e18");
    const uint64_t n_end = n_end_of(h);
    if (n_end == 0) {
        // empty structure: every entry is (inf, none)
        std::vector<double> inf((size_t)nq * k, __builtin_inf());
        HIP_OR_FAIL(hipMemsetAsync(d_ids, 0xFF, sizeof(uint32_t) * nq * k, h->stream));
        HIP_OR_FAIL(hipMemcpyAsync(d_dist, inf.data(), sizeof(double) * inf.size(), hipMemcpyHostToDevice, h->stream));
        HIP_OR_FAIL(hipStreamSynchronize(h->stream));
        return OMPL_GPU_OK;
    }
    ProfileScope prof(h);
    if (large) {
        // distance bound for the histogram range (knn_large.hip)
        double dmax;
        if (h->sp.kind == OMPL_GPU_SPACE_SO3) {
            dmax = 0.5 * M_PI;
        } else if (h->sp.kind == OMPL_GPU_SPACE_SE3) {
            double e = 0.0;
            for (int c = 0; c < 3; ++c) e += (h->hi[c] - h->lo[c]) * (h->hi[c] - h->lo[c]);
            dmax = h->sp.w0 * std::sqrt(e) + h->sp.w1 * 0.5 * M_PI;
        } else if (h->sp.kind == OMPL_GPU_SPACE_KCHAIN) {
            // link * sum_i |P_i(a) - P_i(b)| with |P_i| <= i: at most link * n (n + 1)
            const double n = (double)h->sp.dim;
            dmax = h->sp.link * n * (n + 1.0);
        } else {
            dmax = 2.0 * h->absmax * std::sqrt((double)h->sp.dim);
        }
        dmax = std::max(dmax * 1.0001, 1e-30);
        size_t wsb = knn_large_workspace_bytes(h->sp, h->g, (uint32_t)nq, k, n_end, h->num_cus);
        if (wsb && h->ws.ensure(wsb) != hipSuccess) {  // no room for the select's slabs: the
            (void)hipGetLastError();                    // count / fill / sort form still answers
            wsb = 0;
        }
        if (!h->large_counter.p) {
            HIP_OR_FAIL(h->large_counter.ensure(2 * sizeof(unsigned long long)));
            HIP_OR_FAIL(hipMemsetAsync(h->large_counter.p, 0, 2 * sizeof(unsigned long long), h->stream));
        }
        // the select's exact pass reads one contiguous fp64 row per candidate from the AoS copy of
        // the raw states (features = raw coordinates outside the chain); only the select path
        // reads it, and without room for it the select reads the SoA features instead
        bool aos = wsb && h->sp.kind != OMPL_GPU_SPACE_KCHAIN;
        if (aos && ensure_aos(h) != OMPL_GPU_OK) {
            (void)hipGetLastError();
            aos = false;
        }
        HIP_OR_FAIL(launch_knn_large(h->sp, h->g, h->feat, h->feat32, h->cap, n_end,
                                     aos ? (const double *)h->raw_aos.p : nullptr, aos_width(h), d_qf,
                                     (uint32_t)nq, k, (float)h->absmax * (1.0f + 1e-6f), (float)h->qeta * 1.01f,
                                     (float)dmax, d_dist, d_ids, size_t(4) << 30, h->num_cus, h->stream,
                                     wsb ? h->ws.p : nullptr, wsb ? h->ws.bytes : 0,
                                     (unsigned long long *)h->large_counter.p));
        return OMPL_GPU_OK;
    }
    if (h->fast && screen_safe(h) && fast_k2(h->sp, k, (uint32_t)nq, h->cull) > 0) {
        // fp32 screen + fp64 certificate (knn_fast.hip); uncertified queries re-run exactly
        const bool cull = h->cull && cull_supported(h->sp);
        if (cull) {
            ompl_gpu_status s = ensure_sorted(h);
            if (s != OMPL_GPU_OK) return s;
            if (h->sp.kind == OMPL_GPU_SPACE_KCHAIN)
                HIP_OR_FAIL(refresh_chain_rows16(h->g, &h->sorted, h->stream));
        }
        FastBounds b = current_bounds(h);
        b.absmax = (float)h->absmax * (1.0f + 1e-6f);
        b.n_live = (uint32_t)h->n_live;
        const size_t wsb = knn_fast_workspace_bytes(h->sp, h->g, (uint32_t)nq, k, n_end, h->num_cus, cull);
        HIP_OR_FAIL(h->ws.ensure(wsb));
        // the bounded re-run's counters (below), zeroed by the batch's first kernel
        HIP_OR_FAIL(h->fb_c.ensure(sizeof(uint32_t) * (kBoundedMaxQ + 2 + nq)));
        HIP_OR_FAIL(h->fb_cd.ensure(sizeof(double) * kBoundedMaxQ * kBoundedCap));
        HIP_OR_FAIL(h->fb_ci.ensure(sizeof(uint32_t) * kBoundedMaxQ * kBoundedCap));
        uint32_t *cnt = (uint32_t *)h->fb_c.p;
        b.zero[0] = cnt;
        b.nzero[0] = kBoundedMaxQ + 2;
        uint32_t *d_fail_count = nullptr, *d_fail_list = nullptr;
        HIP_OR_FAIL(launch_knn_fast(h->sp, h->g, h->feat, h->feat32, h->cap, n_end, cull ? &h->sorted : nullptr, d_qf,
                                    (uint32_t)nq, k, b, d_dist, d_ids, h->ws.p, h->ws.bytes, h->num_cus, h->stream,
                                    &d_fail_count, &d_fail_list));
        // exact re-run of the uncertified queries, decided on the device: the bounded pass (one
        // store read for all of them), a full scan for any that overflow its candidate cap
        // (stats_dev: the re-run statistics, accumulated by the re-run's last kernel)
        HIP_OR_FAIL(h->stats_dev.ensure(2 * sizeof(unsigned long long)));
        if (!h->stats_init) {
            HIP_OR_FAIL(hipMemsetAsync(h->stats_dev.p, 0, 2 * sizeof(unsigned long long), h->stream));
            h->stats_init = true;
        }
        HIP_OR_FAIL(launch_knn_bounded(h->sp, h->g, h->feat, h->cap, n_end, d_qf, d_fail_list, d_fail_count, k, d_dist,
                                       d_ids, cnt, (double *)h->fb_cd.p, (uint32_t *)h->fb_ci.p, h->num_cus,
                                       h->stream, (unsigned long long *)h->stats_dev.p));
        h->fast_queries += nq;
        return OMPL_GPU_OK;
    }
    if (h->fast && screen_safe(h) && h->rows32 && stream32_supported(h->sp, h->g, (uint32_t)nq, k)) {
        // one / few queries (RRT's nearest per iteration): stream the fp32 rows, exact by
        // in-chunk fp64 refinement (knn_stream32.hip) — half the bytes of the fp64 stream
        HIP_OR_FAIL(h->ws.ensure(stream32_workspace_bytes((uint32_t)nq, n_end)));
        HIP_OR_FAIL(launch_knn_stream32(h->sp, h->g, h->feat32, h->feat, h->cap, n_end, d_qf, (uint32_t)nq, k,
                                        (float)h->absmax * (1.0f + 1e-6f), (float)h->qeta * 1.01f, d_dist, d_ids,
                                        h->ws.p, h->ws.bytes, h->stream));
        return OMPL_GPU_OK;
    }
    const size_t wsb = knn_workspace_bytes(h->sp, h->g, (uint32_t)nq, k, n_end, h->num_cus);
    HIP_OR_FAIL(h->ws.ensure(wsb));
    HIP_OR_FAIL(launch_knn(h->sp, h->g, h->feat, h->cap, n_end, d_qf, (uint32_t)nq, k, d_dist, d_ids, h->ws.p,
                           h->ws.bytes, h->num_cus, h->stream));
    return OMPL_GPU_OK;
}

static ompl_gpu_status upload_query_features(ompl_gpu_nn *h, const double *queries, size_t nq) {
    const int F = h->g.F, dim = h->sp.dim;
    h->hfeat.resize(nq * F);
    for (size_t i = 0; i < nq; ++i) host_features(h->sp, h->g, queries + i * dim, h->hfeat.data() + i * F);
    HIP_OR_FAIL(h->q.ensure(sizeof(double) * nq * F));
    HIP_OR_FAIL(hipMemcpyAsync(h->q.p, h->hfeat.data(), sizeof(double) * nq * F, hipMemcpyHostToDevice, h->stream));
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_nn_knn(ompl_gpu_nn *h, const double *queries, size_t nq, uint32_t k, uint64_t *out_ids,
                                double *out_dist, uint32_t *out_cnt) {
    if (!h || (nq && (!queries || (k && (!out_ids || !out_dist))))) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    std::lock_guard<std::mutex> lk(h->mu);
    if (nq == 0) return OMPL_GPU_OK;
    if (nq > 0x7FFFFFFFull) return fail(OMPL_GPU_ERR_UNSUPPORTED, "too many queries in one call");
    if (k == 0) {  // NearestNeighborsGNAT.h:226-227
        if (out_cnt) std::fill(out_cnt, out_cnt + nq, 0u);
        return OMPL_GPU_OK;
    }
    HIP_OR_FAIL(hipSetDevice(h->device));
    ompl_gpu_status s = upload_query_features(h, queries, nq);
    if (s != OMPL_GPU_OK) return s;
    HIP_OR_FAIL(h->out_d.ensure(sizeof(double) * nq * k));
    HIP_OR_FAIL(h->out_i.ensure(sizeof(uint32_t) * nq * k));
    s = knn_features_locked(h, (const double *)h->q.p, nq, k, (uint32_t *)h->out_i.p, (double *)h->out_d.p);
    if (s != OMPL_GPU_OK) return s;
    std::vector<uint32_t> ids32(nq * k);
    HIP_OR_FAIL(hipMemcpyAsync(out_dist, h->out_d.p, sizeof(double) * nq * k, hipMemcpyDeviceToHost, h->stream));
    HIP_OR_FAIL(hipMemcpyAsync(ids32.data(), h->out_i.p, sizeof(uint32_t) * nq * k, hipMemcpyDeviceToHost, h->stream));
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    for (size_t q = 0; q < nq; ++q) {
        uint32_t c = 0;
        for (uint32_t j = 0; j < k; ++j) {
            const uint32_t id = ids32[q * k + j];
            out_ids[q * k + j] = id == kNoId ? UINT64_MAX : (uint64_t)id;
            if (id != kNoId) ++c;
        }
        if (out_cnt) out_cnt[q] = c;
    }
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_nn_nearest(ompl_gpu_nn *h, const double *queries, size_t nq, uint64_t *out_ids,
                                    double *out_dist) {
    if (!h) return fail(OMPL_GPU_ERR_INVALID_ARG, "handle is NULL");
    if (h->n_live == 0)  // NearestNeighborsGNAT.h:218
        return fail(OMPL_GPU_ERR_EMPTY, "No elements found in nearest neighbors data structure");
    std::vector<double> tmpd;
    if (!out_dist) {
        tmpd.resize(nq);
        out_dist = tmpd.data();
    }
    return ompl_gpu_nn_knn(h, queries, nq, 1, out_ids, out_dist, nullptr);
}

// nearestR on device-resident query features (caller holds the lock).  Leaves the CSR
// result on device: the per-query offsets (nq + 1 entries) in h->qoff and, inside every
// segment, the (id, distance) pairs sorted by (distance, id) in *res_i / *res_d;
// *total = number of entries.
static ompl_gpu_status radius_features_locked(ompl_gpu_nn *h, const double *d_qf, size_t nq, double r,
                                              uint64_t *total, const uint32_t **res_i, const double **res_d) {
    *total = 0;
    *res_i = nullptr;
    *res_d = nullptr;
    HIP_OR_FAIL(h->qoff.ensure(sizeof(uint64_t) * (nq + 1)));
    uint64_t *d_qoff = (uint64_t *)h->qoff.p;
    const uint64_t n_end = n_end_of(h);
    if (n_end == 0 || !(r >= 0.0)) {  // empty structure, or a radius no distance satisfies
        HIP_OR_FAIL(hipMemsetAsync(d_qoff, 0, sizeof(uint64_t) * (nq + 1), h->stream));
        return OMPL_GPU_OK;
    }
    if (h->fast && h->cull && radius_cull_supported(h->sp) && nq <= 0x7FFFFFFFull && screen_safe(h) && r < kScreenMaxAbs) {
        // culled walk over the Morton-sorted copy (knn_fast_impl.h)
        ompl_gpu_status s = ensure_sorted(h);
        if (s != OMPL_GPU_OK) return s;
        if (h->sp.kind == OMPL_GPU_SPACE_SE3)
            HIP_OR_FAIL(refresh_se3_rows16(h->lo, h->hi, &h->sorted, h->stream));
        FastBounds b = current_bounds(h);
        b.absmax = (float)h->absmax * (1.0f + 1e-6f);
        HIP_OR_FAIL(h->ws.ensure(radius_fast_workspace_bytes(h->sp, h->g, (uint32_t)nq)));
        uint64_t *d_off = nullptr;
        // one walk: hits go to a fixed slab per query (the slab size adapts to the longest
        // segment seen); only if some query overflows its slab does a second (fill) walk run
        uint32_t slab = h->radius_slab;
        while (slab > 16 && (uint64_t)nq * slab > (1ull << 27)) slab >>= 1;
        b.slab = slab;
        HIP_OR_FAIL(h->slab_i.ensure(sizeof(uint32_t) * nq * slab));
        HIP_OR_FAIL(h->slab_d.ensure(sizeof(double) * nq * slab));
        {
            ProfileScope prof(h);
            HIP_OR_FAIL(launch_radius_fast(h->sp, h->g, h->feat, h->cap, &h->sorted, d_qf, (uint32_t)nq, r, b,
                                           h->ws.p, h->ws.bytes, 2, &d_off, (uint32_t *)h->slab_i.p,
                                           (double *)h->slab_d.p, h->stream));
        }
        uint64_t tm[2] = {0, 0};  // total, longest segment
        HIP_OR_FAIL(hipMemcpyAsync(tm, d_off + nq, sizeof(tm), hipMemcpyDeviceToHost, h->stream));
        HIP_OR_FAIL(hipMemcpyAsync(d_qoff, d_off, sizeof(uint64_t) * (nq + 1), hipMemcpyDeviceToDevice, h->stream));
        HIP_OR_FAIL(hipStreamSynchronize(h->stream));
        *total = tm[0];
        if (tm[0] == 0) return OMPL_GPU_OK;
        if (tm[0] > 0x7FFFFFFFull) return fail(OMPL_GPU_ERR_UNSUPPORTED, "radius result above 2^31 entries");
        if (tm[1] <= slab) {  // every segment is complete in its slab: sort into the CSR result
            const uint64_t tot = tm[0];
            h->radius_one_pass += 1;
            HIP_OR_FAIL(h->sorted_ids.ensure(sizeof(uint32_t) * tot));
            HIP_OR_FAIL(h->sorted_d.ensure(sizeof(double) * tot));
            uint32_t *si = (uint32_t *)h->sorted_ids.p;
            double *sd = (double *)h->sorted_d.p;
            HIP_OR_FAIL(launch_segment_rank_sort(d_qoff, (const uint32_t *)h->slab_i.p, (const double *)h->slab_d.p,
                                                 (uint32_t)nq, si, sd, h->stream, slab));
            *res_i = si;
            *res_d = sd;
            return OMPL_GPU_OK;
        }
        // a slab overflowed: its query's count is a candidate count (the exact decisions run on
        // the slab), so recount exactly with the count walk before the fill walk
        h->radius_two_pass += 1;
        HIP_OR_FAIL(launch_radius_fast(h->sp, h->g, h->feat, h->cap, &h->sorted, d_qf, (uint32_t)nq, r, b, h->ws.p,
                                       h->ws.bytes, 0, &d_off, nullptr, nullptr, h->stream));
        HIP_OR_FAIL(hipMemcpyAsync(tm, d_off + nq, sizeof(tm), hipMemcpyDeviceToHost, h->stream));
        HIP_OR_FAIL(hipMemcpyAsync(d_qoff, d_off, sizeof(uint64_t) * (nq + 1), hipMemcpyDeviceToDevice, h->stream));
        HIP_OR_FAIL(hipStreamSynchronize(h->stream));
        *total = tm[0];
        if (tm[0] == 0) return OMPL_GPU_OK;
        if (tm[0] > 0x7FFFFFFFull) return fail(OMPL_GPU_ERR_UNSUPPORTED, "radius result above 2^31 entries");
        const uint64_t tot = tm[0];
        uint32_t grow = 16;
        while (grow < tm[1] && grow < kRankSortMax) grow <<= 1;
        h->radius_slab = grow;  // the next call's slab holds this call's longest segment
        HIP_OR_FAIL(h->ids.ensure(sizeof(uint32_t) * tot));
        HIP_OR_FAIL(h->dists.ensure(sizeof(double) * tot));
        HIP_OR_FAIL(h->sorted_ids.ensure(sizeof(uint32_t) * tot));
        HIP_OR_FAIL(h->sorted_d.ensure(sizeof(double) * tot));
        uint32_t *ui = (uint32_t *)h->ids.p, *si = (uint32_t *)h->sorted_ids.p;
        double *ud = (double *)h->dists.p, *sd = (double *)h->sorted_d.p;
        HIP_OR_FAIL(launch_radius_fast(h->sp, h->g, h->feat, h->cap, &h->sorted, d_qf, (uint32_t)nq, r, b, h->ws.p,
                                       h->ws.bytes, 1, &d_off, ui, ud, h->stream));
        if (tm[1] <= kRankSortMax) {
            HIP_OR_FAIL(launch_segment_rank_sort(d_qoff, ui, ud, (uint32_t)nq, si, sd, h->stream));
            *res_i = si;
            *res_d = sd;
            return OMPL_GPU_OK;
        }
        // long segments: the merge-pass segmented sort by (distance, id)
        HIP_OR_FAIL(h->tmp.ensure(segment_sort_workspace(tot)));
        int second = 0;
        HIP_OR_FAIL(launch_segment_sort(d_qoff, (uint32_t)nq, tot, tm[1], ui, ud, si, sd, h->tmp.p, h->stream, &second));
        *res_i = second ? si : ui;
        *res_d = second ? sd : ud;
        return OMPL_GPU_OK;
    }
    // exact fp64 scan (OMPL_GPU_EXACT_ONLY / set_exact, SO3, KCHAIN): hits per (query, chunk)
    // written in id order, then a stable sort by distance gives (distance, id) order
    const RadiusPlan p = radius_plan((uint32_t)nq, n_end, h->num_cus);
    const size_t nc = nq * p.chunks;
    HIP_OR_FAIL(h->counts.ensure(sizeof(uint32_t) * nc));
    HIP_OR_FAIL(launch_radius_count(h->sp, h->g, p, h->feat, h->cap, n_end, d_qf, (uint32_t)nq, r,
                                    (uint32_t *)h->counts.p, h->stream));
    std::vector<uint32_t> cnt(nc);
    HIP_OR_FAIL(hipMemcpyAsync(cnt.data(), h->counts.p, sizeof(uint32_t) * nc, hipMemcpyDeviceToHost, h->stream));
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    std::vector<uint64_t> off(nc), qoff(nq + 1);
    uint64_t tot = 0, longest = 0;
    for (size_t q = 0; q < nq; ++q) {
        qoff[q] = tot;
        for (uint32_t c = 0; c < p.chunks; ++c) {
            off[q * p.chunks + c] = tot;
            tot += cnt[q * p.chunks + c];
        }
        longest = std::max<uint64_t>(longest, tot - qoff[q]);
    }
    qoff[nq] = tot;
    *total = tot;
    HIP_OR_FAIL(hipMemcpyAsync(d_qoff, qoff.data(), sizeof(uint64_t) * (nq + 1), hipMemcpyHostToDevice, h->stream));
    if (tot > 0x7FFFFFFFull) {
        (void)hipStreamSynchronize(h->stream);
        return fail(OMPL_GPU_ERR_UNSUPPORTED, "radius result above 2^31 entries");
    }
    if (tot > 0) {
        HIP_OR_FAIL(h->offsets.ensure(sizeof(uint64_t) * nc));
        HIP_OR_FAIL(hipMemcpyAsync(h->offsets.p, off.data(), sizeof(uint64_t) * nc, hipMemcpyHostToDevice, h->stream));
        HIP_OR_FAIL(h->ids.ensure(sizeof(uint32_t) * tot));
        HIP_OR_FAIL(h->dists.ensure(sizeof(double) * tot));
        HIP_OR_FAIL(h->sorted_ids.ensure(sizeof(uint32_t) * tot));
        HIP_OR_FAIL(h->sorted_d.ensure(sizeof(double) * tot));
        HIP_OR_FAIL(launch_radius_fill(h->sp, h->g, p, h->feat, h->cap, n_end, d_qf, (uint32_t)nq, r,
                                       (const uint64_t *)h->offsets.p, (uint32_t *)h->ids.p, (double *)h->dists.p,
                                       h->stream));
        HIP_OR_FAIL(h->tmp.ensure(segment_sort_workspace(tot)));
        int second = 0;
        HIP_OR_FAIL(launch_segment_sort(d_qoff, (uint32_t)nq, tot, longest, (uint32_t *)h->ids.p, (double *)h->dists.p,
                                        (uint32_t *)h->sorted_ids.p, (double *)h->sorted_d.p, h->tmp.p, h->stream,
                                        &second));
        *res_i = (const uint32_t *)(second ? h->sorted_ids.p : h->ids.p);
        *res_d = (const double *)(second ? h->sorted_d.p : h->dists.p);
    }
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));  // the host offset vectors are released on return
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_nn_radius(ompl_gpu_nn *h, const double *queries, size_t nq, double r, uint64_t **ids_out,
                                   double **dists_out, uint64_t *offsets_out) {
    if (!h || !ids_out || !offsets_out || (nq && !queries)) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    std::lock_guard<std::mutex> lk(h->mu);
    *ids_out = nullptr;
    if (dists_out) *dists_out = nullptr;
    offsets_out[0] = 0;
    if (nq == 0) return OMPL_GPU_OK;
    HIP_OR_FAIL(hipSetDevice(h->device));
    ompl_gpu_status s = upload_query_features(h, queries, nq);
    if (s != OMPL_GPU_OK) return s;
    uint64_t tot = 0;
    const uint32_t *ri = nullptr;
    const double *rd = nullptr;
    s = radius_features_locked(h, (const double *)h->q.p, nq, r, &tot, &ri, &rd);
    if (s != OMPL_GPU_OK) return s;
    uint64_t *hid = (uint64_t *)std::malloc(sizeof(uint64_t) * std::max<uint64_t>(tot, 1));
    double *hd = (double *)std::malloc(sizeof(double) * std::max<uint64_t>(tot, 1));
    std::vector<uint32_t> i32(tot);
    hipError_t e = hid && hd ? hipSuccess : hipErrorOutOfMemory;
    if (e == hipSuccess)
        e = hipMemcpyAsync(offsets_out, h->qoff.p, sizeof(uint64_t) * (nq + 1), hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess && tot) e = hipMemcpyAsync(i32.data(), ri, sizeof(uint32_t) * tot, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess && tot) e = hipMemcpyAsync(hd, rd, sizeof(double) * tot, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) {
        std::free(hid);
        std::free(hd);
        return fail(e == hipErrorOutOfMemory ? OMPL_GPU_ERR_OOM : OMPL_GPU_ERR_DEVICE,
                    std::string("nearestR copy-back: ") + hipGetErrorString(e));
    }
    for (uint64_t j = 0; j < tot; ++j) hid[j] = i32[j];
    *ids_out = hid;
    if (dists_out)
        *dists_out = hd;
    else
        std::free(hd);
    return OMPL_GPU_OK;
}

// device features of AoS raw queries (the NN's own buffer when they differ from the reals)
static ompl_gpu_status device_query_features(ompl_gpu_nn *h, const double *d_queries, size_t nq, const double **qf) {
    *qf = d_queries;
    const bool raw_is_feat = h->sp.kind == OMPL_GPU_SPACE_SE3 || h->sp.kind == OMPL_GPU_SPACE_SO3 ||
                             (h->sp.kind == OMPL_GPU_SPACE_REALVECTOR && h->g.F == h->sp.dim);
    if (raw_is_feat) return OMPL_GPU_OK;
    HIP_OR_FAIL(h->q.ensure(sizeof(double) * nq * h->g.F));
    HIP_OR_FAIL(launch_features(h->sp, h->g, d_queries, (uint32_t)nq, (double *)h->q.p, h->stream));
    *qf = (const double *)h->q.p;
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_nn_radius_device(ompl_gpu_nn *h, const double *d_queries, size_t nq, double r,
                                          uint64_t *d_offsets, uint32_t *d_ids, double *d_dist, uint64_t capacity,
                                          uint64_t *total) {
    if (!h || !total || (nq && (!d_queries || !d_offsets))) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    std::lock_guard<std::mutex> lk(h->mu);
    *total = 0;
    if (nq == 0) return OMPL_GPU_OK;
    if (nq > 0x7FFFFFFFull) return fail(OMPL_GPU_ERR_UNSUPPORTED, "too many queries in one call");
    HIP_OR_FAIL(hipSetDevice(h->device));
    const double *qf = nullptr;
    ompl_gpu_status s = device_query_features(h, d_queries, nq, &qf);
    if (s != OMPL_GPU_OK) return s;
    uint64_t tot = 0;
    const uint32_t *ri = nullptr;
    const double *rd = nullptr;
    s = radius_features_locked(h, qf, nq, r, &tot, &ri, &rd);
    if (s != OMPL_GPU_OK) return s;
    *total = tot;
    HIP_OR_FAIL(hipMemcpyAsync(d_offsets, h->qoff.p, sizeof(uint64_t) * (nq + 1), hipMemcpyDeviceToDevice, h->stream));
    if (tot > capacity) {
        HIP_OR_FAIL(hipStreamSynchronize(h->stream));
        return fail(OMPL_GPU_ERR_INVALID_ARG, "radius result exceeds the output capacity (see *total)");
    }
    if (tot) {
        if (!d_ids || !d_dist) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL output buffer");
        HIP_OR_FAIL(hipMemcpyAsync(d_ids, ri, sizeof(uint32_t) * tot, hipMemcpyDeviceToDevice, h->stream));
        HIP_OR_FAIL(hipMemcpyAsync(d_dist, rd, sizeof(double) * tot, hipMemcpyDeviceToDevice, h->stream));
    }
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    return OMPL_GPU_OK;
}

// width of the AoS rows of the raw states (edge endpoints gathered by id)
static int aos_width(const ompl_gpu_nn *h) { return (h->sp.dim + 1) & ~1; }

// bring the AoS copy of the raw states up to date: rows of the ids added since the last call
// (ids never move); caller holds the lock
static ompl_gpu_status ensure_aos(ompl_gpu_nn *h) {
    const int da = aos_width(h);
    if (h->aos_n >= h->n_total) return OMPL_GPU_OK;
    if (h->raw_aos.bytes < sizeof(double) * h->n_total * da) {
        DevBuf nb;
        HIP_OR_FAIL(nb.ensure(sizeof(double) * std::max<uint64_t>(h->cap, h->n_total) * da));
        if (h->aos_n)
            HIP_OR_FAIL(hipMemcpyAsync(nb.p, h->raw_aos.p, sizeof(double) * h->aos_n * da, hipMemcpyDeviceToDevice,
                                       h->stream));
        std::swap(h->raw_aos.p, nb.p);
        std::swap(h->raw_aos.bytes, nb.bytes);
        HIP_OR_FAIL(hipStreamSynchronize(h->stream));  // nb (the old buffer) is freed on return
    }
    HIP_OR_FAIL(launch_aos_rows(h->raw, h->cap, h->sp.dim, da, h->aos_n, h->n_total - h->aos_n, (double *)h->raw_aos.p,
                                h->stream));
    h->aos_n = h->n_total;
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_nn_edges_device(ompl_gpu_nn *h, const double *d_queries, size_t nq, const uint64_t *d_offsets,
                                         const uint32_t *d_ids, uint32_t stride, size_t m, int from_query,
                                         double *d_from, double *d_to) {
    if (!h || (m && (!d_queries || !d_ids || !d_from || !d_to))) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    if (!d_offsets && m && (stride == 0 || m != nq * (size_t)stride))
        return fail(OMPL_GPU_ERR_INVALID_ARG, "dense neighbour ids need m == nq * stride");
    std::lock_guard<std::mutex> lk(h->mu);
    if (m == 0) return OMPL_GPU_OK;
    if (nq == 0 || nq > 0xFFFFFFFFull) return fail(OMPL_GPU_ERR_INVALID_ARG, "query count out of range");
    HIP_OR_FAIL(hipSetDevice(h->device));
    // endpoints are gathered by random id: one contiguous row per state instead of one cache
    // line per coordinate of the SoA store
    const int da = aos_width(h);
    if (h->n_total) {
        ompl_gpu_status s = ensure_aos(h);
        if (s != OMPL_GPU_OK) return s;
    }
    uint32_t *qidx = nullptr;  // the CSR segment of every edge (edge_query_kernel)
    if (d_offsets) {
        HIP_OR_FAIL(h->edge_q.ensure(sizeof(uint32_t) * m));
        qidx = (uint32_t *)h->edge_q.p;
    }
    HIP_OR_FAIL(launch_edges(h->sp, h->raw, h->cap, d_queries, (uint32_t)nq, d_offsets, d_ids, stride, m, from_query,
                             d_from, d_to, h->stream, h->n_total ? (const double *)h->raw_aos.p : nullptr, da, qidx));
    return OMPL_GPU_OK;
}


// the walk counters summed over their slot copies (kernels.h kCounterSlots); caller holds the lock
static ompl_gpu_status read_cull_counters(ompl_gpu_nn *h, unsigned long long (&c)[kCullCounters]) {
    for (auto &v : c) v = 0;
    if (!h->cull_counter.p) return OMPL_GPU_OK;
    std::vector<unsigned long long> all((size_t)kCounterSlots * kCounterStride);
    HIP_OR_FAIL(hipSetDevice(h->device));
    HIP_OR_FAIL(hipMemcpyAsync(all.data(), h->cull_counter.p, sizeof(unsigned long long) * all.size(),
                               hipMemcpyDeviceToHost, h->stream));
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    for (int sl = 0; sl < kCounterSlots; ++sl)
        for (int i = 0; i < kCullCounters; ++i) c[i] += all[(size_t)sl * kCounterStride + i];
    return OMPL_GPU_OK;
}

#ifdef OMPL_AMD_PROBE
// probe build only: the raw walk counters
extern "C" ompl_gpu_status ompl_gpu_probe_counters(ompl_gpu_nn *h, uint64_t *out, int n) {
    std::lock_guard<std::mutex> lk(h->mu);
    unsigned long long c[kCullCounters];
    ompl_gpu_status st = read_cull_counters(h, c);
    if (st != OMPL_GPU_OK) return st;
    for (int i = 0; i < n && i < kCullCounters; ++i) out[i] = c[i];
    return OMPL_GPU_OK;
}
#endif

ompl_gpu_status ompl_gpu_nn_radius_cull_stats(ompl_gpu_nn *h, uint64_t *tiles_scanned, uint64_t *query_tiles) {
    if (!h) return fail(OMPL_GPU_ERR_INVALID_ARG, "handle is NULL");
    std::lock_guard<std::mutex> lk(h->mu);
    unsigned long long c[kCullCounters];
    ompl_gpu_status st = read_cull_counters(h, c);
    if (st != OMPL_GPU_OK) return st;
    if (tiles_scanned) *tiles_scanned = c[3];
    if (query_tiles) *query_tiles = c[4];
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_nn_radius_path_stats(ompl_gpu_nn *h, uint64_t *one_pass, uint64_t *two_pass) {
    if (!h) return fail(OMPL_GPU_ERR_INVALID_ARG, "handle is NULL");
    std::lock_guard<std::mutex> lk(h->mu);
    if (one_pass) *one_pass = h->radius_one_pass;
    if (two_pass) *two_pass = h->radius_two_pass;
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_nn_knn_device(ompl_gpu_nn *h, const double *d_queries, size_t nq, uint32_t k,
                                       uint32_t *d_ids, double *d_dist) {
    if (!h || (nq && (!d_queries || !d_ids || !d_dist))) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    std::lock_guard<std::mutex> lk(h->mu);
    if (nq == 0 || k == 0) return OMPL_GPU_OK;
    if (nq > 0x7FFFFFFFull) return fail(OMPL_GPU_ERR_UNSUPPORTED, "too many queries in one call");
    HIP_OR_FAIL(hipSetDevice(h->device));
    const double *qf = nullptr;
    ompl_gpu_status s = device_query_features(h, d_queries, nq, &qf);
    if (s != OMPL_GPU_OK) return s;
    return knn_features_locked(h, qf, nq, k, d_ids, d_dist);
}

ompl_gpu_status ompl_gpu_nn_set_exact(ompl_gpu_nn *h, int exact_only) {
    if (!h) return fail(OMPL_GPU_ERR_INVALID_ARG, "handle is NULL");
    std::lock_guard<std::mutex> lk(h->mu);
    h->fast = exact_only != 1;
    h->cull = exact_only != 2;
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_nn_profile(ompl_gpu_nn *h, int enable) {
    if (!h) return fail(OMPL_GPU_ERR_INVALID_ARG, "handle is NULL");
    std::lock_guard<std::mutex> lk(h->mu);
    h->profile = enable != 0;
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_nn_kernel_time(ompl_gpu_nn *h, double *total_ms, uint64_t *launches,
                                        const char **kernel_name) {
    if (!h) return fail(OMPL_GPU_ERR_INVALID_ARG, "handle is NULL");
    std::lock_guard<std::mutex> lk(h->mu);
    HIP_OR_FAIL(hipSetDevice(h->device));
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    for (KernelTimer &t : h->pending) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, t.begin, t.end) == hipSuccess) {
            h->prof_ms += ms;
            h->prof_launches++;
            h->prof_name = t.name;
        }
        (void)hipEventDestroy(t.begin);
        (void)hipEventDestroy(t.end);
    }
    h->pending.clear();
    if (total_ms) *total_ms = h->prof_ms;
    if (launches) *launches = h->prof_launches;
    if (kernel_name) *kernel_name = h->prof_name.c_str();
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_nn_cull_stats(ompl_gpu_nn *h, uint64_t *tiles_scanned, uint64_t *tiles_total,
                                       uint64_t *query_tiles) {
    if (!h) return fail(OMPL_GPU_ERR_INVALID_ARG, "handle is NULL");
    std::lock_guard<std::mutex> lk(h->mu);
    unsigned long long c[kCullCounters];
    ompl_gpu_status st = read_cull_counters(h, c);
    if (st != OMPL_GPU_OK) return st;
    if (tiles_scanned) *tiles_scanned = c[0];
    if (tiles_total) *tiles_total = c[1];
    if (query_tiles) *query_tiles = c[2];
    return OMPL_GPU_OK;
}

// the re-run counters live on the device (the query path never waits for them): read them here
static ompl_gpu_status read_stats(const ompl_gpu_nn *ch, unsigned long long *c) {
    ompl_gpu_nn *h = const_cast<ompl_gpu_nn *>(ch);
    std::lock_guard<std::mutex> lk(h->mu);
    c[0] = c[1] = 0;
    if (!h->stats_init) return OMPL_GPU_OK;
    HIP_OR_FAIL(hipSetDevice(h->device));
    HIP_OR_FAIL(hipMemcpyAsync(c, h->stats_dev.p, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost, h->stream));
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_nn_stats(const ompl_gpu_nn *h, uint64_t *screened, uint64_t *fallbacks) {
    if (!h) return fail(OMPL_GPU_ERR_INVALID_ARG, "handle is NULL");
    unsigned long long c[2];
    ompl_gpu_status s = read_stats(h, c);
    if (s != OMPL_GPU_OK) return s;
    if (screened) *screened = h->fast_queries;
    if (fallbacks) *fallbacks = c[0];
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_nn_large_stats(ompl_gpu_nn *h, uint64_t *spilled, uint64_t *exact) {
    if (!h) return fail(OMPL_GPU_ERR_INVALID_ARG, "handle is NULL");
    std::lock_guard<std::mutex> lk(h->mu);
    unsigned long long c[2] = {0, 0};
    if (h->large_counter.p) {
        HIP_OR_FAIL(hipSetDevice(h->device));
        HIP_OR_FAIL(hipMemcpyAsync(c, h->large_counter.p, sizeof(c), hipMemcpyDeviceToHost, h->stream));
        HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    }
    if (spilled) *spilled = c[0];
    if (exact) *exact = c[1];
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_nn_rerun_stats(const ompl_gpu_nn *h, uint64_t *full) {
    if (!h) return fail(OMPL_GPU_ERR_INVALID_ARG, "handle is NULL");
    unsigned long long c[2];
    ompl_gpu_status s = read_stats(h, c);
    if (s != OMPL_GPU_OK) return s;
    if (full) *full = c[1];
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_nn_build_index(ompl_gpu_nn *h) {
    if (!h) return fail(OMPL_GPU_ERR_INVALID_ARG, "handle is NULL");
    std::lock_guard<std::mutex> lk(h->mu);
    if (!cull_supported(h->sp) || h->n_total == 0) return OMPL_GPU_OK;
    HIP_OR_FAIL(hipSetDevice(h->device));
    return ensure_sorted(h);
}

ompl_gpu_status ompl_gpu_nn_index_stats(const ompl_gpu_nn *h, uint64_t *builds, uint64_t *appends) {
    if (!h) return fail(OMPL_GPU_ERR_INVALID_ARG, "handle is NULL");
    if (builds) *builds = h->sorted_builds;
    if (appends) *appends = h->sorted_appends;
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_steer_device(ompl_gpu_nn *h, const double *d_queries, size_t nq, const uint32_t *d_nearest,
                                      uint32_t stride, double max_distance, double *d_from, double *d_to) {
    if (!h || (nq && (!d_queries || !d_nearest || !d_from || !d_to))) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    std::lock_guard<std::mutex> lk(h->mu);
    if (nq == 0) return OMPL_GPU_OK;
    if (h->n_total == 0) return fail(OMPL_GPU_ERR_EMPTY, "No elements found in nearest neighbors data structure");
    HIP_OR_FAIL(hipSetDevice(h->device));
    HIP_OR_FAIL(launch_steer(h->sp, h->raw, h->cap, d_queries, (uint32_t)nq, d_nearest, stride, max_distance, d_from,
                             d_to, h->stream));
    return OMPL_GPU_OK;
}

// ------------------------------------------------------------------------------ MV

ompl_gpu_status ompl_gpu_mv_create(ompl_gpu_mv **out, const ompl_gpu_space *space, const ompl_gpu_checker *checker,
                                   int device) {
    if (!out || !checker) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    *out = nullptr;
    DevSpace sp;
    FeatGeom g;
    if (!space_ok(space, &sp, &g)) return fail(OMPL_GPU_ERR_UNSUPPORTED, "unsupported state space");
    if (checker->kind < OMPL_GPU_CHECK_ALL_VALID || checker->kind > OMPL_GPU_CHECK_CIRCLES2D)
        return fail(OMPL_GPU_ERR_UNSUPPORTED, "unknown validity checker");
    size_t per = 0;
    switch (checker->kind) {
    case OMPL_GPU_CHECK_SPHERES: per = 4; break;
    case OMPL_GPU_CHECK_CIRCLES2D: per = 3; break;
    case OMPL_GPU_CHECK_KCHAIN: per = 4; break;
    default: per = 0;
    }
    if (per && checker->count > 0 && !checker->data) return fail(OMPL_GPU_ERR_INVALID_ARG, "checker data is NULL");
    if (checker->kind == OMPL_GPU_CHECK_HYPERCUBE && (checker->ndim < 1 || checker->ndim > sp.dim))
        return fail(OMPL_GPU_ERR_INVALID_ARG, "hypercube ndim out of range");
    if (checker->kind == OMPL_GPU_CHECK_SPHERES && sp.dim < 3) return fail(OMPL_GPU_ERR_INVALID_ARG, "spheres need 3 reals");
    if (checker->kind == OMPL_GPU_CHECK_CIRCLES2D && sp.dim < 2) return fail(OMPL_GPU_ERR_INVALID_ARG, "circles need 2 reals");
    if (checker->kind == OMPL_GPU_CHECK_KCHAIN && sp.kind != OMPL_GPU_SPACE_KCHAIN)
        return fail(OMPL_GPU_ERR_INVALID_ARG, "kinematic chain checker needs a KCHAIN space");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
        return fail(OMPL_GPU_ERR_DEVICE, "no such HIP device");
    HIP_OR_FAIL(hipSetDevice(device));
    auto *h = new ompl_gpu_mv();
    h->device = device;
    h->sp = sp;
    h->g = g;
    h->ck.kind = checker->kind;
    h->ck.ndim = checker->ndim;
    h->ck.edge = checker->edge_width;
    h->ck.count = per ? checker->count : 0;
    h->ck.data = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&h->own, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&h->counters, 4 * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemset(h->counters, 0, 4 * sizeof(unsigned long long));
    if (e == hipSuccess && per && h->ck.count > 0) {
        e = hipMalloc(&h->ck_data, sizeof(double) * per * h->ck.count);
        if (e == hipSuccess)
            e = hipMemcpy(h->ck_data, checker->data, sizeof(double) * per * h->ck.count, hipMemcpyHostToDevice);
        h->ck.data = h->ck_data;
        h->ck_host.assign(checker->data, checker->data + per * h->ck.count);
    }
    h->ck.slack = 0.0;
    if (checker->kind == OMPL_GPU_CHECK_KCHAIN) {  // device_space.h chain_valid's side pre-test
        double M = std::max(1.0, std::fabs(sp.link) * sp.dim + 0.001);
        for (double v : h->ck_host) M = std::max(M, std::fabs(v));
        h->ck.slack = 1e-12 * M * M;
    }
    if (e != hipSuccess) {
        ompl_gpu_mv_destroy(h);
        return fail(OMPL_GPU_ERR_DEVICE, hipGetErrorString(e));
    }
    h->stream = h->own;
    *out = h;
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_mv_destroy(ompl_gpu_mv *h) {
    if (!h) return OMPL_GPU_OK;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->ck_data) (void)hipFree(h->ck_data);
    if (h->counters) (void)hipFree(h->counters);
    if (h->own) (void)hipStreamDestroy(h->own);
    delete h;
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_mv_set_stream(ompl_gpu_mv *h, void *s) {
    if (!h) return fail(OMPL_GPU_ERR_INVALID_ARG, "handle is NULL");
    std::lock_guard<std::mutex> lk(h->mu);
    h->stream = s ? (hipStream_t)s : h->own;
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_mv_sync(ompl_gpu_mv *h) {
    if (!h) return fail(OMPL_GPU_ERR_INVALID_ARG, "handle is NULL");
    HIP_OR_FAIL(hipSetDevice(h->device));
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_mv_check(ompl_gpu_mv *h, const double *s1, const double *s2, size_t m, uint8_t *valid,
                                  int32_t *nd, int32_t *first_invalid) {
    if (!h || (m && (!s1 || !s2 || !valid))) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    std::lock_guard<std::mutex> lk(h->mu);
    if (m == 0) return OMPL_GPU_OK;
    if (m > 0xFFFFFFFFull) return fail(OMPL_GPU_ERR_UNSUPPORTED, "too many edges in one call");
    HIP_OR_FAIL(hipSetDevice(h->device));
    const size_t sb = sizeof(double) * m * h->sp.dim;
    HIP_OR_FAIL(h->s1.ensure(sb));
    HIP_OR_FAIL(h->s2.ensure(sb));
    HIP_OR_FAIL(h->valid.ensure(m));
    if (nd) HIP_OR_FAIL(h->nd.ensure(sizeof(int32_t) * m));
    if (first_invalid) HIP_OR_FAIL(h->fi.ensure(sizeof(int32_t) * m));
    HIP_OR_FAIL(hipMemcpyAsync(h->s1.p, s1, sb, hipMemcpyHostToDevice, h->stream));
    HIP_OR_FAIL(hipMemcpyAsync(h->s2.p, s2, sb, hipMemcpyHostToDevice, h->stream));
    HIP_OR_FAIL(launch_motion(h->sp, h->ck, (const double *)h->s1.p, (const double *)h->s2.p, (uint32_t)m,
                              (uint8_t *)h->valid.p, nd ? (int32_t *)h->nd.p : nullptr,
                              first_invalid ? (int32_t *)h->fi.p : nullptr, h->counters, h->stream));
    HIP_OR_FAIL(hipMemcpyAsync(valid, h->valid.p, m, hipMemcpyDeviceToHost, h->stream));
    if (nd) HIP_OR_FAIL(hipMemcpyAsync(nd, h->nd.p, sizeof(int32_t) * m, hipMemcpyDeviceToHost, h->stream));
    if (first_invalid)
        HIP_OR_FAIL(hipMemcpyAsync(first_invalid, h->fi.p, sizeof(int32_t) * m, hipMemcpyDeviceToHost, h->stream));
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_mv_check_device(ompl_gpu_mv *h, const double *d_s1, const double *d_s2, size_t m,
                                         uint8_t *d_valid, int32_t *d_nd, int32_t *d_first_invalid) {
    if (!h || (m && (!d_s1 || !d_s2 || !d_valid))) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    std::lock_guard<std::mutex> lk(h->mu);
    if (m == 0) return OMPL_GPU_OK;
    if (m > 0xFFFFFFFFull) return fail(OMPL_GPU_ERR_UNSUPPORTED, "too many edges in one call");
    HIP_OR_FAIL(hipSetDevice(h->device));
    HIP_OR_FAIL(launch_motion(h->sp, h->ck, d_s1, d_s2, (uint32_t)m, d_valid, d_nd, d_first_invalid, h->counters,
                              h->stream));
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_mv_check_edges_device(ompl_gpu_mv *mv, ompl_gpu_nn *nn, const double *d_queries, size_t nq,
                                               const uint64_t *d_offsets, const uint32_t *d_ids, uint32_t stride,
                                               size_t m, int from_query, uint8_t *d_valid) {
    if (!mv || !nn || (m && (!d_queries || !d_ids || !d_valid))) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    if (!d_offsets && m && (stride == 0 || m != nq * (size_t)stride))
        return fail(OMPL_GPU_ERR_INVALID_ARG, "dense neighbour ids need m == nq * stride");
    if (mv->sp.kind != nn->sp.kind || mv->sp.dim != nn->sp.dim)
        return fail(OMPL_GPU_ERR_INVALID_ARG, "validator and neighbour structure differ in space");
    if (mv->device != nn->device) return fail(OMPL_GPU_ERR_INVALID_ARG, "validator and neighbour structure on different devices");
    std::scoped_lock lk(nn->mu, mv->mu);
    if (m == 0) return OMPL_GPU_OK;
    if (nq == 0 || nq > 0xFFFFFFFFull) return fail(OMPL_GPU_ERR_INVALID_ARG, "query count out of range");
    if (m > 0xFFFFFFFFull) return fail(OMPL_GPU_ERR_UNSUPPORTED, "too many edges in one call");
    HIP_OR_FAIL(hipSetDevice(mv->device));
    const int da = aos_width(nn);
    if (nn->n_total) {
        ompl_gpu_status s = ensure_aos(nn);
        if (s != OMPL_GPU_OK) return s;
    }
    uint32_t *qidx = nullptr;
    if (d_offsets) {  // validator-owned: written and read on the validator's stream only
        HIP_OR_FAIL(mv->edge_q.ensure(sizeof(uint32_t) * m));
        qidx = (uint32_t *)mv->edge_q.p;
    }
    // `from`'s queued work before `to`'s stream goes on: nn -> mv before the validator reads the
    // neighbour result and the AoS rows; mv -> nn at the end, so no later work on nn's stream (a
    // query overwriting its scratch, an add growing the AoS rows) runs while the motion kernel reads
    auto order = [&](hipStream_t from, hipStream_t to) -> hipError_t {
        if (from == to) return hipSuccess;
        hipEvent_t ev;
        hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        if (e != hipSuccess) return e;
        if ((e = hipEventRecord(ev, from)) == hipSuccess) e = hipStreamWaitEvent(to, ev, 0);
        const hipError_t d = hipEventDestroy(ev);
        return e != hipSuccess ? e : d;
    };
    const double *aos = nn->n_total ? (const double *)nn->raw_aos.p : nullptr;
    HIP_OR_FAIL(order(nn->stream, mv->stream));
    if (qidx) HIP_OR_FAIL(launch_edge_query(d_offsets, (uint32_t)nq, (uint64_t)m, qidx, mv->stream));
    hipError_t e = aos ? launch_motion_edges(mv->sp, mv->ck, d_queries, qidx, d_ids, stride, from_query, aos, da,
                                             (uint32_t)m, d_valid, mv->counters, mv->stream)
                       : hipErrorNotSupported;
    if (e == hipErrorNotSupported) {  // no fixed-width form (or an empty structure): materialise the pairs
        (void)hipGetLastError();
        size_t me = m;  // a CSR's existing edges: e < offsets[nq] (read back: this form synchronises)
        if (d_offsets) {
            uint64_t tot = 0;
            HIP_OR_FAIL(hipMemcpyAsync(&tot, d_offsets + nq, sizeof(tot), hipMemcpyDeviceToHost, mv->stream));
            HIP_OR_FAIL(hipStreamSynchronize(mv->stream));
            me = std::min<size_t>(m, tot);
            if (me < m) HIP_OR_FAIL(hipMemsetAsync(d_valid + me, 0, m - me, mv->stream));
            if (me == 0) return OMPL_GPU_OK;
        }
        m = me;
        const size_t bytes = sizeof(double) * m * mv->sp.dim;
        HIP_OR_FAIL(mv->s1.ensure(bytes));
        HIP_OR_FAIL(mv->s2.ensure(bytes));
        HIP_OR_FAIL(launch_edges(nn->sp, nn->raw, nn->cap, d_queries, (uint32_t)nq, d_offsets, d_ids, stride, m,
                                 from_query, (double *)mv->s1.p, (double *)mv->s2.p, mv->stream, aos, da, qidx));
        HIP_OR_FAIL(launch_motion(mv->sp, mv->ck, (const double *)mv->s1.p, (const double *)mv->s2.p, (uint32_t)m,
                                  d_valid, nullptr, nullptr, mv->counters, mv->stream));
        HIP_OR_FAIL(order(mv->stream, nn->stream));
        return OMPL_GPU_OK;
    }
    HIP_OR_FAIL(e);
    HIP_OR_FAIL(order(mv->stream, nn->stream));
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_mv_counters(ompl_gpu_mv *h, uint64_t *valid, uint64_t *invalid) {
    if (!h) return fail(OMPL_GPU_ERR_INVALID_ARG, "handle is NULL");
    std::lock_guard<std::mutex> lk(h->mu);
    HIP_OR_FAIL(hipSetDevice(h->device));
    unsigned long long c[4];
    HIP_OR_FAIL(hipMemcpyAsync(c, h->counters, sizeof(c), hipMemcpyDeviceToHost, h->stream));
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    if (valid) *valid = c[0];
    if (invalid) *invalid = c[1];
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_mv_state_checks(ompl_gpu_mv *h, uint64_t *checks) {
    if (!h || !checks) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    std::lock_guard<std::mutex> lk(h->mu);
    HIP_OR_FAIL(hipSetDevice(h->device));
    unsigned long long c[4];
    HIP_OR_FAIL(hipMemcpyAsync(c, h->counters, sizeof(c), hipMemcpyDeviceToHost, h->stream));
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    *checks = c[2];
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_mv_reset_counters(ompl_gpu_mv *h) {
    if (!h) return fail(OMPL_GPU_ERR_INVALID_ARG, "handle is NULL");
    std::lock_guard<std::mutex> lk(h->mu);
    HIP_OR_FAIL(hipSetDevice(h->device));
    HIP_OR_FAIL(hipMemsetAsync(h->counters, 0, 4 * sizeof(unsigned long long), h->stream));
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_svc_check(ompl_gpu_mv *h, const double *states, size_t m, uint8_t *valid) {
    if (!h || (m && (!states || !valid))) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    std::lock_guard<std::mutex> lk(h->mu);
    if (m == 0) return OMPL_GPU_OK;
    HIP_OR_FAIL(hipSetDevice(h->device));
    const size_t sb = sizeof(double) * m * h->sp.dim;
    HIP_OR_FAIL(h->s1.ensure(sb));
    HIP_OR_FAIL(h->valid.ensure(m));
    HIP_OR_FAIL(hipMemcpyAsync(h->s1.p, states, sb, hipMemcpyHostToDevice, h->stream));
    HIP_OR_FAIL(launch_state_valid(h->sp, h->ck, (const double *)h->s1.p, (uint32_t)m, (uint8_t *)h->valid.p, h->stream));
    HIP_OR_FAIL(hipMemcpyAsync(valid, h->valid.p, m, hipMemcpyDeviceToHost, h->stream));
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_svc_check_host(ompl_gpu_mv *h, const double *states, size_t m, uint8_t *valid) {
    if (!h || (m && (!states || !valid))) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    DevChecker ck = h->ck;
    ck.data = h->ck_host.empty() ? nullptr : h->ck_host.data();
    const int dim = h->sp.dim;
    for (size_t i = 0; i < m; ++i) valid[i] = is_valid(h->sp, ck, states + i * dim) ? 1 : 0;
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_svc_check_device(ompl_gpu_mv *h, const double *d_states, size_t m, uint8_t *d_valid) {
    if (!h || (m && (!d_states || !d_valid))) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    if (m > 0xFFFFFFFFull) return fail(OMPL_GPU_ERR_UNSUPPORTED, "too many states in one call");
    std::lock_guard<std::mutex> lk(h->mu);
    if (m == 0) return OMPL_GPU_OK;
    HIP_OR_FAIL(hipSetDevice(h->device));
    HIP_OR_FAIL(launch_state_valid(h->sp, h->ck, d_states, (uint32_t)m, d_valid, h->stream));
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_mv_motion_states_device(ompl_gpu_mv *h, const double *d_s1, const double *d_s2, size_t m,
                                                 uint32_t count, int endpoints, double *d_out) {
    if (count > 0xFFFFFFFDu) return fail(OMPL_GPU_ERR_INVALID_ARG, "count above UINT32_MAX - 2");
    const uint64_t per = motion_states_per(count, endpoints);
    if (!h || (m && per && (!d_s1 || !d_s2 || !d_out))) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    if ((uint64_t)m * per > 0xFFFFFFFFull || m > 0xFFFFFFFFull)
        return fail(OMPL_GPU_ERR_UNSUPPORTED, "too many motion states in one call");
    std::lock_guard<std::mutex> lk(h->mu);
    if (m == 0 || per == 0) return OMPL_GPU_OK;
    HIP_OR_FAIL(hipSetDevice(h->device));
    HIP_OR_FAIL(launch_motion_states(h->sp, d_s1, d_s2, (uint32_t)m, count, endpoints ? 1 : 0, d_out, h->stream));
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_mv_motion_states(ompl_gpu_mv *h, const double *s1, const double *s2, size_t m,
                                          uint32_t count, int endpoints, double *out) {
    if (count > 0xFFFFFFFDu) return fail(OMPL_GPU_ERR_INVALID_ARG, "count above UINT32_MAX - 2");
    const uint64_t per = motion_states_per(count, endpoints);
    if (!h || (m && per && (!s1 || !s2 || !out))) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    if ((uint64_t)m * per > 0xFFFFFFFFull || m > 0xFFFFFFFFull)
        return fail(OMPL_GPU_ERR_UNSUPPORTED, "too many motion states in one call");
    std::lock_guard<std::mutex> lk(h->mu);
    if (m == 0 || per == 0) return OMPL_GPU_OK;
    HIP_OR_FAIL(hipSetDevice(h->device));
    const size_t sb = sizeof(double) * m * h->sp.dim, ob = sb * per;
    HIP_OR_FAIL(h->s1.ensure(sb));
    HIP_OR_FAIL(h->s2.ensure(sb));
    HIP_OR_FAIL(h->ms.ensure(ob));
    HIP_OR_FAIL(hipMemcpyAsync(h->s1.p, s1, sb, hipMemcpyHostToDevice, h->stream));
    HIP_OR_FAIL(hipMemcpyAsync(h->s2.p, s2, sb, hipMemcpyHostToDevice, h->stream));
    HIP_OR_FAIL(launch_motion_states(h->sp, (const double *)h->s1.p, (const double *)h->s2.p, (uint32_t)m, count,
                                     endpoints ? 1 : 0, (double *)h->ms.p, h->stream));
    HIP_OR_FAIL(hipMemcpyAsync(out, h->ms.p, ob, hipMemcpyDeviceToHost, h->stream));
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    return OMPL_GPU_OK;
}

// StateSpace::distance / interpolate per pair on the device (see ompl_gpu.h)
ompl_gpu_status ompl_gpu_mv_space_pairs_device(ompl_gpu_mv *h, const double *d_a, const double *d_b, const double *d_t,
                                               size_t m, double *d_out) {
    if (!h || (m && (!d_a || !d_b || !d_out))) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    if (m > 0xFFFFFFFFull) return fail(OMPL_GPU_ERR_UNSUPPORTED, "too many pairs in one call");
    std::lock_guard<std::mutex> lk(h->mu);
    if (m == 0) return OMPL_GPU_OK;
    HIP_OR_FAIL(hipSetDevice(h->device));
    HIP_OR_FAIL(launch_space_pairs(h->sp, d_a, d_b, d_t, (uint32_t)m, d_out, h->stream));
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_mv_space_pairs(ompl_gpu_mv *h, const double *a, const double *b, const double *t, size_t m,
                                        double *out) {
    if (!h || (m && (!a || !b || !out))) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    if (m > 0xFFFFFFFFull) return fail(OMPL_GPU_ERR_UNSUPPORTED, "too many pairs in one call");
    std::lock_guard<std::mutex> lk(h->mu);
    if (m == 0) return OMPL_GPU_OK;
    HIP_OR_FAIL(hipSetDevice(h->device));
    const size_t sb = sizeof(double) * m * h->sp.dim, ob = t ? sb : sizeof(double) * m;
    HIP_OR_FAIL(h->s1.ensure(sb));
    HIP_OR_FAIL(h->s2.ensure(sb));
    HIP_OR_FAIL(h->ms.ensure(ob + (t ? sizeof(double) * m : 0)));
    double *dout = (double *)h->ms.p, *dt = t ? dout + (ob / sizeof(double)) : nullptr;
    HIP_OR_FAIL(hipMemcpyAsync(h->s1.p, a, sb, hipMemcpyHostToDevice, h->stream));
    HIP_OR_FAIL(hipMemcpyAsync(h->s2.p, b, sb, hipMemcpyHostToDevice, h->stream));
    if (t) HIP_OR_FAIL(hipMemcpyAsync(dt, t, sizeof(double) * m, hipMemcpyHostToDevice, h->stream));
    HIP_OR_FAIL(launch_space_pairs(h->sp, (const double *)h->s1.p, (const double *)h->s2.p, dt, (uint32_t)m, dout,
                                   h->stream));
    HIP_OR_FAIL(hipMemcpyAsync(out, dout, ob, hipMemcpyDeviceToHost, h->stream));
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    return OMPL_GPU_OK;
}

// ------------------------------------------------------------------------------ PRM*

namespace {
// One causal batch (PRM::addMilestone / LazyPRM::addMilestone for m milestones); mv == NULL is
// the lazy form (no edge is checked).  Caller holds the locks and validated the arguments.
ompl_gpu_status prm_batch_locked(ompl_gpu_nn *h, ompl_gpu_mv *mv, const double *states, size_t m, size_t j0,
                                 size_t j1, double k_const, uint32_t k_cap, uint32_t *d_nbr, uint32_t *d_cnt,
                                 uint8_t *d_valid, double *d_dist, uint64_t *edges) {
    if (edges) *edges = 0;
    if (m == 0) return OMPL_GPU_OK;
    HIP_OR_FAIL(hipSetDevice(h->device));
    const uint64_t n0 = h->n_total;
    if (n0 + m > 0xFFFFFFF0ull) return fail(OMPL_GPU_ERR_UNSUPPORTED, "more than 2^32-16 states");
    const int F = h->g.F, dim = h->sp.dim;
    // k_i = ceil(k_const * log(n)) with n = the vertex count including milestone i
    // (ConnectionStrategy.h:145-149, milestoneCount(), PRM.cpp:566) — host libm, as the reference
    const size_t rows = j1 - j0;  // this rank's slice: neighbours and edges of milestones [j0, j1)
    std::vector<uint32_t> kj(m);
    uint32_t kmax = 0;
    for (size_t j = 0; j < m; ++j) {
        const double kk = std::ceil(k_const * std::log((double)(n0 + j + 1)));
        kj[j] = kk > 0 ? (uint32_t)kk : 0u;
        kmax = std::max(kmax, kj[j]);
    }
    if (kmax > k_cap) return fail(OMPL_GPU_ERR_INVALID_ARG, "k_cap below the largest k of the batch");
    // the sorted store takes up the previous batch (tail append, 16-bit copy) on the device while
    // the host computes this batch's feature rows (the kNN below finds it current)
    if (n0 && rows && h->fast && h->cull && cull_supported(h->sp) && screen_safe(h)) {
        ompl_gpu_status s = ensure_sorted(h);
        if (s != OMPL_GPU_OK) return s;
        if (h->sp.kind == OMPL_GPU_SPACE_KCHAIN)
            HIP_OR_FAIL(refresh_chain_rows16(h->g, &h->sorted, h->stream));
    }
    // batch features (host, as add() computes them) and raw rows
    h->hfeat.resize(m * F);
    host_features_batch(h->sp, h->g, states, m, h->hfeat.data());
    HIP_OR_FAIL(h->prm_bf.ensure(sizeof(double) * m * F));
    HIP_OR_FAIL(h->prm_raw.ensure(sizeof(double) * m * dim));
    HIP_OR_FAIL(h->prm_kj.ensure(sizeof(uint32_t) * m));
    double *bf = (double *)h->prm_bf.p, *braw = (double *)h->prm_raw.p;
    uint32_t *dkj = (uint32_t *)h->prm_kj.p;
    HIP_OR_FAIL(hipMemcpyAsync(bf, h->hfeat.data(), sizeof(double) * m * F, hipMemcpyHostToDevice, h->stream));
    HIP_OR_FAIL(hipMemcpyAsync(braw, states, sizeof(double) * m * dim, hipMemcpyHostToDevice, h->stream));
    HIP_OR_FAIL(hipMemcpyAsync(dkj, kj.data(), sizeof(uint32_t) * m, hipMemcpyHostToDevice, h->stream));
    if (rows == 0) return add_locked(h, states, m, nullptr, bf, braw);
    // 1. the stored part: batched kNN of the slice's milestones (not yet inserted), k = min(kmax, live)
    const uint32_t kq = (uint32_t)std::min<uint64_t>(kmax, h->n_live);
    HIP_OR_FAIL(h->prm_sd.ensure(sizeof(double) * rows * std::max<uint32_t>(kq, 1)));
    HIP_OR_FAIL(h->prm_si.ensure(sizeof(uint32_t) * rows * std::max<uint32_t>(kq, 1)));
    double *sd = (double *)h->prm_sd.p;
    uint32_t *si = (uint32_t *)h->prm_si.p;
    if (kq > 0) {
        ompl_gpu_status s = knn_features_locked(h, bf + j0 * F, rows, kq, si, sd);
        if (s != OMPL_GPU_OK) return s;
    }
    // 2. in-batch causal candidates: count, offsets, fill, segmented sort by distance (stable:
    //    stored entries first, candidates in id order, so ties resolve by id)
    // prm_len: [0, rows) segment lengths, [rows] 0 (the scan's total), [rows + 1] the longest
    // segment, [rows + 2, 2 rows + 2) the fill's per-milestone cursors (chain tiles)
    HIP_OR_FAIL(h->prm_len.ensure(sizeof(uint64_t) * (2 * rows + 2)));
    HIP_OR_FAIL(h->prm_off.ensure(sizeof(uint64_t) * (rows + 1)));
    uint64_t *len = (uint64_t *)h->prm_len.p, *off = (uint64_t *)h->prm_off.p;
    HIP_OR_FAIL(hipMemsetAsync(len + rows, 0, 2 * sizeof(uint64_t), h->stream));
    float *p32 = nullptr;
    if (h->sp.kind == OMPL_GPU_SPACE_KCHAIN) {  // the causal scan's fp32 screen
        HIP_OR_FAIL(h->prm_p32.ensure(sizeof(float) * m * F));
        p32 = (float *)h->prm_p32.p;
    }
    HIP_OR_FAIL(launch_prm_causal(h->sp, h->g, false, bf, (uint32_t)j0, (uint32_t)rows, (uint32_t)n0, dkj, sd, si, kq,
                                  len, nullptr, nullptr, nullptr, p32, (uint32_t)m,
                                  (unsigned long long *)(len + rows + 1), h->stream));
    HIP_OR_FAIL(h->tmp.ensure(exclusive_scan_u64_workspace(rows)));
    HIP_OR_FAIL(launch_exclusive_scan_u64(len, rows, off, h->tmp.p, h->stream));  // off[rows] = the total
    uint64_t tot = 0, longest = 0;
    HIP_OR_FAIL(hipMemcpyAsync(&tot, off + rows, sizeof(uint64_t), hipMemcpyDeviceToHost, h->stream));
    HIP_OR_FAIL(hipMemcpyAsync(&longest, len + rows + 1, sizeof(uint64_t), hipMemcpyDeviceToHost, h->stream));
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    if (tot > 0x7FFFFFFFull) return fail(OMPL_GPU_ERR_UNSUPPORTED, "in-batch candidate set above 2^31 entries");
    HIP_OR_FAIL(h->dists.ensure(sizeof(double) * std::max<uint64_t>(tot, 1)));
    HIP_OR_FAIL(h->ids.ensure(sizeof(uint32_t) * std::max<uint64_t>(tot, 1)));
    HIP_OR_FAIL(h->sorted_d.ensure(sizeof(double) * std::max<uint64_t>(tot, 1)));
    HIP_OR_FAIL(h->sorted_ids.ensure(sizeof(uint32_t) * std::max<uint64_t>(tot, 1)));
    double *cd = (double *)h->dists.p, *sdd = (double *)h->sorted_d.p;
    uint32_t *ci = (uint32_t *)h->ids.p, *sii = (uint32_t *)h->sorted_ids.p;
    if (tot) {
        HIP_OR_FAIL(launch_prm_causal(h->sp, h->g, true, bf, (uint32_t)j0, (uint32_t)rows, (uint32_t)n0, dkj, sd, si,
                                      kq, nullptr, off, cd, ci, p32, (uint32_t)m, (unsigned long long *)(len + rows + 1),
                                      h->stream));
    }
    if (tot && longest <= kRankSortMax) {  // every segment fits a wave's LDS: rank placement by (distance, id)
        HIP_OR_FAIL(launch_segment_rank_sort(off, ci, cd, (uint32_t)rows, sii, sdd, h->stream));
    } else if (tot) {  // long segments: the merge-pass segmented sort by (distance, id)
        HIP_OR_FAIL(h->tmp.ensure(segment_sort_workspace(tot)));
        int second = 0;
        HIP_OR_FAIL(launch_segment_sort(off, (uint32_t)rows, tot, longest, ci, cd, sii, sdd, h->tmp.p, h->stream,
                                        &second));
        if (!second) {  // the result is in (cd, ci): read it from there
            std::swap(cd, sdd);
            std::swap(ci, sii);
        }
    }
    HIP_OR_FAIL(launch_prm_take(sii, sdd, off, dkj + j0, (uint32_t)rows, k_cap, d_nbr, d_cnt, d_dist, h->stream));
    if (!mv) return add_locked(h, states, m, nullptr, bf, braw);  // lazy: edge validity unknown (LazyPRM.cpp:302)
    // 3. edges checkMotion(state[n], state[m]) (PRM.cpp:582): compact, check, scatter to [m][k_cap]
    HIP_OR_FAIL(h->prm_eoff.ensure(sizeof(uint64_t) * (rows + 1)));
    HIP_OR_FAIL(h->prm_cnt64.ensure(sizeof(uint64_t) * (rows + 1)));
    uint64_t *eoff = (uint64_t *)h->prm_eoff.p, *c64 = (uint64_t *)h->prm_cnt64.p;
    HIP_OR_FAIL(launch_widen_u32(d_cnt, (uint32_t)rows, c64, h->stream));
    HIP_OR_FAIL(h->tmp.ensure(exclusive_scan_u64_workspace(rows)));
    HIP_OR_FAIL(launch_exclusive_scan_u64(c64, rows, eoff, h->tmp.p, h->stream));
    uint64_t E = 0;
    HIP_OR_FAIL(hipMemcpyAsync(&E, eoff + rows, sizeof(uint64_t), hipMemcpyDeviceToHost, h->stream));
    if (n0) {
        ompl_gpu_status s = ensure_aos(h);
        if (s != OMPL_GPU_OK) return s;
    }
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    if (E > 0xFFFFFFFFull) return fail(OMPL_GPU_ERR_UNSUPPORTED, "too many edges in one batch");
    if (E) {
        HIP_OR_FAIL(mv->s1.ensure(sizeof(double) * E * dim));
        HIP_OR_FAIL(mv->s2.ensure(sizeof(double) * E * dim));
        HIP_OR_FAIL(mv->valid.ensure(E));
        HIP_OR_FAIL(launch_prm_edges(d_nbr, d_cnt, eoff, (uint32_t)rows, (uint32_t)j0, k_cap, (uint32_t)n0, dim,
                                     n0 ? (const double *)h->raw_aos.p : nullptr, aos_width(h), braw,
                                     (double *)mv->s1.p, (double *)mv->s2.p, h->stream));
        HIP_OR_FAIL(launch_motion(mv->sp, mv->ck, (const double *)mv->s1.p, (const double *)mv->s2.p, (uint32_t)E,
                                  (uint8_t *)mv->valid.p, nullptr, nullptr, mv->counters, h->stream));
    }
    HIP_OR_FAIL(launch_prm_scatter_valid((const uint8_t *)mv->valid.p, d_cnt, eoff, (uint32_t)rows, k_cap, d_valid,
                                         h->stream));
    if (edges) *edges = E;
    // 4. the milestones join the structure (PRM.cpp:593): the batch's rows are on the device already
    return add_locked(h, states, m, nullptr, bf, braw);
}

ompl_gpu_status prm_check_args(ompl_gpu_nn *h, const double *states, size_t m, size_t j0, size_t j1, uint32_t k_cap) {
    if (j0 > j1 || j1 > m) return fail(OMPL_GPU_ERR_INVALID_ARG, "slice [j0, j1) outside the batch");
    if (m > 0x7FFFFFFFull || k_cap == 0 || k_cap > (uint32_t)kMaxK)
        return fail(OMPL_GPU_ERR_INVALID_ARG, "batch size or k_cap out of range (k_cap in [1, 64])");
    (void)h;
    (void)states;
    return OMPL_GPU_OK;
}
}  // namespace

ompl_gpu_status ompl_gpu_prm_add_milestones(ompl_gpu_nn *h, ompl_gpu_mv *mv, const double *states, size_t m,
                                            size_t j0, size_t j1, double k_const, uint32_t k_cap, uint32_t *d_nbr,
                                            uint32_t *d_cnt, uint8_t *d_valid, uint64_t *edges) {
    if (!h || !mv || (m && !states) || (j1 > j0 && (!d_nbr || !d_cnt || !d_valid)))
        return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    ompl_gpu_status s = prm_check_args(h, states, m, j0, j1, k_cap);
    if (s != OMPL_GPU_OK) return s;
    if (h->device != mv->device) return fail(OMPL_GPU_ERR_INVALID_ARG, "nn and mv handles are on different devices");
    if (h->sp.kind != mv->sp.kind || h->sp.dim != mv->sp.dim)
        return fail(OMPL_GPU_ERR_INVALID_ARG, "nn and mv handles describe different state spaces");
    std::scoped_lock lk(h->mu, mv->mu);
    return prm_batch_locked(h, mv, states, m, j0, j1, k_const, k_cap, d_nbr, d_cnt, d_valid, nullptr, edges);
}

ompl_gpu_status ompl_gpu_lazyprm_add_milestones(ompl_gpu_nn *h, const double *states, size_t m, size_t j0, size_t j1,
                                                double k_const, uint32_t k_cap, uint32_t *d_nbr, uint32_t *d_cnt,
                                                double *d_dist) {
    if (!h || (m && !states) || (j1 > j0 && (!d_nbr || !d_cnt))) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    ompl_gpu_status s = prm_check_args(h, states, m, j0, j1, k_cap);
    if (s != OMPL_GPU_OK) return s;
    std::lock_guard<std::mutex> lk(h->mu);
    return prm_batch_locked(h, nullptr, states, m, j0, j1, k_const, k_cap, d_nbr, d_cnt, nullptr, d_dist, nullptr);
}

// ------------------------------------------------------------------------------ RRT*

namespace {
ompl_gpu_status rrtstar_locked(ompl_gpu_nn *h, ompl_gpu_mv *mv, const double *d_samples, size_t ns, double maxd,
                               double k_rrt, uint32_t *d_nearest, uint32_t *d_added, double *d_inc, double *d_states,
                               ompl_gpu_rrtstar_result *out) {
    auto &R = h->rs;
    const int dim = h->sp.dim, F = h->g.F;
    const uint64_t n0 = h->n_total, nlive0 = h->n_live;
    const uint32_t n = (uint32_t)ns;
    hipStream_t st = h->stream;
    HIP_OR_FAIL(R.near_i.ensure(sizeof(uint32_t) * ns));
    HIP_OR_FAIL(R.near_d.ensure(sizeof(double) * ns));
    HIP_OR_FAIL(R.src.ensure(sizeof(uint32_t) * ns));
    HIP_OR_FAIL(R.xa.ensure(sizeof(double) * ns * dim));
    HIP_OR_FAIL(R.xb.ensure(sizeof(double) * ns * dim));
    HIP_OR_FAIL(R.from.ensure(sizeof(double) * ns * dim));
    HIP_OR_FAIL(R.inc.ensure(sizeof(double) * ns));
    HIP_OR_FAIL(R.va.ensure(ns));
    HIP_OR_FAIL(R.vb.ensure(ns));
    HIP_OR_FAIL(R.rank.ensure(sizeof(uint32_t) * (ns + 1)));
    HIP_OR_FAIL(R.list.ensure(sizeof(uint32_t) * ns));
    HIP_OR_FAIL(R.chg.ensure(sizeof(uint32_t)));
    uint32_t *near_i = (uint32_t *)R.near_i.p, *src = (uint32_t *)R.src.p, *rank = (uint32_t *)R.rank.p,
             *list = (uint32_t *)R.list.p, *chg = (uint32_t *)R.chg.p;
    double *near_d = (double *)R.near_d.p, *xa = (double *)R.xa.p, *xb = (double *)R.xb.p, *from = (double *)R.from.p,
           *inc = (double *)R.inc.p;
    uint8_t *va = (uint8_t *)R.va.p, *vb = (uint8_t *)R.vb.p;
    // 1. every sample against the stored tree: nearest, steer, checkMotion (RRTstar.cpp:266-282)
    const double *qf = nullptr;
    ompl_gpu_status s = device_query_features(h, d_samples, ns, &qf);
    if (s != OMPL_GPU_OK) return s;
    const bool prof = h->profile;  // the profile bracket (ompl_gpu_nn_profile) goes to the neighbourhoods' kNN
    h->profile = false;
    s = knn_features_locked(h, qf, ns, 1, near_i, near_d);
    h->profile = prof;
    if (s != OMPL_GPU_OK) return s;
    HIP_OR_FAIL(hipMemcpyAsync(src, near_i, sizeof(uint32_t) * ns, hipMemcpyDeviceToDevice, st));
    HIP_OR_FAIL(launch_rrtstar_steer(h->sp, h->raw, h->cap, d_samples, n, src, xb, maxd, from, xa, inc, st));
    HIP_OR_FAIL(launch_motion(mv->sp, mv->ck, from, xa, n, va, nullptr, nullptr, nullptr, st));
    // 2. fixed point: the nearest earlier added state of the batch against the stored nearest
    uint32_t rounds = 0;
    for (;;) {
        HIP_OR_FAIL(launch_rrtstar_rank(va, n, rank, list, st));
        HIP_OR_FAIL(launch_rrtstar_causal(h->sp, d_samples, n, xa, rank, list, near_i, near_d, src, st));
        HIP_OR_FAIL(launch_rrtstar_steer(h->sp, h->raw, h->cap, d_samples, n, src, xa, maxd, from, xb, inc, st));
        HIP_OR_FAIL(launch_motion(mv->sp, mv->ck, from, xb, n, vb, nullptr, nullptr, nullptr, st));
        HIP_OR_FAIL(hipMemsetAsync(chg, 0, sizeof(uint32_t), st));
        HIP_OR_FAIL(launch_rrtstar_diff(xa, xb, va, vb, n, dim, chg, st));
        uint32_t changed = 0;
        HIP_OR_FAIL(hipMemcpyAsync(&changed, chg, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        HIP_OR_FAIL(hipStreamSynchronize(st));
        std::swap(xa, xb);
        std::swap(va, vb);
        ++rounds;
        if (changed == 0) break;
        if (rounds > n + 1) return fail(OMPL_GPU_ERR_DEVICE, "RRT* batch: the in-batch nearest states did not settle");
    }
    // the settled state: ranks, ids, the added states in rank order
    HIP_OR_FAIL(launch_rrtstar_rank(va, n, rank, list, st));
    HIP_OR_FAIL(R.xc.ensure(sizeof(double) * ns * dim));
    double *xc = (double *)R.xc.p;
    HIP_OR_FAIL(R.ooff.ensure(sizeof(uint32_t) * 2 * ns));  // nearest / added when the caller passes none
    uint32_t *tmp_near = d_nearest ? d_nearest : (uint32_t *)R.ooff.p, *tmp_added = d_added ? d_added : tmp_near + ns;
    HIP_OR_FAIL(launch_rrtstar_finish(src, va, rank, xa, n, dim, (uint32_t)n0, tmp_near, tmp_added, xc, st));
    if (d_inc) HIP_OR_FAIL(hipMemcpyAsync(d_inc, inc, sizeof(double) * ns, hipMemcpyDeviceToDevice, st));
    if (d_states) HIP_OR_FAIL(hipMemcpyAsync(d_states, xa, sizeof(double) * ns * dim, hipMemcpyDeviceToDevice, st));
    uint32_t m = 0;
    HIP_OR_FAIL(hipMemcpyAsync(&m, rank + ns, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_OR_FAIL(hipStreamSynchronize(st));
    HIP_OR_FAIL(R.soff.ensure(sizeof(uint64_t) * (ns + 1)));
    uint64_t *soff = (uint64_t *)R.soff.p;
    *out = ompl_gpu_rrtstar_result{};
    out->rounds = rounds;
    out->added = m;
    out->offsets = soff;
    if (m == 0) {
        HIP_OR_FAIL(hipMemsetAsync(soff, 0, sizeof(uint64_t) * (ns + 1), st));
        HIP_OR_FAIL(hipStreamSynchronize(st));
        return OMPL_GPU_OK;
    }
    // 3. neighbourhoods of the added states: k_j = ceil(k_rrt ln(size + 1)), size = the tree when
    //    added state j is about to join (getNeighbors, RRTstar.cpp:605-611) — host libm, as the reference
    std::vector<uint32_t> kj(m);
    uint32_t kmax = 0;
    for (uint32_t j = 0; j < m; ++j) {
        const double kk = std::ceil(k_rrt * std::log((double)(nlive0 + j + 1)));
        kj[j] = kk > 0 ? (uint32_t)kk : 0u;
        kmax = std::max(kmax, kj[j]);
    }
    HIP_OR_FAIL(R.kj.ensure(sizeof(uint32_t) * m));
    uint32_t *dkj = (uint32_t *)R.kj.p;
    HIP_OR_FAIL(hipMemcpyAsync(dkj, kj.data(), sizeof(uint32_t) * m, hipMemcpyHostToDevice, st));
    const double *bf = xc;  // the added states' feature rows
    if (!(h->sp.kind == OMPL_GPU_SPACE_SE3 || h->sp.kind == OMPL_GPU_SPACE_SO3 ||
          (h->sp.kind == OMPL_GPU_SPACE_REALVECTOR && F == dim))) {
        HIP_OR_FAIL(R.bf.ensure(sizeof(double) * m * F));
        HIP_OR_FAIL(launch_features(h->sp, h->g, xc, m, (double *)R.bf.p, st));
        bf = (const double *)R.bf.p;
    }
    const uint32_t kq = (uint32_t)std::min<uint64_t>(kmax, nlive0);  // the stored part
    HIP_OR_FAIL(R.sd.ensure(sizeof(double) * (size_t)m * std::max<uint32_t>(kq, 1)));
    HIP_OR_FAIL(R.si.ensure(sizeof(uint32_t) * (size_t)m * std::max<uint32_t>(kq, 1)));
    double *sd = (double *)R.sd.p;
    uint32_t *si = (uint32_t *)R.si.p;
    if (kq > 0) {
        s = knn_features_locked(h, bf, m, kq, si, sd);
        if (s != OMPL_GPU_OK) return s;
    }
    // in-batch candidates (earlier added states within the stored list's k_j-th distance)
    HIP_OR_FAIL(R.len.ensure(sizeof(uint64_t) * (m + 2)));
    HIP_OR_FAIL(R.off.ensure(sizeof(uint64_t) * (m + 1)));
    HIP_OR_FAIL(R.scan.ensure(exclusive_scan_u64_workspace(m + 1)));
    uint64_t *len = (uint64_t *)R.len.p, *off = (uint64_t *)R.off.p;
    HIP_OR_FAIL(hipMemsetAsync(len + m, 0, 2 * sizeof(uint64_t), st));
    float *p32 = nullptr;
    if (h->sp.kind == OMPL_GPU_SPACE_KCHAIN) {
        HIP_OR_FAIL(R.p32.ensure(sizeof(float) * m * F));
        p32 = (float *)R.p32.p;
    }
    HIP_OR_FAIL(launch_prm_causal(h->sp, h->g, false, bf, 0, m, (uint32_t)n0, dkj, sd, si, kq, len, nullptr, nullptr,
                                  nullptr, p32, m, (unsigned long long *)(len + m + 1), st));
    HIP_OR_FAIL(launch_exclusive_scan_u64(len, m, off, R.scan.p, st));
    uint64_t hdr[2] = {0, 0};  // total, longest
    HIP_OR_FAIL(hipMemcpyAsync(&hdr[0], off + m, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    HIP_OR_FAIL(hipMemcpyAsync(&hdr[1], len + m + 1, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    HIP_OR_FAIL(hipStreamSynchronize(st));
    const uint64_t tot = hdr[0];
    HIP_OR_FAIL(R.cd.ensure(sizeof(double) * std::max<uint64_t>(tot, 1)));
    HIP_OR_FAIL(R.ci.ensure(sizeof(uint32_t) * std::max<uint64_t>(tot, 1)));
    double *cd = (double *)R.cd.p;
    uint32_t *ci = (uint32_t *)R.ci.p;
    if (tot)
        HIP_OR_FAIL(launch_prm_causal(h->sp, h->g, true, bf, 0, m, (uint32_t)n0, dkj, sd, si, kq, nullptr, off, cd, ci,
                                      p32, m, (unsigned long long *)(len + m + 1), st));
    // merged lists cut at k_j: counts, offsets
    HIP_OR_FAIL(R.scnt.ensure(sizeof(uint32_t) * m));
    HIP_OR_FAIL(R.ocnt.ensure(sizeof(uint64_t) * (m + 1)));
    HIP_OR_FAIL(R.ovf.ensure(sizeof(uint32_t)));
    uint32_t *scnt = (uint32_t *)R.scnt.p, *ovf = (uint32_t *)R.ovf.p;
    uint64_t *ocnt = (uint64_t *)R.ocnt.p;
    HIP_OR_FAIL(launch_rrtstar_counts(si, kq, dkj, off, m, scnt, ocnt, st));
    HIP_OR_FAIL(R.od.ensure(sizeof(uint64_t) * (m + 1)));
    uint64_t *ooff = (uint64_t *)R.od.p;
    HIP_OR_FAIL(launch_exclusive_scan_u64(ocnt, m, ooff, R.scan.p, st));
    uint64_t E = 0;
    HIP_OR_FAIL(hipMemcpyAsync(&E, ooff + m, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    HIP_OR_FAIL(hipMemsetAsync(ovf, 0, sizeof(uint32_t), st));
    HIP_OR_FAIL(hipStreamSynchronize(st));
    if (E > 0xFFFFFFFFull) return fail(OMPL_GPU_ERR_UNSUPPORTED, "RRT* batch: more than 2^32 neighbourhood entries");
    HIP_OR_FAIL(R.oi.ensure(sizeof(uint32_t) * std::max<uint64_t>(E, 1)));
    HIP_OR_FAIL(R.sortd.ensure(sizeof(double) * std::max<uint64_t>(E, 1)));
    HIP_OR_FAIL(R.oseg.ensure(sizeof(uint32_t) * std::max<uint64_t>(E, 1)));
    uint32_t *oi = (uint32_t *)R.oi.p, *oseg = (uint32_t *)R.oseg.p;
    double *odist = (double *)R.sortd.p;
    HIP_OR_FAIL(launch_rrtstar_merge(off, scnt, dkj, ci, cd, ooff, oi, odist, oseg, m, ovf, st));
    uint32_t overflow = 0;
    HIP_OR_FAIL(hipMemcpyAsync(&overflow, ovf, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_OR_FAIL(hipStreamSynchronize(st));
    if (overflow) {  // a segment with more than kRrtStarMergeCands candidates (a small tree, a large
                     // batch): every segment sorted by two stable radix passes (id, then distance)
        HIP_OR_FAIL(R.sorti.ensure(sizeof(uint32_t) * std::max<uint64_t>(tot, 1)));
        HIP_OR_FAIL(R.bits.ensure(sizeof(double) * std::max<uint64_t>(tot, 1)));
        uint32_t *sii = (uint32_t *)R.sorti.p;
        double *sdd = (double *)R.bits.p;
        HIP_OR_FAIL(h->tmp.ensure(segment_sort_workspace(tot)));
        int second = 0;
        HIP_OR_FAIL(launch_segment_sort(off, (uint32_t)m, tot, std::max<uint64_t>(hdr[1], 1), ci, cd, sii, sdd, h->tmp.p,
                                        st, &second));
        HIP_OR_FAIL(launch_rrtstar_take(off, second ? sii : ci, second ? sdd : cd, ooff, m, oi, odist, oseg, st));
    }
    // 4. both motion bits of every neighbourhood entry: checkMotion(nbh, x_j), checkMotion(x_j, nbh)
    s = ensure_aos(h);
    if (s != OMPL_GPU_OK) return s;
    HIP_OR_FAIL(mv->s1.ensure(sizeof(double) * std::max<uint64_t>(E, 1) * dim));
    HIP_OR_FAIL(mv->s2.ensure(sizeof(double) * std::max<uint64_t>(E, 1) * dim));
    HIP_OR_FAIL(R.fwd.ensure(std::max<uint64_t>(E, 1)));
    HIP_OR_FAIL(R.bwd.ensure(std::max<uint64_t>(E, 1)));
    HIP_OR_FAIL(R.bits.ensure(std::max<uint64_t>(E, 1)));
    double *e1 = (double *)mv->s1.p, *e2 = (double *)mv->s2.p;
    HIP_OR_FAIL(launch_rrtstar_edges(oi, oseg, E, (uint32_t)n0, dim, (const double *)h->raw_aos.p, aos_width(h), xc, e1,
                                     e2, st));
    HIP_OR_FAIL(launch_motion(mv->sp, mv->ck, e1, e2, (uint32_t)E, (uint8_t *)R.fwd.p, nullptr, nullptr, nullptr, st));
    HIP_OR_FAIL(launch_motion(mv->sp, mv->ck, e2, e1, (uint32_t)E, (uint8_t *)R.bwd.p, nullptr, nullptr, nullptr, st));
    HIP_OR_FAIL(launch_rrtstar_bits((const uint8_t *)R.fwd.p, (const uint8_t *)R.bwd.p, E, (uint8_t *)R.bits.p, st));
    HIP_OR_FAIL(launch_rrtstar_sample_offsets(va, rank, ooff, n, soff, st));
    // 5. the added states join the tree (RRTstar.cpp:410), ids n0 + rank
    std::vector<double> hx((size_t)m * dim);
    HIP_OR_FAIL(hipMemcpyAsync(hx.data(), xc, sizeof(double) * m * dim, hipMemcpyDeviceToHost, st));
    HIP_OR_FAIL(hipStreamSynchronize(st));
    uint64_t first = 0;
    s = add_locked(h, hx.data(), m, &first, bf, xc);
    if (s != OMPL_GPU_OK) return s;
    out->ids = oi;
    out->dist = odist;
    out->bits = (const uint8_t *)R.bits.p;
    out->total = E;
    return OMPL_GPU_OK;
}
}  // namespace

ompl_gpu_status ompl_gpu_rrtstar_batch_device(ompl_gpu_nn *h, ompl_gpu_mv *mv, const double *d_samples, size_t ns,
                                              double max_distance, double k_rrt, uint32_t *d_nearest,
                                              uint32_t *d_added, double *d_inc, double *d_states,
                                              ompl_gpu_rrtstar_result *out) {
    if (!h || !mv || !out || (ns && !d_samples)) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    if (h->device != mv->device) return fail(OMPL_GPU_ERR_INVALID_ARG, "nn and mv handles are on different devices");
    if (h->sp.kind != mv->sp.kind || h->sp.dim != mv->sp.dim)
        return fail(OMPL_GPU_ERR_INVALID_ARG, "nn and mv handles describe different state spaces");
    if (h->sp.kind == OMPL_GPU_SPACE_KCHAIN) return fail(OMPL_GPU_ERR_UNSUPPORTED, "RRT* batches: R^n, SO3 or SE3");
    if (ns > 0x7FFFFFFFull) return fail(OMPL_GPU_ERR_UNSUPPORTED, "too many samples in one batch");
    std::scoped_lock lk(h->mu, mv->mu);
    *out = ompl_gpu_rrtstar_result{};
    if (ns == 0) return OMPL_GPU_OK;
    if (h->n_live == 0) return fail(OMPL_GPU_ERR_EMPTY, "No elements found in nearest neighbors data structure");
    HIP_OR_FAIL(hipSetDevice(h->device));
    return rrtstar_locked(h, mv, d_samples, ns, max_distance, k_rrt, d_nearest, d_added, d_inc, d_states, out);
}

// the batch's per-sample outputs and neighbourhoods to the host, queued for ompl_gpu_rrtstar_commit
// (rrtstar_tree.cpp); under nn's lock, so that no later call on nn rewrites them meanwhile
ompl_gpu_status ompl_gpu_rrtstar_stage(ompl_gpu_rrtstar_tree *t, ompl_gpu_nn *h, size_t ns, const uint32_t *d_nearest,
                                       const uint32_t *d_added, const double *d_inc,
                                       const ompl_gpu_rrtstar_result *res) {
    if (!t || !h || !res || (ns && (!d_nearest || !d_added || !d_inc || !res->offsets)))
        return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    if (res->total && (!res->ids || !res->dist || !res->bits)) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    ompl_amd::RrtStarStaged b;
    {
        std::lock_guard<std::mutex> lk(t->mu);
        if (!t->spare.empty()) {
            b = std::move(t->spare.back());
            t->spare.pop_back();
        }
    }
    const size_t E = (size_t)res->total;
    try {
        b.ns = ns;
        b.nearest.resize(ns);
        b.added.resize(ns);
        b.inc.resize(ns);
        b.off.resize(ns + 1);
        b.ids.resize(E);
        b.dist.resize(E);
        b.bits.resize(E);
    } catch (const std::bad_alloc &) {
        return fail(OMPL_GPU_ERR_OOM, "out of host memory");
    }
    if (ns) {
        std::lock_guard<std::mutex> lk(h->mu);
        HIP_OR_FAIL(hipSetDevice(h->device));
        const hipMemcpyKind d2h = hipMemcpyDeviceToHost;
        HIP_OR_FAIL(hipMemcpyAsync(b.nearest.data(), d_nearest, 4 * ns, d2h, h->stream));
        HIP_OR_FAIL(hipMemcpyAsync(b.added.data(), d_added, 4 * ns, d2h, h->stream));
        HIP_OR_FAIL(hipMemcpyAsync(b.inc.data(), d_inc, 8 * ns, d2h, h->stream));
        HIP_OR_FAIL(hipMemcpyAsync(b.off.data(), res->offsets, 8 * (ns + 1), d2h, h->stream));
        if (E) {
            HIP_OR_FAIL(hipMemcpyAsync(b.ids.data(), res->ids, 4 * E, d2h, h->stream));
            HIP_OR_FAIL(hipMemcpyAsync(b.dist.data(), res->dist, 8 * E, d2h, h->stream));
            HIP_OR_FAIL(hipMemcpyAsync(b.bits.data(), res->bits, E, d2h, h->stream));
        }
        HIP_OR_FAIL(hipStreamSynchronize(h->stream));
        if (b.off[ns] != E) return fail(OMPL_GPU_ERR_INVALID_ARG, "result record does not match the offsets");
    } else {
        b.off[0] = 0;
    }
    std::lock_guard<std::mutex> lk(t->mu);
    t->staged.push_back(std::move(b));
    return OMPL_GPU_OK;
}

// ------------------------------------------------------------------------------ RRT

namespace {
ompl_gpu_status rrt_run(ompl_gpu_nn *h, ompl_gpu_mv *mv, const double *d_samples, size_t ns, double max_distance,
                        const double *goal, double goal_threshold, uint32_t *d_nearest, uint32_t *d_added,
                        uint64_t *solved_at, uint32_t *approx_id, double *approx_dist) {
    if (!h || !mv || (ns && (!d_samples || !d_nearest || !d_added))) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    if (h->device != mv->device) return fail(OMPL_GPU_ERR_INVALID_ARG, "nn and mv handles are on different devices");
    if (h->sp.kind != mv->sp.kind || h->sp.dim != mv->sp.dim)
        return fail(OMPL_GPU_ERR_INVALID_ARG, "nn and mv handles describe different state spaces");
    if (h->sp.kind == OMPL_GPU_SPACE_KCHAIN)
        return fail(OMPL_GPU_ERR_UNSUPPORTED, "device RRT growth needs a space whose stored features are its reals");
    if (!(max_distance > 0.0)) return fail(OMPL_GPU_ERR_INVALID_ARG, "max_distance must be positive");
    std::scoped_lock lk(h->mu, mv->mu);
    if (solved_at) *solved_at = ~0ull;
    if (approx_id) *approx_id = kNoId;
    if (approx_dist) *approx_dist = std::numeric_limits<double>::infinity();
    if (ns == 0) return OMPL_GPU_OK;
    if (ns > 0xFFFFFFFFull) return fail(OMPL_GPU_ERR_UNSUPPORTED, "too many samples in one call");
    if (h->n_live == 0) return fail(OMPL_GPU_ERR_EMPTY, "No elements found in nearest neighbors data structure");
    if (h->n_total + ns > 0xFFFFFFF0ull) return fail(OMPL_GPU_ERR_UNSUPPORTED, "more than 2^32-16 states");
    HIP_OR_FAIL(hipSetDevice(h->device));
    ompl_gpu_status s = grow(h, h->n_total + ns);
    if (s != OMPL_GPU_OK) return s;
    // screening bounds: an appended state lies on a segment from a stored state towards a
    // sample, so the box / largest coordinate over stored states and samples still bound it
    const int dim = h->sp.dim;
    std::vector<double> hs((size_t)ns * dim);
    HIP_OR_FAIL(hipMemcpyAsync(hs.data(), d_samples, sizeof(double) * hs.size(), hipMemcpyDeviceToHost, h->stream));
    HIP_OR_FAIL(h->rrt_n.ensure(sizeof(uint64_t)));
    const size_t parts = rrt_part_entries(h->n_total + ns);
    HIP_OR_FAIL(h->rrt_pd.ensure(sizeof(double) * parts));
    HIP_OR_FAIL(h->rrt_pi.ensure(sizeof(uint32_t) * parts));
    const uint64_t n0 = h->n_total;
    HIP_OR_FAIL(hipMemcpyAsync(h->rrt_n.p, &n0, sizeof(uint64_t), hipMemcpyHostToDevice, h->stream));
    if (h->rrt_coop < 0) {
        h->rrt_coop = (int)rrt_coop_blocks(h->device, h->sp, h->g);
        if (h->rrt_coop > 0 && hipExtMallocWithFlags(&h->rrt_sync, rrt_sync_bytes(), hipDeviceMallocUncached) != hipSuccess) {
            (void)hipGetLastError();
            h->rrt_sync = nullptr;
            h->rrt_coop = 0;  // no uncached memory: the two-launch form
        }
    }
    if (h->rrt_sync) HIP_OR_FAIL(hipMemsetAsync(h->rrt_sync, 0, rrt_sync_bytes(), h->stream));
    // goal record {solved iteration, approximate distance, its id} and the goal's reals
    const uint64_t grec0[3] = {~0ull, 0x7FF0000000000000ull, (uint64_t)kNoId};
    HIP_OR_FAIL(h->rrt_goal.ensure(sizeof(uint64_t) * 3 + sizeof(double) * dim));
    uint64_t *grec = (uint64_t *)h->rrt_goal.p;
    double *dgoal = (double *)(grec + 3);
    HIP_OR_FAIL(hipMemcpyAsync(grec, grec0, sizeof(grec0), hipMemcpyHostToDevice, h->stream));
    if (h->rrt_sync)  // the persistent form keeps the record in the uncached words [24, 27)
        HIP_OR_FAIL(hipMemcpyAsync((uint64_t *)h->rrt_sync + 24, grec0, sizeof(grec0), hipMemcpyHostToDevice,
                                   h->stream));
    if (goal) HIP_OR_FAIL(hipMemcpyAsync(dgoal, goal, sizeof(double) * dim, hipMemcpyHostToDevice, h->stream));
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    const int nb = tracked_dims(h->sp);
    const int na = h->sp.kind == OMPL_GPU_SPACE_SE3 ? 3 : (h->sp.kind == OMPL_GPU_SPACE_SO3 ? 0 : dim);
    for (size_t i = 0; i < ns; ++i) {
        const double *x = hs.data() + i * dim;
        for (int c = 0; c < nb; ++c) {
            h->lo[c] = std::min(h->lo[c], x[c]);
            h->hi[c] = std::max(h->hi[c], x[c]);
        }
        for (int c = 0; c < na; ++c) h->absmax = std::max(h->absmax, std::fabs(x[c]));
    }
    // appended states are slerp interpolations of unit quaternions (fp64): a conservative excess
    if (h->sp.kind == OMPL_GPU_SPACE_SE3) h->qeta = std::max(h->qeta, 1e-12);
    // the persistent form screens in fp32 (rrt.hip): it needs the fp32 rows and screenable
    // coordinates, and starts from the store's bounds (words 7 = B, 28 = eta of its record)
    // after two aborts in a row the handle takes the two-launch form for the next kRrtRetryAfter
    // batches (its device is shared with long kernels, and every persistent try would spin up to
    // kSpinLimit first), then tries the persistent form again; clear() resets the latch
    constexpr int kRrtRetryAfter = 64;
    if (h->rrt_abort_streak >= 2 && ++h->rrt_latched > kRrtRetryAfter) {
        h->rrt_abort_streak = 0;
        h->rrt_latched = 0;
    }
    const bool coop = h->rrt_sync && h->rows32 && screen_safe(h) && h->rrt_abort_streak < 2;
    if (coop) {
        // OMPL_GPU_RRT_SPIN_LIMIT (tests): a small spin limit forces the abort-and-re-run path;
        // read once per handle and kept in it, so that the copy needs no synchronisation
        if (!h->rrt_spin_read) {
            const char *lim = std::getenv("OMPL_GPU_RRT_SPIN_LIMIT");
            h->rrt_spin_override = (lim && std::atoll(lim) > 0) ? (uint64_t)std::atoll(lim) : 0ull;
            h->rrt_spin_read = true;
        }
        if (h->rrt_spin_override)
            HIP_OR_FAIL(hipMemcpyAsync((uint64_t *)h->rrt_sync + 4, &h->rrt_spin_override, sizeof(uint64_t),
                                       hipMemcpyHostToDevice, h->stream));
        const double B = h->absmax * (1.0 + 1e-6), eta = h->qeta * 1.01;
        HIP_OR_FAIL(hipMemcpyAsync((uint64_t *)h->rrt_sync + 7, &B, sizeof(double), hipMemcpyHostToDevice, h->stream));
        HIP_OR_FAIL(hipMemcpyAsync((uint64_t *)h->rrt_sync + 28, &eta, sizeof(double), hipMemcpyHostToDevice, h->stream));
    }
    // the persistent grid's counters / goal record / live size are restored if it aborts (a wait
    // past kSpinLimit: the device shared with a long kernel), and the batch re-runs in the
    // two-launch form — the store rows it wrote past n0 are not committed (n_total unchanged)
    if (coop) {
        HIP_OR_FAIL(h->rrt_save.ensure(4 * sizeof(unsigned long long)));
        HIP_OR_FAIL(hipMemcpyAsync(h->rrt_save.p, mv->counters, 4 * sizeof(unsigned long long),
                                   hipMemcpyDeviceToDevice, h->stream));
    }
    HIP_OR_FAIL(launch_rrt_grow(h->sp, mv->sp, mv->ck, h->g, h->feat, h->feat32, h->rows32, h->cap, n0,
                                (uint64_t *)h->rrt_n.p, d_samples, (uint32_t)ns, max_distance, (double *)h->rrt_pd.p,
                                (uint32_t *)h->rrt_pi.p, d_nearest, d_added, mv->counters, (uint64_t *)h->rrt_sync,
                                coop ? (uint32_t)h->rrt_coop : 0u, goal ? dgoal : nullptr, goal_threshold, grec,
                                h->stream));
    if (coop) HIP_OR_FAIL(hipStreamSynchronize(h->stream));  // B / eta above are host locals
    uint64_t grec_h[3] = {~0ull, 0, kNoId};
    uint64_t n1 = n0;
    uint64_t bar_h[3] = {0, 0, 0};
    if (coop) HIP_OR_FAIL(hipMemcpyAsync(bar_h, h->rrt_sync, sizeof(bar_h), hipMemcpyDeviceToHost, h->stream));
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    if (coop) h->rrt_abort_streak = bar_h[2] ? h->rrt_abort_streak + 1 : 0;
    if (bar_h[2]) {  // aborted: restore and re-run the whole batch in the two-launch form
        h->rrt_aborts++;
        HIP_OR_FAIL(hipMemcpyAsync(mv->counters, h->rrt_save.p, 4 * sizeof(unsigned long long),
                                   hipMemcpyDeviceToDevice, h->stream));
        HIP_OR_FAIL(hipMemcpyAsync(h->rrt_n.p, &n0, sizeof(uint64_t), hipMemcpyHostToDevice, h->stream));
        HIP_OR_FAIL(hipMemcpyAsync(grec, grec0, sizeof(grec0), hipMemcpyHostToDevice, h->stream));
        HIP_OR_FAIL(launch_rrt_grow(h->sp, mv->sp, mv->ck, h->g, h->feat, h->feat32, h->rows32, h->cap, n0,
                                    (uint64_t *)h->rrt_n.p, d_samples, (uint32_t)ns, max_distance,
                                    (double *)h->rrt_pd.p, (uint32_t *)h->rrt_pi.p, d_nearest, d_added, mv->counters,
                                    nullptr, 0u, goal ? dgoal : nullptr, goal_threshold, grec, h->stream));
    }
    HIP_OR_FAIL(hipMemcpyAsync(grec_h, grec, sizeof(grec_h), hipMemcpyDeviceToHost, h->stream));
    HIP_OR_FAIL(hipMemcpyAsync(&n1, h->rrt_n.p, sizeof(uint64_t), hipMemcpyDeviceToHost, h->stream));
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    if (goal && grec_h[0] != ~0ull && grec_h[0] + 1 < ns) {  // iterations after the solution did not run
        HIP_OR_FAIL(hipMemsetAsync(d_nearest + grec_h[0] + 1, 0xFF, sizeof(uint32_t) * (ns - grec_h[0] - 1), h->stream));
        HIP_OR_FAIL(hipMemsetAsync(d_added + grec_h[0] + 1, 0xFF, sizeof(uint32_t) * (ns - grec_h[0] - 1), h->stream));
        HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    }
    if (solved_at) *solved_at = grec_h[0];
    if (approx_id) *approx_id = (uint32_t)grec_h[2];
    if (approx_dist) {
        double d;
        std::memcpy(&d, &grec_h[1], sizeof(d));
        *approx_dist = d;
    }
    if (n1 > n0) HIP_OR_FAIL(hipMemsetAsync(h->live + n0, 1, n1 - n0, h->stream));
    h->n_live += n1 - n0;
    h->n_total = n1;
    h->removed.resize(h->n_total, 0);
    return OMPL_GPU_OK;
}
}  // namespace

ompl_gpu_status ompl_gpu_knn_merge_device(const double *d_dist, const uint32_t *d_ids, uint32_t lists, size_t nq,
                                          uint32_t k, double *d_out_dist, uint32_t *d_out_ids, void *stream) {
    if (nq && k && (!d_dist || !d_ids || !d_out_dist || !d_out_ids)) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    if (lists == 0 || lists > 64) return fail(OMPL_GPU_ERR_INVALID_ARG, "lists must be in [1, 64]");
    if (nq > 0xFFFFFFFFull) return fail(OMPL_GPU_ERR_UNSUPPORTED, "too many queries in one call");
    HIP_OR_FAIL(launch_topk_merge(d_dist, d_ids, lists, (uint32_t)nq, k, d_out_dist, d_out_ids, (hipStream_t)stream));
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_csr_merge_device(const uint64_t *d_offsets, uint32_t lists, size_t nq, const uint32_t *d_ids,
                                          const double *d_dist, size_t stride, uint64_t *d_out_offsets,
                                          uint32_t *d_out_ids, double *d_out_dist, void *stream) {
    if (nq && (!d_offsets || !d_out_offsets || ((!d_ids || !d_dist) && stride) || !d_out_ids || !d_out_dist))
        return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    if (lists == 0 || lists > 1024) return fail(OMPL_GPU_ERR_INVALID_ARG, "lists must be in [1, 1024]");
    if (nq > 0x7FFFFFFFull) return fail(OMPL_GPU_ERR_UNSUPPORTED, "too many queries in one call");
    HIP_OR_FAIL(launch_csr_merge(d_offsets, lists, (uint32_t)nq, d_ids, d_dist, stride, d_out_offsets, d_out_ids,
                                 d_out_dist, (hipStream_t)stream));
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_rrt_aborts(const ompl_gpu_nn *h, uint64_t *aborts) {
    if (!h || !aborts) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    *aborts = h->rrt_aborts;
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_rrt_grow_device(ompl_gpu_nn *h, ompl_gpu_mv *mv, const double *d_samples, size_t ns,
                                         double max_distance, uint32_t *d_nearest, uint32_t *d_added) {
    return rrt_run(h, mv, d_samples, ns, max_distance, nullptr, 0.0, d_nearest, d_added, nullptr, nullptr, nullptr);
}

ompl_gpu_status ompl_gpu_rrt_solve_device(ompl_gpu_nn *h, ompl_gpu_mv *mv, const double *d_samples, size_t ns,
                                          double max_distance, const double *goal, double goal_threshold,
                                          uint32_t *d_nearest, uint32_t *d_added, uint64_t *solved_at,
                                          uint32_t *approx_id, double *approx_dist) {
    if (!goal) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL goal");
    return rrt_run(h, mv, d_samples, ns, max_distance, goal, goal_threshold, d_nearest, d_added, solved_at, approx_id,
                   approx_dist);
}

// ------------------------------------------------------------------------------ BIT*

ompl_gpu_status ompl_gpu_bitstar_update_samples(ompl_gpu_nn *h, ompl_gpu_mv *mv, ompl_gpu_sampler *smp,
                                                uint64_t num_samples, uint64_t num_required, uint64_t max_tries,
                                                uint64_t *tries, uint64_t *first_id, uint64_t *added) {
    if (!h || !mv || !smp) return fail(OMPL_GPU_ERR_INVALID_ARG, "NULL argument");
    if (h->device != mv->device) return fail(OMPL_GPU_ERR_INVALID_ARG, "nn and mv handles are on different devices");
    if (h->sp.kind != mv->sp.kind || h->sp.dim != mv->sp.dim || smp->kind != h->sp.kind || smp->dim != h->sp.dim)
        return fail(OMPL_GPU_ERR_INVALID_ARG, "nn, mv and sampler describe different state spaces");
    std::scoped_lock lk(h->mu, mv->mu);
    HIP_OR_FAIL(hipSetDevice(h->device));
    if (first_id) *first_id = h->n_total;
    const int dim = h->sp.dim;
    uint64_t t = 0, have = num_samples, got_all = 0;
    double frac = 1.0;  // valid fraction seen so far: sizes the next batch of tries
    std::vector<double> rows, keep;
    std::vector<uint8_t> bits;
    // ImplicitGraph.cpp:966-990: tries < max_tries && numSamples_ < numRequiredSamples
    while (t < max_tries && have < num_required) {
        const uint64_t need = num_required - have;
        uint64_t chunk = (uint64_t)std::ceil((double)need / std::max(frac, 1e-3) * 1.05) + 32;
        chunk = std::min<uint64_t>({chunk, max_tries - t, (uint64_t)1 << 20});
        const ompl_amd::SamplerMark mark(*smp);
        rows.resize((size_t)chunk * dim);
        bits.resize(chunk);
        smp->sample(chunk, rows.data());
        HIP_OR_FAIL(mv->s1.ensure(sizeof(double) * rows.size()));
        HIP_OR_FAIL(mv->valid.ensure(chunk));
        HIP_OR_FAIL(hipMemcpyAsync(mv->s1.p, rows.data(), sizeof(double) * rows.size(), hipMemcpyHostToDevice,
                                   mv->stream));
        HIP_OR_FAIL(launch_state_valid(mv->sp, mv->ck, (const double *)mv->s1.p, (uint32_t)chunk,
                                       (uint8_t *)mv->valid.p, mv->stream));
        HIP_OR_FAIL(hipMemcpyAsync(bits.data(), mv->valid.p, chunk, hipMemcpyDeviceToHost, mv->stream));
        HIP_OR_FAIL(hipStreamSynchronize(mv->stream));
        // the reference loop stops at the try that brings the count to numRequiredSamples
        uint64_t used = 0, got = 0;
        keep.clear();
        for (; used < chunk && got < need; ++used)
            if (bits[used]) {
                keep.insert(keep.end(), rows.begin() + used * dim, rows.begin() + (used + 1) * dim);
                ++got;
            }
        if (used < chunk) {  // leave the streams exactly after try `used`
            mark.rewind(*smp);
            smp->sample(used, rows.data());
        }
        ompl_gpu_status s = add_locked(h, keep.data(), (size_t)got, nullptr);  // addToSamples (:688-692)
        if (s != OMPL_GPU_OK) return s;
        t += used;
        have += got;
        got_all += got;
        frac = (double)got_all / (double)t;
    }
    if (tries) *tries = t;
    if (added) *added = got_all;
    return OMPL_GPU_OK;
}

}  // extern "C"
