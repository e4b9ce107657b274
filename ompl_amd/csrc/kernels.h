// kernels.h — host-side launch interface of the HIP kernels (knn.hip, motion.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "device_space.h"
#include "kd_order.h"

namespace ompl_amd {

constexpr int kTile = 256;          // states per LDS tile / threads per block
constexpr int kMaxK = 64;           // largest register top-K bucket
// walk statistics counters (SortedStore::counters): kCounterSlots copies of kCounterStride words,
// a wave adds into copy blockIdx.x % kCounterSlots (same-address atomics from every wave of a
// 25,000-wave launch would serialise at the L2); readers sum the copies
constexpr int kCounterSlots = 64, kCounterStride = 24;
constexpr uint32_t kStreamMaxQ = 64; // below this many queries the stream mapping is used

// Optional HIP-event bracket around the dominant kernel of a launch (the scan), armed by
// the C ABI when profiling is enabled (ompl_gpu_nn_profile).  Events are recorded on the
// stream the kernel is launched on.
struct KernelTimer {
    hipEvent_t begin = nullptr, end = nullptr;
    const char *name = "";
};
extern thread_local KernelTimer *g_kernel_timer;
inline void timer_begin(hipStream_t st, const char *name) {
    if (g_kernel_timer) {
        g_kernel_timer->name = name;
        (void)hipEventRecord(g_kernel_timer->begin, st);
    }
}
inline void timer_end(hipStream_t st) {  // one bracket per armed call: disarm after it
    if (g_kernel_timer) (void)hipEventRecord(g_kernel_timer->end, st);
    g_kernel_timer = nullptr;
}

// Feature geometry of a space on device.
struct FeatGeom {
    int F;       // feature slots per state (padded)
    int nmax;    // KCHAIN: link bucket (F = 2*nmax); else 0
};
bool feature_geometry(const DevSpace &sp, FeatGeom *g);  // false if unsupported
// host-side feature computation for one AoS state (glibc cos/sin for KCHAIN)
void host_features(const DevSpace &sp, const FeatGeom &g, const double *raw, double *feat);

int k_bucket(uint32_t k);  // 1,4,16,32,64 or 0 if k > kMaxK

// kNN over features.  feat: SoA [F][cap]; qfeat: AoS [nq][F]; scans ids [0, n_end)
// (n_end a multiple of kTile, entries >= n_total are NaN).  Output [nq][k] sorted by
// (distance, id), missing entries = (inf, 0xFFFFFFFF).  ws: device workspace.
struct KnnWorkspace {
    void *ptr = nullptr;
    size_t bytes = 0;
};
size_t knn_workspace_bytes(const DevSpace &sp, const FeatGeom &g, uint32_t nq, uint32_t k, uint64_t n_end, int num_cus);
hipError_t launch_knn(const DevSpace &sp, const FeatGeom &g, const double *feat, uint64_t cap, uint64_t n_end,
                      const double *qfeat, uint32_t nq, uint32_t k, double *out_d, uint32_t *out_i, void *ws,
                      size_t ws_bytes, int num_cus, hipStream_t st);

// ---- fast exact kNN: fp32 screen (top-K2, K2 > k) + fp64 certify / rerank ----------
// Eligible for REALVECTOR / SO3 / SE3 with nq >= kStreamMaxQ and k + 6 <= kMaxK.  Every
// result is exact: a query whose certificate fails is listed in *fail_list (device) and
// must be re-run on the exact path by the caller (count in *fail_count, device).
constexpr int kKeyDims = 6;  // Morton key over at most 6 coordinates
struct FastBounds {
    float lo[kKeyDims], inv[kKeyDims];  // key box (inv = 1 / extent) of the first nkey key coordinates
    int nkey;                           // SE3: 6 (translation + canonical quaternion xyz); R^n: min(n, 6); SO3: 0
    float absmax;                       // max |coordinate| stored (error bound of the fp32 screen)
    uint32_t slab = 0;                  // radius phase 2: hits kept per query (slab capacity)
    uint32_t n_live = 0;                // live stored states: a screening list that is not full must hold them all
    float qeta = 0.f;                   // SE3: largest |norm^2 - 1| of the stored quaternions (screen_error)
    // per-call scratch words the first kernel of a query batch (query_rows_kernel) zeroes, so the
    // batch needs no memset launches: the re-run counters (C ABI), the home-key bins, the fail count
    uint32_t *zero[3] = {nullptr, nullptr, nullptr};
    uint32_t nzero[3] = {0u, 0u, 0u};
};
// The fp32 screens assume coordinates far from fp32 overflow: with |x| < kScreenMaxAbs every
// squared fp32 distance is finite (the C ABI takes the exact fp64 path otherwise).
constexpr double kScreenMaxAbs = 1e18;

// Spatially sorted fp32 copy of the store for the group walk (SE3 and R^n): states in k-d
// leaf order (kd_order.cpp: median splits along the widest coordinate), 64-state tiles (one
// state per lane, one k-d leaf) and 32-tile super-tiles (subtrees) with axis-aligned boxes over
// every coordinate of the metric (SE3: the translation and the sign-canonical quaternion,
// plus the largest quaternion norm excess, so the box yields a lower bound of the full SE3
// distance).
constexpr int kCullTile = 64;
constexpr int kSuperTiles = 32;
// mega-tiles: 64 consecutive super-tiles (2,048 tiles) with the union of their boxes, so a walk
// over a 10^7-state store tests 77 mega boxes and then only the super-tiles of the megas that
// pass, instead of all 4,883 super-tile boxes (one lane per box, 64 per round)
constexpr int kMegaSupers = 64;
// queries per wave in the group walk.  Measured on MI355X (k=10, 10^5 queries, k-d tiles):
// SE3 10^6 states G=2 2.09 ms, G=4 2.18 ms; R^6 10^5 states G=2 2.20 ms, G=4 1.50 ms.  (With
// Morton-run tiles, SE3: G=8 4.4 ms, G=4 3.5 ms, G=2 3.2 ms; packed two-query math 3.7 ms.)
// The walk is a chain of dependent memory round trips per wave, so narrower waves win where
// the walk is long (SE3, 10^6 states), wider ones where the store is small and L2-resident.
template <int SP>
// queries per wave of the culled kNN walk.  Round 1 measured SE3 G = 2 / 4 / 8 -> 2.04 / 1.41 / 1.73
// ms and R^6 G = 4 / 8 -> 1.01 / 0.70 ms; on round 4's walk (pipelined, packed keys, k-d
// neighbourhood first) fewer queries per wave win: cfg3 G = 2 1.208-1.211 against 1.271 ms at
// G = 4, cfg2 G = 2 / 4 / 8 0.538-0.541 / 0.552-0.562 / 0.655-0.658 ms (profiles/r4_ab)
constexpr int group_queries() { return 2; }
// 16-bit fixed-point coding of an SE3 store's fp32 rows: code = rint((v - lo) * inv) clamped to
// [0, kQ16Max], decoded as lo + code * step (step = 1 / inv); translation over the stored
// states' box, quaternion components over [-1.001, 1.001].  0xFFFF in coordinate 0: NaN row.
constexpr float kQ16Max = 65534.f;
struct Q16Geo {
    float lo[8], step[8], inv[8];
};

// Sorted-store rows are blocked by tile (round 6; were [row][n_pad] SoA): tile t (positions
// 64 t .. 64 t + 63) holds its R rows in segments of 4 rows — the last one R mod 4 wide — and each
// segment is position-major, the 4 values of one position side by side, so a wave reads a tile
// with one 16-byte load per lane per full segment (a contiguous 1 KB per instruction) and one
// narrower load for the remainder, instead of one 4-byte load per row.
__host__ __device__ __forceinline__ uint64_t blk_index(uint64_t p, int r, int R) {
    const int s = r >> 2, w = 4 * s + 4 <= R ? 4 : R - 4 * s;
    return (p >> 6) * (uint64_t)(64 * R) + (uint64_t)s * 256 + (p & 63) * (uint64_t)w + (uint64_t)(r & 3);
}
struct SortedStore {
    float *rows = nullptr;       // R rows per position, blocked by tile (blk_index; SE3 quaternions
                                 // sign-canonical: w >= 0)
    int rw = 0;                  // R: fp32 rows per position
    uint32_t *ids = nullptr;     // [n_pad] original id of each sorted slot (kNoId = padding)
    float *tbox = nullptr;       // [tiles][box_w] lo.., hi.. (, eta, pad)
    float *sbox = nullptr;       // [supers][box_w]
    float *mbox = nullptr;       // [megas][box_w] (kMegaSupers super-tiles each)
    uint32_t *tkey0 = nullptr;   // [tiles] key of each tile = its index (queries' keys are home tiles)
    KdNode *nodes = nullptr;     // internal k-d nodes of the main tiles, pre-order (kd_order.h)
    double *rows64 = nullptr;    // [n_pad][fa] fp64 features in sorted order (AoS: one 64 B row per
                                 // SE3 state), read by the certificate; padding rows are NaN
    uint32_t *inv = nullptr;     // [cap_inv] sorted position of each id (kNoId: not placed)
    int fa = 0;                  // fp64 row width: F rounded up to a multiple of 4
    uint32_t n = 0, n_pad = 0, ntiles = 0, nsuper = 0, nmega = 0, nnodes = 0;
    uint32_t kd_tiles = 0;       // main tiles (leaves of the k-d tree, built on the device)
    // incremental state: the main k-d tiles hold the live ids of [0, main_covered) at the build;
    // states added since then are re-tiled along the Morton curve in the tail region, tiles
    // [tail_t0, tail_t0 + tail_cap_tiles) (tail_t0 a super-tile boundary); removals write a NaN
    // into the state's sorted row (inv) — boxes stay conservative — until a quarter of the
    // main states are gone, which triggers a rebuild
    bool built = false;
    uint32_t main_live = 0, tail_t0 = 0, tail_cap_tiles = 0;
    uint64_t main_covered = 0, covered = 0, removed = 0;
    size_t cap_pos = 0, cap_nodes = 0, cap_inv = 0;  // allocated positions / nodes / inv entries
    uint32_t *qcount = nullptr;  // [pad_tiles + 1] per-tile query counts of the home-key counting sort
    // KinematicChain: the joint positions as 16-bit fixed point, two per word, F / 2 words per
    // position (chain_q16_code), re-encoded from `rows` when the store changed (gen != gen16)
    // SE3 (the radius walk): the 7 coordinates as 16-bit codes over q16 (4 words per position);
    // blocked by tile like `rows` (blk_index with w16 words)
    uint32_t *rows16 = nullptr;
    int w16 = 0;
    size_t cap16 = 0;
    uint64_t gen = 0, gen16 = ~0ull;
    Q16Geo q16{};
    void *scratch = nullptr;     // build / append workspace (grow-only)
    size_t scratch_bytes = 0;
    size_t bytes = 0;
    // optional device counters (owned by the caller), kNN walk: [0] tiles fetched, [1] tiles
    // a brute-force walk of the same query groups would have fetched, [2] (tile, query) pairs
    // scanned; radius walk: [3] tiles fetched, [4] (tile, query) pairs scanned
    unsigned long long *counters = nullptr;
};
bool cull_supported(const DevSpace &sp);
bool radius_cull_supported(const DevSpace &sp);  // the culled radius walk (SE3, R^n)
// full device build of the sorted copy over the live ids of [0, n_total) (live[id] != 0, n_live
// of them); asynchronous on st
hipError_t build_sorted_store(const DevSpace &sp, const FeatGeom &g, const float *feat32, const double *feat64,
                              uint64_t cap, uint64_t n_total, uint32_t n_live, const uint8_t *live, SortedStore *s,
                              hipStream_t st);
// place ids [s->main_covered, n_total) in the tail region; *fits = false when they do not fit (rebuild)
hipError_t append_sorted_store(const DevSpace &sp, const FeatGeom &g, const float *feat32, const double *feat64,
                               uint64_t cap, uint64_t n_total, const FastBounds &b, SortedStore *s, hipStream_t st,
                               bool *fits);
// removal of a placed id: its sorted fp32 row 0 becomes NaN
hipError_t tombstone_sorted_store(SortedStore *s, uint64_t id, hipStream_t st);
// The culled chain scan's 16-bit copy of the joint positions.  Coordinate f of link i = f mod nm
// lies in [-(i + 1), i + 1] (a sum of i + 1 unit vectors); its code is rint((x + i + 1) * S_i),
// S_i = kChainQ16 / (2 (i + 1)), clamped to [0, kChainQ16]; 0xFFFF in coordinate 0 marks a state
// with a NaN row (padding, tombstones).
constexpr float kChainQ16 = 65534.f;
hipError_t refresh_chain_rows16(const FeatGeom &g, SortedStore *s, hipStream_t st);
// bound on |d16 - d32| of one screened chain distance: link * sum_i sqrt(2) * 0.6 quanta * 2 (i + 1) / kChainQ16
// (0.5 for the rounding, the rest for the fp32 scaling of state and query)
double chain_q16_error(const DevSpace &sp);
// SE3 radius walk: the 16-bit copy over the stored box [lo, hi] of the translation, and the
// bound on |d16 - d32| it adds to the threshold.  Measured on cfg5: 1.694 ms per walk against
// 1.741-1.783 on the fp32 rows.  (The kNN group walk on the same copy measured slower — cfg3 1.383
// against 1.263 ms: its decode costs more VALU than the halved tile bytes save.)
hipError_t refresh_se3_rows16(const double *lo, const double *hi, SortedStore *s, hipStream_t st);
double se3_q16_error(const DevSpace &sp, const Q16Geo &q);
void free_sorted_store(SortedStore *s);

int fast_k2(const DevSpace &sp, uint32_t k, uint32_t nq, bool cull);  // screening list size, 0 = not eligible
int fp32_rows(const DevSpace &sp, const FeatGeom &g);     // rows of the fp32 SoA copy
// fp32 screening rows of stored states [first, first + n): the features, or for KCHAIN the
// joint positions (prefix sums of the cos / sin features)
hipError_t launch_rows32(const DevSpace &sp, const FeatGeom &g, const double *feat64, uint64_t cap, uint64_t first,
                         uint64_t n, float *feat32, hipStream_t st);
hipError_t launch_chain_rows32(const double *feat64, uint64_t cap, int nmax, uint64_t first, uint64_t n, float *feat32,
                               hipStream_t st);
size_t knn_fast_workspace_bytes(const DevSpace &sp, const FeatGeom &g, uint32_t nq, uint32_t k, uint64_t n_end,
                                int num_cus, bool cull);
// sorted == nullptr: chunked brute-force screen; else the group walk over *sorted
hipError_t launch_knn_fast(const DevSpace &sp, const FeatGeom &g, const double *feat64, const float *feat32,
                           uint64_t cap, uint64_t n_end, const SortedStore *sorted, const double *qfeat64, uint32_t nq,
                           uint32_t k, const FastBounds &b, double *out_d, uint32_t *out_i, void *ws, size_t ws_bytes,
                           int num_cus, hipStream_t st, uint32_t **fail_count, uint32_t **fail_list);
// ---- small batches (nq < kStreamMaxQ) over the fp32 rows, exact by in-chunk fp64 refinement
// (knn_stream32.hip): SE3 and R^n, k <= kStream32MaxK
constexpr uint32_t kStream32MaxK = 16;
bool stream32_supported(const DevSpace &sp, const FeatGeom &g, uint32_t nq, uint32_t k);
size_t stream32_workspace_bytes(uint32_t nq, uint64_t n_end);
hipError_t launch_knn_stream32(const DevSpace &sp, const FeatGeom &g, const float *feat32, const double *feat64,
                               uint64_t cap, uint64_t n_end, const double *qfeat, uint32_t nq, uint32_t k, float absmax,
                               float qeta, double *out_d, uint32_t *out_i, void *ws, size_t ws_bytes, hipStream_t st);
// ---- large k (k > 32; RRT* k ~ 6e3): histogram threshold + candidate sort (knn_large.hip)
// dmax: bound of the distances between stored states (the histogram's range; larger
// distances fall into an overflow bin and are still handled exactly).
// k <= 8,192 with a workspace of knn_large_workspace_bytes(): sampled thresholds, one fill pass,
// a block-per-query radix select + sort, all on the device (asynchronous); larger k: the
// count / host offsets / fill / segmented sort form (synchronous).
bool large_k_supported(const DevSpace &sp);
size_t knn_large_workspace_bytes(const DevSpace &sp, const FeatGeom &g, uint32_t nq, uint32_t k, uint64_t n_end,
                                 int num_cus);
// aos / da: the raw states by id as AoS rows of da doubles (SE3 / SO3 / R^n: the features), read
// one row per candidate by the exact-distance step (NULL: the SoA features); seta: the store's
// largest |norm^2 - 1| of a quaternion (SE3 fp32 screen bound); stats (device, 2 counters, may be
// NULL): += queries whose candidates spilled to the pool, += queries sent to the exact fallback
hipError_t launch_knn_large(const DevSpace &sp, const FeatGeom &g, const double *feat64, const float *feat32,
                            uint64_t cap, uint64_t n_end, const double *aos, int da, const double *qfeat64, uint32_t nq,
                            uint32_t k, float absmax, float seta, float dmax, double *out_d, uint32_t *out_i,
                            size_t mem_budget, int num_cus, hipStream_t st, void *ws = nullptr, size_t ws_bytes = 0,
                            unsigned long long *stats = nullptr);
hipError_t launch_to_fp32(const double *feat64, uint64_t cap, int rows, uint64_t first, uint64_t n, float *feat32,
                          hipStream_t st);
// exact re-run of the fast path's uncertified queries, with no host round trip: list[0..*d_nlist)
// (device count).  The first kBoundedMaxQ take the bounded pass: od / oi hold the certificate's
// exact lists (row q = query q, k entries), whose k-th distance bounds the answer, and the exact
// top-k overwrites them; queries with more than kBoundedCap candidates (and list entries past
// kBoundedMaxQ) take a full exact scan.  counts (device, kBoundedMaxQ + 2 + nq words, the first
// kBoundedMaxQ + 2 zeroed by the caller) returns at [kBoundedMaxQ] the number of full scans and
// at [kBoundedMaxQ + 2 ..] their query indices ([kBoundedMaxQ + 1]: the launch's grid barrier).
// cand_d / cand_i hold kBoundedMaxQ * kBoundedCap entries.  One launch of num_cus blocks.
constexpr uint32_t kBoundedCap = 1024;
constexpr uint32_t kBoundedMaxQ = 512;
hipError_t launch_knn_bounded(const DevSpace &sp, const FeatGeom &g, const double *feat, uint64_t cap,
                              uint64_t n_end, const double *qf, const uint32_t *list, const uint32_t *d_nlist,
                              uint32_t k, double *od, uint32_t *oi, uint32_t *counts, double *cand_d,
                              uint32_t *cand_i, int num_cus, hipStream_t st, unsigned long long *stats = nullptr);
// gather rows q = list[i] of an AoS [*][F] fp64 array into dst[i]; scatter results back
hipError_t launch_gather_rows(const double *src, int F, const uint32_t *list, uint32_t n, double *dst, hipStream_t st);
hipError_t launch_scatter_results(const double *d, const uint32_t *ids, uint32_t k, const uint32_t *list, uint32_t n,
                                  double *out_d, uint32_t *out_i, hipStream_t st);

// ---- culled radius search (SE3, R^n) over the sorted store (knn_fast_impl.h) ---------------
size_t radius_fast_workspace_bytes(const DevSpace &sp, const FeatGeom &g, uint32_t nq);
// phase 0: queries ordered on the Morton curve and their hits counted; *d_offsets (device,
// inside ws) then holds nq + 2 entries: the exclusive offsets [0, nq] (so [nq] = total) and
// the longest segment at [nq + 1].  phase 1 (same ws, same queries): every hit's (id, fp64
// distance) written into its query's segment, in walk order.  phase 2 (one pass): like
// phase 0, and the first b.slab hits of query q are written to out_i / out_d [q * b.slab ..]
// in walk order; if the longest segment fits in the slab, no phase 1 is needed.
hipError_t launch_radius_fast(const DevSpace &sp, const FeatGeom &g, const double *feat64, uint64_t cap,
                              const SortedStore *sorted, const double *qfeat64, uint32_t nq, double r,
                              const FastBounds &b, void *ws, size_t ws_bytes, int phase, uint64_t **d_offsets,
                              uint32_t *out_i, double *out_d, hipStream_t st);
// sort every CSR segment (at most kRankSortMax long) by (distance, id): rank placement in LDS
constexpr uint32_t kRankSortMax = 1024;
// in_stride != 0: segment q is read from [q * in_stride, ...) (a radius slab) instead of offsets[q]
hipError_t launch_segment_rank_sort(const uint64_t *offsets, const uint32_t *in_i, const double *in_d, uint32_t nq,
                                    uint32_t *out_i, double *out_d, hipStream_t st, uint32_t in_stride = 0);
// every segment [off[s], off[s + 1]) of (i0, d0) sorted by (distance, id), segments of any length
// (max_len >= the longest): bottom-up merge passes between (i0, d0) and (i1, d1); *in_second says
// which pair holds the result.  ws: segment_sort_workspace(n) bytes.
size_t segment_sort_workspace(uint64_t n);
hipError_t launch_segment_sort(const uint64_t *off, uint32_t nseg, uint64_t n, uint64_t max_len, uint32_t *i0,
                               double *d0, uint32_t *i1, double *d1, void *ws, hipStream_t st, int *in_second);
// motion endpoints of neighbour results: edge e pairs query q with stored state ids[e]
// (CSR offsets, or offsets == nullptr and e = q * stride + j)
// aos (optional): [n][da] copy of the raw states (launch_aos_rows), read instead of the SoA store
// the CSR segment (query) of every edge e < m: qidx[e] (kNoId past offsets[nq])
hipError_t launch_edge_query(const uint64_t *offsets, uint32_t nq, uint64_t m, uint32_t *qidx, hipStream_t st);
hipError_t launch_edges(const DevSpace &sp, const double *raw, uint64_t cap, const double *q, uint32_t nq,
                        const uint64_t *offsets, const uint32_t *ids, uint32_t stride, uint64_t m, int from_query,
                        double *from, double *to, hipStream_t st, const double *aos, int da, uint32_t *qidx);
// rows of ids [first, first + n) of the SoA store into aos[id][da]
hipError_t launch_aos_rows(const double *soa, uint64_t cap, int dim, int da, uint64_t first, uint64_t n, double *aos,
                           hipStream_t st);
// ---- PRM* causal milestone batches (prm.hip) ------------------------------------------------
// bf: [m][F] features of the batch; kj[m]: k of each milestone; sd / si: [m][kq] stored kNN lists.
// fill = false: seg_len[j] = stored entries kept + in-batch candidates; fill = true: segments
// written at seg_off (stored entries, then candidates j' < j with d <= the k_j-th stored distance)
// rows j0 .. j0 + rows - 1 of the batch (this rank's slice; sd / si / seg_* indexed by row)
// p32 (KinematicChain; NULL: no screen): workspace of m x F floats for the batch's fp32 joint
// positions (written by the count call, read by both); seg_max (count call): += the longest segment
hipError_t launch_prm_causal(const DevSpace &sp, const FeatGeom &g, bool fill, const double *bf, uint32_t j0,
                             uint32_t rows, uint32_t n0, const uint32_t *kj, const double *sd, const uint32_t *si,
                             uint32_t kq, uint64_t *seg_len, const uint64_t *seg_off, double *out_d, uint32_t *out_i,
                             float *p32, uint32_t m, unsigned long long *seg_max, hipStream_t st);
hipError_t launch_prm_take(const uint32_t *sorted_i, const double *sorted_d, const uint64_t *seg_off,
                           const uint32_t *kj, uint32_t m, uint32_t k_cap, uint32_t *nbr, uint32_t *cnt, double *dist,
                           hipStream_t st);
hipError_t launch_prm_edges(const uint32_t *nbr, const uint32_t *cnt, const uint64_t *eoff, uint32_t m, uint32_t j0,
                            uint32_t k_cap, uint32_t n0, int dim, const double *stored_aos, int da, const double *braw,
                            double *s1, double *s2, hipStream_t st);
hipError_t launch_widen_u32(const uint32_t *a, uint32_t n, uint64_t *b, hipStream_t st);
hipError_t launch_prm_scatter_valid(const uint8_t *vc, const uint32_t *cnt, const uint64_t *eoff, uint32_t m,
                                    uint32_t k_cap, uint8_t *valid, hipStream_t st);

// ---- RRT growth on device (rrt.hip) -------------------------------------------------------
size_t rrt_part_entries(uint64_t n_max);
// blocks of the persistent RRT grid on this device (one per CU, an ordinary launch), 0 when it
// cannot run (the two-launch form is used then); its synchronisation record (uncached device
// memory, zeroed before each launch) holds rrt_sync_bytes()
size_t rrt_sync_bytes();
uint32_t rrt_coop_blocks(int device, const DevSpace &sp, const FeatGeom &g);
hipError_t launch_rrt_grow(const DevSpace &sp, const DevSpace &msp, const DevChecker &ck, const FeatGeom &g,
                           double *feat, float *feat32, int rows32, uint64_t cap, uint64_t n0, uint64_t *n_dev,
                           const double *samples, uint32_t ns, double maxd, double *part_d, uint32_t *part_i,
                           uint32_t *nearest, uint32_t *added, unsigned long long *counters, uint64_t *sync,
                           uint32_t coop_blocks, const double *goal, double goal_threshold, uint64_t *grec,
                           hipStream_t st);
// goal record of a run (64-bit words, zero-initialised by the host as {~0, +inf bits, ~0})
size_t rrt_goal_words();

// ---- RRT* iteration batches (rrtstar.hip) --------------------------------------------------
// nearest sources: a stored id, or kRrtStarInBatch | j (sample j of the batch)
constexpr uint32_t kRrtStarInBatch = 0x80000000u;
hipError_t launch_rrtstar_steer(const DevSpace &sp, const double *raw, uint64_t cap, const double *samples, uint32_t ns,
                                const uint32_t *src, const double *x_prev, double maxd, double *from, double *to,
                                double *inc, hipStream_t st);
hipError_t launch_rrtstar_rank(const uint8_t *valid, uint32_t ns, uint32_t *rank, uint32_t *list, hipStream_t st);
hipError_t launch_rrtstar_causal(const DevSpace &sp, const double *samples, uint32_t ns, const double *x,
                                 const uint32_t *rank, const uint32_t *list, const uint32_t *near_id,
                                 const double *near_d, uint32_t *src, hipStream_t st);
hipError_t launch_rrtstar_diff(const double *xa, const double *xb, const uint8_t *va, const uint8_t *vb, uint32_t ns,
                               int dim, uint32_t *changed, hipStream_t st);
hipError_t launch_rrtstar_finish(const uint32_t *src, const uint8_t *valid, const uint32_t *rank, const double *x,
                                 uint32_t ns, int dim, uint32_t n0, uint32_t *nearest, uint32_t *added, double *xa,
                                 hipStream_t st);
hipError_t launch_rrtstar_counts(const uint32_t *si, uint32_t kq, const uint32_t *kj, const uint64_t *seg_off,
                                 uint32_t rows, uint32_t *stored_cnt, uint64_t *out_cnt, hipStream_t st);
// merge of each segment's sorted stored entries with its (at most kRrtStarMergeCands) in-batch
// candidates, cut at out_off's counts; *overflow += segments with more candidates (not written)
constexpr uint32_t kRrtStarMergeCands = 1024;
hipError_t launch_rrtstar_merge(const uint64_t *seg_off, const uint32_t *stored_cnt, const uint32_t *kj,
                                const uint32_t *in_i, const double *in_d, const uint64_t *out_off, uint32_t *out_i,
                                double *out_d, uint32_t *out_seg, uint32_t rows, uint32_t *overflow, hipStream_t st);
// the same from fully sorted segments (the radix fallback): the first out counts of each segment
hipError_t launch_rrtstar_take(const uint64_t *seg_off, const uint32_t *in_i, const double *in_d, const uint64_t *out_off,
                               uint32_t rows, uint32_t *out_i, double *out_d, uint32_t *out_seg, hipStream_t st);
hipError_t launch_rrtstar_edges(const uint32_t *ids, const uint32_t *seg, uint64_t E, uint32_t n0, int dim,
                                const double *aos, int da, const double *xa, double *s1, double *s2, hipStream_t st);
hipError_t launch_rrtstar_bits(const uint8_t *fwd, const uint8_t *bwd, uint64_t E, uint8_t *bits, hipStream_t st);
hipError_t launch_rrtstar_sample_offsets(const uint8_t *valid, const uint32_t *rank, const uint64_t *out_off,
                                         uint32_t ns, uint64_t *off, hipStream_t st);

// ---- exclusive prefix sums (scan.hip): out[0..n], out[n] = the total; ws of
// exclusive_scan_u64_workspace(n) bytes; asynchronous
size_t exclusive_scan_u64_workspace(uint64_t n);
// max_out (optional, device): the largest of in[0, n)
hipError_t launch_exclusive_scan_u64(const uint64_t *in, uint64_t n, uint64_t *out, void *ws, hipStream_t st,
                                     uint64_t *max_out = nullptr);

// radius search, pass 1 (count per (query, chunk)) and pass 2 (fill CSR in id order).
struct RadiusPlan {
    uint32_t chunks;      // chunks per query
    uint32_t chunk_len;   // states per chunk
    bool stream;          // wave-chunk mapping (small nq) vs tiled mapping
};
RadiusPlan radius_plan(uint32_t nq, uint64_t n_end, int num_cus);
hipError_t launch_radius_count(const DevSpace &sp, const FeatGeom &g, const RadiusPlan &p, const double *feat,
                               uint64_t cap, uint64_t n_end, const double *qfeat, uint32_t nq, double r,
                               uint32_t *counts /* [nq][chunks] */, hipStream_t st);
hipError_t launch_radius_fill(const DevSpace &sp, const FeatGeom &g, const RadiusPlan &p, const double *feat,
                              uint64_t cap, uint64_t n_end, const double *qfeat, uint32_t nq, double r,
                              const uint64_t *offsets /* [nq*chunks] exclusive */, uint32_t *ids, double *dists,
                              hipStream_t st);

// device feature computation for raw AoS queries (device-resident API)
hipError_t launch_features(const DevSpace &sp, const FeatGeom &g, const double *raw, uint32_t n, double *feat,
                           hipStream_t st);
// scatter AoS features of n new states into SoA storage at [first, first+n)
hipError_t launch_store_soa(const double *aos, uint32_t n, int width, double *soa, uint64_t cap, uint64_t first,
                            hipStream_t st);
// tree-sharded kNN: merge `lists` per-shard [nq][k] lists (each sorted by (distance, id)) into one
hipError_t launch_csr_merge(const uint64_t *offs, uint32_t lists, uint32_t nq, const uint32_t *ids, const double *d,
                            uint64_t stride, uint64_t *out_off, uint32_t *out_i, double *out_d, hipStream_t st);
hipError_t launch_topk_merge(const double *d, const uint32_t *ids, uint32_t lists, uint32_t nq, uint32_t k, double *od,
                             uint32_t *oi, hipStream_t st);
// RRT steer: from = raw[nearest], to = q or interpolate(from, q, maxd/d)
hipError_t launch_steer(const DevSpace &sp, const double *raw_soa, uint64_t cap, const double *q, uint32_t nq,
                        const uint32_t *nearest, uint32_t stride, double maxd, double *from, double *to,
                        hipStream_t st);

// motion validation: one thread per edge
hipError_t launch_motion(const DevSpace &sp, const DevChecker &ck, const double *s1, const double *s2, uint32_t m,
                         uint8_t *valid, int32_t *nd, int32_t *first_invalid, unsigned long long *counters,
                         hipStream_t st);
// the edges of a neighbour query (launch_edges' pairs) checked without materialising them; returns
// hipErrorNotSupported for a space / checker without a fixed-width motion form
hipError_t launch_motion_edges(const DevSpace &sp, const DevChecker &ck, const double *q, const uint32_t *qidx,
                               const uint32_t *ids, uint32_t stride, int from_query, const double *aos, int da,
                               uint32_t m, uint8_t *valid, unsigned long long *counters, hipStream_t st);
hipError_t launch_state_valid(const DevSpace &sp, const DevChecker &ck, const double *s, uint32_t m, uint8_t *valid,
                              hipStream_t st);
// getMotionStates: states per motion (SpaceInformation.cpp:201-275 with alloc = true)
// in 64 bits: count near UINT32_MAX must not wrap (the C ABI rejects count > UINT32_MAX - 2)
inline uint64_t motion_states_per(uint32_t count, int endpoints) { return (uint64_t)count + (endpoints ? 2u : 0u); }
hipError_t launch_motion_states(const DevSpace &sp, const double *s1, const double *s2, uint32_t m, uint32_t count,
                                int endpoints, double *out, hipStream_t st);
// StateSpace::distance (t == NULL: out[m]) or StateSpace::interpolate at t[i] (out[m][dim]) per pair
hipError_t launch_space_pairs(const DevSpace &sp, const double *a, const double *b, const double *t, uint32_t m,
                              double *out, hipStream_t st);

}  // namespace ompl_amd
