/*
 * ompl_gpu.h — C ABI of the MI355X (gfx950) backend for OMPL's data-parallel
 * inner loops: NearestNeighbors queries and DiscreteMotionValidator sweeps.
 *
 * The ABI is plain C: pointers, sizes and status codes; no C++ or torch types.
 * It is what the C++ plugin classes in include/ompl_amd/ (drop-ins for the
 * reference's ompl::NearestNeighbors<_T> and ompl::base::MotionValidator)
 * call, and what a ctypes / cgo / JNI binding would bind.
 *
 * Reference interfaces each entry point replaces (paths relative to the
 * reference repo, OMPL 1.6.0):
 *   ompl_gpu_nn_add        NearestNeighbors<_T>::add(data) / add(vector)
 *                          src/ompl/datastructures/NearestNeighbors.h:76-85,
 *                          NearestNeighborsGNAT.h:147-176
 *   ompl_gpu_nn_remove     NearestNeighbors<_T>::remove          NearestNeighbors.h:88,
 *                          NearestNeighborsGNAT.h:190-207
 *   ompl_gpu_nn_clear      NearestNeighbors<_T>::clear           NearestNeighbors.h:73
 *   ompl_gpu_nn_size       NearestNeighbors<_T>::size            NearestNeighbors.h:107
 *   ompl_gpu_nn_knn        nearest (k=1) / nearestK              NearestNeighbors.h:91-98,
 *                          NearestNeighborsGNAT.h:209-233, NearestNeighborsLinear.h:98-131
 *   ompl_gpu_nn_radius     nearestR                              NearestNeighbors.h:100-105,
 *                          NearestNeighborsGNAT.h:236-245, NearestNeighborsLinear.h:135-142
 *   ompl_gpu_mv_check      DiscreteMotionValidator::checkMotion(s1,s2) and
 *                          checkMotion(s1,s2,lastValid)
 *                          src/ompl/base/src/DiscreteMotionValidator.cpp:48-145
 *   ompl_gpu_mv_counters   MotionValidator::getValidMotionCount/getInvalidMotionCount
 *                          src/ompl/base/MotionValidator.h:102-139
 *   ompl_gpu_svc_check     StateValidityChecker::isValid         src/ompl/base/StateValidityChecker.h:111
 *   ompl_gpu_svc_check_host  the same predicate on the host CPU (single-state isValid)
 *   ompl_gpu_nn_distance_host  StateSpace::distance of the handle's space on the host
 *                          (NearestNeighbors::setDistanceFunction verify mode, NearestNeighbors.h:58-61)
 *   ompl_gpu_rng_*         RNG::setSeed / getSeed                src/ompl/util/src/RandomNumbers.cpp:208-216
 *   ompl_gpu_sampler_*     StateSpace::allocStateSampler + StateSampler::sampleUniform
 *                          src/ompl/base/src/StateSpace.cpp:800-806, :1118-1128,
 *                          base/src/StateSampler.cpp:47-52, spaces/src/RealVectorStateSpace.cpp:45-53,
 *                          spaces/src/SO3StateSpace.cpp:99-102
 *   ompl_gpu_steer_device  the RRT extend step (nearest -> interpolate to range)
 *                          src/ompl/geometric/planners/rrt/src/RRT.cpp:137-146
 *   ompl_gpu_rrt_grow_device  the RRT loop itself                 RRT.cpp:128-192
 *   ompl_gpu_rrtstar_batch_device  RRT*'s iterations (geometric part) RRTstar.cpp:247-542, :603-618
 *   ompl_gpu_rrtstar_tree_* / _stage / _commit  RRT*'s cost logic (parent choice, rewiring)
 *                          RRTstar.cpp:285-457, :620-643
 *   ompl_gpu_prm_add_milestones  PRM* causal roadmap batches      prm/src/PRM.cpp:562-596
 *   ompl_gpu_knn_merge_device  per-shard nearestK lists -> global top k (tree-sharded mode)
 *   ompl_gpu_csr_merge_device  per-shard nearestR CSR results -> one CSR (tree-sharded mode)
 *   ompl_gpu_nn_edges_device  the edges PRM / BIT* check after a neighbour query
 *                          prm/src/PRM.cpp:577-582, informedtrees/src/BITstar.cpp:815
 *   ompl_gpu_mv_check_edges_device  checkMotion over those edges, read in place
 *                          BITstar.cpp:815, PRM.cpp:582, DiscreteMotionValidator.cpp:93-145
 *
 * Distances are the reference's fp64 formulas in the reference's operation
 * order (StateSpace.cpp:1068-1076, RealVectorStateSpace.cpp:230-242,
 * SO3StateSpace.cpp:254-262, demos/KinematicChain.h:105-124).
 *
 * State layout across the ABI: AoS rows of `dim` doubles (OMPL copyToReals
 * order): R^n -> n values; SO3 -> qx,qy,qz,qw; SE3 -> x,y,z,qx,qy,qz,qw;
 * KCHAIN -> n joint angles.  Ids are insertion indices (0,1,2,...).
 *
 * Errors: every call returns ompl_gpu_status and never throws or aborts;
 * ompl_gpu_last_error() gives the thread's last message.  nearest on an empty
 * set returns OMPL_GPU_ERR_EMPTY, which the C++ wrapper turns into the
 * reference's ompl::Exception("No elements found in nearest neighbors data
 * structure") (NearestNeighborsGNAT.h:218).
 *
 * Threading: one handle = one device + one HIP stream + an internal mutex;
 * const queries on one handle from several threads are serialised safely.
 * add/remove need external exclusion as in the reference (pRRT.cpp:119-141).
 */
#ifndef OMPL_GPU_H
#define OMPL_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OMPL_GPU_ABI_VERSION 1

typedef enum ompl_gpu_status {
    OMPL_GPU_OK = 0,
    OMPL_GPU_ERR_INVALID_ARG = 1,
    OMPL_GPU_ERR_EMPTY = 2,       /* "No elements found in nearest neighbors data structure" */
    OMPL_GPU_ERR_DEVICE = 3,      /* HIP runtime error / no device */
    OMPL_GPU_ERR_OOM = 4,
    OMPL_GPU_ERR_UNSUPPORTED = 5, /* e.g. k above the largest compiled bucket */
    OMPL_GPU_ERR_NOT_FOUND = 6    /* remove() of an unknown / already removed id */
} ompl_gpu_status;

/* ---- state spaces (closed set of device metrics) --------------------------
 * REALVECTOR : RealVectorStateSpace(n)                 RealVectorStateSpace.cpp:230-265
 * SO3        : SO3StateSpace                           SO3StateSpace.cpp:254-318
 * SE3        : SE3StateSpace = R^3 (w0) + SO3 (w1)     SE3StateSpace.h:114-121, StateSpace.cpp:1068-1116
 * KCHAIN     : KinematicChainSpace(n, linkLength)      demos/KinematicChain.h:87-175
 */
enum {
    OMPL_GPU_SPACE_REALVECTOR = 0,
    OMPL_GPU_SPACE_SO3 = 1,
    OMPL_GPU_SPACE_SE3 = 2,
    OMPL_GPU_SPACE_KCHAIN = 3
};

typedef struct ompl_gpu_space {
    int32_t kind;
    int32_t dim;          /* reals per state: n, 4 (SO3), 7 (SE3) */
    double weight[2];     /* SE3 component weights (CompoundStateSpace::weights_), normally {1,1} */
    double lvs[2];        /* longestValidSegment_ per component: [0] R^n / chain / SE3's R^3, [1] SE3's SO3 */
    uint32_t factor[2];   /* longestValidSegmentCountFactor_ per component (StateSpace.cpp:851-854) */
    double link_length;   /* KCHAIN only */
} ompl_gpu_space;

/* ---- device validity checkers (closed set) --------------------------------
 * ALL_VALID : AllValidStateValidityChecker            StateValidityChecker.h:165-183
 * HYPERCUBE : narrow-passage hypercube on the first ndim reals
 *                                                     demos/HypercubeBenchmark.cpp:57-72
 * SPHERES   : 3-D sphere obstacles on the first 3 reals (SE3 translation); the
 *             3-D extension of Circles2D::noOverlap   tests/resources/circles2D.h:139-150
 * KCHAIN    : KinematicChainValidityChecker           demos/KinematicChain.h:193-277
 * CIRCLES2D : Circles2D::noOverlap on (x,y)            tests/resources/circles2D.h:139-150
 */
enum {
    OMPL_GPU_CHECK_ALL_VALID = 0,
    OMPL_GPU_CHECK_HYPERCUBE = 1,
    OMPL_GPU_CHECK_SPHERES = 2,
    OMPL_GPU_CHECK_KCHAIN = 3,
    OMPL_GPU_CHECK_CIRCLES2D = 4
};

typedef struct ompl_gpu_checker {
    int32_t kind;
    int32_t ndim;         /* HYPERCUBE: number of leading reals tested */
    double edge_width;    /* HYPERCUBE */
    int32_t count;        /* SPHERES / CIRCLES2D: obstacles; KCHAIN: environment segments */
    int32_t reserved;
    const double *data;   /* SPHERES: count x (cx,cy,cz,r^2); CIRCLES2D: count x (x,y,r^2);
                             KCHAIN: count x (x0,y0,x1,y1).  Copied at create time. */
} ompl_gpu_checker;

typedef struct ompl_gpu_nn ompl_gpu_nn;
typedef struct ompl_gpu_mv ompl_gpu_mv;

/* ---- library ---------------------------------------------------------------- */
int ompl_gpu_abi_version(void);
const char *ompl_gpu_last_error(void);
ompl_gpu_status ompl_gpu_device_count(int *count);
void ompl_gpu_free(void *p); /* frees buffers the library returned (radius CSR) */

/* ---- nearest neighbours ----------------------------------------------------- */
ompl_gpu_status ompl_gpu_nn_create(ompl_gpu_nn **out, const ompl_gpu_space *space, int device);
ompl_gpu_status ompl_gpu_nn_destroy(ompl_gpu_nn *h);
/* Launch on a caller-owned hipStream_t (NULL restores the handle's own stream). */
ompl_gpu_status ompl_gpu_nn_set_stream(ompl_gpu_nn *h, void *hip_stream);
ompl_gpu_status ompl_gpu_nn_sync(ompl_gpu_nn *h);
/* Append n AoS states; *first_id (may be NULL) receives the id of the first one. */
ompl_gpu_status ompl_gpu_nn_add(ompl_gpu_nn *h, const double *states, size_t n, uint64_t *first_id);
ompl_gpu_status ompl_gpu_nn_remove(ompl_gpu_nn *h, uint64_t id);
ompl_gpu_status ompl_gpu_nn_clear(ompl_gpu_nn *h);
ompl_gpu_status ompl_gpu_nn_size(const ompl_gpu_nn *h, size_t *live, size_t *total);
/* Copy back the stored states (AoS), ids [first, first+n). */
ompl_gpu_status ompl_gpu_nn_get_states(ompl_gpu_nn *h, uint64_t first, size_t n, double *out);
/* k nearest per query, host buffers, synchronous.  Results sorted by
 * (distance, id) ascending; out_ids/out_dist are nq x k, out_cnt[q] = number
 * of valid results (min(k, live)).  k == 0 returns counts of 0.  With no live
 * element, counts are 0 and the call returns OMPL_GPU_ERR_EMPTY only if k==1
 * was requested through ompl_gpu_nn_nearest. */
ompl_gpu_status ompl_gpu_nn_knn(ompl_gpu_nn *h, const double *queries, size_t nq, uint32_t k,
                                uint64_t *out_ids, double *out_dist, uint32_t *out_cnt);
ompl_gpu_status ompl_gpu_nn_nearest(ompl_gpu_nn *h, const double *queries, size_t nq,
                                    uint64_t *out_ids, double *out_dist);
/* All elements with distance <= r (inclusive), sorted by (distance, id).
 * *ids / *dists are library-allocated CSR payloads (free with ompl_gpu_free);
 * offsets has nq+1 entries. */
ompl_gpu_status ompl_gpu_nn_radius(ompl_gpu_nn *h, const double *queries, size_t nq, double r,
                                   uint64_t **ids, double **dists, uint64_t *offsets);
/* The handle's metric on the host: out[i] = distance(a[i], b[i]) for m pairs of AoS states, in
 * the reference's operation order (host libm). */
ompl_gpu_status ompl_gpu_nn_distance_host(const ompl_gpu_nn *h, const double *a, const double *b, size_t m,
                                          double *out);
/* Device-resident variants: all pointers are device memory, the call is
 * asynchronous on the handle's stream.  queries are AoS fp64; ids are uint32
 * (0xFFFFFFFF = no result); dist fp64. */
ompl_gpu_status ompl_gpu_nn_knn_device(ompl_gpu_nn *h, const double *d_queries, size_t nq, uint32_t k,
                                       uint32_t *d_ids, double *d_dist);
/* Path selection and counters.  mode (exact_only) 0 = default: batched R^n / SO3 / SE3
 * queries use the fp32 screen + fp64 certificate, culled over a Morton-sorted copy of the
 * store for R^n and SE3; 1 = the exact fp64 scan only; 2 = the screen without culling.
 * Results are identical in every mode (uncertified queries are re-run exactly).
 * *screened counts queries that took the screen, *fallbacks those re-run exactly. */
ompl_gpu_status ompl_gpu_nn_set_exact(ompl_gpu_nn *h, int exact_only);
ompl_gpu_status ompl_gpu_nn_stats(const ompl_gpu_nn *h, uint64_t *screened, uint64_t *fallbacks);
/* Of those *fallbacks: *full counts the queries whose bounded exact re-run (one pass over the
 * store for all uncertified queries, keeping d <= the certificate's exact k-th distance)
 * exceeded its candidate cap and took the full exact scan. */
ompl_gpu_status ompl_gpu_nn_rerun_stats(const ompl_gpu_nn *h, uint64_t *full);
/* Large-k select (k > 61 on SE3 / R^n, RRT*'s k = 6,169): queries whose candidates overflowed a
 * per-chunk slab into the query's pool (a store whose id order follows space), and queries the
 * select could not answer (sampling short-count, pool overflow) and re-ran on the exact fallback,
 * summed over calls.  Synchronises the handle's stream. */
ompl_gpu_status ompl_gpu_nn_large_stats(ompl_gpu_nn *h, uint64_t *spilled, uint64_t *exact);
/* Bring the culled walks' sorted copy up to date now (a device k-d build, or placing the states
 * added since the last call in its tail) instead of at the next batched query; asynchronous on
 * the handle's stream.  No-op for spaces without a culled walk (SO3, KCHAIN). */
ompl_gpu_status ompl_gpu_nn_build_index(ompl_gpu_nn *h);
/* The culled walks' sorted copy: device k-d builds and tail appends (states added since the
 * last build placed along the Morton curve without a rebuild) performed so far. */
ompl_gpu_status ompl_gpu_nn_index_stats(const ompl_gpu_nn *h, uint64_t *builds, uint64_t *appends);
/* Group walk: 64-state tiles fetched, summed over query groups, vs the tiles a full scan
 * by the same groups would have touched; *query_tiles counts (tile, query) scans, i.e.
 * 64 distance evaluations each.  Any output may be NULL. */
ompl_gpu_status ompl_gpu_nn_cull_stats(ompl_gpu_nn *h, uint64_t *tiles_scanned, uint64_t *tiles_total,
                                       uint64_t *query_tiles);
/* Profiling: when enabled, each query call brackets its dominant scan kernel with HIP
 * events recorded on the launch stream; kernel_time synchronises the stream and returns
 * the summed duration, the number of bracketed launches and the kernel's name. */
ompl_gpu_status ompl_gpu_nn_profile(ompl_gpu_nn *h, int enable);
ompl_gpu_status ompl_gpu_nn_kernel_time(ompl_gpu_nn *h, double *total_ms, uint64_t *launches,
                                        const char **kernel_name);
/* Device-resident nearestR: d_queries AoS fp64 (device).  The CSR result goes to
 * caller-owned device buffers: d_offsets (nq+1 entries, uint64), d_ids (uint32) / d_dist
 * (fp64) of `capacity` entries, sorted by (distance, id) inside each query's segment
 * (NearestNeighborsGNAT.h:236-245, NearestNeighborsLinear.h:135-142).  *total receives the
 * number of results; when it exceeds capacity only d_offsets is written and the call
 * returns OMPL_GPU_ERR_INVALID_ARG (call again with *total entries).  Synchronous. */
ompl_gpu_status ompl_gpu_nn_radius_device(ompl_gpu_nn *h, const double *d_queries, size_t nq, double r,
                                          uint64_t *d_offsets, uint32_t *d_ids, double *d_dist, uint64_t capacity,
                                          uint64_t *total);
/* Radius walk: 64-state tiles fetched and (tile, query) pairs scanned (64 distance
 * evaluations each), summed over nearestR calls.  Either output may be NULL. */
ompl_gpu_status ompl_gpu_nn_radius_cull_stats(ompl_gpu_nn *h, uint64_t *tiles_scanned, uint64_t *query_tiles);
/* Culled nearestR calls answered by the one walk into per-query slabs, and those whose longest
 * segment overflowed the slab (count walk + fill walk; the next call's slab grows to it). */
ompl_gpu_status ompl_gpu_nn_radius_path_stats(ompl_gpu_nn *h, uint64_t *one_pass, uint64_t *two_pass);
/* Motion endpoints of a batch of neighbour results — the edges the planners check after a
 * neighbour query: PRM checkMotion(state[n], state[m]) (PRM.cpp:577-582, from_query = 0),
 * BIT* checkMotion(vertex, sample) (BITstar.cpp:815, from_query = 1).  Edge e pairs query q
 * (d_queries, AoS) with stored state d_ids[e]: e in [d_offsets[q], d_offsets[q+1]) for a CSR
 * result (nn_radius_device), or, with d_offsets NULL, e = q * stride + j for a dense
 * nq x stride id matrix (nn_knn_device; m == nq * stride).  A missing id (0xFFFFFFFF)
 * pairs q with itself.  Writes m AoS rows to d_from / d_to; asynchronous.  With a CSR,
 * m may differ from d_offsets[nq]: only edges e < min(m, d_offsets[nq]) are written. */
ompl_gpu_status ompl_gpu_nn_edges_device(ompl_gpu_nn *h, const double *d_queries, size_t nq, const uint64_t *d_offsets,
                                         const uint32_t *d_ids, uint32_t stride, size_t m, int from_query,
                                         double *d_from, double *d_to);
/* RRT extend on device: for each query q with nearest id nid[q*stride]:
 * from = state[nid]; to = q; if d(from,q) > max_distance, to = interpolate(from,
 * q, max_distance/d).  Writes AoS from/to rows (RRT.cpp:137-146).  A missing id (0xFFFFFFFF)
 * gives from = to = q (a motion of length 0: checkMotion then tests q alone). */
ompl_gpu_status ompl_gpu_steer_device(ompl_gpu_nn *h, const double *d_queries, size_t nq,
                                      const uint32_t *d_nearest, uint32_t stride, double max_distance,
                                      double *d_from, double *d_to);

/* ---- motion validation ------------------------------------------------------ */
ompl_gpu_status ompl_gpu_mv_create(ompl_gpu_mv **out, const ompl_gpu_space *space,
                                   const ompl_gpu_checker *checker, int device);
ompl_gpu_status ompl_gpu_mv_destroy(ompl_gpu_mv *h);
ompl_gpu_status ompl_gpu_mv_set_stream(ompl_gpu_mv *h, void *hip_stream);
ompl_gpu_status ompl_gpu_mv_sync(ompl_gpu_mv *h);
/* m edges (s1[i] -> s2[i]), host AoS.  valid[i] = checkMotion(s1,s2) (s1 is
 * assumed valid and never checked, DiscreteMotionValidator.cpp:95-96);
 * nd[i] = validSegmentCount; first_invalid[i] = first invalid sample of the
 * lastValid variant (j in [1,nd-1]; nd when only s2 fails; -1 when valid).
 * nd / first_invalid may be NULL.  Updates the valid/invalid counters. */
ompl_gpu_status ompl_gpu_mv_check(ompl_gpu_mv *h, const double *s1, const double *s2, size_t m,
                                  uint8_t *valid, int32_t *nd, int32_t *first_invalid);
ompl_gpu_status ompl_gpu_mv_check_device(ompl_gpu_mv *h, const double *d_s1, const double *d_s2, size_t m,
                                         uint8_t *d_valid, int32_t *d_nd, int32_t *d_first_invalid);
/* checkMotion over the edges of a neighbour result, without materialising them: edge e is the pair
 * ompl_gpu_nn_edges_device(nn, ...) would write (the same d_queries / d_offsets / d_ids / stride /
 * from_query meaning), read in place from the query rows and the stored states of nn —
 * BITstar.cpp:815 checkMotion(vertex, sample), PRM.cpp:582 checkMotion(state[n], state[m]).
 * d_valid[e] and the counters as ompl_gpu_mv_check_device; an edge past the last CSR segment
 * (e >= d_offsets[nq]) reports 0 and is not counted.  Runs on the validator's stream, after the
 * work queued on nn's stream; asynchronous.  Spaces / checkers without a fixed-width motion form
 * (the KinematicChain, R^n other than 2 / 3 / 6) materialise the pairs in the validator's scratch
 * (that form reads d_offsets[nq] back: it synchronises). */
ompl_gpu_status ompl_gpu_mv_check_edges_device(ompl_gpu_mv *mv, ompl_gpu_nn *nn, const double *d_queries, size_t nq,
                                               const uint64_t *d_offsets, const uint32_t *d_ids, uint32_t stride,
                                               size_t m, int from_query, uint8_t *d_valid);
ompl_gpu_status ompl_gpu_mv_counters(ompl_gpu_mv *h, uint64_t *valid, uint64_t *invalid);
ompl_gpu_status ompl_gpu_mv_reset_counters(ompl_gpu_mv *h);
/* total isValid() evaluations the bisection variant made (the reference's work). */
ompl_gpu_status ompl_gpu_mv_state_checks(ompl_gpu_mv *h, uint64_t *checks);
/* isValid per state (host AoS, evaluated on the device). */
ompl_gpu_status ompl_gpu_svc_check(ompl_gpu_mv *h, const double *states, size_t m, uint8_t *valid);
/* the same predicate evaluated on the host CPU, from the same source as the device code
 * (bit-identical wherever the predicate calls no libm function; the KCHAIN checker's cos / sin
 * are glibc's here, the device math library's there).  For single-state isValid calls, where a
 * device round trip costs more than the predicate. */
ompl_gpu_status ompl_gpu_svc_check_host(ompl_gpu_mv *h, const double *states, size_t m, uint8_t *valid);
/* device-resident batch: d_states AoS fp64, d_valid one byte per state; asynchronous. */
ompl_gpu_status ompl_gpu_svc_check_device(ompl_gpu_mv *h, const double *d_states, size_t m, uint8_t *d_valid);
/* SpaceInformation::getMotionStates(s1, s2, states, count, endpoints, alloc = true)
 * (src/ompl/base/src/SpaceInformation.cpp:201-275) for m motions: out = [m][per][dim] with
 * per = count + (endpoints ? 2 : 0) = the function's return value — [s1], the states at
 * j / (count + 1) for j in [1, count], [s2].  Host AoS / device-resident variants. */
ompl_gpu_status ompl_gpu_mv_motion_states(ompl_gpu_mv *h, const double *s1, const double *s2, size_t m,
                                          uint32_t count, int endpoints, double *out);
ompl_gpu_status ompl_gpu_mv_motion_states_device(ompl_gpu_mv *h, const double *d_s1, const double *d_s2, size_t m,
                                                 uint32_t count, int endpoints, double *d_out);
/* StateSpace::distance(a[i], b[i]) (t == NULL: out[m]) or StateSpace::interpolate(a[i], b[i], t[i])
 * (out[m][dim], AoS) for m pairs, evaluated by the device fp64 code the kernels use — the
 * reference's virtuals RealVectorStateSpace.cpp:230-265, SO3StateSpace.cpp:254-318 (arcLength,
 * slerp), CompoundStateSpace StateSpace.cpp:1068-1116 (SE3), KinematicChain.h:105-175.  Host AoS
 * (synchronous) / device-resident (asynchronous on the handle's stream) variants. */
ompl_gpu_status ompl_gpu_mv_space_pairs(ompl_gpu_mv *h, const double *a, const double *b, const double *t, size_t m,
                                        double *out);
ompl_gpu_status ompl_gpu_mv_space_pairs_device(ompl_gpu_mv *h, const double *d_a, const double *d_b, const double *d_t,
                                               size_t m, double *d_out);

/* ---- PRM* roadmap construction, causal batches ------------------------------------
 * PRM::addMilestone (geometric/planners/prm/src/PRM.cpp:562-596) with KStarStrategy
 * (ConnectionStrategy.h:124-156) for m new milestones (host AoS, in insertion order) after the
 * n0 states already stored: milestone j (id n0 + j) connects to its
 * k_j = ceil(k_const * ln(n0 + j + 1)) nearest among ALL earlier vertices — the stored states and
 * the milestones j' < j of the batch — sorted by (distance, id); every edge is checked with mv's
 * checkMotion(state[neighbour], state[milestone]) (PRM.cpp:582, counters updated); then the m
 * milestones are added to nn (PRM.cpp:593).  k_const = e + e / dim (PRM*).  Only milestones
 * [j0, j1) get neighbours and edges (a rank's share of a batch every rank inserts whole; the full
 * batch is [0, m)).  Outputs (device, caller-owned, (j1 - j0) x k_cap, k_cap >= the batch's largest
 * k, <= 64): d_nbr neighbour ids (0xFFFFFFFF past d_cnt[r]), d_cnt, d_valid (1 = the edge is
 * valid).  *edges (may be NULL) = edges checked.  Synchronous; equal to the sequential loop's
 * result (tests/test_gpu_prm.py). */
ompl_gpu_status ompl_gpu_prm_add_milestones(ompl_gpu_nn *nn, ompl_gpu_mv *mv, const double *states, size_t m,
                                            size_t j0, size_t j1, double k_const, uint32_t k_cap, uint32_t *d_nbr,
                                            uint32_t *d_cnt, uint8_t *d_valid, uint64_t *edges);

/* LazyPRM::addMilestone (geometric/planners/prm/src/LazyPRM.cpp:285-309) with its star strategy
 * (LazyPRM.cpp:238-239): the same neighbours as ompl_gpu_prm_add_milestones, but no edge is
 * checked (validity stays unknown until a path search needs it); d_dist (may be NULL) receives each
 * edge's weight, motionCost = distance(milestone, neighbour) under the path-length objective
 * (LazyPRM.cpp:299), +inf past d_cnt[r].  Synchronous. */
ompl_gpu_status ompl_gpu_lazyprm_add_milestones(ompl_gpu_nn *nn, const double *states, size_t m, size_t j0, size_t j1,
                                                double k_const, uint32_t k_cap, uint32_t *d_nbr, uint32_t *d_cnt,
                                                double *d_dist);

/* ---- RRT growth on device ----------------------------------------------------
 * The RRT loop (RRT.cpp:128-192) without its goal test, for ns samples in order: nearest
 * stored state (:137), steer to max_distance (:141-146), mv's checkMotion(nearest,
 * steered) (:148) and, when valid, append the steered state to the NN store (:170-173).
 * Sample i sees every state samples < i appended, as in the sequential loop.
 * d_nearest[i] = id of sample i's nearest state, d_added[i] = id of the appended state or
 * 0xFFFFFFFF.  d_samples are ns AoS rows (device).  Both handles must describe the same
 * space (R^n, SO3 or SE3) on the same device; mv's valid / invalid counters are updated.
 * All iterations are queued on the NN handle's stream with no host round trip;
 * synchronous on return.  The persistent one-launch form gives up when a grid-wide wait
 * outlives its spin limit (the device shared with a long kernel); the batch is then re-run in
 * the two-launch form from the same start (counters restored), with identical results. */
ompl_gpu_status ompl_gpu_rrt_grow_device(ompl_gpu_nn *nn, ompl_gpu_mv *mv, const double *d_samples, size_t ns,
                                         double max_distance, uint32_t *d_nearest, uint32_t *d_added);
/* The same loop with RRT's goal test (RRT.cpp:175-187): after each added state,
 * GoalRegion::isSatisfied — distance(state, goal) < goal_threshold (GoalRegion.cpp:52-58; the
 * threshold of ProblemDefinition::setStartAndGoalStates defaults to DBL_EPSILON) — ends the run:
 * *solved_at = that iteration (~0 if none), the samples after it are not processed (their
 * d_nearest / d_added are 0xFFFFFFFF).  Otherwise the added state strictly closest to the goal
 * is the approximate solution: *approx_id / *approx_dist (0xFFFFFFFF / +inf if nothing was
 * added).  goal: host, dim reals.  Output pointers may be NULL. */
/* Tree-sharded nearestK (SURVEY §8e "state set sharded, queries broadcast"): every shard's
 * [nq][k] result of the same queries — ids already global, each list sorted by (distance, id),
 * missing entries (+inf, 0xFFFFFFFF) — stacked as d_dist / d_ids [lists][nq][k] (the layout an
 * all_gather produces), merged into the global top k by (distance, id): the order of
 * NearestNeighborsGNAT::nearestK over the union (NearestNeighborsGNAT.h:222-233).  Device
 * pointers, asynchronous on `stream` (a hipStream_t; NULL = the null stream).  lists <= 64. */
ompl_gpu_status ompl_gpu_knn_merge_device(const double *d_dist, const uint32_t *d_ids, uint32_t lists, size_t nq,
                                          uint32_t k, double *d_out_dist, uint32_t *d_out_ids, void *stream);
/* Tree-sharded nearestR (SURVEY §8e "Radius search"): `lists` shards' CSR results of the same nq
 * queries — shard l: offsets d_offsets[l * (nq + 1) + 0..nq] (uint64), ids (global, uint32) and
 * distances at d_ids / d_dist + l * stride, each segment sorted by (distance, id) — merged into
 * one CSR: d_out_offsets[nq + 1], segment q the union of the shards' segments in (distance, id)
 * order (NearestNeighborsGNAT.h:236-245).  d_out_ids / d_out_dist hold sum_l d_offsets[l][nq]
 * entries.  Device pointers, asynchronous on `stream`.  lists <= 1024. */
ompl_gpu_status ompl_gpu_csr_merge_device(const uint64_t *d_offsets, uint32_t lists, size_t nq, const uint32_t *d_ids,
                                          const double *d_dist, size_t stride, uint64_t *d_out_offsets,
                                          uint32_t *d_out_ids, double *d_out_dist, void *stream);
/* Persistent RRT runs that gave up and were re-run in the two-launch form (diagnostics). */
ompl_gpu_status ompl_gpu_rrt_aborts(const ompl_gpu_nn *nn, uint64_t *aborts);
ompl_gpu_status ompl_gpu_rrt_solve_device(ompl_gpu_nn *nn, ompl_gpu_mv *mv, const double *d_samples, size_t ns,
                                          double max_distance, const double *goal, double goal_threshold,
                                          uint32_t *d_nearest, uint32_t *d_added, uint64_t *solved_at,
                                          uint32_t *approx_id, double *approx_dist);

/* ---- RRT* iteration batches ----------------------------------------------------
 * RRTstar::solve (geometric/planners/rrt/src/RRTstar.cpp:247-542) with its defaults (k-nearest
 * neighbourhoods, useKNearest_ RRTstar.h:445; delayed collision checking, delayCC_ :458; no
 * new-state rejection or pruning) for ns samples in order: nmotion = nearest(s_i) (:266); x_i =
 * s_i, or interpolate(nmotion, s_i, max_distance / d) when d > max_distance (:271-279); when
 * mv's checkMotion(nmotion, x_i) holds (:282), x_i joins the tree (:410) after its neighbourhood
 * nearestK(x_i, k_i), k_i = ceil(k_rrt * ln(size + 1)) over the tree as it stands (getNeighbors
 * :603-618), is taken.  Sample i sees every state samples < i added, as in the sequential loop.
 * This is the geometric part of every iteration: which states join, the neighbourhoods, and both
 * motion bits of every (neighbour, x_i) pair — checkMotion(nbh, x_i) for the parent choice in
 * cost order (:319-357) and checkMotion(x_i, nbh) for the rewiring (:414-440) — so the planner's
 * cost logic needs only lookups (ompl_gpu_rrtstar_commit below).  None of it depends on costs.
 * Inputs: d_samples ns AoS rows (device).  Outputs (device, caller-owned, ns entries each, may be
 * NULL): d_nearest[i] = id of nmotion; d_added[i] = the id x_i got, or 0xFFFFFFFF; d_inc[i] =
 * distance(nmotion, x_i) (the motion's incCost, :288); d_states[i] = x_i (dim reals).  The
 * neighbourhoods are library-owned device arrays, valid until the next call on nn: a CSR over the
 * samples (out->offsets, ns + 1 entries; empty for samples not added) of neighbour ids, their
 * distances distance(nbh, x_i) and bits (bit 0 = checkMotion(nbh, x_i), bit 1 = checkMotion(x_i,
 * nbh)), each segment sorted by (distance, id) and k_i long (fewer if the tree was smaller).
 * mv's counters are not updated (the planner performs only the checks its cost logic asks for).
 * Both handles describe the same space (R^n, SO3 or SE3) on the same device.  Synchronous. */
typedef struct ompl_gpu_rrtstar_result {
    const uint64_t *offsets; /* device, ns + 1 */
    const uint32_t *ids;     /* device, total */
    const double *dist;      /* device, total */
    const uint8_t *bits;     /* device, total */
    uint64_t total;          /* neighbourhood entries */
    uint64_t added;          /* samples whose state joined the tree */
    uint32_t rounds;         /* fixed-point rounds over the batch's in-batch nearest states */
    uint32_t reserved;
} ompl_gpu_rrtstar_result;
ompl_gpu_status ompl_gpu_rrtstar_batch_device(ompl_gpu_nn *nn, ompl_gpu_mv *mv, const double *d_samples, size_t ns,
                                              double max_distance, double k_rrt, uint32_t *d_nearest,
                                              uint32_t *d_added, double *d_inc, double *d_states,
                                              ompl_gpu_rrtstar_result *out);

/* ---- RRT* cost logic -----------------------------------------------------------
 * The tree's costs as RRTstar keeps them in its Motions (RRTstar.h:347-372: parent, incCost,
 * cost, children), indexed by the nearest-neighbour ids, and the cost part of every iteration
 * (RRTstar.cpp:285-457, delayCC, the path-length objective) over the device batch's results:
 * the parent in cost order among the neighbours (:319-357), the rewiring (:414-457) with
 * removeFromParent / updateChildCosts (:620-643), each sample in order.  Host-side; a tree
 * belongs to one planner.  ompl_gpu_rrtstar_stage copies a batch's results to the host (device ->
 * host, synchronous on nn's stream, under nn's lock) and queues them; ompl_gpu_rrtstar_commit
 * processes the oldest queued batch.  stage and commit may run on two threads (the next device
 * batch then overlaps the previous batch's cost logic); commit, add and read must not overlap.
 * tree_add appends states: parent[j] is -1 (a start state, cost = the identity 0) or an earlier
 * id; NULL arrays mean -1 / 0 / 0.  commit writes per sample (when not NULL; ns_cap entries
 * available) the nearest id, the added id or -1, and the parent chosen or -1.
 * totals: [0] rewires, [1] checkMotion calls the sequential loop makes (the bits it looks up),
 * [2] states added, [3] neighbourhood entries, [4] samples, [5] child costs updateChildCosts
 * rewrote. */
typedef struct ompl_gpu_rrtstar_tree ompl_gpu_rrtstar_tree;
ompl_gpu_status ompl_gpu_rrtstar_tree_create(ompl_gpu_rrtstar_tree **out);
void ompl_gpu_rrtstar_tree_destroy(ompl_gpu_rrtstar_tree *t);
ompl_gpu_status ompl_gpu_rrtstar_tree_add(ompl_gpu_rrtstar_tree *t, size_t m, const int64_t *parent,
                                          const double *inc, const double *cost);
ompl_gpu_status ompl_gpu_rrtstar_tree_size(const ompl_gpu_rrtstar_tree *t, size_t *n);
ompl_gpu_status ompl_gpu_rrtstar_tree_read(const ompl_gpu_rrtstar_tree *t, size_t first, size_t m, int64_t *parent,
                                           double *inc, double *cost);
ompl_gpu_status ompl_gpu_rrtstar_tree_totals(const ompl_gpu_rrtstar_tree *t, uint64_t totals[6]);
ompl_gpu_status ompl_gpu_rrtstar_stage(ompl_gpu_rrtstar_tree *t, ompl_gpu_nn *nn, size_t ns, const uint32_t *d_nearest,
                                       const uint32_t *d_added, const double *d_inc,
                                       const ompl_gpu_rrtstar_result *res);
/* the same from host arrays (offsets: ns + 1 entries; a planner whose geometric part ran elsewhere) */
ompl_gpu_status ompl_gpu_rrtstar_stage_host(ompl_gpu_rrtstar_tree *t, size_t ns, const uint32_t *nearest,
                                            const uint32_t *added, const double *inc, const uint64_t *offsets,
                                            const uint32_t *ids, const double *dist, const uint8_t *bits);
ompl_gpu_status ompl_gpu_rrtstar_commit(ompl_gpu_rrtstar_tree *t, double max_distance, size_t ns_cap,
                                        int64_t *nearest, int64_t *added, int64_t *chosen, size_t *ns_out);

/* ---- BIT* batch sampling -----------------------------------------------------
 * BITstar::ImplicitGraph::updateSamples before a solution exists (ImplicitGraph.cpp:924-1000: the
 * informed sampler draws from its base sampler while the cost bound is infinite,
 * PathLengthDirectInfSampler.cpp:350-368): tries = 0; while tries < max_tries and
 * numSamples < num_required: draw one state from smp (sampleUniform), check it with mv's
 * StateValidityChecker, keep it if valid; then addToSamples appends the kept states to nn
 * (ImplicitGraph.cpp:682-692).  The caller passes num_samples = numSamples_ and
 * num_required = numSamples_ + numNewSamplesInCurrentBatch_, max_tries =
 * averageNumOfAllowedFailedAttemptsWhenSampling_ (2) * num_required.  The validity checks run
 * on the device in batches; smp's streams are left exactly after the last try the sequential
 * loop makes.  *tries = states drawn (= isValid calls, numStateCollisionChecks_), *first_id =
 * the first new id, *added = states appended.  nn, mv and smp describe the same space.
 * Synchronous.  Output pointers may be NULL. */
typedef struct ompl_gpu_sampler ompl_gpu_sampler;
ompl_gpu_status ompl_gpu_bitstar_update_samples(ompl_gpu_nn *nn, ompl_gpu_mv *mv, ompl_gpu_sampler *smp,
                                                uint64_t num_samples, uint64_t num_required, uint64_t max_tries,
                                                uint64_t *tries, uint64_t *first_id, uint64_t *added);

/* ---- the reference's input streams (host) ------------------------------------
 * ompl::RNG restated on the same standard-library engines (std::ranlux24_base seed generator,
 * std::mt19937 + std::uniform_real_distribution per RNG, RandomNumbers.cpp:53-279).
 * ompl_gpu_rng_set_seed = RNG::setSeed (call before any RNG is constructed for deterministic
 * streams); every sampler created afterwards draws its RNG seeds from that generator in the
 * reference's construction order. */
void ompl_gpu_rng_set_seed(uint32_t seed);
uint32_t ompl_gpu_rng_get_seed(void);
uint64_t ompl_gpu_rng_seeds_drawn(void); /* seeds handed out so far (observability) */
/* the seed an RNG() constructed now would take (RandomNumbers.cpp:218-223): draws it from the
 * generator — for mirroring the construction of an RNG that lives outside this library (a
 * planner's rng_, a GNAT's pivot selector) in the reference's order */
uint32_t ompl_gpu_rng_next_seed(void);
/* n x RNG(local_seed).uniformReal(low, high): an explicitly seeded RNG (RandomNumbers.cpp:225-228),
 * which draws nothing from the seed generator */
ompl_gpu_status ompl_gpu_rng_uniform_real(uint32_t local_seed, size_t n, double low, double high, double *out);
/* allocStateSampler of the space: SE3 = CompoundStateSampler + R^3 + SO3 samplers (3 seeds),
 * R^n / KCHAIN one RealVectorStateSampler, SO3 one SO3StateSampler.  low / high: bounds of the
 * R^n part (dim reals; SE3: 3), NULL = [0, 1] (KCHAIN: [-pi, pi], KinematicChain.h:87-100). */
ompl_gpu_status ompl_gpu_sampler_create(ompl_gpu_sampler **out, const ompl_gpu_space *space, const double *low,
                                        const double *high);
ompl_gpu_status ompl_gpu_sampler_destroy(ompl_gpu_sampler *s);
/* n successive sampleUniform calls, AoS rows (copyToReals order) */
ompl_gpu_status ompl_gpu_sampler_sample_uniform(ompl_gpu_sampler *s, size_t n, double *out);
/* local seeds of the sampler's RNGs in construction order (at most 3) */
ompl_gpu_status ompl_gpu_sampler_local_seeds(const ompl_gpu_sampler *s, uint32_t *seeds, int *count);

#ifdef __cplusplus
}
#endif
#endif /* OMPL_GPU_H */
