/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, IEEE double, no FMA contraction) of the reference
 * OMPL hot path that the MI355X backend replaces.  Only tests/, the smoke()
 * entry point and bench.py's cpu_baseline leg may load this library, and only
 * as the checker / the timed CPU baseline — never as the product path.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * the reference repo root, OMPL 1.6.0 fork).
 *
 * Parity pinning:
 *   - ranking / tie / empty / k>n semantics are checked against the reference's
 *     own NearestNeighborsLinear.h compiled unmodified (oracle/ref_linear.cpp,
 *     built into oracle/_ref/ by oracle/Makefile);
 *   - distance / interpolation formulas are checked against the reference
 *     tests' known answers (tests/base/state_spaces.cpp:197-300,
 *     tests/base/StateSpaceTest.h:72-112) in tests/test_oracle.py;
 *   - GNAT (oracle/gnat.cpp) is checked against Linear exactly as the
 *     reference test does (tests/datastructures/nearestneighbors.cpp:147-184).
 *   The motion validator and the validity checkers live in reference sources
 *   that need Boost/Eigen (absent here) and cannot be compiled: they are pinned
 *   only by restatement + the property tests; see DESIGN.md "Oracle".
 */
#ifndef OMPL_AMD_ORACLE_H
#define OMPL_AMD_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/ompl_gpu.h" /* shared space / checker descriptors */

#ifdef __cplusplus
extern "C" {
#endif

/* ---- state-space leaves ------------------------------------------------ */
double oracle_distance(const ompl_gpu_space *sp, const double *a, const double *b);
void oracle_interpolate(const ompl_gpu_space *sp, const double *from, const double *to, double t,
                        double *out);
uint32_t oracle_valid_segment_count(const ompl_gpu_space *sp, const double *a, const double *b);
/* SpaceInformation::getMotionStates(s1, s2, states, count, endpoints, alloc = true) for m
 * motions; out = [m][count + (endpoints ? 2 : 0)][dim]; returns the states per motion. */
uint32_t oracle_motion_states(const ompl_gpu_space *sp, const double *s1, const double *s2, size_t m,
                              uint32_t count, int endpoints, double *out);

/* ---- validity + motion -------------------------------------------------- */
int oracle_is_valid(const ompl_gpu_space *sp, const ompl_gpu_checker *ck, const double *s);
/* DiscreteMotionValidator::checkMotion(s1,s2) (bisection, s2 first) for m edges.
 * valid[i] in {0,1}; nd[i] = validSegmentCount; first_invalid[i] = first invalid
 * sample of the linear (lastValid) variant: j in [1,nd-1], nd for s2, -1 if valid.
 * Any output pointer may be NULL.  Returns the number of states isValid() was
 * called on by the bisection variant (the reference's work count). */
uint64_t oracle_check_motions(const ompl_gpu_space *sp, const ompl_gpu_checker *ck, const double *s1,
                              const double *s2, size_t m, uint8_t *valid, int32_t *nd,
                              int32_t *first_invalid);

/* ---- brute-force nearest neighbours (NearestNeighborsLinear semantics) --
 * data: n AoS states (sp->dim reals each).  Results per query sorted by
 * (distance, index) ascending; k > n returns n results; out arrays are nq*k,
 * counts[q] = min(k, n). */
void oracle_knn(const ompl_gpu_space *sp, const double *data, size_t n, const double *q, size_t nq,
                uint32_t k, uint32_t *ids, double *dists, uint32_t *counts);
/* radius: pass 1 with ids==NULL fills counts; pass 2 writes CSR at offsets[q]. */
void oracle_radius(const ompl_gpu_space *sp, const double *data, size_t n, const double *q, size_t nq,
                   double r, const uint64_t *offsets, uint32_t *ids, double *dists, uint64_t *counts);

/* ---- GNAT restatement (oracle/gnat.cpp): exact metric tree, CPU baseline --- */
typedef struct oracle_gnat oracle_gnat;
oracle_gnat *oracle_gnat_create(const ompl_gpu_space *sp, uint32_t degree, uint32_t min_degree,
                                uint32_t max_degree, uint32_t max_pts_per_leaf, uint64_t seed);
void oracle_gnat_destroy(oracle_gnat *g);
void oracle_gnat_add(oracle_gnat *g, const double *states, size_t n); /* ids = insertion order */
void oracle_gnat_add_bulk(oracle_gnat *g, const double *states, size_t n);
size_t oracle_gnat_size(const oracle_gnat *g);
/* nthreads>1 runs independent const queries on std::threads (thread-safe GNAT). */
void oracle_gnat_knn(const oracle_gnat *g, const double *q, size_t nq, uint32_t k, uint32_t *ids,
                     double *dists, uint32_t *counts, int nthreads);
uint64_t oracle_gnat_radius_count(const oracle_gnat *g, const double *q, size_t nq, double r,
                                  uint64_t *counts, int nthreads);
/* nearestR with the results: CSR offsets[nq + 1], returns the total; the (distance, id)-sorted
 * ids / distances stay in the handle until oracle_gnat_radius_fetch copies them out */
uint64_t oracle_gnat_radius(oracle_gnat *g, const double *q, size_t nq, double r, uint64_t *offsets,
                            int nthreads);
void oracle_gnat_radius_fetch(oracle_gnat *g, uint32_t *ids, double *dists);
/* multi-threaded motion checks (for the all-cores CPU baseline) */
uint64_t oracle_check_motions_mt(const ompl_gpu_space *sp, const ompl_gpu_checker *ck, const double *s1,
                                 const double *s2, size_t m, uint8_t *valid, int nthreads);

/* PRM* roadmap construction, sequential (PRM.cpp:562-596): out [n][k_cap] neighbours / validity,
 * cnt[n] neighbours per vertex */
void oracle_prm_causal(const ompl_gpu_space *sp, const ompl_gpu_checker *ck, const double *states, size_t n,
                       double k_const, uint32_t k_cap, uint32_t *nbr, uint32_t *cnt, uint8_t *valid);

/* RRT*'s iteration, sequential (oracle/rrtstar.cpp; RRTstar.cpp:247-542 with its defaults) from
 * the tree (states0, parent0 (-1 = root), inc0, cost0) over the given samples; use_gnat: the GNAT
 * restatement as the neighbour structure (else brute force); time_budget_s > 0 stops early.
 * Per sample: nearest_out, added_out (0xFFFFFFFF: not added), parent_choice (-1); the final tree
 * (n0 + added entries) in parent_out / inc_out / cost_out (may be NULL); stats[5] = samples
 * processed, added, rewires, checkMotion calls, nanoseconds in the loop (the neighbour structure's
 * build excluded).  Returns the samples processed. */
uint64_t oracle_rrtstar(const ompl_gpu_space *sp, const ompl_gpu_checker *ck, const double *states0, size_t n0,
                        const int64_t *parent0, const double *inc0, const double *cost0, const double *samples,
                        size_t ns, double maxd, double k_rrt, int use_gnat, double time_budget_s, uint32_t *nearest_out,
                        uint32_t *added_out, int64_t *parent_choice, int64_t *parent_out, double *inc_out,
                        double *cost_out, uint64_t *stats);

/* ---- the reference's input streams (oracle/rng.cpp) ------------------- */
uint32_t oracle_mt19937_10000th(void);
uint32_t oracle_ranlux24_base_10000th(void);
/* the first n RNG() seeds after RNG::setSeed(seed) */
void oracle_seed_stream(uint32_t seed, size_t n, uint32_t *out);
/* n sampleUniform() of the space's default sampler whose RNGs have the given local seeds
 * (SE3: compound, R^3, SO3; SO3: one; R^n / KCHAIN: one); low/high: bounds of the R^n part */
void oracle_sample_uniform(const ompl_gpu_space *sp, const uint32_t *local_seeds, const double *low,
                           const double *high, size_t n, double *out);

#ifdef __cplusplus
}
#endif
#endif
