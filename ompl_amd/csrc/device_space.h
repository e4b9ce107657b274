// device_space.h — device restatement of the reference's state-space leaves in
// IEEE fp64 with the reference's operation order.  Every function is __host__ __device__:
// the library's host side runs the same code (StateValidityCheckerGPU's single-state isValid,
// the distance the NN plugin's verify mode compares against), so host and device agree bit for
// bit.  The KinematicChain's cos / sin are glibc's own algorithm (glibc_sincos.h: the device math
// library differs from glibc by an ulp on 3 % of the arguments, enough to flip validity bits and
// segment counts at the chain's knife edges); SO3's acos is glibc's own too (glibc_acos.h: the
// device library's differs from glibc's by an ulp on up to 2 % of the arguments near 1, which moved
// SO3 / SE3 distances, steered rotations and segment counts off the reference's bits).  This translation unit is
// compiled with -ffp-contract=off: no multiply-add is fused, matching the
// reference x86-64 build (CMakeModules/CompilerSettings.cmake:8, no -march).
//
//   distance   RealVectorStateSpace.cpp:230-242, SO3StateSpace.cpp:254-262,
//              StateSpace.cpp:1068-1076 (compound), demos/KinematicChain.h:105-124
//   interpolate RealVectorStateSpace.cpp:257-265, SO3StateSpace.cpp:289-318,
//              StateSpace.cpp:1109-1116, demos/KinematicChain.h:150-175
//   segments   StateSpace.cpp:851-854, :1085-1097
//   isValid    demos/HypercubeBenchmark.cpp:57-72, tests/resources/circles2D.h:139-150,
//              demos/KinematicChain.h:200-276
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ompl_gpu.h"
#include "glibc_acos.h"
#include "glibc_sincos.h"

namespace ompl_amd {

constexpr double kPi = 3.141592653589793238462643383279502884;
constexpr double kQuatNormErr = 1e-9;                    // SO3StateSpace.cpp:47
constexpr double kDblEps = 2.220446049250313080847e-16;  // numeric_limits<double>::epsilon()
constexpr double kFltEps = 1.1920928955078125e-07;       // numeric_limits<float>::epsilon()

// Plain-old-data copy of ompl_gpu_space passed by value to kernels.
struct DevSpace {
    int kind;
    int dim;
    double w0, w1;
    double lvs0, lvs1;
    uint32_t f0, f1;
    double link;
};

// Feature layout per state (what the NN kernels stream):
//   REALVECTOR(n): n coordinates, zero-padded to the bucket (adding 0*0 to the
//                  running sum is exact, so padding preserves the bits)
//   SO3          : qx,qy,qz,qw
//   SE3          : x,y,z,qx,qy,qz,qw
//   KCHAIN(n)    : cos(theta_1..n), sin(theta_1..n) of the cumulative angles —
//                  the reference recomputes them per pair; they are a pure
//                  function of the state, so precomputing them is bit-identical.
__host__ __device__ inline int feature_count(int kind, int dim) {
    return kind == OMPL_GPU_SPACE_KCHAIN ? 2 * dim : dim;
}

__host__ __device__ __forceinline__ double l2_dist(const double *a, const double *b, int n) {
    double acc = 0.0;
    for (int i = 0; i < n; ++i) {
        double diff = a[i] - b[i];
        acc += diff * diff;
    }
    return sqrt(acc);
}

__host__ __device__ __forceinline__ double so3_arc(const double *p, const double *q) {
    double dq = fabs(p[0] * q[0] + p[1] * q[1] + p[2] * q[2] + p[3] * q[3]);
    if (dq > 1.0 - kQuatNormErr) return 0.0;
    return glibc_acos(dq);
}

// chain distance from precomputed cumulative cos/sin features (cs[0..n) = cos, cs[n..2n) = sin)
template <int NMAX>
__host__ __device__ __forceinline__ double chain_dist_feat(const double *a, const double *b, int n, double link) {
    double dx = 0., dy = 0., dist = 0.;
#pragma unroll
    for (int i = 0; i < NMAX; ++i) {
        if (i < n) {
            dx += a[i] - b[i];
            dy += a[NMAX + i] - b[NMAX + i];
            dist += sqrt(dx * dx + dy * dy);
        }
    }
    return dist * link;
}

// raw-angle chain distance (motion validator: validSegmentCount on raw states)
__host__ __device__ __forceinline__ double chain_dist_raw(const double *a, const double *b, int n, double link,
                                                          const double *tab = gsc::kSinCosTab) {
    double th1 = 0., th2 = 0., dx = 0., dy = 0., dist = 0.;
    for (int i = 0; i < n; ++i) {
        th1 += a[i];
        th2 += b[i];
        double s1, c1, s2, c2;
        glibc_sincos(th1, s1, c1, tab);
        glibc_sincos(th2, s2, c2, tab);
        dx += c1 - c2;
        dy += s1 - s2;
        dist += sqrt(dx * dx + dy * dy);
    }
    return dist * link;
}

__host__ __device__ __forceinline__ double se3_dist(const double *a, const double *b, double w0, double w1) {
    double dist = 0.0;
    dist += w0 * l2_dist(a, b, 3);
    dist += w1 * so3_arc(a + 3, b + 3);
    return dist;
}

// distance on raw AoS states (dim reals)
__host__ __device__ inline double raw_distance(const DevSpace &sp, const double *a, const double *b) {
    switch (sp.kind) {
    case OMPL_GPU_SPACE_REALVECTOR: return l2_dist(a, b, sp.dim);
    case OMPL_GPU_SPACE_SO3: return so3_arc(a, b);
    case OMPL_GPU_SPACE_SE3: return se3_dist(a, b, sp.w0, sp.w1);
    default: return chain_dist_raw(a, b, sp.dim, sp.link);
    }
}

__host__ __device__ __forceinline__ uint32_t seg_count(double d, double lvs, uint32_t f) {
    return f * (uint32_t)ceil(d / lvs);
}

__host__ __device__ inline uint32_t valid_segment_count(const DevSpace &sp, const double *a, const double *b,
                                                        const double *tab = gsc::kSinCosTab) {
    switch (sp.kind) {
    case OMPL_GPU_SPACE_REALVECTOR: return seg_count(l2_dist(a, b, sp.dim), sp.lvs0, sp.f0);
    case OMPL_GPU_SPACE_SO3: return seg_count(so3_arc(a, b), sp.lvs0, sp.f0);
    case OMPL_GPU_SPACE_SE3: {
        uint32_t sc = 0;
        uint32_t s0 = seg_count(l2_dist(a, b, 3), sp.lvs0, sp.f0);
        if (s0 > sc) sc = s0;
        uint32_t s1 = seg_count(so3_arc(a + 3, b + 3), sp.lvs1, sp.f1);
        if (s1 > sc) sc = s1;
        return sc;
    }
    default: return seg_count(chain_dist_raw(a, b, sp.dim, sp.link, tab), sp.lvs0, sp.f0);
    }
}

__host__ __device__ __forceinline__ void lerp(const double *f, const double *t_, double t, double *o, int n) {
    for (int i = 0; i < n; ++i) o[i] = f[i] + (t_[i] - f[i]) * t;
}

__host__ __device__ inline void slerp(const double *f, const double *to, double t, double *o) {
    double theta = so3_arc(f, to);
    if (theta > kDblEps) {
        double d = 1.0 / glibc_sin(theta);
        double s0 = glibc_sin((1.0 - t) * theta);
        double s1 = glibc_sin(t * theta);
        double dq = f[0] * to[0] + f[1] * to[1] + f[2] * to[2] + f[3] * to[3];
        if (dq < 0) s1 = -s1;
        o[0] = (f[0] * s0 + to[0] * s1) * d;
        o[1] = (f[1] * s0 + to[1] * s1) * d;
        o[2] = (f[2] * s0 + to[2] * s1) * d;
        o[3] = (f[3] * s0 + to[3] * s1) * d;
    } else {
        o[0] = f[0]; o[1] = f[1]; o[2] = f[2]; o[3] = f[3];
    }
}

__host__ __device__ inline void chain_interp(const double *f, const double *to, double t, double *o, int n) {
    for (int i = 0; i < n; ++i) {
        double diff = to[i] - f[i];
        if (fabs(diff) <= kPi) {
            o[i] = f[i] + diff * t;
        } else {
            if (diff > 0.0)
                diff = 2.0 * kPi - diff;
            else
                diff = -2.0 * kPi - diff;
            double v = f[i] - diff * t;
            if (v > kPi)
                v -= 2.0 * kPi;
            else if (v < -kPi)
                v += 2.0 * kPi;
            o[i] = v;
        }
    }
}

// interpolate; rot=false skips the SO3 part of SE3 when the validity checker only
// reads the translation (its output is then unused: the result bit is unchanged).
__host__ __device__ inline void interpolate(const DevSpace &sp, const double *f, const double *to, double t, double *o,
                                   bool rot = true) {
    switch (sp.kind) {
    case OMPL_GPU_SPACE_REALVECTOR: lerp(f, to, t, o, sp.dim); break;
    case OMPL_GPU_SPACE_SO3: slerp(f, to, t, o); break;
    case OMPL_GPU_SPACE_SE3:
        lerp(f, to, t, o, 3);
        if (rot) slerp(f + 3, to + 3, t, o + 3);
        break;
    default: chain_interp(f, to, t, o, sp.dim); break;
    }
}

// ---- validity checkers --------------------------------------------------------

struct DevChecker {
    int kind;
    int ndim;
    double edge;
    int count;
    const double *data;  // device copy
    // KinematicChain: the rounding slack of the segment-side pre-test (chain_valid), >= every
    // difference between a side value computed here and the reference's s / t numerators:
    // 1e-12 * M^2, M = max(1, the chain's reach, the largest |environment coordinate|)
    double slack;
};

__host__ __device__ __forceinline__ bool hypercube_valid(const double *s, int ndim, double edge) {
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

__host__ __device__ __forceinline__ bool spheres_valid(const double *s, const double *c, int count) {
    for (int i = 0; i < count; ++i) {
        double dx = c[4 * i + 0] - s[0];
        double dy = c[4 * i + 1] - s[1];
        double dz = c[4 * i + 2] - s[2];
        if (dx * dx + dy * dy + dz * dz < c[4 * i + 3]) return false;
    }
    return true;
}

__host__ __device__ __forceinline__ bool circles_valid(const double *s, const double *c, int count) {
    for (int i = 0; i < count; ++i) {
        double dx = c[3 * i + 0] - s[0];
        double dy = c[3 * i + 1] - s[1];
        if (dx * dx + dy * dy < c[3 * i + 2]) return false;
    }
    return true;
}

__host__ __device__ __forceinline__ bool seg_intersect(double a0x, double a0y, double a1x, double a1y, double b0x, double b0y,
                                              double b1x, double b1y) {
    double s10_x = a1x - a0x;
    double s10_y = a1y - a0y;
    double s32_x = b1x - b0x;
    double s32_y = b1y - b0y;
    double denom = s10_x * s32_y - s32_x * s10_y;
    if (fabs(denom) < kDblEps) return false;
    bool denomPositive = denom > 0;
    double s02_x = a0x - b0x;
    double s02_y = a0y - b0y;
    double s_numer = s10_x * s02_y - s10_y * s02_x;
    if ((s_numer < kFltEps) == denomPositive) return false;
    double t_numer = s32_x * s02_y - s32_y * s02_x;
    if ((t_numer < kFltEps) == denomPositive) return false;
    if (((s_numer - denom > -kFltEps) == denomPositive) || ((t_numer - denom > kFltEps) == denomPositive))
        return false;
    return true;
}

constexpr int kChainMaxLinks = 32;

// KinematicChainValidityChecker::isValid (demos/KinematicChain.h:200-276): the chain's link
// endpoints, then every pair of its segments and every (segment, environment segment) pair
// through intersectionTest (seg_intersect) — the result is the AND of those tests, so the order
// of the pairs does not matter.  A pair is tested only when a necessary condition for the test to
// return true holds.  For a = (a0, a1) against b = (b0, b1), with v = b1 - b0 and the side value
// side(p) = v x (p - b0), the test's t numerator is side(a0) and its t numerator minus the
// denominator is side(a1) up to rounding; it returns true only if (denom > 0) t >= eps >= t - denom,
// or (denom < 0) t < eps < t - denom — in both cases eps lies between side(a0) and side(a1)
// (eps = FLT_EPSILON, the test's own threshold).  So when both endpoints of a have side values
// above eps + slack, or both below eps - slack, the test returns false and is skipped (slack:
// DevChecker::slack, far above the rounding of either computation).  For an environment
// segment the side values of the whole chain are first bounded over the chain's bounding box
// (side() is affine): a box entirely on one side skips all of that segment's tests.
__host__ __device__ inline bool chain_valid(const double *s, int n, double link, const double *env, int nenv,
                                            double slack, const double *tab = gsc::kSinCosTab) {
    double px[kChainMaxLinks + 2], py[kChainMaxLinks + 2];  // segment i = (p[i], p[i+1])
    double theta = 0., x = 0., y = 0.;
    px[0] = 0.;
    py[0] = 0.;
    double st = 0.0, ct = 1.0;
    for (int i = 0; i < n; ++i) {
        theta += s[i];
        glibc_sincos(theta, st, ct, tab);
        double xN = x + ct * link;
        double yN = y + st * link;
        px[i + 1] = xN;
        py[i + 1] = yN;
        x = xN;
        y = yN;
    }
    if (n == 0) glibc_sincos(theta, st, ct, tab);
    px[n + 1] = x + ct * 0.001;
    py[n + 1] = y + st * 0.001;
    const int ns = n + 1;
    const double lo_t = kFltEps - slack, hi_t = kFltEps + slack;
    // segment pairs (i, j), i < j: b = segment j
    for (int j = 1; j < ns; ++j) {
        const double bx = px[j], by = py[j], vx = px[j + 1] - bx, vy = py[j + 1] - by;
        double sa = vx * (py[0] - by) - vy * (px[0] - bx);
        for (int i = 0; i < j; ++i) {
            const double sb = vx * (py[i + 1] - by) - vy * (px[i + 1] - bx);
            if (!((sa > hi_t && sb > hi_t) || (sa < lo_t && sb < lo_t)) &&
                seg_intersect(px[i], py[i], px[i + 1], py[i + 1], px[j], py[j], px[j + 1], py[j + 1]))
                return false;
            sa = sb;
        }
    }
    double xmin = px[0], xmax = px[0], ymin = py[0], ymax = py[0];
    for (int i = 1; i <= ns; ++i) {
        xmin = fmin(xmin, px[i]);
        xmax = fmax(xmax, px[i]);
        ymin = fmin(ymin, py[i]);
        ymax = fmax(ymax, py[i]);
    }
    for (int j = 0; j < nenv; ++j) {
        const double bx = env[4 * j], by = env[4 * j + 1], vx = env[4 * j + 2] - bx, vy = env[4 * j + 3] - by;
        const double y0 = vx * (ymin - by), y1 = vx * (ymax - by), x0 = vy * (xmin - bx), x1 = vy * (xmax - bx);
        const double smax = fmax(y0, y1) - fmin(x0, x1), smin = fmin(y0, y1) - fmax(x0, x1);
        if (smin > hi_t || smax < lo_t) continue;  // the whole chain on one side of b's line
        double sa = vx * (py[0] - by) - vy * (px[0] - bx);
        for (int i = 0; i < ns; ++i) {
            const double sb = vx * (py[i + 1] - by) - vy * (px[i + 1] - bx);
            if (!((sa > hi_t && sb > hi_t) || (sa < lo_t && sb < lo_t)) &&
                seg_intersect(px[i], py[i], px[i + 1], py[i + 1], env[4 * j], env[4 * j + 1], env[4 * j + 2],
                              env[4 * j + 3]))
                return false;
            sa = sb;
        }
    }
    return true;
}

// chain_valid with the link endpoints in registers: NP >= n + 2 points, every loop unrolled to
// NP with guards on the runtime n, so every index is a constant (the runtime form's arrays live
// in scratch).  angle(i) yields the state's i-th joint angle — a stored state, or an interpolated
// one computed on the fly in chain_interp's arithmetic (no state array either).  The same tests
// in the same arithmetic as chain_valid: identical results.
template <int NP, class Angle>
__device__ __forceinline__ bool chain_valid_np(Angle angle, int n, double link, const double *env, int nenv,
                                               double slack, const double *tab) {
    double px[NP], py[NP];
    double theta = 0., x = 0., y = 0., st = 0.0, ct = 1.0;
    px[0] = 0.;
    py[0] = 0.;
#pragma unroll
    for (int i = 0; i < NP - 2; ++i) {
        if (i < n) {
            __builtin_amdgcn_sched_barrier(0);  // one link at a time: no hoisted state loads
            theta += angle(i);
            glibc_sincos(theta, st, ct, tab);
            x = x + ct * link;
            y = y + st * link;
        }
        px[i + 1] = x;  // past n: copies of the last point (never read as a segment)
        py[i + 1] = y;
    }
    if (n == 0) glibc_sincos(theta, st, ct, tab);
    const double tx = x + ct * 0.001, ty = y + st * 0.001;
#pragma unroll
    for (int i = 1; i < NP; ++i)
        if (i == n + 1) {
            px[i] = tx;
            py[i] = ty;
        }
    const int ns = n + 1;
    const double lo_t = kFltEps - slack, hi_t = kFltEps + slack;
#pragma unroll
    for (int j = 1; j < NP - 1; ++j) {
        if (j < ns) {
            __builtin_amdgcn_sched_barrier(0);  // one segment j at a time (live ranges)
            const double bx = px[j], by = py[j], vx = px[j + 1] - bx, vy = py[j + 1] - by;
            double sa = vx * (py[0] - by) - vy * (px[0] - bx);
#pragma unroll
            for (int i = 0; i < j; ++i) {
                const double sb = vx * (py[i + 1] - by) - vy * (px[i + 1] - bx);
                if (!((sa > hi_t && sb > hi_t) || (sa < lo_t && sb < lo_t)) &&
                    seg_intersect(px[i], py[i], px[i + 1], py[i + 1], px[j], py[j], px[j + 1], py[j + 1]))
                    return false;
                sa = sb;
            }
        }
    }
    double xmin = 0., xmax = 0., ymin = 0., ymax = 0.;  // point 0 is the origin
#pragma unroll
    for (int i = 1; i < NP; ++i) {
        if (i <= ns) {
            xmin = fmin(xmin, px[i]);
            xmax = fmax(xmax, px[i]);
            ymin = fmin(ymin, py[i]);
            ymax = fmax(ymax, py[i]);
        }
    }
    for (int j = 0; j < nenv; ++j) {
        const double bx = env[4 * j], by = env[4 * j + 1], ex = env[4 * j + 2], ey = env[4 * j + 3];
        const double vx = ex - bx, vy = ey - by;
        const double y0 = vx * (ymin - by), y1 = vx * (ymax - by), x0 = vy * (xmin - bx), x1 = vy * (xmax - bx);
        const double smax = fmax(y0, y1) - fmin(x0, x1), smin = fmin(y0, y1) - fmax(x0, x1);
        if (smin > hi_t || smax < lo_t) continue;
        double sa = vx * (py[0] - by) - vy * (px[0] - bx);
#pragma unroll
        for (int i = 0; i < NP - 1; ++i) {
            if (i < ns) {
                const double sb = vx * (py[i + 1] - by) - vy * (px[i + 1] - bx);
                if (!((sa > hi_t && sb > hi_t) || (sa < lo_t && sb < lo_t)) &&
                    seg_intersect(px[i], py[i], px[i + 1], py[i + 1], bx, by, ex, ey))
                    return false;
                sa = sb;
            }
        }
    }
    return true;
}

// chain_interp's coordinate i (demos/KinematicChain.h:150-175), for chain_valid_np
__host__ __device__ __forceinline__ double chain_interp1(double f, double to, double t) {
    double diff = to - f;
    if (fabs(diff) <= kPi) return f + diff * t;
    if (diff > 0.0)
        diff = 2.0 * kPi - diff;
    else
        diff = -2.0 * kPi - diff;
    double v = f - diff * t;
    if (v > kPi)
        v -= 2.0 * kPi;
    else if (v < -kPi)
        v += 2.0 * kPi;
    return v;
}

__host__ __device__ inline bool is_valid(const DevSpace &sp, const DevChecker &ck, const double *s,
                                         const double *tab = gsc::kSinCosTab) {
    switch (ck.kind) {
    case OMPL_GPU_CHECK_ALL_VALID: return true;
    case OMPL_GPU_CHECK_HYPERCUBE: return hypercube_valid(s, ck.ndim, ck.edge);
    case OMPL_GPU_CHECK_SPHERES: return spheres_valid(s, ck.data, ck.count);
    case OMPL_GPU_CHECK_CIRCLES2D: return circles_valid(s, ck.data, ck.count);
    default: return chain_valid(s, sp.dim, sp.link, ck.data, ck.count, ck.slack, tab);
    }
}

// Does the checker read the SO3 part of an SE3 state?  (None of the closed set does.)
__host__ __device__ inline bool checker_reads_rotation(int kind) { return false; }

// ---- fixed-width forms (device) ------------------------------------------------
// Kernels specialised on the space kind SP and a compile-time state width DIM (DIM = 0: the
// runtime width, up to kChainMaxLinks).  With DIM fixed every state array is indexed by
// constants after unrolling and lives in registers; the runtime-width form keeps them in
// scratch.  The arithmetic is the same code either way, so results are identical.
template <int DIM>
struct Width {
    static constexpr int N = DIM > 0 ? DIM : kChainMaxLinks;
};

template <int DIM>
__device__ __forceinline__ void load_state(const double *__restrict__ p, int dim, double *o) {
    if constexpr (DIM > 0) {
#pragma unroll
        for (int c = 0; c < DIM; ++c) o[c] = p[c];
    } else {
        for (int c = 0; c < dim; ++c) o[c] = p[c];
    }
}

// the space descriptor with the specialisation's constants folded in
template <int SP, int DIM>
__device__ __forceinline__ DevSpace fixed_space(DevSpace sp) {
    if constexpr (DIM > 0) {
        sp.kind = SP;
        sp.dim = DIM;
    }
    return sp;
}

// HypercubeBenchmark's predicate (device_space.h hypercube_valid, HypercubeBenchmark.cpp:57-72)
// unrolled over the fixed width: the reference's loop i = ndim - 1 .. 0 with the same early
// exit (a violation decides the result; later indices no longer matter)
template <int DIM>
__device__ __forceinline__ bool hypercube_valid_fixed(const double *s, int ndim, double edge) {
    bool found = false, ok = true;
#pragma unroll
    for (int i = DIM - 1; i >= 0; i--) {
        if (i < ndim && ok) {
            if (!found) {
                if (s[i] > edge) found = true;
            } else if (s[i] < (1. - edge)) {
                ok = false;
            }
        }
    }
    return ok;
}

// is_valid (device_space.h) for the fixed forms, which never see the KinematicChain checker
// (dispatch_width sends it to the runtime-width form)
template <int DIM>
__device__ __forceinline__ bool valid_t(const DevSpace &sp, const DevChecker &ck, const double *s,
                                        const double *tab = gsc::kSinCosTab) {
    if constexpr (DIM > 0) {
        switch (ck.kind) {
        case OMPL_GPU_CHECK_ALL_VALID: return true;
        case OMPL_GPU_CHECK_HYPERCUBE: return hypercube_valid_fixed<DIM>(s, ck.ndim, ck.edge);
        case OMPL_GPU_CHECK_SPHERES: return spheres_valid(s, ck.data, ck.count);
        default: return circles_valid(s, ck.data, ck.count);
        }
    } else {
        return is_valid(sp, ck, s, tab);
    }
}

// valid_t for a kernel's (space kind, width) specialisation (the KinematicChain checker only ever
// takes the runtime width, DIM = 0)
template <int SP, int DIM>
__device__ __forceinline__ bool valid_sp(const DevSpace &sp, const DevChecker &ck, const double *s,
                                         const double *tab = gsc::kSinCosTab) {
    static_assert(SP != OMPL_GPU_SPACE_KCHAIN || DIM == 0, "the chain checker runs at the runtime width");
    return valid_t<DIM>(sp, ck, s, tab);
}

}  // namespace ompl_amd
