// host_features.cpp — host-side feature rows (kernels.h FeatGeom), compiled with the
// system C++ compiler (g++) against glibc's libm: the KinematicChain features
// cos/sin of the cumulative joint angles must be the very values the reference computes
// (demos/KinematicChain.h:113-116), which a HIP-compiled host path does not guarantee.
#include <cmath>
#include <cstdint>

namespace ompl_amd {

struct DevSpace {  // layout-identical to device_space.h (kept POD; no HIP headers here)
    int kind;
    int dim;
    double w0, w1;
    double lvs0, lvs1;
    uint32_t f0, f1;
    double link;
};
struct FeatGeom {
    int F;
    int nmax;
};

constexpr int kKindKChain = 3;  // OMPL_GPU_SPACE_KCHAIN

void host_features(const DevSpace &sp, const FeatGeom &g, const double *s, double *o) {
    if (sp.kind == kKindKChain) {
        double th = 0.;
        for (int j = 0; j < g.nmax; ++j) {
            if (j < sp.dim) {
                th += s[j];
                o[j] = std::cos(th);
                o[g.nmax + j] = std::sin(th);
            } else {
                o[j] = 0.;
                o[g.nmax + j] = 0.;
            }
        }
    } else {
        for (int j = 0; j < g.F; ++j) o[j] = j < sp.dim ? s[j] : 0.0;
    }
}

}  // namespace ompl_amd
