// Resource-usage probe (not product): instantiates only the group walk kernels so that their
// VGPR / scratch figures come out of one short device-only compile:
//   hipcc --offload-arch=gfx950 --cuda-device-only -O3 -std=c++17 -ffp-contract=off -I include \
//         -Rpass-analysis=kernel-resource-usage -c tools/kexp.hip -o /tmp/kexp.o
#include "../ompl_amd/csrc/knn_fast_impl.h"
namespace ompl_amd {
namespace {
template __global__ void knn32_group_kernel<OMPL_GPU_SPACE_SE3, 7, 16, 4, 1, true>(
    const float *, uint32_t, const uint32_t *, uint32_t, const float *, const float *, uint32_t, const uint32_t *,
    const float *, const uint32_t *, uint32_t, float, float, float *, uint32_t *, unsigned long long *, int, int, int);
}  // namespace
}  // namespace ompl_amd
namespace ompl_amd {
namespace {
template __global__ void radius32_group_kernel<OMPL_GPU_SPACE_SE3, 7, 4, 2>(
    const float *, uint32_t, const uint32_t *, uint32_t, const float *, const float *, uint32_t, const float *,
    const uint32_t *, uint32_t, const double *, const double *, DevSpace, float, float, double, uint64_t *,
    const uint64_t *, uint32_t *, double *, unsigned long long *, uint32_t);
template __global__ void radius32_group_kernel<OMPL_GPU_SPACE_SE3, 7, 4, 1>(
    const float *, uint32_t, const uint32_t *, uint32_t, const float *, const float *, uint32_t, const float *,
    const uint32_t *, uint32_t, const double *, const double *, DevSpace, float, float, double, uint64_t *,
    const uint64_t *, uint32_t *, double *, unsigned long long *, uint32_t);
}  // namespace
}  // namespace ompl_amd
