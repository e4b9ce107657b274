// kd_order.cpp — k-d leaf order of the sorted store (host, plain C++).
//
// The culled walks (knn_fast_impl.h) skip a tile when its bounding box is farther than a
// query's current threshold, so their cost is the number of tiles whose box reaches into the
// query's neighbourhood.  Median splits along the widest coordinate, down to leaves of exactly
// one tile, give compact, well-proportioned boxes; runs of a space-filling curve straddle
// curve cells and give long thin ones (measured on 2e5 SE(3) states: 47 vs 136 tiles reach a
// query's 16-NN ball).  A tile is a leaf, a super-tile a subtree of 32 leaves.  The internal
// nodes are kept (pre-order) so the device can send each query down to its home leaf, which
// orders the queries into coherent groups and starts the walk there.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <numeric>
#include <vector>

#include "kd_order.h"

namespace ompl_amd {

namespace {

struct Builder {
    const float *x;
    size_t stride;
    int dims;
    uint32_t tile;
    std::vector<KdNode> *nodes;

    void run(uint32_t *idx, size_t cnt, uint32_t tiles) {
        if (tiles <= 1 || cnt == 0) return;
        float lo[kKdMaxDims], hi[kKdMaxDims];
        for (int d = 0; d < dims; ++d) {
            lo[d] = INFINITY;
            hi[d] = -INFINITY;
        }
        for (size_t i = 0; i < cnt; ++i)
            for (int d = 0; d < dims; ++d) {
                const float v = x[(size_t)d * stride + idx[i]];
                lo[d] = std::min(lo[d], v);
                hi[d] = std::max(hi[d], v);
            }
        int bd = 0;
        float be = -1.f;
        for (int d = 0; d < dims; ++d)
            if (hi[d] - lo[d] > be) {
                be = hi[d] - lo[d];
                bd = d;
            }
        const uint32_t tl = tiles / 2;  // the left subtree holds tl full tiles
        const size_t lt = std::min<size_t>((size_t)tl * tile, cnt);
        const float *col = x + (size_t)bd * stride;
        std::nth_element(idx, idx + lt, idx + cnt, [col](uint32_t a, uint32_t b) { return col[a] < col[b]; });
        const float split = lt < cnt ? col[idx[lt]] : hi[bd];
        const size_t me = nodes->size();
        nodes->push_back(KdNode{(uint32_t)bd, split, tl, 0u});
        run(idx, lt, tl);
        (*nodes)[me].right = (uint32_t)nodes->size();
        run(idx + lt, cnt - lt, tiles - tl);
    }
};

}  // namespace

void kd_tile_order(const float *x, size_t stride, uint32_t n, int dims, uint32_t tile, std::vector<uint32_t> &perm,
                   std::vector<KdNode> &nodes) {
    perm.resize(n);
    nodes.clear();
    // live states (finite first coordinate) are split; removed ones (NaN) go to the end, where
    // their rows stay NaN and the tile boxes ignore them
    size_t live = 0;
    for (uint32_t i = 0; i < n; ++i)
        if (x[i] == x[i]) perm[live++] = i;
    size_t dead = live;
    for (uint32_t i = 0; i < n; ++i)
        if (!(x[i] == x[i])) perm[dead++] = i;
    const uint32_t tiles = (uint32_t)((live + tile - 1) / tile);
    Builder b{x, stride, std::min(dims, kKdMaxDims), tile, &nodes};
    b.run(perm.data(), live, tiles);
}

}  // namespace ompl_amd
