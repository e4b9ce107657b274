// kd_order.h — k-d leaf order of the sorted store (kd_order.cpp, host) and its node record,
// which the device walks to find a query's home leaf (knn_fast_impl.h).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace ompl_amd {

constexpr int kKdMaxDims = 16;

// internal node, pre-order: its left subtree (left_tiles leaves) follows it directly, its
// right subtree starts at node `right`; states with coordinate `dim` < split went left
struct KdNode {
    uint32_t dim;
    float split;
    uint32_t left_tiles;
    uint32_t right;
};

// x: rows [dims][stride] of n states.  perm: the states in leaf order (leaves of `tile`
// states; removed states, NaN in row 0, last); nodes: the internal nodes, pre-order.
void kd_tile_order(const float *x, size_t stride, uint32_t n, int dims, uint32_t tile, std::vector<uint32_t> &perm,
                   std::vector<KdNode> &nodes);

}  // namespace ompl_amd
