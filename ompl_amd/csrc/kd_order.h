// kd_order.h — the node record of the sorted store's k-d tree (built on the device,
// knn_fast_impl.h build_sorted), which the device walks to find a query's home leaf.
#pragma once
#include <stddef.h>
#include <stdint.h>


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

}  // namespace ompl_amd
