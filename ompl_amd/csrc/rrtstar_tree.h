// rrtstar_tree.h — the RRT* tree's cost bookkeeping on the host (internal; the C-ABI is in
// include/ompl_gpu.h, "RRT* cost logic").  RRTstar's Motion (RRTstar.h:347-372) holds parent,
// incCost, cost and the children list; here they are arrays over the nearest-neighbour ids.
// A device batch's results are staged (copied to the host, ompl_gpu_rrtstar_stage, capi.hip) and
// then committed in sample order (rrtstar_tree.cpp): staging and committing may run on two
// threads, so the next device batch overlaps the cost logic of the previous one.
#pragma once

#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <vector>

namespace ompl_amd {

struct RrtStarStaged {
    size_t ns = 0;
    std::vector<uint32_t> nearest, added;  // per sample
    std::vector<double> inc;               // per sample: distance(nmotion, x_i)
    std::vector<uint64_t> off;             // ns + 1
    std::vector<uint32_t> ids;             // neighbourhood entries, each segment by (distance, id)
    std::vector<double> dist;
    std::vector<uint8_t> bits;             // bit 0: checkMotion(nbh, x_i), bit 1: checkMotion(x_i, nbh)
};

}  // namespace ompl_amd

struct ompl_gpu_rrtstar_tree {
    std::vector<int64_t> parent;  // -1: a start state
    std::vector<double> inc, cost;
    std::vector<std::vector<uint32_t>> children;
    std::vector<uint32_t> slot;  // each state's index in its parent's children list
    bool consistent = true;      // every cost = its parent's cost + incCost (tree_add checks)
    // staged batches, oldest first, and recycled buffers (stage and commit may be on two threads)
    std::mutex mu;
    std::deque<ompl_amd::RrtStarStaged> staged;
    std::vector<ompl_amd::RrtStarStaged> spare;
    // commit's scratch
    std::vector<uint32_t> stack;
    std::vector<double> costs, cv;
    std::vector<std::vector<uint32_t>> cand;  // per pool thread: rewiring candidates (neighbour index)
    std::vector<uint64_t> cand_checks;        // per pool thread: parent-choice checkMotion count
    std::shared_ptr<void> touched, pool;  // rrtstar_tree.cpp Touched, Pool
    // totals: [0] rewires, [1] checkMotion calls the sequential loop would make, [2] states added,
    // [3] neighbourhood entries, [4] samples, [5] child costs updateChildCosts rewrote
    uint64_t totals[6] = {0, 0, 0, 0, 0, 0};
};
