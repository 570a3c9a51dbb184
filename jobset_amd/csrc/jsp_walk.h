// jsp_walk.h — host half of the split placement service: the lowest-index
// 1:1 greedy over the feasibility the
// resident tiles hand back. The tiles do the streaming part (predicate +
// capacity tally over every node row, per-leaf feasibility, partial sums per
// upper-level domain); what is left is sequential across jobs and small
// (O(J + C D / 64) word operations), so it runs on the host, next to the
// caller, instead of on one GPU wave.
#pragma once
#include <stdint.h>

#include <vector>

#include "jsp_internal.h"

namespace jsp {

// The waves of the largest tally row block that hold leaves (64 leaves each,
// at most 4): the split service's line layout (jsp_internal.h SplitArgs).
uint32_t split_waves(const std::vector<uint32_t>& blk_l0, const std::vector<uint32_t>& blk_l1);

class HostWalk {
public:
    // topology: first_leaf per level (identity at the leaves), child_start
    // per level k < K-1, parent per level k >= 1 (the engine's upload tables)
    void set_topology(uint32_t K, const uint32_t* D, const std::vector<uint32_t>* fl,
                      const std::vector<uint32_t>* cs, const std::vector<int32_t>* par);
    // classes: level and pods of each (the engine's class upload)
    void set_classes(const std::vector<DevClass>& cls);
    // tiles of the split service: row block leaf ranges (blk table, first and
    // end leaf per block), class groups and classes per group
    void set_tiles(const std::vector<uint32_t>& blk_l0, const std::vector<uint32_t>& blk_l1, uint32_t groups,
                   uint32_t cpg);

    // One request: feasibility from the tiles' slots (jsp_internal.h
    // SplitArgs), then the walk over runs in global order. Returns the
    // number of placed jobs; assign[j] = domain at the job's class level or -1.
    uint32_t place(const uint64_t* slots, const uint32_t* run_class, const uint32_t* run_len, uint32_t n_runs,
                   int32_t* assign);

    // The walk alone over feasibility bitmaps the GPU built (feas_kernel's
    // layout: class c's words at the cumulative offset of (D[level] + 63) / 64
    // words per class -- the engine's word_off). The device paths' walk for
    // the shapes whose GPU walk is a one-wave dependent chain.
    uint32_t walk(const uint64_t* feas, const uint32_t* run_class, const uint32_t* run_len, uint32_t n_runs,
                  int32_t* assign);
    // start loading the walk's own state (cold host core: the call after a
    // sleep), while the device works
    void prefetch_state() const;

    // Tile t (= row block t / groups, class group t % groups) has answered:
    // start loading its slot lines into the host cache while the other tiles
    // finish (pinned memory the device just wrote misses every cache level;
    // read one by one in the walk, the misses cost cfg3 ~3.9 us, cfg5 ~7.4 us).
    void prefetch_tile(const uint64_t* slots, uint32_t t) const;

    // Tile t's answer to request seq has arrived whole: every entry of its
    // lines carries seq and every record its wave counts carries the
    // request's record tag (jsp_internal.h SplitArgs).
    bool tile_ready(const uint64_t* slots, uint32_t t, uint32_t seq) const;

    // The feasibility bitmaps of the last request (tests / diagnostics):
    // words [woff[c], woff[c+1]) of class c.
    const std::vector<uint64_t>& feas() const { return feas_; }
    // the feasibility build alone (timing: tools/walk_bench.py)
    void feasibility_only(const uint64_t* slots) { build_feasibility(slots); }

private:
    void build_feasibility(const uint64_t* slots);
    void take_marks(uint32_t d, uint32_t k);

    struct ClassWalk {
        const uint64_t* F;  // feasibility words
        uint64_t* T;        // taken words at the class's level
        uint32_t D, nw, k;  // domains at that level, their words, the level
        uint32_t cursor;    // first domain not yet passed
    };

    uint32_t K_ = 0, L_ = 0, C_ = 0, groups_ = 1, cpg_ = 1, nw_ = 1;
    uint32_t D_[kMaxLevels] = {0, 0, 0, 0};
    std::vector<uint32_t> fl_[kMaxLevels], cs_[kMaxLevels];
    std::vector<int32_t> par_[kMaxLevels];
    std::vector<uint32_t> level_, pods_, woff_, toff_, uoff_;
    std::vector<uint32_t> l0_, l1_;          // per row block
    std::vector<uint64_t> occ_;              // occupied leaves (bitmap)
    std::vector<uint64_t> occ_lvl_;          // occupied domains per level above the leaves (toff_ layout)
    std::vector<uint64_t> feas_;             // feasibility words of every class (woff_ layout)
    std::vector<uint64_t> sums_;             // clamped capacity sums of every upper class's domains (uoff_ layout)
    std::vector<uint64_t> taken_;            // taken domains per level (toff_ layout)
    std::vector<ClassWalk> cw_;              // per class, set up per request
    // per level, set up per walk: taken words, first leaf, child start, parent
    uint64_t* lv_t_[kMaxLevels] = {nullptr, nullptr, nullptr, nullptr};
    const uint32_t* lv_fl_[kMaxLevels] = {nullptr, nullptr, nullptr, nullptr};
    const uint32_t* lv_cs_[kMaxLevels] = {nullptr, nullptr, nullptr, nullptr};
    const int32_t* lv_par_[kMaxLevels] = {nullptr, nullptr, nullptr, nullptr};
    bool any_upper_ = false;
};

}  // namespace jsp
