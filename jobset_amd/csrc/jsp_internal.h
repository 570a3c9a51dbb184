// jsp_internal.h — shared declarations between the engine host code and the
// gfx950 kernels (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace jsp {

constexpr int kTallyThreads = 256;                 // 4 waves
constexpr int kTallyWaves = kTallyThreads / 64;
constexpr int kRowsPerThread = 4;                  // 16-B column loads
constexpr int kChunkRows = kTallyThreads * kRowsPerThread;
constexpr int kMaxBlkLeaves = 256;                 // leaves one tally workgroup may own
constexpr int kTallyClasses = 16;                  // classes per tally pass
constexpr int kAssignThreads = 1024;               // 16 waves, one workgroup
constexpr int kAssignWaves = kAssignThreads / 64;
constexpr int kMaxClasses = 64;
constexpr uint32_t kMaxTakenWords = 18432;         // 144 KiB of LDS: 1.18M domain bits over all levels

// Device copy of a jsp_job_class (+ reciprocals of the per-pod requests).
struct alignas(16) DevClass {
    uint64_t req[4];
    uint64_t forbid[4];
    uint32_t tol;
    uint32_t level;
    uint32_t pods;
    uint32_t pad;
    uint32_t res[4];
    float rcp[4];
};

// Domain hierarchy on the device (passed by value).
struct TopoDev {
    uint32_t K;
    uint32_t D[4];
    const uint32_t* fl[4];   // first_leaf[k] [D_k+1], k < K-1
    const uint32_t* cs[4];   // child_start[k] [D_k+1]: range at level k+1, k < K-1
    const int32_t* par[4];   // parent[k] [D_k]: domain at level k-1, k >= 1
};

struct TallyArgs {
    const uint64_t* labels;
    const uint32_t* taints;
    const uint32_t* freer;
    const int32_t* excl;
    uint32_t npad;
    const uint32_t* leaf_start;
    const uint32_t* blk_leaf;
    uint32_t n_blocks;
    const DevClass* cls;
    uint32_t c0, nc;
    int do_occ;
    uint32_t* cap_out;
    uint32_t* occ_out;
    uint32_t ld, leaf_base;
    int W, R;
};

hipError_t launch_tally(const TallyArgs& a, hipStream_t s);
hipError_t launch_feas(const uint32_t* cap, const uint32_t* occ, uint32_t ld, const DevClass* cls, uint32_t C,
                       const uint32_t* word_off, uint32_t total_words, const TopoDev& topo, uint64_t* feas,
                       hipStream_t s);
hipError_t launch_assign(const uint64_t* feas, const uint32_t* word_off, const DevClass* cls, uint32_t C,
                         const TopoDev& topo, const uint32_t* t_off, uint32_t t_words, const uint32_t* job_class,
                         uint32_t J, int32_t* assign, uint32_t* stats, hipStream_t s);
hipError_t launch_resolve(const int32_t* rows, const uint32_t* levels, uint32_t n, uint32_t n_rows,
                          const uint32_t* leaf_start, uint32_t n_leaves, uint32_t leaf_base, const TopoDev& topo,
                          int32_t* out, hipStream_t s);
hipError_t launch_audit(const int32_t* leader_rows, const uint32_t* levels, const uint32_t* foff,
                        const int32_t* fdom, uint32_t n_jobs, uint32_t n_rows, const uint32_t* leaf_start,
                        uint32_t n_leaves, uint32_t leaf_base, const TopoDev& topo, uint32_t* bad, hipStream_t s);

hipError_t launch_patch(const uint32_t* rows, uint32_t n, uint32_t npad, uint32_t W, uint32_t R,
                        const uint64_t* dlab, const uint32_t* dtaint, const uint32_t* dfree, const int32_t* dexcl,
                        uint64_t* labels, uint32_t* taints, uint32_t* freer, int32_t* excl, hipStream_t s);

}  // namespace jsp
