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
constexpr uint32_t kMaxTakenWords = 16384;         // 128 KiB of LDS: 1M domain bits over all levels

// Device copy of a jsp_job_class, pre-digested for the tally's inner loop:
// one mask test per label word, one AND per taint word, and an exact
// division-free floor(free / req) per resource (multiply-high by an
// invariant-divisor magic number, branch-free form).
struct alignas(16) DevClass {
    uint64_t req[4];      // bits that must be set
    uint64_t mask[4];     // req | forbid: a row passes when (labels & mask) == req
    uint32_t tol_inv;     // ~tolerated_taints: a row passes when (taints & tol_inv) == 0
    uint32_t level;
    uint32_t pods;
    uint32_t pad;
    uint32_t res[4];      // per-pod request, 0 = none
    uint32_t magic[4];    // floor(n / res) = (((n - mulhi(n, magic)) >> 1) + mulhi(n, magic)) >> shift
    uint32_t shift[4];    // kDivIdentity marks res == 1
};
constexpr uint32_t kDivIdentity = 0xFFFFFFFFu;

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
    const uint4* blk;           // per workgroup {first leaf, end leaf, first row, end row}
    uint32_t n_blocks;
    const DevClass* cls;
    uint32_t c0, nc;
    int do_occ;
    uint32_t* cap_out;
    uint32_t* occ_out;
    uint32_t ld, leaf_base;
    int W, R;
};

// Tail of place_fused_kernel (the last tally workgroup runs the assignment).
struct FusedArgs {
    unsigned long long* ticket;  // zeroed at snapshot upload, grows by n_blocks per launch
    uint32_t C;
    TopoDev topo;
    const uint32_t* t_off;
    uint32_t t_words;
    const uint32_t* word_off;
    uint32_t feas_words;
    const uint32_t* run_class;
    const uint32_t* run_len;
    uint32_t n_runs;
    uint32_t J;
    int32_t* assign;
    uint32_t* stats;
    size_t lds_bytes;
};

// Single-class leaf-level placement as one compaction pass (decoupled look-back).
struct CompactArgs {
    unsigned long long* ticket;    // shared with FusedArgs::ticket
    unsigned long long* granules;  // [n_blocks] {epoch|status, value}, zeroed at snapshot upload
    uint32_t pods;
    uint32_t n_runs;
    uint32_t J;
    int32_t* assign;
    uint32_t* stats;               // [0] runs [1] placed [2] look-back timeout flag
    uint32_t epoch;                // per-launch tag (host counter), 30-bit, never 0
    uint32_t coresident;           // 1: every workgroup is resident at once, tile = blockIdx.x
};

constexpr int assign_small_words(int nt) { return 2 * (nt / 64) + 8 + 3 * kMaxClasses + (kMaxClasses + 1) + 8 + 2 * nt; }
constexpr uint32_t kFusedMaxWords = 6144;  // taken + feasibility words the fused tail keeps in LDS (48 KiB)

hipError_t launch_tally(const TallyArgs& a, hipStream_t s);
hipError_t launch_fused(const TallyArgs& a, const FusedArgs& f, hipStream_t s);
hipError_t launch_compact(const TallyArgs& a, const CompactArgs& f, hipStream_t s);
size_t compact_lds_bytes();
size_t fused_lds_bytes(uint32_t t_words, uint32_t feas_words, uint32_t nv);
size_t assign_lds_bytes(uint32_t t_words);
hipError_t launch_feas(const uint32_t* cap, const uint32_t* occ, uint32_t ld, const DevClass* cls, uint32_t C,
                       const uint32_t* word_off, uint32_t total_words, const TopoDev& topo, uint64_t* feas,
                       hipStream_t s);
hipError_t launch_assign(const uint64_t* feas, const uint32_t* word_off, const DevClass* cls, uint32_t C,
                         const TopoDev& topo, uint32_t t_words, const uint32_t* run_class, const uint32_t* run_len,
                         uint32_t n_runs, uint32_t J, int32_t* assign, uint32_t* stats, hipStream_t s);
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
