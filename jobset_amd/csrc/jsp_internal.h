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
constexpr int kWaveTileRows = 256;                 // one wave's chunk: 64 lanes x 4 rows
constexpr int kWaveTileLeaves = 64;                // leaves of a multi-leaf wave tile (one per lane)
constexpr int kTallyClasses = 16;                  // classes per tally pass
constexpr int kAssignThreads = 1024;               // 16 waves, one workgroup
constexpr int kAssignWaves = kAssignThreads / 64;
constexpr int kMaxClasses = 64;
constexpr uint32_t kMaxLevels = 4;                 // JSP_MAX_LEVELS
constexpr uint32_t kMaxTakenWords = 16384;         // 128 KiB of LDS: 1M domain bits over all levels

// Device copy of a jsp_job_class, pre-digested for the tally's inner loop:
// one mask test per label word, one AND per taint word, and an exact
// floor(free / req) per resource as one f64 multiply by a pre-rounded
// reciprocal (no integer division).
struct alignas(16) DevClass {
    uint64_t req[4];      // bits that must be set
    uint64_t mask[4];     // req | forbid: a row passes when (labels & mask) == req
    uint32_t tol_inv;     // ~tolerated_taints: a row passes when (taints & tol_inv) == 0
    uint32_t level;
    uint32_t pods;
    uint32_t pad;
    uint32_t res[4];      // per-pod request, 0 = none
    double rcp[4];        // res >= 2: floor(n / res) = (uint32)(double(n) * rcp), exact for every u32 n
                          //   (rcp = 1/res (1 + 2^-45)); res == 1: 1.0
};

// A long run's step gives away the taken bits of a window word: one record per
// such word (assign_kernel), expanded to assign[] by expand_kernel. Each taken
// domain is in exactly one record, so J records always suffice.
struct alignas(16) AssignRec {
    uint32_t dom0;   // domain of bit 0 of the word
    uint32_t base;   // job of the lowest taken bit
    uint64_t took;   // taken bits
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
    const uint4* blk;           // per workgroup {first leaf, end leaf, first row, end row}
    uint32_t n_blocks;
    uint32_t la;                // leaf stride of the LDS tallies: max leaves of a block, rounded up to 4
    const DevClass* cls;
    uint32_t c0, nc;
    int do_occ;
    uint32_t* cap_out;
    uint32_t* occ_out;
    uint32_t ld, leaf_base;
    int W, R;
    int sc1_out;                // write cap/occ write-through (sc1): the fused kernel's hand-off to its tail
    // Feasibility folded into the wave tally (every class of the pass at the
    // leaf level, unsharded snapshot): each wave tile sets its leaves' bits of
    // class c's words at feas_fold + c * fold_nw (an atomic AND of its bit
    // range, then an OR of its bits), so no feasibility launch follows. Null: off.
    uint64_t* feas_fold;
    uint32_t fold_nw;
    // In-kernel span of the one-tile wave tally (jspb_tally_device_spans):
    // lane 0 of every wave stores {its start, its end after its stores
    // drained} (100 MHz clock) at [2 t, 2 t + 1] for wave tile t. Null: off.
    unsigned long long* wstamps;
};

// Single-launch kernels run an oversubscribed grid (n_blocks + kSpareBlocks
// workgroups): each workgroup draws a tile from a ticket and workgroups that
// draw past the last tile exit at once. On an idle GPU the XCDs start a
// launch's workgroups up to ~4 us apart, so the tiles go to the
// workgroups that started first instead of waiting for the last XCD.
constexpr uint32_t kSpareBlocks = 64;

// Bounded waits inside a launch (the pipelined batch walk's polls of an
// earlier batch, the level walk's expanders' wait for the walker): a wait
// that gives up writes `tag` to the engine's host-mapped error word, which the
// host reports as JSP_EHIP (jsp_engine.cc check_launch_error) -- never a stale
// assign[] with success. The tag's top two bits say which wait (kErr*); the
// compaction's look-back writes its launch number (kind 0).
// kErrMicro: a resident compaction tile whose microbox wait gave up (its
// registers may lack the request's patched rows; it writes no answer line)
constexpr uint32_t kErrLookback = 0u, kErrExpand = 1u << 30, kErrPipe = 2u << 30, kErrMicro = 3u << 30,
                   kErrKindMask = 3u << 30;
struct WaitErr {
    uint32_t* err;         // host-mapped error word (null: no report)
    uint32_t tag;          // written there by a wait that gave up
    uint32_t pipe_spins;   // polls of the pipelined batch walk before it gives up
    uint64_t wait_ticks;   // 100 MHz ticks the level walk's expanders wait for the walker
};

// Tail of place_fused_kernel (the last tally workgroup runs the assignment).
struct FusedArgs {
    unsigned long long* ticket;  // [0] tile ticket, [1] finished-tile count; zeroed at snapshot upload
    unsigned long long tile_base;  // ticket[0] before this launch (the host counts every draw)
    unsigned long long done_base;  // ticket[1] before this launch
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
    uint32_t topo_in_lds;        // hierarchy tables staged in LDS for the tail
    uint32_t topo_lds_words;     // their size (0 when not staged)
    uint32_t fscr_words;         // LDS scratch (u64) for upper-level domain sums + occupancy bits, 0 = none
    uint32_t* done;              // host-mapped completion word (host path) or null
    uint32_t epoch;              // value written to *done when the tail has finished
    uint32_t groups;             // class groups: tile t tallies row block t / groups, classes of group t % groups
    uint32_t cpg;                // classes per group (group 0 also counts occupancy)
    WaitErr we;                  // the pipelined batch walk's bounded wait
};

// A fused tile's share: row block and class range.
struct FusedTile {
    uint32_t blk, c0, nc;
    int do_occ;
};
__host__ __device__ inline FusedTile fused_tile(uint32_t t, uint32_t groups, uint32_t cpg, uint32_t C) {
    FusedTile x;
    x.blk = t / groups;
    const uint32_t g = t % groups;
    x.c0 = g * cpg;
    x.nc = C > x.c0 ? (C - x.c0 < cpg ? C - x.c0 : cpg) : 0u;
    x.do_occ = g == 0 ? 1 : 0;
    return x;
}

// Single-class leaf-level placement as one compaction pass (decoupled look-back).
struct CompactArgs {
    unsigned long long* ticket;    // shared with FusedArgs::ticket ([0] only)
    unsigned long long tile_base;  // ticket[0] before this launch
    unsigned long long* granules;  // [n_blocks] {epoch|status, value}, zeroed at snapshot upload
    uint32_t pods;
    uint32_t n_runs;
    uint32_t J;
    int32_t* assign;
    uint32_t* stats;               // [0] runs [1] placed
    uint32_t epoch;                // per-launch tag (host counter), 30-bit, never 0
    uint32_t* err;                 // host-mapped error word: a tile whose look-back timed out writes epoch
    uint32_t* done;                // host-mapped [n_blocks] completion words (host path) or null
    uint32_t spin_limit;           // look-back polls before a tile gives up (JSP_LOOKBACK_SPINS in tests)
};

// Resident placement service (place_service_kernel): the compaction shape kept
// on the GPU between host-API placements, fed through a host-mapped request
// word instead of a launch.
constexpr uint32_t kSvcStop = 0xFFFFFFFFu;  // request word's low half: every workgroup leaves
constexpr uint32_t kSvcClkSlots = 8;        // per tile: seen, acquired, tallied, scanned, looked back, drained
// A snapshot patch the service's dispatcher applies (request bit kReqPatch):
// host-mapped, written by the host before the request is posted.
struct PatchDesc {
    const uint32_t* rows;     // [n] row ids
    const uint64_t* dlab;     // [W][n] or null
    const uint32_t* dtaint;   // [n] or null
    const uint32_t* dfree;    // [R][n] or null
    const int32_t* dexcl;     // [n] or null
    uint32_t n;
    uint32_t seq;             // written to ServiceArgs::pdone once every row is in memory
};
// Request word bits above J (J < 2^28): 31 rows patched since the tiles'
// previous request, 30 apply the staged patch first, 29 nothing behind it,
// 28 the patch is inline (below) and the request's n_runs word is
// n | column flags << 16.
constexpr uint32_t kReqDirty = 1u << 31, kReqPatch = 1u << 30, kReqPatchOnly = 1u << 29,
                   kReqPatchInline = 1u << 28;
// The bell's J word (the dispatcher's copy of the request): bit 31 the rows
// changed (every tile reloads them), bit 30 the request's micro-patch rows
// are in the microbox (ServiceArgs::mbox: the resident tiles take them from
// there instead of reloading), bits 0..27 J.
constexpr uint32_t kBellMicro = 1u << 30;
// Inline patch staging (ServiceArgs::pstage, host-mapped, one fixed buffer per
// service): a 64-B header {seq}, then rows[n], then (8-B aligned) the present
// columns in the order labels [W][n] u64, taints [n], free [R][n], excl [n].
// Its layout follows from n and the flags alone, so the dispatcher issues
// every load of a patch at once -- one host-link round trip, no pointer chase.
constexpr uint32_t kPatchInlineRows = 4096;
constexpr uint32_t kPatchLab = 1, kPatchTaint = 2, kPatchFree = 4, kPatchExcl = 8;
struct PatchInlineLayout {
    size_t rows, lab, taint, free, excl, bytes;
};
__host__ __device__ inline PatchInlineLayout patch_inline_layout(uint32_t n, uint32_t flags, uint32_t W, uint32_t R) {
    PatchInlineLayout L{};
    L.rows = 64;
    size_t o = (64 + (size_t)n * 4 + 7) & ~size_t(7);
    L.lab = o;
    if (flags & kPatchLab) o += (size_t)W * n * 8;
    L.taint = o;
    if (flags & kPatchTaint) o += (size_t)n * 4;
    L.free = o;
    if (flags & kPatchFree) o += (size_t)R * n * 4;
    L.excl = o;
    if (flags & kPatchExcl) o += (size_t)n * 4;
    L.bytes = o;
    return L;
}

// The request line in pinned host memory (ServiceArgs::mailbox), read by the
// dispatcher in one load of kMailboxChunks 16-byte chunks, each written by one
// 16-byte host store and tagged with the request's seq (a torn read shows two
// seqs and is read again):
//   chunk 0 {seq, J | request bits, seq, n_runs (or an inline patch's n | flags << 16)}
//   chunk 1 {seq, micro rows m, patch number, column flags}
//   chunks 2.. {seq, 3 payload words}: m micro-patch rows of 3 + 2W + R words
//     each {row, labels (u32 halves) [W], taint, free [R], excl} -- a patch
//     small enough to ride in the request itself (no staging read)
// A patch number equal to the one the dispatcher applied last is not applied
// again (a request carrying a patch whose completion word had not come back).
constexpr uint32_t kMailboxChunks = 8;
constexpr uint32_t kMailboxPayload = 3 * (kMailboxChunks - 2);  // micro-patch words per request
constexpr uint32_t kMailboxBytes = 16 * kMailboxChunks;
__host__ __device__ constexpr uint32_t micro_row_words(uint32_t W, uint32_t R) { return 3u + 2u * W + R; }
__host__ __device__ constexpr uint32_t micro_rows_max(uint32_t W, uint32_t R) {
    return kMailboxPayload / micro_row_words(W, R);
}

struct ServiceArgs {
    const unsigned long long* mailbox;  // host-mapped kMailboxBytes request line (above)
    unsigned long long* granules;       // [n_blocks] the service's own look-back granules (tag = seq)
    unsigned long long* bell;           // device word: the dispatcher's copy of the request word (sc1)
    uint32_t pods;
    uint32_t seq0;                      // the request word's seq at launch (already answered)
    int32_t* assign;                    // host-mapped [capacity >= J of every request]
    uint32_t* stats;                    // host-mapped [2]: runs (1), placed
    uint32_t* done;                     // host-mapped [n_blocks]: seq of the last answered request
    uint32_t* err;                      // host-mapped: a tile whose look-back timed out writes its epoch
    uint32_t* clk;                      // host-mapped [kSvcClkSlots (n_tiles + 1)] 100 MHz phase stamps, or null:
                                        //   a row per tile, then the dispatcher's {request seen, bell rung}
    uint32_t n_tiles;                   // tiles of the grid (the dispatcher's clk row follows theirs)
    uint32_t spin_limit;
    unsigned long long idle_ticks;      // 100 MHz ticks without a request before a workgroup leaves
    uint32_t* ready;                    // host-mapped: the dispatcher writes gen once it polls
    uint32_t gen;                       // service launch number
    uint32_t row_cache_words;           // split shape: LDS word offset of the tiles' row copy, 0 = none
    uint32_t anc_words;                 // split shape: LDS word offset of the tiles' ancestor words
                                        //   (split_anc_words), 0 = none
    // XCD co-location (compaction shape): the grid is spread x (tiles + 1)
    // workgroups and only those with blockIdx % spread == 0 stay -- one XCD
    // under the round-robin dealing of workgroups to XCDs. Each survivor
    // publishes its XCC id in xcc[] (tagged with gen); when all agree, the
    // bell and the look-back granules are written as plain stores that stay
    // in that XCD's L2 (the sc1 loads that poll them are L2 hits); otherwise
    // they stay write-through (correct on any placement). spread 1: off.
    uint32_t spread;
    uint32_t* xcc;                      // device [tiles + 1] vote words
    // compaction shape, every tile one chunk: the tile's rows stay in
    // registers between requests, its class in scalar registers and its
    // leaves' row bounds in registers (place_service_kernel's resident path)
    uint32_t resident;
    const PatchDesc* pdesc;             // host-mapped patch descriptor (kReqPatch)
    const char* pstage;                 // host-mapped inline patch staging (kReqPatchInline)
    uint32_t* pdone;                    // host-mapped: the applied patch's seq
    uint32_t* taken;                    // host-mapped: the seq of the request the dispatcher took last
    // compaction shape: the bitmap answer -- per tile one 64-byte line of its
    // leaves' feasibility (four 64-leaf ballots, each as two (seq << 32 |
    // 32 bits) halves); the host gives job j the j-th feasible leaf. null: the
    // per-job (seq << 32 | domain) entries in `assign` after a look-back.
    unsigned long long* bits;
    // the co-located resident compaction: the dispatcher's copy of a
    // micro-patch for its tiles (kBellMicro), device memory, each word tagged
    // with the request's seq (seq << 32 | word): [0] m | flags << 16, then
    // the m rows of micro_row_words; or null
    unsigned long long* mbox;
    uint32_t micro_spins;               // passes over the microbox before a tile gives up (kErrMicro)
    // split shape launched for one request (launch_split_oneshot): the
    // request's seq, tiles only (no dispatcher), rows from memory; 0 = service
    uint32_t oneshot;
};

// Split service (place_split_service_kernel): the fused shape's tiles stay
// resident and hand the host, per request, only what the sequential greedy
// needs -- per tile and class, the feasibility bits of its leaves (leaf-level
// classes) or its partial capacity sums per upper-level domain (upper
// classes), plus its leaves' occupancy bits -- through pinned host memory; the
// host runs the O(J + C D / 64) walk.
// Per tile, split_tile_words(cpg, nw) u64 (nw: the waves of the largest tile
// that hold leaves, 64 leaves each), every one tagged with the request, so its
// arrival is the signal (no done word, no store-retirement wait). First the
// tile's lines: for class slot j (j = cpg: the leaves' occupancy) and wave
// w < nw, entries 2 (j nw + w) and + 1 = (seq << 32) | 32 bits -- the low and
// high halves of the ballot of leaves [64w, 64w + 64) of the tile (a
// leaf-level class, the occupancy), or the wave's record count and 0 (an upper
// class) -- rounded up to whole 64-byte lines: the host reads every line a
// device write just invalidated, one miss each, so the layout is dense (cfg3:
// one line per tile, not one per class and wave). Then, per upper class slot j
// and wave w, kSplitRecs records (split_rec_tag(seq) << 50) | (domain << 30) |
// partial clamped capacity sum (< 2^30). Upper-level domains must number
// < 2^20 (split_ok).
constexpr uint32_t kSplitRecs = 64;
constexpr uint32_t kSplitMaxDomains = 1u << 20;
__host__ __device__ constexpr uint32_t split_line_words(uint32_t cpg, uint32_t nw) {
    return (2u * (cpg + 1u) * nw + 7u) & ~7u;
}
__host__ __device__ constexpr uint32_t split_tile_words(uint32_t cpg, uint32_t nw) {
    return split_line_words(cpg, nw) + nw * kSplitRecs * cpg;
}
__host__ __device__ constexpr uint64_t split_rec_tag(uint32_t seq) { return (uint64_t)(seq % 16383u + 1u); }
struct SplitArgs {
    uint32_t groups, cpg, C;
    uint32_t nw;    // waves of the largest tile that hold leaves (1..4)
    uint64_t* out;  // host-mapped [n_tiles][split_tile_words(cpg, nw)]
    TopoDev topo;
    // one-request launch of a device-resident run list (ServiceArgs::oneshot):
    // tile 0 copies it to run_dst (host-mapped, class then length) before its
    // lines, so the host has it once every tile's lines are in; null: none
    const uint32_t* run_class;
    const uint32_t* run_len;
    uint32_t* run_dst;
    uint32_t n_runs;
    // ... and its assign[] copy in one extra workgroup (null flag: none):
    // after the host walk's release of cw_tag in cw_flag, cw_n words from the
    // host-mapped cw_src to the device buffer cw_dst (copy_after_release)
    const uint32_t* cw_flag;
    uint32_t cw_tag;
    const uint32_t* cw_src;
    uint32_t* cw_dst;
    uint32_t cw_n;
    uint32_t* cw_err;
    uint32_t cw_err_tag;
    unsigned long long cw_ticks;
};

constexpr int assign_small_words(int nt) { return 2 * (nt / 64) + 8 + 3 * kMaxClasses + (kMaxClasses + 1) + 4 * 8 + 3 * nt + 64; }
constexpr uint32_t kFusedMaxWords = 6144;  // taken + feasibility words the fused tail keeps in LDS (48 KiB)
constexpr uint32_t kFusedStage = 2048;     // ranks the fused tail stages per long-run step (8 KiB)
constexpr uint32_t kMinStage = 4096;       // assign_kernel stages the bitmaps in LDS only if this much stage remains
constexpr uint32_t kMaxStage = 32768;
constexpr uint32_t kFusedTopoMax = 8192;   // hierarchy-table words the fused tail stages in LDS (32 KiB)
constexpr uint32_t kFusedScrMax = 4096;    // upper-level feasibility scratch of the fused tail (u64 words, 32 KiB)
constexpr size_t kLdsBytes = 160 * 1024;   // gfx950 LDS per workgroup
// window of a long-run step: NT u64 words + NT u32 ranks, in u64 units
constexpr uint32_t kAssignWinWords64 = kAssignThreads + kAssignThreads / 2;
constexpr uint32_t kFusedWinWords64 = kTallyThreads + kTallyThreads / 2;

// Words of the LDS copy of the hierarchy tables (parent[k] for k >= 1,
// child_start[k] for k < K-1), in the order stage_meta numbers them.
__host__ __device__ inline uint32_t topo_table_words(uint32_t K, const uint32_t* D) {
    uint32_t t = 0;
    for (uint32_t k = 0; k < K; ++k) {
        if (k >= 1) t += D[k];
        if (k + 1 < K) t += D[k] + 1;
    }
    return t;
}

// LDS plan of assign_kernel: the hierarchy tables, then the feasibility
// bitmaps, are staged in LDS when they fit beside the taken bitmaps.
struct AssignPlan {
    uint32_t feas_in_lds;
    uint32_t topo_in_lds;
    uint32_t stage_cap;  // ranks per long-run step
    size_t lds_bytes;    // 0: does not fit
};
AssignPlan plan_assign(uint32_t t_words, uint32_t feas_words, uint32_t topo_words);

// While set (non-null), every launch records `ev` at its kernel's completion
// (the device-path calls' end-of-call marker); launch_stop_used() says whether
// a launch did since the last set.
void set_launch_stop(hipEvent_t ev);
void set_launch_start(hipEvent_t ev);  // the next launch's start event (then cleared)
bool launch_stop_used();
// the stop event set for the coming launches, cleared (a call whose last
// launch alone should carry it sets it back with set_launch_stop)
hipEvent_t take_launch_stop();
// host-link floor probe (instrumentation): four polling waves answer request
// numbers 1..n of *req in ack[16 w] (pinned host memory)
hipError_t launch_link_probe(const uint32_t* req, uint32_t* ack, uint32_t n, uint64_t wait_ticks, hipStream_t s);
// an empty launch of `grid` 256-thread workgroups (instrumentation)
hipError_t launch_empty(uint32_t grid, hipStream_t s);
// read-only cache scrub of `bytes` (instrumentation: cold-cache timings)
hipError_t launch_scrub(const void* p, size_t bytes, uint32_t* sink, hipStream_t s);
hipError_t launch_tally(const TallyArgs& a, hipStream_t s);
// Wave-tile tally (tally_wave_kernel): tiles {first leaf, end leaf, first row,
// end row} of up to kWaveTileLeaves whole leaves in <= kWaveTileRows - 4 rows
// (snapshots with a larger leaf use the workgroup tally), 1-4 classes and the
// occupancy count in one pass; `grid` workgroups of 4 waves take them in turn. Every column's bytes must stay below 2^31
// (buffer offsets; the host checks).
hipError_t launch_tally_wave(const TallyArgs& a, const uint4* tiles, uint32_t n_tiles, uint32_t n_leaves, uint32_t grid,
                             hipStream_t s);
size_t tally_wave_lds_bytes(uint32_t nc, uint32_t nv);
hipError_t launch_fused(const TallyArgs& a, const FusedArgs& f, hipStream_t s);
hipError_t launch_compact(const TallyArgs& a, const CompactArgs& f, hipStream_t s);
hipError_t launch_service(const TallyArgs& a, const ServiceArgs& v, hipStream_t s);
// LDS of the compaction service: the compaction's, then (row_cache) the tile's
// rows kept between requests, from word service_row_cache_words(la) on
uint32_t service_row_cache_words(uint32_t la);
size_t service_lds_bytes(uint32_t la, int W, int R, bool row_cache);
size_t compact_lds_bytes(uint32_t la);
hipError_t launch_split_service(const TallyArgs& a, const SplitArgs& sp, const ServiceArgs& v, hipStream_t s);
// the split tiles for one request (ServiceArgs::oneshot): grid = tiles
hipError_t launch_split_oneshot(const TallyArgs& a, const SplitArgs& sp, const ServiceArgs& v, hipStream_t s);
size_t split_lds_bytes(uint32_t cpg, uint32_t la);
// the split service's LDS: split_lds_bytes, then (row_cache) the tile's rows
uint32_t split_row_cache_words(uint32_t cpg, uint32_t la);
uint32_t split_anc_words(uint32_t cpg, uint32_t la, int W, int R, bool row_cache);
size_t split_service_lds_bytes(uint32_t cpg, uint32_t la, int W, int R, bool row_cache);
// Workgroups of the resident service kernel (shape 2 compaction, 3 split) of
// this W/R that one CU holds at once with lds_bytes each (occupancy API).
hipError_t service_occupancy(const TallyArgs& a, int shape, size_t lds_bytes, int* blocks_per_cu);
size_t fused_lds_bytes(uint32_t t_words, uint32_t feas_words, uint32_t nc, uint32_t nv, uint32_t la,
                       uint32_t topo_words, uint32_t fscr_words);
// u64 words of the fused tail's upper-level feasibility scratch: one sum per
// domain of every class above the leaves, one occupancy bit per domain of
// every level above the leaves; 0 when there is no such class or it exceeds
// kFusedScrMax (the tail then builds those words one wave per word).
uint32_t fused_scratch_words(uint32_t K, const uint32_t* D, const uint32_t* class_level, uint32_t C);
hipError_t launch_copy_u32(const uint32_t* src, uint32_t* dst, uint32_t n, hipStream_t s);
hipError_t launch_tag(uint32_t* dst, uint32_t v, hipStream_t s);
hipError_t launch_copy_wait(const uint32_t* flag, uint32_t tag, const uint32_t* src, uint32_t* dst, uint32_t n,
                            uint32_t* err, uint32_t err_tag, unsigned long long ticks, hipStream_t s);
// kind of a timed-out device-path copy wait in the engine's error word
constexpr uint32_t kErrCopyWait = 3u << 30;
hipError_t launch_feas(const uint32_t* cap, const uint32_t* occ, uint32_t ld, const DevClass* cls, uint32_t C,
                       const uint32_t* word_off, uint32_t total_words, const TopoDev& topo, uint64_t* feas,
                       hipStream_t s);
hipError_t launch_assign(const uint64_t* feas, const uint32_t* word_off, const DevClass* cls, uint32_t C,
                         const TopoDev& topo, uint32_t t_words, uint32_t feas_words, const uint32_t* run_class,
                         const uint32_t* run_len, uint32_t n_runs, uint32_t J, int32_t* assign, uint32_t* stats,
                         uint32_t* rec_count, AssignRec* recs, hipStream_t s, const WaitErr& we);
// The level walker (assign_level_kernel): every class at one topology level
// of nw <= kLevelMaxWords words and at most kLevelMaxRuns runs. 256 threads
// hold the taken bits of their words in registers and walk the runs in
// order; per run one block scan of the free feasible counts hands the run its
// lowest free feasible domains; one record per word that gives domains away
// (expand_kernel writes assign[]). Returns hipErrorInvalidValue when the
// shape does not fit (the caller runs assign_kernel).
constexpr uint32_t kLevelMaxWords = 256 * 8;
constexpr uint32_t kLevelMaxRuns = 32;
size_t level_walk_lds_bytes(uint32_t C, uint32_t nw);
// ready (device u64): the walker publishes (epoch << 32 | 1 << 31 | record
// count) there once its records are written, and the launch's other
// workgroups expand them (epoch: new per launch, != 0); an expander that
// waits longer than we.wait_ticks writes we.tag to the error word.
hipError_t launch_assign_level(const uint64_t* feas, uint32_t C, uint32_t nw, const uint32_t* run_class,
                               const uint32_t* run_len, uint32_t n_runs, uint32_t J, int32_t* assign, uint32_t* stats,
                               uint32_t* rec_count, AssignRec* recs, hipStream_t s, unsigned long long* ready,
                               uint32_t epoch, const WaitErr& we);
hipError_t launch_resolve(const int32_t* rows, const uint32_t* levels, uint32_t n, uint32_t n_rows,
                          const uint32_t* leaf_start, uint32_t n_leaves, uint32_t leaf_base, const TopoDev& topo,
                          int32_t* out, hipStream_t s);
hipError_t launch_audit(const int32_t* leader_rows, const uint32_t* levels, const uint32_t* foff,
                        const int32_t* fdom, uint32_t n_jobs, uint32_t n_rows, const uint32_t* leaf_start,
                        uint32_t n_leaves, uint32_t leaf_base, const TopoDev& topo, uint32_t* bad, hipStream_t s);

// dst += src (n words, 16-B aligned buffers): shards of a device set on one device
hipError_t launch_add_u32(uint32_t* dst, const uint32_t* src, size_t n, hipStream_t s);

// A snapshot patch: n rows overwritten from a dense delta in pinned host
// memory ([n] rows, [W][n] labels, [n] taints, [R][n] free, [n] excl; a null
// column is left as is). done != nullptr: the last workgroup to finish writes
// seq there (host-mapped) after every row store has drained; counter is a
// device word every launch adds its grid to, target = its value after this one.
struct PatchArgs {
    const uint32_t* rows;
    uint32_t n, npad, W, R;
    const uint64_t* dlab;
    const uint32_t* dtaint;
    const uint32_t* dfree;
    const int32_t* dexcl;
    uint64_t* labels;
    uint32_t* taints;
    uint32_t* freer;
    int32_t* excl;
    unsigned long long* counter;
    unsigned long long target;
    uint32_t* done;
    uint32_t seq;
};
hipError_t launch_patch(const PatchArgs& a, hipStream_t s);

}  // namespace jsp
