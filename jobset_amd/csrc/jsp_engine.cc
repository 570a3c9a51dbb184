// jsp_engine.cc — host side of the exclusive-topology placement engine:
// the C ABI of include/jsplace.h over HIP device buffers and the kernels of
// jsp_kernels.hip. See DESIGN.md for the data layout and the rules.
#include <emmintrin.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/jsplace_bench.h"
#include "jsp_internal.h"
#include "jsp_multi.h"
#include "jsp_walk.h"

namespace {

thread_local std::string g_err;

int set_err(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

// One value into a log2 histogram (jsplace.h jsp_hist): bucket 0 below lo,
// bucket i in [lo 2^(i-1), lo 2^i), the last one the rest.
void hist_add(jsp_hist& h, double v, double lo) {
    h.count += 1;
    h.sum += v;
    if (v > h.max) h.max = v;
    int i = 0;
    if (v >= lo) {
        int ex = 0;
        (void)std::frexp(v / lo, &ex);
        i = std::min(ex, JSP_HIST_BUCKETS - 1);
    }
    h.bucket[i] += 1;
}

#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t _e = (expr);                                                              \
        if (_e != hipSuccess)                                                                \
            return set_err(JSP_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e),  \
                           __FILE__, __LINE__);                                              \
    } while (0)

// Buffers a grow-only buffer gave up while the resident service ran: hipFree
// and hipHostFree wait for every kernel on the device, the resident service
// included, which leaves only after JSP_SERVICE_IDLE_MS without a request --
// a free while it runs stalls the caller for up to that long
// (tools/block_probe.hip). They are freed once the service has stopped.
struct Grave {
    std::vector<void*> dev, host;
    void flush() {
        for (void* p : dev) (void)hipFree(p);
        for (void* p : host) (void)hipHostFree(p);
        dev.clear();
        host.clear();
    }
    ~Grave() { flush(); }
};

// Grow-only device buffer. `g`: where the old buffer goes when it must grow
// while a kernel that never ends by itself runs (nullptr: freed at once).
// The calling thread's current device, restored when an entry point that
// switches devices returns (the device-set engine walks its devices; a
// caller -- a torch rank, a Go thread -- keeps the device it had).
struct DeviceGuard {
    int prev = -1;
    DeviceGuard() { (void)hipGetDevice(&prev); }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    hipError_t reserve(size_t n, Grave* g = nullptr) {
        if (n <= bytes && p) return hipSuccess;
        if (g && p) {
            g->dev.push_back(p);
            p = nullptr;
            bytes = 0;
        }
        release();
        hipError_t e = hipMalloc(&p, n ? n : 16);
        if (e == hipSuccess) bytes = n ? n : 16;
        return e;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

// Pinned, device-mapped host memory: the host placement path hands run lists
// to the kernels and takes assign[] back through it without DMA copies
// (kernels read and write it over the host link directly).
struct HostBuf {
    void* p = nullptr;
    size_t bytes = 0;
    ~HostBuf() { release(); }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        bytes = 0;
    }
    hipError_t reserve(size_t n, Grave* g = nullptr) {
        if (n <= bytes && p) return hipSuccess;
        if (g && p) {
            g->host.push_back(p);
            p = nullptr;
            bytes = 0;
        }
        release();
        hipError_t e = hipHostMalloc(&p, n ? n : 16, hipHostMallocMapped | hipHostMallocCoherent);
        if (e == hipSuccess) bytes = n ? n : 16;
        return e;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

struct EvPair {
    hipEvent_t a = nullptr, b = nullptr;
    int tag = 0;  // 0 tally, 1 feas, 2 assign, 3 fused
};

// Test hooks: JSP_TEST_HOOKS="name=value,...", read at engine creation and
// again at each snapshot upload. They force, at test sizes, the shapes the
// engine otherwise picks only for large geometries (the double-buffered and
// workgroup tallies, multi-chunk tally blocks), shorten the kernels' bounded
// waits so that their error path runs, and stand in for a smaller GPU. The
// library's other environment switches are operational only: JSP_SERVICE,
// JSP_SERVICE_IDLE_MS and (device sets) JSP_RCCL_LIB.
struct TestHooks {
    bool tally_one = true;          // tally_one=0: the double-buffered wave tally at any size
    bool tally_block = false;       // tally_block=1: the workgroup tally instead of the wave tiles
    uint32_t block_chunks = 1;      // block_chunks=N (1..8): 1024-row chunks per tally workgroup
    uint32_t block_rows = 0;        // block_rows=N (>= 60): smaller tally row blocks (more tiles)
    uint32_t lookback_spins = 1u << 22;  // lookback_spins=N: compaction look-back polls before giving up
    uint32_t pipe_spins = 1u << 24;      // pipe_spins=N: the pipelined batch walk's polls of an earlier batch
    uint64_t wait_ticks = 200000000ull;  // wait_us=N: the level walk's expanders' wait (100 MHz ticks; 2 s)
    int cu_limit = 0;               // cu_limit=N: CUs the resident service may count on
    bool svc_xcd = true;            // svc_xcd=0: the compaction service spread over the XCDs (the
                                    //   write-through protocol a partition mode would run)
    uint32_t seq0 = 0;              // seq0=N: the service's first request number
    bool have_seq0 = false;
    bool svc_entries = false;       // svc_entries=1: the compaction service answers with per-job entries
                                    //   after a look-back instead of tile bitmaps (A/B)
    uint32_t loop_gap_ns = 0;       // loop_gap_ns=N: jspb_place_loop spins N ns between calls (diagnostic)
    uint32_t wait_delay_ns = 0;     // wait_delay_ns=N: the split wait spins N ns after the post (diagnostic)
    bool warm = true;               // warm=0: no call-entry prefetch of the engine's lines (A/B)
    uint32_t micro_spins = 1u << 22;  // micro_spins=N: a resident tile's passes over the microbox (kErrMicro)
    uint32_t waker_poll_us = 200;   // waker_poll_us=N: the armed waker's poll period; 0 = condition variable only
    bool waker_spin = false;        // waker_spin=1: the armed waker spins instead of sleeping (A/B: a host core
                                    //   kept awake, as the CPU evaluator's pool threads are)
};

TestHooks read_hooks() {
    TestHooks h;
    const char* s = std::getenv("JSP_TEST_HOOKS");
    if (!s) return h;
    std::string all(s);
    size_t p = 0;
    while (p < all.size()) {
        size_t q = all.find(',', p);
        if (q == std::string::npos) q = all.size();
        const std::string kv = all.substr(p, q - p);
        p = q + 1;
        const size_t eq = kv.find('=');
        if (eq == std::string::npos) continue;
        const std::string k = kv.substr(0, eq);
        const unsigned long long v = std::strtoull(kv.c_str() + eq + 1, nullptr, 0);
        if (k == "tally_one") h.tally_one = v != 0;
        else if (k == "tally_block") h.tally_block = v != 0;
        else if (k == "block_chunks" && v >= 1 && v <= 8) h.block_chunks = (uint32_t)v;
        else if (k == "block_rows" && v >= 60) h.block_rows = (uint32_t)v;
        else if (k == "lookback_spins") h.lookback_spins = (uint32_t)v;
        else if (k == "pipe_spins") h.pipe_spins = (uint32_t)v;
        else if (k == "wait_us") h.wait_ticks = v * 100ull;
        else if (k == "cu_limit") h.cu_limit = (int)v;
        else if (k == "svc_xcd") h.svc_xcd = v != 0;
        else if (k == "svc_entries") h.svc_entries = v != 0;
        else if (k == "loop_gap_ns") h.loop_gap_ns = (uint32_t)v;
        else if (k == "wait_delay_ns") h.wait_delay_ns = (uint32_t)v;
        else if (k == "warm") h.warm = v != 0;
        else if (k == "micro_spins") h.micro_spins = (uint32_t)v;
        else if (k == "waker_poll_us") h.waker_poll_us = (uint32_t)v;
        else if (k == "waker_spin") h.waker_spin = v != 0;
        else if (k == "seq0") {
            h.seq0 = (uint32_t)v;
            h.have_seq0 = true;
        }
    }
    return h;
}

}  // namespace

int jsp_internal_set_err(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

struct jsp_engine {
    int device = 0;
    jspm::Multi* multi = nullptr;  // a device-set engine (jsp_engine_create_multi): every call goes there
    int n_cu = 0;  // compute units (multiProcessorCount)
    hipStream_t stream = nullptr;
    std::mutex mu;

    // topology
    bool have_topo = false;
    uint32_t K = 0;
    uint32_t D[JSP_MAX_LEVELS] = {0, 0, 0, 0};
    uint32_t L_total = 0;
    DevBuf fl[JSP_MAX_LEVELS], cs[JSP_MAX_LEVELS], par[JSP_MAX_LEVELS];
    uint32_t t_off_h[JSP_MAX_LEVELS + 1] = {0, 0, 0, 0, 0};
    DevBuf t_off;
    jsp::TopoDev topo{};
    // host copies of the hierarchy tables (the split service's host walk)
    std::vector<uint32_t> h_fl[JSP_MAX_LEVELS], h_cs[JSP_MAX_LEVELS];
    std::vector<int32_t> h_par[JSP_MAX_LEVELS];
    std::vector<uint32_t> blk_l0, blk_l1;  // leaf range of each tally row block
    uint32_t max_blk_span = 0;             // rows a tally block's first chunk spans, max over blocks
    TestHooks hooks;                       // JSP_TEST_HOOKS (tests only; defaults otherwise)
    jsp::HostWalk walk;

    // snapshot
    bool have_snap = false;
    uint32_t N = 0, npad = 0, W = 0, R = 0, leaf_begin = 0, n_leaves = 0, max_leaf_rows = 0;
    uint32_t blk_leaves = 4;  // most leaves any tally workgroup owns, rounded up to 4 (LDS tally stride)
    DevBuf labels, taints, freer, excl, leaf_start, blk;
    DevBuf wtiles;              // wave tiles of the three-launch tally (tally_wave_kernel)
    uint32_t n_wtiles = 0;
    uint32_t n_blocks = 0;
    uint32_t epoch = 0;  // compaction launches so far (granule tags)

    // classes
    bool have_cls = false;
    uint32_t C = 0;
    std::vector<jsp::DevClass> cls_h;
    DevBuf cls, word_off, feas;
    uint32_t feas_words = 0;

    // scratch
    DevBuf cap, occ, run_class, run_len, assign, stats, ticket, granules, recs;
    HostBuf h_runs, h_assign, h_stats;  // zero-copy staging of the host placement path
    HostBuf h_done;                     // [n_blocks] completion words of the host placement path
    HostBuf h_err;                      // [1] error word: a failed launch writes its epoch (sticky)
    // snapshot patches run asynchronously: the delta is staged in pinned
    // memory the patch kernel reads in place, whose last workgroup writes
    // patch_seq to h_patch_done (patch_wait)
    HostBuf h_patch, h_patch_done;
    HostBuf h_batch;                    // pinned staging of the webhook / reconciler batches (A5, A9)
    DevBuf patch_ctr;                   // workgroups of every patch launch so far (device counter)
    unsigned long long patch_target = 0;
    uint32_t patch_seq = 0;
    bool patch_pending = false;
    // the device paths' host walks (host_walk_impl, split_oneshot): the
    // feasibility words (and a completion tag) in pinned memory, and a ring
    // of staging slots for the device paths' run list and assign[]:
    // a back-to-back call never waits for the previous call's assign[] copy
    // (it waited ~12 us for that copy's completion report, profiles/r06)
    struct WalkStage {
        HostBuf io;
        hipEvent_t ev = nullptr;
        bool pending = false;
    };
    static constexpr int kWalkStages = 4;
    WalkStage hw_stage[kWalkStages];
    uint32_t hw_next = 0;
    uint32_t hw_tag = 0;
    HostBuf hw_feas;
    // the split tiles launched for one request (split_oneshot): their answer
    // lines (pinned), the geometry the host walk's tile table was set for,
    // and the request numbers of these launches
    HostBuf os_split;
    unsigned long long os_key = ~0ull;
    uint32_t os_seq = 0;
    DevBuf lvl_ready;                   // the one-launch level walk's published record count
    uint32_t lvl_epoch = 0;
    uint32_t err_tag = 0;               // launches that may report a timed-out wait (kernel error words)
    bool patch_svc = false;             // the pending patch goes to the service's dispatcher
    bool patch_deferred = false;        // ... and is held back for the next request (not posted yet)
    uint32_t patch_bits = 0;            // its request bits (kReqPatch, kReqPatchInline)
    uint32_t patch_nf = 0;              // inline: n | column flags << 16 (the request's n_runs word)
    uint32_t patch_req = 0;             // the request that posted it alone (0: none)
    // A micro-patch (jsp_internal.h kMailbox*): a patch small enough to ride
    // in the next request's line, held back until a request carries it (no
    // staging read, no post of its own); patches of the same columns merge
    // into it while it is held
    bool patch_micro = false;
    uint32_t micro_n = 0, micro_fl = 0;  // its rows (distinct) and column flags
    uint32_t micro_w[jsp::kMailboxPayload] = {};
    // The waker: a host thread that restarts the service for a recovery's
    // first patch off the caller's thread (the launch after an idle period
    // costs ~10 us of host time). wake_job is guarded by mu; the thread
    // sleeps on wake_cv (wake_ring / wake_quit under wake_mu).
    bool wake_job = false;
    std::thread waker;
    std::mutex wake_mu;
    std::condition_variable wake_cv;
    std::atomic<bool> wake_ring{false}, wake_quit{false};
    // a ring is delivered after the caller releases mu (wake_notify) -- only
    // while the waker sleeps on wake_cv: while the service is armed it polls
    // wake_ring instead (waker_poll), so a recovery's first patch call makes
    // no system call
    std::atomic<bool> wake_notify{false};
    std::atomic<bool> waker_poll{false};     // the service is armed: the waker polls
    std::atomic<bool> waker_polling{false};  // the waker is in its polling loop
    jsp::PatchArgs last_patch{};        // its kernel form (the fallback when the service left without it)
    uint32_t err_ack = 0;               // last error word value reported to a caller
    uint32_t* stats_override = nullptr;  // kernels' stats go here when set (host path)
    int fused_mode = JSP_FUSED_AUTO;
    uint32_t last_shape = 0;  // 0 three launches, 1 fused tail, 2 single-class compaction
    // draws on the single-launch kernels' tickets so far (DevBuf ticket [0]
    // tiles, [1] finished tiles): every launch adds its grid / tile count
    unsigned long long tile_draws = 0, done_draws = 0;
    // look-back polls before a compaction tile gives up (hooks.lookback_spins,
    // taken at snapshot upload)
    uint32_t spin_limit = 1u << 22;

    // stream ordering: work is enqueued on the engine stream or a caller's;
    // the first call on a different stream waits for the previous one. A
    // caller's stream is touched only inside the call that was given it: the
    // call records ev_last on it before returning, and later calls wait on
    // that engine-owned event (the caller may destroy its stream meanwhile).
    hipStream_t last_stream = nullptr;  // compared, never used after its call returned
    bool foreign_pending = false;       // device-path work on a caller's stream not yet waited for (ev_last)
    bool have_last = false;
    bool last_foreign = false;          // the last call enqueued on a caller's stream
    hipEvent_t ev_switch = nullptr;     // recorded on the engine stream
    hipEvent_t ev_last = nullptr;       // recorded on the last caller stream, at the end of its call
    // ev_last alternates between two events: a launch that carries an event
    // still pending from the previous call (its kernel running) waits in the
    // runtime for it -- ~7 us of host time per device-path call (profiles/r06)
    hipEvent_t ev_ring[2] = {nullptr, nullptr};
    int ev_i = 0;

    // resident placement service: the compaction shape kept on the GPU
    // between host-API placements (place_service_kernel), fed by a host-mapped
    // request word instead of a launch
    struct Service {
        bool running = false;
        hipStream_t stream = nullptr;
        hipEvent_t ev_exit = nullptr;  // recorded behind the kernel at its stop (svc_stop)
        HostBuf box;     // request: [0] (J << 32) | seq, [1] (n_runs << 32) | seq; u32 [8] ready
        HostBuf words;   // done[nb] | stats[2] | err[1] | clk[kSvcClkSlots nb]
        HostBuf assign;  // [cap]
        HostBuf bits;    // compaction: the bitmap answer, one 64-byte line per tile (ServiceArgs::bits)
        DevBuf granules; // compaction granules | bell, one 128-B line each after the granules | XCC votes
        HostBuf split;   // split shape: the tiles' feasibility slots (jsp_internal.h SplitArgs)
        HostBuf pdesc;   // the patch descriptor its dispatcher reads (kReqPatch)
        HostBuf pstage;  // inline patch staging (kReqPatchInline, jsp_internal.h), sized at snapshot upload
        uint32_t groups = 1, cpg = 1;  // split shape: class groups of its tiles
        uint32_t blocks = 0;           // row blocks the running service was started for
        uint32_t cap = 0, nb = 0, seq = 0, err_ack = 0, gen = 0;
        int shape = 0;   // 2 compaction, 3 split
        bool clk = false;
        bool rows_dirty = true;  // a patch since the last request: its tiles reload their rows from memory
        // a micro-patch since the last request: the request that carries it
        // hands its rows to the resident tiles (the dispatcher's microbox), any
        // other request reloads them (rows_dirty)
        bool micro_dirty = false;
        uint32_t pending = 0;    // a compaction request answered early: its tiles' done words still to come
        bool resume = false;  // an upload stopped it: start it again once the engine is ready
        bool pending_ready = false;  // launched; the dispatcher's ready word not seen yet
        std::chrono::steady_clock::time_point t_launch{};
        bool broken = false;  // the service cannot run on this geometry (its grid is not co-resident): the
                              // launch path answers until the next upload (every upload clears it)
        bool start_failed = false;  // the last start never saw its dispatcher poll (-> broken)
        bool armed = false;   // the host API was answered by the service: a patch (re)starts it (svc_wake)
        unsigned long long zero_key = ~0ull;  // geometry the granule / bell lines were last zeroed for
        unsigned long long layout_key = ~0ull;  // geometry the host-side slots / words were laid out for
        unsigned long long occ_key = ~0ull;   // (shape, LDS, grid) whose co-residency was last checked
        int occ_fit = 0;
        std::chrono::steady_clock::time_point last{};
        std::chrono::steady_clock::time_point first_seen{};  // the current request's first answer entry (svc_wait_entries)
        bool bitmap = false;  // compaction answers with tile bitmaps (ServiceArgs::bits)
    } svc;
    int svc_mode = JSP_SERVICE_AUTO;
    Grave grave;  // buffers replaced while the service ran: freed when it stops

    // metrics (jsp_engine_get_metrics): their own lock, so that reading them
    // never waits for a placement; taken after mu where both are held
    std::mutex met_mu;
    jsp_metrics met{};

    // timing
    bool timing = false;
    std::vector<EvPair> tev;  // jsp_*_device_timed: one start/stop pair per step
    DevBuf tmp_scrub;         // the scrub kernel's sink word
    std::vector<EvPair> ev;
    size_t ev_used = 0;
    jsp_timing acc{};

    ~jsp_engine() {
        if (waker.joinable()) {  // jsp_engine_destroy joins it; any other delete too
            {
                std::lock_guard<std::mutex> l(wake_mu);
                wake_quit.store(true);
            }
            wake_cv.notify_one();
            waker.join();
        }
        if (multi) jspm::destroy(multi);
        (void)hipSetDevice(device);
        for (auto* v : {&ev, &tev})
            for (auto& p : *v) {
                if (p.a) (void)hipEventDestroy(p.a);
                if (p.b) (void)hipEventDestroy(p.b);
            }
        if (ev_switch) (void)hipEventDestroy(ev_switch);
        for (auto& w : hw_stage)
            if (w.ev) (void)hipEventDestroy(w.ev);
        for (hipEvent_t x : ev_ring)
            if (x) (void)hipEventDestroy(x);
        if (stream) (void)hipStreamDestroy(stream);
        if (svc.ev_exit) (void)hipEventDestroy(svc.ev_exit);
        if (svc.stream) (void)hipStreamDestroy(svc.stream);
    }
};

namespace {

// 1024-row chunks per tally workgroup: one (hooks.block_chunks in tests).
// Measured on MI355X (cfg4, 1M rows, C=4) the tally takes 14.2 / 18.9 / 23.2 /
// 28.4 / 39.2 us at 1/2/3/4/8 chunks per workgroup -- the chunk's row/leaf
// passes, not its HBM loads, set a workgroup's time, and more, smaller-grid
// workgroups hide each other's latency better than a next-chunk prefetch does.
constexpr size_t kMaxEvents = 3 * 4096;
// Above this many tally workgroups the three-launch shape wins: the fused tail
// runs feasibility + assignment on one 256-thread workgroup.
constexpr uint32_t kFusedMaxBlocks = 256;

// Make stream s wait for everything the engine enqueued before (on any
// stream): the engine stream's work through an event recorded on it now, a
// caller stream's through ev_last, recorded at the end of the call that used
// it (that stream itself is never touched again: it may be gone). ev_last
// rides on the call's kernel launches as their stop event
// (jsp::set_launch_stop), so it completes with the last kernel and no marker
// packet follows it; a call that launched nothing records it. Its release is
// device scope: ordering a later stream after the device call needs no more.
int wait_prior(jsp_engine* e, hipStream_t s) {
    if (!e->have_last) return JSP_OK;
    if (e->last_foreign) {
        HIP_TRY(hipStreamWaitEvent(s, e->ev_last, 0));
    } else {
        if (!e->ev_switch) HIP_TRY(hipEventCreateWithFlags(&e->ev_switch, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(e->ev_switch, e->stream));
        HIP_TRY(hipStreamWaitEvent(s, e->ev_switch, 0));
    }
    return JSP_OK;
}

// Order work on stream s after everything the engine enqueued before on
// another stream (uploads and jsp_place use the engine stream, the device
// entry points the caller's). Calls on one stream cost nothing here.
int patch_fence(jsp_engine* e);
int enter_stream(jsp_engine* e, hipStream_t s) {
    // a patch the service applies is not stream-ordered: wait for its word
    if (int rc = patch_fence(e)) return rc;
    if (e->have_last && e->last_stream != s)
        if (int rc = wait_prior(e, s)) return rc;
    if (s != e->stream) jsp::set_launch_stop(e->ev_ring[e->ev_i ^ 1]);  // this call's end (ev_last after it)
    return JSP_OK;
}

// After a call enqueued its work on s: a caller's stream gets ev_last
// recorded on it (when no launch carried it) while the handle is known to be
// valid.
int leave_stream(jsp_engine* e, hipStream_t s) {
    const bool launched = jsp::launch_stop_used();
    jsp::set_launch_stop(nullptr);
    e->last_stream = s;
    e->have_last = true;
    e->last_foreign = s != e->stream;
    e->foreign_pending = e->last_foreign;
    if (e->last_foreign) {
        e->ev_i ^= 1;
        e->ev_last = e->ev_ring[e->ev_i];
        if (!launched) HIP_TRY(hipEventRecord(e->ev_last, s));
    }
    return JSP_OK;
}

// Host wait for the last caller-stream call's work.
int wait_last_foreign(jsp_engine* e) {
    HIP_TRY(hipEventSynchronize(e->ev_last));
    return JSP_OK;
}

// Entry of a call that enqueues on the engine's own stream: ordered after
// earlier caller-stream work, and later calls order after it by an event on
// the engine stream (no HIP call needed at its end).
int use_engine_stream(jsp_engine* e) {
    if (int rc = enter_stream(e, e->stream)) return rc;
    return leave_stream(e, e->stream);
}

// Non-blocking: a launch whose bounded wait timed out has written its tag to
// the host-mapped error word (jsp_internal.h kErr*: the kind in the top two
// bits). Reported once, by the next call.
int check_launch_error(jsp_engine* e) {
    const uint32_t w = __atomic_load_n(e->h_err.as<uint32_t>(), __ATOMIC_ACQUIRE);
    if (w != e->err_ack) {
        e->err_ack = w;
        const uint32_t kind = w & jsp::kErrKindMask, n = w & ~jsp::kErrKindMask;
        if (kind == jsp::kErrExpand)
            return set_err(JSP_EHIP, "placement launch %u failed: the level walk's expanders timed out waiting for "
                                     "the walker's records; that launch's assign[] is invalid", n);
        if (kind == jsp::kErrPipe)
            return set_err(JSP_EHIP, "placement launch %u failed: the pipelined batch walk timed out waiting for an "
                                     "earlier batch; that launch's assign[] is invalid", n);
        if (kind == jsp::kErrCopyWait)
            return set_err(JSP_EHIP, "placement launch %u failed: its assign[] copy timed out waiting for the host "
                                     "walk; that launch's assign[] is invalid", n);
        return set_err(JSP_EHIP, "placement launch %u failed: the compaction look-back timed out (a workgroup "
                                 "never published its count); that launch's assign[] is invalid", n);
    }
    return JSP_OK;
}

// The next error tag of a launch that may time out in a bounded wait (never
// 0 in the low 30 bits, so it always differs from an acknowledged word).
uint32_t next_err_tag(jsp_engine* e, uint32_t kind) {
    e->err_tag = e->err_tag % 0x3FFFFFFFu + 1u;
    return kind | e->err_tag;
}

// A wait's occasional HIP status query (has the stream finished, or failed?):
// at most once per 20 us. A query is a runtime call whose code and data a
// cold host core must first fetch, and the waits it guards mostly end within
// a few microseconds.
struct QueryPacer {
    std::chrono::steady_clock::time_point next = std::chrono::steady_clock::now() + std::chrono::microseconds(20);
    bool due() {
        const auto t = std::chrono::steady_clock::now();
        if (t < next) return false;
        next = t + std::chrono::microseconds(20);
        return true;
    }
};

// Host placement path: wait for the kernel's completion words (one per
// signalling workgroup) instead of the kernel-end signal. A finished stream
// whose words are missing, or a failed stream, is an error.
int wait_done(jsp_engine* e, hipStream_t s, uint32_t n, uint32_t epoch) {
    const uint32_t* words = e->h_done.as<uint32_t>();
    uint32_t i = 0;
    QueryPacer qp;
    for (uint64_t spins = 1;; ++spins) {
        while (i < n && __atomic_load_n(words + i, __ATOMIC_ACQUIRE) == epoch) ++i;
        if (i == n) return JSP_OK;
        if ((spins & 255) == 0 && qp.due()) {
            const hipError_t q = hipStreamQuery(s);
            if (q == hipSuccess) {
                for (; i < n; ++i)
                    if (__atomic_load_n(words + i, __ATOMIC_ACQUIRE) != epoch)
                        return set_err(JSP_EHIP, "placement kernel ended without completion word %u", i);
                return JSP_OK;
            }
            if (q != hipErrorNotReady) return set_err(JSP_EHIP, "placement kernel failed: %s", hipGetErrorString(q));
        }
    }
}

int resolve_timing(jsp_engine* e) {
    if (e->ev_used == 0) return JSP_OK;
    HIP_TRY(hipEventSynchronize(e->ev[e->ev_used - 1].b));
    for (size_t i = 0; i < e->ev_used; ++i) {
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, e->ev[i].a, e->ev[i].b));
        if (e->ev[i].tag == 0) e->acc.tally_ms += ms;
        else if (e->ev[i].tag == 1) e->acc.feas_ms += ms;
        else if (e->ev[i].tag == 2) e->acc.assign_ms += ms;
        else {
            e->acc.fused_ms += ms;
            std::lock_guard<std::mutex> l(e->met_mu);
            hist_add(e->met.device_us, ms * 1e3, JSP_HIST_LO_US);
        }
    }
    e->ev_used = 0;
    return JSP_OK;
}

// Returns the pair to bracket a launch with (nullptr when timing is off).
EvPair* ev_begin(jsp_engine* e, int tag, hipStream_t s) {
    if (!e->timing) return nullptr;
    if (e->ev_used == kMaxEvents && resolve_timing(e) != JSP_OK) return nullptr;
    if (e->ev_used == e->ev.size()) {
        EvPair p;
        if (hipEventCreate(&p.a) != hipSuccess || hipEventCreate(&p.b) != hipSuccess) return nullptr;
        e->ev.push_back(p);
    }
    EvPair* p = &e->ev[e->ev_used++];
    p->tag = tag;
    if (tag == 0 || tag == 3) e->acc.calls += 1;
    if (tag == 3) e->acc.fused_calls += 1;
    (void)hipEventRecord(p->a, s);
    return p;
}

void ev_end(EvPair* p, hipStream_t s) {
    if (p) (void)hipEventRecord(p->b, s);
}

// The caller's stream is used as given: NULL is the HIP null stream (what
// torch's default stream is), jsp_engine_stream(e) the engine's own.
hipStream_t pick(jsp_engine*, void* s) { return static_cast<hipStream_t>(s); }

int check_engine(jsp_engine* e) {
    if (!e) return set_err(JSP_EINVAL, "engine is NULL");
    if (hipSetDevice(e->device) != hipSuccess) return set_err(JSP_EHIP, "hipSetDevice(%d) failed", e->device);
    return JSP_OK;
}

// Where a buffer that must grow now leaves its old allocation: the grave
// while the resident service runs (freed when it stops), else nowhere.
Grave* grave(jsp_engine* e) { return e->svc.running ? &e->grave : nullptr; }

template <class T>
hipError_t upload(DevBuf& b, const T* src, size_t n, hipStream_t s, Grave* g = nullptr) {
    hipError_t err = b.reserve(n * sizeof(T), g);
    if (err != hipSuccess || n == 0) return err;
    return hipMemcpyAsync(b.p, src, n * sizeof(T), hipMemcpyHostToDevice, s);
}

jsp::TallyArgs tally_args(jsp_engine* e, uint32_t* d_cap, uint32_t* d_occ, uint32_t ld) {
    jsp::TallyArgs a{};
    a.labels = e->labels.as<uint64_t>();
    a.taints = e->taints.as<uint32_t>();
    a.freer = e->freer.as<uint32_t>();
    a.excl = e->excl.as<int32_t>();
    a.npad = e->npad;
    a.leaf_start = e->leaf_start.as<uint32_t>();
    a.blk = e->blk.as<uint4>();
    a.n_blocks = e->n_blocks;
    a.la = e->blk_leaves;
    a.cls = e->cls.as<jsp::DevClass>();
    a.cap_out = d_cap;
    a.occ_out = d_occ;
    a.ld = ld;
    a.leaf_base = e->leaf_begin;
    a.W = (int)e->W;
    a.R = (int)e->R;
    a.c0 = 0;
    a.nc = std::min<uint32_t>(e->C, jsp::kTallyClasses);
    a.do_occ = 1;
    return a;
}

// Workgroups of the wave-tile tally: 4 waves per SIMD (best warm and cold of
// 1-8 on cfg4, profiles/r03) over the CUs, never more than the tiles need and
// never fewer than 64 tiles per wave allow.
uint32_t tally_wave_grid(jsp_engine* e) {
    // one tile per wave (grid 0: the one-set kernel) while every tile fits
    // 6 waves per SIMD; beyond that the double-buffered kernel
    if (e->hooks.tally_one && e->n_wtiles <= (uint32_t)std::max(e->n_cu, 1) * 4u * 6u) return 0;
    constexpr uint32_t wps = 4;
    // at least n_wtiles / 64 waves: a wave holds at most 64 tile descriptors
    const uint32_t waves = std::max<uint32_t>(std::min<uint32_t>(e->n_wtiles, (uint32_t)std::max(e->n_cu, 1) * 4u * wps),
                                              (e->n_wtiles + 63) / 64);
    return std::max<uint32_t>(1, (waves + jsp::kTallyWaves - 1) / jsp::kTallyWaves);
}

// Whether the wave tally can fold the feasibility words into itself (the
// three-launch shape on the engine's own unsharded tallies): at most 4
// classes (one wave pass), all at the leaf level, wave tiles available.
bool fold_ok(jsp_engine* e, bool shard = false) {
    if (e->C < 1 || e->C > 4 || e->n_wtiles == 0 || e->hooks.tally_block) return false;
    if (!shard && (e->leaf_begin != 0 || e->n_leaves != e->L_total)) return false;
    for (const auto& c : e->cls_h)
        if (c.level + 1 != e->K) return false;
    return (uint64_t)(e->C + 1) * e->L_total * 4 < (1ull << 31);
}

// The tally alone (three-launch shape, jsp_tally_device): the wave-tile
// kernel when every leaf fits a wave tile, else the workgroup-block kernel.
// fold_feas (null: none): the wave tally sets the leaf classes' feasibility
// words there (fold_ok's shape; a shard of a device set folds into the words
// of the set's assigning engine)
int tally_impl(jsp_engine* e, uint32_t* d_cap, uint32_t* d_occ, uint32_t ld, hipStream_t s,
               uint64_t* fold_feas = nullptr) {
    jsp::TallyArgs a = tally_args(e, d_cap, d_occ, ld);
    if (fold_feas) {
        a.feas_fold = fold_feas;
        a.fold_nw = (e->L_total + 63) / 64;
    }
    if (e->n_blocks == 0) return JSP_OK;
    const bool block = e->hooks.tally_block;
    EvPair* p = ev_begin(e, 0, s);
    uint32_t c0 = 0;
    do {
        a.c0 = c0;
        a.nc = std::min<uint32_t>(e->C - c0, jsp::kTallyClasses);
        a.do_occ = (c0 == 0);
        // the wave-tile kernel takes 1-4 classes with the occupancy count in one pass
        const bool wave = !block && e->n_wtiles > 0 && a.do_occ && a.nc >= 1 && a.nc <= 4 &&
                          (uint64_t)(e->C + 1) * ld * 4 < (1ull << 31);
        if (!wave) HIP_TRY(jsp::launch_tally(a, s));
        else HIP_TRY(jsp::launch_tally_wave(a, e->wtiles.as<uint4>(), e->n_wtiles, e->n_leaves, tally_wave_grid(e), s));
        c0 += a.nc;
    } while (c0 < e->C);
    ev_end(p, s);
    return JSP_OK;
}

uint32_t* stats_ptr(jsp_engine* e) { return e->stats_override ? e->stats_override : e->stats.as<uint32_t>(); }

// The level walker's shape: every class at one level of <= kLevelMaxWords
// words, <= kLevelMaxRuns runs.
bool level_walk_ok(jsp_engine* e, uint32_t n_runs) {
    if (e->C < 1 || n_runs > jsp::kLevelMaxRuns) return false;
    const uint32_t lvl = e->cls_h[0].level;
    for (const auto& c : e->cls_h)
        if (c.level != lvl) return false;
    const uint32_t nw = (e->D[lvl] + 63) / 64;
    return nw >= 1 && nw <= jsp::kLevelMaxWords && jsp::level_walk_lds_bytes(e->C, nw) <= 128u * 1024u;
}

// The walk on the host (ABI v7) for every shape the level walker does not
// take -- several levels, or many runs -- up to kHostWalkMaxJobs jobs: there
// the GPU walk is one wave's dependent scalar chain at ~100 shader cycles per
// job visit (cfg5: 49.6 us, SQ_WAIT_ANY 82 % of its wave cycles, DESIGN.md
// §4.2), while the host walks the same bitmaps in ~2.5 us (jsp_walk.cc, the
// split service's walk; SURVEY.md §7 step 5 allows the sequential part of A7
// on the host). The GPU computes the feasibility words; the host reads them,
// walks, and writes assign[].
constexpr uint32_t kHostWalkMaxJobs = 1u << 16;
// Below this many jobs the GPU walk (~40 ns per job visit) costs less than the
// host round trip of the walk on the host (~15 us: the answer out, the copy
// of assign[] back): cfg3's 64 jobs take 16.6 us on the fused launch against
// 26.8 us walked on the host; cfg5's 500 take 49.6 against 30.5 (profiles/r06).
constexpr uint32_t kHostWalkMinJobs = 256;

// (JSP_FUSED_OFF keeps every walk on the GPU: the three-launch shape, which
// the tests use to exercise the GPU walkers on the shapes AUTO walks here)
bool host_walk_ok(jsp_engine* e, uint32_t n_runs, uint32_t J) {
    return e->fused_mode == JSP_FUSED_AUTO && e->C >= 1 && n_runs > 0 && J >= kHostWalkMinJobs &&
           J <= kHostWalkMaxJobs && !level_walk_ok(e, n_runs);
}

// The next staging slot of the device paths' walks, `bytes` large: its last
// copy has long finished by the time the ring comes round (a wait only then).
int walk_stage(jsp_engine* e, size_t bytes, jsp_engine::WalkStage** out) {
    jsp_engine::WalkStage& w = e->hw_stage[e->hw_next];
    if (w.pending) {
        HIP_TRY(hipEventSynchronize(w.ev));
        w.pending = false;
    }
    if (!w.ev) HIP_TRY(hipEventCreateWithFlags(&w.ev, hipEventDisableTiming));
    HIP_TRY(w.io.reserve(bytes + 64, grave(e)));  // + the host's release word of the copy (copy_wait_kernel)
    *out = &w;
    return JSP_OK;
}

// The assign[] copy of a device-path walk, launched before the host walks:
// it waits for the host's release of the slot's flag (walk_release), so the
// copy needs no launch after the walk. Carries the call's stop event.
int walk_copy_launch(jsp_engine* e, jsp_engine::WalkStage* w, size_t flag_off, const int32_t* staged, int32_t* d_assign,
                     uint32_t J, hipStream_t s, uint32_t* tag) {
    uint32_t* flag = reinterpret_cast<uint32_t*>(static_cast<char*>(w->io.p) + flag_off);
    e->hw_tag = e->hw_tag % 0x7FFFFFFFu + 1u;
    *tag = e->hw_tag;
    __atomic_store_n(flag, 0u, __ATOMIC_RELEASE);
    HIP_TRY(jsp::launch_copy_wait(flag, *tag, reinterpret_cast<const uint32_t*>(staged),
                                  reinterpret_cast<uint32_t*>(d_assign), J, e->h_err.as<uint32_t>(),
                                  next_err_tag(e, jsp::kErrCopyWait), e->hooks.wait_ticks, s));
    return JSP_OK;
}

// The host's side of walk_copy_launch: the walk's assign[] is in the staging
// (ok), or the call fails and nothing is copied (!ok).
void walk_release(jsp_engine::WalkStage* w, size_t flag_off, uint32_t tag, bool ok) {
    uint32_t* flag = reinterpret_cast<uint32_t*>(static_cast<char*>(w->io.p) + flag_off);
    __atomic_store_n(flag, ok ? tag : (tag | 0x80000000u), __ATOMIC_RELEASE);
}

// After the assign[] copy out of slot w was launched on stream s.
int walk_stage_done(jsp_engine* e, jsp_engine::WalkStage* w, hipStream_t s) {
    HIP_TRY(hipEventRecord(w->ev, s));
    w->pending = true;
    e->hw_next = (e->hw_next + 1) % jsp_engine::kWalkStages;
    return JSP_OK;
}

// Feasibility (feas_kernel into pinned memory, or the folded words copied
// there), the run list staged when it is device-resident, one wait, the walk,
// and assign[] copied back when it is device-resident. host_io: run_class,
// run_len and d_assign are pinned host memory (the host API's staging) -- no
// copies, the walk writes assign[] in place and the stats too. The call's
// stop event (a caller stream's end-of-call marker) rides on its last launch,
// the assign[] copy.
int host_walk_impl(jsp_engine* e, const uint32_t* d_cap, const uint32_t* d_occ, uint32_t ld,
                   const uint32_t* run_class, const uint32_t* run_len, uint32_t n_runs, uint32_t J, int32_t* assign,
                   hipStream_t s, bool folded, bool host_io) {
    const uint32_t fw = std::max<uint32_t>(e->feas_words, 1);
    HIP_TRY(e->hw_feas.reserve((size_t)fw * 8 + 64, grave(e)));  // + the tag word
    jsp_engine::WalkStage* st = nullptr;
    if (!host_io)
        if (int rc = walk_stage(e, (size_t)n_runs * 8 + (size_t)J * 4, &st)) return rc;
    uint32_t* hrc = host_io ? const_cast<uint32_t*>(run_class) : st->io.as<uint32_t>();
    uint32_t* hrl = host_io ? const_cast<uint32_t*>(run_len) : hrc + n_runs;
    int32_t* out = host_io ? assign : reinterpret_cast<int32_t*>(hrc + 2 * (size_t)n_runs);
    // a caller stream's end-of-call event rides on the last launch only (each
    // launch that carries one costs its dispatch an event write)
    const hipEvent_t stop = jsp::take_launch_stop();
    EvPair* p = ev_begin(e, 1, s);
    if (folded)
        HIP_TRY(jsp::launch_copy_u32(e->feas.as<uint32_t>(), e->hw_feas.as<uint32_t>(), 2 * e->feas_words, s));
    else
        HIP_TRY(jsp::launch_feas(d_cap, d_occ, ld, e->cls.as<jsp::DevClass>(), e->C, e->word_off.as<uint32_t>(),
                                 e->feas_words, e->topo, e->hw_feas.as<uint64_t>(), s));
    ev_end(p, s);
    if (!host_io) {
        HIP_TRY(jsp::launch_copy_u32(run_class, hrc, n_runs, s));
        HIP_TRY(jsp::launch_copy_u32(run_len, hrl, n_runs, s));
    }
    // a tag written behind them on the stream tells the host they are done
    // (an event's completion reaches the host microseconds later)
    uint32_t* tag = e->hw_feas.as<uint32_t>() + 2 * (size_t)fw;
    e->hw_tag = e->hw_tag % 0x7FFFFFFFu + 1u;
    const uint32_t want = e->hw_tag;
    HIP_TRY(jsp::launch_tag(tag, want, s));
    // the assign[] copy is queued now (it waits for the walk's release): no
    // launch between the walk and the copy
    const size_t flag_off = (size_t)n_runs * 8 + (size_t)J * 4;
    uint32_t ctag = 0;
    if (!host_io) {
        jsp::set_launch_stop(stop);
        if (int rc = walk_copy_launch(e, st, flag_off, out, assign, J, s, &ctag)) return rc;
        if (int rc = walk_stage_done(e, st, s)) {
            walk_release(st, flag_off, ctag, false);
            return rc;
        }
    }
    e->walk.prefetch_state();  // while the device works
    {
        const auto t0 = std::chrono::steady_clock::now();
        QueryPacer qp;
        int rc = JSP_OK;
        for (uint64_t spins = 1; __atomic_load_n(tag, __ATOMIC_ACQUIRE) != want; ++spins) {
            if ((spins & 255) == 0 && qp.due()) {
                const hipError_t q = hipStreamQuery(s);
                if (q == hipSuccess && __atomic_load_n(tag, __ATOMIC_ACQUIRE) == want) break;
                if (q == hipSuccess) rc = set_err(JSP_EHIP, "host walk: the feasibility ended without its tag");
                else if (q != hipErrorNotReady) rc = set_err(JSP_EHIP, "host walk: feasibility failed: %s", hipGetErrorString(q));
                else if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10))
                    rc = set_err(JSP_EHIP, "host walk: the device feasibility did not complete within 10 s");
                if (rc) break;
            }
            _mm_pause();
        }
        if (rc) {
            if (!host_io) walk_release(st, flag_off, ctag, false);
            return rc;
        }
    }
    p = ev_begin(e, 2, s);
    const uint32_t placed = e->walk.walk(e->hw_feas.as<uint64_t>(), hrc, hrl, n_runs, out);
    if (e->stats_override) {  // the host API reads them (pinned)
        e->stats_override[0] = n_runs;
        e->stats_override[1] = placed;
    }
    if (!host_io) walk_release(st, flag_off, ctag, true);
    else jsp::set_launch_stop(stop);
    ev_end(p, s);
    return JSP_OK;
}

int assign_impl(jsp_engine* e, const uint32_t* d_cap, const uint32_t* d_occ, uint32_t ld,
                const uint32_t* d_run_class, const uint32_t* d_run_len, uint32_t n_runs, uint32_t J,
                int32_t* d_assign, hipStream_t s, bool folded = false, bool host_io = false) {
    if (host_walk_ok(e, n_runs, J))
        return host_walk_impl(e, d_cap, d_occ, ld, d_run_class, d_run_len, n_runs, J, d_assign, s, folded, host_io);
    EvPair* p = ev_begin(e, 1, s);
    if (!folded)
        HIP_TRY(jsp::launch_feas(d_cap, d_occ, ld, e->cls.as<jsp::DevClass>(), e->C, e->word_off.as<uint32_t>(),
                                 e->feas_words, e->topo, e->feas.as<uint64_t>(), s));
    ev_end(p, s);
    p = ev_begin(e, 2, s);
    if (e->recs.reserve(sizeof(jsp::AssignRec) * (size_t)std::max<uint32_t>(J, 1), grave(e)) != hipSuccess)
        return set_err(JSP_ENOMEM, "assignment records (%u jobs)", J);
    jsp::WaitErr we{e->h_err.as<uint32_t>(), 0u, e->hooks.pipe_spins, e->hooks.wait_ticks};
    if (level_walk_ok(e, n_runs)) {
        // the expansion rides in the walker's launch: its expanders wait
        // (bounded) for the walker's record count, and one that gives up
        // writes the launch's tag to the error word (kErrExpand)
        const uint32_t nw = (e->D[e->cls_h[0].level] + 63) / 64;
        if (!e->lvl_ready.p) {
            HIP_TRY(e->lvl_ready.reserve(64));
            HIP_TRY(hipMemsetAsync(e->lvl_ready.p, 0, 64, s));
        }
        e->lvl_epoch = e->lvl_epoch % 0x7FFFFFFFu + 1u;
        we.tag = next_err_tag(e, jsp::kErrExpand);
        HIP_TRY(jsp::launch_assign_level(e->feas.as<uint64_t>(), e->C, nw, d_run_class, d_run_len, n_runs, J, d_assign,
                                         stats_ptr(e), e->stats.as<uint32_t>() + 3, e->recs.as<jsp::AssignRec>(), s,
                                         e->lvl_ready.as<unsigned long long>(), e->lvl_epoch, we));
        ev_end(p, s);
        return JSP_OK;
    }
    we.tag = next_err_tag(e, jsp::kErrPipe);
    HIP_TRY(jsp::launch_assign(e->feas.as<uint64_t>(), e->word_off.as<uint32_t>(), e->cls.as<jsp::DevClass>(),
                               e->C, e->topo, e->t_off_h[e->K], e->feas_words, d_run_class, d_run_len, n_runs, J,
                               d_assign, stats_ptr(e), e->stats.as<uint32_t>() + 3, e->recs.as<jsp::AssignRec>(), s,
                               we));
    ev_end(p, s);
    return JSP_OK;
}

bool fused_ok(jsp_engine* e) {
    return e->fused_mode == JSP_FUSED_AUTO && e->n_blocks > 0 && e->n_blocks <= kFusedMaxBlocks &&
           e->C <= (uint32_t)jsp::kTallyClasses &&
           e->leaf_begin == 0 && e->n_leaves == e->L_total &&
           e->t_off_h[e->K] + e->feas_words <= jsp::kFusedMaxWords;
}

// One class at the leaf level: job j takes the j-th feasible leaf (any size).
bool compact_ok(jsp_engine* e) {
    return e->fused_mode == JSP_FUSED_AUTO && e->n_blocks > 0 && e->C == 1 && e->cls_h[0].level + 1 == e->K &&
           e->leaf_begin == 0 && e->n_leaves == e->L_total;
}

// Launch arguments of the fused shape (the launch path and the resident
// service); sets a.sc1_out, the tallies' write-through hand-off to the tail.
jsp::FusedArgs fused_args(jsp_engine* e, jsp::TallyArgs& a, const uint32_t* d_run_class, const uint32_t* d_run_len,
                          uint32_t n_runs, uint32_t J, int32_t* d_assign, uint32_t* stats) {
    jsp::FusedArgs f{};
    f.ticket = e->ticket.as<unsigned long long>();
    f.tile_base = e->tile_draws;
    f.done_base = e->done_draws;
    f.C = e->C;
    f.topo = e->topo;
    f.t_off = e->t_off.as<uint32_t>();
    f.t_words = e->t_off_h[e->K];
    f.word_off = e->word_off.as<uint32_t>();
    f.feas_words = e->feas_words;
    f.run_class = d_run_class;
    f.run_len = d_run_len;
    f.n_runs = n_runs;
    f.J = J;
    f.assign = d_assign;
    f.stats = stats;
    const uint32_t topo_words = e->K > 1 ? jsp::topo_table_words(e->K, e->topo.D) : 0u;
    f.topo_in_lds = topo_words > 0 && topo_words <= jsp::kFusedTopoMax ? 1u : 0u;
    f.topo_lds_words = f.topo_in_lds ? topo_words : 0u;
    {
        uint32_t lv[jsp::kMaxClasses];
        for (uint32_t c = 0; c < e->C; ++c) lv[c] = e->cls_h[c].level;
        f.fscr_words = jsp::fused_scratch_words(e->K, e->topo.D, lv, e->C);
        bool upper = false;
        for (uint32_t c = 0; c < e->C; ++c) upper |= lv[c] + 1 < e->K;
        // write-through hand-off of the tallies to the tail (no release/acquire
        // fences) unless the tail's per-wave upper-class path, which reads them
        // with plain loads, will run
        a.sc1_out = !upper || f.fscr_words != 0 ? 1 : 0;
    }
    // class groups: a small snapshot's tiles are VALU-bound over many classes;
    // splitting the classes over up to 4 groups of >= 2 multiplies the tiles
    // (each row block read once per group), within 128 tiles
    f.groups = 1;
    if (e->C > 2) {
        const uint32_t by_c = std::min<uint32_t>(4, (e->C + 1) / 2);
        const uint32_t by_t = std::max<uint32_t>(1, 128 / std::max<uint32_t>(e->n_blocks, 1));
        f.groups = std::max<uint32_t>(1, std::min(by_c, by_t));
    }
    f.cpg = (a.nc + f.groups - 1) / f.groups;
    f.we = jsp::WaitErr{e->h_err.as<uint32_t>(), next_err_tag(e, jsp::kErrPipe), e->hooks.pipe_spins,
                        e->hooks.wait_ticks};
    f.lds_bytes = jsp::fused_lds_bytes(f.t_words, f.feas_words, f.cpg, f.cpg + a.do_occ, a.la,
                                       f.topo_in_lds ? topo_words : 0u, f.fscr_words);
    return f;
}

bool split_ok(jsp_engine* e);
uint32_t split_groups(jsp_engine* e);
uint32_t next_seq(uint32_t q);

// The split shape launched for one request (ABI v7, shape 8): the resident
// split service's tiles (tally, per-leaf feasibility ballots, upper-domain
// partial sums, tagged lines into pinned memory) as one launch of tiles only
// -- no dispatcher, no residency -- and the host walk over their lines, as
// the service's answer is walked. The launch path and the device paths of
// every multi-class / multi-level shape the split service takes, up to
// kHostWalkMaxJobs jobs. host_io: the run list and assign[] are pinned host
// memory (the host API's staging); otherwise they are device buffers, staged
// through pinned memory by copy launches on the same stream.
bool split_oneshot_ok(jsp_engine* e, uint32_t n_runs, uint32_t J) {
    return e->fused_mode == JSP_FUSED_AUTO && n_runs > 0 && J >= kHostWalkMinJobs && J <= kHostWalkMaxJobs &&
           split_ok(e);
}

int split_oneshot(jsp_engine* e, const uint32_t* run_class, const uint32_t* run_len, uint32_t n_runs, uint32_t J,
                  int32_t* assign, hipStream_t s, bool host_io) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    const uint32_t g = split_groups(e), cpg = (e->C + g - 1) / g, nb = e->n_blocks, n_tiles = nb * g;
    const uint32_t nw = jsp::split_waves(e->blk_l0, e->blk_l1);
    const size_t sb = (size_t)n_tiles * jsp::split_tile_words(cpg, nw) * 8;
    if (sb > e->os_split.bytes || !e->os_split.p) {
        HIP_TRY(e->os_split.reserve(sb, grave(e)));
        std::memset(e->os_split.p, 0, e->os_split.bytes);  // tags: request 0 is never posted
    }
    const unsigned long long key = ((unsigned long long)nb << 40) | ((unsigned long long)g << 32) | cpg;
    if (e->os_key != key) {
        e->walk.set_tiles(e->blk_l0, e->blk_l1, g, cpg);
        e->os_key = key;
        e->svc.layout_key = ~0ull;  // the service re-lays its own slots (and the walk's tiles) at its next start
    }
    jsp_engine::WalkStage* st = nullptr;
    if (!host_io)
        if (int rc = walk_stage(e, (size_t)n_runs * 8 + (size_t)J * 4, &st)) return rc;
    uint32_t* hrc = host_io ? const_cast<uint32_t*>(run_class) : st->io.as<uint32_t>();
    uint32_t* hrl = host_io ? const_cast<uint32_t*>(run_len) : hrc + n_runs;
    int32_t* out = host_io ? assign : reinterpret_cast<int32_t*>(hrc + 2 * (size_t)n_runs);
    e->os_seq = next_seq(e->os_seq);
    const uint32_t seq = e->os_seq;
    const jsp::TallyArgs ta = tally_args(e, nullptr, nullptr, e->L_total);
    jsp::SplitArgs sp{};
    sp.groups = g;
    sp.cpg = cpg;
    sp.nw = nw;
    sp.C = e->C;
    sp.out = e->os_split.as<uint64_t>();
    sp.topo = e->topo;
    if (!host_io) {  // the device-resident run list comes out with tile 0's answer
        sp.run_class = run_class;
        sp.run_len = run_len;
        sp.run_dst = hrc;
        sp.n_runs = n_runs;
    }
    jsp::ServiceArgs a{};
    a.oneshot = seq;
    a.anc_words = jsp::split_anc_words(cpg, e->blk_leaves, (int)e->W, (int)e->R, false);
    // the assign[] copy rides in the same launch: one extra workgroup waits
    // for the walk's release and copies (no launch between walk and copy)
    const size_t flag_off = (size_t)n_runs * 8 + (size_t)J * 4;
    uint32_t ctag = 0;
    if (!host_io) {
        uint32_t* flag = reinterpret_cast<uint32_t*>(static_cast<char*>(st->io.p) + flag_off);
        e->hw_tag = e->hw_tag % 0x7FFFFFFFu + 1u;
        ctag = e->hw_tag;
        __atomic_store_n(flag, 0u, __ATOMIC_RELEASE);
        sp.cw_flag = flag;
        sp.cw_tag = ctag;
        sp.cw_src = reinterpret_cast<const uint32_t*>(out);
        sp.cw_dst = reinterpret_cast<uint32_t*>(assign);
        sp.cw_n = J;
        sp.cw_err = e->h_err.as<uint32_t>();
        sp.cw_err_tag = next_err_tag(e, jsp::kErrCopyWait);
        sp.cw_ticks = e->hooks.wait_ticks;
    }
    EvPair* p = ev_begin(e, 3, s);
    const auto tl = clk::now();
    // one launch (the copy as a kernel of its own behind the tiles measured the
    // same: 20.9 against 21.7 us per back-to-back call, profiles/r06/g2)
    HIP_TRY(jsp::launch_split_oneshot(ta, sp, a, s));  // carries the call's stop event, if any
    e->acc.oneshot_stage_us += std::chrono::duration<double, std::micro>(tl - t0).count();
    ev_end(p, s);
    if (!host_io)
        if (int rc = walk_stage_done(e, st, s)) {
            walk_release(st, flag_off, ctag, false);
            return rc;
        }
    const auto t1 = clk::now();
    e->walk.prefetch_state();
    // every tile's tagged lines (the answer), bounded; a failed stream is an error
    const uint64_t* slots = e->os_split.as<uint64_t>();
    uint32_t t = 0;
    QueryPacer qp;
    int wrc = JSP_OK;
    for (uint64_t spins = 1; wrc == JSP_OK; ++spins) {
        while (t < n_tiles && e->walk.tile_ready(slots, t, seq)) ++t;
        if (t == n_tiles) break;
        if ((spins & 7) == 1)
            for (uint32_t u = t + 1; u < n_tiles; ++u) e->walk.prefetch_tile(slots, u);
        if ((spins & 255) == 0 && qp.due()) {
            // (the stream also holds the queued copy, which waits for this
            // walk: a query reports the split launch's failure, never success)
            const hipError_t q = hipStreamQuery(s);
            if (q == hipSuccess) {
                while (t < n_tiles && e->walk.tile_ready(slots, t, seq)) ++t;
                if (t == n_tiles) break;
                wrc = set_err(JSP_EHIP, "split launch ended without the answer of tile %u", t);
            } else if (q != hipErrorNotReady) {
                wrc = set_err(JSP_EHIP, "split launch failed: %s", hipGetErrorString(q));
            } else if (clk::now() - t1 > std::chrono::seconds(10)) {
                wrc = set_err(JSP_EHIP, "split launch: no answer within 10 s");
            }
        }
    }
    if (wrc) {
        if (!host_io) walk_release(st, flag_off, ctag, false);
        return wrc;
    }
    // (a device-resident run list came out with tile 0's lines: its stores
    // were released before them)
    const auto t2 = clk::now();
    const uint32_t placed = e->walk.place(slots, hrc, hrl, n_runs, out);
    if (e->stats_override) {
        e->stats_override[0] = n_runs;
        e->stats_override[1] = placed;
    }
    if (!host_io) walk_release(st, flag_off, ctag, true);
    // the phases (jspb_get_timing): set-up and launch, the wait for the
    // tiles' lines, the walk and the copy launch
    using us = std::chrono::duration<double, std::micro>;
    const auto t3 = clk::now();
    e->acc.oneshot_calls += 1;
    e->acc.oneshot_launch_us += us(t1 - t0).count();
    e->acc.oneshot_wait_us += us(t2 - t1).count();
    e->acc.oneshot_walk_us += us(t3 - t2).count();
    return JSP_OK;
}

// Whole placement on the engine's own tally buffers: one compaction launch for
// a single leaf-level class, one fused launch when the snapshot is small, else
// tally -> feas -> assign. `signal`: the single-launch shapes write host
// completion words (e->h_done) tagged e->epoch; *n_signals says how many.
int place_impl(jsp_engine* e, const uint32_t* d_run_class, const uint32_t* d_run_len, uint32_t n_runs, uint32_t J,
               int32_t* d_assign, hipStream_t s, bool signal = false, uint32_t* n_signals = nullptr,
               bool want_tally = false, bool host_io = false) {
    e->epoch = e->epoch % 0x3FFFFFFFu + 1u;
    if (n_signals) *n_signals = 0;
    if (compact_ok(e)) {
        e->last_shape = 2;
        // the compaction keeps its sums in LDS; they go out only when asked for
        jsp::TallyArgs a = want_tally ? tally_args(e, e->cap.as<uint32_t>(), e->occ.as<uint32_t>(), e->L_total)
                                      : tally_args(e, nullptr, nullptr, e->L_total);
        jsp::CompactArgs f{};
        f.ticket = e->ticket.as<unsigned long long>();
        f.tile_base = e->tile_draws;
        f.granules = e->granules.as<unsigned long long>();
        f.pods = e->cls_h[0].pods;
        f.n_runs = n_runs;
        f.J = J;
        f.assign = d_assign;
        f.stats = stats_ptr(e);
        f.epoch = e->epoch;
        f.err = e->h_err.as<uint32_t>();
        f.spin_limit = e->spin_limit;
        f.done = signal ? e->h_done.as<uint32_t>() : nullptr;
        if (n_signals && signal) *n_signals = e->n_blocks;
        EvPair* p = ev_begin(e, 3, s);
        HIP_TRY(jsp::launch_compact(a, f, s));
        ev_end(p, s);
        e->tile_draws += e->n_blocks + jsp::kSpareBlocks;
        return JSP_OK;
    }
    // the split tiles launched for this request, the walk on the host (shape
    // 8: no tallies wanted -- they stay in the tiles' LDS)
    if (!want_tally && split_oneshot_ok(e, n_runs, J)) {
        e->last_shape = 8;
        return split_oneshot(e, d_run_class, d_run_len, n_runs, J, d_assign, s, host_io);
    }
    // the walk on the host after the GPU's tally and feasibility (shape 7), or
    // on the GPU: one fused launch (shape 1), three launches (shape 0)
    const bool hw = host_walk_ok(e, n_runs, J);
    e->last_shape = hw ? 7 : fused_ok(e) ? 1 : 0;
    if (e->last_shape != 1) {
        const bool fold = fold_ok(e);
        if (int rc = tally_impl(e, e->cap.as<uint32_t>(), e->occ.as<uint32_t>(), e->L_total, s,
                                fold ? e->feas.as<uint64_t>() : nullptr))
            return rc;
        return assign_impl(e, e->cap.as<uint32_t>(), e->occ.as<uint32_t>(), e->L_total, d_run_class, d_run_len,
                           n_runs, J, d_assign, s, fold, host_io);
    }
    jsp::TallyArgs a = tally_args(e, e->cap.as<uint32_t>(), e->occ.as<uint32_t>(), e->L_total);
    jsp::FusedArgs f = fused_args(e, a, d_run_class, d_run_len, n_runs, J, d_assign, stats_ptr(e));
    f.done = signal ? e->h_done.as<uint32_t>() : nullptr;
    f.epoch = e->epoch;
    if (n_signals && signal) *n_signals = 1;
    EvPair* p = ev_begin(e, 3, s);
    HIP_TRY(jsp::launch_fused(a, f, s));
    ev_end(p, s);
    e->tile_draws += e->n_blocks * f.groups + jsp::kSpareBlocks;
    e->done_draws += e->n_blocks * f.groups;
    return JSP_OK;
}

// ---- resident placement service ----
// Host side of place_service_kernel. The request word is written last with one
// 64-bit store (x86 keeps store order; the kernel reads it with system-scope
// vector loads). The host answers from the done words, as for a launch.
// Idle exit: a workgroup leaves after JSP_SERVICE_IDLE_MS without a request;
// the host restarts the service when its own last request is older than half
// of that, so it never posts into an exit (and if it ever did, the dead
// service is seen by a stream query and the request re-posted once).
constexpr uint32_t kSvcMaxBlocks = 255;  // one tile per workgroup + the dispatcher, all co-resident (<= one per CU)
constexpr int kSvcGone = 1;
constexpr int kSvcFailed = 3;  // a tile reported a failed wait through the service's error word
// svc_stop's bound on the kernel's exit after the stop word (it leaves within
// ~2 us; the runtime reports it ~8 us later)
constexpr std::chrono::milliseconds kStopLimit{2000};

double svc_idle_ms() {
    static const double ms = [] {
        const char* v = std::getenv("JSP_SERVICE_IDLE_MS");
        const double x = v ? std::strtod(v, nullptr) : 50.0;
        return x >= 1.0 && x <= 5000.0 ? x : 50.0;
    }();
    return ms;
}

// The engine's idle limit: JSP_SERVICE_PARKED never idles out (a dedicated
// GPU; the service leaves on jsp_engine_service_stop, an upload or destroy).
constexpr double kParkedIdleMs = 1e15;
double idle_ms(const jsp_engine* e) { return e->svc_mode == JSP_SERVICE_PARKED ? kParkedIdleMs : svc_idle_ms(); }

// Class groups of the split service's tiles: as the fused shape's (up to 4
// groups of >= 2 classes, within 128 tiles), capped by the co-resident tile
// limit.
uint32_t split_groups(jsp_engine* e) {
    uint32_t g = 1;
    if (e->C > 2) {
        const uint32_t by_c = std::min<uint32_t>(4, (e->C + 1) / 2);
        const uint32_t by_t = std::max<uint32_t>(1, 128 / std::max<uint32_t>(e->n_blocks, 1));
        g = std::max<uint32_t>(1, std::min(by_c, by_t));
    }
    while (g > 1 && e->n_blocks * g > kSvcMaxBlocks) --g;
    return g;
}

// The split shape (tiles resident, the walk on the host): any snapshot whose
// tiles fit the service, all classes in <= 16 per group.
bool split_ok(jsp_engine* e) {
    if (e->fused_mode != JSP_FUSED_AUTO || e->n_blocks == 0 || e->leaf_begin != 0 || e->n_leaves != e->L_total)
        return false;
    const uint32_t g = split_groups(e);
    // an upper class's records carry its domain in 20 bits (jsp_internal.h SplitArgs)
    for (uint32_t c = 0; c < e->C; ++c)
        if (e->cls_h[c].level + 1 < e->K && e->D[e->cls_h[c].level] >= jsp::kSplitMaxDomains) return false;
    return e->n_blocks * g <= kSvcMaxBlocks && (e->C + g - 1) / g <= (uint32_t)jsp::kTallyClasses && e->C > 0;
}

// The shape the service would run for the engine's current state (2
// compaction, 3 split), 0 = none. The split shape answers every multi-class
// or multi-level shape the fused launch would (and more: no LDS limit on the
// walk, which runs on the host).
int svc_shape(jsp_engine* e) {
    if (e->svc_mode == JSP_SERVICE_OFF || !e->have_topo || !e->have_snap || !e->have_cls ||
        e->n_blocks > kSvcMaxBlocks || e->svc.broken)
        return 0;
    if (compact_ok(e)) return 2;
    if (split_ok(e)) return 3;
    return 0;
}
bool svc_ok(jsp_engine* e) { return svc_shape(e) != 0; }

// The request line (pinned host memory the dispatcher polls, jsp_internal.h
// kMailbox*) and, on a line of its own after it, the dispatcher's ready word.
// A request line in device memory written through the BAR was measured
// slower on every shape.
constexpr size_t kBoxBytes = jsp::kMailboxBytes + 128;
constexpr size_t kReadyWord = jsp::kMailboxBytes / 4 + 16;

// One 16-byte chunk of the request line in one store (aligned 16-byte SSE
// stores are single-copy atomic on x86-64 processors with AVX).
inline void store16(uint32_t* p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    _mm_store_si128(reinterpret_cast<__m128i*>(p), _mm_set_epi32((int)d, (int)c, (int)b, (int)a));
}

// Post request `seq`: the micro-patch payload chunks (micro: the held-back
// micro-patch rides in it), chunk 1 {seq, rows, patch number, flags}, then
// chunk 0 -- its second half first: the dispatcher reads the whole line in
// one load and takes a read whose chunks disagree on seq for none.
void svc_request(jsp_engine* e, uint32_t seq, uint32_t jw, uint32_t w2, bool micro = false) {
    uint32_t* b = e->svc.box.as<uint32_t>();
    uint32_t m = 0, fl = 0, pseq = (jw & jsp::kReqPatch) ? e->patch_seq : 0u;
    if (micro && e->micro_n > 0) {
        m = e->micro_n;
        fl = e->micro_fl;
        pseq = e->patch_seq;
        const uint32_t words = m * jsp::micro_row_words(e->W, e->R);
        for (uint32_t c = 0; 3 * c < words; ++c)
            store16(b + 4 * (2 + c), seq, e->micro_w[3 * c], e->micro_w[3 * c + 1], e->micro_w[3 * c + 2]);
    }
    store16(b + 4, seq, m, pseq, fl);
    unsigned long long* r = reinterpret_cast<unsigned long long*>(b);
    __atomic_store_n(r + 1, ((unsigned long long)w2 << 32) | seq, __ATOMIC_RELEASE);
    __atomic_store_n(r, ((unsigned long long)jw << 32) | seq, __ATOMIC_RELEASE);
}

// The stop word (every workgroup of the service leaves).
void svc_post_stop(jsp_engine* e) {
    __atomic_store_n(e->svc.box.as<unsigned long long>(), (unsigned long long)jsp::kSvcStop, __ATOMIC_RELEASE);
}

int patch_wait(jsp_engine* e);
int svc_stop(jsp_engine* e) {
    auto& v = e->svc;
    // a patch posted to the dispatcher lands first (the stop word would
    // replace its request); one held back stays so (patch_wait applies it)
    if (e->patch_pending && e->patch_svc && !e->patch_deferred)
        if (int rc = patch_wait(e)) return rc;
    v.pending = 0;  // the stop waits for the kernel to leave, i.e. for every tile to finish
    if (!v.running) return JSP_OK;
    v.running = false;
    // The kernel leaves within ~2 us of the stop word; the runtime reports it
    // complete ~7-9 us later whatever the host does (tools/stop_anatomy.hip,
    // profiles/r05/probes/stop_anatomy.txt). An event recorded behind it
    // (before the stop word: the record's own host time overlaps the exit)
    // and its synchronize report it soonest: 7.7 us from the stop word,
    // against 9.3 us polling hipStreamQuery.
    if (!v.ev_exit) HIP_TRY(hipEventCreateWithFlags(&v.ev_exit, hipEventDisableTiming));
    const hipError_t rec = hipEventRecord(v.ev_exit, v.stream);
    svc_post_stop(e);
    // Bounded: a kernel that never reads the stop word -- a wedged
    // dispatcher -- would hold a blocking synchronize forever. The event is
    // polled instead, up to kStopLimit; past it the service is marked broken
    // (the launch path answers until the next upload) and the call fails.
    hipError_t q = hipSuccess;
    if (rec == hipSuccess) {
        const auto t0 = std::chrono::steady_clock::now();
        while ((q = hipEventQuery(v.ev_exit)) == hipErrorNotReady) {
            if (std::chrono::steady_clock::now() - t0 > kStopLimit) {
                v.broken = true;
                return set_err(JSP_EHIP, "placement service did not leave within %lld ms of its stop word",
                               (long long)std::chrono::duration_cast<std::chrono::milliseconds>(kStopLimit).count());
            }
            _mm_pause();
        }
    } else {
        q = hipStreamSynchronize(v.stream);
    }
    if (q != hipSuccess) return set_err(JSP_EHIP, "placement service failed: %s", hipGetErrorString(q));
    e->grave.flush();  // nothing resident any more: a free no longer waits
    return JSP_OK;
}

// Uploads stop the service (it holds the old buffers and geometry) and start
// it again at their end when it was running, so the next jsp_place -- the
// recovery path: post-delete snapshot uploaded, then placed -- finds it ready.
int svc_suspend(jsp_engine* e) {
    // every patch lands before an upload replaces what it patched
    if (int rc = patch_wait(e)) return rc;
    e->svc.resume |= e->svc.running;
    e->svc.broken = false;  // new geometry: the service may fit again
    e->svc.zero_key = ~0ull;  // and its lines are zeroed again at the next start
    e->svc.layout_key = ~0ull;
    return svc_stop(e);
}

int svc_start(jsp_engine* e, uint32_t J, bool wait_ready);
int svc_wait_ready(jsp_engine* e);
// The upload returns once the new service polls, so the recovery's "post-delete
// snapshot uploaded -> jsp_place" finds it ready instead of waiting for its
// launch inside the placement (a failure here resurfaces at the next jsp_place).
void svc_resume(jsp_engine* e) {
    if (e->svc.resume && svc_ok(e)) {
        e->svc.resume = false;
        (void)svc_start(e, 0, true);
    }
}

void start_waker(jsp_engine* e);
void notify_waker_poll(jsp_engine* e);

int svc_start(jsp_engine* e, uint32_t J, bool wait_ready) {
    auto& v = e->svc;
    if (!v.stream) HIP_TRY(hipStreamCreateWithFlags(&v.stream, hipStreamNonBlocking));
    start_waker(e);  // created with the first service, never on a recovery's path
    const uint32_t nb = e->n_blocks;
    if (J > v.cap || !v.assign.p) {
        const uint32_t cap = std::max<uint32_t>(4096, J + J / 2);
        HIP_TRY(v.assign.reserve((size_t)cap * 8));  // compaction: u64 (seq << 32 | domain) entries
        v.cap = cap;
    }
    const int shape = svc_shape(e);
    if (shape == 0) return set_err(JSP_ESTATE, "no resident-service shape for this engine state");
    uint32_t n_tiles = nb;  // workgroups that answer (and write a done word), dispatcher excluded
    // The host-side layout (split slots, the host walk's tile table, the done
    // and stamp words) is rebuilt only when the geometry changes: every
    // request rewrites the slots the walk reads, done words are compared with
    // request numbers that never repeat, and the error word is acknowledged at
    // its current value -- so a restart after an idle exit (a recovery's cold
    // start) costs the launch alone.
    if (shape == 3) {
        v.groups = split_groups(e);
        v.cpg = (e->C + v.groups - 1) / v.groups;
        n_tiles = nb * v.groups;
    }
    const unsigned long long lkey = ((unsigned long long)nb << 40) | ((unsigned long long)v.groups << 32) |
                                    ((unsigned long long)v.cpg << 8) | (unsigned)shape;
    const size_t nw = (size_t)(1 + jsp::kSvcClkSlots) * n_tiles + 3 + jsp::kSvcClkSlots;  // + the dispatcher's clk row
    if (v.layout_key != lkey || !v.words.p || nw * 4 > v.words.bytes) {
        if (shape == 3) {
            const size_t sb = (size_t)n_tiles * jsp::split_tile_words(v.cpg, jsp::split_waves(e->blk_l0, e->blk_l1)) * 8;
            HIP_TRY(v.split.reserve(sb));
            std::memset(v.split.p, 0, sb);
            e->walk.set_tiles(e->blk_l0, e->blk_l1, v.groups, v.cpg);
        }
        HIP_TRY(v.words.reserve(nw * 4));
        std::memset(v.words.p, 0, nw * 4);  // done words: seq 0 is never posted
        if (shape == 2) {
            HIP_TRY(v.bits.reserve((size_t)64 * std::max<uint32_t>(n_tiles, 1)));
            std::memset(v.bits.p, 0, (size_t)64 * std::max<uint32_t>(n_tiles, 1));  // tags: seq 0 is never posted
        }
        v.layout_key = lkey;
    }
    HIP_TRY(v.box.reserve(kBoxBytes));
    const size_t gbytes = (size_t)8 * std::max<uint32_t>(nb, 1), gpad = (gbytes + 127) & ~size_t(127);
    // granules, then the bell on a line of its own, then the XCC votes.
    // Zeroed only when allocated or the geometry changes: granule tags and
    // request numbers never repeat across starts and a stop in the bell
    // carries its service's generation -- so a restart after an idle exit
    // (the recovery's cold start) costs the launch alone. Every write the
    // service stages from (uploads) was synchronous, and rows are fenced per
    // request (patch_wait), so the launch need not wait for the engine's
    // streams.
    const size_t xbytes = ((size_t)4 * (nb + 1) + 127) & ~size_t(127);  // XCC vote words (co-located service)
    const size_t mbytes = (size_t)8 * (1 + jsp::kMailboxPayload);       // the microbox (not zeroed: seq-tagged)
    if (gpad + 128 + xbytes + mbytes > v.granules.bytes || !v.granules.p) v.zero_key = ~0ull;
    HIP_TRY(v.granules.reserve(gpad + 128 + xbytes + mbytes));
    const unsigned long long key = ((unsigned long long)nb << 8) | ((unsigned long long)n_tiles << 40) | (unsigned)shape;
    if (v.zero_key != key) {
        HIP_TRY(hipMemsetAsync(v.granules.p, 0, gpad + 128, v.stream));
        v.zero_key = key;
    }
    svc_request(e, v.seq, 0u, 0u);  // already answered: the new dispatcher starts after it
    v.gen = v.gen % 0x7FFFFFFFu + 1u;
    uint32_t* ready = v.box.as<uint32_t>() + kReadyWord;
    __atomic_store_n(ready, 0u, __ATOMIC_RELEASE);
    uint32_t* w = v.words.as<uint32_t>();
    jsp::ServiceArgs a{};
    a.mailbox = v.box.as<unsigned long long>();
    a.granules = v.granules.as<unsigned long long>();
    a.bell = reinterpret_cast<unsigned long long*>(static_cast<char*>(v.granules.p) + gpad);
    a.xcc = reinterpret_cast<uint32_t*>(static_cast<char*>(v.granules.p) + gpad + 128);
    if (!v.pdesc.p) HIP_TRY(v.pdesc.reserve(sizeof(jsp::PatchDesc)));
    if (!e->h_patch_done.p) {
        HIP_TRY(e->h_patch_done.reserve(128));
        std::memset(e->h_patch_done.p, 0, 128);
    }
    // the inline staging was sized for this W/R at snapshot upload (the
    // service was stopped then, and no patch was pending): never reallocated
    // here, where a staged patch may be waiting in it
    if (jsp::patch_inline_layout(jsp::kPatchInlineRows, 15u, e->W, e->R).bytes > v.pstage.bytes)
        return set_err(JSP_ESTATE, "inline patch staging not sized for W=%u R=%u", e->W, e->R);
    a.pstage = v.pstage.as<const char>();
    a.pdesc = v.pdesc.as<jsp::PatchDesc>();
    a.pdone = e->h_patch_done.as<uint32_t>();
    a.taken = e->h_patch_done.as<uint32_t>() + 16;  // its own line
    // co-located compaction service: all its workgroups on one XCD when it
    // fits one (32 CUs, one workgroup per CU)
    a.spread = shape == 2 && nb + 1 <= 32 && e->hooks.svc_xcd ? 8u : 1u;
    a.pods = e->cls_h[0].pods;
    a.seq0 = v.seq;
    a.assign = v.assign.as<int32_t>();
    // the bitmap answer (test hook svc_entries=1: the per-job entries after a
    // look-back, for A/B runs)
    v.bitmap = shape == 2 && !e->hooks.svc_entries;
    a.bits = v.bitmap ? v.bits.as<unsigned long long>() : nullptr;
    // the microbox: a micro-patch's rows for the co-located resident tiles
    a.mbox = shape == 2 ? reinterpret_cast<unsigned long long*>(static_cast<char*>(v.granules.p) + gpad + 128 + xbytes) : nullptr;
    a.micro_spins = e->hooks.micro_spins;
    a.done = w;
    a.stats = w + n_tiles;
    a.err = w + n_tiles + 2;
    a.clk = e->timing && (shape == 2 || shape == 3) ? w + n_tiles + 3 : nullptr;
    a.n_tiles = n_tiles;
    a.spin_limit = e->spin_limit;
    // 100 MHz ticks; parked: 2^62 (never reached, and twice it does not wrap)
    a.idle_ticks = e->svc_mode == JSP_SERVICE_PARKED ? (1ull << 62) : (unsigned long long)(svc_idle_ms() * 1e5);
    a.ready = ready;
    a.gen = v.gen;
    v.err_ack = __atomic_load_n(w + n_tiles + 2, __ATOMIC_ACQUIRE);  // an earlier instance's error is not ours
    v.nb = n_tiles;
    v.blocks = nb;
    v.clk = e->timing;
    v.shape = shape;
    // Every workgroup of the grid must be resident at once (tiles wait on each
    // other and on the dispatcher): check the grid against what the CUs hold
    // at this LDS size before launching; a service that cannot fit is not
    // started and the launch path answers instead.
    const jsp::TallyArgs ta0 = tally_args(e, nullptr, nullptr, e->L_total);
    size_t lds = 0;
    uint32_t grid = 0;
    jsp::SplitArgs sp{};
    // the tiles keep their rows on chip between requests when each is one
    // chunk: the compaction tiles in registers (the resident path), the
    // split tiles in LDS
    const bool one_chunk = e->max_blk_span <= (uint32_t)jsp::kChunkRows;
    if (shape == 2) {
        a.resident = one_chunk ? 1u : 0u;
        a.row_cache_words = 0u;
        lds = jsp::service_lds_bytes(e->blk_leaves, (int)e->W, (int)e->R, false);
        grid = nb + 1;
    } else {
        sp.groups = v.groups;
        sp.cpg = v.cpg;
        sp.nw = jsp::split_waves(e->blk_l0, e->blk_l1);
        sp.C = e->C;
        sp.out = v.split.as<uint64_t>();
        sp.topo = e->topo;
        a.row_cache_words = one_chunk ? jsp::split_row_cache_words(v.cpg, e->blk_leaves) : 0u;
        a.anc_words = jsp::split_anc_words(v.cpg, e->blk_leaves, (int)e->W, (int)e->R, one_chunk);
        lds = jsp::split_service_lds_bytes(v.cpg, e->blk_leaves, (int)e->W, (int)e->R, one_chunk);
        grid = n_tiles + 1;
    }
    {
        // the API answer can be one workgroup per CU high at high SGPR counts
        // (MI355X_MICROARCH.md, Residency): keep that margin. Asked once per
        // (shape, W, R, LDS size).
        const unsigned long long okey = ((unsigned long long)lds << 16) | ((unsigned long long)shape << 8) |
                                        ((unsigned long long)e->W << 4) | e->R;
        if (v.occ_key != okey) {
            int per_cu = 0;
            HIP_TRY(jsp::service_occupancy(ta0, shape, lds, &per_cu));
            v.occ_fit = std::max(per_cu > 1 ? per_cu - 1 : per_cu, 0);
            v.occ_key = okey;
        }
        const int64_t fit = (int64_t)v.occ_fit * e->n_cu;
        if ((int64_t)grid > fit)
            return set_err(JSP_ERANGE, "placement service needs %u co-resident workgroups; %d CUs hold %lld at %zu B "
                                       "of LDS each", grid, e->n_cu, (long long)fit, lds);
    }
    if (shape == 2) HIP_TRY(jsp::launch_service(ta0, a, v.stream));
    else HIP_TRY(jsp::launch_split_service(ta0, sp, a, v.stream));
    v.running = true;
    v.pending_ready = true;
    v.t_launch = std::chrono::steady_clock::now();
    v.last = v.t_launch;
    e->acc.svc_starts += 1;
    {
        std::lock_guard<std::mutex> l(e->met_mu);
        e->met.svc_starts += 1;
    }
    return wait_ready ? svc_wait_ready(e) : JSP_OK;
}

// Return once the dispatcher polls: a request posted then is answered without
// waiting for the launch (bounded: a dispatcher that cannot get a CU within
// 2 s means the grid is not co-resident).
int svc_wait_ready(jsp_engine* e) {
    auto& v = e->svc;
    if (!v.pending_ready) return JSP_OK;
    const uint32_t* ready = v.box.as<uint32_t>() + kReadyWord;
    const auto t_start = v.t_launch;
    QueryPacer qp;
    for (uint64_t spins = 1; __atomic_load_n(ready, __ATOMIC_ACQUIRE) != v.gen; ++spins) {
        if ((spins & 255) == 0 && qp.due()) {
            const hipError_t q = hipStreamQuery(v.stream);
            if (q != hipErrorNotReady) {
                v.running = false;
                return set_err(JSP_EHIP, "placement service ended before it started polling: %s",
                               hipGetErrorString(q));
            }
            if (std::chrono::steady_clock::now() - t_start > std::chrono::seconds(2)) {
                (void)svc_stop(e);
                v.start_failed = true;  // not co-resident on this GPU as launched: off until the next upload
                return set_err(JSP_EHIP, "placement service did not start polling within 2 s");
            }
        }
    }
    v.pending_ready = false;
    e->acc.svc_ready_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_start).count();
    v.last = std::chrono::steady_clock::now();
    return JSP_OK;
}

// Tile t's bitmap answer line to request seq has arrived whole (its 8
// halves carry seq): the tile is past its row reads -- the bitmap answer's
// done signal (timing off: the tiles write no done word then).
static inline bool bits_line_done(const unsigned long long* b, uint32_t t, uint32_t seq) {
    uint32_t bad = 0;
    for (int k = 0; k < 8; ++k) bad |= (uint32_t)(__atomic_load_n(b + 8u * t + k, __ATOMIC_ACQUIRE) >> 32) ^ seq;
    return bad == 0;
}

// Waits for every tile's done word == seq (timing off, the bitmap answer:
// every tile's tagged line instead). kSvcGone: the service left before answering (its stream
// finished).
int svc_wait(jsp_engine* e, uint32_t seq, uint32_t J) {
    auto& v = e->svc;
    const uint32_t* words = v.words.as<uint32_t>();
    const unsigned long long* lines = v.bitmap && !v.clk ? v.bits.as<unsigned long long>() : nullptr;
    const uint32_t n = v.nb;
    const bool split = v.shape == 3;
    // (the split service writes done words for requests without jobs, the
    // only ones this waits for; with jobs the host reads its lines,
    // svc_wait_split)
    // every tile's line(s) at once: read one after another they would miss
    // one after another (a settle usually comes after the host slept or
    // worked, with none of them cached)
    if (lines)
        for (uint32_t t = 0; t < n; ++t) __builtin_prefetch(lines + 8u * t, 0, 3);

    // compaction: tiles 0..i-1 have answered, so assign[] up to about i/n of
    // J is final (tiles own consecutive ranges of roughly equal size): start
    // those lines' misses before the copy-out (cfg2 copy-out 0.55 us cold)
    const char* as = v.shape == 2 ? static_cast<const char*>(v.assign.p) : nullptr;
    size_t pf = 0;
    uint32_t i = 0;
    QueryPacer qp;
    for (uint64_t spins = 1;; ++spins) {
        while (i < n && (lines ? bits_line_done(lines, i, seq) : __atomic_load_n(words + i, __ATOMIC_ACQUIRE) == seq)) {
            if (split) e->walk.prefetch_tile(v.split.as<uint64_t>(), i);  // its slots are final: start their misses
            ++i;
            if (as) {
                const size_t upto = ((size_t)J * 8 * i / n) & ~size_t(63);
                for (; pf + 64 <= upto; pf += 64) __builtin_prefetch(as + pf, 0, 3);
            }
        }
        if (i == n) return JSP_OK;
        // a tile whose microbox wait gave up writes no line, but the error word
        if ((spins & 255) == 0 && lines && __atomic_load_n(words + n + 2, __ATOMIC_ACQUIRE) != v.err_ack)
            return kSvcFailed;
        if ((spins & 255) == 0 && qp.due()) {
            const hipError_t q = hipStreamQuery(v.stream);
            if (q == hipSuccess) {
                for (; i < n; ++i)
                    if (lines ? !bits_line_done(lines, i, seq) : __atomic_load_n(words + i, __ATOMIC_ACQUIRE) != seq)
                        return kSvcGone;
                return JSP_OK;
            }
            if (q != hipErrorNotReady) return set_err(JSP_EHIP, "placement service failed: %s", hipGetErrorString(q));
        }
    }
}

// The compaction request the host returned from early (its assign[] entries
// had all arrived): wait for its tiles' done words before anything that needs
// them idle -- the next request (tiles past the J-th feasible leaf may still be
// tallying, and the look-back granules are per tile), a patch of the rows.
int svc_settle(jsp_engine* e) {
    auto& v = e->svc;
    if (v.pending == 0) return JSP_OK;
    const uint32_t q = v.pending;
    v.pending = 0;
    if (!v.running) return JSP_OK;
    const int rc = svc_wait(e, q, 0);
    if (rc == kSvcGone) {  // it left after answering: nothing is outstanding
        v.running = false;
        return JSP_OK;
    }
    if (rc == kSvcFailed) {
        // a tile past the early answer's last job gave up its microbox wait
        // (the answer itself was complete: that tile's line was not needed).
        // Its registers may be stale: the service is stopped, and the next
        // request starts it afresh from the rows in memory.
        v.err_ack = __atomic_load_n(v.words.as<uint32_t>() + v.nb + 2, __ATOMIC_ACQUIRE);
        return svc_stop(e);
    }
    // The early answer had all J entries, so a tile past them that timed out
    // in its look-back (it scattered nothing) did not touch it: acknowledge
    // its error word here rather than blame the next request for it.
    if (rc == JSP_OK && v.words.p)
        v.err_ack = __atomic_load_n(v.words.as<uint32_t>() + v.nb + 2, __ATOMIC_ACQUIRE);
    return rc;
}


// The compaction service's answer read from the entries themselves: entry j
// is (seq << 32 | domain) in one 8-byte store, so the host copies each out as
// soon as it carries this request's seq and returns when all J have -- before
// the tiles drain and publish their done words (those gate the next request:
// svc_settle). kSvcGone: the service left; kSvcFailed: a tile timed out.
int svc_wait_entries(jsp_engine* e, uint32_t seq, uint32_t J, int32_t* out, uint32_t* placed) {
    auto& v = e->svc;
    const unsigned long long* a = v.assign.as<unsigned long long>();
    const uint32_t* w = v.words.as<uint32_t>();
    uint32_t i = 0, n = 0;
    QueryPacer qp;
    for (uint64_t spins = 1;; ++spins) {
        const uint32_t i0 = i;
        while (i < J) {
            const unsigned long long x = __atomic_load_n(a + i, __ATOMIC_ACQUIRE);
            if ((uint32_t)(x >> 32) != seq) break;
            const int32_t d = (int32_t)(uint32_t)x;
            out[i++] = d;
            n += d >= 0 ? 1u : 0u;
        }
        if (i0 == 0 && i > 0) v.first_seen = std::chrono::steady_clock::now();
        if (i == J) {
            *placed = n;
            return JSP_OK;
        }
        if ((spins & 255) == 0) {
            if (__atomic_load_n(w + v.nb + 2, __ATOMIC_ACQUIRE) != v.err_ack) return kSvcFailed;
            if (!qp.due()) continue;
            const hipError_t q = hipStreamQuery(v.stream);
            if (q == hipSuccess) {  // it left: whatever arrived is all there is
                for (; i < J; ++i) {
                    const unsigned long long x = __atomic_load_n(a + i, __ATOMIC_ACQUIRE);
                    if ((uint32_t)(x >> 32) != seq) return kSvcGone;
                    out[i] = (int32_t)(uint32_t)x;
                    n += out[i] >= 0 ? 1u : 0u;
                }
                *placed = n;
                return JSP_OK;
            }
            if (q != hipErrorNotReady) return set_err(JSP_EHIP, "placement service failed: %s", hipGetErrorString(q));
        }
    }
}

// The compaction service's bitmap answer (ServiceArgs::bits): tile t's line
// holds its leaves' feasibility as four 64-leaf words, each as two (seq << 32
// | 32 bits) halves. Tiles own consecutive leaf ranges in leaf order, so job
// j's domain is the j-th feasible leaf: the host takes the lines in tile
// order as they arrive, bit by bit, and returns once J jobs have a leaf or
// every tile has answered (the rest get -1). kSvcGone: the service left.
// *all: every tile's line arrived -- each tile then has read its rows and
// holds no state of this request that a patch or the next request could
// disturb, so neither waits for the tiles' done words (svc_settle); after an
// answer complete before its last tiles, they do.
constexpr uint32_t kPrefetchAhead = 8;  // answer lines in flight ahead of the one expanded

int svc_wait_bits(jsp_engine* e, uint32_t seq, uint32_t J, int32_t* out, uint32_t* placed, bool* all) {
    auto& v = e->svc;
    const unsigned long long* b = v.bits.as<unsigned long long>();
    const uint32_t n = v.nb, base = e->leaf_begin;
    const uint32_t* l0 = e->blk_l0.data();
    uint32_t t = 0, j = 0;
    QueryPacer qp;
    for (uint64_t spins = 1;; ++spins) {
        // touch every line still to come (independent loads: their misses
        // overlap), so a line that has landed is in cache when its turn comes
        // -- not one miss after another in tile order
        for (uint32_t u = t + 1; u < n; ++u) __builtin_prefetch(b + 8u * u, 0, 3);
        while (t < n && j < J) {
            const unsigned long long* L = b + 8u * t;
            unsigned long long x[8];
            uint32_t bad = 0;
            for (int k = 0; k < 8; ++k) {
                x[k] = __atomic_load_n(L + k, __ATOMIC_ACQUIRE);
                bad |= (uint32_t)(x[k] >> 32) ^ seq;
            }
            if (bad) break;
            if (t == 0) v.first_seen = std::chrono::steady_clock::now();
            // the tiles answer within ~0.1 us of each other: once a line is in,
            // the next ones have landed too (and the copies the spin's
            // prefetches brought in before they landed are gone). Keep the
            // lines kPrefetchAhead ahead in flight while this one is expanded.
            if (t == 0)
                for (uint32_t u = 1; u < n && u <= kPrefetchAhead; ++u) __builtin_prefetch(b + 8u * u, 0, 3);
            else if (t + kPrefetchAhead < n)
                __builtin_prefetch(b + 8u * (t + kPrefetchAhead), 0, 3);
            const uint32_t d0 = base + l0[t];
            for (uint32_t w = 0; w < 4 && j < J; ++w) {
                // run by run: feasible leaves come in long runs (a word of 64
                // is the common case), each written by a loop that vectorizes
                uint64_t m = (x[2 * w] & 0xFFFFFFFFull) | (x[2 * w + 1] << 32);
                const int32_t dw = (int32_t)(d0 + 64u * w);
                while (m != 0ull && j < J) {
                    const uint32_t s0 = (uint32_t)__builtin_ctzll(m);
                    const uint64_t sh = m >> s0;
                    const uint32_t r = ~sh == 0ull ? 64u - s0 : (uint32_t)__builtin_ctzll(~sh);
                    const uint32_t take = std::min(r, J - j);
                    int32_t* o = out + j;
                    const int32_t d = dw + (int32_t)s0;
                    for (uint32_t k = 0; k < take; ++k) o[k] = d + (int32_t)k;
                    j += take;
                    m = s0 + r >= 64u ? 0ull : m & (~0ull << (s0 + r));
                }
            }
            ++t;
        }
        if (t == n || j == J) {
            *placed = j;
            *all = t == n;
            for (uint32_t i = j; i < J; ++i) out[i] = -1;
            return JSP_OK;
        }
        // a tile whose microbox wait gave up writes no line, but the error word
        if ((spins & 255) == 0 && __atomic_load_n(e->svc.words.as<uint32_t>() + n + 2, __ATOMIC_ACQUIRE) != v.err_ack)
            return kSvcFailed;
        if ((spins & 255) == 0 && qp.due()) {
            const hipError_t q = hipStreamQuery(v.stream);
            if (q == hipSuccess) {  // it left: only a line already complete counts
                const unsigned long long* L = b + 8u * t;
                uint32_t bad = 0;
                for (int k = 0; k < 8; ++k) bad |= (uint32_t)(__atomic_load_n(L + k, __ATOMIC_ACQUIRE) >> 32) ^ seq;
                if (bad) return kSvcGone;
                continue;
            }
            if (q != hipErrorNotReady) return set_err(JSP_EHIP, "placement service failed: %s", hipGetErrorString(q));
        }
    }
}

// The split service's answer (jsp_internal.h SplitArgs): every tile's lines and
// records carry the request, so the host takes tile after tile as each has
// arrived whole -- touching the lines still to come every few polls, so
// their misses overlap -- with no done word in between. kSvcGone: the
// service left.
int svc_wait_split(jsp_engine* e, uint32_t seq) {
    auto& v = e->svc;
    const uint64_t* s = v.split.as<uint64_t>();
    const uint32_t n = v.nb;
    uint32_t t = 0;
    if (e->hooks.wait_delay_ns) {  // diagnostic: let the answer land before reading it
        const auto until = std::chrono::steady_clock::now() + std::chrono::nanoseconds(e->hooks.wait_delay_ns);
        while (std::chrono::steady_clock::now() < until) __builtin_ia32_pause();
    }
    QueryPacer qp;
    for (uint64_t spins = 1;; ++spins) {
        while (t < n && e->walk.tile_ready(s, t, seq)) ++t;
        if (t == n) return JSP_OK;
        if ((spins & 7) == 1)
            for (uint32_t u = t + 1; u < n; ++u) e->walk.prefetch_tile(s, u);
        if ((spins & 255) == 0 && qp.due()) {
            const hipError_t q = hipStreamQuery(v.stream);
            if (q == hipSuccess) {  // it left: only tiles already complete count
                while (t < n && e->walk.tile_ready(s, t, seq)) ++t;
                return t == n ? JSP_OK : kSvcGone;
            }
            if (q != hipErrorNotReady) return set_err(JSP_EHIP, "placement service failed: %s", hipGetErrorString(q));
        }
    }
}

// The request number after q. Never 0 (the done words' initial value) or
// kSvcStop, and never a value whose low 30 bits are 0: the compaction tiles
// tag their look-back granules with seq & 0x3FFFFFFF (0 -> 1), so 2^30 would
// share its tag with the request after it and a tile could take that request
// predecessor's stale granule as current.
uint32_t next_seq(uint32_t q) {
    uint32_t s = q + 1;
    while (s == 0 || s == jsp::kSvcStop || (s & 0x3FFFFFFFu) == 0) ++s;
    return s;
}


// Wait for the last snapshot patch's completion word (the rows are then in
// memory for every later reader, the resident tiles' `sc1` loads included).
// A patch held back for the next request, posted on its own now (a service
// that has left meanwhile is caught by patch_wait, and the patch kernel
// applies it).
void patch_post_deferred(jsp_engine* e) {
    if (!e->patch_deferred) return;
    e->patch_deferred = false;
    auto& v = e->svc;
    const uint32_t seq = next_seq(v.seq);
    v.seq = seq;
    v.last = std::chrono::steady_clock::now();
    svc_request(e, seq, e->patch_bits | jsp::kReqPatchOnly, e->patch_nf, e->patch_micro);
    e->patch_req = seq;
    // applied on its own: the next request's tiles reload the rows
    v.rows_dirty |= v.micro_dirty;
    v.micro_dirty = false;
}

int patch_wait(jsp_engine* e) {
    if (!e->patch_pending) return JSP_OK;
    e->wake_job = false;  // a reader other than a placement: no wake, the patch lands now
    if (e->patch_deferred && !e->svc.running) {
        // held back for a service that is not up: the patch kernel applies it
        e->patch_deferred = false;
        e->patch_svc = false;
        if (int rc = use_engine_stream(e)) return rc;
        e->patch_target += (e->last_patch.n + 255) / 256;
        e->last_patch.target = e->patch_target;
        HIP_TRY(jsp::launch_patch(e->last_patch, e->stream));
    }
    patch_post_deferred(e);
    const uint32_t* w = e->h_patch_done.as<uint32_t>();
    const auto t0 = std::chrono::steady_clock::now();
    const auto limit = std::chrono::duration<double, std::milli>(2.0 * svc_idle_ms() + 100.0);
    for (uint64_t spins = 1; __atomic_load_n(w, __ATOMIC_ACQUIRE) != e->patch_seq; ++spins) {
        if ((spins & 255) == 0 && e->patch_svc) {
            // posted to the dispatcher: if the service left without taking it
            // (an idle exit racing the post), apply it with the patch kernel.
            // A live service that never takes it (bounded: it polls every few
            // microseconds) is stopped, and the patch kernel applies it too
            // (the staged delta is unchanged: writing it twice writes the
            // same values)
            const hipError_t q = hipStreamQuery(e->svc.stream);
            if (q == hipErrorNotReady && std::chrono::steady_clock::now() - t0 < limit) continue;
            if (__atomic_load_n(w, __ATOMIC_ACQUIRE) == e->patch_seq) break;
            e->patch_svc = false;
            if (q == hipErrorNotReady) {
                e->svc.pending = 0;
                if (int rc = svc_stop(e)) return rc;  // patch_svc is off: the stop does not wait for it
            }
            e->svc.running = false;
            if (int rc = use_engine_stream(e)) return rc;
            e->patch_target += (e->last_patch.n + 255) / 256;
            e->last_patch.target = e->patch_target;
            HIP_TRY(jsp::launch_patch(e->last_patch, e->stream));
            continue;
        }
        if ((spins & 255) == 0) {
            const hipError_t q = hipStreamQuery(e->stream);
            if (q == hipErrorNotReady) continue;
            if (__atomic_load_n(w, __ATOMIC_ACQUIRE) == e->patch_seq) break;
            e->patch_pending = false;
            if (q == hipSuccess) return set_err(JSP_EHIP, "snapshot patch %u ended without its completion word", e->patch_seq);
            return set_err(JSP_EHIP, "snapshot patch %u failed: %s", e->patch_seq, hipGetErrorString(q));
        }
    }
    e->patch_pending = false;
    e->patch_svc = false;
    return JSP_OK;
}

// Launches that read the rows are stream-ordered after a patch kernel, but
// not after a patch the service applies: they wait for its word first.
int patch_fence(jsp_engine* e) { return e->patch_pending && e->patch_svc ? patch_wait(e) : JSP_OK; }

// How patches reach the resident service's dispatcher: posted at once, so the
// dispatcher applies them during the gap before the next request (a
// recovery's deletions take milliseconds), and a request posted before the
// patch's completion word came back carries it again (applying a staged
// patch twice writes the same values; the request may have replaced the
// patch's own in the mailbox).

// A snapshot patch is the first sign of a recovery: the watch events of the
// deleted Jobs' pods arrive while the reconciler deletes them in the
// foreground, before it recreates and places them
// (pkg/controllers/jobset_controller.go:553-576, 698-709). When the host API
// has been answered by the resident service (armed), a patch (re)starts it
// here without waiting: the GPU wakes from idle and the grid comes up while
// the deletions finish, and the recreate's jsp_place finds it polling.
// Whether a patch should (re)start the service: the host API has been
// answered by it and it is not up (or about to idle out).
bool svc_wake_wanted(jsp_engine* e) {
    auto& v = e->svc;
    if (!v.armed || !svc_ok(e)) return false;
    const double since = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - v.last).count();
    return !(v.running && since <= 0.5 * idle_ms(e));
}

// (Re)start the service without waiting for its dispatcher to poll. Long
// idle (a recovery after hours): the service has left by itself and its
// stream is done -- a query, not a synchronize, tells; otherwise it is
// stopped. On failure it stays stopped (the next jsp_place starts it, or
// answers on the launch path) and the error is dropped.
int svc_restart_quiet(jsp_engine* e) {
    auto& v = e->svc;
    const double since = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - v.last).count();
    if (v.running && since > idle_ms(e) + 5.0 && hipStreamQuery(v.stream) == hipSuccess) {
        v.running = false;
        v.pending = 0;
        e->grave.flush();
    }
    if (svc_stop(e) != JSP_OK || svc_start(e, 0, false) != JSP_OK) {
        (void)svc_stop(e);
        g_err.clear();
        return JSP_EHIP;
    }
    v.resume = false;
    return JSP_OK;
}

void svc_wake(jsp_engine* e) {
    auto& v = e->svc;
    if (!svc_wake_wanted(e) || svc_restart_quiet(e) != JSP_OK) return;
    // A warm-up request (no jobs, rows marked patched): the fresh tiles load
    // their rows, run every phase once and pull the kernel's code into the
    // instruction caches while the deletions finish, so the recreate's
    // request runs warm. Posted without waiting (the dispatcher finds it when
    // it starts polling); the next request settles it first (svc_settle).
    const uint32_t seq = next_seq(v.seq);
    v.seq = seq;
    v.last = std::chrono::steady_clock::now();
    svc_request(e, seq, jsp::kReqDirty, 0u);
    // rows marked patched, and they stay marked: the patch kernel may not
    // have landed when the warm-up loads them, so the next request (which
    // waits for the patch's completion word) loads them again
    v.pending = seq;
}

// The waker's job (or the next caller's, whichever takes the engine lock
// first): restart the service, post the held-back patch and, for the tile
// shapes, a warm-up request (no jobs) behind it -- the fresh tiles load the
// patched rows and pull the code into the instruction caches while the
// deletions finish, so the recreate's request runs warm. A patch already
// taken care of (patch_wait) leaves nothing to do; a start that fails
// leaves the patch held back, and patch_wait hands it to the patch kernel.
void run_wake(jsp_engine* e) {
    if (!e->wake_job) return;
    e->wake_job = false;
    if (!(e->patch_pending && e->patch_svc && e->patch_deferred)) return;
    const auto t0 = std::chrono::steady_clock::now();
    if (svc_restart_quiet(e) != JSP_OK) return;
    auto& v = e->svc;
    const uint32_t seq = next_seq(v.seq);
    v.seq = seq;
    v.last = std::chrono::steady_clock::now();
    svc_request(e, seq, e->patch_bits | jsp::kReqDirty, (e->patch_bits & jsp::kReqPatchInline) ? e->patch_nf : 0u,
                e->patch_micro);
    e->patch_req = seq;
    e->patch_deferred = false;
    v.pending = seq;
    v.rows_dirty = v.micro_dirty = false;  // the warm-up loads the patched rows
    e->acc.wake_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
}

// The waker's loop. While the service is armed (a placement it answered may
// be followed by a recovery's first patch, hours later) the waker polls the
// ring every waker_poll_us (200 us: ~5k sleeps a second, ~1 % of one core),
// so the patch call that rings it only stores a flag -- a futex wake from a
// core that slept was the default service's cold-recovery tail (patch call
// p95 9.9 us against 4.7 us with no wake, profiles/r06/g2). Otherwise it
// sleeps on wake_cv. The ring is consumed whichever way it arrives; a ring
// the waker has not taken yet is run by the next placement itself (run_wake).
void waker_main(jsp_engine* e) {
    // Normal priority: at SCHED_IDLE (measured, profiles/r05) a waker
    // preempted while it held the engine lock stalled the next placement by
    // milliseconds (a 5.2 ms cold-recovery p99 on a shared host).
    (void)hipSetDevice(e->device);
    const auto period = std::chrono::microseconds(e->hooks.waker_poll_us);
    for (;;) {
        if (e->wake_quit.load(std::memory_order_acquire)) return;
        if (e->wake_ring.exchange(false, std::memory_order_acq_rel)) {
            std::lock_guard<std::mutex> g(e->mu);
            run_wake(e);
            continue;
        }
        if (period.count() > 0 && e->waker_poll.load(std::memory_order_acquire)) {
            e->waker_polling.store(true, std::memory_order_release);
            if (e->hooks.waker_spin) {
                for (int i = 0; i < 64; ++i) __builtin_ia32_pause();
            } else {
                std::this_thread::sleep_for(period);
            }
            continue;
        }
        e->waker_polling.store(false, std::memory_order_release);
        std::unique_lock<std::mutex> l(e->wake_mu);
        e->wake_cv.wait_for(l, std::chrono::milliseconds(50), [e, period] {
            return e->wake_ring.load() || e->wake_quit.load() || (period.count() > 0 && e->waker_poll.load());
        });
    }
}

// The waker thread, created with the engine's first service (thread creation
// costs ~100 us, which must never land in a recovery's patch call).
void start_waker(jsp_engine* e) {
    if (!e->waker.joinable()) e->waker = std::thread(waker_main, e);
}

// Hand the wake to the waker thread. Called with mu held; the caller delivers
// it (notify_waker) after releasing mu, so the waker never wakes into a held
// lock. (Diagnostic A/B build tools/bin/ab_inlinewake, -DJSP_AB_INLINE_WAKE:
// the patch call runs the wake itself; never the product library.)
void ring_waker(jsp_engine* e) {
    e->wake_job = true;
#ifdef JSP_AB_INLINE_WAKE
    run_wake(e);
    return;
#endif
    start_waker(e);
    e->wake_ring.store(true, std::memory_order_release);
    if (e->waker_polling.load(std::memory_order_acquire)) return;  // it polls: no notify
    {
        std::lock_guard<std::mutex> l(e->wake_mu);  // no lost wake-up between its predicate and its wait
    }
    e->wake_notify.store(true, std::memory_order_relaxed);
}

// The service became armed: the waker leaves its condition variable for its
// polling loop (once per arming; a waiter that misses it polls within 50 ms).
void notify_waker_poll(jsp_engine* e) { e->wake_cv.notify_one(); }

// Deliver a ring (mu not held). Keeping the waker off the ringing thread's
// CPU (an affinity change when the caller's CPU changed) was measured and
// dropped: the affinity call costs the patch call 6-15 us at p50
// (profiles/r05/probes/cold4_waker_affinity_ab.txt).
void notify_waker(jsp_engine* e) {
    if (!e->wake_notify.exchange(false, std::memory_order_relaxed)) return;
    e->wake_cv.notify_one();
}

// One placement through the service: J jobs of the engine's one class.
int svc_place(jsp_engine* e, const uint32_t* run_class, const uint32_t* run_len, uint32_t n_runs, uint32_t J,
              int32_t* assign_out, uint32_t* placed) {
    auto& v = e->svc;
    const auto t_in = std::chrono::steady_clock::now();
    run_wake(e);  // a recovery's wake the waker has not run yet: run it here
    const auto now = std::chrono::steady_clock::now();
    const int shape = svc_shape(e);
    bool restart = !v.running || J > v.cap || v.clk != e->timing || v.blocks != e->n_blocks || v.shape != shape ||
                   std::chrono::duration<double, std::milli>(now - v.last).count() > 0.5 * idle_ms(e);
    // the request's tiles must read the patched rows: a patch held back for
    // the running service rides on this request (its dispatcher applies it
    // before ringing the tiles); any other is waited for
    bool carry = !restart && e->patch_pending && e->patch_svc;
    if (!carry)
        if (int rc = patch_wait(e)) return rc;
    // A cold start -- the first request after an idle exit (recoveries are
    // hours apart, and a recovery's first patch has normally restarted it
    // already), an upload or a geometry change -- launches the service, waits
    // for its dispatcher to poll and posts to it. Measured after 60 ms idle on
    // MI355X (profiles/r03): cfg2 p50 33 us, max 67 us this way, against 66 /
    // 428 us when the launch path answered the cold call while the service
    // came up -- the polling dispatcher brings the GPU out of its idle state
    // while the host waits, and a launch after idling pays that wake-up inside
    // the kernel.
    if (!restart) {
        if (int rc = svc_wait_ready(e)) return rc;
        if (int rc = svc_settle(e)) return rc;
        if (!v.running) {  // the settle stopped it (kSvcFailed): a fresh start, the patch applied first
            restart = true;
            if (carry) {
                carry = false;
                if (int rc = patch_wait(e)) return rc;
            }
        }
    }
    if (carry) {  // held back, or posted and its completion word not back yet
        // (a posted patch the dispatcher has taken is applied before it takes
        // this request: no need to carry it again)
        const uint32_t* pw = e->h_patch_done.as<uint32_t>();
        carry = e->patch_deferred || (__atomic_load_n(pw, __ATOMIC_ACQUIRE) != e->patch_seq &&
                                      __atomic_load_n(pw + 16, __ATOMIC_ACQUIRE) != e->patch_req);
        e->patch_deferred = false;
    }
    // the compaction answer is read from its tagged entries (timing on: the
    // done words, which carry the per-tile stamps)
    // (timing on too: the stamps are read once the tiles' done words are in)
    const bool early = shape == 2 && J > 0;
    uint32_t seq = 0, n_early = 0;
    bool all_tiles = false;
    std::chrono::steady_clock::time_point t_post{};
    for (int attempt = 0;; ++attempt) {
        if (restart) {
            if (int rc = svc_stop(e)) return rc;
            if (int rc = svc_start(e, J, true)) return rc;
        }
        seq = next_seq(v.seq);
        v.seq = seq;
        v.last = std::chrono::steady_clock::now();
        // second half first: the dispatcher reads both halves in one 16-byte
        // load (an inline patch carried here: its n | flags in place of n_runs,
        // which the tiles do not read)
        const uint32_t w2 = carry && (e->patch_bits & jsp::kReqPatchInline) ? e->patch_nf : n_runs;
        // the tiles keep their rows on chip: bit 31 of J tells them the
        // snapshot was patched since their previous request (J < 2^28)
        // (a micro-patch carried here: the dispatcher hands its rows to the
        // resident tiles, or marks the rows patched itself)
        const bool micro = carry && e->patch_micro;
        const bool dirty = v.rows_dirty || (v.micro_dirty && !micro);
        const uint32_t jw = J | (dirty ? jsp::kReqDirty : 0u) | (carry ? e->patch_bits : 0u);
        carry = false;  // a retry finds it applied, or applied by the patch kernel (patch_wait)
        v.rows_dirty = v.micro_dirty = false;
        if (attempt == 0) {
            t_post = std::chrono::steady_clock::now();
            e->acc.svc_pre_us += std::chrono::duration<double, std::micro>(t_post - t_in).count();
        }
        svc_request(e, seq, jw, w2, micro);
        // (the split shape, timing off and J > 0: its tagged lines; with the
        // stamps on, the done words, which follow the stamps)
        const int rc = !early ? (v.shape == 3 && !v.clk && J > 0 ? svc_wait_split(e, seq) : svc_wait(e, seq, J))
                       : v.bitmap ? svc_wait_bits(e, seq, J, assign_out, &n_early, &all_tiles)
                                  : svc_wait_entries(e, seq, J, assign_out, &n_early);
        if (rc == kSvcFailed) {
            const uint32_t ew = __atomic_load_n(v.words.as<uint32_t>() + v.nb + 2, __ATOMIC_ACQUIRE);
            v.err_ack = ew;
            (void)svc_stop(e);
            return set_err(JSP_EHIP, "placement service request %u failed: %s; its assign[] is invalid", seq,
                           (ew & jsp::kErrKindMask) == jsp::kErrMicro
                               ? "a resident tile's wait for the request's micro-patch rows gave up"
                               : "the compaction look-back timed out");
        }
        if (rc == kSvcGone && attempt == 0) {
            v.running = false;
            restart = true;
            continue;
        }
        if (rc == kSvcGone) return set_err(JSP_EHIP, "placement service left before answering request %u", seq);
        if (rc) return rc;
        break;
    }
    e->acc.svc_answer_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_post).count();
    if (early && J > 0) e->acc.svc_first_us += std::chrono::duration<double, std::micro>(v.first_seen - t_post).count();
    if (v.clk && v.nb > 0) {
        if (early) {  // the tiles' stamps land with their done words
            v.pending = seq;
            if (int rc = svc_settle(e)) return rc;
        }
        // the request's device time: first tile saw it -> last tile drained
        const uint32_t* clk = v.words.as<uint32_t>() + v.nb + 3;
        const uint32_t ref = clk[0];
        int32_t lo = 0, hi = 0;
        for (uint32_t t = 0; t < v.nb; ++t) {
            lo = std::min(lo, (int32_t)(clk[jsp::kSvcClkSlots * t] - ref));
            hi = std::max(hi, (int32_t)(clk[jsp::kSvcClkSlots * t + 5] - ref));
        }
        e->acc.svc_us += (double)(hi - lo) / 100.0;
        std::lock_guard<std::mutex> l(e->met_mu);
        hist_add(e->met.device_us, (double)(hi - lo) / 100.0, JSP_HIST_LO_US);
    }
    if (v.shape == 3) {  // the tiles answered: the walk, into the caller's buffer
        const auto tw = std::chrono::steady_clock::now();
        *placed = e->walk.place(v.split.as<uint64_t>(), run_class, run_len, n_runs, assign_out);
        // the host walk's share of the wait (jsp_timing.host_post_us on this path)
        e->acc.host_post_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tw).count();
        e->acc.svc_calls += 1;
        return JSP_OK;
    }
    if (early) {
        v.pending = all_tiles ? 0u : seq;
        *placed = n_early;
        e->acc.svc_calls += 1;
        return JSP_OK;
    }
    const uint32_t* w = v.words.as<uint32_t>();
    const uint32_t ew = __atomic_load_n(w + v.nb + 2, __ATOMIC_ACQUIRE);
    if (ew != v.err_ack) {
        v.err_ack = ew;
        (void)svc_stop(e);
        return set_err(JSP_EHIP, "placement service request %u failed: the compaction look-back timed out; "
                                 "its assign[] is invalid", seq);
    }
    const auto tc = std::chrono::steady_clock::now();
    {  // u64 entries: the domain is the low half
        const unsigned long long* a = v.assign.as<unsigned long long>();
        for (uint32_t j = 0; j < J; ++j) assign_out[j] = (int32_t)(uint32_t)a[j];
    }
    // (the bitmap answer writes no stats: it runs this path only for J = 0)
    *placed = v.bitmap ? 0u : __atomic_load_n(w + v.nb + 1, __ATOMIC_ACQUIRE);
    // the copy-out's share of the wait (jsp_timing.host_post_us on this path)
    e->acc.host_post_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tc).count();
    e->acc.svc_calls += 1;
    return JSP_OK;
}

// ---- micro-patches (jsp_internal.h kMailbox*)
// Whether the resident service is up and fresh enough to take a patch
// through its dispatcher (not about to idle out, the engine's shape).
bool svc_up(jsp_engine* e) {
    auto& v = e->svc;
    const double since = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - v.last).count();
    return v.running && since <= 0.5 * idle_ms(e) && svc_ok(e) && svc_shape(e) == v.shape;
}

// Merge n rows of one patch call (columns fl) into the held micro-patch: a
// row already held takes the new values, a new row is appended. All or
// nothing: false when the rows do not fit.
bool micro_merge(jsp_engine* e, const uint32_t* rows, uint32_t n, const uint64_t* labels, const uint32_t* taints,
                 const uint32_t* free_res, const int32_t* excl) {
    const uint32_t W = e->W, R = e->R, rw = jsp::micro_row_words(W, R), cap = jsp::micro_rows_max(W, R);
    uint32_t w[jsp::kMailboxPayload];
    std::memcpy(w, e->micro_w, sizeof w);
    uint32_t m = e->micro_n;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t r = 0;
        while (r < m && w[r * rw] != rows[i]) ++r;
        if (r == m) {
            if (m == cap) return false;
            std::memset(w + r * rw, 0, rw * 4);
            w[r * rw] = rows[i];
            ++m;
        }
        uint32_t* x = w + r * rw;
        if (labels)
            for (uint32_t k = 0; k < W; ++k) {
                const uint64_t l = labels[(size_t)k * n + i];
                x[1 + 2 * k] = (uint32_t)l;
                x[2 + 2 * k] = (uint32_t)(l >> 32);
            }
        if (taints) x[1 + 2 * W] = taints[i];
        if (free_res)
            for (uint32_t k = 0; k < R; ++k) x[2 + 2 * W + k] = free_res[(size_t)k * n + i];
        if (excl) x[2 + 2 * W + R] = (uint32_t)excl[i];
    }
    std::memcpy(e->micro_w, w, sizeof w);
    e->micro_n = m;
    return true;
}

// The held micro-patch in its kernel form too (engine staging, pinned): the
// patch kernel applies it if the service leaves before a request carries it.
int micro_stage_kernel_form(jsp_engine* e) {
    const uint32_t W = e->W, R = e->R, rw = jsp::micro_row_words(W, R), m = e->micro_n, fl = e->micro_fl;
    const jsp::PatchInlineLayout L = jsp::patch_inline_layout(m, 15u, W, R);
    HIP_TRY(e->h_patch.reserve(L.bytes, grave(e)));
    char* hp = static_cast<char*>(e->h_patch.p) - 64;  // the inline layout without its header
    for (uint32_t r = 0; r < m; ++r) {
        const uint32_t* x = e->micro_w + r * rw;
        reinterpret_cast<uint32_t*>(hp + L.rows)[r] = x[0];
        for (uint32_t k = 0; k < W; ++k)
            reinterpret_cast<uint64_t*>(hp + L.lab)[(size_t)k * m + r] = ((uint64_t)x[2 + 2 * k] << 32) | x[1 + 2 * k];
        reinterpret_cast<uint32_t*>(hp + L.taint)[r] = x[1 + 2 * W];
        for (uint32_t k = 0; k < R; ++k) reinterpret_cast<uint32_t*>(hp + L.free)[(size_t)k * m + r] = x[2 + 2 * W + k];
        reinterpret_cast<uint32_t*>(hp + L.excl)[r] = x[2 + 2 * W + R];
    }
    jsp::PatchArgs& a = e->last_patch;
    a = jsp::PatchArgs{};
    a.rows = reinterpret_cast<const uint32_t*>(hp + L.rows);
    a.n = m;
    a.npad = e->npad;
    a.W = W;
    a.R = R;
    a.dlab = (fl & jsp::kPatchLab) ? reinterpret_cast<const uint64_t*>(hp + L.lab) : nullptr;
    a.dtaint = (fl & jsp::kPatchTaint) ? reinterpret_cast<const uint32_t*>(hp + L.taint) : nullptr;
    a.dfree = (fl & jsp::kPatchFree) ? reinterpret_cast<const uint32_t*>(hp + L.free) : nullptr;
    a.dexcl = (fl & jsp::kPatchExcl) ? reinterpret_cast<const int32_t*>(hp + L.excl) : nullptr;
    a.labels = e->labels.as<uint64_t>();
    a.taints = e->taints.as<uint32_t>();
    a.freer = e->freer.as<uint32_t>();
    a.excl = e->excl.as<int32_t>();
    a.counter = e->patch_ctr.as<unsigned long long>();
    a.done = e->h_patch_done.as<uint32_t>();
    a.seq = e->patch_seq;
    return JSP_OK;
}

// Host-side validation of a run list; returns the job count through *J.
int check_runs(jsp_engine* e, const uint32_t* run_class, const uint32_t* run_len, uint32_t n_runs, uint64_t* J) {
    uint64_t n = 0;
    for (uint32_t i = 0; i < n_runs; ++i) {
        if (run_class[i] >= e->C) return set_err(JSP_EINVAL, "run %u: class %u out of range (%u classes)", i,
                                                  run_class[i], e->C);
        n += run_len[i];
    }
    if (n > (1u << 30)) return set_err(JSP_ERANGE, "%llu jobs exceed the 2^30 limit", (unsigned long long)n);
    *J = n;
    return JSP_OK;
}

// The f64 reciprocal r of d >= 2 with floor(double(n) * r) == floor(n / d)
// for every u32 n (the device truncates fl(n * r) to u32). With r = (1/d)(1 + e):
// fl(n * r) >= n/d needs e above the two roundings (2^-52); below q + 1 it
// needs (n/d)(1 + e + 2^-52) < q + 1, i.e. e < 1/(n + d) - 2^-52, which holds
// for e < 2^-34 as n + d < 2^33. r = fl(fl(1/d) (1 + 2^-45)) has e within
// 2^-45 +- 2^-52. tests/test_engine_gpu.py checks the edges (n = kd - 1, kd).
double divisor_rcp(uint32_t d) { return d >= 2 ? (1.0 / (double)d) * (1.0 + 0x1p-45) : d == 1 ? 1.0 : 0.0; }

int ready(jsp_engine* e, bool need_cls) {
    if (!e->have_topo) return set_err(JSP_ESTATE, "no topology uploaded");
    if (!e->have_snap) return set_err(JSP_ESTATE, "no snapshot uploaded");
    if (need_cls && !e->have_cls) return set_err(JSP_ESTATE, "no job classes uploaded");
    return JSP_OK;
}

// `iters` back-to-back device steps on the engine stream, each bracketed by
// a start event on its first dispatch and a stop event on its last
// (hipExtLaunchKernel: the dispatch packets' own timestamps, as a kernel
// trace reports them -- no host submit time, no marker packets). With a
// scrub buffer, a read-only sweep of it precedes every step (cold caches).
// out_us[0] median, out_us[1] mean over the steps.
template <class Step>
int time_steps(jsp_engine* e, uint32_t iters, const void* d_scrub, size_t scrub_bytes, double* out_us, Step step) {
    if (iters == 0 || iters > 4096) return set_err(JSP_EINVAL, "iters %u out of range [1,4096]", iters);
    if (!out_us) return set_err(JSP_EINVAL, "out_us is NULL");
    if (scrub_bytes > 0 && !d_scrub) return set_err(JSP_EINVAL, "scrub buffer is NULL");
    if (int rc = check_launch_error(e)) return rc;
    hipStream_t s = e->stream;
    if (int rc = use_engine_stream(e)) return rc;
    while (e->tev.size() < iters) {
        EvPair p;
        HIP_TRY(hipEventCreate(&p.a));
        HIP_TRY(hipEventCreate(&p.b));
        e->tev.push_back(p);
    }
    if (scrub_bytes > 0) HIP_TRY(e->tmp_scrub.reserve(64, grave(e)));
    int rc = JSP_OK;
    for (uint32_t i = 0; i < iters && rc == JSP_OK; ++i) {
        if (scrub_bytes > 0) HIP_TRY(jsp::launch_scrub(d_scrub, scrub_bytes, e->tmp_scrub.as<uint32_t>(), s));
        jsp::set_launch_start(e->tev[i].a);
        jsp::set_launch_stop(e->tev[i].b);
        rc = step(s);
        jsp::set_launch_start(nullptr);
        jsp::set_launch_stop(nullptr);
    }
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(s));
    std::vector<double> us(iters);
    double sum = 0.0;
    for (uint32_t i = 0; i < iters; ++i) {
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, e->tev[i].a, e->tev[i].b));
        us[i] = ms * 1e3;
        sum += us[i];
    }
    std::sort(us.begin(), us.end());
    out_us[0] = us[iters / 2];
    out_us[1] = sum / iters;
    return check_launch_error(e);
}
}  // namespace

extern "C" {

int jsp_abi_version(void) { return JSP_ABI_VERSION; }

const char* jsp_last_error(void) { return g_err.c_str(); }

int jsp_device_count(int* out) {
    if (!out) return set_err(JSP_EINVAL, "out is NULL");
    int n = 0;
    hipError_t err = hipGetDeviceCount(&n);
    if (err != hipSuccess) {
        *out = 0;
        return set_err(JSP_EHIP, "hipGetDeviceCount: %s", hipGetErrorString(err));
    }
    *out = n;
    return JSP_OK;
}

int jsp_engine_create(int device_id, jsp_engine** out) {
    DeviceGuard dg;
    if (!out) return set_err(JSP_EINVAL, "out is NULL");
    *out = nullptr;
    int n = 0;
    hipError_t err = hipGetDeviceCount(&n);
    if (err != hipSuccess || n == 0)
        return set_err(JSP_EHIP, "no HIP device available (%s)", hipGetErrorString(err));
    if (device_id < 0 || device_id >= n) return set_err(JSP_EINVAL, "device %d out of range [0,%d)", device_id, n);
    HIP_TRY(hipSetDevice(device_id));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device_id));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return set_err(JSP_EHIP, "device %d is %s; this engine is built for gfx950 (MI355X) only", device_id,
                       prop.gcnArchName);
    auto* e = new (std::nothrow) jsp_engine();
    if (!e) return set_err(JSP_ENOMEM, "engine allocation failed");
    e->device = device_id;
    e->n_cu = prop.multiProcessorCount;
    err = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
    if (err != hipSuccess) {
        delete e;
        return set_err(JSP_EHIP, "hipStreamCreate: %s", hipGetErrorString(err));
    }
    if (hipEventCreateWithFlags(&e->ev_ring[0], hipEventDisableTiming | hipEventReleaseToDevice) != hipSuccess ||
        hipEventCreateWithFlags(&e->ev_ring[1], hipEventDisableTiming | hipEventReleaseToDevice) != hipSuccess) {
        delete e;
        return set_err(JSP_EHIP, "hipEventCreate failed");
    }
    if (e->stats.reserve(16) != hipSuccess || hipMemset(e->stats.p, 0, 16) != hipSuccess) {
        delete e;
        return set_err(JSP_ENOMEM, "stats buffer");
    }
    if (e->h_err.reserve(64) != hipSuccess) {
        delete e;
        return set_err(JSP_ENOMEM, "error word");
    }
    std::memset(e->h_err.p, 0, 64);
    // operational: JSP_SERVICE=0 keeps the resident service off
    if (const char* v = std::getenv("JSP_SERVICE"))
        e->svc_mode = std::strcmp(v, "0") == 0 ? JSP_SERVICE_OFF
                      : std::strcmp(v, "parked") == 0 ? JSP_SERVICE_PARKED : JSP_SERVICE_AUTO;
    e->hooks = read_hooks();
    // test hooks: CUs the service may count on (stands in for a smaller GPU
    // or a partition), the service's first request number (next to 2^30)
    if (e->hooks.cu_limit > 0) e->n_cu = std::min<int>(e->n_cu, e->hooks.cu_limit);
    if (e->hooks.have_seq0) e->svc.seq = e->hooks.seq0;
    *out = e;
    return JSP_OK;
}

int jsp_engine_create_multi(const int* device_ids, int n_devices, jsp_engine** out) {
    DeviceGuard dg;
    if (!out) return set_err(JSP_EINVAL, "out is NULL");
    *out = nullptr;
    jspm::Multi* m = nullptr;
    if (int rc = jspm::create(device_ids, n_devices, &m)) return rc;
    auto* e = new (std::nothrow) jsp_engine();
    if (!e) {
        jspm::destroy(m);
        return set_err(JSP_ENOMEM, "engine allocation failed");
    }
    e->device = jspm::device_of(m);
    e->multi = m;
    *out = e;
    return JSP_OK;
}

int jsp_engine_shards(jsp_engine* e, int* shards, int* devices) {
    if (!e) return set_err(JSP_EINVAL, "engine is NULL");
    if (shards) *shards = e->multi ? jspm::shard_count(e->multi) : 1;
    if (devices) *devices = e->multi ? jspm::n_devices(e->multi) : 1;
    return JSP_OK;
}

void jsp_engine_destroy(jsp_engine* e) {
    if (!e) return;
    DeviceGuard dg;
    if (e->multi) {
        delete e;  // the destructor tears the device set down
        return;
    }
    if (e->waker.joinable()) {  // not under mu: the waker may be waiting for it
        {
            std::lock_guard<std::mutex> l(e->wake_mu);
            e->wake_quit.store(true);
        }
        e->wake_cv.notify_one();
        e->waker.join();
    }
    {
        std::lock_guard<std::mutex> g(e->mu);
        (void)hipSetDevice(e->device);
        e->wake_job = false;
        (void)svc_stop(e);
        if (e->stream) (void)hipStreamSynchronize(e->stream);
    }
    delete e;
}

int jsp_topology_upload(jsp_engine* e, const jsp_topology* t) {
    if (int rc = check_engine(e)) return rc;
    if (e->multi) { DeviceGuard dg; return jspm::topology_upload(e->multi, t); }
    std::lock_guard<std::mutex> g(e->mu);
    if (int rc = svc_suspend(e)) return rc;  // it holds the old buffers and geometry
    if (!t) return set_err(JSP_EINVAL, "topology is NULL");
    // a failed upload leaves the engine without topology (buffers may be gone)
    e->have_topo = e->have_snap = e->have_cls = false;
    const uint32_t K = t->n_levels;
    if (K < 1 || K > JSP_MAX_LEVELS) return set_err(JSP_EINVAL, "n_levels %u out of range [1,%d]", K, JSP_MAX_LEVELS);
    const uint32_t L = t->n_domains[K - 1];
    std::vector<std::vector<uint32_t>> fl(K);
    for (uint32_t k = 0; k < K; ++k) {
        const uint32_t D = t->n_domains[k];
        fl[k].resize(D + 1);
        if (k + 1 == K || t->first_leaf[k] == nullptr) {
            if (k + 1 != K) return set_err(JSP_EINVAL, "first_leaf[%u] is NULL", k);
            for (uint32_t d = 0; d <= D; ++d) fl[k][d] = d;
        } else {
            std::memcpy(fl[k].data(), t->first_leaf[k], sizeof(uint32_t) * (D + 1));
        }
        if (fl[k][0] != 0 || fl[k][D] != L) return set_err(JSP_EINVAL, "first_leaf[%u] must run 0..%u", k, L);
        for (uint32_t d = 0; d < D; ++d)
            if (fl[k][d] > fl[k][d + 1]) return set_err(JSP_EINVAL, "first_leaf[%u] not monotone at %u", k, d);
    }
    for (uint32_t k = 0; k + 1 < K; ++k)
        for (uint32_t d = 0; d <= t->n_domains[k]; ++d)
            if (!std::binary_search(fl[k + 1].begin(), fl[k + 1].end(), fl[k][d]))
                return set_err(JSP_EINVAL, "level %u is not nested in level %u (boundary %u)", k, k + 1, fl[k][d]);
    // taken-bitmap layout in LDS
    uint32_t off = 0;
    for (uint32_t k = 0; k < K; ++k) {
        e->t_off_h[k] = off;
        off += (t->n_domains[k] + 63) / 64;
    }
    e->t_off_h[K] = off;
    if (off > jsp::kMaxTakenWords)
        return set_err(JSP_ERANGE, "topology has %u bitmap words over all levels; engine limit is %u (%u domains)",
                       off, jsp::kMaxTakenWords, jsp::kMaxTakenWords * 64);
    hipStream_t s = e->stream;
    if (int rc = use_engine_stream(e)) return rc;
    jsp::TopoDev td{};
    td.K = K;
    for (uint32_t k = 0; k < K; ++k) {
        td.D[k] = t->n_domains[k];
        HIP_TRY(upload(e->fl[k], fl[k].data(), fl[k].size(), s));
        td.fl[k] = e->fl[k].as<uint32_t>();
        if (k + 1 < K) {  // child_start: level-(k+1) range of each level-k domain
            std::vector<uint32_t> cs(t->n_domains[k] + 1);
            for (uint32_t d = 0; d <= t->n_domains[k]; ++d)
                cs[d] = (uint32_t)(std::lower_bound(fl[k + 1].begin(), fl[k + 1].end(), fl[k][d]) - fl[k + 1].begin());
            HIP_TRY(upload(e->cs[k], cs.data(), cs.size(), s));
            td.cs[k] = e->cs[k].as<uint32_t>();
            e->h_cs[k] = cs;
        }
        if (k > 0) {  // parent at level k-1 of each level-k domain (by its first leaf)
            std::vector<int32_t> par(std::max<uint32_t>(t->n_domains[k], 1));
            for (uint32_t d = 0; d < t->n_domains[k]; ++d)
                par[d] = (int32_t)(std::upper_bound(fl[k - 1].begin(), fl[k - 1].end(), fl[k][d]) - fl[k - 1].begin()) - 1;
            HIP_TRY(upload(e->par[k], par.data(), par.size(), s));
            td.par[k] = e->par[k].as<int32_t>();
            e->h_par[k] = par;
        }
    }
    HIP_TRY(upload(e->t_off, e->t_off_h, K + 1, s));
    HIP_TRY(hipStreamSynchronize(s));
    e->topo = td;
    for (uint32_t k = 0; k < K; ++k) e->h_fl[k] = fl[k];
    e->walk.set_topology(K, t->n_domains, e->h_fl, e->h_cs, e->h_par);
    e->K = K;
    for (uint32_t k = 0; k < JSP_MAX_LEVELS; ++k) e->D[k] = k < K ? t->n_domains[k] : 0;
    e->L_total = L;
    e->have_topo = true;
    e->have_snap = false;  // a snapshot is tied to its topology
    e->have_cls = false;
    return JSP_OK;
}

int jsp_snapshot_upload(jsp_engine* e, const jsp_nodes* nd) {
    if (int rc = check_engine(e)) return rc;
    if (e->multi) { DeviceGuard dg; return jspm::snapshot_upload(e->multi, nd); }
    std::lock_guard<std::mutex> g(e->mu);
    if (int rc = svc_suspend(e)) return rc;  // it holds the old buffers and geometry
    if (!e->have_topo) return set_err(JSP_ESTATE, "upload the topology first");
    if (!nd || !nd->leaf_start) return set_err(JSP_EINVAL, "nodes / leaf_start is NULL");
    e->have_snap = false;  // until every column is resident again
    const uint32_t N = nd->n_nodes, W = nd->n_label_words, R = nd->n_res, NL = nd->n_leaves;
    if (W < 1 || W > JSP_MAX_LABEL_WORDS) return set_err(JSP_EINVAL, "n_label_words %u out of range", W);
    if (R < 1 || R > JSP_MAX_RES) return set_err(JSP_EINVAL, "n_res %u out of range", R);
    if ((uint64_t)nd->leaf_begin + NL > e->L_total)
        return set_err(JSP_EINVAL, "leaves [%u,%u) exceed topology (%u leaves)", nd->leaf_begin,
                       nd->leaf_begin + NL, e->L_total);
    if (N > 0 && (!nd->labels || !nd->taints || !nd->free_res || !nd->excl_owner))
        return set_err(JSP_EINVAL, "a node column is NULL");
    if (N > (1u << 30)) return set_err(JSP_ERANGE, "%u rows exceed the 2^30 row limit", N);
    const uint32_t* ls = nd->leaf_start;
    if (ls[0] != 0 || ls[NL] != N) return set_err(JSP_EINVAL, "leaf_start must run 0..%u", N);
    uint32_t max_rows = 0;
    for (uint32_t l = 0; l < NL; ++l) {
        if (ls[l] > ls[l + 1]) return set_err(JSP_EINVAL, "leaf_start not monotone at %u", l);
        max_rows = std::max(max_rows, ls[l + 1] - ls[l]);
    }
    // workgroup partition: whole leaves, <= 256 leaves each, one 1024-row
    // chunk each (test hooks: more chunks, or smaller row blocks)
    e->hooks = read_hooks();
    const uint32_t chunks = e->hooks.block_chunks;
    uint32_t target_rows = chunks * (uint32_t)jsp::kChunkRows - 4;  // fits even when unaligned
    if (e->hooks.block_rows >= 60 && e->hooks.block_rows < target_rows) target_rows = e->hooks.block_rows;
    std::vector<uint32_t> blk{0};
    {
        uint32_t rows = 0, leaves = 0;
        for (uint32_t l = 0; l < NL; ++l) {
            const uint32_t r = ls[l + 1] - ls[l];
            if (leaves > 0 && (rows + r > target_rows || leaves == (uint32_t)jsp::kMaxBlkLeaves)) {
                blk.push_back(l);
                rows = 0;
                leaves = 0;
            }
            rows += r;
            ++leaves;
        }
        if (NL > 0) blk.push_back(NL);
    }
    const uint32_t npad = ((N + 63) / 64) * 64 + 64;
    hipStream_t s = e->stream;
    if (int rc = use_engine_stream(e)) return rc;
    HIP_TRY(e->labels.reserve((size_t)W * npad * 8));
    HIP_TRY(e->taints.reserve((size_t)npad * 4));
    HIP_TRY(e->freer.reserve((size_t)R * npad * 4));
    HIP_TRY(e->excl.reserve((size_t)npad * 4));
    HIP_TRY(hipMemsetAsync(e->labels.p, 0, (size_t)W * npad * 8, s));
    HIP_TRY(hipMemsetAsync(e->taints.p, 0, (size_t)npad * 4, s));
    HIP_TRY(hipMemsetAsync(e->freer.p, 0, (size_t)R * npad * 4, s));
    HIP_TRY(hipMemsetAsync(e->excl.p, 0xFF, (size_t)npad * 4, s));
    if (N > 0) {
        for (uint32_t w = 0; w < W; ++w)
            HIP_TRY(hipMemcpyAsync(e->labels.as<uint64_t>() + (size_t)w * npad, nd->labels + (size_t)w * N,
                                   (size_t)N * 8, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(e->taints.p, nd->taints, (size_t)N * 4, hipMemcpyHostToDevice, s));
        for (uint32_t r = 0; r < R; ++r)
            HIP_TRY(hipMemcpyAsync(e->freer.as<uint32_t>() + (size_t)r * npad, nd->free_res + (size_t)r * N,
                                   (size_t)N * 4, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(e->excl.p, nd->excl_owner, (size_t)N * 4, hipMemcpyHostToDevice, s));
    }
    HIP_TRY(upload(e->leaf_start, ls, (size_t)NL + 1, s));
    std::vector<uint4> bt(blk.size() > 0 ? blk.size() - 1 : 0);
    uint32_t span = 0;
    for (size_t b = 0; b + 1 < blk.size(); ++b) {
        bt[b] = make_uint4(blk[b], blk[b + 1], ls[blk[b]], ls[blk[b + 1]]);
        span = std::max(span, bt[b].w - (bt[b].z & ~3u));
    }
    e->blk_l0.assign(blk.begin(), blk.end() - (blk.empty() ? 0 : 1));
    e->blk_l1.assign(blk.begin() + (blk.empty() ? 0 : 1), blk.end());
    if (bt.empty()) bt.push_back(make_uint4(0, 0, 0, 0));  // no rows: never read
    HIP_TRY(upload(e->blk, bt.data(), bt.size(), s));
    {
        // wave tiles: up to kWaveTileLeaves whole leaves in <= kWaveTileRows - 4
        // rows (one wave chunk at any row alignment), or one larger leaf alone
        // (none when a leaf is larger than a tile or a column reaches 2^31 bytes:
        // the workgroup tally then runs)
        std::vector<uint4> wt;
        const uint32_t max_rows = (uint32_t)jsp::kWaveTileRows - 4;
        bool ok = (uint64_t)W * npad * 8 < (1ull << 31) && (uint64_t)R * npad * 4 < (1ull << 31) &&
                  (uint64_t)jsp::kMaxClasses * std::max<uint32_t>(e->L_total, 1) * 4 < (1ull << 31);
        for (uint32_t l = 0; l < NL && ok; ++l) ok = ls[l + 1] - ls[l] <= max_rows;
        for (uint32_t l = 0; ok && l < NL;) {
            const uint32_t r0 = ls[l];
            uint32_t end = l;
            while (end < NL && end - l < (uint32_t)jsp::kWaveTileLeaves && ls[end + 1] - r0 <= max_rows) ++end;
            wt.push_back(make_uint4(l, end, r0, ls[end]));
            l = end;
        }
        e->n_wtiles = (uint32_t)wt.size();
        if (wt.empty()) wt.push_back(make_uint4(0, 0, 0, 0));  // never read (n_wtiles == 0)
        HIP_TRY(upload(e->wtiles, wt.data(), wt.size(), s));
    }
    HIP_TRY(e->ticket.reserve(16));
    HIP_TRY(hipMemsetAsync(e->ticket.p, 0, 16, s));  // single-launch tickets (tile draws, finished tiles)
    HIP_TRY(e->granules.reserve(8 * blk.size()));
    HIP_TRY(hipMemsetAsync(e->granules.p, 0, 8 * blk.size(), s));  // look-back granules (epoch 0 never matches)
    HIP_TRY(e->h_done.reserve(4 * blk.size()));
    // the service's inline patch staging, sized for this W/R now: the service
    // is stopped and no patch is pending (svc_suspend), so nothing staged can
    // be lost, and svc_start never reallocates it under a staged patch
    HIP_TRY(e->svc.pstage.reserve(jsp::patch_inline_layout(jsp::kPatchInlineRows, 15u, W, R).bytes));
    HIP_TRY(hipStreamSynchronize(s));
    std::memset(e->h_done.p, 0, 4 * blk.size());  // completion words (epoch 0 never matches)
    e->N = N;
    e->npad = npad;
    e->W = W;
    e->R = R;
    e->leaf_begin = nd->leaf_begin;
    e->n_leaves = NL;
    e->max_leaf_rows = max_rows;
    e->n_blocks = (uint32_t)blk.size() - 1;
    e->max_blk_span = span;
    {
        uint32_t most = 1;
        for (size_t b = 0; b + 1 < blk.size(); ++b) most = std::max(most, blk[b + 1] - blk[b]);
        e->blk_leaves = (most + 3) & ~3u;
    }
    e->tile_draws = e->done_draws = 0;
    e->spin_limit = e->hooks.lookback_spins;
    e->have_snap = true;
    if (e->have_cls) {
        for (auto& c : e->cls_h)
            if ((uint64_t)c.pods * max_rows >= (1ull << 32)) {
                e->have_cls = false;
                return set_err(JSP_ERANGE, "pods x rows per leaf overflows 32-bit tallies; re-upload classes");
            }
    }
    svc_resume(e);
    return JSP_OK;
}

static int snapshot_patch_locked(jsp_engine* e, const uint32_t* rows, uint32_t n, const uint64_t* labels,
                                 const uint32_t* taints, const uint32_t* free_res, const int32_t* excl_owner,
                                 std::chrono::steady_clock::time_point t0);

// The first calls of a recovery run on a host core that slept for hours (or
// for the bench's 60 ms): its caches are gone, and every line a call touches
// would miss in turn -- the engine's fields, the request and answer lines in
// pinned memory, the tables the answer is expanded with. Touched up front by
// independent prefetches their misses overlap instead. (On a warm core: ~100
// prefetches of lines already cached.) Measured on the cold recovery, data
// lines only (tools/warm_ab.py, profiles/r05/probes/warm_ab.txt): cfg2 p50
// 11.0 -> 9.4 us at a 10 ms gap on one box, 16.7 -> 11.8 us at 1 ms on a
// slower-waking one; prefetching the hot code into L2 as well showed no
// consistent gain and is not done.
static inline void warm_lines(const void* p, size_t bytes) {
    const char* c = static_cast<const char*>(p);
    if (!c) return;
    for (size_t i = 0; i < bytes; i += 64) __builtin_prefetch(c + i, 0, 3);
}

static void warm_engine(const jsp_engine* e, bool place) {
    if (!e->hooks.warm) return;
    warm_lines(e, std::min<size_t>(sizeof(jsp_engine), 16384));
    warm_lines(e->svc.box.p, 128);
    warm_lines(e->h_patch_done.p, 128);
    if (place) {
        warm_lines(e->svc.words.p, std::min<size_t>(e->svc.words.bytes, 4096));
        warm_lines(e->svc.bits.p, std::min<size_t>(e->svc.bits.bytes, 8192));
        warm_lines(e->blk_l0.data(), 4 * e->blk_l0.size());
        // the split service's host walk: its bitmaps, sums, taken words and
        // hierarchy tables (a cold core's walk was ~2 us slower, cfg5)
        if (e->svc.shape == 3) e->walk.prefetch_state();
    } else {
        warm_lines(e->h_patch.p, std::min<size_t>(e->h_patch.bytes, 1024));
        warm_lines(e->svc.pstage.p, 256);
    }
}

static int snapshot_patch_call(jsp_engine* e, const uint32_t* rows, uint32_t n, const uint64_t* labels,
                               const uint32_t* taints, const uint32_t* free_res, const int32_t* excl_owner) {
    if (e->multi) { DeviceGuard dg; return jspm::snapshot_patch(e->multi, rows, n, labels, taints, free_res, excl_owner); }
    const auto t0 = std::chrono::steady_clock::now();
    int rc;
    {
        std::lock_guard<std::mutex> g(e->mu);
        warm_engine(e, false);  // under the lock: the waker may be replacing the buffers it touches
        rc = snapshot_patch_locked(e, rows, n, labels, taints, free_res, excl_owner, t0);
    }
    notify_waker(e);
    return rc;
}

int jsp_snapshot_patch(jsp_engine* e, const uint32_t* rows, uint32_t n, const uint64_t* labels,
                       const uint32_t* taints, const uint32_t* free_res, const int32_t* excl_owner) {
    if (int rc = check_engine(e)) return rc;
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = snapshot_patch_call(e, rows, n, labels, taints, free_res, excl_owner);
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    std::lock_guard<std::mutex> l(e->met_mu);
    hist_add(e->met.patch_us, us, JSP_HIST_LO_US);
    if (rc != JSP_OK) e->met.patch_errors += 1;
    return rc;
}

static int snapshot_patch_locked(jsp_engine* e, const uint32_t* rows, uint32_t n, const uint64_t* labels,
                                 const uint32_t* taints, const uint32_t* free_res, const int32_t* excl_owner,
                                 std::chrono::steady_clock::time_point t0) {
    if (!e->have_snap) return set_err(JSP_ESTATE, "no snapshot uploaded");
    if (n == 0) return JSP_OK;
    if (!rows) return set_err(JSP_EINVAL, "rows is NULL");
    for (uint32_t i = 0; i < n; ++i)
        if (rows[i] >= e->N) return set_err(JSP_EINVAL, "row %u out of range (%u rows)", rows[i], e->N);
    run_wake(e);  // an earlier patch's wake still queued: run it (that patch then goes to the service)
    // A patch the service's dispatcher applies is not stream-ordered: device-
    // path work still in flight on a caller's stream (it may be reading the
    // rows) finishes first. (The patch kernel is ordered by the stream.)
    if (e->foreign_pending) {
        HIP_TRY(hipEventSynchronize(e->ev_last));
        e->foreign_pending = false;
    }
    const uint32_t fl = (labels ? jsp::kPatchLab : 0u) | (taints ? jsp::kPatchTaint : 0u) |
                        (free_res ? jsp::kPatchFree : 0u) | (excl_owner ? jsp::kPatchExcl : 0u);
    // A patch small enough to ride in the next request's line, while the
    // service is up: held back (a watch event's few rows; more of the same
    // columns merge into it) and applied by the dispatcher from the request
    // itself -- no staging read, no request of its own. Whatever else reads
    // the rows first posts it alone and waits (patch_wait).
    const bool small = n <= jsp::micro_rows_max(e->W, e->R);
    bool micro = false;
    if (small && e->patch_pending && e->patch_micro && e->patch_deferred && e->micro_fl == fl && svc_up(e))
        micro = micro_merge(e, rows, n, labels, taints, free_res, excl_owner);  // same patch number: not sent yet
    if (!micro) {
        if (int rc = svc_settle(e)) return rc;  // no tile may still be reading the rows of the last request
        if (int rc = patch_wait(e)) return rc;  // the staging buffer is free again
    }
    hipStream_t s = e->stream;
    auto& v = e->svc;
    if (!e->patch_ctr.p) {
        if (int rc = use_engine_stream(e)) return rc;
        HIP_TRY(e->patch_ctr.reserve(64));
        HIP_TRY(hipMemsetAsync(e->patch_ctr.p, 0, 64, s));
    }
    if (!e->h_patch_done.p) {
        HIP_TRY(e->h_patch_done.reserve(128));
        std::memset(e->h_patch_done.p, 0, 128);
    }
    if (!micro && small && svc_up(e)) {
        e->micro_n = 0;
        e->micro_fl = fl;
        micro = micro_merge(e, rows, n, labels, taints, free_res, excl_owner);  // fits: n <= the row capacity
        if (micro) {
            e->patch_seq = e->patch_seq % 0x7FFFFFFFu + 1u;
            e->patch_bits = 0u;  // the request's chunk 1 says it carries micro rows
            e->patch_nf = 0u;
            e->patch_req = 0;
            e->patch_micro = e->patch_pending = e->patch_svc = e->patch_deferred = true;
        }
    }
    if (micro) {
        e->svc.micro_dirty = true;  // the resident tiles' on-chip row copies are stale
        if (int rc = micro_stage_kernel_form(e)) return rc;
        const auto t2 = std::chrono::steady_clock::now();
        e->acc.patches += 1;
        e->acc.patch_us += std::chrono::duration<double, std::micro>(t2 - t0).count();
        return JSP_OK;
    }
    e->patch_micro = false;
    e->svc.rows_dirty = true;  // the resident tiles' on-chip row copies are stale
    // Who applies it: the running service's dispatcher (posted at once; a
    // request that finds it not yet taken carries it again; whatever else
    // reads the rows first waits for it, patch_wait); after the service left,
    // a recovery's first patch restarts it (the waker thread: its grid comes
    // up while the deletions finish) and the dispatcher applies it followed by
    // a warm-up request; otherwise the patch kernel.
    const auto t1 = std::chrono::steady_clock::now();
    const double since = std::chrono::duration<double, std::milli>(t1 - v.last).count();
    const bool up = v.running && since <= 0.5 * idle_ms(e) && svc_ok(e) && svc_shape(e) == v.shape;
    const bool wake = !up && svc_wake_wanted(e);
    // The delta into pinned staging, read in place. Patches for the service
    // of up to kPatchInlineRows rows go to its fixed inline buffer (layout
    // from n and the column flags, which ride in the request; sized for this
    // W/R at snapshot upload); larger ones, and the patch kernel's, to the
    // engine's staging through a descriptor.
    const uint32_t W = e->W, R = e->R;
    const bool inl = (up || wake) && n <= jsp::kPatchInlineRows && v.pstage.p &&
                     jsp::patch_inline_layout(jsp::kPatchInlineRows, 15u, W, R).bytes <= v.pstage.bytes;
    const jsp::PatchInlineLayout L = jsp::patch_inline_layout(n, inl ? fl : 15u, W, R);
    char* hp;
    size_t base = 0;
    if (inl) {
        hp = static_cast<char*>(v.pstage.p);
    } else {
        base = 64;  // the same layout without its header
        HIP_TRY(e->h_patch.reserve(L.bytes, grave(e)));
        hp = static_cast<char*>(e->h_patch.p) - base;
    }
    std::memcpy(hp + L.rows, rows, (size_t)n * 4);
    if (labels) std::memcpy(hp + L.lab, labels, (size_t)W * n * 8);
    if (taints) std::memcpy(hp + L.taint, taints, (size_t)n * 4);
    if (free_res) std::memcpy(hp + L.free, free_res, (size_t)R * n * 4);
    if (excl_owner) std::memcpy(hp + L.excl, excl_owner, (size_t)n * 4);
    e->patch_seq = e->patch_seq % 0x7FFFFFFFu + 1u;
    if (inl) __atomic_store_n(reinterpret_cast<uint32_t*>(hp), e->patch_seq, __ATOMIC_RELAXED);  // header
    jsp::PatchArgs a{};
    a.rows = reinterpret_cast<const uint32_t*>(hp + L.rows);
    a.n = n;
    a.npad = e->npad;
    a.W = W;
    a.R = R;
    a.dlab = labels ? reinterpret_cast<const uint64_t*>(hp + L.lab) : nullptr;
    a.dtaint = taints ? reinterpret_cast<const uint32_t*>(hp + L.taint) : nullptr;
    a.dfree = free_res ? reinterpret_cast<const uint32_t*>(hp + L.free) : nullptr;
    a.dexcl = excl_owner ? reinterpret_cast<const int32_t*>(hp + L.excl) : nullptr;
    a.labels = e->labels.as<uint64_t>();
    a.taints = e->taints.as<uint32_t>();
    a.freer = e->freer.as<uint32_t>();
    a.excl = e->excl.as<int32_t>();
    a.counter = e->patch_ctr.as<unsigned long long>();
    a.done = e->h_patch_done.as<uint32_t>();
    a.seq = e->patch_seq;
    e->last_patch = a;
    e->patch_bits = jsp::kReqPatch | (inl ? jsp::kReqPatchInline : 0u);
    e->patch_req = 0;
    e->patch_nf = inl ? (n | fl << 16) : 0u;
    if (up || wake) {
        if (!inl && v.pdesc.p) *v.pdesc.as<jsp::PatchDesc>() = jsp::PatchDesc{a.rows, a.dlab, a.dtaint, a.dfree, a.dexcl, n, a.seq};
        e->patch_pending = e->patch_svc = true;
    }
    // No wait here: later work is ordered after the patch -- service requests
    // and launches by its completion word (patch_wait / patch_fence), or by
    // the stream for the patch kernel.
    if (up) {
        e->patch_deferred = true;
        patch_post_deferred(e);  // posted now: it lands during the gap before the next request
    } else if (wake) {
        // held back; the waker restarts the service and posts it (run_wake)
        e->patch_deferred = true;
        ring_waker(e);
    } else {
        if (int rc = use_engine_stream(e)) return rc;
        // the patch kernel's workgroups count up to the target (patches the
        // service applied do not touch the counter)
        e->patch_target += (n + 255) / 256;
        a.target = e->patch_target;
        HIP_TRY(jsp::launch_patch(a, s));
        e->patch_pending = true;
        e->patch_svc = false;
        svc_resume(e);
        svc_wake(e);
    }
    const auto t2 = std::chrono::steady_clock::now();
    using us = std::chrono::duration<double, std::micro>;
    e->acc.patches += 1;
    e->acc.patch_us += us(t2 - t0).count();
    if (!wake) e->acc.wake_us += us(t2 - t1).count();  // a wake's own time is counted where it runs
    return JSP_OK;
}

int jsp_classes_upload(jsp_engine* e, const jsp_job_class* classes, uint32_t C) {
    if (int rc = check_engine(e)) return rc;
    if (e->multi) { DeviceGuard dg; return jspm::classes_upload(e->multi, classes, C); }
    std::lock_guard<std::mutex> g(e->mu);
    if (int rc = svc_suspend(e)) return rc;  // it holds the old buffers and geometry
    if (!e->have_topo) return set_err(JSP_ESTATE, "upload the topology first");
    if (C > (uint32_t)jsp::kMaxClasses) return set_err(JSP_ERANGE, "%u classes exceed the limit of %d", C, jsp::kMaxClasses);
    if (C > 0 && !classes) return set_err(JSP_EINVAL, "classes is NULL");
    e->have_cls = false;  // until the new classes are resident
    std::vector<jsp::DevClass> h(std::max<uint32_t>(C, 1));
    std::vector<uint32_t> woff(C + 1, 0);
    for (uint32_t c = 0; c < C; ++c) {
        const jsp_job_class& x = classes[c];
        if (x.level >= e->K) return set_err(JSP_EINVAL, "class %u: level %u >= n_levels %u", c, x.level, e->K);
        if (x.pods < 1) return set_err(JSP_EINVAL, "class %u: pods must be >= 1", c);
        if (x.pods > (1u << 22)) return set_err(JSP_ERANGE, "class %u: pods %u exceed 2^22", c, x.pods);
        if (e->have_snap && (uint64_t)x.pods * e->max_leaf_rows >= (1ull << 32))
            return set_err(JSP_ERANGE, "class %u: pods x rows per leaf overflows 32-bit tallies", c);
        jsp::DevClass& d = h[c];
        std::memset(&d, 0, sizeof d);
        for (int w = 0; w < 4; ++w) {
            d.req[w] = x.req_labels[w];
            d.mask[w] = x.req_labels[w] | x.forbid_labels[w];
        }
        d.tol_inv = ~x.tolerated_taints;
        d.level = x.level;
        d.pods = x.pods;
        for (int r = 0; r < 4; ++r) {
            d.res[r] = x.req_res[r];
            d.rcp[r] = divisor_rcp(x.req_res[r]);
        }
        woff[c + 1] = woff[c] + (e->D[x.level] + 63) / 64;
    }
    hipStream_t s = e->stream;
    if (int rc = use_engine_stream(e)) return rc;
    HIP_TRY(upload(e->cls, h.data(), h.size(), s));
    HIP_TRY(upload(e->word_off, woff.data(), woff.size(), s));
    HIP_TRY(e->feas.reserve((size_t)std::max<uint32_t>(woff[C], 1) * 8));
    // the folded feasibility (fold_ok) never writes the bits past the last leaf
    HIP_TRY(hipMemsetAsync(e->feas.p, 0, (size_t)std::max<uint32_t>(woff[C], 1) * 8, s));
    HIP_TRY(e->cap.reserve((size_t)std::max<uint32_t>(C, 1) * std::max<uint32_t>(e->L_total, 1) * 4));
    HIP_TRY(e->occ.reserve((size_t)std::max<uint32_t>(e->L_total, 1) * 4));
    HIP_TRY(hipStreamSynchronize(s));
    e->cls_h.assign(h.begin(), h.begin() + C);
    e->walk.set_classes(e->cls_h);
    e->C = C;
    e->feas_words = woff[C];
    e->have_cls = true;
    svc_resume(e);
    return JSP_OK;
}

int jsp_tally_device(jsp_engine* e, uint32_t* d_cap, uint32_t* d_occ, uint32_t ld, void* stream) {
    if (int rc = check_engine(e)) return rc;
    if (e->multi) return set_err(JSP_ESTATE, "device-set engine: use jsp_place (the shards tally and combine inside it)");
    std::lock_guard<std::mutex> g(e->mu);
    if (int rc = ready(e, true)) return rc;
    if (!d_occ || (e->C > 0 && !d_cap)) return set_err(JSP_EINVAL, "output buffer is NULL");
    if (ld < e->L_total) return set_err(JSP_EINVAL, "ld %u < total leaves %u", ld, e->L_total);
    if (int rc = check_launch_error(e)) return rc;
    hipStream_t s = pick(e, stream);
    if (int rc = enter_stream(e, s)) return rc;
    const int rc = tally_impl(e, d_cap, d_occ, ld, s);
    if (int lr = leave_stream(e, s)) return lr;
    return rc;
}

int jsp_assign_device(jsp_engine* e, const uint32_t* d_cap, const uint32_t* d_occ, uint32_t ld,
                      const uint32_t* d_run_class, const uint32_t* d_run_len, uint32_t n_runs, uint32_t n_jobs,
                      int32_t* d_assign, void* stream) {
    if (int rc = check_engine(e)) return rc;
    if (e->multi) return set_err(JSP_ESTATE, "device-set engine: use jsp_place");
    std::lock_guard<std::mutex> g(e->mu);
    if (int rc = ready(e, true)) return rc;
    if (ld < e->L_total) return set_err(JSP_EINVAL, "ld %u < total leaves %u", ld, e->L_total);
    if (!d_cap || !d_occ) return set_err(JSP_EINVAL, "tally buffers are NULL");
    if (n_runs > 0 && (!d_run_class || !d_run_len)) return set_err(JSP_EINVAL, "run buffers are NULL");
    if (n_jobs > 0 && !d_assign) return set_err(JSP_EINVAL, "assign buffer is NULL");
    if (int rc = check_launch_error(e)) return rc;
    hipStream_t s = pick(e, stream);
    if (int rc = enter_stream(e, s)) return rc;
    const int rc = assign_impl(e, d_cap, d_occ, ld, d_run_class, d_run_len, n_runs, n_jobs, d_assign, s);
    if (int lr = leave_stream(e, s)) return lr;
    return rc;
}

int jsp_place_device(jsp_engine* e, const uint32_t* d_run_class, const uint32_t* d_run_len, uint32_t n_runs,
                     uint32_t n_jobs, int32_t* d_assign, void* stream) {
    if (int rc = check_engine(e)) return rc;
    if (e->multi) return set_err(JSP_ESTATE, "device-set engine: use jsp_place");
    std::lock_guard<std::mutex> g(e->mu);
    if (int rc = ready(e, true)) return rc;
    if (e->leaf_begin != 0 || e->n_leaves != e->L_total)
        return set_err(JSP_ESTATE, "sharded engine: use jsp_tally_device + all-reduce + jsp_assign_device");
    if (n_runs > 0 && (!d_run_class || !d_run_len)) return set_err(JSP_EINVAL, "run buffers are NULL");
    if (n_jobs > 0 && !d_assign) return set_err(JSP_EINVAL, "assign buffer is NULL");
    if (int rc = check_launch_error(e)) return rc;
    hipStream_t s = pick(e, stream);
    if (int rc = enter_stream(e, s)) return rc;
    const int rc = place_impl(e, d_run_class, d_run_len, n_runs, n_jobs, d_assign, s);
    if (int lr = leave_stream(e, s)) return lr;
    return rc;
}


int jspb_tally_device_timed(jsp_engine* e, uint32_t* d_cap, uint32_t* d_occ, uint32_t ld, uint32_t iters,
                           const void* d_scrub, size_t scrub_bytes, double* out_us) {
    if (int rc = check_engine(e)) return rc;
    if (e->multi) return set_err(JSP_ESTATE, "device-set engine: time its shard engines");
    std::lock_guard<std::mutex> g(e->mu);
    if (int rc = ready(e, true)) return rc;
    if (!d_occ || (e->C > 0 && !d_cap)) return set_err(JSP_EINVAL, "output buffer is NULL");
    if (ld < e->L_total) return set_err(JSP_EINVAL, "ld %u < total leaves %u", ld, e->L_total);
    return time_steps(e, iters, d_scrub, scrub_bytes, out_us,
                      [&](hipStream_t s) { return tally_impl(e, d_cap, d_occ, ld, s); });
}

int jspb_tally_device_spans(jsp_engine* e, uint32_t* d_cap, uint32_t* d_occ, uint32_t ld, uint32_t iters,
                           double* out_us) {
    if (int rc = check_engine(e)) return rc;
    if (e->multi) return set_err(JSP_ESTATE, "device-set engine: time its shard engines");
    std::lock_guard<std::mutex> g(e->mu);
    if (int rc = ready(e, true)) return rc;
    if (!d_occ || (e->C > 0 && !d_cap)) return set_err(JSP_EINVAL, "output buffer is NULL");
    if (ld < e->L_total) return set_err(JSP_EINVAL, "ld %u < total leaves %u", ld, e->L_total);
    if (iters == 0 || iters > 1024) return set_err(JSP_EINVAL, "iters %u out of range [1,1024]", iters);
    if (!out_us) return set_err(JSP_EINVAL, "out_us is NULL");
    if (e->n_wtiles == 0 || e->C < 1 || e->C > 4 || tally_wave_grid(e) != 0 || e->hooks.tally_block)
        return set_err(JSP_ESTATE, "the span probe times the one-tile wave tally; this snapshot runs another shape");
    if (int rc = check_launch_error(e)) return rc;
    hipStream_t s = e->stream;
    if (int rc = use_engine_stream(e)) return rc;
    const size_t per = (size_t)2 * e->n_wtiles;
    DevBuf st;
    HIP_TRY(st.reserve(per * iters * 8));
    for (uint32_t i = 0; i < iters; ++i) {
        jsp::TallyArgs a = tally_args(e, d_cap, d_occ, ld);
        a.wstamps = st.as<unsigned long long>() + per * i;
        HIP_TRY(jsp::launch_tally_wave(a, e->wtiles.as<uint4>(), e->n_wtiles, e->n_leaves, 0, s));
    }
    std::vector<unsigned long long> h(per * iters);
    HIP_TRY(hipMemcpyAsync(h.data(), st.p, per * iters * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    std::vector<double> us(iters);
    double sum = 0.0;
    unsigned long long lo0 = 0, lo_last = 0;
    for (uint32_t i = 0; i < iters; ++i) {
        unsigned long long lo = ~0ull, hi = 0;
        for (size_t k = 0; k < per; k += 2) {
            lo = std::min(lo, h[per * i + k]);
            hi = std::max(hi, h[per * i + k + 1]);
        }
        us[i] = (double)(hi - lo) / 100.0;  // 100 MHz ticks
        sum += us[i];
        if (i == 0) lo0 = lo;
        lo_last = lo;
    }
    std::sort(us.begin(), us.end());
    out_us[0] = us[iters / 2];
    out_us[1] = sum / iters;
    // the launches' period by the kernels' own clock: first wave of launch 0
    // to first wave of the last launch, per launch (execution + the gap the
    // dispatch leaves between back-to-back launches)
    out_us[3] = iters > 1 ? (double)(lo_last - lo0) / 100.0 / (iters - 1) : out_us[1];
    // an empty one-workgroup launch timed by events on its dispatch packet:
    // the fixed cost events add to a kernel's own span
    const uint32_t grid = 1;  // the launch's fixed packet and completion cost (a grid's dispatch overlaps its work)
    std::vector<EvPair> ev(iters);
    for (auto& p : ev) {
        HIP_TRY(hipEventCreate(&p.a));
        HIP_TRY(hipEventCreate(&p.b));
    }
    int rc = JSP_OK;
    for (uint32_t i = 0; i < iters && rc == JSP_OK; ++i) {
        jsp::set_launch_start(ev[i].a);
        jsp::set_launch_stop(ev[i].b);
        if (jsp::launch_empty(grid, s) != hipSuccess) rc = set_err(JSP_EHIP, "empty launch failed");
        jsp::set_launch_start(nullptr);
        jsp::set_launch_stop(nullptr);
    }
    if (rc == JSP_OK && hipStreamSynchronize(s) != hipSuccess) rc = set_err(JSP_EHIP, "empty launches failed");
    std::vector<double> eu(iters, 0.0);
    for (uint32_t i = 0; i < iters && rc == JSP_OK; ++i) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, ev[i].a, ev[i].b) != hipSuccess) rc = set_err(JSP_EHIP, "event time failed");
        eu[i] = ms * 1e3;
    }
    for (auto& p : ev) {
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    if (rc) return rc;
    std::sort(eu.begin(), eu.end());
    out_us[2] = eu[iters / 2];
    return check_launch_error(e);
}

int jspb_place_device_timed(jsp_engine* e, const uint32_t* d_run_class, const uint32_t* d_run_len, uint32_t n_runs,
                           uint32_t n_jobs, int32_t* d_assign, uint32_t iters, const void* d_scrub, size_t scrub_bytes,
                           double* out_us) {
    if (int rc = check_engine(e)) return rc;
    if (e->multi) return set_err(JSP_ESTATE, "device-set engine: use jsp_place");
    std::lock_guard<std::mutex> g(e->mu);
    if (int rc = ready(e, true)) return rc;
    if (e->leaf_begin != 0 || e->n_leaves != e->L_total)
        return set_err(JSP_ESTATE, "sharded engine: use jsp_tally_device + all-reduce + jsp_assign_device");
    if (n_runs > 0 && (!d_run_class || !d_run_len)) return set_err(JSP_EINVAL, "run buffers are NULL");
    if (n_jobs > 0 && !d_assign) return set_err(JSP_EINVAL, "assign buffer is NULL");
    return time_steps(e, iters, d_scrub, scrub_bytes, out_us, [&](hipStream_t s) {
        return place_impl(e, d_run_class, d_run_len, n_runs, n_jobs, d_assign, s);
    });
}

static int place_call(jsp_engine* e, const uint32_t* run_class, const uint32_t* run_len, uint32_t n_runs,
                      int32_t* assign_out, uint32_t* tally_out, uint32_t* occ_out, jsp_stats* stats) {
    if (e->multi) { DeviceGuard dg; return jspm::place(e->multi, run_class, run_len, n_runs, assign_out, tally_out, occ_out, stats); }
    auto t0 = std::chrono::steady_clock::now();
    std::lock_guard<std::mutex> g(e->mu);
    warm_engine(e, true);  // under the lock: the waker may be replacing the buffers it touches
    if (int rc = ready(e, true)) return rc;
    if (e->leaf_begin != 0 || e->n_leaves != e->L_total)
        return set_err(JSP_ESTATE, "sharded engine: use jsp_tally_device + all-reduce + jsp_assign_device");
    if (n_runs > 0 && (!run_class || !run_len)) return set_err(JSP_EINVAL, "run buffers are NULL");
    uint64_t J64 = 0;
    if (int rc = check_runs(e, run_class, run_len, n_runs, &J64)) return rc;
    const uint32_t J = (uint32_t)J64;
    if (J > 0 && !assign_out) return set_err(JSP_EINVAL, "assign_out is NULL");
    if (e->hooks.warm)  // the caller's assign[], written by the answer's expansion: for write, ahead of the wait
        for (size_t i = 0; i < std::min<size_t>((size_t)J * 4, 16384); i += 64)
            __builtin_prefetch(reinterpret_cast<char*>(assign_out) + i, 1, 3);
    const bool want_tally = (tally_out && e->C > 0) || occ_out;
    if (!want_tally && J < jsp::kReqPatchInline && svc_ok(e)) {  // J and the request bits share a word
        const auto t1 = std::chrono::steady_clock::now();
        uint32_t placed = 0;
        const int src = svc_place(e, run_class, run_len, n_runs, J, assign_out, &placed);
        if (src != JSP_OK) {
            // the service could not answer: stop it and answer this call on the
            // launch path. A geometry failure (its grid cannot be co-resident,
            // JSP_ERANGE, or its dispatcher never polled) keeps it off until
            // the next upload; a transient one (it left twice, a look-back
            // timed out) lets the next call start it again.
            (void)svc_stop(e);
            if (src == JSP_ERANGE || e->svc.start_failed) e->svc.broken = true;
            e->svc.start_failed = false;
            e->acc.svc_fallbacks += 1;
            {
                std::lock_guard<std::mutex> l(e->met_mu);
                e->met.svc_fallbacks += 1;
            }
            g_err.clear();  // answered: the call succeeds (jsp_timing.svc_fallbacks counts it)
            goto launch_path;
        }
        {
        const auto t2 = std::chrono::steady_clock::now();
        e->svc.armed = true;
        if (!e->waker_poll.load(std::memory_order_relaxed)) {
            e->waker_poll.store(true, std::memory_order_release);
            notify_waker_poll(e);
        }
        e->last_shape = e->svc.shape == 3 ? 5 : 3;
        if (stats) {
            stats->jobs = J;
            stats->runs = n_runs;
            stats->placed = n_runs > 0 ? placed : 0;
            stats->fused = e->last_shape;
            stats->wall_us = std::chrono::duration<double, std::micro>(t2 - t0).count();
        }
        using us = std::chrono::duration<double, std::micro>;
        e->acc.host_calls += 1;
        e->acc.host_prep_us += us(t1 - t0).count();
        e->acc.host_wait_us += us(t2 - t1).count();
        return JSP_OK;
        }
    }
launch_path:
    hipStream_t s = e->stream;
    if (int rc = check_launch_error(e)) return rc;
    if (int rc = use_engine_stream(e)) return rc;
    // runs in, assign[] and stats out through pinned mapped host memory: one
    // launch sequence, no DMA round trips. The single-launch shapes signal
    // completion through host words (wait_done); the others, and calls that
    // copy the tallies out, synchronise the stream.
    HIP_TRY(e->h_runs.reserve((size_t)std::max<uint32_t>(n_runs, 1) * 8, grave(e)));
    HIP_TRY(e->h_assign.reserve((size_t)std::max<uint32_t>(J, 1) * 4, grave(e)));
    HIP_TRY(e->h_stats.reserve(16));
    uint32_t* h_rc = e->h_runs.as<uint32_t>();
    uint32_t* h_rl = h_rc + std::max<uint32_t>(n_runs, 1);
    if (n_runs > 0) {
        std::memcpy(h_rc, run_class, (size_t)n_runs * 4);
        std::memcpy(h_rl, run_len, (size_t)n_runs * 4);
    }
    e->stats_override = e->h_stats.as<uint32_t>();
    uint32_t n_sig = 0;
    const auto t1 = std::chrono::steady_clock::now();
    const int prc = place_impl(e, h_rc, h_rl, n_runs, J, e->h_assign.as<int32_t>(), s, !want_tally, &n_sig,
                               want_tally, true);
    e->stats_override = nullptr;
    if (prc) return prc;
    const auto t2 = std::chrono::steady_clock::now();
    if (want_tally) {
        if (tally_out && e->C > 0)
            HIP_TRY(hipMemcpyAsync(tally_out, e->cap.p, (size_t)e->C * e->L_total * 4, hipMemcpyDeviceToHost, s));
        if (occ_out) HIP_TRY(hipMemcpyAsync(occ_out, e->occ.p, (size_t)e->L_total * 4, hipMemcpyDeviceToHost, s));
    }
    if (!want_tally && (e->last_shape == 7 || e->last_shape == 8)) {
        // the host walked: assign[] is complete, and nothing the stream still
        // runs writes what the caller reads
    } else if (n_sig > 0) {
        if (int rc = wait_done(e, s, n_sig, e->epoch)) return rc;
    } else {
        HIP_TRY(hipStreamSynchronize(s));
    }
    const auto t3 = std::chrono::steady_clock::now();
    if (J > 0) std::memcpy(assign_out, e->h_assign.p, (size_t)J * 4);
    if (int rc = check_launch_error(e)) return rc;
    uint32_t st[2];
    std::memcpy(st, e->h_stats.p, sizeof st);
    if (stats) {
        stats->jobs = J;
        stats->runs = n_runs > 0 ? st[0] : 0;
        stats->placed = n_runs > 0 ? st[1] : 0;
        stats->fused = e->last_shape;
        stats->wall_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    }
    const auto t4 = std::chrono::steady_clock::now();
    using us = std::chrono::duration<double, std::micro>;
    e->acc.host_calls += 1;
    e->acc.host_prep_us += us(t1 - t0).count();
    e->acc.host_launch_us += us(t2 - t1).count();
    e->acc.host_wait_us += us(t3 - t2).count();
    e->acc.host_post_us += us(t4 - t3).count();
    return JSP_OK;
}

int jsp_place(jsp_engine* e, const uint32_t* run_class, const uint32_t* run_len, uint32_t n_runs,
              int32_t* assign_out, uint32_t* tally_out, uint32_t* occ_out, jsp_stats* stats) {
    if (int rc = check_engine(e)) return rc;
    const auto t0 = std::chrono::steady_clock::now();
    jsp_stats local{};
    jsp_stats* st = stats ? stats : &local;
    const int rc = place_call(e, run_class, run_len, n_runs, assign_out, tally_out, occ_out, st);
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    std::lock_guard<std::mutex> l(e->met_mu);
    hist_add(e->met.place_us, us, JSP_HIST_LO_US);
    if (rc != JSP_OK) {
        e->met.place_errors += 1;
        return rc;
    }
    hist_add(e->met.batch_jobs, (double)st->jobs, JSP_HIST_LO_JOBS);
    e->met.placed += st->placed;
    e->met.unplaceable += st->jobs - st->placed;
    if (st->fused == 3 || st->fused == 5) e->met.svc_calls += 1;
    return rc;
}

int jsp_engine_get_metrics(jsp_engine* e, jsp_metrics* out, int reset) {
    if (!e) return set_err(JSP_EINVAL, "engine is NULL");
    if (!out && !reset) return set_err(JSP_EINVAL, "out is NULL");
    std::lock_guard<std::mutex> l(e->met_mu);
    if (out) *out = e->met;
    if (reset) e->met = jsp_metrics{};
    return JSP_OK;
}

int jspb_place_loop(jsp_engine* e, const uint32_t* run_class, const uint32_t* run_len, uint32_t n_runs,
                   int32_t* assign_out, uint32_t iters, const uint32_t* patch_rows, const uint32_t* patch_taints,
                   uint32_t n_patch, double* out_us) {
    if (int rc = check_engine(e)) return rc;
    if (iters == 0 || iters > 1000000) return set_err(JSP_EINVAL, "iters %u out of range [1,1000000]", iters);
    if (!out_us) return set_err(JSP_EINVAL, "out_us is NULL");
    if (n_patch > 0 && (!patch_rows || !patch_taints)) return set_err(JSP_EINVAL, "patch rows / taints are NULL");
    std::vector<double> us(iters);
    const auto t0 = std::chrono::steady_clock::now();
    auto tp = t0;
    const auto gap = std::chrono::nanoseconds(e->hooks.loop_gap_ns);
    for (uint32_t i = 0; i < iters; ++i) {
        if (gap.count() > 0) {  // test hook: a caller that does other work between calls
            const auto until = std::chrono::steady_clock::now() + gap;
            while (std::chrono::steady_clock::now() < until) __builtin_ia32_pause();
            tp = std::chrono::steady_clock::now();
        }
        if (n_patch > 0) {
            const uint32_t k = i % n_patch;
            if (int rc = jsp_snapshot_patch(e, patch_rows + k, 1, nullptr, patch_taints + k, nullptr, nullptr)) return rc;
        }
        if (int rc = jsp_place(e, run_class, run_len, n_runs, assign_out, nullptr, nullptr, nullptr)) return rc;
        const auto t = std::chrono::steady_clock::now();
        us[i] = std::chrono::duration<double, std::micro>(t - tp).count();
        tp = t;
    }
    out_us[0] = std::chrono::duration<double, std::micro>(tp - t0).count();
    std::sort(us.begin(), us.end());
    out_us[1] = us[iters / 2];
    out_us[2] = us[std::min<size_t>(iters - 1, (size_t)(0.99 * iters))];
    return JSP_OK;
}

// The idle period or gap of jspb_recovery_loop: slept, or spun (a busy caller).
static void recovery_wait(double us, bool spin) {
    if (us <= 0.0) return;
    const auto end = std::chrono::steady_clock::now() + std::chrono::duration<double, std::micro>(us);
    if (!spin) {
        std::this_thread::sleep_until(end);
        return;
    }
    while (std::chrono::steady_clock::now() < end) __builtin_ia32_pause();
}

int jspb_recovery_loop(jsp_engine* e, const uint32_t* run_class, const uint32_t* run_len, uint32_t n_runs,
                      int32_t* assign_out, uint32_t trials, double idle_us, double gap_us, int spin,
                      const uint32_t* patch_rows, const uint32_t* patch_taints, uint32_t n_patch, double* out_us) {
    if (int rc = check_engine(e)) return rc;
    if (trials == 0 || trials > 100000) return set_err(JSP_EINVAL, "trials %u out of range [1,100000]", trials);
    if (!out_us) return set_err(JSP_EINVAL, "out_us is NULL");
    if (!(idle_us >= 0.0 && idle_us <= 1e7 && gap_us >= 0.0 && gap_us <= 1e7))
        return set_err(JSP_EINVAL, "idle / gap out of range [0, 10 s]");
    if (n_patch > 0 && (!patch_rows || !patch_taints)) return set_err(JSP_EINVAL, "patch rows / taints are NULL");
    using clk = std::chrono::steady_clock;
    const auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    for (uint32_t t = 0; t < trials; ++t) {
        recovery_wait(idle_us, spin != 0);
        const uint32_t k = n_patch ? t % n_patch : 0u;
        const auto t0 = clk::now();
        if (n_patch > 0)
            if (int rc = jsp_snapshot_patch(e, patch_rows + k, 1, nullptr, patch_taints + k, nullptr, nullptr)) return rc;
        const auto t1 = clk::now();
        recovery_wait(gap_us, spin != 0);
        const auto t2 = clk::now();
        if (int rc = jsp_place(e, run_class, run_len, n_runs, assign_out, nullptr, nullptr, nullptr)) return rc;
        const auto t3 = clk::now();
        out_us[3 * t] = us(t0, t1);
        out_us[3 * t + 1] = us(t2, t3);
        out_us[3 * t + 2] = us(t1, t2);
    }
    return JSP_OK;
}

int jsp_place_jobs(jsp_engine* e, const uint32_t* job_class, uint32_t n_jobs, int32_t* assign_out,
                   uint32_t* tally_out, uint32_t* occ_out, jsp_stats* stats) {
    if (n_jobs > 0 && !job_class) return set_err(JSP_EINVAL, "job_class is NULL");
    std::vector<uint32_t> rc, rl;
    for (uint32_t j = 0; j < n_jobs; ++j) {
        if (rc.empty() || rc.back() != job_class[j]) {
            rc.push_back(job_class[j]);
            rl.push_back(0);
        }
        ++rl.back();
    }
    return jsp_place(e, rc.data(), rl.data(), (uint32_t)rc.size(), assign_out, tally_out, occ_out, stats);
}

int jsp_resolve_leader_domains(jsp_engine* e, const int32_t* leader_rows, const uint32_t* levels, uint32_t n,
                               int32_t* domain_out) {
    if (int rc = check_engine(e)) return rc;
    if (e->multi) { DeviceGuard dg; return jspm::resolve(e->multi, leader_rows, levels, n, domain_out); }
    std::lock_guard<std::mutex> g(e->mu);
    if (int rc = ready(e, false)) return rc;
    if (n == 0) return JSP_OK;
    if (!leader_rows || !levels || !domain_out) return set_err(JSP_EINVAL, "NULL buffer");
    hipStream_t s = e->stream;
    if (int rc = use_engine_stream(e)) return rc;
    // inputs and output through pinned staging the kernel reads and writes in
    // place: no copy launches (a pageable copy can stall behind the resident
    // service, tools/block_probe.hip)
    HIP_TRY(e->h_batch.reserve((size_t)n * 12, grave(e)));
    int32_t* hr = e->h_batch.as<int32_t>();
    uint32_t* hl = reinterpret_cast<uint32_t*>(hr + n);
    int32_t* ho = hr + 2 * (size_t)n;
    std::memcpy(hr, leader_rows, (size_t)n * 4);
    std::memcpy(hl, levels, (size_t)n * 4);
    HIP_TRY(jsp::launch_resolve(hr, hl, n, e->N, e->leaf_start.as<uint32_t>(), e->n_leaves, e->leaf_begin, e->topo, ho,
                                s));
    HIP_TRY(hipStreamSynchronize(s));
    std::memcpy(domain_out, ho, (size_t)n * 4);
    return JSP_OK;
}

int jsp_audit_placements(jsp_engine* e, const int32_t* leader_rows, const uint32_t* levels,
                         const uint32_t* follower_off, const int32_t* follower_domains, uint32_t n_jobs,
                         uint32_t* bad_out) {
    if (int rc = check_engine(e)) return rc;
    if (e->multi) { DeviceGuard dg; return jspm::audit(e->multi, leader_rows, levels, follower_off, follower_domains, n_jobs, bad_out); }
    std::lock_guard<std::mutex> g(e->mu);
    if (int rc = ready(e, false)) return rc;
    if (n_jobs == 0) return JSP_OK;
    if (!leader_rows || !levels || !follower_off || !bad_out) return set_err(JSP_EINVAL, "NULL buffer");
    const uint32_t M = follower_off[n_jobs];
    if (follower_off[0] != 0) return set_err(JSP_EINVAL, "follower_off[0] must be 0");
    for (uint32_t i = 0; i < n_jobs; ++i)
        if (follower_off[i] > follower_off[i + 1]) return set_err(JSP_EINVAL, "follower_off not monotone at %u", i);
    if (M > 0 && !follower_domains) return set_err(JSP_EINVAL, "follower_domains is NULL");
    hipStream_t s = e->stream;
    if (int rc = use_engine_stream(e)) return rc;
    // pinned staging read and written in place by the kernel (as the resolve)
    const size_t n = n_jobs;
    HIP_TRY(e->h_batch.reserve((n * 4 + 1 + (size_t)M) * 4, grave(e)));
    int32_t* hr = e->h_batch.as<int32_t>();
    uint32_t* hl = reinterpret_cast<uint32_t*>(hr + n);
    uint32_t* hf = hl + n;
    int32_t* hd = reinterpret_cast<int32_t*>(hf + n + 1);
    uint32_t* ho = reinterpret_cast<uint32_t*>(hd + M);
    std::memcpy(hr, leader_rows, n * 4);
    std::memcpy(hl, levels, n * 4);
    std::memcpy(hf, follower_off, (n + 1) * 4);
    if (M > 0) std::memcpy(hd, follower_domains, (size_t)M * 4);
    HIP_TRY(jsp::launch_audit(hr, hl, hf, hd, n_jobs, e->N, e->leaf_start.as<uint32_t>(), e->n_leaves, e->leaf_begin,
                              e->topo, ho, s));
    HIP_TRY(hipStreamSynchronize(s));
    std::memcpy(bad_out, ho, n * 4);
    return JSP_OK;
}

int jspb_set_fused(jsp_engine* e, int mode) {
    if (int rc = check_engine(e)) return rc;
    if (e->multi) { DeviceGuard dg; return jspm::forward(e->multi, 0, mode); }
    std::lock_guard<std::mutex> g(e->mu);
    if (mode != JSP_FUSED_OFF && mode != JSP_FUSED_AUTO) return set_err(JSP_EINVAL, "fused mode %d", mode);
    if (mode != e->fused_mode) {
        if (int rc = svc_stop(e)) return rc;
        e->svc.zero_key = ~0ull;
    }
    e->fused_mode = mode;
    return JSP_OK;
}

int jsp_engine_set_service(jsp_engine* e, int mode) {
    if (int rc = check_engine(e)) return rc;
    if (e->multi) { DeviceGuard dg; return jspm::forward(e->multi, 1, mode); }
    std::lock_guard<std::mutex> g(e->mu);
    if (mode != JSP_SERVICE_OFF && mode != JSP_SERVICE_AUTO && mode != JSP_SERVICE_PARKED)
        return set_err(JSP_EINVAL, "service mode %d", mode);
    if (mode != e->svc_mode) {  // the running service's shape may change
        e->svc.resume = false;
        e->svc.armed = false;
        e->waker_poll.store(false, std::memory_order_release);
        if (int rc = svc_stop(e)) return rc;
        e->svc.zero_key = ~0ull;
    }
    e->svc_mode = mode;
    return JSP_OK;
}

int jspb_service_clock(jsp_engine* e, uint32_t* out, uint32_t cap, uint32_t* n_tiles) {
    if (int rc = check_engine(e)) return rc;
    if (e->multi) { if (n_tiles) *n_tiles = 0; return JSP_OK; }
    std::lock_guard<std::mutex> g(e->mu);
    if (!n_tiles) return set_err(JSP_EINVAL, "n_tiles is NULL");
    *n_tiles = 0;
    const auto& v = e->svc;
    if (!v.clk || !v.words.p) return JSP_OK;
    const uint32_t n = std::min<uint32_t>(cap / jsp::kSvcClkSlots, v.nb);
    if (n > 0 && !out) return set_err(JSP_EINVAL, "out is NULL");
    // the tiles' rows, then (room permitting) the dispatcher's {request seen, bell rung}
    const uint32_t rows = n == v.nb && cap / jsp::kSvcClkSlots > v.nb ? n + 1 : n;
    std::memcpy(out, v.words.as<uint32_t>() + v.nb + 3, (size_t)rows * jsp::kSvcClkSlots * 4);
    *n_tiles = n;
    return JSP_OK;
}

int jsp_engine_service_stop(jsp_engine* e) {
    if (int rc = check_engine(e)) return rc;
    if (e->multi) return JSP_OK;
    std::lock_guard<std::mutex> g(e->mu);
    e->svc.resume = false;
    e->svc.armed = false;  // no patch restarts it until a jsp_place is answered by it again
    e->waker_poll.store(false, std::memory_order_release);
    e->wake_job = false;   // nor a wake still queued (its patch lands through patch_wait)
    return svc_stop(e);
}

}  // extern "C"

// ---- internal entry points of the device-set engine (jsp_multi.h)
bool jspi_fold_ok(jsp_engine* e) {
    std::lock_guard<std::mutex> g(e->mu);
    return e->have_cls && e->have_snap && fold_ok(e, true);
}

uint64_t* jspi_feas(jsp_engine* e, uint32_t* words) {
    std::lock_guard<std::mutex> g(e->mu);
    if (words) *words = e->feas_words;
    return e->feas.as<uint64_t>();
}

int jspi_tally(jsp_engine* e, uint32_t* d_cap, uint32_t* d_occ, uint32_t ld, uint64_t* fold_feas) {
    if (int rc = check_engine(e)) return rc;
    std::lock_guard<std::mutex> g(e->mu);
    if (int rc = ready(e, true)) return rc;
    if (ld < e->L_total) return set_err(JSP_EINVAL, "ld %u < total leaves %u", ld, e->L_total);
    if (fold_feas && !fold_ok(e, true)) return set_err(JSP_ESTATE, "this shard cannot fold its feasibility");
    if (int rc = check_launch_error(e)) return rc;
    if (int rc = enter_stream(e, e->stream)) return rc;
    const int rc = tally_impl(e, d_cap, d_occ, ld, e->stream, fold_feas);
    if (int lr = leave_stream(e, e->stream)) return lr;
    return rc;
}

int jspi_assign(jsp_engine* e, const uint32_t* d_cap, const uint32_t* d_occ, uint32_t ld, const uint32_t* run_class,
                const uint32_t* run_len, uint32_t n_runs, uint32_t J, int32_t* assign, bool folded) {
    if (int rc = check_engine(e)) return rc;
    std::lock_guard<std::mutex> g(e->mu);
    if (int rc = ready(e, true)) return rc;
    if (int rc = check_launch_error(e)) return rc;
    if (int rc = enter_stream(e, e->stream)) return rc;
    const int rc = assign_impl(e, d_cap, d_occ, ld, run_class, run_len, n_runs, J, assign, e->stream, folded, true);
    if (int lr = leave_stream(e, e->stream)) return lr;
    return rc;
}

int jspi_check(jsp_engine* e) {
    std::lock_guard<std::mutex> g(e->mu);
    return check_launch_error(e);
}

extern "C" {

int jspb_link_floor(jsp_engine* e, uint32_t iters, double* out_us) {
    if (int rc = check_engine(e)) return rc;
    if (e->multi) return set_err(JSP_ESTATE, "device-set engine: probe a shard engine");
    std::lock_guard<std::mutex> g(e->mu);
    if (iters == 0 || iters > 100000) return set_err(JSP_EINVAL, "iters %u out of range [1,100000]", iters);
    if (!out_us) return set_err(JSP_EINVAL, "out_us is NULL");
    HostBuf box;
    HIP_TRY(box.reserve(512));
    uint32_t* req = box.as<uint32_t>();
    uint32_t* ack = req + 32;  // four ack words, 64 B apart, on lines of their own
    std::memset(box.p, 0, 512);
    hipStream_t s = e->stream;
    if (int rc = use_engine_stream(e)) return rc;
    const uint32_t warm = std::min<uint32_t>(50, iters);
    const uint32_t n = iters + warm;
    HIP_TRY(jsp::launch_link_probe(req, ack, n, 100000000ull, s));  // a wave waits <= 1 s per request
    auto acked = [&](uint32_t i) {
        for (int w = 0; w < 4; ++w)
            if (__atomic_load_n(ack + 16 * w, __ATOMIC_ACQUIRE) >= i) return true;
        return false;
    };
    std::vector<double> us;
    us.reserve(iters);
    int rc = JSP_OK;
    for (uint32_t i = 1; i <= n && rc == JSP_OK; ++i) {
        const auto t0 = std::chrono::steady_clock::now();
        __atomic_store_n(req, i, __ATOMIC_RELEASE);
        while (!acked(i)) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(500)) {
                rc = set_err(JSP_EHIP, "host-link probe: request %u not answered within 500 ms", i);
                break;
            }
        }
        if (i > warm) us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    if (rc != JSP_OK) __atomic_store_n(req, n, __ATOMIC_RELEASE);  // let every wave finish
    HIP_TRY(hipStreamSynchronize(s));
    if (rc != JSP_OK) return rc;
    std::sort(us.begin(), us.end());
    double sum = 0;
    for (double x : us) sum += x;
    out_us[0] = us[us.size() / 2];
    out_us[1] = us[std::min(us.size() - 1, (size_t)(0.99 * us.size()))];
    out_us[2] = sum / us.size();
    return JSP_OK;
}

int jspb_set_timing(jsp_engine* e, int enable) {
    if (int rc = check_engine(e)) return rc;
    if (e->multi) { DeviceGuard dg; return jspm::forward(e->multi, 2, enable); }
    std::lock_guard<std::mutex> g(e->mu);
    e->timing = enable != 0;
    return JSP_OK;
}

int jspb_get_timing(jsp_engine* e, jsp_timing* out, int reset) {
    if (int rc = check_engine(e)) return rc;
    if (e->multi) { DeviceGuard dg; return jspm::get_timing(e->multi, out, reset); }
    std::lock_guard<std::mutex> g(e->mu);
    if (int rc = resolve_timing(e)) return rc;
    if (out) *out = e->acc;
    if (reset) e->acc = jsp_timing{};
    return JSP_OK;
}

void* jsp_engine_stream(jsp_engine* e) {
    if (e && e->multi) return jspm::stream(e->multi);
    return e ? static_cast<void*>(e->stream) : nullptr;
}

int jsp_engine_sync(jsp_engine* e) {
    if (int rc = check_engine(e)) return rc;
    if (e->multi) { DeviceGuard dg; return jspm::sync(e->multi); }
    std::lock_guard<std::mutex> g(e->mu);
    if (int rc = svc_settle(e)) return rc;  // the service's last request finished on every tile
    if (int rc = patch_wait(e)) return rc;  // and every patch landed
    HIP_TRY(hipStreamSynchronize(e->stream));
    if (e->have_last && e->last_foreign) {
        if (int rc = wait_last_foreign(e)) return rc;
    }
    return JSP_OK;
}

int jsp_engine_check(jsp_engine* e) {
    if (int rc = check_engine(e)) return rc;
    if (e->multi) { DeviceGuard dg; return jspm::check(e->multi); }
    std::lock_guard<std::mutex> g(e->mu);
    // everything enqueued so far is ordered before the last call's work, so
    // waiting for that (an engine-owned event, or the engine stream) suffices
    if (e->have_last) {
        if (e->last_foreign) {
            if (int rc = wait_last_foreign(e)) return rc;
        } else {
            HIP_TRY(hipStreamSynchronize(e->stream));
        }
    }
    return check_launch_error(e);
}

}  // extern "C"
