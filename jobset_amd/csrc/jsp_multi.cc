// jsp_multi.cc — the device-set engine (jsp_multi.h). Built only on the
// public C ABI of the shard engines plus HIP and RCCL: RCCL is loaded at run
// time (dlopen of librccl.so.1, the library torch's own RCCL also answers to)
// when a set spans more than one device, so a single-device build or caller
// never needs it.
#include "jsp_multi.h"

#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "jsp_internal.h"

namespace jspm {

namespace {

// ---- RCCL, resolved at run time (rccl.h types restated: opaque comm, int result,
// ncclInt32 = 2, ncclSum = 0)
typedef struct ncclComm* ncclComm_t;
typedef int (*InitAllFn)(ncclComm_t*, int, const int*);
typedef int (*AllReduceFn)(const void*, void*, size_t, int, int, ncclComm_t, hipStream_t);
typedef int (*GroupFn)();
typedef int (*DestroyFn)(ncclComm_t);
typedef const char* (*ErrStrFn)(int);
constexpr int kNcclInt32 = 2, kNcclUint64 = 5, kNcclSum = 0;

struct Rccl {
    void* so = nullptr;
    InitAllFn init_all = nullptr;
    AllReduceFn all_reduce = nullptr;
    GroupFn group_start = nullptr, group_end = nullptr;
    DestroyFn destroy = nullptr;
    ErrStrFn err = nullptr;
};

// JSP_RCCL_LIB names the library to load instead of the default search (a
// test hook: a name that does not exist stands in for a host without RCCL).
int load_rccl(Rccl* r) {
    if (r->so) return JSP_OK;
    const char* forced = std::getenv("JSP_RCCL_LIB");
    const char* err = nullptr;
    if (forced && forced[0]) {
        r->so = dlopen(forced, RTLD_NOW | RTLD_GLOBAL);
        if (!r->so) err = dlerror();
    } else {
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            r->so = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
            if (r->so) break;
            err = dlerror();
        }
    }
    if (!r->so)
        return jsp_internal_set_err(JSP_EHIP,
                                    "device set spans several GPUs but RCCL (%s) cannot be loaded: %s; a device set "
                                    "over one GPU (repeated ids) needs no RCCL",
                                    forced && forced[0] ? forced : "librccl.so.1", err ? err : "?");
    r->init_all = (InitAllFn)dlsym(r->so, "ncclCommInitAll");
    r->all_reduce = (AllReduceFn)dlsym(r->so, "ncclAllReduce");
    r->group_start = (GroupFn)dlsym(r->so, "ncclGroupStart");
    r->group_end = (GroupFn)dlsym(r->so, "ncclGroupEnd");
    r->destroy = (DestroyFn)dlsym(r->so, "ncclCommDestroy");
    r->err = (ErrStrFn)dlsym(r->so, "ncclGetErrorString");
    if (!r->init_all || !r->all_reduce || !r->group_start || !r->group_end || !r->destroy || !r->err)
        return jsp_internal_set_err(JSP_EHIP, "librccl.so.1 lacks an RCCL entry point");
    return JSP_OK;
}

#define MHIP(expr)                                                                                  \
    do {                                                                                            \
        hipError_t _e = (expr);                                                                     \
        if (_e != hipSuccess)                                                                       \
            return jsp_internal_set_err(JSP_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                                        __FILE__, __LINE__);                                        \
    } while (0)

#define MTRY(expr)                      \
    do {                                \
        int _rc = (expr);               \
        if (_rc != JSP_OK) return _rc;  \
    } while (0)

struct DevMem {
    int dev = 0;
    void* p = nullptr;
    size_t bytes = 0;
    void release() {
        if (p) {
            (void)hipSetDevice(dev);
            (void)hipFree(p);
        }
        p = nullptr;
        bytes = 0;
    }
    hipError_t reserve(int d, size_t n) {
        if (p && dev == d && n <= bytes) return hipSuccess;
        release();
        dev = d;
        hipError_t e = hipSetDevice(d);
        if (e != hipSuccess) return e;
        e = hipMalloc(&p, n ? n : 16);
        if (e == hipSuccess) bytes = n ? n : 16;
        return e;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

// pinned, device-mapped host memory (run lists in, assign[] out: the kernels
// read and write it in place, no copy launches)
struct PinMem {
    void* p = nullptr;
    size_t bytes = 0;
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        bytes = 0;
    }
    hipError_t reserve(size_t n) {
        if (p && n <= bytes) return hipSuccess;
        release();
        hipError_t e = hipHostMalloc(&p, n ? n : 16, hipHostMallocMapped | hipHostMallocCoherent);
        if (e == hipSuccess) bytes = n ? n : 16;
        return e;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

}  // namespace

struct Multi {
    std::mutex mu;
    int n = 0;
    std::vector<int> dev;              // device of each shard
    std::vector<jsp_engine*> sh;       // shard engines
    std::vector<hipEvent_t> ev;        // per shard: its tally enqueued
    // device groups: shards sharing a device; the first shard of a group leads it
    std::vector<int> gdev, glead;      // per group: device, leading shard
    std::vector<int> group_of;         // per shard
    Rccl rccl;
    std::vector<ncclComm_t> comm;      // per group when there are several devices
    // topology (host copy of what the shards hold)
    bool have_topo = false, have_snap = false, have_cls = false;
    uint32_t K = 0, L = 0, C = 0;
    std::vector<uint32_t> fl0;         // level-0 first_leaf
    // snapshot partition
    uint32_t N = 0, W = 0, R = 0;
    std::vector<uint32_t> r0, r1;      // per shard: global row range
    // per group: its shards' [C+1][L] tallies, each shard writing only its own
    // leaf columns (every other column stays zero); with several devices the
    // all-reduce sums them into `sum` (out of place: `red` keeps its zeros)
    std::vector<DevMem> red, sum;
    // folded feasibility (every class at the leaf level, <= 4 classes): per
    // group its shards' bits of the [C][ceil(L/64)] words (zero elsewhere);
    // one device: the assigning engine's own words, no all-reduce
    bool fold = false;
    bool leaf_classes = false;
    std::vector<DevMem> fl_local, fl_sum;
    PinMem h_runs, h_assign;           // run list in, assign[] out (pinned)
};

int reset_buffers(Multi* m);

int create(const int* ids, int n, Multi** out) {
    *out = nullptr;
    if (!ids || n < 1) return jsp_internal_set_err(JSP_EINVAL, "device set is empty");
    if (n > 64) return jsp_internal_set_err(JSP_ERANGE, "%d shards exceed the limit of 64", n);
    auto* m = new (std::nothrow) Multi();
    if (!m) return jsp_internal_set_err(JSP_ENOMEM, "device set allocation failed");
    m->n = n;
    for (int i = 0; i < n; ++i) {
        jsp_engine* e = nullptr;
        if (int rc = jsp_engine_create(ids[i], &e)) {
            destroy(m);
            return rc;
        }
        (void)jsp_engine_set_service(e, JSP_SERVICE_OFF);  // shards are driven through the device path
        m->sh.push_back(e);
        m->dev.push_back(ids[i]);
        hipEvent_t ev = nullptr;
        if (hipSetDevice(ids[i]) != hipSuccess || hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
            destroy(m);
            return jsp_internal_set_err(JSP_EHIP, "event creation on device %d failed", ids[i]);
        }
        m->ev.push_back(ev);
        int g = -1;
        for (size_t k = 0; k < m->gdev.size(); ++k)
            if (m->gdev[k] == ids[i]) g = (int)k;
        if (g < 0) {
            g = (int)m->gdev.size();
            m->gdev.push_back(ids[i]);
            m->glead.push_back(i);
        }
        m->group_of.push_back(g);
    }
    m->red.resize(m->gdev.size());
    m->sum.resize(m->gdev.size());
    m->fl_local.resize(m->gdev.size());
    m->fl_sum.resize(m->gdev.size());
    if (m->gdev.size() > 1) {
        if (int rc = load_rccl(&m->rccl)) {
            destroy(m);
            return rc;
        }
        m->comm.assign(m->gdev.size(), nullptr);
        const int r = m->rccl.init_all(m->comm.data(), (int)m->gdev.size(), m->gdev.data());
        if (r != 0) {
            const char* msg = m->rccl.err(r);
            m->comm.clear();
            destroy(m);
            return jsp_internal_set_err(JSP_EHIP, "ncclCommInitAll over %d devices failed: %s", (int)m->gdev.size(),
                                        msg ? msg : "?");
        }
    }
    *out = m;
    return JSP_OK;
}

void destroy(Multi* m) {
    if (!m) return;
    for (ncclComm_t c : m->comm)
        if (c && m->rccl.destroy) (void)m->rccl.destroy(c);
    for (size_t i = 0; i < m->ev.size(); ++i) {
        (void)hipSetDevice(m->dev[i]);
        (void)hipEventDestroy(m->ev[i]);
    }
    for (auto* v : {&m->red, &m->sum, &m->fl_local, &m->fl_sum})
        for (auto& b : *v) b.release();
    m->h_runs.release();
    m->h_assign.release();
    for (jsp_engine* e : m->sh) jsp_engine_destroy(e);
    delete m;
}

int device_of(const Multi* m) { return m->dev.empty() ? 0 : m->dev[0]; }
int shard_count(const Multi* m) { return m->n; }
int n_devices(const Multi* m) { return (int)m->gdev.size(); }
void* stream(Multi* m) { return m->sh.empty() ? nullptr : jsp_engine_stream(m->sh[0]); }

int topology_upload(Multi* m, const jsp_topology* t) {
    std::lock_guard<std::mutex> g(m->mu);
    m->have_topo = m->have_snap = m->have_cls = false;
    if (!t) return jsp_internal_set_err(JSP_EINVAL, "topology is NULL");
    for (jsp_engine* e : m->sh) MTRY(jsp_topology_upload(e, t));
    m->K = t->n_levels;
    m->L = t->n_domains[m->K - 1];
    const uint32_t D0 = t->n_domains[0];
    m->fl0.resize(D0 + 1);
    if (m->K == 1) {
        for (uint32_t d = 0; d <= D0; ++d) m->fl0[d] = d;
    } else {
        std::memcpy(m->fl0.data(), t->first_leaf[0], sizeof(uint32_t) * (D0 + 1));
    }
    m->have_topo = true;
    return JSP_OK;
}

// Level-0 domains split into n contiguous groups of about equal row count
// (jobset_amd/snapshot.py shard_problem restates the same rule), so every
// domain at every level lives wholly on one shard.
int snapshot_upload(Multi* m, const jsp_nodes* nd) {
    std::lock_guard<std::mutex> g(m->mu);
    if (!m->have_topo) return jsp_internal_set_err(JSP_ESTATE, "upload the topology first");
    if (!nd || !nd->leaf_start) return jsp_internal_set_err(JSP_EINVAL, "nodes / leaf_start is NULL");
    if (nd->leaf_begin != 0 || nd->n_leaves != m->L)
        return jsp_internal_set_err(JSP_EINVAL, "a device-set engine takes the whole snapshot (leaves 0..%u)", m->L);
    m->have_snap = false;
    const uint32_t N = nd->n_nodes, W = nd->n_label_words, R = nd->n_res;
    if (W < 1 || W > JSP_MAX_LABEL_WORDS || R < 1 || R > JSP_MAX_RES)
        return jsp_internal_set_err(JSP_EINVAL, "n_label_words %u / n_res %u out of range", W, R);
    if (N > 0 && (!nd->labels || !nd->taints || !nd->free_res || !nd->excl_owner))
        return jsp_internal_set_err(JSP_EINVAL, "a node column is NULL");
    const uint32_t* ls = nd->leaf_start;
    if (ls[0] != 0 || ls[m->L] != N) return jsp_internal_set_err(JSP_EINVAL, "leaf_start must run 0..%u", N);
    // the cuts and the column slices below index the caller's columns by
    // leaf_start: validate it whole first (as jsp_snapshot_upload does for a
    // single engine), so no slice can wrap or read past a column
    for (uint32_t l = 0; l < m->L; ++l)
        if (ls[l] > ls[l + 1] || ls[l + 1] > N)
            return jsp_internal_set_err(JSP_EINVAL, "leaf_start not monotone at %u", l);
    const uint32_t D0 = (uint32_t)m->fl0.size() - 1;
    std::vector<uint32_t> cuts{0};
    for (int r = 1; r < m->n; ++r) {
        const uint64_t target = (uint64_t)N * (uint64_t)r / (uint64_t)m->n;
        uint32_t i = 0;  // first level-0 boundary whose row offset >= target
        {
            uint32_t lo = 0, hi = D0 + 1;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) / 2;
                if ((uint64_t)ls[m->fl0[mid]] < target) lo = mid + 1;
                else hi = mid;
            }
            i = lo;
        }
        i = std::min(std::max(i, cuts.back()), D0);
        cuts.push_back(i);
    }
    cuts.push_back(D0);
    m->r0.assign(m->n, 0);
    m->r1.assign(m->n, 0);
    for (int s = 0; s < m->n; ++s) {
        const uint32_t l0 = m->fl0[cuts[s]], l1 = m->fl0[cuts[s + 1]];
        const uint32_t a = ls[l0], b = ls[l1], ns = b - a;
        std::vector<uint32_t> sls(l1 - l0 + 1);
        for (uint32_t l = l0; l <= l1; ++l) sls[l - l0] = ls[l] - a;
        std::vector<uint64_t> lab((size_t)W * ns);
        std::vector<uint32_t> fr((size_t)R * ns);
        for (uint32_t w = 0; w < W; ++w)
            if (ns) std::memcpy(lab.data() + (size_t)w * ns, nd->labels + (size_t)w * N + a, (size_t)ns * 8);
        for (uint32_t r = 0; r < R; ++r)
            if (ns) std::memcpy(fr.data() + (size_t)r * ns, nd->free_res + (size_t)r * N + a, (size_t)ns * 4);
        jsp_nodes v{};
        v.n_nodes = ns;
        v.leaf_begin = l0;
        v.n_leaves = l1 - l0;
        v.leaf_start = sls.data();
        v.n_label_words = W;
        v.labels = lab.data();
        v.taints = ns ? nd->taints + a : nullptr;
        v.n_res = R;
        v.free_res = fr.data();
        v.excl_owner = ns ? nd->excl_owner + a : nullptr;
        MTRY(jsp_snapshot_upload(m->sh[s], &v));
        m->r0[s] = a;
        m->r1[s] = b;
    }
    m->N = N;
    m->W = W;
    m->R = R;
    m->have_snap = true;
    if (m->have_cls) MTRY(reset_buffers(m));  // new leaf columns per shard
    return JSP_OK;
}

// The per-group buffers for the current snapshot and classes, zeroed: every
// shard rewrites only its own columns and feasibility bits, so the others
// stay zero from here on. The fold is on when every shard can fold.
int reset_buffers(Multi* m) {
    const size_t words = (size_t)(m->C + 1) * std::max<uint32_t>(m->L, 1);
    m->fold = m->leaf_classes;
    for (jsp_engine* e : m->sh) m->fold = m->fold && jspi_fold_ok(e);
    uint32_t fw = 0;
    uint64_t* f0 = jspi_feas(m->sh[0], &fw);
    const bool multi = m->gdev.size() > 1;
    for (size_t k = 0; k < m->gdev.size(); ++k) {
        MHIP(m->red[k].reserve(m->gdev[k], words * 4));
        MHIP(hipMemset(m->red[k].p, 0, words * 4));
        if (multi) MHIP(m->sum[k].reserve(m->gdev[k], words * 4));
        if (m->fold && multi) {
            MHIP(m->fl_local[k].reserve(m->gdev[k], (size_t)std::max<uint32_t>(fw, 1) * 8));
            MHIP(hipMemset(m->fl_local[k].p, 0, m->fl_local[k].bytes));
            if (k != (size_t)m->group_of[0]) MHIP(m->fl_sum[k].reserve(m->gdev[k], (size_t)std::max<uint32_t>(fw, 1) * 8));
        }
    }
    if (m->fold && !multi) {  // the shards fold straight into the assigning engine's words
        MHIP(hipSetDevice(m->dev[0]));
        MHIP(hipMemset(f0, 0, (size_t)std::max<uint32_t>(fw, 1) * 8));
    }
    return JSP_OK;  // hipMemset returns once the bytes are set (no device-wide wait: a resident service runs)
}

// the shard holding global row `row` (r0 ascending; empty shards skipped)
int shard_of(const Multi* m, uint32_t row) {
    int s = (int)(std::upper_bound(m->r0.begin(), m->r0.end(), row) - m->r0.begin()) - 1;
    while (s >= 0 && !(row >= m->r0[s] && row < m->r1[s])) --s;
    return s;
}

int snapshot_patch(Multi* m, const uint32_t* rows, uint32_t n, const uint64_t* labels, const uint32_t* taints,
                   const uint32_t* free_res, const int32_t* excl_owner) {
    std::lock_guard<std::mutex> g(m->mu);
    if (!m->have_snap) return jsp_internal_set_err(JSP_ESTATE, "no snapshot uploaded");
    if (n == 0) return JSP_OK;
    if (!rows) return jsp_internal_set_err(JSP_EINVAL, "rows is NULL");
    std::vector<std::vector<uint32_t>> idx(m->n);
    for (uint32_t i = 0; i < n; ++i) {
        if (rows[i] >= m->N) return jsp_internal_set_err(JSP_EINVAL, "row %u out of range (%u rows)", rows[i], m->N);
        idx[shard_of(m, rows[i])].push_back(i);
    }
    for (int s = 0; s < m->n; ++s) {
        const auto& id = idx[s];
        const uint32_t k = (uint32_t)id.size();
        if (k == 0) continue;
        std::vector<uint32_t> lr(k), t(k), f((size_t)m->R * k);
        std::vector<uint64_t> lab((size_t)m->W * k);
        std::vector<int32_t> ex(k);
        for (uint32_t j = 0; j < k; ++j) {
            const uint32_t i = id[j];
            lr[j] = rows[i] - m->r0[s];
            if (labels)
                for (uint32_t w = 0; w < m->W; ++w) lab[(size_t)w * k + j] = labels[(size_t)w * n + i];
            if (taints) t[j] = taints[i];
            if (free_res)
                for (uint32_t r = 0; r < m->R; ++r) f[(size_t)r * k + j] = free_res[(size_t)r * n + i];
            if (excl_owner) ex[j] = excl_owner[i];
        }
        MTRY(jsp_snapshot_patch(m->sh[s], lr.data(), k, labels ? lab.data() : nullptr, taints ? t.data() : nullptr,
                                free_res ? f.data() : nullptr, excl_owner ? ex.data() : nullptr));
    }
    return JSP_OK;
}

int classes_upload(Multi* m, const jsp_job_class* classes, uint32_t C) {
    std::lock_guard<std::mutex> g(m->mu);
    m->have_cls = false;
    for (jsp_engine* e : m->sh) MTRY(jsp_classes_upload(e, classes, C));
    m->C = C;
    m->leaf_classes = C >= 1;
    for (uint32_t c = 0; c < C; ++c) m->leaf_classes &= classes[c].level + 1 == m->K;
    m->have_cls = true;
    if (m->have_snap) MTRY(reset_buffers(m));
    return JSP_OK;
}

int place(Multi* m, const uint32_t* run_class, const uint32_t* run_len, uint32_t n_runs, int32_t* assign_out,
          uint32_t* tally_out, uint32_t* occ_out, jsp_stats* stats) {
    const auto t0 = std::chrono::steady_clock::now();
    std::lock_guard<std::mutex> g(m->mu);
    if (!m->have_topo || !m->have_snap || !m->have_cls)
        return jsp_internal_set_err(JSP_ESTATE, "device set: topology, snapshot and classes must be uploaded");
    if (n_runs > 0 && (!run_class || !run_len)) return jsp_internal_set_err(JSP_EINVAL, "run buffers are NULL");
    uint64_t J64 = 0;
    for (uint32_t i = 0; i < n_runs; ++i) {
        if (run_class[i] >= m->C)
            return jsp_internal_set_err(JSP_EINVAL, "run %u: class %u out of range (%u classes)", i, run_class[i], m->C);
        J64 += run_len[i];
    }
    if (J64 > (1u << 30)) return jsp_internal_set_err(JSP_ERANGE, "%llu jobs exceed the 2^30 limit", (unsigned long long)J64);
    const uint32_t J = (uint32_t)J64;
    if (J > 0 && !assign_out) return jsp_internal_set_err(JSP_EINVAL, "assign_out is NULL");
    const uint32_t L = m->L, C = m->C;
    const size_t words = (size_t)(C + 1) * L;
    const bool multi = m->gdev.size() > 1;
    const int g0 = m->group_of[0];
    uint32_t fw = 0;
    uint64_t* f0 = jspi_feas(m->sh[0], &fw);
    // 1. every shard tallies straight into its device's buffer (its own leaf
    //    columns) on its own stream -- shards of one device run side by side
    //    -- folding its leaves' feasibility bits when every class is a leaf class
    for (int s = 0; s < m->n; ++s) {
        const int k = m->group_of[s];
        uint32_t* b = m->red[k].as<uint32_t>();
        uint64_t* fb = !m->fold ? nullptr : multi ? m->fl_local[k].as<uint64_t>() : f0;
        MTRY(jspi_tally(m->sh[s], b, b + (size_t)C * L, L, fb));
    }
    // 2. per device: the group's leader waits for its other shards (an event each)
    for (int s = 0; s < m->n; ++s) {
        const int lead = m->glead[m->group_of[s]];
        if (s == lead) continue;
        MHIP(hipSetDevice(m->dev[s]));
        MHIP(hipEventRecord(m->ev[s], static_cast<hipStream_t>(jsp_engine_stream(m->sh[s]))));
        MHIP(hipStreamWaitEvent(static_cast<hipStream_t>(jsp_engine_stream(m->sh[lead])), m->ev[s], 0));
    }
    // 3. between devices: one group of SUM all-reduces over RCCL, out of place
    //    (each device's own buffers keep their zeros): the tallies, and the
    //    folded feasibility words (disjoint bits: their sum is their OR) into
    //    the assigning engine's words
    const uint32_t* tallies = m->red[g0].as<uint32_t>();
    if (multi) {
        if (m->rccl.group_start() != 0) return jsp_internal_set_err(JSP_EHIP, "ncclGroupStart failed");
        for (size_t k = 0; k < m->gdev.size(); ++k) {
            MHIP(hipSetDevice(m->gdev[k]));
            hipStream_t ls = static_cast<hipStream_t>(jsp_engine_stream(m->sh[m->glead[k]]));
            int r = m->rccl.all_reduce(m->red[k].p, m->sum[k].p, words, kNcclInt32, kNcclSum, m->comm[k], ls);
            if (r == 0 && m->fold)
                r = m->rccl.all_reduce(m->fl_local[k].p, (int)k == g0 ? (void*)f0 : m->fl_sum[k].p, fw, kNcclUint64,
                                       kNcclSum, m->comm[k], ls);
            if (r != 0) {
                (void)m->rccl.group_end();
                return jsp_internal_set_err(JSP_EHIP, "ncclAllReduce failed: %s", m->rccl.err(r));
            }
        }
        const int r = m->rccl.group_end();
        if (r != 0) return jsp_internal_set_err(JSP_EHIP, "ncclGroupEnd failed: %s", m->rccl.err(r));
        tallies = m->sum[g0].as<uint32_t>();
    }
    // 4. the assignment on shard 0 (the leader of its device group): the run
    //    list read and assign[] written in pinned memory by the kernels
    jsp_engine* e0 = m->sh[0];
    hipStream_t s0 = static_cast<hipStream_t>(jsp_engine_stream(e0));
    MHIP(m->h_runs.reserve((size_t)std::max<uint32_t>(n_runs, 1) * 8));
    MHIP(m->h_assign.reserve((size_t)std::max<uint32_t>(J, 1) * 4));
    uint32_t* hr = m->h_runs.as<uint32_t>();
    if (n_runs > 0) {
        std::memcpy(hr, run_class, (size_t)n_runs * 4);
        std::memcpy(hr + n_runs, run_len, (size_t)n_runs * 4);
    }
    MTRY(jspi_assign(e0, tallies, tallies + (size_t)C * L, L, hr, hr + n_runs, n_runs, J, m->h_assign.as<int32_t>(),
                     m->fold));
    MHIP(hipSetDevice(m->dev[0]));
    if (tally_out && C > 0) MHIP(hipMemcpyAsync(tally_out, tallies, (size_t)C * L * 4, hipMemcpyDeviceToHost, s0));
    if (occ_out) MHIP(hipMemcpyAsync(occ_out, tallies + (size_t)C * L, (size_t)L * 4, hipMemcpyDeviceToHost, s0));
    // everything above is ordered before this stream's end (events, the
    // all-reduce group on the leaders' streams): one wait, then every shard's
    // error word without another synchronisation
    MHIP(hipStreamSynchronize(s0));
    if (J > 0) std::memcpy(assign_out, m->h_assign.p, (size_t)J * 4);
    for (int s = 0; s < m->n; ++s) MTRY(jspi_check(m->sh[s]));
    if (stats) {
        uint32_t placed = 0;
        for (uint32_t j = 0; j < J; ++j) placed += assign_out[j] >= 0;
        stats->jobs = J;
        stats->placed = placed;
        stats->runs = n_runs;
        stats->fused = 6;
        stats->wall_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    }
    return JSP_OK;
}

int resolve(Multi* m, const int32_t* rows, const uint32_t* levels, uint32_t n, int32_t* out) {
    std::lock_guard<std::mutex> g(m->mu);
    if (!m->have_topo || !m->have_snap) return jsp_internal_set_err(JSP_ESTATE, "no snapshot uploaded");
    if (n == 0) return JSP_OK;
    if (!rows || !levels || !out) return jsp_internal_set_err(JSP_EINVAL, "NULL buffer");
    std::vector<std::vector<uint32_t>> idx(m->n);
    for (uint32_t i = 0; i < n; ++i) {
        out[i] = -1;
        if (rows[i] >= 0 && (uint32_t)rows[i] < m->N) idx[shard_of(m, (uint32_t)rows[i])].push_back(i);
    }
    for (int s = 0; s < m->n; ++s) {
        const uint32_t k = (uint32_t)idx[s].size();
        if (!k) continue;
        std::vector<int32_t> lr(k), o(k);
        std::vector<uint32_t> lv(k);
        for (uint32_t j = 0; j < k; ++j) {
            lr[j] = rows[idx[s][j]] - (int32_t)m->r0[s];
            lv[j] = levels[idx[s][j]];
        }
        MTRY(jsp_resolve_leader_domains(m->sh[s], lr.data(), lv.data(), k, o.data()));
        for (uint32_t j = 0; j < k; ++j) out[idx[s][j]] = o[j];
    }
    return JSP_OK;
}

int audit(Multi* m, const int32_t* leader_rows, const uint32_t* levels, const uint32_t* foff, const int32_t* fdom,
          uint32_t n_jobs, uint32_t* bad) {
    std::lock_guard<std::mutex> g(m->mu);
    if (!m->have_topo || !m->have_snap) return jsp_internal_set_err(JSP_ESTATE, "no snapshot uploaded");
    if (n_jobs == 0) return JSP_OK;
    if (!leader_rows || !levels || !foff || !bad) return jsp_internal_set_err(JSP_EINVAL, "NULL buffer");
    if (foff[0] != 0) return jsp_internal_set_err(JSP_EINVAL, "follower_off[0] must be 0");
    for (uint32_t i = 0; i < n_jobs; ++i)
        if (foff[i] > foff[i + 1]) return jsp_internal_set_err(JSP_EINVAL, "follower_off not monotone at %u", i);
    if (foff[n_jobs] > 0 && !fdom) return jsp_internal_set_err(JSP_EINVAL, "follower_domains is NULL");
    std::vector<std::vector<uint32_t>> idx(m->n);
    for (uint32_t i = 0; i < n_jobs; ++i) {
        bad[i] = 0xFFFFFFFFu;  // leader node unknown
        if (leader_rows[i] >= 0 && (uint32_t)leader_rows[i] < m->N)
            idx[shard_of(m, (uint32_t)leader_rows[i])].push_back(i);
    }
    for (int s = 0; s < m->n; ++s) {
        const uint32_t k = (uint32_t)idx[s].size();
        if (!k) continue;
        std::vector<int32_t> lr(k), fd;
        std::vector<uint32_t> lv(k), off(k + 1, 0), o(k);
        for (uint32_t j = 0; j < k; ++j) {
            const uint32_t i = idx[s][j];
            lr[j] = leader_rows[i] - (int32_t)m->r0[s];
            lv[j] = levels[i];
            fd.insert(fd.end(), fdom + foff[i], fdom + foff[i + 1]);
            off[j + 1] = (uint32_t)fd.size();
        }
        MTRY(jsp_audit_placements(m->sh[s], lr.data(), lv.data(), off.data(), fd.empty() ? nullptr : fd.data(), k,
                                  o.data()));
        for (uint32_t j = 0; j < k; ++j) bad[idx[s][j]] = o[j];
    }
    return JSP_OK;
}

int forward(Multi* m, int what, int value) {
    std::lock_guard<std::mutex> g(m->mu);
    for (jsp_engine* e : m->sh) {
        if (what == 0) MTRY(jspb_set_fused(e, value));
        else if (what == 1) MTRY(jsp_engine_set_service(e, JSP_SERVICE_OFF));  // shards stay on the device path
        else MTRY(jspb_set_timing(e, value));
    }
    return JSP_OK;
}

int sync(Multi* m) {
    std::lock_guard<std::mutex> g(m->mu);
    for (jsp_engine* e : m->sh) MTRY(jsp_engine_sync(e));
    return JSP_OK;
}

int check(Multi* m) {
    std::lock_guard<std::mutex> g(m->mu);
    for (jsp_engine* e : m->sh) MTRY(jsp_engine_check(e));
    return JSP_OK;
}

int get_timing(Multi* m, jsp_timing* out, int reset) {
    std::lock_guard<std::mutex> g(m->mu);
    jsp_timing sum{};
    for (jsp_engine* e : m->sh) {
        jsp_timing t{};
        MTRY(jspb_get_timing(e, &t, reset));
        sum.calls += t.calls;
        sum.tally_ms += t.tally_ms;
        sum.feas_ms += t.feas_ms;
        sum.assign_ms += t.assign_ms;
        sum.fused_ms += t.fused_ms;
        sum.fused_calls += t.fused_calls;
    }
    if (out) *out = sum;
    return JSP_OK;
}

}  // namespace jspm
