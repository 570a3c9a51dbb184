// jsp_walk.cc — host half of the split placement service (jsp_walk.h).
//
// Feasibility: a leaf-level class's domain (leaf) is feasible
// when its capacity covers the job's pods and no foreign exclusive job covers
// one of its rows: the tiles' ballots give the first, the group-0 tiles'
// occupancy ballots the second. An upper-level class's domain is feasible
// when the sum over its leaves of min(cap, pods) reaches pods (the tiles'
// clamped partial sums per domain, added here) and none of its leaves is
// occupied. The walk is the lowest-index rule of oracle/cpu_ref.c: jobs in
// global order, each takes the lowest feasible domain at its class's level
// not yet taken; taking a domain takes its ancestors and descendants.
#include "jsp_walk.h"

#include <algorithm>
#include <chrono>
#include <cstring>

namespace jsp {

namespace {

inline void set_range(uint64_t* t, uint32_t lo, uint32_t hi) {
    while (lo < hi) {
        const uint32_t w = lo >> 6, b = lo & 63u;
        const uint32_t n = (hi - lo) < (64u - b) ? (hi - lo) : (64u - b);
        t[w] |= (n == 64u) ? ~0ull : (((1ull << n) - 1ull) << b);
        lo += n;
    }
}

// any bit of g in [lo, hi)
inline bool any_bits(const uint64_t* g, uint32_t lo, uint32_t hi) {
    while (lo < hi) {
        const uint32_t w = lo >> 6, b = lo & 63u;
        const uint32_t n = (hi - lo) < (64u - b) ? (hi - lo) : (64u - b);
        const uint64_t m = (n == 64u) ? ~0ull : (((1ull << n) - 1ull) << b);
        if (g[w] & m) return true;
        lo += n;
    }
    return false;
}

}  // namespace

void HostWalk::set_topology(uint32_t K, const uint32_t* D, const std::vector<uint32_t>* fl,
                            const std::vector<uint32_t>* cs, const std::vector<int32_t>* par) {
    K_ = K;
    uint32_t off = 0;
    toff_.assign(K + 1, 0);
    for (uint32_t k = 0; k < kMaxLevels; ++k) {
        D_[k] = k < K ? D[k] : 0;
        fl_[k] = k < K ? fl[k] : std::vector<uint32_t>();
        cs_[k] = k + 1 < K ? cs[k] : std::vector<uint32_t>();
        par_[k] = k >= 1 && k < K ? par[k] : std::vector<int32_t>();
        if (k < K) {
            toff_[k] = off;
            off += (D_[k] + 63) / 64;
        }
    }
    toff_[K] = off;
    L_ = D_[K - 1];
    taken_.assign(off + 1, 0);
    occ_lvl_.assign(off + 1, 0);
    occ_.assign((L_ + 63) / 64 + 1, 0);
}

void HostWalk::set_classes(const std::vector<DevClass>& cls) {
    C_ = (uint32_t)cls.size();
    level_.resize(C_);
    pods_.resize(C_);
    woff_.assign(C_ + 1, 0);
    uoff_.assign(C_ + 1, 0);
    any_upper_ = false;
    for (uint32_t c = 0; c < C_; ++c) {
        level_[c] = cls[c].level;
        pods_[c] = cls[c].pods;
        const uint32_t D = D_[level_[c]];
        woff_[c + 1] = woff_[c] + (D + 63) / 64;
        const bool upper = level_[c] + 1 < K_;
        uoff_[c + 1] = uoff_[c] + (upper ? D : 0u);
        any_upper_ |= upper;
    }
    feas_.assign(woff_[C_] + 1, 0);
    sums_.assign(uoff_[C_] + 1, 0);
    cw_.assign(C_, ClassWalk{});
}

void HostWalk::set_tiles(const std::vector<uint32_t>& blk_l0, const std::vector<uint32_t>& blk_l1, uint32_t groups,
                         uint32_t cpg) {
    l0_ = blk_l0;
    l1_ = blk_l1;
    groups_ = groups;
    cpg_ = cpg;
    nw_ = split_waves(blk_l0, blk_l1);
}

uint32_t split_waves(const std::vector<uint32_t>& blk_l0, const std::vector<uint32_t>& blk_l1) {
    uint32_t m = 1;
    for (size_t b = 0; b < blk_l0.size() && b < blk_l1.size(); ++b) m = std::max(m, blk_l1[b] - blk_l0[b]);
    return std::min<uint32_t>((m + 63) / 64, 4u);
}

void HostWalk::prefetch_tile(const uint64_t* slots, uint32_t t) const {
    const uint32_t b = t / groups_;
    if (b >= l0_.size()) return;
    const uint64_t* s = slots + (size_t)t * split_tile_words(cpg_, nw_);
    const uint32_t n_line = split_line_words(cpg_, nw_);
    for (uint32_t i = 0; i < n_line; i += 8) __builtin_prefetch(s + i, 0, 3);
    if (!any_upper_) return;
    const uint32_t nl = l1_[b] - l0_[b], g = t % groups_;
    for (uint32_t j = 0; j < cpg_; ++j) {
        const uint32_t c = g * cpg_ + j;
        if (c >= C_ || level_[c] + 1 == K_) continue;
        for (uint32_t w = 0; 64 * w < nl; ++w)
            __builtin_prefetch(s + n_line + ((size_t)j * nw_ + w) * kSplitRecs, 0, 3);
    }
}

bool HostWalk::tile_ready(const uint64_t* slots, uint32_t t, uint32_t seq) const {
    const uint64_t* s = slots + (size_t)t * split_tile_words(cpg_, nw_);
    const uint32_t n_line = split_line_words(cpg_, nw_);
    uint32_t bad = 0;
    for (uint32_t i = 0; i < n_line; ++i) bad |= (uint32_t)(__atomic_load_n(s + i, __ATOMIC_ACQUIRE) >> 32) ^ seq;
    if (bad) return false;
    if (!any_upper_) return true;
    const uint32_t b = t / groups_, g = t % groups_;
    const uint32_t nl = l1_[b] - l0_[b];
    const uint64_t rtag = split_rec_tag(seq);
    for (uint32_t j = 0; j < cpg_; ++j) {
        const uint32_t c = g * cpg_ + j;
        if (c >= C_ || level_[c] + 1 == K_) continue;
        for (uint32_t w = 0; 64 * w < nl; ++w) {
            const uint32_t n = std::min<uint32_t>((uint32_t)s[2 * (j * nw_ + w)], kSplitRecs);
            const uint64_t* r = s + n_line + ((size_t)j * nw_ + w) * kSplitRecs;
            for (uint32_t i = 0; i < n; ++i)
                if ((__atomic_load_n(r + i, __ATOMIC_ACQUIRE) >> 50) != rtag) return false;
        }
    }
    return true;
}

// A ballot word of a tile's lines: class slot j, wave w's halves (the low 32
// bits of entries 2 (j nw + w) and + 1).
static inline uint64_t line_word(const uint64_t* lines, uint32_t nw, uint32_t j, uint32_t w) {
    const uint64_t* p = lines + 2 * (j * nw + w);
    return (p[0] & 0xFFFFFFFFull) | (p[1] << 32);
}

// Bitmap words built from 64-bit pieces at nondecreasing bit positions (the
// tiles' ballots, in leaf order) into a zeroed bitmap: the two words a piece
// touches are kept in registers and written once they are passed, instead of
// a read-modify-write per piece (cfg3's 80 tiles: a store-to-load chain).
struct BitAppender {
    uint64_t* g;
    uint32_t w = 0;
    uint64_t a0 = 0, a1 = 0;
    explicit BitAppender(uint64_t* g_) : g(g_) {}
    inline void add(uint32_t pos, uint64_t x) {
        const uint32_t pw = pos >> 6, b = pos & 63u;
        if (pw != w) {
            g[w] |= a0;
            if (pw == w + 1) {
                a0 = a1;
            } else {
                g[w + 1] |= a1;
                a0 = 0;
            }
            a1 = 0;
            w = pw;
        }
        a0 |= x << b;
        if (b != 0) a1 |= x >> (64u - b);
    }
    inline void flush() {
        g[w] |= a0;
        g[w + 1] |= a1;
    }
};

void HostWalk::build_feasibility(const uint64_t* slots) {
    const size_t tile_words = split_tile_words(cpg_, nw_);
    const uint32_t n_line = split_line_words(cpg_, nw_);
    const uint32_t nb = (uint32_t)l0_.size();
    // occupied leaves, from the group-0 tiles
    std::fill(occ_.begin(), occ_.end(), 0ull);
    {
        BitAppender ap(occ_.data());
        for (uint32_t b = 0; b < nb; ++b) {
            const uint64_t* s = slots + (size_t)(b * groups_) * tile_words;
            const uint32_t nl = l1_[b] - l0_[b];
            for (uint32_t w = 0; 64 * w < nl; ++w) ap.add(l0_[b] + 64 * w, line_word(s, nw_, cpg_, w));
        }
        ap.flush();
    }
    // occupied domains above the leaves (only levels some class places at)
    if (any_upper_) {
        std::fill(occ_lvl_.begin(), occ_lvl_.end(), 0ull);
        for (uint32_t k = 0; k + 1 < K_; ++k) {
            bool used = false;
            for (uint32_t c = 0; c < C_ && !used; ++c) used = level_[c] == k;
            if (!used) continue;
            uint64_t* o = occ_lvl_.data() + toff_[k];
            const uint32_t* fl = fl_[k].data();
            for (uint32_t d = 0; d < D_[k]; ++d)
                if (any_bits(occ_.data(), fl[d], fl[d + 1])) o[d >> 6] |= 1ull << (d & 63);
        }
    }
    std::fill(feas_.begin(), feas_.end(), 0ull);
    for (uint32_t c = 0; c < C_; ++c) {
        const uint32_t g = c / cpg_, j = c % cpg_, k = level_[c], pods = pods_[c];
        uint64_t* F = feas_.data() + woff_[c];
        if (k + 1 == K_) {
            BitAppender ap(F);
            for (uint32_t b = 0; b < nb; ++b) {
                const uint64_t* s = slots + (size_t)(b * groups_ + g) * tile_words;
                const uint32_t nl = l1_[b] - l0_[b];
                for (uint32_t w = 0; 64 * w < nl; ++w) ap.add(l0_[b] + 64 * w, line_word(s, nw_, j, w));
            }
            ap.flush();
            const uint32_t nw = woff_[c + 1] - woff_[c];
            for (uint32_t w = 0; w < nw; ++w) F[w] &= ~occ_[w];
        } else {
            uint64_t* S = sums_.data() + uoff_[c];
            std::fill(S, S + D_[k], 0ull);
            for (uint32_t b = 0; b < nb; ++b) {
                const uint64_t* s = slots + (size_t)(b * groups_ + g) * tile_words;
                const uint32_t nl = l1_[b] - l0_[b];
                for (uint32_t w = 0; 64 * w < nl; ++w) {
                    const uint32_t n = std::min<uint32_t>((uint32_t)s[2u * (j * nw_ + w)], kSplitRecs);
                    const uint64_t* q = s + n_line + ((size_t)j * nw_ + w) * kSplitRecs;
                    for (uint32_t i = 0; i < n; ++i) {
                        const uint64_t r = q[i];
                        const uint32_t d = (uint32_t)(r >> 30) & (kSplitMaxDomains - 1u);
                        if (d < D_[k]) S[d] += (uint32_t)(r & 0x3FFFFFFFull);
                    }
                }
            }
            const uint64_t* O = occ_lvl_.data() + toff_[k];
            for (uint32_t d = 0; d < D_[k]; ++d)
                if (S[d] >= pods && !((O[d >> 6] >> (d & 63)) & 1ull)) F[d >> 6] |= 1ull << (d & 63);
        }
    }
}

// Taking domain d at level k (its own bit is set by the caller) takes its
// ancestors and its descendants at every other level.
// (the per-level table pointers are set up by walk(): raw pointers, not a
// vector lookup per level and job)
void HostWalk::take_marks(uint32_t d, uint32_t k) {
    if (k + 1 < K_ && lv_fl_[k][d] == lv_fl_[k][d + 1]) return;  // an empty domain intersects nothing
    uint32_t dd = d;
    for (int kk = (int)k - 1; kk >= 0; --kk) {
        dd = (uint32_t)lv_par_[kk + 1][dd];
        lv_t_[kk][dd >> 6] |= 1ull << (dd & 63);
    }
    uint32_t lo = d, hi = d + 1;
    for (uint32_t kk = k + 1; kk < K_; ++kk) {
        lo = lv_cs_[kk - 1][lo];
        hi = lv_cs_[kk - 1][hi];
        set_range(lv_t_[kk], lo, hi);
    }
}

uint32_t HostWalk::place(const uint64_t* slots, const uint32_t* run_class, const uint32_t* run_len, uint32_t n_runs,
                         int32_t* assign) {
    build_feasibility(slots);
    return walk(feas_.data(), run_class, run_len, n_runs, assign);
}

static inline void prefetch_vec(const void* p, size_t bytes) {
    const char* c = static_cast<const char*>(p);
    for (size_t i = 0; c && i < bytes; i += 64) __builtin_prefetch(c + i, 0, 3);
}

void HostWalk::prefetch_state() const {
    prefetch_vec(taken_.data(), taken_.size() * 8);
    prefetch_vec(feas_.data(), feas_.size() * 8);
    prefetch_vec(occ_.data(), occ_.size() * 8);
    prefetch_vec(sums_.data(), std::min<size_t>(sums_.size() * 8, 65536));
    prefetch_vec(cw_.data(), cw_.size() * sizeof(ClassWalk));
    prefetch_vec(level_.data(), level_.size() * 4);
    prefetch_vec(pods_.data(), pods_.size() * 4);
    prefetch_vec(woff_.data(), woff_.size() * 4);
    prefetch_vec(uoff_.data(), uoff_.size() * 4);
    prefetch_vec(l0_.data(), l0_.size() * 4);
    prefetch_vec(l1_.data(), l1_.size() * 4);
    for (uint32_t k = 0; k < K_; ++k) {
        prefetch_vec(fl_[k].data(), std::min<size_t>(fl_[k].size() * 4, 65536));
        prefetch_vec(cs_[k].data(), std::min<size_t>(cs_[k].size() * 4, 65536));
        prefetch_vec(par_[k].data(), std::min<size_t>(par_[k].size() * 4, 65536));
    }
}

uint32_t HostWalk::walk(const uint64_t* feas, const uint32_t* run_class, const uint32_t* run_len, uint32_t n_runs,
                        int32_t* assign) {
    std::fill(taken_.begin(), taken_.end(), 0ull);
    for (uint32_t k = 0; k < K_; ++k) {
        lv_t_[k] = taken_.data() + toff_[k];
        lv_fl_[k] = fl_[k].data();
        lv_cs_[k] = cs_[k].data();
        lv_par_[k] = par_[k].data();
    }
    // per class, everything a run needs in one record (cfg5: ~500 runs of one
    // job each, so the per-run set-up is most of the walk)
    cw_.resize(C_);
    for (uint32_t c = 0; c < C_; ++c) {
        const uint32_t k = level_[c];
        cw_[c] = ClassWalk{feas + woff_[c], taken_.data() + toff_[k], D_[k], (D_[k] + 63) / 64, k, 0u};
    }
    uint32_t placed = 0;
    size_t j = 0;
    const bool marks = K_ > 1;
    for (uint32_t r = 0; r < n_runs; ++r) {
        ClassWalk& cw = cw_[run_class[r]];
        const uint32_t n = run_len[r];
        uint32_t cur = cw.cursor, i = 0;
        if (cur < cw.D) {
            // The run's jobs take the free feasible bits in order. Taking a
            // domain marks other levels only (ancestors above, descendants
            // below), so at this level the only bits that change are the ones
            // the run itself takes: the current word's free bits are kept
            // across jobs and re-read only when a new word starts.
            const uint64_t* F = cw.F;
            uint64_t* T = cw.T;
            uint32_t w = cur >> 6;
            uint64_t bits = F[w] & ~T[w] & (~0ull << (cur & 63));
            for (; i < n; ++i) {
                while (bits == 0 && ++w < cw.nw) bits = F[w] & ~T[w];
                if (bits == 0) break;
                const uint32_t b = (uint32_t)__builtin_ctzll(bits);
                const uint32_t d = w * 64 + b;
                bits &= bits - 1;
                assign[j + i] = (int32_t)d;
                T[w] |= 1ull << b;
                if (marks) take_marks(d, cw.k);
                cur = d + 1;
            }
            placed += i;
            cw.cursor = i < n ? cw.D : cur;
        }
        for (; i < n; ++i) assign[j + i] = -1;
        j += n;
    }
    return placed;
}

}  // namespace jsp

// Internal entries for the CPU tests of the host walk (tests/test_host_walk.py)
// and its timing (tools/walk_bench.py): not part of include/jsplace.h. The
// hierarchy tables are derived from first_leaf as jsp_topology_upload derives
// them.
static bool walk_setup(jsp::HostWalk& w, uint32_t K, const uint32_t* D, const uint32_t* const* first_leaf, uint32_t C,
                       const uint32_t* cls_level, const uint32_t* cls_pods, uint32_t n_blocks, const uint32_t* blk_l0,
                       const uint32_t* blk_l1, uint32_t groups, uint32_t cpg) {
    using jsp::kMaxLevels;
    if (K < 1 || K > kMaxLevels) return false;
    std::vector<uint32_t> fl[kMaxLevels], cs[kMaxLevels];
    std::vector<int32_t> par[kMaxLevels];
    for (uint32_t k = 0; k < K; ++k) fl[k].assign(first_leaf[k], first_leaf[k] + D[k] + 1);
    for (uint32_t k = 0; k < K; ++k) {
        if (k + 1 < K) {
            cs[k].resize(D[k] + 1);
            for (uint32_t d = 0; d <= D[k]; ++d)
                cs[k][d] = (uint32_t)(std::lower_bound(fl[k + 1].begin(), fl[k + 1].end(), fl[k][d]) - fl[k + 1].begin());
        }
        if (k > 0) {
            par[k].resize(std::max<uint32_t>(D[k], 1));
            for (uint32_t d = 0; d < D[k]; ++d)
                par[k][d] = (int32_t)(std::upper_bound(fl[k - 1].begin(), fl[k - 1].end(), fl[k][d]) - fl[k - 1].begin()) - 1;
        }
    }
    std::vector<jsp::DevClass> cls(C);
    for (uint32_t c = 0; c < C; ++c) {
        std::memset(&cls[c], 0, sizeof cls[c]);
        cls[c].level = cls_level[c];
        cls[c].pods = cls_pods[c];
    }
    w.set_topology(K, D, fl, cs, par);
    w.set_classes(cls);
    w.set_tiles(std::vector<uint32_t>(blk_l0, blk_l0 + n_blocks), std::vector<uint32_t>(blk_l1, blk_l1 + n_blocks),
                groups, cpg);
    return true;
}

extern "C" int jspi_walk_test(uint32_t K, const uint32_t* D, const uint32_t* const* first_leaf, uint32_t C,
                              const uint32_t* cls_level, const uint32_t* cls_pods, uint32_t n_blocks,
                              const uint32_t* blk_l0, const uint32_t* blk_l1, uint32_t groups, uint32_t cpg,
                              const uint64_t* slots, const uint32_t* run_class, const uint32_t* run_len,
                              uint32_t n_runs, int32_t* assign) {
    jsp::HostWalk w;
    if (!walk_setup(w, K, D, first_leaf, C, cls_level, cls_pods, n_blocks, blk_l0, blk_l1, groups, cpg)) return -1;
    return (int)w.place(slots, run_class, run_len, n_runs, assign);
}

// The same walk `iters` times on one set-up walker: mean ns per place() in
// out_ns[0], and in out_ns[1] the feasibility build alone.
extern "C" int jspi_walk_bench(uint32_t K, const uint32_t* D, const uint32_t* const* first_leaf, uint32_t C,
                               const uint32_t* cls_level, const uint32_t* cls_pods, uint32_t n_blocks,
                               const uint32_t* blk_l0, const uint32_t* blk_l1, uint32_t groups, uint32_t cpg,
                               const uint64_t* slots, const uint32_t* run_class, const uint32_t* run_len,
                               uint32_t n_runs, int32_t* assign, uint32_t iters, double* out_ns) {
    jsp::HostWalk w;
    if (!walk_setup(w, K, D, first_leaf, C, cls_level, cls_pods, n_blocks, blk_l0, blk_l1, groups, cpg)) return -1;
    uint32_t placed = 0;
    auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 0; i < iters; ++i) placed = w.place(slots, run_class, run_len, n_runs, assign);
    auto t1 = std::chrono::steady_clock::now();
    for (uint32_t i = 0; i < iters; ++i) w.feasibility_only(slots);
    auto t2 = std::chrono::steady_clock::now();
    out_ns[0] = std::chrono::duration<double, std::nano>(t1 - t0).count() / std::max<uint32_t>(iters, 1);
    out_ns[1] = std::chrono::duration<double, std::nano>(t2 - t1).count() / std::max<uint32_t>(iters, 1);
    return (int)placed;
}
