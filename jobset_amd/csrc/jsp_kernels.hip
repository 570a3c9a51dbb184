// jsp_kernels.hip — gfx950 kernels of the exclusive-topology placement engine.
//
// A placement is (SURVEY.md §8a rows A8 then A7):
//   tally   HBM-streaming predicate + per-(class, leaf) pod-capacity tally.
//           One workgroup owns a contiguous run of whole leaves, so every leaf
//           sum finishes inside one workgroup: no global atomics, no memset,
//           bit-exact integer sums, each written exactly once.
//   feas    per-(class, domain) feasibility bitmap at the class's topology
//           level (wave64 ballot -> one 64-bit word per wave).
//   assign  lowest-index 1:1 assignment, walked as replicated-job runs (one
//           class each): a block-wide prefix of word popcounts hands the k-th
//           available domain to the k-th job of the run.
// Two launch shapes:
//   large snapshots: tally_kernel (grid) -> feas_kernel (grid) -> assign_kernel
//                    (one 1024-thread workgroup);
//   small snapshots: place_fused_kernel — the tally grid, after which the last
//                    workgroup to finish (agent-scope release/acquire ticket)
//                    builds the bitmaps in LDS and runs the assignment; one
//                    launch per placement.
// Plus gather kernels for the webhook / reconciler batch paths (A5, A9) and the
// snapshot patch.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "jsp_internal.h"

namespace jsp {

// Diagnostic build only (-DJSP_STAMPS, tools/stamps.py): per-workgroup phase
// timestamps of the constant 100 MHz clock, for finding where a launch's
// time goes. The product library is built without it.
#ifdef JSP_STAMPS
__device__ unsigned long long jsp_dbg[4096 * 8];
#define JSP_STAMP(blk, i)                                                                 \
    do {                                                                                  \
        if (threadIdx.x == 0 && (blk) < 4096) jsp_dbg[(blk) * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
// shader-clock stamp (s_memtime) beside a real-time one: the effective clock of a phase
#define JSP_CLK(blk, i)                                                                   \
    do {                                                                                  \
        if (threadIdx.x == 0 && (blk) < 4096) jsp_dbg[(blk) * 8 + (i)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#define JSP_DBGV(row, i, v)                                                               \
    do {                                                                                  \
        if (threadIdx.x == 0 && (row) < 4096) jsp_dbg[(row) * 8 + (i)] = (unsigned long long)(v); \
    } while (0)
// per-wave real-time stamp (lane 0 of each wave), and a shader-clock one
#define JSP_WSTAMP(w, i)                                                                  \
    do {                                                                                  \
        if ((threadIdx.x & 63) == 0 && (w) < 4096) jsp_dbg[(w) * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#define JSP_WCLK(w, i)                                                                    \
    do {                                                                                  \
        if ((threadIdx.x & 63) == 0 && (w) < 4096) jsp_dbg[(w) * 8 + (i)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define JSP_WSTAMP(w, i) \
    do {                 \
    } while (0)
#define JSP_WCLK(w, i) \
    do {               \
    } while (0)
#define JSP_DBGV(row, i, v) \
    do {                    \
    } while (0)
#define JSP_CLK(blk, i) \
    do {                \
    } while (0)
#define JSP_STAMP(blk, i) \
    do {                  \
    } while (0)
#endif

// ----------------------------------------------------------------- helpers
// LDS pointers typed as such: where LDS tables are reached through a struct or
// a carved-up generic pointer the compiler can lose their address space and
// emit flat loads and atomics (each waiting on both the vector and the LDS
// counters; a release or acquire on one also drains global traffic)
#define JSP_LDS __attribute__((address_space(3)))
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // a 16-B LDS store in any address space

template <typename T>
__device__ __forceinline__ JSP_LDS T* lds_ptr(T* p) {
    return (JSP_LDS T*)p;
}
// Inclusive wave64 prefix sum on the VALU with DPP (no LDS traffic):
// row_shr 1/2/4/8 scan each 16-lane row, row_bcast15 / row_bcast31 carry the
// row totals across rows (GFX9/CDNA DPP controls).
// s_waitcnt vmcnt(0) with the other counters unconstrained (gfx9 encoding:
// vmcnt bits 3:0 and 15:14, expcnt 6:4, lgkmcnt 11:8), as the builtin's
// immediate: the compiler's wait insertion sees it, unlike inline asm.
constexpr int kWaitVmcnt0 = 0x0F70;

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x, int /*lane*/) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}

// Wave64 OR / unsigned-min of a value, uniform result (DPP row steps within
// each 16-lane row, row_bcast15/31 across rows; lane 63 holds the total).
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_or(uint32_t x) {
    return x | (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROW_MASK, 0xf, false);
}
__device__ __forceinline__ uint64_t wave_or64(uint64_t v) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    lo = dpp_or<0x111, 0xf>(lo); hi = dpp_or<0x111, 0xf>(hi);  // row_shr:1
    lo = dpp_or<0x112, 0xf>(lo); hi = dpp_or<0x112, 0xf>(hi);  // row_shr:2
    lo = dpp_or<0x114, 0xf>(lo); hi = dpp_or<0x114, 0xf>(hi);  // row_shr:4
    lo = dpp_or<0x118, 0xf>(lo); hi = dpp_or<0x118, 0xf>(hi);  // row_shr:8
    lo = dpp_or<0x142, 0xa>(lo); hi = dpp_or<0x142, 0xa>(hi);  // row_bcast:15
    lo = dpp_or<0x143, 0xc>(lo); hi = dpp_or<0x143, 0xc>(hi);  // row_bcast:31
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, 63) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)lo, 63);
}
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_and(uint32_t x) {
    return x & (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)x, CTRL, ROW_MASK, 0xf, false);
}
__device__ __forceinline__ uint64_t wave_and64(uint64_t v) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    lo = dpp_and<0x111, 0xf>(lo); hi = dpp_and<0x111, 0xf>(hi);
    lo = dpp_and<0x112, 0xf>(lo); hi = dpp_and<0x112, 0xf>(hi);
    lo = dpp_and<0x114, 0xf>(lo); hi = dpp_and<0x114, 0xf>(hi);
    lo = dpp_and<0x118, 0xf>(lo); hi = dpp_and<0x118, 0xf>(hi);
    lo = dpp_and<0x142, 0xa>(lo); hi = dpp_and<0x142, 0xa>(hi);
    lo = dpp_and<0x143, 0xc>(lo); hi = dpp_and<0x143, 0xc>(hi);
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, 63) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)lo, 63);
}
// number of set bits of a uniform 64-bit mask below this lane
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
    // bound_ctrl off: lanes without a source keep their own value (old = x)
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x111, 0xf, 0xf, false));
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x112, 0xf, 0xf, false));
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x114, 0xf, 0xf, false));
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x118, 0xf, 0xf, false));
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x142, 0xa, 0xf, false));
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x143, 0xc, 0xf, false));
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

// Completion word of the host placement path: every wave's stores of this
// workgroup (assign[] and stats, in pinned host memory) are drained, then one
// lane publishes `value` (vector store, system scope). The host spins on the
// word instead of waiting for the kernel-end signal, which saves the ~5 us of
// the end-of-kernel completion path. `fence`: a system-scope
// release first -- needed when the workgroup's output went out as plain
// stores; output written with system-scope stores (store_sys) is already at
// the host once its wave's vmcnt has drained.
__device__ __forceinline__ void signal_host(uint32_t* word, uint32_t value, bool fence) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        if (fence) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(word, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// An output word: to pinned host memory as a system-scope (write-through)
// store when `sys`, else a plain store.
template <class T>
__device__ __forceinline__ void store_out(T* p, T v, bool sys) {
    if (sys) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else *p = v;
}

// Store of bytes another workgroup of the same launch reads: write-through
// (agent-scope relaxed = `sc1`) when `sc1`, so the writer needs no release fence
// and a reader using `sc1` loads no acquire (cdna_hip_programming.md G16).
__device__ __forceinline__ void store_handoff(uint32_t* p, uint32_t v, int sc1) {
    if (sc1) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}
__device__ __forceinline__ uint32_t load_handoff(const uint32_t* p) {
    return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// last leaf index l in [0, n) with ls[l] <= row (ls ascending, n+1 entries)
__device__ __forceinline__ uint32_t leaf_search(const uint32_t* ls, uint32_t n, uint32_t row) {
    uint32_t lo = 0, hi = n;  // invariant: ls[lo] <= row, answer < hi
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (ls[mid] <= row) lo = mid; else hi = mid;
    }
    return lo;
}

constexpr uint32_t kSvcStaggerTicks = 50;  // 100 MHz ticks between the dispatcher's polling waves

// Request phase stamp of the resident service (timing on): thread 0 stores the
// 100 MHz clock into the tile's host-mapped clock slots (posted system-scope
// stores; nothing waits on them). Slots: 0 request seen, 1 request broadcast
// to the workgroup, 2 tallied, 3 feasible count scanned, 4 look-back done,
// 5 assign[] drained, 6 row pass done, 7 leaf pass done.
// The stamps are kept in LDS (s_clk, static) and go out with the request's
// done word (signal_host_clk): a system-scope store in the request path would
// put a host-link round trip into the next wait on vmcnt (the row pass's
// register waits), which is what the round-3 stamps measured as the row pass.
__device__ __forceinline__ void svc_stamp(JSP_LDS uint32_t* clk, int slot) {
#ifdef JSP_AB_CLKFREQ
    // A/B build: slots 6 and 7 carry the shader clock at slots 1 and 2 (the
    // effective clock of the row and leaf passes), not the real-time stamps
    if (clk && threadIdx.x == 0) {
        if (slot == 1) clk[6] = (uint32_t)__builtin_amdgcn_s_memtime();
        if (slot == 2) clk[7] = (uint32_t)__builtin_amdgcn_s_memtime();
        if (slot != 6 && slot != 7) clk[slot] = (uint32_t)wall_clock64();
    }
#else
    if (clk && threadIdx.x == 0) clk[slot] = (uint32_t)wall_clock64();
#endif
}

// signal_host with the request's stamps: every wave's stores drained, then
// lane 0 takes stamp 5 (drained), writes the tile's stamps to the host and,
// once they have landed, the done word -- the host reads the stamps after it.
__device__ __forceinline__ void signal_host_clk(uint32_t* word, uint32_t value, JSP_LDS uint32_t* s_clk,
                                                uint32_t* clk_out) {
    if (s_clk == nullptr || clk_out == nullptr) {
        signal_host(word, value, false);
        return;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        s_clk[5] = (uint32_t)wall_clock64();
        for (int i = 0; i < (int)kSvcClkSlots; ++i)
            __hip_atomic_store(clk_out + i, s_clk[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(word, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ----------------------------------------------------------------- A8 tally (one workgroup)
// LDS carve (uint32 words), sized per launch by nv = classes in this pass + 1:
//   [classes nc x DevClass][acc nv x la][wsum nv x 4]
//   [leaf starts la+1 (+3 pad)][row prefixes nv x kChunkRows]
// Class records are staged in LDS once per workgroup (read per row from global
// memory they were re-fetched by vector loads: a generic pointer may alias
// LDS, and SGPRs are too few to hold them).
// Sized per launch: nc classes, nv values, la = the leaf stride of acc (the
// most leaves any workgroup of the snapshot owns, rounded up to 4), so a
// snapshot of small racks does not reserve 256 leaves' worth per value --
// LDS per workgroup decides how many tally workgroups a CU holds at once.
__host__ __device__ constexpr int tally_acc_off(int nc) { return nc * (int)(sizeof(DevClass) / 4); }
__host__ __device__ constexpr int tally_wsum_off(int nc, int nv, int la) { return tally_acc_off(nc) + nv * la; }
__host__ __device__ constexpr int tally_ls_off(int nc, int nv, int la) { return tally_wsum_off(nc, nv, la) + nv * kTallyWaves; }
__host__ __device__ constexpr int tally_pre_off(int nc, int nv, int la) { return tally_ls_off(nc, nv, la) + la + 4; }
__host__ __device__ constexpr int tally_lds_words(int nc, int nv, int la) {
    return tally_pre_off(nc, nv, la) + nv * kChunkRows;
}
__host__ __device__ inline int tally_lds_words(const TallyArgs& a) {
    return tally_lds_words((int)a.nc, (int)a.nc + a.do_occ, (int)a.la);
}

// Rows of the workgroup: [r0, r1) = leaves [l0, l1). Per chunk of 1024 rows
// each thread holds 4 consecutive rows (16-B column loads: a wave streams
// 1 KiB per column instruction), evaluates every class on them, and writes its
// rows' in-wave inclusive prefixes (DPP wave scan) to LDS — a pure streaming
// pass, no branches on leaf boundaries. Then one thread per leaf adds
// prefix(last row in chunk) - prefix(row before first in chunk) of its leaf
// (plus the earlier waves' totals) to acc[v][leaf]; the leaf is owned by that
// thread, so no atomics.
// One thread's 4 consecutive rows of every column (16-B loads).
template <int W, int R>
struct RowRegs {
    uint64_t lab[W][4];
    uint32_t tn[4], fr[R][4];
    int32_t ex[4];
};

// 16 bytes of a column at byte offset `off`, `sc1` (agent scope): bypasses
// this CU's L1, so rows another launch patched since this workgroup last read
// them are never served from stale L1 lines (the resident service has no
// kernel-start invalidate between requests). Offsets are 32-bit: the service
// runs for <= 255 tiles (~261k rows).
__device__ __forceinline__ uint4 load16_sc1(const void* base, uint32_t off) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                                                       0x7FFFFFF0, 0x00020000);
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));
}

// The same with a bound: bytes at offsets >= n_bytes read as 0 (the
// descriptor's range check, per dword).
__device__ __forceinline__ uint4 load16_sc1_n(const void* base, uint32_t off, uint32_t n_bytes) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                                                       (int)n_bytes, 0x00020000);
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));
}

template <int W, int R, bool SC1 = false>
__device__ __forceinline__ void load_rows(const TallyArgs& a, uint32_t row, bool any, RowRegs<W, R>& x) {
    if (SC1 && any) {
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const uint64_t* col = a.labels + (size_t)w * a.npad;
            const uint4 u = load16_sc1(col, row * 8u), v = load16_sc1(col, row * 8u + 16u);
            x.lab[w][0] = ((uint64_t)u.y << 32) | u.x; x.lab[w][1] = ((uint64_t)u.w << 32) | u.z;
            x.lab[w][2] = ((uint64_t)v.y << 32) | v.x; x.lab[w][3] = ((uint64_t)v.w << 32) | v.z;
        }
        const uint4 t4 = load16_sc1(a.taints, row * 4u);
        x.tn[0] = t4.x; x.tn[1] = t4.y; x.tn[2] = t4.z; x.tn[3] = t4.w;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint4 f4 = load16_sc1(a.freer + (size_t)r * a.npad, row * 4u);
            x.fr[r][0] = f4.x; x.fr[r][1] = f4.y; x.fr[r][2] = f4.z; x.fr[r][3] = f4.w;
        }
        const uint4 e4 = load16_sc1(a.excl, row * 4u);
        x.ex[0] = (int32_t)e4.x; x.ex[1] = (int32_t)e4.y; x.ex[2] = (int32_t)e4.z; x.ex[3] = (int32_t)e4.w;
    } else if (any) {
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const ulonglong2* p = reinterpret_cast<const ulonglong2*>(a.labels + (size_t)w * a.npad + row);
            const ulonglong2 u = p[0], v = p[1];
            x.lab[w][0] = u.x; x.lab[w][1] = u.y; x.lab[w][2] = v.x; x.lab[w][3] = v.y;
        }
        const uint4 t4 = *reinterpret_cast<const uint4*>(a.taints + row);
        x.tn[0] = t4.x; x.tn[1] = t4.y; x.tn[2] = t4.z; x.tn[3] = t4.w;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint4 f4 = *reinterpret_cast<const uint4*>(a.freer + (size_t)r * a.npad + row);
            x.fr[r][0] = f4.x; x.fr[r][1] = f4.y; x.fr[r][2] = f4.z; x.fr[r][3] = f4.w;
        }
        const int4 e4 = *reinterpret_cast<const int4*>(a.excl + row);
        x.ex[0] = e4.x; x.ex[1] = e4.y; x.ex[2] = e4.z; x.ex[3] = e4.w;
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
            for (int w = 0; w < W; ++w) x.lab[w][i] = 0;
#pragma unroll
            for (int r = 0; r < R; ++r) x.fr[r][i] = 0;
            x.tn[i] = 0;
            x.ex[i] = -1;
        }
    }
}

// On-chip copy of a thread's 4 rows (the resident compaction service keeps
// its tile's rows in LDS between requests while no patch touched the
// snapshot): 2W + 2 + R uint4 per thread, column-major by thread so each
// 16-B access of a wave is contiguous (no bank conflicts).
template <int W, int R>
constexpr int row_cache_vecs() { return 2 * W + 2 + R; }

template <int W, int R>
__device__ __forceinline__ void rows_to_lds(JSP_LDS u32x4* c, int tid, const RowRegs<W, R>& x) {
    int k = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        c[(k++) * kTallyThreads + tid] = u32x4{(uint32_t)x.lab[w][0], (uint32_t)(x.lab[w][0] >> 32),
                                               (uint32_t)x.lab[w][1], (uint32_t)(x.lab[w][1] >> 32)};
        c[(k++) * kTallyThreads + tid] = u32x4{(uint32_t)x.lab[w][2], (uint32_t)(x.lab[w][2] >> 32),
                                               (uint32_t)x.lab[w][3], (uint32_t)(x.lab[w][3] >> 32)};
    }
    c[(k++) * kTallyThreads + tid] = u32x4{x.tn[0], x.tn[1], x.tn[2], x.tn[3]};
#pragma unroll
    for (int r = 0; r < R; ++r) c[(k++) * kTallyThreads + tid] = u32x4{x.fr[r][0], x.fr[r][1], x.fr[r][2], x.fr[r][3]};
    c[k * kTallyThreads + tid] = u32x4{(uint32_t)x.ex[0], (uint32_t)x.ex[1], (uint32_t)x.ex[2], (uint32_t)x.ex[3]};
}

template <int W, int R>
__device__ __forceinline__ void rows_from_lds(const JSP_LDS u32x4* c, int tid, RowRegs<W, R>& x) {
    int k = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        const u32x4 u = c[(k++) * kTallyThreads + tid], v = c[(k++) * kTallyThreads + tid];
        x.lab[w][0] = ((uint64_t)u[1] << 32) | u[0]; x.lab[w][1] = ((uint64_t)u[3] << 32) | u[2];
        x.lab[w][2] = ((uint64_t)v[1] << 32) | v[0]; x.lab[w][3] = ((uint64_t)v[3] << 32) | v[2];
    }
    const u32x4 t4 = c[(k++) * kTallyThreads + tid];
    x.tn[0] = t4[0]; x.tn[1] = t4[1]; x.tn[2] = t4[2]; x.tn[3] = t4[3];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const u32x4 f4 = c[(k++) * kTallyThreads + tid];
        x.fr[r][0] = f4[0]; x.fr[r][1] = f4[1]; x.fr[r][2] = f4[2]; x.fr[r][3] = f4[3];
    }
    const u32x4 e4 = c[k * kTallyThreads + tid];
    x.ex[0] = (int32_t)e4[0]; x.ex[1] = (int32_t)e4[1]; x.ex[2] = (int32_t)e4[2]; x.ex[3] = (int32_t)e4[3];
}

// The fields of one class the row pass reads, moved to SGPRs: every lane
// reads the same LDS words, so readfirstlane is exact, and the row pass then
// takes them as scalar operands and branches on them without exec masking
// (read as VGPRs, each use waited on its own LDS round trip).
template <int W, int R>
struct ClassRegs {
    uint64_t req[W], mask[W];
    uint32_t tol_inv, pods, res[R];
    double rcp[R];
};

// floor(n / res) for one row of a resource, res >= 2: the f64 reciprocal,
// truncated (exact for every u32 n: DESIGN.md §4.1). 3 VALU ops at the f64
// rate; the invariant-divisor multiply-high it replaced issues v_mul_hi_u32 at
// a quarter of the full rate on gfx950 (8.6 cycles per wave-instruction,
// tools/valu_rate.hip) and took SGPRs for its constants.
// A class's capacity on 4 rows: min(pods, min over its requested resources of
// floor(free / req)). floor is monotone, so the minimum is taken over the f64
// products fl(free * rcp) -- each floors to the exact quotient (rcp = 1.0 for
// req == 1) -- and ONE truncation to u32 ends it: per resource and row one
// v_mul_f64 and one v_min_f64, per row one v_cvt_u32_f64 (the per-resource
// truncation and integer min it replaces cost two more instructions each).
template <int W, int R>
__device__ __forceinline__ void row_caps(const ClassRegs<W, R>& k, const uint32_t (&fr)[R][4], uint32_t (&cap)[4]) {
    const double pods = (double)k.pods;
    double m[4] = {pods, pods, pods, pods};
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (k.res[r] == 0) continue;  // scalar branch (SGPR operand)
#pragma unroll
        for (int i = 0; i < 4; ++i) m[i] = __builtin_fmin(m[i], (double)fr[r][i] * k.rcp[r]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) cap[i] = (uint32_t)m[i];
}

__device__ __forceinline__ uint32_t to_sgpr(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint64_t to_sgpr64(uint64_t x) {
    return ((uint64_t)to_sgpr((uint32_t)(x >> 32)) << 32) | to_sgpr((uint32_t)x);
}

template <int W, int R>
__device__ __forceinline__ ClassRegs<W, R> class_regs(const DevClass& d) {
    ClassRegs<W, R> k;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        k.req[w] = to_sgpr64(d.req[w]);
        k.mask[w] = to_sgpr64(d.mask[w]);
    }
    k.tol_inv = to_sgpr(d.tol_inv);
    k.pods = to_sgpr(d.pods);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        k.res[r] = to_sgpr(d.res[r]);
        const uint32_t* rw = reinterpret_cast<const uint32_t*>(&d.rcp[r]);  // the two halves, moved to SGPRs
        k.rcp[r] = __hiloint2double((int)to_sgpr(rw[1]), (int)to_sgpr(rw[0]));
    }
    return k;
}

// STAGED (resident service): the class records and the tile's leaf starts are
// already in LDS (staged once per service lifetime: they change only with an
// upload, which restarts the service) and `bt` is the tile's geometry, so the
// first chunk's row loads are the request's first memory access.
// row_cache (resident compaction service, single-chunk tiles only): the
// tile's rows are read from this LDS copy when use_cache, else loaded and
// copied into it.
// staged_rt (the resident split service after its first request): the same
// as STAGED at run time -- the class records and leaf starts an earlier
// request staged are still in LDS (nothing else writes those words; an
// upload restarts the service), and bt_staged is the tile's geometry. A
// request answered from the row copy then issues no global load before its
// row pass (cfg3: 0.52 us from the broadcast to the first chunk, one memory
// round trip for words that never change).
template <int W, int R, bool STAGED = false, bool SC1 = STAGED>
__device__ __forceinline__ void tally_block(const TallyArgs& a, uint32_t blk, uint32_t* lds,
                                            uint4 bt_staged = make_uint4(0, 0, 0, 0), JSP_LDS uint32_t* clk = nullptr,
                                            JSP_LDS u32x4* row_cache = nullptr, bool use_cache = false,
                                            bool staged_rt = false) {
    const int nc = (int)a.nc;
    const int nv = nc + a.do_occ;
    DevClass* s_cls = reinterpret_cast<DevClass*>(lds);
    const int la = (int)a.la;
    uint32_t* s_acc = lds + tally_acc_off(nc);
    uint32_t* s_wsum = lds + tally_wsum_off(nc, nv, la);
    uint32_t* s_ls = lds + tally_ls_off(nc, nv, la);
    uint32_t* s_pre = lds + tally_pre_off(nc, nv, la);

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
#ifdef JSP_AB_ENTRYSTAMP
    svc_stamp(clk, 2);  // A/B build: slots 2-4 at the block's entry, after its row copy, after the first barrier
#endif
    const bool staged = STAGED || staged_rt;
    const uint4 bt = staged ? bt_staged : a.blk[blk];  // {first leaf, end leaf, first row, end row}
    const uint32_t l0 = bt.x, nl = bt.y - bt.x, r0 = bt.z, r1 = bt.w;

    // Every global load a workgroup needs before its first barrier is issued
    // back to back -- staging words (class records, leaf starts) first, then
    // the first chunk's rows -- and only then are the staging words written to
    // LDS, so the wait for them (vmcnt counts in issue order) leaves the row
    // loads in flight: one memory round trip before the row pass, not two.
    constexpr int kClsVec = (int)(sizeof(DevClass) / 16);
    static_assert(kTallyClasses * kClsVec <= kTallyThreads, "one class vector per thread");
    static_assert(kMaxBlkLeaves + 1 <= 2 * kTallyThreads, "two leaf starts per thread");
    const bool st_cls = !staged && tid < nc * kClsVec;
    const bool st_ls0 = !staged && (uint32_t)tid <= nl, st_ls1 = !staged && (uint32_t)tid + kTallyThreads <= nl;
    uint4 cls_v = make_uint4(0, 0, 0, 0);
    uint32_t ls0 = 0, ls1 = 0;
    if (st_cls) cls_v = reinterpret_cast<const uint4*>(a.cls + a.c0)[tid];
    if (st_ls0) ls0 = a.leaf_start[l0 + tid];
    if (st_ls1) ls1 = a.leaf_start[l0 + tid + kTallyThreads];

    // A workgroup of a large snapshot owns several chunks: the next chunk's rows
    // are loaded (into a second register set) before this chunk is evaluated,
    // so its HBM latency hides behind the row and leaf passes.
    const uint32_t base0 = r0 & ~3u;
    RowRegs<W, R> cur;
    if (row_cache != nullptr && use_cache) {
        rows_from_lds<W, R>(row_cache, tid, cur);
#ifdef JSP_AB_ENTRYSTAMP
        svc_stamp(clk, 3);
#endif
    } else {
        const uint32_t row = base0 + 4u * tid;
        load_rows<W, R, SC1>(a, row, (row < r1) && (row + 3 >= r0), cur);
        if (row_cache != nullptr) rows_to_lds<W, R>(row_cache, tid, cur);
    }
    for (int i = tid; i < nv * la; i += kTallyThreads) s_acc[i] = 0;
    if (st_cls) reinterpret_cast<uint4*>(s_cls)[tid] = cls_v;
    if (st_ls0) s_ls[tid] = ls0;
    if (st_ls1) s_ls[tid + kTallyThreads] = ls1;
    for (uint32_t base = base0; base < r1; base += kChunkRows) {
        const uint32_t row = base + 4u * tid;
        const bool any = (row < r1) && (row + 3 >= r0);
        bool valid[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) valid[i] = any && (row + i >= r0) && (row + i < r1);
        __syncthreads();  // s_cls / s_ls / s_acc ready (first chunk); previous leaf pass done (later ones)
        JSP_STAMP(blk, 1);
#ifdef JSP_AB_ENTRYSTAMP
        if (base == base0) svc_stamp(clk, 4);
#endif
#ifdef JSP_AB_FINESTAMP
        svc_stamp(clk, 2);  // A/B build: slots 2-4 inside the row pass (compact_tile's are dropped)
#endif
        const bool more = base + kChunkRows < r1;  // workgroup-uniform
        RowRegs<W, R> nxt;
        if (more) {
            const uint32_t nrow = row + kChunkRows;
            load_rows<W, R, SC1>(a, nrow, (nrow < r1) && (nrow + 3 >= r0), nxt);
        }
        const auto& lab = cur.lab;
        const auto& tn = cur.tn;
        const auto& fr = cur.fr;
        const auto& ex = cur.ex;

        // ---- row pass: per value, evaluate 4 rows, scan, store row prefixes.
        // Two values per step: their evaluations and their DPP scans are
        // independent, so the two dependent chains interleave (cfg3's split
        // tiles: 2 classes + occupancy, row pass 1.6 us one value at a time).
        auto eval = [&](int c, uint32_t (&v)[4]) {
            if (c < nc) {
                const ClassRegs<W, R> k = class_regs<W, R>(s_cls[c]);
                uint32_t cap[4];
                row_caps<W, R>(k, fr, cap);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    bool ok = valid[i] & ((tn[i] & k.tol_inv) == 0);
#pragma unroll
                    for (int w = 0; w < W; ++w) ok = ok & ((lab[w][i] & k.mask[w]) == k.req[w]);
                    v[i] = ok ? cap[i] : 0u;
                }
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = (valid[i] && ex[i] != -1) ? 1u : 0u;
            }
        };
#ifdef JSP_AB_FINESTAMP
        svc_stamp(clk, 3);
#endif
        for (int c = 0; c < nv; c += 2) {
            const bool two = c + 1 < nv;  // workgroup-uniform
            uint32_t v[4], u[4] = {0u, 0u, 0u, 0u};
            eval(c, v);
            if (two) eval(c + 1, u);
            const uint32_t p0 = v[0], p1 = p0 + v[1], p2 = p1 + v[2], p3 = p2 + v[3];
            const uint32_t q0 = u[0], q1 = q0 + u[1], q2 = q1 + u[2], q3 = q2 + u[3];
            const uint32_t incl = wave_incl_scan(p3, lane), incl2 = wave_incl_scan(q3, lane);
#ifdef JSP_AB_FINESTAMP
            if (c == 0 && incl != 0xFFFFFFFFu) svc_stamp(clk, 4);
#endif
            const uint32_t wex = incl - p3;
            reinterpret_cast<uint4*>(s_pre + c * kChunkRows)[tid] = make_uint4(wex + p0, wex + p1, wex + p2, incl);
            if (lane == 63) s_wsum[c * kTallyWaves + wid] = incl;
            if (two) {
                const uint32_t wex2 = incl2 - q3;
                reinterpret_cast<uint4*>(s_pre + (c + 1) * kChunkRows)[tid] =
                    make_uint4(wex2 + q0, wex2 + q1, wex2 + q2, incl2);
                if (lane == 63) s_wsum[(c + 1) * kTallyWaves + wid] = incl2;
            }
        }
        __syncthreads();
        JSP_STAMP(blk, 6);
        svc_stamp(clk, 6);

        // ---- leaf pass: one thread per leaf folds its rows of this chunk.
        // Chunk prefix at row x = wave-local prefix + the totals of the waves
        // before x's wave; every LDS read of a value is independent (one
        // round trip), the wave offsets come from one 16-B read.
        // One thread per (value, leaf): a tile of few large leaves (cfg3: 2
        // leaves, 3 values) reads its prefixes in one LDS round trip instead
        // of a chain of nv per leaf thread (leaf pass 0.52 us on cfg3's split
        // tiles, profiles/r06/probes). Each (value, leaf) sum has one owner.
        static_assert(kTallyWaves == 4, "wave-offset select assumes 4 waves");
        for (uint32_t q = tid; q < nl * (uint32_t)nv; q += kTallyThreads) {
            const uint32_t c = q / nl, li = q - c * nl;
            const uint32_t s = s_ls[li], e = s_ls[li + 1];
            const uint32_t lo = s > base ? s : base;
            const uint32_t hi = e < base + kChunkRows ? e : base + kChunkRows;
            if (lo >= hi) continue;
            const uint32_t xh = hi - 1 - base;                       // chunk-local last row
            const uint32_t xb = lo > base ? lo - 1 - base : 0u;      // row before the first (if any)
            const bool has_lo = lo > base;
            const uint32_t wh = xh >> 8, wb = xb >> 8;               // their waves (256 rows per wave)
            const uint32_t* pre = s_pre + c * kChunkRows;
            const uint4 ws = reinterpret_cast<const uint4*>(s_wsum)[c];
            const uint32_t e1 = ws.x, e2 = e1 + ws.y, e3 = e2 + ws.z;
            // all four reads unconditional (xb = 0 when the leaf starts the chunk), then selects
            const uint32_t ph = pre[xh], pb = pre[xb];
            const uint32_t hi_p = ph + (wh == 0 ? 0u : wh == 1 ? e1 : wh == 2 ? e2 : e3);
            const uint32_t lo_p = has_lo ? pb + (wb == 0 ? 0u : wb == 1 ? e1 : wb == 2 ? e2 : e3) : 0u;
            s_acc[c * la + li] += hi_p - lo_p;
        }
        if (more) cur = nxt;
    }
    __syncthreads();
    JSP_STAMP(blk, 7);
    svc_stamp(clk, 7);
    if (a.cap_out == nullptr) return;  // the caller keeps the sums in LDS (compaction without tally output)
    for (uint32_t li = tid; li < nl; li += kTallyThreads) {
        const uint32_t leaf = a.leaf_base + l0 + li;
        for (int c = 0; c < nc; ++c) store_handoff(a.cap_out + (size_t)(a.c0 + c) * a.ld + leaf, s_acc[c * la + li], a.sc1_out);
        if (a.do_occ) store_handoff(a.occ_out + leaf, s_acc[nc * la + li], a.sc1_out);
    }
}

template <int W, int R>
__global__ __launch_bounds__(kTallyThreads) void tally_kernel(TallyArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    JSP_STAMP(blockIdx.x, 0);
    tally_block<W, R>(a, blockIdx.x, lds);
    JSP_STAMP(blockIdx.x, 5);
}


// ---- wave-tile tally (the three-launch shape's tally: large snapshots)
// Every wave works alone -- no workgroup barrier after the class records are
// staged -- on a stream of wave tiles (jsp_internal.h kWaveTile*): up to 64
// whole leaves in <= 252 rows, one 256-row chunk (lane i holds rows base + 4i
// .. + 3). A wave takes tiles gw, gw + waves, ... with two register sets in
// turn: while it evaluates one tile, the next tile's rows (and leaf starts)
// are already in flight in the other set. Loads and stores go through buffer
// resources, so a load of a tile past the end (or a store of a lane without a
// leaf) is issued all the same and reads zeros (or is dropped): every
// iteration issues the same memory instructions, the compiler's vmcnt waits
// count exactly the older set (no vmcnt(0) per tile), and no register set is
// copied while its loads are in flight. Per tile and value: the 4-row partial
// sums, a DPP wave scan, the row prefixes into the wave's own LDS slice; lane
// li then forms leaf li's sum as prefix(last row) - prefix(row before its
// first) and stores it (a tile's leaves are consecutive: one coalesced store
// per value). Snapshots with a leaf over 252 rows use the workgroup tally.
struct WaveRsrc {
    __amdgpu_buffer_rsrc_t lab, tn, fr, ex, ls;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint4 rload16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

template <int W, int R>
struct WaveSet {
    RowRegs<W, R> x;
    uint32_t ls_lo, ls_hi;  // lane li: rows of leaf first + li
};

// Issue one tile's loads into `v` (base row `base`; a tile past the end reads
// zeros: off is pushed beyond every resource's range).
template <int W, int R>
__device__ __forceinline__ void wave_issue(const TallyArgs& a, const WaveRsrc& rs, uint32_t base, uint32_t leaf0,
                                           bool live, int lane, WaveSet<W, R>& v) {
    const uint32_t row = base + 4u * (uint32_t)lane;
    const uint32_t bad = live ? 0u : 0x80000000u;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        const uint32_t off = ((uint32_t)w * a.npad + row) * 8u | bad;
        const uint4 u = rload16(rs.lab, off), q = rload16(rs.lab, off + 16u);
        v.x.lab[w][0] = ((uint64_t)u.y << 32) | u.x; v.x.lab[w][1] = ((uint64_t)u.w << 32) | u.z;
        v.x.lab[w][2] = ((uint64_t)q.y << 32) | q.x; v.x.lab[w][3] = ((uint64_t)q.w << 32) | q.z;
    }
    const uint4 t4 = rload16(rs.tn, (row * 4u) | bad);
    v.x.tn[0] = t4.x; v.x.tn[1] = t4.y; v.x.tn[2] = t4.z; v.x.tn[3] = t4.w;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint4 f4 = rload16(rs.fr, (((uint32_t)r * a.npad + row) * 4u) | bad);
        v.x.fr[r][0] = f4.x; v.x.fr[r][1] = f4.y; v.x.fr[r][2] = f4.z; v.x.fr[r][3] = f4.w;
    }
    const uint4 e4 = rload16(rs.ex, (row * 4u) | bad);
    v.x.ex[0] = (int32_t)e4.x; v.x.ex[1] = (int32_t)e4.y; v.x.ex[2] = (int32_t)e4.z; v.x.ex[3] = (int32_t)e4.w;
    // leaf starts: lane li's leaf [ls[leaf0 + li], ls[leaf0 + li + 1]) (beyond the table: zeros)
    const uint32_t lo = ((leaf0 + (uint32_t)lane) * 4u) | bad;
    v.ls_lo = __builtin_amdgcn_raw_buffer_load_b32(rs.ls, lo, 0, 0);
    v.ls_hi = __builtin_amdgcn_raw_buffer_load_b32(rs.ls, lo + 4u, 0, 0);
}

// Evaluate one tile from `v` and store its leaves' sums: NV values, the
// first NV - 1 classes and the occupancy count (compile-time, so every store
// of the unrolled loop is counted by the compiler's waits).
// Class records read through the constant address space: uniform addresses
// become scalar loads (s_load, scalar cache), so a class reaches SGPRs with
// no LDS staging, workgroup barrier or readfirstlane (the wave tally).
#define JSP_CONST __attribute__((address_space(4)))
template <int W, int R>
__device__ __forceinline__ ClassRegs<W, R> class_regs_k(const JSP_CONST DevClass& d) {
    ClassRegs<W, R> k;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        k.req[w] = d.req[w];
        k.mask[w] = d.mask[w];
    }
    k.tol_inv = d.tol_inv;
    k.pods = d.pods;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        k.res[r] = d.res[r];
        k.rcp[r] = d.rcp[r];
    }
    return k;
}

// Evaluate one tile from `v` and keep its leaves' sums: NV values, the first
// NV - 1 classes and the occupancy count (compile-time, so every store of the
// unrolled loop is counted by the compiler's waits). In three batched phases:
// every value's 4-row partial sums, then the NV wave scans (independent DPP
// chains the scheduler interleaves), then all row prefixes into the wave's LDS
// slice behind ONE wave barrier and every leaf's difference read back (one
// LDS round trip per tile instead of one per value). Rows outside the tile's
// leaves are evaluated like any other and not masked: a leaf's sum is
// prefix(its last row) - prefix(the row before its first), and a row before
// the tile's first leaf is in both prefixes, a row after its last leaf in
// neither (the u32 differences are exact: a tile's prefix stays below
// 256 x 2^22 -- pods <= 2^22, checked at class upload).
template <int W, int R, int NV>
__device__ __forceinline__ void wave_eval(const TallyArgs& a, const JSP_CONST DevClass* k_cls, JSP_LDS uint32_t* s_pre, uint4 bt,
                                          int lane, const WaveSet<W, R>& v, uint32_t (&sums)[NV]) {
    constexpr int nc = NV - 1;
    const uint32_t base = bt.z & ~3u;
    const uint32_t nl = bt.y - bt.x;
    const bool has_leaf = (uint32_t)lane < nl;
    uint32_t part[NV][4];  // inclusive sums of the lane's 4 rows, per value
    // re-read the class records per tile (scalar-cache hits): hoisted out of
    // the tile loop, 4 classes' constants overflow the SGPRs and every use
    // becomes a v_readlane of a spill lane
    const JSP_CONST DevClass* kc = k_cls;
    asm volatile("" : "+s"(kc));
#pragma unroll
    for (int c = 0; c < NV; ++c) {
        uint32_t val[4];
        if (c < nc) {
            const ClassRegs<W, R> k = class_regs_k<W, R>(kc[c]);
            uint32_t cap[4];
            row_caps<W, R>(k, v.x.fr, cap);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                bool ok = (v.x.tn[i] & k.tol_inv) == 0;
#pragma unroll
                for (int w = 0; w < W; ++w) ok = ok & ((v.x.lab[w][i] & k.mask[w]) == k.req[w]);
                val[i] = ok ? cap[i] : 0u;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) val[i] = v.x.ex[i] != -1 ? 1u : 0u;
        }
        part[c][0] = val[0];
        part[c][1] = part[c][0] + val[1];
        part[c][2] = part[c][1] + val[2];
        part[c][3] = part[c][2] + val[3];
    }
    uint32_t incl[NV];
#pragma unroll
    for (int c = 0; c < NV; ++c) incl[c] = wave_incl_scan(part[c][3], lane);
#pragma unroll
    for (int c = 0; c < NV; ++c) {
        const uint32_t wex = incl[c] - part[c][3];
        reinterpret_cast<JSP_LDS u32x4*>(s_pre + c * kWaveTileRows)[lane] =
            u32x4{wex + part[c][0], wex + part[c][1], wex + part[c][2], incl[c]};
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t lo = v.ls_lo, hi = v.ls_hi;
    const bool live = has_leaf && lo < hi;
    const bool before = lo > base;
    // a lane without a leaf reads row 0 of each slice (and discards it)
    const uint32_t ih = live ? hi - 1 - base : 0u, ib = live && before ? lo - 1 - base : 0u;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
        const uint32_t hp = s_pre[c * kWaveTileRows + ih];
        const uint32_t bp = s_pre[c * kWaveTileRows + ib];
        sums[c] = live ? hp - (before ? bp : 0u) : 0u;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Store a tile's leaf sums: value c's column is cap[c0 + c][leaf] (occ[leaf]
// for the last); a lane without a leaf stores out of range (dropped). Issued
// after the next tile's loads, so no load waits on these stores' registers.
template <int NV>
__device__ __forceinline__ void wave_store(const TallyArgs& a, __amdgpu_buffer_rsrc_t cap_rsrc,
                                           __amdgpu_buffer_rsrc_t occ_rsrc, uint4 bt, int lane,
                                           const uint32_t (&sums)[NV]) {
    const bool has_leaf = (uint32_t)lane < bt.y - bt.x;
    const uint32_t leaf = a.leaf_base + bt.x + (uint32_t)lane;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
        const uint32_t col = c < NV - 1 ? (a.c0 + (uint32_t)c) * a.ld : 0u;
        const uint32_t off = has_leaf ? (col + leaf) * 4u : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b32(sums[c], c < NV - 1 ? cap_rsrc : occ_rsrc, off, 0, 0);
    }
}

// The tile's leaves' feasibility bits (leaf-level classes: capacity >= pods
// and no rows of other exclusive jobs), set in the class's words: the tile's
// bit range is cleared and its bits or-ed in, in one word or two (every leaf
// belongs to one tile, so after the launch each word is exact; bits past the
// last leaf are never set). Agent-scope atomics: the next launch reads them.
template <int NV>
__device__ __forceinline__ void wave_fold(const TallyArgs& a, const JSP_CONST DevClass* k_cls, uint4 bt, int lane,
                                          const uint32_t (&sums)[NV]) {
    const uint32_t nl = bt.y - bt.x;
    const bool free_leaf = (uint32_t)lane < nl && sums[NV - 1] == 0u;
    const uint32_t gl0 = a.leaf_base + bt.x;
    const uint32_t w0 = gl0 >> 6, sh = gl0 & 63u;
    const uint64_t lmask = nl >= 64u ? ~0ull : ((1ull << nl) - 1ull);
#pragma unroll
    for (int c = 0; c < NV - 1; ++c) {
        const uint32_t pods = k_cls[c].pods;
        const uint64_t m = __ballot(free_leaf && sums[c] >= pods);
        if (lane == 0) {
            uint64_t* f = a.feas_fold + (size_t)(a.c0 + (uint32_t)c) * a.fold_nw + w0;
            __hip_atomic_fetch_and(f, ~(lmask << sh), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_or(f, m << sh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (sh != 0u && sh + nl > 64u) {
                __hip_atomic_fetch_and(f + 1, ~(lmask >> (64u - sh)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_fetch_or(f + 1, m >> (64u - sh), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

template <int W, int R, int NV>
__global__ __launch_bounds__(kTallyThreads) void tally_wave_kernel(TallyArgs a, const uint4* __restrict__ tiles,
                                                                   uint32_t n_tiles, uint32_t n_leaves) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    constexpr int nc = NV - 1;  // this launch: NV - 1 classes and the occupancy count
    constexpr int nv = NV;
    const int tid = threadIdx.x, lane = tid & 63;
    // wave-uniform in SGPRs, so every tile index and descriptor below is scalar
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t waves = gridDim.x * kTallyWaves;
    const uint32_t t0 = blockIdx.x * kTallyWaves + wid;
    // the wave's tiles are t0, t0 + waves, ...: lane k holds the k-th one's
    // descriptor (<= 64, checked by the host), loaded once, so no later tile
    // waits on a descriptor load. No workgroup barrier: the classes are read
    // by scalar loads and each wave has its own LDS slice.
    JSP_WSTAMP(t0, 0);
    if (t0 >= n_tiles) return;
    uint4 dl = make_uint4(0, 0, 0, 0);
    if (t0 + (uint32_t)lane * waves < n_tiles) dl = tiles[t0 + (uint32_t)lane * waves];
    JSP_WSTAMP(t0, 1);
    const uint32_t nt = (n_tiles - t0 + waves - 1) / waves;  // this wave's tiles
    const JSP_CONST DevClass* k_cls = (const JSP_CONST DevClass*)(a.cls + a.c0);
    JSP_LDS uint32_t* s_pre = lds_ptr(lds + wid * nv * kWaveTileRows);
    auto desc = [&](uint32_t k) {
        const int l = (int)(k < nt ? k : nt - 1);
        return make_uint4(__builtin_amdgcn_readlane(dl.x, l), __builtin_amdgcn_readlane(dl.y, l),
                          __builtin_amdgcn_readlane(dl.z, l), __builtin_amdgcn_readlane(dl.w, l));
    };
    const WaveRsrc rs{make_rsrc(a.labels, (uint32_t)W * a.npad * 8u), make_rsrc(a.taints, a.npad * 4u),
                      make_rsrc(a.freer, (uint32_t)R * a.npad * 4u), make_rsrc(a.excl, a.npad * 4u),
                      make_rsrc(a.leaf_start, (n_leaves + 1u) * 4u)};
    const __amdgpu_buffer_rsrc_t cap_r = make_rsrc(a.cap_out, (a.c0 + (uint32_t)nc) * a.ld * 4u);
    const __amdgpu_buffer_rsrc_t occ_r = make_rsrc(a.occ_out, a.do_occ ? a.ld * 4u : 0u);
    WaveSet<W, R> A, B;
    uint32_t kA = 0, kB = 1;
    uint4 btA = desc(kA);
    wave_issue<W, R>(a, rs, btA.z & ~3u, btA.x, true, lane, A);
    // keep set A's loads ahead of set B's: the loop header's waits merge this
    // order with the loop's, and an interleaved prologue would make them wait
    // for nearly every load in flight
    __builtin_amdgcn_sched_barrier(0);
    uint4 btB = desc(kB);
    wave_issue<W, R>(a, rs, btB.z & ~3u, btB.x, kB < nt, lane, B);
    uint32_t sums[NV];
    bool first = true;
    while (true) {
        wave_eval<W, R, NV>(a, k_cls, s_pre, btA, lane, A, sums);
        if (first) JSP_WSTAMP(t0, 2);
        const uint4 done_a = btA;
        kA = kB + 1;
        btA = desc(kA);
        wave_issue<W, R>(a, rs, btA.z & ~3u, btA.x, kA < nt, lane, A);
        wave_store<NV>(a, cap_r, occ_r, done_a, lane, sums);
        if (a.feas_fold) wave_fold<NV>(a, k_cls, done_a, lane, sums);
        if (kB >= nt) break;
#ifdef JSP_STAMPS
        if (first) {  // diagnostic only: the next tile's rows in registers, then time its evaluation alone
            __builtin_amdgcn_s_waitcnt(0);
            JSP_WSTAMP(t0, 3);
            JSP_WCLK(t0, 6);
        }
#endif
        wave_eval<W, R, NV>(a, k_cls, s_pre, btB, lane, B, sums);
        if (first) {
            JSP_WSTAMP(t0, 4);
            JSP_WCLK(t0, 7);
        }
        first = false;
        const uint4 done_b = btB;
        kB = kA + 1;
        btB = desc(kB);
        wave_issue<W, R>(a, rs, btB.z & ~3u, btB.x, kB < nt, lane, B);
        wave_store<NV>(a, cap_r, occ_r, done_b, lane, sums);
        if (a.feas_fold) wave_fold<NV>(a, k_cls, done_b, lane, sums);
        if (kA >= nt) break;
    }
    JSP_WSTAMP(t0, 5);
}

// One tile per wave (the grid covers every tile): a single register set, no
// descriptor table in lanes -- the tile's descriptor is one scalar load -- so
// the kernel holds fewer VGPRs and more waves stay resident per SIMD to hide
// each other's row latency and evaluation.
template <int W, int R, int NV>
__global__ __launch_bounds__(kTallyThreads) void tally_wave1_kernel(TallyArgs a, const uint4* __restrict__ tiles,
                                                                    uint32_t n_tiles, uint32_t n_leaves) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    constexpr int nc = NV - 1;
    constexpr int nv = NV;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t t = blockIdx.x * kTallyWaves + wid;
    if (t >= n_tiles) return;
#ifdef JSP_AB_FAKE_DESC
    // diagnostic A/B build only (wrong sums): the descriptor from the tile
    // index (12 leaves in 252 rows, cfg4's shape), no dependent load before
    // the rows -- what a fixed-window tiling would save cold
    (void)tiles;
    const uint32_t fl0 = t * 12u < n_leaves ? t * 12u : n_leaves;
    const uint4 bt = make_uint4(fl0, fl0 + 12u < n_leaves ? fl0 + 12u : n_leaves, t * 252u, t * 252u + 252u);
#else
    const uint4 bt = tiles[t];
#endif
    const uint64_t t_in = a.wstamps ? wall_clock64() : 0ull;
    const JSP_CONST DevClass* k_cls = (const JSP_CONST DevClass*)(a.cls + a.c0);
    JSP_LDS uint32_t* s_pre = lds_ptr(lds + wid * nv * kWaveTileRows);
    const WaveRsrc rs{make_rsrc(a.labels, (uint32_t)W * a.npad * 8u), make_rsrc(a.taints, a.npad * 4u),
                      make_rsrc(a.freer, (uint32_t)R * a.npad * 4u), make_rsrc(a.excl, a.npad * 4u),
                      make_rsrc(a.leaf_start, (n_leaves + 1u) * 4u)};
    const __amdgpu_buffer_rsrc_t cap_r = make_rsrc(a.cap_out, (a.c0 + (uint32_t)nc) * a.ld * 4u);
    const __amdgpu_buffer_rsrc_t occ_r = make_rsrc(a.occ_out, a.do_occ ? a.ld * 4u : 0u);
    WaveSet<W, R> A;
    wave_issue<W, R>(a, rs, bt.z & ~3u, bt.x, true, lane, A);
    uint32_t sums[NV];
    wave_eval<W, R, NV>(a, k_cls, s_pre, bt, lane, A, sums);
    wave_store<NV>(a, cap_r, occ_r, bt, lane, sums);
    if (a.feas_fold) wave_fold<NV>(a, k_cls, bt, lane, sums);
    if (a.wstamps) {  // the span probe: this wave's start and end (its stores drained)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) {
            a.wstamps[2 * t] = t_in;
            a.wstamps[2 * t + 1] = wall_clock64();
        }
    }
}

// ----------------------------------------------------------------- feasibility
// Bit d of class c's word w: capsum(c, d) >= pods[c] && occsum(d) == 0 over the
// leaves of domain d = 64w + lane at level lvl. One wave computes one word.
__device__ __forceinline__ uint64_t feas_word(const uint32_t* __restrict__ cap, const uint32_t* __restrict__ occ,
                                              uint32_t ld, uint32_t lvl, uint32_t pods, uint32_t c, uint32_t w,
                                              const TopoDev& topo, int lane) {
    const uint32_t d = w * 64 + lane;
    bool ok = false;
    if (d < topo.D[lvl]) {
        uint32_t lo = d, hi = d + 1;
        if (lvl + 1 < topo.K) { lo = topo.fl[lvl][d]; hi = topo.fl[lvl][d + 1]; }
        uint64_t cs = 0, os = 0;
        const uint32_t* cp = cap + (size_t)c * ld;
        for (uint32_t leaf = lo; leaf < hi; ++leaf) { cs += cp[leaf]; os += occ[leaf]; }
        ok = (cs >= pods) && (os == 0);
    }
    return __ballot(ok);
}

// Inclusive wave64 prefix sum of a 64-bit value: the DPP steps of
// wave_incl_scan on both halves, carry propagated from the low half.
__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t x) {
    uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
#define JSP_SCAN64_STEP(CTRL, RM)                                                              \
    {                                                                                          \
        const uint32_t a = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, CTRL, RM, 0xf, false); \
        const uint32_t b = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, CTRL, RM, 0xf, false); \
        const uint32_t n = lo + a;                                                             \
        hi += b + (n < lo ? 1u : 0u);                                                          \
        lo = n;                                                                                \
    }
    JSP_SCAN64_STEP(0x111, 0xf)
    JSP_SCAN64_STEP(0x112, 0xf)
    JSP_SCAN64_STEP(0x114, 0xf)
    JSP_SCAN64_STEP(0x118, 0xf)
    JSP_SCAN64_STEP(0x142, 0xa)
    JSP_SCAN64_STEP(0x143, 0xc)
#undef JSP_SCAN64_STEP
    return ((uint64_t)hi << 32) | lo;
}

// Feasibility word w of class c at a level above the leaves. Lane i owns
// domain 64w + i with leaves [lo_i, hi_i); the word's leaves [A, B) are one
// contiguous range, which the wave streams in coalesced 64-leaf chunks
// (kUpperBatch chunks of loads in flight at once). A 64-bit running prefix of
// min(cap, pods) — the clamp keeps `capsum >= pods` exact — and a 32-bit one of
// occ give each lane P(hi_i) when hi_i falls in a chunk; P(lo_i) is the
// previous lane's P(hi). One pass, no per-domain serial loops, so a zone of
// thousands of racks costs ~(leaves / 512) memory round trips, not one per leaf.
constexpr int kUpperBatch = 8;
__device__ __forceinline__ uint64_t feas_word_upper(const uint32_t* __restrict__ cap, const uint32_t* __restrict__ occ, uint32_t ld,
                                    uint32_t lvl, uint32_t pods, uint32_t c, uint32_t w, const TopoDev& topo,
                                    int lane) {
    const uint32_t D = topo.D[lvl];
    const uint32_t d0 = w * 64;
    const uint32_t nd = (D - d0) < 64u ? (D - d0) : 64u;
    const uint32_t* fl = topo.fl[lvl];
    const uint32_t hi_i = (uint32_t)lane < nd ? fl[d0 + lane + 1] : 0u;
    const uint32_t A = fl[d0];
    const uint32_t B = (uint32_t)__builtin_amdgcn_readlane((int)hi_i, (int)nd - 1);
    const uint32_t* cp = cap + (size_t)c * ld;
    uint64_t carry = 0, p_hi = 0;
    uint32_t ocarry = 0, o_hi = 0;
    for (uint32_t base = A; base < B; base += 64u * kUpperBatch) {
        uint32_t v[kUpperBatch], o[kUpperBatch];
#pragma unroll
        for (int u = 0; u < kUpperBatch; ++u) {
            const uint32_t leaf = base + 64u * u + (uint32_t)lane;
            v[u] = 0;
            o[u] = 0;
            if (leaf < B) {
                const uint32_t x = cp[leaf];
                v[u] = x < pods ? x : pods;
                o[u] = occ[leaf];
            }
        }
#pragma unroll
        for (int u = 0; u < kUpperBatch; ++u) {
            const uint32_t sb = base + 64u * u;
            if (sb >= B) break;  // wave-uniform
            const uint64_t s = wave_incl_scan64(v[u]);
            const uint32_t os = wave_incl_scan(o[u], lane);
            // P(hi_i) = carry + s[hi_i - 1 - sb] when hi_i in (sb, sb + 64]
            const bool mine = hi_i > sb && hi_i <= sb + 64u;
            const int src = mine ? (int)(hi_i - 1 - sb) : 0;
            const uint32_t slo = (uint32_t)__shfl((int)(uint32_t)s, src, 64);
            const uint32_t shi = (uint32_t)__shfl((int)(uint32_t)(s >> 32), src, 64);
            const uint32_t so = (uint32_t)__shfl((int)os, src, 64);
            if (mine) {
                p_hi = carry + (((uint64_t)shi << 32) | slo);
                o_hi = ocarry + so;
            }
            carry += ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(s >> 32), 63) << 32) |
                     (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)s, 63);
            ocarry += (uint32_t)__builtin_amdgcn_readlane((int)os, 63);
        }
    }
    // P(lo_i) = P(hi_{i-1}); P(A) = 0. Empty domains read equal prefixes.
    const uint32_t plo_l = (uint32_t)__shfl_up((int)(uint32_t)p_hi, 1, 64);
    const uint32_t plo_h = (uint32_t)__shfl_up((int)(uint32_t)(p_hi >> 32), 1, 64);
    const uint32_t olo_s = (uint32_t)__shfl_up((int)o_hi, 1, 64);
    const uint64_t p_lo = lane == 0 ? 0ull : (((uint64_t)plo_h << 32) | plo_l);
    const uint32_t o_lo = lane == 0 ? 0u : olo_s;
    const bool ok = (uint32_t)lane < nd && (p_hi - p_lo) >= pods && (o_hi - o_lo) == 0u;
    return __ballot(ok);
}

// Word w of class c at its level, leaves or above.
__device__ __forceinline__ uint64_t feas_word_any(const uint32_t* __restrict__ cap, const uint32_t* __restrict__ occ,
                                                  uint32_t ld, uint32_t lvl, uint32_t pods, uint32_t c, uint32_t w,
                                                  const TopoDev& topo, int lane) {
    if (lvl + 1 < topo.K) return feas_word_upper(cap, occ, ld, lvl, pods, c, w, topo, lane);
    return feas_word(cap, occ, ld, lvl, pods, c, w, topo, lane);
}

__global__ __launch_bounds__(256) void feas_kernel(const uint32_t* __restrict__ cap,
                                                   const uint32_t* __restrict__ occ, uint32_t ld,
                                                   const DevClass* __restrict__ cls, uint32_t C,
                                                   const uint32_t* __restrict__ word_off, TopoDev topo,
                                                   uint64_t* __restrict__ feas) {
    const int lane = threadIdx.x & 63;
    const uint32_t gw = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (gw >= word_off[C]) return;
    uint32_t c = 0;
    while (word_off[c + 1] <= gw) ++c;  // wave-uniform, C <= 64
    const uint64_t word = feas_word_any(cap, occ, ld, cls[c].level, cls[c].pods, c, gw - word_off[c], topo, lane);
    if (lane == 0) feas[gw] = word;
}

// ----------------------------------------------------------------- A7 assignment (one workgroup)
__device__ __forceinline__ void lds_set_bit(uint64_t* t, uint32_t d) {
    atomicOr(reinterpret_cast<unsigned long long*>(&t[d >> 6]), 1ull << (d & 63));
}

__device__ void lds_set_range(uint64_t* t, uint32_t lo, uint32_t hi) {
    while (lo < hi) {
        const uint32_t w = lo >> 6, b = lo & 63;
        const uint32_t n = (hi - lo) < (64 - b) ? (hi - lo) : (64 - b);
        const uint64_t m = (n == 64) ? ~0ull : (((1ull << n) - 1) << b);
        atomicOr(reinterpret_cast<unsigned long long*>(&t[w]), (unsigned long long)m);
        lo += n;
    }
}

// Block-wide exclusive scan with ONE barrier: each wave publishes its total
// in region `slot` of s_w, then every wave combines the NT/64 totals itself
// (lanes < NT/64 read them) instead of waiting for wave 0 to scan them behind
// a second barrier. A region is free again after the next barrier, so two
// scans with no barrier between them use different slots (0, 1).
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t* s_w, uint32_t* total, int slot = 0) {
    constexpr int NW = NT / 64;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    uint32_t* w = s_w + slot * NW;
    const uint32_t incl = wave_incl_scan(x, lane);
    if (lane == 63) w[wid] = incl;
    __syncthreads();
    const uint32_t v = lane < NW ? w[lane] : 0u;
    const uint32_t sc = wave_incl_scan(v, lane);
    *total = (uint32_t)__builtin_amdgcn_readlane((int)sc, NW - 1);
    const uint32_t before = wid > 0 ? (uint32_t)__builtin_amdgcn_readlane((int)sc, wid - 1) : 0u;
    return before + incl - x;
}

// Small LDS tables of the assignment (all filled in one round of loads):
// per class its level, pods, bitmap word offset and cursor; per level the
// offset of its taken bitmap (computed from topo.D, no memory).
struct AssignMeta {
    uint32_t* s_w;       // 2*NW + 4 (block scans: two NW-word slots)
    uint32_t* s_misc;    // 4
    uint32_t* s_cursor;  // kMaxClasses
    uint32_t* s_lvl;     // kMaxClasses
    uint32_t* s_pods;    // kMaxClasses
    uint32_t* s_woff;    // kMaxClasses + 1
    uint32_t* s_toff;    // 8
    uint32_t* s_D;       // 8: domains per level
    uint32_t* s_poff;    // 8: parent[k] offset in the LDS topology tables
    uint32_t* s_coff;    // 8: child_start[k] offset in the LDS topology tables
    uint32_t* s_rc;      // NT run classes (tile)
    uint32_t* s_ro;      // NT run job offsets (tile)
    uint32_t* s_long;    // NT indices of the tile's long runs
    uint32_t* s_bcls;    // 64: class of each run start of a wave-0 batch (job offset -> class)
};

template <int NT>
__device__ __forceinline__ AssignMeta carve_meta(uint32_t* s_small) {
    constexpr int NW = NT / 64;
    AssignMeta m;
    m.s_w = s_small;
    m.s_misc = m.s_w + 2 * NW + 4;
    m.s_cursor = m.s_misc + 4;
    m.s_lvl = m.s_cursor + kMaxClasses;
    m.s_pods = m.s_lvl + kMaxClasses;
    m.s_woff = m.s_pods + kMaxClasses;
    m.s_toff = m.s_woff + kMaxClasses + 1;
    m.s_D = m.s_toff + 8;
    m.s_poff = m.s_D + 8;
    m.s_coff = m.s_poff + 8;
    m.s_rc = m.s_coff + 8;
    m.s_ro = m.s_rc + NT;
    m.s_long = m.s_ro + NT;
    m.s_bcls = m.s_long + NT;
    return m;
}

// Issue every small-table load at once (no barrier inside: the caller's next
// barrier publishes them).
template <int NT>
__device__ __forceinline__ void stage_meta(const AssignMeta& m, const DevClass* __restrict__ cls, uint32_t C,
                                           const uint32_t* __restrict__ word_off, const TopoDev& topo) {
    const int tid = threadIdx.x;
    for (uint32_t i = tid; i < C; i += NT) {
        m.s_cursor[i] = 0;
        m.s_lvl[i] = cls[i].level;
        m.s_pods[i] = cls[i].pods;
    }
    for (uint32_t i = tid; i <= C; i += NT) m.s_woff[i] = word_off[i];
    if (tid == 0) {
        uint32_t off = 0, t = 0;
        for (uint32_t k = 0; k < topo.K; ++k) {
            m.s_toff[k] = off;
            m.s_D[k] = topo.D[k];
            off += (topo.D[k] + 63) >> 6;
            if (k >= 1) { m.s_poff[k] = t; t += topo.D[k]; }
            if (k + 1 < topo.K) { m.s_coff[k] = t; t += topo.D[k] + 1; }
        }
        m.s_toff[topo.K] = off;
    }
}

// Copy the hierarchy tables into LDS (no barrier inside).
template <int NT>
__device__ __forceinline__ void stage_topo(uint32_t* s_topo, const TopoDev& topo) {
    uint32_t t = 0;
    for (uint32_t k = 0; k < topo.K; ++k) {
        if (k >= 1) {
            for (uint32_t i = threadIdx.x; i < topo.D[k]; i += NT) s_topo[t + i] = (uint32_t)topo.par[k][i];
            t += topo.D[k];
        }
        if (k + 1 < topo.K) {
            for (uint32_t i = threadIdx.x; i <= topo.D[k]; i += NT) s_topo[t + i] = topo.cs[k][i];
            t += topo.D[k] + 1;
        }
    }
}

__device__ __forceinline__ uint32_t taken_words(const TopoDev& topo) {
    uint32_t off = 0;
    for (uint32_t k = 0; k < topo.K; ++k) off += (topo.D[k] + 63) >> 6;
    return off;
}

// Taking domain d at level lvl also takes, at every other level, each domain
// whose leaf range intersects d's: its ancestors (one bit per level) and its
// descendants (a bit range per level). LDS atomics: other lanes may mark the
// same words. The hierarchy tables are read from LDS when staged there.
template <bool TOPO_LDS>
__device__ __forceinline__ void mark_other_levels(uint32_t d, uint32_t lvl, uint32_t K, const TopoDev& topo,
                                                  uint64_t* s_taken, const AssignMeta& m, const uint32_t* s_topo) {
    uint32_t dd = d;  // ancestors
    for (int kk = (int)lvl - 1; kk >= 0; --kk) {
        if constexpr (TOPO_LDS) dd = s_topo[m.s_poff[kk + 1] + dd];
        else dd = (uint32_t)topo.par[kk + 1][dd];
        lds_set_bit(s_taken + m.s_toff[kk], dd);
    }
    uint32_t lo = d, hi = d + 1;  // descendants
    for (uint32_t kk = lvl + 1; kk < K; ++kk) {
        if constexpr (TOPO_LDS) {
            const uint32_t* cs = s_topo + m.s_coff[kk - 1];
            lo = cs[lo];
            hi = cs[hi];
        } else {
            lo = topo.cs[kk - 1][lo];
            hi = topo.cs[kk - 1][hi];
        }
        lds_set_range(s_taken + m.s_toff[kk], lo, hi);
    }
}

// Position of the r-th (0-based) set bit of x; r < popcount(x).
__device__ __forceinline__ uint32_t select_bit(uint64_t x, uint32_t r) {
    uint32_t pos = 0;
    uint32_t c = (uint32_t)__popc((uint32_t)x);
    if (r >= c) { r -= c; x >>= 32; pos += 32; }
    c = (uint32_t)__popc((uint32_t)x & 0xFFFFu);
    if (r >= c) { r -= c; x >>= 16; pos += 16; }
    c = (uint32_t)__popc((uint32_t)x & 0xFFu);
    if (r >= c) { r -= c; x >>= 8; pos += 8; }
    c = (uint32_t)__popc((uint32_t)x & 0xFu);
    if (r >= c) { r -= c; x >>= 4; pos += 4; }
    c = (uint32_t)__popc((uint32_t)x & 0x3u);
    if (r >= c) { r -= c; x >>= 2; pos += 2; }
    c = (uint32_t)(x & 1u);
    if (r >= c) pos += 1;
    return pos;
}

// Runs with at most this many jobs are placed by wave 0 alone: no workgroup
// barrier, a 64-word (4096-domain) window per step, per-class state in wave
// 0's registers (lane c holds class c). Longer runs use the whole workgroup on
// an NT-word window per step.
constexpr uint32_t kWaveRunMax = 64;

// One long run (jobs [j0, jend) of class c), executed by every wave of the
// workgroup. Per step: a block scan gives each window word its first rank;
// each word's owner marks what the step takes from it; every thread then
// emits an equal share of the step's ranks (merge-path split: binary search
// of its first rank over the word ranks, select of the bit, then a walk)
// into LDS in rank order; the ranks leave for assign[] in coalesced stores.
// Returns the class's new cursor.
template <int NT, bool TOPO_LDS>
__device__ uint32_t long_run(uint32_t c, uint32_t j0, uint32_t jend, const uint64_t* __restrict__ feas,
                             const TopoDev& topo, int32_t* __restrict__ assign, uint64_t* s_taken,
                             const AssignMeta& m, const uint32_t* s_topo, uint64_t* s_win, uint32_t* s_stage,
                             uint32_t stage_cap, AssignRec* __restrict__ recs, uint32_t& placed) {
    const int tid = threadIdx.x;
    const uint32_t K = topo.K;
    uint32_t* s_wpre = reinterpret_cast<uint32_t*>(s_win + NT);
    __syncthreads();  // wave 0's short-run state (taken words, cursors) visible
    JSP_STAMP(4001u + (c & 7u), 0);
    const uint32_t lvl = m.s_lvl[c];
    const uint32_t D = m.s_D[lvl];
    const uint32_t nw = (D + 63) >> 6;
    uint64_t* Tk = s_taken + m.s_toff[lvl];
    const uint64_t* F = feas + m.s_woff[c];
    uint32_t cur = m.s_cursor[c];
    uint32_t need = jend - j0, jpos = j0;
    while (need > 0 && cur < D) {
        const uint32_t cap = (recs != nullptr || need < stage_cap) ? need : stage_cap;
        const uint32_t wb0 = cur >> 6;
        const uint32_t w = wb0 + tid;
        uint64_t bits = 0;
        if (w < nw) {
            bits = F[w] & ~Tk[w];
            if (w == wb0) bits &= ~0ull << (cur & 63);
        }
        const uint32_t cnt = (uint32_t)__popcll(bits);
        // one scan counts both the ranks (low 20 bits: <= 64 NT) and the words
        // holding any (high bits): a record's slot is its word's rank among the
        // nonzero words, as the taking words are the first nonzero ones
        const uint32_t rec_base = recs != nullptr ? m.s_misc[1] : 0u;  // read before the scan's barriers
        uint32_t total_p;
        const uint32_t pre_p = block_excl_scan<NT>(cnt | (cnt != 0u ? 1u << 20 : 0u), m.s_w, &total_p);
        const uint32_t pre = pre_p & 0xFFFFFu, total = total_p & 0xFFFFFu;
        JSP_STAMP(4001u + (c & 7u), 1);
        const uint32_t used = total < cap ? total : cap;
        // the owner of each word marks the ranks [pre, min(pre + cnt, used)) taken
        uint64_t took = 0;
        if (cnt != 0 && pre < used) {
            took = pre + cnt <= used ? bits : bits & ((1ull << select_bit(bits, used - pre)) - 1ull);
            Tk[w] |= took;
        }
        if (recs != nullptr) {
            // record mode: one {word, first job, taken bits} record per word that
            // gives domains away; expand_kernel turns them into assign[] with the
            // whole GPU. The last taking word publishes the next record base.
            if (took != 0) {
                const uint32_t slot = rec_base + (pre_p >> 20);
                if (pre + cnt >= used) m.s_misc[1] = slot + 1u;
                AssignRec r;
                r.dom0 = w * 64;
                r.base = jpos + pre;
                r.took = took;
                recs[slot] = r;
                if (K > 1) {
                    uint64_t x = took;
                    while (x) {
                        mark_other_levels<TOPO_LDS>(w * 64 + (uint32_t)__builtin_ctzll(x), lvl, K, topo, s_taken, m,
                                                    s_topo);
                        x &= x - 1;
                    }
                }
                if (pre + cnt >= used) m.s_misc[0] = w * 64 + 64 - (uint32_t)__builtin_clzll(took);  // last taken + 1
            }
            __syncthreads();
            cur = total >= cap ? m.s_misc[0] : (wb0 + NT) * 64u;
            need -= used;
            jpos += used;
            placed += used;
            continue;  // the next step's scan barriers order s_misc[0] reuse
        }
        s_win[tid] = bits;
        s_wpre[tid] = pre;
        __syncthreads();
        JSP_STAMP(4001u + (c & 7u), 2);
        // this thread's share of the ranks: [i0, i1)
        const uint32_t i0 = (uint32_t)(((uint64_t)tid * used) / NT);
        const uint32_t i1 = (uint32_t)(((uint64_t)(tid + 1) * used) / NT);
        if (i0 < i1) {
            uint32_t lo = 0, hi = NT;  // last word k with s_wpre[k] <= i0: it holds rank i0
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_wpre[mid] <= i0) lo = mid; else hi = mid;
            }
            uint32_t k = lo;
            uint64_t x = s_win[k];
            x &= ~0ull << select_bit(x, i0 - s_wpre[k]);
            for (uint32_t i = i0; i < i1; ++i) {
                while (x == 0) x = s_win[++k];
                const uint32_t d = (wb0 + k) * 64 + (uint32_t)__builtin_ctzll(x);
                x &= x - 1;
                s_stage[i] = d;
                if (K > 1) mark_other_levels<TOPO_LDS>(d, lvl, K, topo, s_taken, m, s_topo);
                if (i + 1 == used) m.s_misc[0] = d + 1;
            }
        }
        __syncthreads();
        JSP_STAMP(4001u + (c & 7u), 3);
        for (uint32_t i = tid; i < used; i += NT) assign[jpos + i] = (int32_t)s_stage[i];
        cur = total >= cap ? m.s_misc[0] : (wb0 + NT) * 64u;
        need -= used;
        jpos += used;
        placed += used;
        __syncthreads();  // window, stage and s_misc free again
        JSP_STAMP(4001u + (c & 7u), 4);
    }
    for (uint32_t j = jpos + tid; j < jend; j += NT) assign[j] = -1;
    JSP_STAMP(4001u + (c & 7u), 5);
    return cur < D ? cur : D;
}

// ---- register-resident walker for small hierarchies: when the taken
// bitmaps of all levels together are <= 64 words (s_taken's layout: level k at
// words [toff_k, toff_k + nw_k)), wave 0 keeps them in one register, lane w =
// word w, so a short run touches no LDS state. The only memory access per job
// is its class's feasibility word, loaded one run ahead. Taking a domain marks
// its descendants at once (ranges from the child_start tables); its ancestors
// are marked lazily: taken bits below level 0 stay pending until a job at a
// coarser level, or a long run, needs them, and are then folded upwards (one
// parent lookup per distinct parent per word) through the LDS image s_taken.
constexpr uint32_t kRegMaxWords = 64;

struct RegState {
    uint64_t T;  // taken (lane w: word w of the concatenated level bitmaps)
    uint64_t P;  // taken directly at a level >= 1, ancestors not yet marked
    int pend;    // highest level with pending bits, -1 none (wave-uniform)
};

// bits of [lo, hi) in word `wi` (domains [64 wi, 64 wi + 64))
__device__ __forceinline__ uint64_t range_word(uint32_t wi, uint32_t lo, uint32_t hi) {
    const uint32_t w0 = wi * 64, a = lo > w0 ? lo : w0, b = hi < w0 + 64 ? hi : w0 + 64;
    if (a >= b) return 0ull;
    const uint32_t n = b - a;
    return (n == 64 ? ~0ull : ((1ull << n) - 1ull)) << (a - w0);
}

template <bool TOPO_LDS>
__device__ __forceinline__ uint32_t topo_cs(const TopoDev& topo, const uint32_t* s_topo, const AssignMeta& m,
                                            uint32_t k, uint32_t i) {
    if constexpr (TOPO_LDS) return s_topo[m.s_coff[k] + i];
    else return topo.cs[k][i];
}

template <bool TOPO_LDS>
__device__ __forceinline__ uint32_t topo_par(const TopoDev& topo, const uint32_t* s_topo, const AssignMeta& m,
                                             uint32_t k, uint32_t i) {
    if constexpr (TOPO_LDS) return s_topo[m.s_poff[k] + i];
    else return (uint32_t)topo.par[k][i];
}

// Mark the descendants of every taken bit of `took` (level lvl, its words at
// lanes [t0, ...)) at all finer levels: contiguous taken bits of one word are
// one domain range, whose descendants are one range per level.
template <bool TOPO_LDS>
__device__ void reg_mark_desc(RegState& s, uint64_t took, uint32_t lvl, uint32_t t0, uint32_t K, const TopoDev& topo,
                              const uint32_t* s_topo, const AssignMeta& m, int lane) {
    uint64_t lanes = __ballot(took != 0);
    while (lanes) {
        const int k = __builtin_ctzll(lanes);
        lanes &= lanes - 1;
        uint64_t word = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(took >> 32), k) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)took, k);
        while (word) {
            const uint32_t b = (uint32_t)__builtin_ctzll(word);
            const uint64_t sh = word >> b;
            const uint32_t len = ~sh == 0ull ? 64u - b : (uint32_t)__builtin_ctzll(~sh);
            word &= len >= 64u ? 0ull : ~(((1ull << len) - 1ull) << b);
            uint32_t lo = ((uint32_t)k - t0) * 64 + b, hi = lo + len;
            for (uint32_t kk = lvl + 1; kk < K; ++kk) {
                lo = topo_cs<TOPO_LDS>(topo, s_topo, m, kk - 1, lo);
                hi = topo_cs<TOPO_LDS>(topo, s_topo, m, kk - 1, hi);
                const uint32_t tk = m.s_toff[kk], nwk = (m.s_D[kk] + 63) >> 6;
                const uint32_t wi = (uint32_t)lane - tk;
                if (wi < nwk) s.T |= range_word(wi, lo, hi);
            }
        }
    }
}

// Fold the pending bits into their ancestors, finest level first, so marks
// made at level k-1 propagate further up. Lanes scatter the ancestor bits
// into other lanes' words with LDS atomics on the image s_taken (written from
// the register first, read back after); one parent lookup per distinct parent
// per word (parents are monotone: skip the bits below the next parent's first
// child).
template <bool TOPO_LDS>
__device__ void reg_flush(RegState& s, uint32_t K, const TopoDev& topo, uint64_t* s_taken, uint32_t t_words,
                          const uint32_t* s_topo, const AssignMeta& m, int lane) {
    if ((uint32_t)lane < t_words) s_taken[lane] = s.T;
    for (uint32_t kk = K - 1; kk >= 1; --kk) {
        const uint32_t tk = m.s_toff[kk], nwk = (m.s_D[kk] + 63) >> 6;
        const uint32_t wi = (uint32_t)lane - tk;
        uint64_t pb = wi < nwk ? s.P : 0ull;
        if (__ballot(pb != 0) == 0) continue;
        const uint32_t tu = m.s_toff[kk - 1], nwu = (m.s_D[kk - 1] + 63) >> 6;
        const uint64_t before = s.T;
        while (__ballot(pb != 0)) {
            if (pb) {
                const uint32_t d = wi * 64 + (uint32_t)__builtin_ctzll(pb);
                const uint32_t p = topo_par<TOPO_LDS>(topo, s_topo, m, kk, d);
                lds_set_bit(s_taken + tu, p);
                const uint32_t end = topo_cs<TOPO_LDS>(topo, s_topo, m, kk - 1, p + 1);  // p's children end
                const uint32_t w0 = wi * 64;
                pb = end >= w0 + 64 ? 0ull : pb & (~0ull << (end - w0));
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if ((uint32_t)lane < t_words) s.T = s_taken[lane];
        if (wi < nwk) s.P = 0;  // level kk done
        const uint32_t wu = (uint32_t)lane - tu;
        if (kk - 1 >= 1 && wu < nwu) s.P |= s.T & ~before;  // new marks propagate further up
        if (kk == 1) break;
    }
    s.pend = -1;
}

// Scalar chain of a dense word, unrolled: packed lane k (< n) holds the k-th
// visiting job's class word (bits 0..62); job k takes the lowest bit of it not
// yet taken, and its lane of `res` gets the bit (-1: none). Lanes >= n hold 0:
// their s_ff1 gives -1 and the s_bitset1 after it sets bit 63, which no job's
// word holds (the caller clears it and settles bit 63 itself).
#define JSP_CHAIN_STEP(K)                                                                                 \
    do {                                                                                                  \
        const uint64_t g_ = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)gh, (K)) << 32) |         \
                            (uint32_t)__builtin_amdgcn_readlane((int)gl, (K));                            \
        uint64_t t_;                                                                                      \
        int32_t b_;                                                                                       \
        asm("s_andn2_b64 %[t], %[g], %[tk]\n\t"                                                          \
            "s_ff1_i32_b64 %[b], %[t]\n\t"                                                               \
            "s_bitset1_b64 %[tk], %[b]"                                                                   \
            : [tk] "+s"(taken), [t] "=&s"(t_), [b] "=&s"(b_)                                              \
            : [g] "s"(g_)                                                                                 \
            : "scc");                                                                                     \
        asm("v_writelane_b32 %0, %1, %2" : "+v"(res) : "s"(b_), "i"(K));                                  \
    } while (0)
#define JSP_CHAIN_8(B)                                                                                    \
    JSP_CHAIN_STEP((B) + 0); JSP_CHAIN_STEP((B) + 1); JSP_CHAIN_STEP((B) + 2); JSP_CHAIN_STEP((B) + 3);   \
    JSP_CHAIN_STEP((B) + 4); JSP_CHAIN_STEP((B) + 5); JSP_CHAIN_STEP((B) + 6); JSP_CHAIN_STEP((B) + 7)

__device__ __forceinline__ void chain_unrolled(uint32_t gl, uint32_t gh, uint32_t n, uint64_t& taken, int32_t& res) {
    JSP_CHAIN_8(0);
    if (n <= 8) return;
    JSP_CHAIN_8(8);
    if (n <= 16) return;
    JSP_CHAIN_8(16);
    if (n <= 24) return;
    JSP_CHAIN_8(24);
    if (n <= 32) return;
    JSP_CHAIN_8(32);
    if (n <= 40) return;
    JSP_CHAIN_8(40);
    if (n <= 48) return;
    JSP_CHAIN_8(48);
    if (n <= 56) return;
    JSP_CHAIN_8(56);
}
#undef JSP_CHAIN_8
#undef JSP_CHAIN_STEP
constexpr uint32_t kChainUnrollMin = 6;
#ifndef JSP_PIPE_WAVES
#define JSP_PIPE_WAVES 4
#endif
constexpr uint32_t kPipeWaves = JSP_PIPE_WAVES;    // waves of the pipelined batch walk

// One word of a batch (wave-wide): lane c holds class c's free feasible bits
// `g` of word w; the batch's jobs still without a domain (R; lane j = job j of
// class `cls`) take, in job order, the lowest free bit of their class's word.
// Job lanes that took one get res = 64 w + bit and leave R; returns the bits
// taken.
__device__ __forceinline__ uint64_t walk_word(uint64_t g, uint32_t cls, bool job, uint64_t& R, int32_t& res, uint32_t w,
                                              int lane) {
    // job lane j: its class's word
    const uint32_t gl = (uint32_t)__shfl((int)(uint32_t)g, (int)cls);
    const uint32_t gh = (uint32_t)__shfl((int)(uint32_t)(g >> 32), (int)cls);
    const uint64_t gj = ((uint64_t)gh << 32) | gl;
    const uint64_t V0 = R & __ballot(job && gj != 0ull);  // jobs that can take something here
    if (V0 == 0ull) return 0ull;
    // The chain runs on bits 0..62: s_ff1 of an empty word is -1, and the
    // s_bitset1 that follows then sets bit 63, which the chain never reads.
    // Bit 63 goes afterwards to the first visited job left without a domain
    // whose class has it (job order inside the word: it is the word's last
    // domain, so only jobs that found nothing below it can want it).
    const uint32_t gh62 = gh & 0x7FFFFFFFu;
    uint64_t taken = 0;
    int32_t wres = -1;
    const uint32_t nv = (uint32_t)__popcll(V0);
    if (nv >= kChainUnrollMin) {
        // Dense word: the visiting jobs' class words are packed into
        // lanes 0..nv-1 (job order), then an unrolled chain reads
        // them with constant-lane readlanes and writes each result
        // into its packed lane: per job two readlanes, and-not,
        // lowest-bit, bit-set and one writelane -- half the
        // instructions of the loop below, no loop control.
        // (the permutes run on every lane: a source lane outside a
        // branch's exec mask would read as 0)
        const uint32_t src = (uint32_t)lane < nv ? select_bit(V0, (uint32_t)lane) : 0u;
        const uint32_t pgl = (uint32_t)__shfl((int)gl, (int)src);
        const uint32_t pgh = (uint32_t)__shfl((int)gh62, (int)src);
        const uint32_t cgl = (uint32_t)lane < nv ? pgl : 0u;
        const uint32_t cgh = (uint32_t)lane < nv ? pgh : 0u;
        int32_t cres = -1;
        chain_unrolled(cgl, cgh, nv, taken, cres);
        const uint32_t pos = mbcnt64(V0);
        const int32_t back = __shfl(cres, (int)(pos & 63u));
        if ((V0 >> lane) & 1ull) wres = back;
    } else {
    uint64_t V = V0;
    // software-pipelined: the next job's class word is read (two
    // readlanes) before the current job's scalar chain runs. Measured
    // ~100 shader cycles per job visit (tools/stamps_words.py): about
    // 7 per instruction of the 14-instruction loop on one wave; a
    // two-job unroll compiled to the same count per job.
    uint32_t j;  // current job: lowest bit of V, cleared
    asm("s_ff1_i32_b64 %[j], %[V]\n\t"
        "s_bitset0_b64 %[V], %[j]"
        : [V] "+s"(V), [j] "=&s"(j));
    uint64_t gc = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)gh62, (int)j) << 32) |
                  (uint32_t)__builtin_amdgcn_readlane((int)gl, (int)j);
    while (true) {
        uint32_t jn;  // next job (-1: none; V stays 0)
        asm("s_ff1_i32_b64 %[j], %[V]\n\t"
            "s_bitset0_b64 %[V], %[j]"
            : [V] "+s"(V), [j] "=&s"(jn));
        const uint64_t gn =
            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)gh62, (int)(jn & 63u)) << 32) |
            (uint32_t)__builtin_amdgcn_readlane((int)gl, (int)(jn & 63u));
        uint64_t t;
        int32_t bpos;
        // taken |= lowest bit of (gc & ~taken); job j's lane gets its
        // position (-1: none). SALU only, plus one writelane whose lane
        // select (m0) a SALU move wrote three instructions earlier.
        asm("s_mov_b32 m0, %[j]\n\t"
            "s_andn2_b64 %[t], %[g], %[tk]\n\t"
            "s_ff1_i32_b64 %[b], %[t]\n\t"
            "s_bitset1_b64 %[tk], %[b]\n\t"
            "v_writelane_b32 %[w], %[b], m0"
            : [tk] "+s"(taken), [w] "+v"(wres), [t] "=&s"(t), [b] "=&s"(bpos)
            : [g] "s"(gc), [j] "s"(j)
            : "m0", "scc");  // s_andn2 sets SCC
        if ((int32_t)jn < 0) break;
        j = jn;
        gc = gn;
    }
    }
    taken &= ~(1ull << 63);
    const uint64_t m63 = __ballot(((V0 >> lane) & 1ull) && wres < 0 && (gh >> 31) != 0u);
    if (m63 != 0ull) {
        if ((uint32_t)lane == (uint32_t)__builtin_ctzll(m63)) wres = 63;
        taken |= 1ull << 63;
    }
    if (wres >= 0) res = (int32_t)(w * 64u + (uint32_t)wres);
    R &= ~__ballot(wres >= 0);
    return taken;
}

// Runs walk (A7). Requires stage_meta (+ stage_topo when TOPO_LDS) and a
// barrier first, s_taken zeroed, and `feas` holding every class's bitmap words
// (LDS or global). Jobs are taken in global order, run by run; a run of class
// c takes the lowest free feasible domains at c's level from c's cursor on
// (domains below the cursor are taken or infeasible: the cursor only grows).
// Wave 0 walks every run; the other waves only join the long ones.
template <int NT, bool TOPO_LDS>
__device__ __forceinline__ void assign_block(const uint64_t* __restrict__ feas, uint32_t C, const TopoDev& topo,
                             const uint32_t* __restrict__ run_class, const uint32_t* __restrict__ run_len,
                             uint32_t n_runs, uint32_t J, int32_t* __restrict__ assign, uint32_t* __restrict__ stats,
                             uint64_t* s_taken, const AssignMeta& m, const uint32_t* s_topo, uint64_t* s_win,
                             uint32_t* s_stage, uint32_t stage_cap, AssignRec* __restrict__ recs,
                             uint32_t* __restrict__ rec_count, const WaitErr& wait, uint32_t len0 = ~0u,
                             uint32_t rc0 = 0u) {
    // len0 != ~0u: the caller loaded the first tile's run (thread tid's) already
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t K = topo.K;
    // the pipelined walk keeps its batch table and progress words in the stage
    const bool pipe_ok = NT >= 64 * (int)kPipeWaves && stage_cap >= 4u * NT + 2u * kPipeWaves + 8u;
    // a pipelined wait that gave up (wait.pipe_spins polls): the launch
    // reports it through wait.err at the end instead of a stale assign[]
    bool pipe_fail = false;
    // wave 0: class state in registers, lane c = class c (C <= kMaxClasses = 64)
    uint32_t my_cur = 0, my_lvl = 0, my_woff = 0, my_D = 0, my_toff = 0;
    if (wid == 0 && (uint32_t)lane < C) {
        my_lvl = m.s_lvl[lane];
        my_woff = m.s_woff[lane];
        my_D = m.s_D[my_lvl];
        my_toff = m.s_toff[my_lvl];
        my_cur = m.s_cursor[lane];
    }
    uint32_t placed = 0, jbase = 0;
    // register mode: the taken bitmaps of all levels fit one word per lane
    const uint32_t t_words = m.s_toff[K];
    const bool regmode = t_words <= kRegMaxWords;
    RegState rs;
    rs.T = rs.P = 0;  // s_taken starts zeroed
    rs.pend = -1;
    // Register mode: classes with no feasible domain at all ("dead") take
    // nothing and block nothing, so their jobs (-1) join a batch of any level
    // instead of cutting the level's job sequence into separate batches.
    uint64_t dead = 0;
    if (regmode) {
        uint64_t* s_alive = reinterpret_cast<uint64_t*>(m.s_misc + 2);
        if (tid == 0) *s_alive = 0;
        __syncthreads();
        const uint32_t nfw = m.s_woff[C];
        for (uint32_t wi = tid; wi < nfw; wi += NT) {
            if (feas[wi] == 0ull) continue;
            uint32_t c = 0;
            while (m.s_woff[c + 1] <= wi) ++c;  // C <= kMaxClasses
            atomicOr(reinterpret_cast<unsigned long long*>(s_alive), (unsigned long long)(1ull << c));
        }
        __syncthreads();
        dead = ~*s_alive & (C >= 64 ? ~0ull : ((1ull << C) - 1ull));
    }
    for (uint32_t r0 = 0; r0 < n_runs; r0 += NT) {
        // ---- a tile of runs: job offsets (block scan of run lengths) and the long-run list
        const uint32_t ri = r0 + tid;
        const bool pre = r0 == 0 && len0 != ~0u;
        const uint32_t len = pre ? len0 : ri < n_runs ? run_len[ri] : 0u;
        const uint32_t rc = pre ? rc0 : ri < n_runs ? run_class[ri] : 0u;
        m.s_rc[tid] = rc;
        uint32_t tile_total, n_long;
        const uint32_t off = block_excl_scan<NT>(len, m.s_w, &tile_total);
        m.s_ro[tid] = off;
        const bool is_long = len > kWaveRunMax && rc < C;
        const uint32_t lrank = block_excl_scan<NT>(is_long ? 1u : 0u, m.s_w, &n_long, 1);
        if (is_long) m.s_long[lrank] = (uint32_t)tid;
        __syncthreads();
        const uint32_t nr = (n_runs - r0) < (uint32_t)NT ? (n_runs - r0) : (uint32_t)NT;
        // Pipelined batches (a tile of short leaf-level runs, no long run): batch
        // b runs on wave b % kPipeWaves and may take word w as soon as every
        // earlier batch has passed w (words go in increasing order), so a
        // batch's sparse words and setup overlap the previous batch's dense word.
        bool pipe = false;
        if (regmode && pipe_ok) {
            const bool ok_run = ri >= n_runs || len == 0 ||
                                (rc < C && len <= kWaveRunMax && (((dead >> rc) & 1ull) || m.s_lvl[rc] + 1 == K));
            uint32_t n_bad;  // block count of runs outside the pipelined form (no static LDS of __syncthreads_and)
            (void)block_excl_scan<NT>(ok_run ? 0u : 1u, m.s_w, &n_bad);
            pipe = n_bad == 0 && n_long == 0;
        }
        if (pipe) {
            uint32_t* s_desc = s_stage;  // [4 per batch] {first run, runs, first job, jobs}
            JSP_LDS unsigned long long* s_prog = lds_ptr(reinterpret_cast<unsigned long long*>(
                (reinterpret_cast<uintptr_t>(s_stage + 4 * NT) + 7) & ~static_cast<uintptr_t>(7)));
            JSP_LDS uint32_t* s_pcnt = reinterpret_cast<JSP_LDS uint32_t*>(s_prog + kPipeWaves);
            JSP_LDS uint32_t* s_cur = lds_ptr(m.s_cursor);
            if (wid == 0) {
                if ((uint32_t)lane < t_words) s_taken[lane] = rs.T;
                if ((uint32_t)lane < C) m.s_cursor[lane] = my_cur;
                uint32_t q = 0, nbat = 0;
                while (q < nr) {
                    const uint32_t rk = q + (uint32_t)lane;
                    const bool in = rk < nr;
                    const uint32_t rc_v = in ? m.s_rc[rk] : 0xFFFFFFFFu;
                    const uint32_t ro_v = in ? m.s_ro[rk] : tile_total;
                    const uint32_t re_v = rk + 1 < nr ? m.s_ro[rk + 1] : tile_total;
                    const uint32_t o0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)ro_v);
                    const uint32_t o1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)re_v);
                    const uint32_t j0 = jbase + o0;
                    const uint32_t jend = jbase + o1 < J ? jbase + o1 : J;
                    if (j0 >= jend) {
                        ++q;
                        continue;
                    }
                    // every run of the tile is short and valid; a batch ends within 64 jobs of o0
                    const bool ok_v = in && rc_v < C && re_v - o0 <= 64u;
                    const uint64_t okm = __ballot(ok_v);
                    const uint32_t nrb = ~okm == 0ull ? 64u : (uint32_t)__builtin_ctzll(~okm);
                    uint32_t nb = (uint32_t)__builtin_amdgcn_readlane((int)re_v, (int)nrb - 1) - o0;
                    if (j0 + nb > J) nb = J - j0;
                    if (lane == 0) {
                        s_desc[4 * nbat + 0] = q;
                        s_desc[4 * nbat + 1] = nrb;
                        s_desc[4 * nbat + 2] = j0;
                        s_desc[4 * nbat + 3] = nb;
                    }
                    q += nrb;
                    ++nbat;
                }
                if (lane == 0) {
                    m.s_misc[0] = nbat;
                    s_pcnt[0] = 0;
                    s_pcnt[1] = 0;  // timed-out flag
                }
                if (lane < (int)kPipeWaves) s_prog[lane] = 0ull;
            }
            __syncthreads();
            const uint32_t nbat = m.s_misc[0];
            const uint32_t lvl = K - 1;
            const uint32_t D = m.s_D[lvl], tl = m.s_toff[lvl], nwl = (D + 63) >> 6;
            const uint32_t w_woff = (uint32_t)lane < C ? m.s_woff[lane] : 0u;
            uint32_t* s_bc = m.s_long + 64 * wid;  // this wave's job offset -> class table
            uint32_t my_placed = 0;
            for (uint32_t bi = (uint32_t)wid; wid < (int)kPipeWaves && bi < nbat; bi += kPipeWaves) {
                const uint32_t bid = bi + 1;  // progress words hold batch index + 1 (0: none yet)
                const uint32_t q = s_desc[4 * bi], nrb = s_desc[4 * bi + 1], j0 = s_desc[4 * bi + 2],
                               nb = s_desc[4 * bi + 3];
                const uint32_t rk = q + (uint32_t)lane, o0 = j0 - jbase;
                const bool inr = (uint32_t)lane < nrb;
                const uint32_t rc_v = inr ? m.s_rc[rk] : 0u;
                const uint32_t ro_v = inr ? m.s_ro[rk] : 0u;
                const uint32_t re_v = inr ? (rk + 1 < nr ? m.s_ro[rk + 1] : tile_total) : 0u;
                const bool starts = inr && re_v > ro_v;
                if (starts) s_bc[ro_v - o0] = rc_v;
                const uint64_t smask = wave_or64(starts ? 1ull << (ro_v - o0) : 0ull);
                const uint64_t le = (uint32_t)lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
                const bool job = (uint32_t)lane < nb;
                const uint32_t my_start = job ? 63u - (uint32_t)__builtin_clzll(smask & le) : 0u;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const uint32_t cls = job ? s_bc[my_start] : 0u;
                const uint64_t cmask = wave_or64(job ? 1ull << cls : 0ull) & ~dead;
                const bool cl = (uint32_t)lane < C && ((cmask >> lane) & 1ull);
                const uint32_t curc = cl ? __hip_atomic_load(s_cur + lane, __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_WORKGROUP)
                                         : D;  // a stale (lower) cursor only widens the scan
                const uint32_t d0 = wave_min_u32(curc);
                uint64_t R = __ballot(job);
                int32_t res = -1;
                uint32_t w = d0 >> 6 < nwl ? d0 >> 6 : nwl;
                if (lane == 0)
                    __hip_atomic_store(s_prog + wid, ((unsigned long long)bid << 32) | w, __ATOMIC_RELEASE,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
                // words each of the previous kPipeWaves - 1 batches is known to have
                // passed (0xFFFFFFFF: finished); polled only when a word needs it
                uint32_t known[kPipeWaves - 1];
#pragma unroll
                for (uint32_t k = 0; k + 1 < kPipeWaves; ++k) known[k] = k + 1 < bid ? 0u : 0xFFFFFFFFu;
                uint64_t fcur = cl && w < nwl ? feas[w_woff + w] : 0ull;
                for (; w < nwl && R != 0ull; ++w) {
                    const uint64_t fnx = cl && w + 1 < nwl ? feas[w_woff + w + 1] : 0ull;  // static: prefetch
                    // every earlier batch has passed word w: the previous kPipeWaves - 1
                    // batches by their progress words (older ones ran on this wave,
                    // or on a wave whose newer batch waited for them)
#pragma unroll
                    for (uint32_t k = 1; k < kPipeWaves; ++k) {
                        if (known[k - 1] > w) continue;
                        const uint32_t a = bid - k;
                        JSP_LDS unsigned long long* pw = s_prog + (a - 1) % kPipeWaves;
                        for (uint32_t spins = 0;; ++spins) {
                            const unsigned long long x =
                                __hip_atomic_load(pw, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                            const uint32_t pb = (uint32_t)(x >> 32), pr = (uint32_t)x;
                            known[k - 1] = pb > a ? 0xFFFFFFFFu : pb == a ? pr : 0u;
                            if (known[k - 1] > w) break;
                            if (spins >= wait.pipe_spins) {  // never waits forever: reported, never silent
                                __hip_atomic_store(s_pcnt + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                                break;
                            }
                            __builtin_amdgcn_s_sleep(1);
                        }
                    }
                    const uint64_t tw = s_taken[tl + w];
                    const uint64_t g = cl ? fcur & ~tw : 0ull;
                    fcur = fnx;
                    const uint64_t taken = walk_word(g, cls, job, R, res, w, lane);
                    if (lane == 0) {
                        if (taken) s_taken[tl + w] = tw | taken;
                        __hip_atomic_store(s_prog + wid, ((unsigned long long)bid << 32) | (w + 1), __ATOMIC_RELEASE,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
                if (lane == 0)
                    __hip_atomic_store(s_prog + wid, ((unsigned long long)bid << 32) | 0xFFFFFFFFull, __ATOMIC_RELEASE,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
                if (job) assign[j0 + lane] = res;
                my_placed += (uint32_t)__popcll(__ballot(job && res >= 0));
                uint64_t cm = cmask;
                while (cm != 0ull) {
                    const uint32_t cc = (uint32_t)__builtin_ctzll(cm);
                    cm &= cm - 1ull;
                    const uint64_t lanes_c = __ballot(job && cls == cc);
                    const int32_t last = __builtin_amdgcn_readlane(res, 63 - __builtin_clzll(lanes_c));
                    if ((uint32_t)lane == cc)
                        __hip_atomic_fetch_max(s_cur + cc, last < 0 ? D : (uint32_t)last + 1u, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
            if (lane == 0 && my_placed)
                __hip_atomic_fetch_add(s_pcnt, my_placed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __syncthreads();
            if (wid == 0) {
                const uint64_t Tn = (uint32_t)lane < t_words ? s_taken[lane] : rs.T;
                const uint64_t fresh = Tn & ~rs.T;
                if (lvl >= 1 && __ballot(fresh != 0ull) != 0ull) {
                    rs.P |= fresh;
                    rs.pend = rs.pend > (int)lvl ? rs.pend : (int)lvl;
                }
                rs.T = Tn;
                if ((uint32_t)lane < C) my_cur = m.s_cursor[lane];
            }
            if (tid == 0) {
                placed += s_pcnt[0];
                pipe_fail |= s_pcnt[1] != 0u;
            }
        } else if (wid == 0 && regmode) {
            // Short runs are taken in batches: up to 64 consecutive jobs (lane = job)
            // of short runs at one level. Within a batch the lowest-index greedy
            // ("each job in order takes its lowest free feasible domain") equals the
            // domain-order greedy ("each domain in order goes to the earliest
            // untaken job that finds it feasible": with one priority order per
            // side, both are the same unique stable matching). So the batch scans
            // the level's words from the lowest class cursor; per word each lane
            // holds its job's free feasible bits and every candidate domain costs
            // one ballot plus a few scalar ops -- no per-job chain of dependent
            // vector work.
            uint32_t q = 0, nbatch = 0;
            while (q < nr) {
                const uint32_t rk = q + (uint32_t)lane;
                const bool in = rk < nr;
                const uint32_t rc_v = in ? m.s_rc[rk] : 0xFFFFFFFFu;
                const uint32_t ro_v = in ? m.s_ro[rk] : tile_total;
                const uint32_t re_v = rk + 1 < nr ? m.s_ro[rk + 1] : tile_total;
                const uint32_t c = (uint32_t)__builtin_amdgcn_readfirstlane((int)rc_v);
                const uint32_t o0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)ro_v);
                const uint32_t o1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)re_v);
                const uint32_t j0 = jbase + o0;
                const uint32_t jend = jbase + o1 < J ? jbase + o1 : J;
                if (j0 >= jend) {
                    ++q;
                    continue;
                }
                if (c >= C) {  // malformed run: its jobs are unplaceable
                    for (uint32_t j = j0 + lane; j < jend; j += 64) assign[j] = -1;
                    ++q;
                    continue;
                }
                if (o1 - o0 > kWaveRunMax) {
                    // long run: fold pending ancestors, publish the bitmaps, join the
                    // workgroup (cursor 0: the whole level is one window), reload
                    if (rs.pend >= 1) reg_flush<TOPO_LDS>(rs, K, topo, s_taken, t_words, s_topo, m, lane);
                    if ((uint32_t)lane < t_words) s_taken[lane] = rs.T;
                    if (lane == 0) m.s_cursor[c] = 0;
                    long_run<NT, TOPO_LDS>(c, j0, jend, feas, topo, assign, s_taken, m, s_topo, s_win, s_stage,
                                           stage_cap, recs, placed);
                    if ((uint32_t)lane < t_words) rs.T = s_taken[lane];
                    ++q;
                    continue;
                }
                const uint32_t sb = 4010u + (nbatch < 39u ? nbatch : 39u);
                (void)sb;
                ++nbatch;
                JSP_STAMP(sb, 0);
                // ---- the batch: runs q .. q+nrb-1 (lane k = run q+k), all short, valid,
                // at level lvl (the level of its first live run; dead runs fit any
                // level), ending within 64 jobs of o0
                const uint32_t lvl_v = (uint32_t)__shfl((int)my_lvl, (int)(rc_v < C ? rc_v : 0u));
                const bool dead_v = rc_v < C && ((dead >> rc_v) & 1ull);
                const uint64_t live_runs = __ballot(in && rc_v < C && !dead_v);
                const uint32_t lvl = live_runs != 0ull
                                         ? (uint32_t)__builtin_amdgcn_readlane((int)lvl_v, __builtin_ctzll(live_runs))
                                         : (uint32_t)__builtin_amdgcn_readlane((int)my_lvl, (int)c);
                const bool ok_v = in && rc_v < C && (lvl_v == lvl || dead_v) && re_v - ro_v <= kWaveRunMax &&
                                  re_v - o0 <= 64u;
                const uint64_t okm = __ballot(ok_v);
                const uint32_t nrb = ~okm == 0ull ? 64u : (uint32_t)__builtin_ctzll(~okm);  // >= 1: run q qualifies
                uint32_t nb = (uint32_t)__builtin_amdgcn_readlane((int)re_v, (int)nrb - 1) - o0;
                if (j0 + nb > J) nb = J - j0;
                // job offset -> class: each non-empty run writes its class at its first
                // job; a job takes the class of the last run start at or below it
                const bool starts = (uint32_t)lane < nrb && re_v > ro_v;
                if (starts) m.s_bcls[ro_v - o0] = rc_v;
                const uint64_t smask = wave_or64(starts ? 1ull << (ro_v - o0) : 0ull);
                const uint64_t le = (uint32_t)lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
                const bool job = (uint32_t)lane < nb;
                const uint32_t my_start = job ? 63u - (uint32_t)__builtin_clzll(smask & le) : 0u;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const uint32_t cls = job ? m.s_bcls[my_start] : 0u;
                q += nrb;
                // live classes of the batch; the scan starts at their lowest cursor
                // (every class's domains below its cursor are taken or infeasible)
                const uint64_t cmask = wave_or64(job ? 1ull << cls : 0ull) & ~dead;
                if (cmask != 0ull && rs.pend > (int)lvl) reg_flush<TOPO_LDS>(rs, K, topo, s_taken, t_words, s_topo, m, lane);
                const uint32_t D = m.s_D[lvl];
                const uint32_t curc = (uint32_t)lane < C && ((cmask >> lane) & 1ull) ? my_cur : D;
                const uint32_t d0 = wave_min_u32(curc);
                const uint32_t tl = m.s_toff[lvl], nwl = (D + 63) >> 6;
                uint64_t R = __ballot(job);  // jobs of the batch without a domain yet
                int32_t res = -1;
                uint64_t tookv = 0;
                const bool cl = (uint32_t)lane < C && ((cmask >> lane) & 1ull);
                JSP_STAMP(sb, 1);
                // Domain words in order; in each, the jobs still without a domain take,
                // in job order, the lowest free bit of their class's word (job order
                // and domain order give the same matching inside one word, see above).
                // The per-job step is a scalar chain -- two readlanes of the job's
                // class word, and-not / lowest-bit / or on the word's taken mask, one
                // select into the job's lane -- so its cost is a dozen instructions of one
                // wave, whatever the classes' feasibility patterns.
                // class lanes' feasibility word, one word ahead: the next word's
                // load is in flight while this word's chain runs
                uint64_t fcur = cl && (d0 >> 6) < nwl ? feas[my_woff + (d0 >> 6)] : 0ull, fnx = 0ull;
                for (uint32_t w = d0 >> 6; w < nwl && R != 0ull; ++w, fcur = fnx) {
                    fnx = cl && w + 1 < nwl ? feas[my_woff + w + 1] : 0ull;
                    const uint64_t tw =
                        ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(rs.T >> 32), (int)(tl + w)) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)rs.T, (int)(tl + w));
                    const uint64_t g = cl ? fcur & ~tw : 0ull;  // lane c: class c's free feasible bits
                    // job lane j: its class's word
                    const uint64_t taken = walk_word(g, cls, job, R, res, w, lane);
                    if ((uint32_t)lane == tl + w) tookv |= taken;
                }
                JSP_STAMP(sb, 2);
                if (job) assign[j0 + lane] = res;
                placed += (uint32_t)__popcll(__ballot(job && res >= 0));
                // cursors: a class's last job in the batch holds its largest domain
                // (or -1: the class has nothing left at this level)
                uint64_t cm = cmask;
                while (cm != 0ull) {
                    const uint32_t cc = (uint32_t)__builtin_ctzll(cm);
                    cm &= cm - 1ull;
                    const uint64_t lanes_c = __ballot(job && cls == cc);
                    const int32_t last = __builtin_amdgcn_readlane(res, 63 - __builtin_clzll(lanes_c));
                    if ((uint32_t)lane == cc) my_cur = last < 0 ? D : (uint32_t)last + 1u;
                }
                rs.T |= tookv;
                if (lvl >= 1) {
                    rs.P |= tookv;
                    rs.pend = rs.pend > (int)lvl ? rs.pend : (int)lvl;
                }
                if (lvl + 1 < K) reg_mark_desc<TOPO_LDS>(rs, tookv, lvl, tl, K, topo, s_topo, m, lane);
                JSP_STAMP(sb, 3);
            }
        } else if (wid == 0) {
            for (uint32_t t0 = 0; t0 < nr; t0 += 64) {
                const uint32_t tl = t0 + (uint32_t)lane;
                const uint32_t rc_l = tl < nr ? m.s_rc[tl] : 0u;
                const uint32_t ro_l = tl < nr ? m.s_ro[tl] : 0u;
                const uint32_t rn_l = tl + 1 < nr ? m.s_ro[tl + 1] : tile_total;
                const uint32_t nb = (nr - t0) < 64u ? (nr - t0) : 64u;
                for (uint32_t q = 0; q < nb; ++q) {
                    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)rc_l, (int)q);
                    const uint32_t o0 = (uint32_t)__builtin_amdgcn_readlane((int)ro_l, (int)q);
                    const uint32_t o1 = (uint32_t)__builtin_amdgcn_readlane((int)rn_l, (int)q);
                    const uint32_t j0 = jbase + o0;
                    const uint32_t jend = jbase + o1 < J ? jbase + o1 : J;
                    if (j0 >= jend) continue;
                    if (c >= C) {  // malformed run: its jobs are unplaceable
                        for (uint32_t j = j0 + lane; j < jend; j += 64) assign[j] = -1;
                        continue;
                    }
                    if (o1 - o0 > kWaveRunMax) {  // long run: publish the cursors, join the workgroup
                        if ((uint32_t)lane < C) m.s_cursor[lane] = my_cur;
                        const uint32_t nc = long_run<NT, TOPO_LDS>(c, j0, jend, feas, topo, assign, s_taken, m, s_topo,
                                                                   s_win, s_stage, stage_cap, recs, placed);
                        if ((uint32_t)lane == c) my_cur = nc;
                        continue;
                    }
                    // ---- short run, wave 0 alone
                    const uint32_t lvl = (uint32_t)__builtin_amdgcn_readlane((int)my_lvl, (int)c);
                    const uint32_t D = (uint32_t)__builtin_amdgcn_readlane((int)my_D, (int)c);
                    const uint32_t nw = (D + 63) >> 6;
                    uint64_t* Tk = s_taken + (uint32_t)__builtin_amdgcn_readlane((int)my_toff, (int)c);
                    const uint64_t* F = feas + (uint32_t)__builtin_amdgcn_readlane((int)my_woff, (int)c);
                    uint32_t cur = (uint32_t)__builtin_amdgcn_readlane((int)my_cur, (int)c);
                    uint32_t need = jend - j0, jpos = j0;
                    while (need > 0 && cur < D) {
                        const uint32_t w = (cur >> 6) + lane;
                        uint64_t bits = 0;
                        if (w < nw) {
                            bits = F[w] & ~Tk[w];
                            if (w == (cur >> 6)) bits &= ~0ull << (cur & 63);
                        }
                        const uint32_t cnt = (uint32_t)__popcll(bits);
                        const uint32_t incl = wave_incl_scan(cnt, lane);
                        const uint32_t pre = incl - cnt;
                        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
                        // emission, one useful word at a time, its bits across the
                        // lanes: lane b takes bit b at rank pre_k + (bits below b)
                        uint64_t todo = __ballot(cnt != 0 && pre < need);
                        uint32_t next = ((cur >> 6) + 64) * 64;
                        while (todo) {
                            const int k = __builtin_ctzll(todo);
                            todo &= todo - 1;
                            const uint32_t blo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)bits, k);
                            const uint32_t bhi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(bits >> 32), k);
                            const uint64_t wbits = ((uint64_t)bhi << 32) | blo;
                            const uint32_t rank = (uint32_t)__builtin_amdgcn_readlane((int)pre, k) +
                                                  (uint32_t)__popcll(wbits & ((1ull << lane) - 1ull));
                            const bool take = ((wbits >> lane) & 1ull) && rank < need;
                            const uint32_t d = ((cur >> 6) + (uint32_t)k) * 64 + (uint32_t)lane;
                            if (take) {
                                assign[jpos + rank] = (int32_t)d;
                                if (K > 1) mark_other_levels<TOPO_LDS>(d, lvl, K, topo, s_taken, m, s_topo);
                            }
                            const uint64_t took = __ballot(take);
                            if (lane == k) Tk[w] |= took;  // lane k owns word k of the window
                            const uint64_t lastm = __ballot(take && rank + 1 == need);
                            if (lastm) next = (uint32_t)__builtin_amdgcn_readlane((int)d, __builtin_ctzll(lastm)) + 1;
                        }
                        cur = next;
                        const uint32_t used = total < need ? total : need;
                        need -= used;
                        jpos += used;
                        placed += used;
                    }
                    for (uint32_t j = jpos + lane; j < jend; j += 64) assign[j] = -1;
                    if ((uint32_t)lane == c) my_cur = cur < D ? cur : D;
                }
            }
        } else {
            for (uint32_t q = 0; q < n_long; ++q) {
                const uint32_t t = m.s_long[q];
                const uint32_t j0 = jbase + m.s_ro[t];
                uint32_t jend = (t + 1 < nr) ? jbase + m.s_ro[t + 1] : jbase + tile_total;
                if (jend > J) jend = J;
                if (j0 >= jend) continue;
                long_run<NT, TOPO_LDS>(m.s_rc[t], j0, jend, feas, topo, assign, s_taken, m, s_topo, s_win, s_stage,
                                       stage_cap, recs, placed);
            }
        }
        jbase += tile_total;
        __syncthreads();  // tile tables free again; short-run state visible
    }
    if (tid == 0 && stats != nullptr) {
        stats[0] = n_runs;
        stats[1] = placed;
    }
    if (tid == 0 && pipe_fail && wait.err != nullptr)
        __hip_atomic_store(wait.err, wait.tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (tid == 0 && rec_count != nullptr) *rec_count = m.s_misc[1];  // records for expand_kernel
    JSP_STAMP(4000u, 7);
}

// LDS: [taken t_words u64][window NT u64 + NT u32][feasibility feas_words u64, when staged]
//      [small tables][hierarchy tables, when staged][stage stage_cap u32]
__global__ __launch_bounds__(kAssignThreads) void assign_kernel(
    const uint64_t* __restrict__ feas, const uint32_t* __restrict__ word_off, const DevClass* __restrict__ cls,
    uint32_t C, TopoDev topo, const uint32_t* __restrict__ run_class, const uint32_t* __restrict__ run_len,
    uint32_t n_runs, uint32_t J, int32_t* __restrict__ assign, uint32_t* __restrict__ stats, uint32_t feas_words,
    uint32_t feas_in_lds, uint32_t topo_in_lds, uint32_t topo_words, uint32_t stage_cap, AssignRec* __restrict__ recs,
    uint32_t* __restrict__ rec_count, WaitErr wait) {
    extern __shared__ __attribute__((aligned(16))) uint64_t s_dyn[];
    const uint32_t tw = taken_words(topo);
    uint64_t* s_win = s_dyn + tw;
    uint64_t* s_feas = s_win + kAssignWinWords64;
    const uint32_t fw = feas_in_lds ? feas_words : 0u;
    uint32_t* s_small = reinterpret_cast<uint32_t*>(s_feas + fw);
    const AssignMeta m = carve_meta<kAssignThreads>(s_small);
    uint32_t* s_topo = s_small + assign_small_words(kAssignThreads);
    uint32_t* s_stage = s_topo + (topo_in_lds ? topo_words : 0u);
    JSP_STAMP(4000u, 0);
    // the first tile of runs and up to 4 feasibility words per thread are
    // loaded before any staging store, so their latencies overlap (the run
    // table otherwise waited for the staging barrier)
    const uint32_t tid = threadIdx.x;
    const uint32_t len0 = tid < n_runs ? run_len[tid] : 0u;
    const uint32_t rc0 = tid < n_runs ? run_class[tid] : 0u;
    uint64_t f4[4];
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t i = tid + k * kAssignThreads;
        f4[k] = i < fw ? feas[i] : 0ull;
    }
    stage_meta<kAssignThreads>(m, cls, C, word_off, topo);
    if (tid == 0) m.s_misc[1] = 0;
    if (topo_in_lds) stage_topo<kAssignThreads>(s_topo, topo);
    for (uint32_t i = tid; i < tw; i += kAssignThreads) s_dyn[i] = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t i = tid + k * kAssignThreads;
        if (i < fw) s_feas[i] = f4[k];
    }
    for (uint32_t i = tid + 4 * kAssignThreads; i < fw; i += kAssignThreads) s_feas[i] = feas[i];
    __syncthreads();
    JSP_STAMP(4000u, 1);
    const uint64_t* F = feas_in_lds ? s_feas : feas;
    if (topo_in_lds)
        assign_block<kAssignThreads, true>(F, C, topo, run_class, run_len, n_runs, J, assign, stats, s_dyn, m, s_topo,
                                           s_win, s_stage, stage_cap, recs, rec_count, wait, len0, rc0);
    else
        assign_block<kAssignThreads, false>(F, C, topo, run_class, run_len, n_runs, J, assign, stats, s_dyn, m,
                                            s_topo, s_win, s_stage, stage_cap, recs, rec_count, wait, len0, rc0);
}

// Records per expanding wave: 1, 4 and 16 are equal within noise on cfg4, 64
// is slower.
constexpr uint32_t kExpandRpw = 16;

// Expansion of assign_kernel's records: a wave owns rpw (<= 64) consecutive
// records of the host's bound (records <= min(J, feas_words + runs)); lane i
// loads record r0 + i in one coalesced load issued beside the count's, then
// the wave writes them one at a time: lane b of a record with bit b taken
// writes job base + (taken bits below b), so each store is one run. A small
// grid (tens of blocks, not one wave per job) is most of this kernel's time.
__global__ __launch_bounds__(256) void expand_kernel(const AssignRec* __restrict__ recs,
                                                     const uint32_t* __restrict__ rec_count, uint32_t bound,
                                                     uint32_t rpw, int32_t* __restrict__ assign) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t r0 = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * rpw;
    if (r0 >= bound) return;  // wave-uniform
    AssignRec x{0u, 0u, 0ull};
    if (lane < rpw && r0 + lane < bound) x = recs[r0 + lane];
    const uint32_t n = *rec_count;
    if (r0 >= n) return;
    const uint32_t m = n - r0 < rpw ? n - r0 : rpw;
    const uint64_t below = (1ull << lane) - 1ull;
    const uint32_t t_lo = (uint32_t)x.took, t_hi = (uint32_t)(x.took >> 32);
    for (uint32_t i = 0; i < m; ++i) {
        const uint64_t t = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)t_hi, (int)i) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((int)t_lo, (int)i);
        const uint32_t base = (uint32_t)__builtin_amdgcn_readlane((int)x.base, (int)i);
        const uint32_t dom0 = (uint32_t)__builtin_amdgcn_readlane((int)x.dom0, (int)i);
        if ((t >> lane) & 1ull) assign[base + (uint32_t)__popcll(t & below)] = (int32_t)(dom0 + lane);
    }
}

// The expanders of the one-launch level walk: wave g owns records
// [g rpw, g rpw + rpw). It waits (bounded) for the walker's published count
// of this launch (epoch-tagged), reads its records write-through and writes
// their jobs' domains as expand_kernel does. A wave that gives up (the
// walker, dispatched first, never published within wait.wait_ticks) writes
// the launch's tag to the error word: the call fails, never a stale assign[].
__device__ void level_expand(const AssignRec* recs, const unsigned long long* ready, uint32_t epoch, uint32_t bound,
                             uint32_t rpw, int32_t* assign, const WaitErr& wait) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t r0 = ((blockIdx.x - 1) * (blockDim.x >> 6) + (threadIdx.x >> 6)) * rpw;
    if (r0 >= bound) return;  // wave-uniform
    const uint64_t t0 = wall_clock64();
    uint32_t n = 0;
    while (true) {
        const unsigned long long x = __hip_atomic_load(ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)(x >> 32) == epoch && (x & 0x80000000ull)) {  // this launch's final count
            n = (uint32_t)x & 0x7FFFFFFFu;
            break;
        }
        if (wall_clock64() - t0 >= wait.wait_ticks) {
            if (lane == 0 && wait.err != nullptr)
                __hip_atomic_store(wait.err, wait.tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    if (r0 >= n) return;
    const uint32_t m = n - r0 < rpw ? n - r0 : rpw;
    uint32_t dom0 = 0, base = 0, t_lo = 0, t_hi = 0;
    if (lane < m) {
        const unsigned long long* rp = reinterpret_cast<const unsigned long long*>(recs + r0 + lane);
        const unsigned long long a = __hip_atomic_load(rp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long b = __hip_atomic_load(rp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        dom0 = (uint32_t)a;
        base = (uint32_t)(a >> 32);
        t_lo = (uint32_t)b;
        t_hi = (uint32_t)(b >> 32);
    }
    const uint64_t below = (1ull << lane) - 1ull;
    for (uint32_t i = 0; i < m; ++i) {
        const uint64_t t = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)t_hi, (int)i) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((int)t_lo, (int)i);
        const uint32_t bs = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)i);
        const uint32_t d0 = (uint32_t)__builtin_amdgcn_readlane((int)dom0, (int)i);
        if ((t >> lane) & 1ull) assign[bs + (uint32_t)__popcll(t & below)] = (int32_t)(d0 + lane);
    }
}

// ---- level walker (jsp_internal.h launch_assign_level): every class at one
// level, few runs. The workgroup (256 threads) stages the classes'
// feasibility words in LDS (word-major by thread: thread t owns words
// [t WPT, t WPT + WPT), stored [class][k][t] so every read is conflict-free)
// and keeps the taken bits of its words in registers. Per run, ONE block scan
// (one barrier) of a packed (nonzero words << 18 | free feasible count) gives
// each thread its first rank and its first record slot: the run takes its
// `used` lowest free feasible domains, and the words that give domains away
// are the first nonzero ones, so a word's record slot is its rank among the
// nonzero words. The thread holding the run's last taking word publishes the
// next run's record base (read after the next scan's barrier). A one-wave
// version (all words in one wave's registers) was instruction-bound: a wave64
// VALU op takes 4 cycles of its SIMD, ~3 us per run on cfg4.
// NT threads (256, or 1024 for more than 256 words: one or two words per
// thread, 4 waves per SIMD to hide each other's latency in the per-run chain)
template <int WPT, int NT>
__global__ __launch_bounds__(NT) void assign_level_kernel(const uint64_t* __restrict__ feas, uint32_t C,
                                                                     uint32_t nw, const uint32_t* __restrict__ run_class,
                                                                     const uint32_t* __restrict__ run_len, uint32_t n_runs,
                                                                     int32_t* __restrict__ assign,
                                                                     uint32_t* __restrict__ stats,
                                                                     uint32_t* __restrict__ rec_count,
                                                                     AssignRec* __restrict__ recs,
                                                                     unsigned long long* __restrict__ ready,
                                                                     uint32_t epoch, uint32_t bound, uint32_t rpw,
                                                                     WaitErr wait) {
    // Expansion in the same launch (ready != null): workgroups 1.. wait for
    // the walker (workgroup 0, dispatched first, never waits for them) to
    // publish its record count, then expand the records as expand_kernel
    // does -- no second launch and no launch gap between walk and expansion.
    if (ready != nullptr && blockIdx.x > 0) {
        level_expand(recs, ready, epoch, bound, rpw, assign, wait);
        return;
    }
    extern __shared__ __attribute__((aligned(16))) uint64_t s_f[];  // [C][WPT][NT]
    JSP_LDS uint64_t* sf = lds_ptr(s_f);
    __shared__ uint32_t s_rc[kLevelMaxRuns], s_rl[kLevelMaxRuns];
    __shared__ uint32_t s_scan[2 * (NT / 64)];
    __shared__ uint32_t s_base[2];
    __shared__ uint32_t s_u0[kLevelMaxRuns], s_u1[kLevelMaxRuns];
    const uint32_t tid = threadIdx.x;
    JSP_STAMP(4050u, 0);
    // the run table beside the words: one round trip, however far the runs
    // live (pinned host memory on the host path)
    if (tid < n_runs) {
        s_rc[tid] = run_class[tid];
        s_rl[tid] = run_len[tid];
    }
    if (tid == 0) s_base[0] = 0u;
    // 16 loads per thread in flight before their LDS stores
    constexpr uint32_t kBatch = 16;
    const uint32_t total = C * (uint32_t)NT * (uint32_t)WPT;
    for (uint32_t b0 = 0; b0 < total; b0 += (uint32_t)NT * kBatch) {
        uint64_t f[kBatch];
#pragma unroll
        for (uint32_t q = 0; q < kBatch; ++q) {
            const uint32_t i = b0 + q * (uint32_t)NT + tid;  // i = c * (256 WPT) + word
            const uint32_t c = i / ((uint32_t)NT * WPT), w = i - c * ((uint32_t)NT * WPT);
            f[q] = (i < total && w < nw) ? feas[(size_t)c * nw + w] : 0ull;
        }
#pragma unroll
        for (uint32_t q = 0; q < kBatch; ++q) {
            const uint32_t i = b0 + q * (uint32_t)NT + tid;
            const uint32_t c = i / ((uint32_t)NT * WPT), w = i - c * ((uint32_t)NT * WPT);
            if (i < total) sf[(c * WPT + w % WPT) * (uint32_t)NT + w / WPT] = f[q];
        }
    }
    __syncthreads();
    JSP_STAMP(4050u, 1);
    uint64_t T[WPT];
#pragma unroll
    for (int k = 0; k < WPT; ++k) T[k] = 0;
    uint32_t jpos = 0, placed = 0;
    for (uint32_t r = 0; r < n_runs; ++r) {
        const uint32_t c = s_rc[r], n = s_rl[r];
        uint64_t A[WPT];
        uint32_t cnt = 0, nzw = 0;
#pragma unroll
        for (int k = 0; k < WPT; ++k) {
            A[k] = sf[(c * WPT + k) * (uint32_t)NT + tid] & ~T[k];
            cnt += (uint32_t)__popcll(A[k]);
            nzw += A[k] != 0ull ? 1u : 0u;
        }
        uint32_t tot_p;
        const uint32_t pre_p = block_excl_scan<NT>((nzw << 18) | cnt, s_scan, &tot_p, (int)(r & 1u));
        const uint32_t pre = pre_p & 0x3FFFFu, total_free = tot_p & 0x3FFFFu;
        const uint32_t used = total_free < n ? total_free : n;
        if (r < 4) JSP_STAMP(4051u, r);  // diagnostic: this run's scan is done
        const uint32_t rec_base = s_base[r & 1u];  // published by run r - 1 before this scan's barrier
        uint32_t rem = used > pre ? used - pre : 0u;
        uint32_t slot = rec_base + (pre_p >> 18);
        uint32_t base = jpos + pre;
#pragma unroll
        for (int k = 0; k < WPT; ++k) {
            if (rem != 0u && A[k] != 0ull) {
                const uint32_t pc = (uint32_t)__popcll(A[k]);
                uint64_t took = A[k];
                if (pc > rem) took &= (1ull << select_bit(took, rem)) - 1ull;
                const uint32_t tk = pc > rem ? rem : pc;
                rem -= tk;
                T[k] |= took;
                const uint32_t dom0 = (tid * (uint32_t)WPT + (uint32_t)k) * 64u;
                if (ready != nullptr) {  // read by other workgroups of this launch: write-through
                    unsigned long long* rp = reinterpret_cast<unsigned long long*>(recs + slot);
                    __hip_atomic_store(rp, ((unsigned long long)base << 32) | dom0, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(rp + 1, (unsigned long long)took, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } else {
                    AssignRec x;
                    x.dom0 = dom0;
                    x.base = base;
                    x.took = took;
                    recs[slot] = x;
                }
                ++slot;
                base += tk;
                // the run's last taking word: the next run's records start after it
                if (rem == 0u) s_base[(r + 1) & 1u] = slot;
            }
        }
        if (used == 0u && tid == 0) s_base[(r + 1) & 1u] = rec_base;
        if (r < 4) JSP_STAMP(4051u, 4 + r);  // diagnostic: this run's records issued
        if (tid == 0) {  // the run's unplaceable tail, written after the walk (off the runs' chain)
            s_u0[r] = jpos + used;
            s_u1[r] = jpos + n;
        }
        placed += used;
        jpos += n;
        if (r < 5) JSP_STAMP(4050u, 2 + r);
    }
    if (ready != nullptr) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's records are out
    __syncthreads();  // the last run's record base
    if (tid == 0) {
        *rec_count = s_base[n_runs & 1u];
        stats[0] = n_runs;
        stats[1] = placed;
        if (ready != nullptr)
            __hip_atomic_store(ready, ((unsigned long long)epoch << 32) | 0x80000000ull | s_base[n_runs & 1u],
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the unplaceable tails (-1), while the expanders work: 16-byte stores
    // between the 4-aligned bounds when assign[] is 16-byte aligned
    const bool vec = (reinterpret_cast<uintptr_t>(assign) & 15u) == 0u;
    for (uint32_t r = 0; r < n_runs; ++r) {
        const uint32_t j0 = s_u0[r], j1 = s_u1[r];
        if (j0 >= j1) continue;
        uint32_t a0 = j1, a1 = j1;
        if (vec) {
            a0 = (j0 + 3u) & ~3u;
            a1 = j1 & ~3u;
            if (a0 > a1) a0 = a1 = j1;
        }
        for (uint32_t j = j0 + tid; j < a0; j += (uint32_t)NT) assign[j] = -1;
        for (uint32_t q = a0 / 4u + tid; q < a1 / 4u; q += (uint32_t)NT)
            reinterpret_cast<int4*>(assign)[q] = make_int4(-1, -1, -1, -1);
        for (uint32_t j = a1 + tid; j < j1; j += (uint32_t)NT) assign[j] = -1;
    }
    JSP_STAMP(4050u, 7);
}

// ---- fused tail: leaf pass of the feasibility build (see place_fused_kernel)
struct TailFeasArgs {
    const uint32_t* cap;
    const uint32_t* occ;
    uint32_t ld, L;
    uint64_t pass_cls, leaf_cls;
    uint32_t npc;
    bool scr;
    uint32_t K;
    uint32_t ooff0, ooff1, ooff2;  // occupancy-bit word offset of upper levels 0..2 (no arrays: they
                                   // would be indexed at run time and live in scratch)
    uint64_t* s_uocc;
    uint64_t* s_usum;
    uint64_t* s_feas;
    uint32_t c_pods, c_beg, c_lvl, c_uoff;  // lane c: class c's fields
    const uint32_t* s_topo;  // hierarchy tables in LDS, or null
    const uint32_t* s_poff;  // parent-table offsets in s_topo per level
    const int32_t *par1, *par2, *par3;  // the same tables in global memory (levels 1..3)
};
static_assert(kMaxLevels == 4, "TailFeasArgs spells out the levels");


__device__ __forceinline__ uint32_t tail_ooff(const TailFeasArgs& t, uint32_t k) {
    const uint32_t o0 = t.ooff0, o1 = t.ooff1, o2 = t.ooff2;  // values: a conditional of lvalues would select
    return k == 0 ? o0 : k == 1 ? o1 : o2;                    // field addresses and keep t in scratch
}

// ancestor at level lvl of leaf l (hierarchy tables from LDS when staged)
__device__ __forceinline__ uint32_t tail_up_dom(const TailFeasArgs& t, uint32_t l, uint32_t lvl) {
    if (t.s_topo) {
        JSP_LDS const uint32_t* st = lds_ptr(t.s_topo);
        JSP_LDS const uint32_t* po = lds_ptr(t.s_poff);
        for (uint32_t k = t.K - 1; k > lvl; --k) l = st[po[k] + l];
        return l;
    }
    const int32_t *p1 = t.par1, *p2 = t.par2, *p3 = t.par3;  // values, as in tail_ooff
    for (uint32_t k = t.K - 1; k > lvl; --k) l = (uint32_t)(k == 1 ? p1 : k == 2 ? p2 : p3)[l];
    return l;
}

// Every thread takes 4-leaf chunks, loads occupancy once and the capacities of
// the NG classes of the pass, then ORs each leaf-level class's 4 feasibility
// bits into its LDS word and adds each upper class's clamped capacities into
// its domain sums (and flags occupied leaves' domains).
template <int NG>
__device__ __forceinline__ void tail_leaf_pass(const TailFeasArgs& t) {
    const uint32_t L = t.L, npc = t.npc;
    // the pass's classes and their capacity rows, wave-uniform (SGPRs): each
    // load below is one instruction on a scalar base and a shared lane offset
    uint32_t cid[NG];
    {
        uint64_t m = t.pass_cls;
#pragma unroll
        for (int u = 0; u < NG; ++u) {
            const uint32_t c = (uint32_t)__builtin_ctzll(m);  // past npc: the last class again
            if ((uint32_t)u + 1 < npc) m &= m - 1ull;
            cid[u] = to_sgpr(c);
        }
    }
    // one buffer resource over the capacity rows of classes 0..highest of the
    // pass (a resource or a pointer per row would cost 4 or 2 SGPRs each, and
    // this kernel already spills SGPRs)
    const uint32_t n_rows = 64u - (uint32_t)__builtin_clzll(t.pass_cls);
    const __amdgpu_buffer_rsrc_t cap_r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(t.cap), (short)0, (int)(n_rows * t.ld * 4u), 0x00020000);
    JSP_STAMP(4008u, 3);
    // wave-uniform trip count (lanes past L run with masked values): the
    // leaf-level classes' words are formed by a DPP OR across each 16-lane row
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t qb = threadIdx.x - lane; qb * 4u < L; qb += kTallyThreads) {
        const uint32_t q = qb + lane;
        const uint32_t l0 = q * 4u;
        // every load at a clamped index (classes past npc repeat the last one,
        // leaves past L the last leaf) and masked afterwards: straight-line
        // code, so all of them are in flight before the first wait
        // one 16-B sc1 buffer load per row and thread (its 4 leaves; rows
        // need not be 16-B aligned), bounded by the row's end
        uint32_t ov[4], cv[NG][4];
        if (l0 + 4u <= L) {
            const uint4 o4 = load16_sc1_n(t.occ, l0 * 4u, L * 4u);
            ov[0] = o4.x; ov[1] = o4.y; ov[2] = o4.z; ov[3] = o4.w;
#pragma unroll
            for (int u = 0; u < NG; ++u) {
                const uint4 c4 = __builtin_bit_cast(
                    uint4, __builtin_amdgcn_raw_buffer_load_b128(cap_r, cid[u] * t.ld * 4u + l0 * 4u, 0, 16));
                cv[u][0] = c4.x; cv[u][1] = c4.y; cv[u][2] = c4.z; cv[u][3] = c4.w;
            }
        } else {  // the last, partial chunk (and lanes past L): clamped dword loads
            uint32_t ix[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) ix[i] = l0 + i < L ? l0 + i : L - 1;
#pragma unroll
            for (int i = 0; i < 4; ++i) ov[i] = load_handoff(t.occ + ix[i]);
#pragma unroll
            for (int u = 0; u < NG; ++u)
#pragma unroll
                for (int i = 0; i < 4; ++i) cv[u][i] = load_handoff(t.cap + (size_t)cid[u] * t.ld + ix[i]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const bool in = l0 + i < L;
            ov[i] = in ? ov[i] : 1u;
#pragma unroll
            for (int u = 0; u < NG; ++u) cv[u][i] = in ? cv[u][i] : 0u;
        }
#ifdef JSP_STAMPS
        JSP_STAMP(4008u, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        JSP_STAMP(4008u, 1);
#endif
        if (t.scr) {  // occupied leaves flag their domain at every level above the leaves
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (l0 + i >= L || ov[i] == 0u) continue;
                for (uint32_t k = 0; k + 1 < t.K; ++k) {
                    const uint32_t d = tail_up_dom(t, l0 + i, k);
                    __hip_atomic_fetch_or(lds_ptr(t.s_uocc) + tail_ooff(t, k) + (d >> 6), 1ull << (d & 63u),
                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
        }
        JSP_STAMP(4008u, 2);
        // leaf-level classes, unrolled: a 16-lane row covers one 64-leaf word;
        // OR the lanes' nibbles across the row (DPP row_shr 1/2/4/8), its last
        // lane stores it
#pragma unroll
        for (int u = 0; u < NG; ++u) {
            if ((uint32_t)u >= npc || ((t.leaf_cls >> cid[u]) & 1ull) == 0ull) continue;
            if (u < 8) JSP_STAMP(4009u, u);
            const uint32_t pods = (uint32_t)__builtin_amdgcn_readlane((int)t.c_pods, (int)cid[u]);
            const uint32_t wo = (uint32_t)__builtin_amdgcn_readlane((int)t.c_beg, (int)cid[u]);
            uint32_t nib = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) nib |= (cv[u][i] >= pods && ov[i] == 0u) ? (1u << i) : 0u;
            const uint32_t sh = 4u * (lane & 7u);
            uint32_t lo = (lane & 8u) ? 0u : nib << sh, hi = (lane & 8u) ? nib << sh : 0u;
            lo |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, 0x111, 0xf, 0xf, true);  // row_shr:1
            hi |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, 0x111, 0xf, 0xf, true);
            lo |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, 0x112, 0xf, 0xf, true);  // row_shr:2
            hi |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, 0x112, 0xf, 0xf, true);
            lo |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, 0x114, 0xf, 0xf, true);  // row_shr:4
            hi |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, 0x114, 0xf, 0xf, true);
            lo |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, 0x118, 0xf, 0xf, true);  // row_shr:8
            hi |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, 0x118, 0xf, 0xf, true);
            if ((lane & 15u) == 15u && (l0 & ~63u) < L) lds_ptr(t.s_feas)[wo + (l0 >> 6)] = ((uint64_t)hi << 32) | lo;
        }
        JSP_STAMP(4008u, 5);
        // upper-level classes (few), in a rolled loop so that the pass's code
        // stays small: the tail runs once per launch on whichever CU drew the
        // last ticket, from a cold instruction cache. Each class's 4 values are
        // picked from the unrolled registers by its slot in the pass.
        if (t.scr) {
            uint32_t dl[4] = {0u, 0u, 0u, 0u}, dl_lvl = 0xFFFFFFFFu;  // wave-uniform level of dl
            uint64_t um = t.pass_cls & ~t.leaf_cls;
            while (um != 0ull) {
                const uint32_t c = (uint32_t)__builtin_ctzll(um);
                um &= um - 1ull;
                const uint32_t u = (uint32_t)__popcll(t.pass_cls & ((1ull << c) - 1ull));  // slot in the pass
                uint32_t v[4] = {cv[0][0], cv[0][1], cv[0][2], cv[0][3]};
#pragma unroll
                for (int k = 1; k < NG; ++k)
                    if (u == (uint32_t)k) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) v[i] = cv[k][i];
                    }
                const uint32_t pods = (uint32_t)__builtin_amdgcn_readlane((int)t.c_pods, (int)c);
                const uint32_t lvl = (uint32_t)__builtin_amdgcn_readlane((int)t.c_lvl, (int)c);
                JSP_LDS uint64_t* sum =
                    lds_ptr(t.s_usum) + (uint32_t)__builtin_amdgcn_readlane((int)t.c_uoff, (int)c);
                if (lvl != dl_lvl) {  // the 4 leaves' domains at this level, shared by its classes
#pragma unroll
                    for (int i = 0; i < 4; ++i) dl[i] = l0 + i < L ? tail_up_dom(t, l0 + i, lvl) : 0u;
                    dl_lvl = lvl;
                }
                uint32_t dcur = dl[0];  // lanes past L add nothing (the loop below stops at once)
                uint64_t acc = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    if (l0 + i >= L) break;
                    const uint32_t d = dl[i];
                    if (d != dcur) {
                        if (acc) __hip_atomic_fetch_add(sum + dcur, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        acc = 0;
                        dcur = d;
                    }
                    acc += v[i] < pods ? v[i] : pods;
                }
                if (acc) __hip_atomic_fetch_add(sum + dcur, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        JSP_STAMP(4008u, 4);
    }
}

// ----------------------------------------------------------------- fused small-snapshot placement
// Tally workgroups publish their leaf sums (plain stores, every wave drains
// vmcnt, workgroup barrier, one lane: agent release fence, drain, relaxed agent
// ticket add). The workgroup that draws the last ticket of this launch
// acquires (agent fence + drain + barrier), builds every class's feasibility
// bitmap in LDS and runs the assignment (cdna_hip_programming.md §6 G16).
// Tiles come from ticket[0] (oversubscribed grid, kSpareBlocks); ticket[1]
// counts finished tiles. Both 64-bit counters are zeroed at snapshot upload
// and the host adds every launch's draws to its bases, so "my tile" =
// old - tile_base and "last" = old + 1 - done_base == n_blocks.
// The fused kernel's tail, run by the workgroup whose tile finished last: the
// feasibility bitmaps of every class into LDS from the tiles' published sums,
// then the assignment walk; done (host path) gets epoch at the end.
template <int W, int R>
__device__ __forceinline__ void fused_tail(const TallyArgs& a, const FusedArgs& f, uint32_t* lds, uint32_t J,
                                           uint32_t n_runs, uint32_t epoch, uint32_t* done) {
    JSP_STAMP(4000u, 1);
    // the tail: small tables first (independent of the other workgroups' sums)
    uint64_t* s_taken = reinterpret_cast<uint64_t*>(lds);
    uint64_t* s_win = s_taken + f.t_words;
    uint64_t* s_feas = s_win + kFusedWinWords64;
    uint32_t* s_small = reinterpret_cast<uint32_t*>(s_feas + f.feas_words);
    const AssignMeta m = carve_meta<kTallyThreads>(s_small);
    uint32_t* s_topo = s_small + assign_small_words(kTallyThreads);
    uint32_t* s_stage = s_topo + f.topo_lds_words;
    stage_meta<kTallyThreads>(m, a.cls, f.C, f.word_off, f.topo);
    if (threadIdx.x == 0) m.s_misc[1] = 0;
    if (f.topo_in_lds) stage_topo<kTallyThreads>(s_topo, f.topo);
    for (uint32_t i = threadIdx.x; i < f.t_words; i += kTallyThreads) s_taken[i] = 0;
    for (uint32_t i = threadIdx.x; i < f.feas_words; i += kTallyThreads) s_feas[i] = 0;
    // With sc1_out every load of the other tiles' sums below is an sc1 load
    // (load_handoff) issued after the ticket add returned and this barrier, so
    // no acquire is needed; the per-wave upper-class path reads them with plain
    // loads and keeps it (the host sets sc1_out only when that path cannot run).
    if (threadIdx.x == 0 && !a.sc1_out) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    JSP_STAMP(4000u, 3);
    // feasibility bitmaps of every class into LDS. The tallies were written by
    // other workgroups (after the acquire every load misses to HBM/MALL), so
    // loads are issued in bulk before they are used.
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t Kt = f.topo.K;
    // per-class fields in registers (lane c = class c)
    const bool c_in = (uint32_t)lane < f.C;
    const uint32_t c_beg = c_in ? m.s_woff[lane] : 0u;
    const uint32_t c_end = c_in ? m.s_woff[lane + 1] : 0u;
    const uint32_t c_lvl = c_in ? m.s_lvl[lane] : 0u;
    const uint32_t c_pods = c_in ? m.s_pods[lane] : 0u;
    const uint64_t leaf_cls = __ballot(c_in && c_lvl + 1 == Kt);
    const uint64_t upper_cls = __ballot(c_in && c_lvl + 1 < Kt);
    // Upper-level classes with the scratch: every leaf's capacity (clamped to
    // pods, which keeps capsum >= pods exact) is added into its domain's 64-bit
    // LDS sum and its occupancy into the domain's bit, in the same pass over
    // the leaves as the leaf-level classes; the words follow from the sums.
    // Scratch: [sums of each upper class's domains][occupancy bits per upper level].
    const bool scr = f.fscr_words != 0 && upper_cls != 0ull;
    uint64_t* s_usum = reinterpret_cast<uint64_t*>(
        (reinterpret_cast<uintptr_t>(s_stage + kFusedStage) + 7) & ~static_cast<uintptr_t>(7));
    const uint32_t usz = scr && ((upper_cls >> lane) & 1ull) ? f.topo.D[c_lvl] : 0u;
    const uint32_t uincl = wave_incl_scan(usz, lane);
    const uint32_t c_uoff = uincl - usz;  // lane c: first sum of class c
    uint64_t* s_uocc = s_usum + (uint32_t)__builtin_amdgcn_readlane((int)uincl, 63);
    const uint32_t ooff0 = 0, ooff1 = (f.topo.D[0] + 63) >> 6, ooff2 = ooff1 + ((f.topo.D[1] + 63) >> 6);
    if (scr) {
        for (uint32_t i = threadIdx.x; i < f.fscr_words; i += kTallyThreads) lds_ptr(s_usum)[i] = 0;
        __syncthreads();
    }
    // every thread takes 4-leaf chunks, loads occupancy once and the capacities
    // of every class in the pass (8 classes per group, all loads first), then
    // ORs each leaf-level class's 4 feasibility bits into its LDS word and adds
    // each upper class's clamped capacities into its domain sums
    {
        const uint32_t L = f.topo.D[Kt - 1];
        const uint64_t pass_cls = leaf_cls | (scr ? upper_cls : 0ull);
        const uint32_t npc = (uint32_t)__popcll(pass_cls);
        static_assert(kTallyClasses <= 16, "the fused tail's leaf pass takes at most 16 classes");
        const TailFeasArgs t{a.cap_out, a.occ_out, a.ld, L, pass_cls, leaf_cls, npc, scr, Kt, ooff0, ooff1, ooff2,
                             s_uocc, s_usum, s_feas, c_pods, c_beg, c_lvl, c_uoff,
                             f.topo_in_lds ? s_topo : nullptr, m.s_poff, f.topo.par[1], f.topo.par[2], f.topo.par[3]};
        if (npc > 8) tail_leaf_pass<16>(t);
        else if (npc > 0) tail_leaf_pass<8>(t);
    }
    JSP_STAMP(4000u, 4);
    if (scr) {
        __syncthreads();
        // upper classes' words from the sums: one wave per word, words dealt to the waves in turn
        uint64_t uc = upper_cls;
        uint32_t base = 0;
        while (uc != 0ull) {
            const uint32_t c = (uint32_t)__builtin_ctzll(uc);
            uc &= uc - 1ull;
            const uint32_t wb = (uint32_t)__builtin_amdgcn_readlane((int)c_beg, (int)c);
            const uint32_t we = (uint32_t)__builtin_amdgcn_readlane((int)c_end, (int)c);
            const uint32_t lvl = (uint32_t)__builtin_amdgcn_readlane((int)c_lvl, (int)c);
            const uint32_t pods = (uint32_t)__builtin_amdgcn_readlane((int)c_pods, (int)c);
            JSP_LDS const uint64_t* sum = lds_ptr(s_usum) + (uint32_t)__builtin_amdgcn_readlane((int)c_uoff, (int)c);
            JSP_LDS const uint64_t* uocc = lds_ptr(s_uocc);
            const uint32_t D = f.topo.D[lvl];
            for (uint32_t gw = wb + (wid + kTallyWaves - base % kTallyWaves) % kTallyWaves; gw < we;
                 gw += kTallyWaves) {
                const uint32_t d = (gw - wb) * 64u + (uint32_t)lane;
                const bool ok = d < D && sum[d] >= pods && ((uocc[(lvl == 0 ? ooff0 : lvl == 1 ? ooff1 : ooff2) + (d >> 6)] >> (d & 63u)) & 1ull) == 0ull;
                const uint64_t word = __ballot(ok);
                if (lane == 0) s_feas[gw] = word;
            }
            base += we - wb;
        }
    } else {
        // classes above the leaves: one wave per word (prefix sums over the word's
        // leaf range, feas_word_upper), words dealt to the waves in turn
        uint64_t uc = upper_cls;
        uint32_t base = 0;
        while (uc != 0ull) {
            const uint32_t c = (uint32_t)__builtin_ctzll(uc);
            uc &= uc - 1ull;
            const uint32_t wb = (uint32_t)__builtin_amdgcn_readlane((int)c_beg, (int)c);
            const uint32_t we = (uint32_t)__builtin_amdgcn_readlane((int)c_end, (int)c);
            const uint32_t lvl = (uint32_t)__builtin_amdgcn_readlane((int)c_lvl, (int)c);
            const uint32_t pods = (uint32_t)__builtin_amdgcn_readlane((int)c_pods, (int)c);
            for (uint32_t gw = wb; gw < we; ++gw) {
                if ((base + gw - wb) % kTallyWaves == (uint32_t)wid) {
                    const uint64_t word = feas_word_upper(a.cap_out, a.occ_out, a.ld, lvl, pods, c, gw - wb, f.topo, lane);
                    if (lane == 0) s_feas[gw] = word;
                }
            }
            base += we - wb;
        }
    }
    __syncthreads();
    JSP_STAMP(4000u, 2);
    JSP_CLK(4090u, 0);
    JSP_STAMP(4090u, 1);
    if (f.topo_in_lds)
        assign_block<kTallyThreads, true>(s_feas, f.C, f.topo, f.run_class, f.run_len, n_runs, J, f.assign,
                                          f.stats, s_taken, m, s_topo, s_win, s_stage, kFusedStage, nullptr, nullptr,
                                          f.we);
    else
        assign_block<kTallyThreads, false>(s_feas, f.C, f.topo, f.run_class, f.run_len, n_runs, J, f.assign,
                                           f.stats, s_taken, m, s_topo, s_win, s_stage, kFusedStage, nullptr, nullptr,
                                           f.we);
    JSP_CLK(4090u, 2);
    JSP_STAMP(4090u, 3);
    if (done) signal_host(done, epoch, true);
}

// Small words after a fused tile's tally carve (sized for class group 0).
__device__ __forceinline__ uint32_t* fused_flags(uint32_t* lds, const TallyArgs& a, const FusedArgs& f) {
    return lds + tally_lds_words((int)f.cpg, (int)f.cpg + 1, (int)a.la);
}

template <int W, int R>
__global__ __launch_bounds__(kTallyThreads) void place_fused_kernel(TallyArgs a, FusedArgs f) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* s_flag = fused_flags(lds, a, f);
    if (threadIdx.x == 0)
        *s_flag = (uint32_t)(__hip_atomic_fetch_add(f.ticket, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) -
                             f.tile_base);
    __syncthreads();
    const uint32_t tile = *s_flag;
    const uint32_t n_tiles = a.n_blocks * f.groups;
    if (tile >= n_tiles) return;  // a spare workgroup: every tile is taken
    JSP_STAMP(tile, 0);
    {
        // this tile's row block and class group (the LDS carve is sized for group 0)
        const FusedTile ft = fused_tile(tile, f.groups, f.cpg, f.C);
        TallyArgs ag = a;
        ag.c0 = ft.c0;
        ag.nc = ft.nc;
        ag.do_occ = ft.do_occ;
        tally_block<W, R>(ag, ft.blk, lds);
    }

    // publish. With sc1_out the sums went out write-through, so every storing
    // wave's wait and the barrier order them before the ticket add (G16 R1: no
    // release fence); otherwise the agent release writes this XCD's L2 back.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        if (!a.sc1_out) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned long long old =
            __hip_atomic_fetch_add(f.ticket + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *s_flag = (old + 1 - f.done_base) == n_tiles ? 1u : 0u;
    }
    __syncthreads();
    JSP_STAMP(tile, 5);
    if (*s_flag == 0) return;
    fused_tail<W, R>(a, f, lds, f.J, f.n_runs, f.epoch, f.done);
}

// ----------------------------------------------------------------- single-class compaction
// When the engine holds one class and it sits at the leaf level, the greedy is
// a stream compaction: job j gets the j-th feasible leaf. Each workgroup
// tallies its leaves, counts its feasible ones, and learns how many feasible
// leaves precede it by a decoupled look-back over 8-byte {epoch|status, value}
// granules (sc1 stores / loads: the data is the flag, G16 R2). Tile order comes
// from a ticket, so a workgroup only ever waits on tiles that already started.
constexpr uint32_t kAggregate = 1, kPrefix = 2;
static_assert(kMaxBlkLeaves <= kTallyThreads, "compaction keeps one leaf per thread");

// `local`: every tile of the launch runs on one XCD (the service's XCC vote):
// a plain store keeps the line in that XCD's L2, where the other tiles' sc1
// loads find it; otherwise write-through (sc1), correct across XCDs.
__device__ __forceinline__ void put_granule(unsigned long long* g, uint32_t epoch, uint32_t status, uint32_t v,
                                            bool local = false) {
    const unsigned long long x = ((unsigned long long)((epoch << 2) | status) << 32) | v;
    if (local) __hip_atomic_store(g, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else __hip_atomic_store(g, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The compaction after the tally: `ok` = this thread's leaf (l0 + tid) is
// feasible. Scan of the feasible count, look back for the feasible leaves
// before the tile, scatter its jobs' domains. `sys`: assign[] and stats are in
// pinned host memory (system-scope stores). s_x: the small LDS words after
// the tally carve ([2] prefix [3] timeout [4..16] scan). tag != 0 (the
// resident service): assign is a u64 array and entry j is written as
// (tag << 32) | domain in ONE system-scope store, so the host knows each entry
// has arrived from the entry itself and returns without waiting for the
// tiles' done words (which then only gate the next request).
__device__ __forceinline__ void compact_finish(const TallyArgs& a, uint32_t tile, uint32_t l0, bool ok, uint32_t epoch,
                                               uint32_t J, uint32_t n_runs, unsigned long long* g, uint32_t spin_limit,
                                               int32_t* assign, uint32_t* stats, uint32_t* err, bool sys, uint32_t* s_x,
                                               JSP_LDS uint32_t* clk, uint32_t tag, bool local) {
    unsigned long long* assign64 = reinterpret_cast<unsigned long long*>(assign);
    const unsigned long long tag_hi = (unsigned long long)tag << 32;
    const int tid = threadIdx.x, lane = tid & 63;
    uint32_t total;
    const uint32_t rank = block_excl_scan<kTallyThreads>(ok ? 1u : 0u, s_x + 4, &total);
    JSP_STAMP(tile, 3);
#ifndef JSP_AB_FINESTAMP
    svc_stamp(clk, 3);
#endif
    if (tid == 0) put_granule(g + tile, epoch, tile == 0 ? kPrefix : kAggregate, total, local);
    if (tid < 64) {  // wave 0: look back
        uint32_t prefix = 0, spins = 0;
        bool timeout = false;
        for (int p = (int)tile - 1; p >= 0; p -= 64) {
            const int idx = p - lane;
            uint32_t st = 0, v = 0;
            while (true) {
                if (idx >= 0) {
                    const unsigned long long x = __hip_atomic_load(g + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const uint32_t tag = (uint32_t)(x >> 32);
                    st = (tag >> 2) == epoch ? (tag & 3u) : 0u;
                    v = (uint32_t)x;
                }
                if (__all(idx < 0 || st != 0)) break;
                if (++spins > spin_limit) { timeout = true; break; }
                __builtin_amdgcn_s_sleep(1);
            }
            const unsigned long long pm = __ballot(idx >= 0 && st == kPrefix);
            const int stop = pm ? __builtin_ctzll(pm) : 64;
            uint32_t x = (idx >= 0 && lane <= stop) ? v : 0u;
            for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
            prefix += x;
            if (pm || timeout) break;
        }
        if (lane == 0) {
            // A tile that timed out knows no prefix: it publishes none (its
            // aggregate stays visible, so later tiles still sum correctly past
            // it), scatters nothing and reports the launch as failed.
            if (tile != 0 && !timeout) put_granule(g + tile, epoch, kPrefix, prefix + total, local);
            s_x[2] = prefix;
            s_x[3] = timeout ? 1u : 0u;
        }
    }
    __syncthreads();
    JSP_STAMP(tile, 4);
#ifndef JSP_AB_FINESTAMP
    svc_stamp(clk, 4);
#endif
    const uint32_t prefix = s_x[2];
    const bool failed = s_x[3] != 0;
    if (!failed) {
        if (ok && prefix + rank < J) {
            const uint32_t d = a.leaf_base + l0 + tid;
            if (tag) store_out(assign64 + prefix + rank, tag_hi | d, true);
            else store_out(assign + prefix + rank, (int32_t)d, sys);
        }
        if (tile + 1 == a.n_blocks) {
            const uint32_t placed = prefix + total < J ? prefix + total : J;
            for (uint32_t j = placed + tid; j < J; j += kTallyThreads) {
                if (tag) store_out(assign64 + j, tag_hi | 0xFFFFFFFFull, true);
                else store_out(assign + j, -1, sys);
            }
            if (tid == 0 && stats) {
                store_out(stats, n_runs, sys);
                store_out(stats + 1, placed, sys);
            }
        }
    } else if (tid == 0) {
        __hip_atomic_store(err, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// The bitmap answer of the resident service (ServiceArgs::bits): the tile's
// feasible leaves (thread t: leaf l0 + t) as four 64-leaf wave ballots, each
// sent as two tagged halves (tag << 32 | 32 bits: one atomic 8-byte store
// each) into the tile's own 64-byte line of pinned host memory. The host takes
// the tiles' lines in order and gives job j the j-th feasible leaf -- no
// look-back between tiles, no per-job scatter, one line per tile on the link.
// The four ballots meet in LDS (s_w: 8 words) and wave 0's lanes 0-7 write the
// line with one store instruction: one whole-line write to host memory
// instead of four partial ones (each a read-modify-write there, and a
// snoop of the host's polling copy).
// The line goes out from the last wave, not wave 0: a host store retires
// only after a link round trip, and wave 0's thread 0 polls the bell for the
// next request -- its first poll would wait (vmcnt) for these stores.
__device__ __forceinline__ void bitmap_finish(uint32_t tile, bool ok, uint32_t tag, unsigned long long* bits,
                                              uint32_t* s_w) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t word = __ballot(ok);
    if (lane < 2) s_w[2 * wid + lane] = lane == 0 ? (uint32_t)word : (uint32_t)(word >> 32);
    __syncthreads();
    if (wid == kTallyWaves - 1 && lane < 8)
        __hip_atomic_store(bits + 8u * tile + (uint32_t)lane, ((unsigned long long)tag << 32) | s_w[lane],
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
static_assert(kTallyThreads == 256, "bitmap_finish: four waves, eight halves per tile line");

// One compaction tile: tally its leaves (sums in LDS), then compact_finish
// (or bitmap_finish when `bits` is given: the resident service).
template <int W, int R, bool STAGED = false>
__device__ __forceinline__ void compact_tile(const TallyArgs& a, uint32_t tile, uint4 bt, uint32_t epoch, uint32_t pods,
                                             uint32_t J, uint32_t n_runs, unsigned long long* g, uint32_t spin_limit,
                                             int32_t* assign, uint32_t* stats, uint32_t* err, bool sys, uint32_t* lds,
                                             uint32_t* s_x, JSP_LDS uint32_t* clk = nullptr, JSP_LDS u32x4* row_cache = nullptr,
                                             bool use_cache = false, uint32_t tag = 0, bool local = false,
                                             unsigned long long* bits = nullptr) {
    const int tid = threadIdx.x;
    // ends with the leaf sums in LDS (acc[0] cap, acc[1] occ)
    tally_block<W, R, STAGED>(a, tile, lds, bt, clk, row_cache, use_cache);
    JSP_STAMP(tile, 2);
#ifndef JSP_AB_FINESTAMP
    svc_stamp(clk, 2);
#endif
    const uint32_t* s_acc = lds + tally_acc_off(1);
    const uint32_t nl = bt.y - bt.x;
    const bool ok = (uint32_t)tid < nl && s_acc[tid] >= pods && s_acc[a.la + tid] == 0;
    if (bits) bitmap_finish(tile, ok, tag, bits, s_x + 4);
    else compact_finish(a, tile, bt.x, ok, epoch, J, n_runs, g, spin_limit, assign, stats, err, sys, s_x, clk, tag, local);
}

template <int W, int R>
__global__ __launch_bounds__(kTallyThreads) void place_compact_kernel(TallyArgs a, CompactArgs f) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* s_x = lds + tally_lds_words(a);  // [0] tile [2] prefix [3] timeout [4..] scan scratch
    // tiles in start order (oversubscribed grid): a tile only ever waits on
    // tiles that workgroups already hold, and the first-started take them all
    if (threadIdx.x == 0)
        s_x[0] = (uint32_t)(__hip_atomic_fetch_add(f.ticket, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) -
                            f.tile_base);
    __syncthreads();
    const uint32_t tile = s_x[0];
    if (tile >= a.n_blocks) return;  // a spare workgroup: every tile is taken
    JSP_STAMP(tile, 0);
    const bool sys = f.done != nullptr;  // host path: assign[] and stats are in pinned host memory
    compact_tile<W, R>(a, tile, a.blk[tile], f.epoch, f.pods, f.J, f.n_runs, f.granules, f.spin_limit, f.assign,
                       f.stats, f.err, sys, lds, s_x);
    if (sys) signal_host(f.done + tile, f.epoch, false);
    JSP_STAMP(tile, 5);
}

// ----------------------------------------------------------------- resident placement service
// The compaction kept resident between placements: one
// workgroup per tile, each polling the host-mapped request word (vector
// system-scope loads; the host writes it with one 64-bit store). A request is
// (J << 32) | seq; the tile runs compact_tile with granules tagged by seq,
// writes assign[] / stats into pinned host memory and publishes done[tile] =
// seq. Every workgroup leaves on kSvcStop or after idle_ticks of the 100 MHz
// clock without a request, so the grid always drains; a tile whose look-back
// partner left (the host posted into an exit) times out and reports it.
// Dispatcher workgroup of the service (the grid's last block): lane 0 of
// each of its 4 waves polls the host request word, one system-scope load in
// flight each, the waves a quarter of a host-link round trip apart, so a
// request is seen ~1/4 round trip after it lands. It rings the device bell
// (one sc1 8-byte store, tag = seq), which the tiles poll close by. Only this
// workgroup reads host memory: tiles polling it themselves see a request up
// to a whole round trip apart and load the link with reads.
// A snapshot patch the dispatcher applies itself (ServiceArgs::pdesc,
// request bit kReqPatch): the whole workgroup overwrites the rows from the
// staged delta in pinned memory with write-through stores, every wave
// drains, and lane 0 publishes the patch's number in the host word -- no
// launch per patch while the service is up, and none besides the service's
// own when a patch wakes it.
__device__ void service_apply_patch(const ServiceArgs& v, const TallyArgs& a) {
    // the descriptor and the staged delta are rewritten by the host for every
    // patch: drop what this CU's caches hold of the last one
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    const PatchDesc* d = v.pdesc;
    const uint32_t n = d->n;
    for (uint32_t i = threadIdx.x; i < n; i += kTallyThreads) {
        const uint32_t row = d->rows[i];
        if (d->dlab)
            for (int w = 0; w < a.W; ++w)
                __hip_atomic_store(const_cast<uint64_t*>(a.labels) + (size_t)w * a.npad + row, d->dlab[(size_t)w * n + i],
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (d->dtaint)
            __hip_atomic_store(const_cast<uint32_t*>(a.taints) + row, d->dtaint[i], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        if (d->dfree)
            for (int r = 0; r < a.R; ++r)
                __hip_atomic_store(const_cast<uint32_t*>(a.freer) + (size_t)r * a.npad + row, d->dfree[(size_t)r * n + i],
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (d->dexcl)
            __hip_atomic_store(const_cast<int32_t*>(a.excl) + row, d->dexcl[i], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(v.pdone, d->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The inline form: n and the column flags come with the request, the layout
// follows from them, so each thread issues every load of its rows (and lane 0
// the header) before the first store -- one round trip over the host link.
__device__ void service_apply_inline(const ServiceArgs& v, const TallyArgs& a, uint32_t nf) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    const uint32_t n = nf & 0xFFFFu, fl = nf >> 16;
    const PatchInlineLayout L = patch_inline_layout(n, fl, (uint32_t)a.W, (uint32_t)a.R);
    const char* b = v.pstage;
    uint32_t seq = 0;
    if (threadIdx.x == 0) seq = *reinterpret_cast<const uint32_t*>(b);
    for (uint32_t i = threadIdx.x; i < n; i += kTallyThreads) {
        const uint32_t row = reinterpret_cast<const uint32_t*>(b + L.rows)[i];
        uint64_t lab[4];
        uint32_t fr[4];
        uint32_t tn = 0;
        int32_t ex = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w)
            if ((fl & kPatchLab) && w < a.W) lab[w] = reinterpret_cast<const uint64_t*>(b + L.lab)[(size_t)w * n + i];
        if (fl & kPatchTaint) tn = reinterpret_cast<const uint32_t*>(b + L.taint)[i];
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if ((fl & kPatchFree) && r < a.R) fr[r] = reinterpret_cast<const uint32_t*>(b + L.free)[(size_t)r * n + i];
        if (fl & kPatchExcl) ex = reinterpret_cast<const int32_t*>(b + L.excl)[i];
#pragma unroll
        for (int w = 0; w < 4; ++w)
            if ((fl & kPatchLab) && w < a.W)
                __hip_atomic_store(const_cast<uint64_t*>(a.labels) + (size_t)w * a.npad + row, lab[w], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        if (fl & kPatchTaint)
            __hip_atomic_store(const_cast<uint32_t*>(a.taints) + row, tn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if ((fl & kPatchFree) && r < a.R)
                __hip_atomic_store(const_cast<uint32_t*>(a.freer) + (size_t)r * a.npad + row, fr[r], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        if (fl & kPatchExcl)
            __hip_atomic_store(const_cast<int32_t*>(a.excl) + row, ex, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(v.pdone, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// A micro-patch carried in the request line (jsp_internal.h kMailbox*): the
// rows' words are already in LDS (s_w: m records of 3 + 2W + R words, row ids
// distinct); one thread per word stores it (agent scope: the tiles' sc1
// reloads find it in L2), every store drains, and thread 0 publishes the
// patch number. No host-link round trip beyond the request's own.
// A micro-patch's row stores (the rows ride in the request line, s_w). `plain`:
// the co-located service -- plain stores that stay in this XCD's L2, where the
// tiles' sc1 reloads find them, retired in an L2 round trip; otherwise
// write-through (agent scope), which retires only once the memory side has the
// data. Each thread stores one word; the barrier ends with every store retired.
__device__ void service_micro_stores(const TallyArgs& a, const uint32_t* s_w, uint32_t m, uint32_t fl, bool plain) {
    const uint32_t W = (uint32_t)a.W, R = (uint32_t)a.R, rw = 3u + 2u * W + R;
    const uint32_t t = threadIdx.x;
    if (t < m * rw) {
        const uint32_t r = t / rw, k = t - r * rw;
        const uint32_t row = s_w[r * rw], val = s_w[t];
        uint32_t* p = nullptr;
        if (k == 0u || row >= a.npad) {
            // the row id itself
        } else if (k <= 2u * W) {
            if (fl & kPatchLab)
                p = reinterpret_cast<uint32_t*>(const_cast<uint64_t*>(a.labels) + (size_t)((k - 1) >> 1) * a.npad + row) +
                    ((k - 1) & 1u);
        } else if (k == 2u * W + 1u) {
            if (fl & kPatchTaint) p = const_cast<uint32_t*>(a.taints) + row;
        } else if (k < 2u * W + 2u + R) {
            if (fl & kPatchFree) p = const_cast<uint32_t*>(a.freer) + (size_t)(k - 2u * W - 2u) * a.npad + row;
        } else if (k == 2u * W + 2u + R) {
            if (fl & kPatchExcl) p = reinterpret_cast<uint32_t*>(const_cast<int32_t*>(a.excl)) + row;
        }
        if (p) {
            if (plain) __hip_atomic_store(p, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            else __hip_atomic_store(p, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

// Whether request q's micro-patch goes to the resident tiles through the
// microbox (their rows in registers, patched there, no reload): m rows, a
// patch number this dispatcher has not applied (pseq != last), a co-located
// resident service, and rows not marked patched otherwise (a dirty request
// reloads them anyway; a patch-only request has no tiles to ring).
__device__ __forceinline__ bool microbox_ring(const ServiceArgs& v, uint32_t m, uint32_t jw, uint32_t pseq,
                                              uint32_t last, bool local) {
    return m > 0u && pseq != last && v.mbox != nullptr && v.resident != 0u && local &&
           (jw & (kReqDirty | kReqPatchOnly)) == 0u;
}

// The dispatcher's LDS words (s_p): [0] claimed request seq [1] J word [2]
// stop [3] second request word [4] micro rows [5] patch number [6] column
// flags [7] last applied patch number [8 .. 8 + kMailboxPayload) micro words
// [8 + kMailboxPayload] the request's seen stamp, [9 + kMailboxPayload] its
// rung stamp when the claiming wave rang (timing on).
__device__ __forceinline__ void service_dispatch(const ServiceArgs& v, const TallyArgs& a, uint32_t* s_p,
                                                 bool local = false) {
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t rw = 3u + 2u * (uint32_t)a.W + (uint32_t)a.R;  // words of a micro-patch row
    uint32_t seq = v.seq0;
    if (threadIdx.x == 0) {
        s_p[0] = 0;
        s_p[2] = 0;
        s_p[7] = 0;  // patch numbers are never 0
        __hip_atomic_store(v.ready, v.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __syncthreads();
    const uint32_t* mb = reinterpret_cast<const uint32_t*>(v.mailbox);
    while (true) {
        {
            // every wave polls, the waves a quarter of the host-link round trip apart
            const uint64_t t0 = wall_clock64();
            while (wall_clock64() - t0 < (uint64_t)w * kSvcStaggerTicks) __builtin_amdgcn_s_sleep(1);
            while (true) {
                if (__hip_atomic_load(s_p + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0 ||
                    __hip_atomic_load(s_p + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0)
                    break;
                // the request line in one load: lane c < kMailboxChunks reads
                // 16-byte chunk c (each chunk carries the request's seq: a torn
                // read shows two seqs)
                uint4 x = make_uint4(0u, 0u, 0u, 0u);
                if (lane < kMailboxChunks)
                    asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)"
                                 : "=v"(x) : "v"(mb + 4 * lane) : "memory");
                const uint32_t q = (uint32_t)__builtin_amdgcn_readlane((int)x.x, 0);
                if (q == kSvcStop) {
                    if (lane == 0) __hip_atomic_store(s_p + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    break;
                }
                const uint32_t jw = (uint32_t)__builtin_amdgcn_readlane((int)x.y, 0);
                const uint32_t z0 = (uint32_t)__builtin_amdgcn_readlane((int)x.z, 0);
                const uint32_t w2 = (uint32_t)__builtin_amdgcn_readlane((int)x.w, 0);
                const uint32_t tag1 = (uint32_t)__builtin_amdgcn_readlane((int)x.x, 1);
                const uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)x.y, 1);
                const uint32_t nch = m > 0u ? (m * rw + 2u) / 3u : 0u;  // payload chunks in use (3 words each)
                const bool mine = lane >= 2u && lane < 2u + nch;
                const bool torn = __ballot(mine && x.x != q) != 0ull;
                if (q != seq && q != 0 && z0 == q && tag1 == q && !torn && 2u + nch <= kMailboxChunks) {
                    // claim it (two waves may see it; one hands it on)
                    uint32_t won = 0;
                    if (lane == 0) won = atomicCAS(s_p + 0, 0u, q) == 0u ? 1u : 0u;
                    if (__builtin_amdgcn_readlane((int)won, 0) == 0) break;
                    const bool patch = (jw & kReqPatch) != 0u || m > 0u;
                    const uint32_t t_seen = (uint32_t)wall_clock64();
                    if (!patch && lane == 0) {
                        // ring at once: nothing to apply first
                        const unsigned long long mm = ((unsigned long long)jw << 32) | q;
                        if (local) __hip_atomic_store(v.bell, mm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        else __hip_atomic_store(v.bell, mm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                    if (microbox_ring(v, m, jw, (uint32_t)__builtin_amdgcn_readlane((int)x.z, 1), s_p[7], local)) {
                        // a micro-patch for the resident tiles: its words into
                        // the microbox and the bell rung from this wave, at
                        // once (the barrier below waits for the other waves'
                        // host polls in flight, up to a link round trip)
                        const uint32_t mw = m * rw;
                        const uint32_t b = 3u * (lane - 2u);
                        const unsigned long long tq = (unsigned long long)q << 32;
                        if (mine) {
                            if (b < mw)
                                __hip_atomic_store(v.mbox + 1 + b, tq | x.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            if (b + 1 < mw)
                                __hip_atomic_store(v.mbox + 2 + b, tq | x.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            if (b + 2 < mw)
                                __hip_atomic_store(v.mbox + 3 + b, tq | x.w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        }
                        if (lane == 0) {
                            const uint32_t fl1 = (uint32_t)__builtin_amdgcn_readlane((int)x.w, 1);
                            __hip_atomic_store(v.mbox, tq | m | (fl1 << 16), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            const uint32_t bj = (jw & ~(kReqPatch | kReqPatchOnly | kReqPatchInline)) | kBellMicro;
                            __hip_atomic_store(v.bell, ((unsigned long long)bj << 32) | q, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
                            s_p[9 + kMailboxPayload] = (uint32_t)wall_clock64();
                        }
                    }
                    if (v.clk && lane == 0) {  // timing on: the dispatcher's row after the tiles' (seen, rung)
                        if (patch) {
                            // written after the apply: a host store here would sit in
                            // the apply's wait for its row stores
                            s_p[8 + kMailboxPayload] = t_seen;
                        } else {
                            uint32_t* dc = v.clk + kSvcClkSlots * v.n_tiles;
                            __hip_atomic_store(dc, t_seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                            __hip_atomic_store(dc + 1, (uint32_t)wall_clock64(), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_SYSTEM);
                        }
                    }
                    if (lane == 1) {
                        s_p[1] = jw;
                        s_p[3] = w2;
                        s_p[4] = m;
                        s_p[5] = x.z;  // patch number
                        s_p[6] = x.w;  // column flags
                    }
                    if (mine) {
                        s_p[8 + 3 * (lane - 2)] = x.y;
                        s_p[9 + 3 * (lane - 2)] = x.z;
                        s_p[10 + 3 * (lane - 2)] = x.w;
                    }
                    break;
                }
                if (w == 0 && wall_clock64() - t0 > v.idle_ticks) {
                    if (lane == 0) __hip_atomic_store(s_p + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    break;
                }
            }
        }
        __syncthreads();
        const uint32_t q = s_p[0], jw = s_p[1], nr = s_p[3], m = s_p[4], pseq = s_p[5], fl = s_p[6];
        if (q == 0) {  // stop or idle: every tile leaves too (a request claimed beside an idle exit is answered first)
            if (threadIdx.x == 0)
                __hip_atomic_store(v.bell, ((unsigned long long)v.gen << 32) | kSvcStop, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        const bool patch = (jw & kReqPatch) != 0u || m > 0u;
        if (patch) {
            // a patch this dispatcher applied already (carried again by a
            // request posted before its completion word came back) is not
            // applied twice; each apply ends with a barrier and the completion word
            const bool fresh = pseq != s_p[7];
            // a micro-patch handed to the resident tiles in the microbox: the
            // claiming wave has rung the bell already (the rows are written
            // through below)
            const bool mb = microbox_ring(v, m, jw, pseq, s_p[7], local);
            if (fresh && !mb) {
                if (m > 0u) {
                    // a micro-patch on a co-located service: into this XCD's L2
                    // first (the tiles reload from there), written through for
                    // every other reader after the bell
                    service_micro_stores(a, s_p + 8, m, fl, local);
                } else if (jw & kReqPatchInline) {
                    service_apply_inline(v, a, nr);
                } else {
                    service_apply_patch(v, a);
                }
            }
            if (threadIdx.x == 0 && (jw & kReqPatchOnly) == 0u) {  // the request behind the patch
                // rows changed (and not handed over in the microbox): every tile reloads
                if (!mb) {
                    const uint32_t bj = (jw & ~(kReqPatch | kReqPatchOnly | kReqPatchInline)) |
                                        (fresh && m > 0u ? kReqDirty : 0u);
                    const unsigned long long mm = ((unsigned long long)bj << 32) | q;
                    if (local) __hip_atomic_store(v.bell, mm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    else __hip_atomic_store(v.bell, mm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                if (v.clk) {
                    const uint32_t t_rung = mb ? s_p[9 + kMailboxPayload] : (uint32_t)wall_clock64();
                    __hip_atomic_store(v.clk + kSvcClkSlots * v.n_tiles, s_p[8 + kMailboxPayload], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store(v.clk + kSvcClkSlots * v.n_tiles + 1, t_rung, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
            if (fresh && m > 0u) {
                if (local || mb) service_micro_stores(a, s_p + 8, m, fl, false);  // in memory for every other reader
                // its completion word: readers other than this service's
                // tiles (launches, uploads, jsp_engine_sync) wait for it
                if (threadIdx.x == 0) __hip_atomic_store(v.pdone, pseq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            if (threadIdx.x == 0) {
                if (fresh) s_p[7] = pseq;
                // the host learns that a request with a patch was taken (a
                // later request then need not carry the patch again); after
                // the stores, whose retirement waits would otherwise include
                // this host store's link round trip
                __hip_atomic_store(v.taken, q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        seq = q;
        // the next request comes only after every tile has answered this one
        // (the host waits for all done words), so polling may resume at once
        __syncthreads();
        if (threadIdx.x == 0) s_p[0] = 0;
        __syncthreads();
    }
}

// The micro-patch rows of request q from the microbox (ServiceArgs::mbox):
// every wave loads the whole box in one pass (lane k word k, sc1: L2 hits on
// the co-located service) and takes the words by readlane. The dispatcher
// stores the words and rings the bell without waiting between them, so a
// word may land after the bell: the pass repeats until every word in use
// carries q (bounded; the stores were issued before the bell's). Thread t
// holds rows mine .. mine + 3 in registers, and a patched row among them
// takes the columns the patch carries (micro_row_words layout: row id, W
// label words as lo/hi halves, taint, R free, excl).
// Returns false (wave-uniform) when the words still lack q after `spins`
// passes: the registers are then left as they were, and the tile reports the
// failure instead of answering (place_service_kernel: kErrMicro).
template <int W, int R>
__device__ __forceinline__ bool apply_microbox(const unsigned long long* mb, uint32_t q, uint32_t mine,
                                               RowRegs<W, R>& x, uint32_t spins) {
    constexpr uint32_t rw = 3u + 2u * W + R;
    const uint32_t lane = threadIdx.x & 63u;
    unsigned long long t = 0;
    bool got = false;
    for (uint32_t s = 0; s < spins; ++s) {
        if (lane <= kMailboxPayload) t = __hip_atomic_load(mb + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t m0 = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)t, 0) & 0xFFFFu;
        const bool ok = lane > kMailboxPayload || lane > m0 * rw || (uint32_t)(t >> 32) == q;
        if (__ballot(!ok) == 0ull) {
            got = true;
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    if (!got) return false;
    const int word = (int)(uint32_t)t;
    const uint32_t mf = (uint32_t)__builtin_amdgcn_readlane(word, 0);
    const uint32_t m = mf & 0xFFFFu, fl = mf >> 16;
    for (uint32_t r = 0; r < m && (r + 1) * rw <= kMailboxPayload; ++r) {
        const uint32_t b = 1 + r * rw;
        const uint32_t i = (uint32_t)__builtin_amdgcn_readlane(word, b) - mine;
        uint32_t v[rw];
#pragma unroll
        for (uint32_t k = 1; k < rw; ++k) v[k] = (uint32_t)__builtin_amdgcn_readlane(word, b + k);
        if (i >= 4u) continue;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            if ((uint32_t)s != i) continue;
            if (fl & kPatchLab) {
#pragma unroll
                for (int w = 0; w < W; ++w) x.lab[w][s] = ((uint64_t)v[2 + 2 * w] << 32) | v[1 + 2 * w];
            }
            if (fl & kPatchTaint) x.tn[s] = v[1 + 2 * W];
            if (fl & kPatchFree) {
#pragma unroll
                for (int r2 = 0; r2 < R; ++r2) x.fr[r2][s] = v[2 + 2 * W + r2];
            }
            if (fl & kPatchExcl) x.ex[s] = (int32_t)v[2 + 2 * W + R];
        }
    }
    return true;
}

// ---- resident compaction tile (ServiceArgs::resident): every tile is one
// chunk, so thread t's 4 rows and leaf t never change while the service
// lives. The rows stay in registers (reloaded with sc1 loads when a patch
// marked them dirty), the class in scalar registers, and each leaf's
// chunk-local row bounds in registers: a request evaluates the rows, scans
// them (two independent DPP chains), stores the row prefixes, crosses ONE
// barrier and forms each leaf's capacity and occupancy from two prefix
// differences -- no class-record or leaf-start LDS round trips, no
// accumulation buffer, no second barrier before the feasible-count scan.
struct ResidentLeaf {
    uint32_t xh, xb;  // chunk-local last row of the leaf, row before its first
    uint32_t wh, wb;  // their waves (256 rows per wave)
    bool live, has_lo;
};

__device__ __forceinline__ ResidentLeaf resident_leaf(const TallyArgs& a, uint4 bt) {
    ResidentLeaf f{0u, 0u, 0u, 0u, false, false};
    const uint32_t nl = bt.y - bt.x, li = threadIdx.x;
    if (li < nl) {
        const uint32_t base = bt.z & ~3u;
        const uint32_t s = a.leaf_start[bt.x + li], e = a.leaf_start[bt.x + li + 1];
        f.live = s < e;
        f.xh = f.live ? e - 1 - base : 0u;
        f.has_lo = f.live && s > base;
        f.xb = f.has_lo ? s - 1 - base : 0u;
        f.wh = f.xh >> 8;
        f.wb = f.xb >> 8;
    }
    return f;
}

// Sum of the wave totals before wave w (0..3), branch-free: three selects and
// an add (a nested conditional compiled to divergent branches here).
__device__ __forceinline__ uint32_t wave_off(uint4 ws, uint32_t w) {
    return (w > 0u ? ws.x : 0u) + (w > 1u ? ws.y : 0u) + (w > 2u ? ws.z : 0u);
}

// A/B build (tools/bin/ab_eval, -DJSP_AB_EVALSTAMP): real-time stamps inside
// the resident evaluation, in the service's stamp slots the bitmap path leaves
// free (3 after the row predicates, 4 after the scans' LDS stores, 6 after the
// barrier, 7 at the end). Diagnostic only.
#ifdef JSP_AB_EVALSTAMP
#define JSP_EVAL_STAMP(clk, s) \
    do {                       \
        if ((clk) && threadIdx.x == 0) (clk)[s] = (uint32_t)wall_clock64(); \
    } while (0)
#else
#define JSP_EVAL_STAMP(clk, s) \
    do {                       \
    } while (0)
#endif

template <int W, int R>
__device__ __forceinline__ bool resident_eval(const ClassRegs<W, R>& k, const RowRegs<W, R>& x, const bool (&valid)[4],
                                              const ResidentLeaf& lf, JSP_LDS uint32_t* s_pre,
                                              JSP_LDS uint32_t* s_wsum, JSP_LDS uint32_t* clk = nullptr) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    uint32_t cap[4];
    row_caps<W, R>(k, x.fr, cap);
    uint32_t v0[4], v1[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        bool ok = valid[i] & ((x.tn[i] & k.tol_inv) == 0);
#pragma unroll
        for (int w = 0; w < W; ++w) ok = ok & ((x.lab[w][i] & k.mask[w]) == k.req[w]);
        v0[i] = ok ? cap[i] : 0u;
        v1[i] = (valid[i] && x.ex[i] != -1) ? 1u : 0u;
    }
    const uint32_t a0 = v0[0], a1 = a0 + v0[1], a2 = a1 + v0[2], a3 = a2 + v0[3];
    const uint32_t b0 = v1[0], b1 = b0 + v1[1], b2 = b1 + v1[2], b3 = b2 + v1[3];
    JSP_EVAL_STAMP(clk, 3);
    const uint32_t ia = wave_incl_scan(a3, lane), ib = wave_incl_scan(b3, lane);
    const uint32_t wa = ia - a3, wb = ib - b3;
    reinterpret_cast<JSP_LDS u32x4*>(s_pre)[tid] = u32x4{wa + a0, wa + a1, wa + a2, ia};
    reinterpret_cast<JSP_LDS u32x4*>(s_pre + kChunkRows)[tid] = u32x4{wb + b0, wb + b1, wb + b2, ib};
    if (lane == 63) {
        s_wsum[wid] = ia;
        s_wsum[kTallyWaves + wid] = ib;
    }
    JSP_EVAL_STAMP(clk, 4);
    __syncthreads();
    JSP_EVAL_STAMP(clk, 6);
    if (!lf.live) return false;
    const u32x4 va = *reinterpret_cast<const JSP_LDS u32x4*>(s_wsum);
    const u32x4 vb = *reinterpret_cast<const JSP_LDS u32x4*>(s_wsum + kTallyWaves);
    const uint4 wsa = make_uint4(va[0], va[1], va[2], va[3]), wsb = make_uint4(vb[0], vb[1], vb[2], vb[3]);
    // all four prefix reads unconditional (xb = 0 when the leaf starts the
    // chunk: a valid address whose value is dropped), then selects -- no
    // divergent branches around the LDS reads
    const uint32_t ha = s_pre[lf.xh], hb = s_pre[kChunkRows + lf.xh];
    const uint32_t la = s_pre[lf.xb], lb = s_pre[kChunkRows + lf.xb];
    const uint32_t capsum = (ha + wave_off(wsa, lf.wh)) - (lf.has_lo ? la + wave_off(wsa, lf.wb) : 0u);
    const uint32_t occsum = (hb + wave_off(wsb, lf.wh)) - (lf.has_lo ? lb + wave_off(wsb, lf.wb) : 0u);
    JSP_EVAL_STAMP(clk, 7);
    return capsum >= k.pods && occsum == 0u;
}

// The XCC vote of a co-located service (ServiceArgs::spread): workgroup
// `slot` of n publishes its XCC id (tagged with the launch generation, so a
// vote left by an earlier launch is not counted) and wave 0 reads all n:
// true when every workgroup of the service runs on one XCD. Bounded: a vote
// missing after idle_ticks counts as a disagreement (the write-through
// protocol is correct on any placement).
__device__ bool service_xcc_vote(const ServiceArgs& v, uint32_t slot, uint32_t n, uint32_t* s_flag) {
    if (threadIdx.x == 0) {
        uint32_t x;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
        __hip_atomic_store(v.xcc + slot, ((v.gen & 0x0FFFFFFFu) << 4) | (x & 15u), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x < 64) {
        const uint32_t lane = threadIdx.x, tag = v.gen & 0x0FFFFFFFu;
        uint32_t lo = 15u, hi = 0u;
        bool ok = true;
        const uint64_t t0 = wall_clock64();
        // bounded by the idle limit, at most 50 ms (a parked service's is unbounded)
        const uint64_t limit = v.idle_ticks < 5000000ull ? v.idle_ticks : 5000000ull;
        for (uint32_t base = 0; base < n && ok; base += 64) {
            const uint32_t i = base + lane;
            uint32_t x = 0;
            while (true) {
                if (i < n) x = __hip_atomic_load(v.xcc + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (__all(i >= n || (x >> 4) == tag)) break;
                if (wall_clock64() - t0 > limit) {
                    ok = false;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (i < n) {
                lo = min(lo, x & 15u);
                hi = max(hi, x & 15u);
            }
        }
        lo = wave_min_u32(lo);
        hi = ~wave_min_u32(~hi);
        if (lane == 0) s_flag[0] = ok && lo == hi ? 1u : 0u;
    }
    __syncthreads();
    const bool local = s_flag[0] != 0u;
    __syncthreads();
    return local;
}

template <int W, int R>
__global__ __launch_bounds__(kTallyThreads) void place_service_kernel(TallyArgs a, ServiceArgs v) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* s_x = lds + tally_lds_words(a);  // compact_tile's words, then [16] request seq [17] J
    // co-located launch: only every spread-th workgroup stays (one XCD under
    // round-robin dealing), and the survivors vote on whether they share one
    if (v.spread > 1 && blockIdx.x % v.spread != 0) return;
    const uint32_t tile = blockIdx.x / (v.spread > 1 ? v.spread : 1u);
    const bool local = v.spread > 1 ? service_xcc_vote(v, tile, a.n_blocks + 1, s_x + 18) : false;
    if (tile == a.n_blocks) {
        service_dispatch(v, a, s_x + 16, local);
        return;
    }
    uint32_t seq = v.seq0;
    // this request's phase stamps (timing on). One word in: the array sits at
    // LDS address 0, which compares equal to a null LDS pointer
    __shared__ uint32_t s_clk[kSvcClkSlots + 1];
    JSP_LDS uint32_t* clk = v.clk ? lds_ptr(s_clk + 1) : nullptr;
    uint32_t* clk_out = v.clk ? v.clk + kSvcClkSlots * tile : nullptr;
    // the tile's constants, staged once: geometry, class record, leaf starts
    const uint4 bt = a.blk[tile];
    // the tile's rows stay in LDS between requests (v.row_cache_words != 0:
    // every tile is one chunk); a request whose bell carries the "rows
    // patched" bit (bit 63: the host patched the snapshot since its previous
    // request) reloads them
    JSP_LDS u32x4* row_cache = v.row_cache_words ? lds_ptr(reinterpret_cast<u32x4*>(lds + v.row_cache_words)) : nullptr;
    bool cached = false;
    // resident path: the tile's rows, class and leaf bounds held across requests
    const bool resident = v.resident != 0u;
    RowRegs<W, R> rows;
    bool valid[4] = {false, false, false, false};
    ResidentLeaf lf{0u, 0u, 0u, 0u, false, false};
    ClassRegs<W, R> kreg{};
    if (resident) {
        lf = resident_leaf(a, bt);
        kreg = class_regs_k<W, R>(*(const JSP_CONST DevClass*)a.cls);
        const uint32_t row = (bt.z & ~3u) + 4u * threadIdx.x;
#pragma unroll
        for (int i = 0; i < 4; ++i) valid[i] = row + i >= bt.z && row + i < bt.w;
    }
    {
        constexpr int kClsVec = (int)(sizeof(DevClass) / 16);
        const int tid = threadIdx.x;
        const uint32_t nl = bt.y - bt.x;
        const int la = (int)a.la;
        if (tid < kClsVec) reinterpret_cast<uint4*>(lds)[tid] = reinterpret_cast<const uint4*>(a.cls)[tid];
        uint32_t* s_ls = lds + tally_ls_off(1, 2, la);
        for (uint32_t i = tid; i <= nl; i += kTallyThreads) s_ls[i] = a.leaf_start[bt.x + i];
    }
    __syncthreads();
    while (true) {
        if (threadIdx.x == 0) {
            // the bell (device memory, sc1 loads: the dispatcher stores it sc1);
            // a tile also leaves on its own after twice the idle time, in case
            // the dispatcher never ran
            uint32_t next = 0, J = 0;  // next == 0: leave
            const uint64_t t0 = wall_clock64();
            while (true) {
                const unsigned long long m = __hip_atomic_load(v.bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t q = (uint32_t)m;
                // a stop carries its service's generation: one left by an
                // earlier service in this (unzeroed) bell is not for us
                if (q == kSvcStop && (uint32_t)(m >> 32) == v.gen) break;
                if (q != seq && q != 0 && q != kSvcStop) {
                    next = q;
                    J = (uint32_t)(m >> 32);  // bit 31: rows patched since the previous request
                    break;
                }
                if (wall_clock64() - t0 > 2 * v.idle_ticks) break;
                __builtin_amdgcn_s_sleep(1);
            }
            if (next != 0) svc_stamp(clk, 0);
            s_x[16] = next;
            s_x[17] = J;
            s_x[19] = 0u;  // a wave whose microbox wait gave up sets it
        }
        __syncthreads();
        const uint32_t next = s_x[16], Jw = s_x[17];
        if (next == 0) return;
        const uint32_t J = Jw & ~(kReqDirty | kBellMicro);
        const bool use_cache = cached && (Jw >> 31) == 0u;
        svc_stamp(clk, 1);
        const uint32_t epoch = next & 0x3FFFFFFFu;
        if (resident) {
            if (!use_cache) {  // first request, or rows patched since the last one: from memory (sc1, no stale L1)
                const uint32_t row = (bt.z & ~3u) + 4u * threadIdx.x;
                load_rows<W, R, true>(a, row, row < bt.w && row + 3 >= bt.z, rows);
                // waited for here, on this path only: otherwise the waits the
                // compiler places at the rows' first use, in code both paths
                // share, would make the cached path wait for the previous
                // request's host stores too (vmcnt counts them)
                __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);
            }
            // this request's micro-patch rows, from the microbox (their stores
            // to memory may land after this tile's loads)
            if (Jw & kBellMicro)
                if (!apply_microbox<W, R>(v.mbox, next, (bt.z & ~3u) + 4u * threadIdx.x, rows, v.micro_spins) &&
                    (threadIdx.x & 63u) == 0u)
                    s_x[19] = 1u;
            const bool ok = resident_eval<W, R>(kreg, rows, valid, lf, lds_ptr(lds + tally_pre_off(1, 2, (int)a.la)),
                                                lds_ptr(lds + tally_wsum_off(1, 2, (int)a.la)), clk);
            svc_stamp(clk, 2);
            // (resident_eval's barrier orders the flag's LDS stores before this read)
            const bool mb_fail = s_x[19] != 0u;
            if (mb_fail) {
                // a microbox wait gave up: this tile's registers may lack the
                // request's patched rows. No answer line (the host never takes
                // the request as answered) and the error word instead, which
                // the host's waits poll; the rows come from memory next time
                // (the dispatcher wrote them through before its completion word)
                if (threadIdx.x == 0)
                    __hip_atomic_store(v.err, kErrMicro | (next & ~kErrKindMask), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
                if (!v.bits)
                    compact_finish(a, tile, bt.x, ok, epoch == 0 ? 1u : epoch, J, 1u, v.granules, v.spin_limit,
                                   v.assign, v.stats, v.err, true, s_x, clk, next, local);
            } else if (v.bits) {
                bitmap_finish(tile, ok, next, v.bits, s_x + 4);
            } else {
                compact_finish(a, tile, bt.x, ok, epoch == 0 ? 1u : epoch, J, 1u, v.granules, v.spin_limit, v.assign,
                               v.stats, v.err, true, s_x, clk, next, local);
            }
            cached = !mb_fail;
        } else {
            compact_tile<W, R, true>(a, tile, bt, epoch == 0 ? 1u : epoch, v.pods, J, 1u, v.granules, v.spin_limit,
                                     v.assign, v.stats, v.err, true, lds, s_x, clk, row_cache, use_cache, next, local,
                                     v.bits);
            cached = row_cache != nullptr;
        }
        if (v.bits && !clk_out) {
            // bitmap answer: no done word. It would only say that this tile is
            // past its row reads, and the tile's answer line (every half
            // tagged with the request) says as much: the host's settle reads
            // the lines (svc_wait) -- one host write per tile and request, not two
        } else {
            signal_host_clk(v.done + tile, next, clk, clk_out);
        }
        // The host may patch the snapshot before its next request (another
        // launch): drop this CU's L1 lines now, off the request path -- no
        // snapshot load happens until the next request, which the host posts
        // after the patch has finished. The invalidate alone: an acquire fence
        // would first wait for this tile's posted host stores (vmcnt(0)).
        if (threadIdx.x == 0) asm volatile("buffer_inv sc1" ::: "memory");
        seq = next;
        __syncthreads();  // s_x[16..17] and the tally carve are rewritten by the next request
    }
}

// The split service (jsp_internal.h SplitArgs): the fused shape's tiles kept
// resident, each answering a request with its feasibility ballots / partial
// domain sums in pinned host memory and a done word; the host walks. One
// workgroup per (row block, class group) tile + the dispatcher.
// The tile's sums are in LDS after tally_block (cap_out == nullptr); for an
// upper class the clamped per-leaf values min(cap, pods) are block-scanned
// (exact: capsum >= pods iff the clamped sum is, and the clamped partial sums
// of <= 256 leaves stay below 2^30) and every leaf that ends its level-k
// domain inside the tile emits that domain's partial sum.
__device__ __forceinline__ uint32_t leaf_ancestor(uint32_t leaf, uint32_t level, const TopoDev& topo) {
    uint32_t d = leaf;
    for (uint32_t k = topo.K - 1; k > level; --k) d = (uint32_t)topo.par[k][d];
    return d;
}

// The device paths' assign[] copy, launched before the host walks (so no
// launch sits between the walk and the copy): each workgroup waits (bounded)
// for the host's release of `tag` in the host-mapped word `flag`, then copies
// n words from the host-mapped staging into the device buffer. The host
// writes tag | 0x80000000 when it cannot deliver (the call fails): nothing is
// copied. A wait that times out writes err_tag to err (the engine reports it).
__device__ __forceinline__ void copy_after_release(const uint32_t* flag, uint32_t tag, const uint32_t* __restrict__ src,
                                                   uint32_t* __restrict__ dst, uint32_t n, uint32_t* err,
                                                   uint32_t err_tag, unsigned long long ticks, uint32_t wg,
                                                   uint32_t n_wg) {
    __shared__ uint32_t s_go;
    if (threadIdx.x == 0) {
        const uint64_t t0 = wall_clock64();
        uint32_t f = 0;
        while (true) {
            f = __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
            if ((f & 0x7FFFFFFFu) == tag) break;
            if (wall_clock64() - t0 > ticks) {
                if (err != nullptr) __hip_atomic_store(err, err_tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                f = 0x80000000u;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        s_go = (f & 0x80000000u) ? 0u : 1u;
    }
    __syncthreads();
    if (s_go == 0u) return;
    for (uint32_t i = wg * blockDim.x + threadIdx.x; i < n; i += n_wg * blockDim.x)
        dst[i] = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void copy_wait_kernel(const uint32_t* flag, uint32_t tag,
                                                        const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                                        uint32_t n, uint32_t* err, uint32_t err_tag,
                                                        unsigned long long ticks) {
    copy_after_release(flag, tag, src, dst, n, err, err_tag, ticks, blockIdx.x, gridDim.x);
}

// anc: per (upper level k, leaf thread) one LDS word d | first << 20 |
// last << 28 -- the leaf's level-k domain, the block-local index of that
// domain's first leaf, whether the leaf ends it. The first upper class of a
// level walks the hierarchy tables (dependent global loads) and leaves the
// words there; the level's other classes, and a resident tile's later
// requests (anc_ready: topology only, an upload restarts the service), read
// them. On gfx9 vmcnt counts stores, so each of those global loads also
// waited for the previous class's system-scope record stores (a link round
// trip): cfg5's resident request 4.99 -> 3.89 us on the device.
// d < 2^20 as in the records; first < 256 (a split tile's leaves fit its
// four waves).
// The tile's answer line words start at zero (split_emit writes only the
// ballots and counts it has); zeroed before the tally, whose barriers order
// it before split_emit's writes (no barrier of its own).
__device__ __forceinline__ void split_zero_line(const SplitArgs& sp, uint32_t* s_x) {
    JSP_LDS uint32_t* s_line = lds_ptr(s_x + 16 + kTallyThreads);
    if ((uint32_t)threadIdx.x < split_line_words(sp.cpg, sp.nw)) s_line[threadIdx.x] = 0u;
}

__device__ __forceinline__ void split_emit(const TallyArgs& ag, const SplitArgs& sp, uint4 bt, uint64_t* out,
                                           uint32_t seq, uint32_t* lds, uint32_t* s_x,
                                           JSP_LDS uint32_t* anc = nullptr, bool anc_ready = false) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int nc = (int)ag.nc;
    JSP_LDS const DevClass* cls_l = lds_ptr(reinterpret_cast<const DevClass*>(lds));
    JSP_LDS const uint32_t* s_acc = lds_ptr(lds + tally_acc_off(nc));
    JSP_LDS uint32_t* s_pre = lds_ptr(s_x + 16);
    // the tile's lines, gathered here and written by one pass of stores
    JSP_LDS uint32_t* s_line = lds_ptr(s_x + 16 + kTallyThreads);
    const uint32_t nw = sp.nw, n_line = split_line_words(sp.cpg, nw);
    const uint32_t la = ag.la;
    const uint32_t l0 = bt.x, nl = bt.y - bt.x;
    const bool in = (uint32_t)tid < nl;
    // s_line was zeroed before the tally (split_zero_line), whose barriers order it
    const uint32_t K = sp.topo.K;
    uint32_t anc_lv = anc_ready ? 0xFu : 0u;  // bit k: level k's words are in anc
    const unsigned long long rtag = (unsigned long long)split_rec_tag(seq) << 50;
    for (int c = 0; c < nc; ++c) {
        const uint32_t level = to_sgpr(cls_l[c].level), pods = to_sgpr(cls_l[c].pods);
        const uint32_t cap_r = s_acc[c * la + tid];  // in the tally carve for every tid: read with the class words
        const uint32_t cap = in ? cap_r : 0u;
        if (level + 1 == K) {
            const uint64_t word = __ballot(in && cap >= pods);
            if (lane < 2 && (uint32_t)wid < nw)
                s_line[2 * (c * nw + wid) + lane] = lane == 0 ? (uint32_t)word : (uint32_t)(word >> 32);
        } else {
            const uint32_t v = cap < pods ? cap : pods;
            uint32_t total;
            const uint32_t incl = block_excl_scan<kTallyThreads>(v, s_x + 4, &total) + v;
            s_pre[tid] = incl;
            __syncthreads();
            bool last = false;
            unsigned long long rec = 0;
            if (in) {
                uint32_t d, first;
                if (anc != nullptr && ((anc_lv >> level) & 1u)) {
                    const uint32_t w = anc[level * kTallyThreads + tid];
                    d = w & 0xFFFFFu;
                    first = (w >> 20) & 0xFFu;
                    last = (w >> 28) != 0u;
                } else {
                    const uint32_t l = l0 + (uint32_t)tid;
                    d = leaf_ancestor(l, level, sp.topo);
                    const uint32_t beg = sp.topo.fl[level][d], end = sp.topo.fl[level][d + 1];
                    last = (uint32_t)tid + 1 == nl || l + 1 == end;
                    first = (beg > l0 ? beg : l0) - l0;
                    if (anc != nullptr) anc[level * kTallyThreads + tid] = d | (first << 20) | ((last ? 1u : 0u) << 28);
                }
                const uint32_t partial = incl - (first > 0 ? s_pre[first - 1] : 0u);
                rec = rtag | ((unsigned long long)d << 30) | partial;
            }
            if (anc != nullptr) anc_lv |= 1u << level;  // each thread reads back only its own words
            const uint64_t m = __ballot(last);
            uint64_t* recs = out + n_line + ((size_t)c * nw + wid) * kSplitRecs;
            if (last) __hip_atomic_store(recs + mbcnt64(m), rec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (lane == 0 && (uint32_t)wid < nw) s_line[2 * (c * nw + wid)] = (uint32_t)__popcll(m);
            __syncthreads();  // s_pre and the scan scratch are rewritten by the next upper class
        }
    }
    if (ag.do_occ) {
        const uint32_t o_r = s_acc[nc * la + tid];
        const uint32_t o = in ? o_r : 0u;
        const uint64_t word = __ballot(in && o != 0u);
        if (lane < 2 && (uint32_t)wid < nw)
            s_line[2 * (sp.cpg * nw + wid) + lane] = lane == 0 ? (uint32_t)word : (uint32_t)(word >> 32);
    }
    __syncthreads();
    if ((uint32_t)tid < n_line)
        __hip_atomic_store(out + tid, ((unsigned long long)seq << 32) | s_line[tid], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int W, int R>
__global__ __launch_bounds__(kTallyThreads) void place_split_service_kernel(TallyArgs a, SplitArgs sp, ServiceArgs v) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t tile = blockIdx.x;
    const uint32_t n_tiles = a.n_blocks * sp.groups;
    uint32_t* s_x = lds + tally_lds_words((int)sp.cpg, (int)sp.cpg + 1, (int)a.la);  // [0] seq [4..16) scan [16..) prefixes
    if (v.oneshot != 0u && tile == n_tiles) {
        // the one-request launch's assign[] copy: waits for the host walk's
        // release, then copies (split_oneshot; no launch after the walk)
        copy_after_release(sp.cw_flag, sp.cw_tag, sp.cw_src, sp.cw_dst, sp.cw_n, sp.cw_err, sp.cw_err_tag, sp.cw_ticks, 0u,
                           1u);
        return;
    }
    if (tile == n_tiles) {
        service_dispatch(v, a, s_x);
        return;
    }
    const FusedTile ft = fused_tile(tile, sp.groups, sp.cpg, sp.C);
    TallyArgs ag = a;
    ag.c0 = ft.c0;
    ag.nc = ft.nc;
    ag.do_occ = ft.do_occ;
    ag.cap_out = nullptr;  // the sums stay in LDS
    const uint4 bt = a.blk[ft.blk];
    uint64_t* out = sp.out + (size_t)tile * split_tile_words(sp.cpg, sp.nw);
    if (v.oneshot != 0u) {
        // one launch, one request (the launch path and the device paths of the
        // split shape, ABI v7): no dispatcher, no bell, rows from memory; the
        // tile answers request v.oneshot through its tagged lines and leaves
        if (tile == 0 && sp.run_dst != nullptr) {
            for (uint32_t i = threadIdx.x; i < sp.n_runs; i += kTallyThreads) {
                sp.run_dst[i] = sp.run_class[i];
                sp.run_dst[sp.n_runs + i] = sp.run_len[i];
            }
            __threadfence_system();  // before this tile's lines, which the host waits for
        }
        split_zero_line(sp, s_x);
        tally_block<W, R, false, true>(ag, ft.blk, lds, make_uint4(0, 0, 0, 0), nullptr, nullptr, false);
        split_emit(ag, sp, bt, out, v.oneshot, lds, s_x, v.anc_words ? lds_ptr(lds + v.anc_words) : nullptr, false);
        return;
    }
    uint32_t seq = v.seq0;
    // the tile's rows stay in LDS between requests (as the compaction
    // service's; bit 63 of the bell: the snapshot was patched since the
    // previous request)
    JSP_LDS u32x4* row_cache = v.row_cache_words ? lds_ptr(reinterpret_cast<u32x4*>(lds + v.row_cache_words)) : nullptr;
    bool cached = false;
    // the first request stages the class records, leaf starts and ancestor
    // words in LDS; the later ones reuse them (tally_block staged_rt, split_emit anc)
    bool staged = false;
    JSP_LDS uint32_t* anc = v.anc_words ? lds_ptr(lds + v.anc_words) : nullptr;
    // this request's phase stamps (timing on). One word in: the array sits at
    // LDS address 0, which compares equal to a null LDS pointer
    __shared__ uint32_t s_clk[kSvcClkSlots + 1];
    JSP_LDS uint32_t* clk = v.clk ? lds_ptr(s_clk + 1) : nullptr;
    uint32_t* clk_out = v.clk ? v.clk + kSvcClkSlots * tile : nullptr;
    while (true) {
        // the bell is polled from the last wave: wave 0 issues the tile's
        // host stores (its lines, the done word; the last wave holds leaves
        // only in tiles of more than 192), and a poll from it would first
        // wait for them to retire, a link round trip (vmcnt counts stores)
        if (threadIdx.x == kTallyThreads - 64) {
            uint32_t next = 0, dirty = 0, jobs = 0;  // next 0: leave
            const uint64_t t0 = wall_clock64();
            while (true) {
                const unsigned long long m = __hip_atomic_load(v.bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t q = (uint32_t)m;
                // a stop carries its service's generation: one left by an
                // earlier service in this (unzeroed) bell is not for us
                if (q == kSvcStop && (uint32_t)(m >> 32) == v.gen) break;
                if (q != seq && q != 0 && q != kSvcStop) {
                    next = q;
                    dirty = (uint32_t)(m >> 63);
                    jobs = (uint32_t)(m >> 32) & ~(kReqDirty | kBellMicro);
                    break;
                }
                if (wall_clock64() - t0 > 2 * v.idle_ticks) break;
                __builtin_amdgcn_s_sleep(1);
            }
            if (next != 0 && clk) clk[0] = (uint32_t)wall_clock64();  // svc_stamp's slot 0, from this thread
            s_x[0] = next;
            s_x[1] = dirty;
            s_x[2] = jobs;
        }
        __syncthreads();
        const uint32_t next = s_x[0];
        if (next == 0) return;
        const bool use_cache = cached && s_x[1] == 0u;
        const bool job_less = s_x[2] == 0u;  // a request without jobs: this tile writes its done word
        svc_stamp(clk, 1);
        split_zero_line(sp, s_x);
        tally_block<W, R, false, true>(ag, ft.blk, lds, bt, clk, row_cache, use_cache, staged);
        cached = row_cache != nullptr;
#if !defined(JSP_AB_FINESTAMP) && !defined(JSP_AB_ENTRYSTAMP)
    svc_stamp(clk, 2);
#endif
        split_emit(ag, sp, bt, out, next, lds, s_x, anc, staged);
        staged = true;
#if !defined(JSP_AB_FINESTAMP) && !defined(JSP_AB_ENTRYSTAMP)
    svc_stamp(clk, 4);
#endif
        if (!clk_out) {
            // the tagged lines are the answer, and the host waits for them
            // (svc_wait_split); a done word -- this tile is past its row reads
            // -- only for a request without jobs (the warm-up after a wake),
            // which the host settles later from the done words, contiguous
            // where the lines are not: one host write per tile and request
            if (job_less && threadIdx.x == 0)
                __hip_atomic_store(v.done + tile, next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        } else {
            signal_host_clk(v.done + tile, next, clk, clk_out);
        }
        // drop this CU's L1 lines before the next request (patches come from
        // other launches), off the request path
#ifndef JSP_AB_NOINV
        if (threadIdx.x == 0) asm volatile("buffer_inv sc1" ::: "memory");  // no wait for the done word's store
#endif
        seq = next;
        __syncthreads();  // s_x and the tally carve are rewritten by the next request
    }
}

// ----------------------------------------------------------------- A5 / A9 batch kernels
__device__ __forceinline__ uint32_t upper_bound_u32(const uint32_t* a, uint32_t n, uint32_t x) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] <= x) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// domain id at `level` of local row `row` (-1 when row < 0 or out of range)
__device__ __forceinline__ int32_t row_domain(int32_t row, uint32_t level, uint32_t n_rows,
                                              const uint32_t* leaf_start, uint32_t n_leaves,
                                              uint32_t leaf_base, const TopoDev& topo) {
    if (row < 0 || (uint32_t)row >= n_rows || level >= topo.K) return -1;
    const uint32_t l = upper_bound_u32(leaf_start, n_leaves + 1, (uint32_t)row) - 1 + leaf_base;
    if (level + 1 == topo.K) return (int32_t)l;
    return (int32_t)(upper_bound_u32(topo.fl[level], topo.D[level] + 1, l) - 1);
}

__global__ void resolve_kernel(const int32_t* __restrict__ rows, const uint32_t* __restrict__ levels,
                               uint32_t n, uint32_t n_rows, const uint32_t* __restrict__ leaf_start,
                               uint32_t n_leaves, uint32_t leaf_base, TopoDev topo, int32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = row_domain(rows[i], levels[i], n_rows, leaf_start, n_leaves, leaf_base, topo);
}

__global__ void audit_kernel(const int32_t* __restrict__ leader_rows, const uint32_t* __restrict__ levels,
                             const uint32_t* __restrict__ foff, const int32_t* __restrict__ fdom,
                             uint32_t n_jobs, uint32_t n_rows, const uint32_t* __restrict__ leaf_start,
                             uint32_t n_leaves, uint32_t leaf_base, TopoDev topo, uint32_t* __restrict__ bad) {
    // one wave per job: lanes stride over the job's followers
    const int lane = threadIdx.x & 63;
    const uint32_t job = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (job >= n_jobs) return;
    const int32_t ld = row_domain(leader_rows[job], levels[job], n_rows, leaf_start, n_leaves, leaf_base, topo);
    if (ld < 0) {
        if (lane == 0) bad[job] = 0xFFFFFFFFu;
        return;
    }
    uint32_t cnt = 0;
    for (uint32_t f = foff[job] + lane; f < foff[job + 1]; f += 64) cnt += (fdom[f] != ld);
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off, 64);
    if (lane == 0) bad[job] = cnt;
}

// ----------------------------------------------------------------- snapshot patch
// Overwrite n rows of the resident columns from a dense delta (watch events).
// The delta is read straight from pinned host memory (no copy launch), the
// rows are written through to memory (agent-scope `sc1` stores: the resident
// service's tiles re-read patched rows with `sc1` loads on any XCD), and the
// workgroup whose arrival completes the launch's count publishes `seq` to a
// host-mapped word once every workgroup's stores have drained
// (MI355X_MICROARCH.md hand-off table, first row: each workgroup adds after
// its own vmcnt wait, the last adder signals). The host orders its next
// service request after that word instead of synchronising the stream.
__global__ __launch_bounds__(256) void patch_kernel(PatchArgs a) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < a.n) {
        const uint32_t row = a.rows[i];
        if (a.dlab)
            for (uint32_t w = 0; w < a.W; ++w)
                __hip_atomic_store(a.labels + (size_t)w * a.npad + row, a.dlab[(size_t)w * a.n + i], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        if (a.dtaint) __hip_atomic_store(a.taints + row, a.dtaint[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a.dfree)
            for (uint32_t r = 0; r < a.R; ++r)
                __hip_atomic_store(a.freer + (size_t)r * a.npad + row, a.dfree[(size_t)r * a.n + i], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        if (a.dexcl) __hip_atomic_store(a.excl + row, a.dexcl[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (a.done == nullptr) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long old =
            __hip_atomic_fetch_add(a.counter, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old + 1 == a.target) __hip_atomic_store(a.done, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ----------------------------------------------------------------- shard tally sum
// dst += src over n words (the device-set engine's shards on one device: the
// on-device stand-in for the RCCL all-reduce between devices).
__global__ __launch_bounds__(256) void add_u32_kernel(uint32_t* __restrict__ dst, const uint32_t* __restrict__ src,
                                                      size_t n) {
    const size_t n4 = n / 4;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        uint4 a = reinterpret_cast<const uint4*>(dst)[i];
        const uint4 b = reinterpret_cast<const uint4*>(src)[i];
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
        reinterpret_cast<uint4*>(dst)[i] = a;
    }
    for (size_t i = n4 * 4 + (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] += src[i];
}

// ----------------------------------------------------------------- host-link floor (instrumentation)
// jspb_link_floor: the dispatcher's polling alone -- lane 0 of four
// waves a quarter of a round trip apart, system-scope loads of one request
// word in pinned host memory -- answering request number i with an ack word
// of its own in pinned memory, which the host spins on: the host -> device ->
// host round trip every host-API request pays at least once. Every wave gives
// up after wait_ticks without a request, so the grid always drains.
__global__ __launch_bounds__(256) void link_probe_kernel(const uint32_t* req, uint32_t* ack, uint32_t n,
                                                         uint64_t wait_ticks) {
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane != 0) return;
    const uint64_t ts = wall_clock64();
    while (wall_clock64() - ts < (uint64_t)w * kSvcStaggerTicks) __builtin_amdgcn_s_sleep(1);
    for (uint32_t i = 1; i <= n; ++i) {
        const uint64_t t0 = wall_clock64();
        uint32_t q = 0;
        while (true) {
            asm volatile("global_load_dword %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(q) : "v"(req) : "memory");
            if (q >= i) break;
            if (wall_clock64() - t0 > wait_ticks) return;
        }
        i = q;
        __hip_atomic_store(ack + 16u * w, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// An empty kernel (instrumentation): the dispatch-event time of a launch of
// a given grid that does nothing -- the packet and workgroup-dispatch
// overhead that dispatch events add to a kernel's own span.
__global__ __launch_bounds__(256) void empty_kernel() {}

// ----------------------------------------------------------------- cache scrub (instrumentation)
// Reads n16 16-byte words (a buffer larger than the Infinity Cache), so the
// next launch finds its bytes in HBM only; nothing is dirtied. The sum goes
// to sink[0] only when it equals a value it never takes (keeps the loads).
__global__ __launch_bounds__(256) void scrub_kernel(const uint4* __restrict__ p, size_t n16, uint32_t* sink) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u && sink) sink[0] = acc;
}

// ----------------------------------------------------------------- launchers
// Every launch goes through jsp_launch. While a device-path call on a caller's
// stream is being enqueued, the engine names an event (set_launch_stop): each
// launch then carries it as its stop event (hipExtLaunchKernel), so the event
// completes with the call's last kernel -- the kernel's own completion signal,
// with no marker packet behind it on the caller's stream (an hipEventRecord
// after each call cost 2-3 us of GPU time per call, profiles/r03).
// set_launch_start names a start event the NEXT launch carries (then
// cleared): with a stop event it brackets the dispatches themselves, as a
// kernel trace does (jspb_tally_device_timed).
namespace {
thread_local hipEvent_t t_stop = nullptr;
thread_local hipEvent_t t_start = nullptr;
thread_local bool t_stop_used = false;
}  // namespace
void set_launch_stop(hipEvent_t ev) {
    t_stop = ev;
    t_stop_used = false;
}
void set_launch_start(hipEvent_t ev) { t_start = ev; }
hipEvent_t take_launch_stop() {
    hipEvent_t ev = t_stop;
    t_stop = nullptr;
    return ev;
}
bool launch_stop_used() { return t_stop_used; }

template <typename F, typename... Args>
static inline void jsp_launch(F kernel, const dim3& grid, const dim3& block, uint32_t lds, hipStream_t s,
                              Args... args) {
    hipExtLaunchKernelGGL(kernel, grid, block, lds, s, t_start, t_stop, 0u, args...);
    t_start = nullptr;
    if (t_stop) t_stop_used = true;
}

template <int W, int R>
static hipError_t launch_tally_wr(const TallyArgs& a, hipStream_t s) {
    jsp_launch((tally_kernel<W, R>), dim3(a.n_blocks), dim3(kTallyThreads),
                       sizeof(uint32_t) * tally_lds_words(a), s, a);
    return hipGetLastError();
}

template <int W, int R>
static hipError_t launch_tally_wave_wr(const TallyArgs& a, const uint4* tiles, uint32_t n_tiles, uint32_t n_leaves,
                                       uint32_t grid, hipStream_t s) {
    const size_t lds = tally_wave_lds_bytes(a.nc, a.nc + 1);
    if (grid == 0) {  // one tile per wave: the grid covers every tile
        const uint32_t g1 = (n_tiles + kTallyWaves - 1) / kTallyWaves;
        switch (a.nc) {
            case 1: jsp_launch((tally_wave1_kernel<W, R, 2>), dim3(g1), dim3(kTallyThreads), lds, s, a, tiles, n_tiles, n_leaves); break;
            case 2: jsp_launch((tally_wave1_kernel<W, R, 3>), dim3(g1), dim3(kTallyThreads), lds, s, a, tiles, n_tiles, n_leaves); break;
            case 3: jsp_launch((tally_wave1_kernel<W, R, 4>), dim3(g1), dim3(kTallyThreads), lds, s, a, tiles, n_tiles, n_leaves); break;
            case 4: jsp_launch((tally_wave1_kernel<W, R, 5>), dim3(g1), dim3(kTallyThreads), lds, s, a, tiles, n_tiles, n_leaves); break;
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    // a wave holds at most 64 tile descriptors, one per lane
    if ((uint64_t)grid * kTallyWaves * 64u < n_tiles) return hipErrorInvalidValue;
    switch (a.nc) {
        case 1: jsp_launch((tally_wave_kernel<W, R, 2>), dim3(grid), dim3(kTallyThreads), lds, s, a, tiles, n_tiles, n_leaves); break;
        case 2: jsp_launch((tally_wave_kernel<W, R, 3>), dim3(grid), dim3(kTallyThreads), lds, s, a, tiles, n_tiles, n_leaves); break;
        case 3: jsp_launch((tally_wave_kernel<W, R, 4>), dim3(grid), dim3(kTallyThreads), lds, s, a, tiles, n_tiles, n_leaves); break;
        case 4: jsp_launch((tally_wave_kernel<W, R, 5>), dim3(grid), dim3(kTallyThreads), lds, s, a, tiles, n_tiles, n_leaves); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <int W, int R>
static hipError_t launch_fused_wr(const TallyArgs& a, const FusedArgs& f, hipStream_t s) {
    jsp_launch((place_fused_kernel<W, R>), dim3(a.n_blocks * f.groups + kSpareBlocks), dim3(kTallyThreads), f.lds_bytes,
                       s, a, f);
    return hipGetLastError();
}

template <int W, int R>
static hipError_t launch_compact_wr(const TallyArgs& a, const CompactArgs& f, hipStream_t s) {
    jsp_launch((place_compact_kernel<W, R>), dim3(a.n_blocks + kSpareBlocks), dim3(kTallyThreads),
                       compact_lds_bytes(a.la), s, a, f);
    return hipGetLastError();
}

#define JSP_DISPATCH_WR_OR(DEF, FN, ...)     \
    switch (a.W * 8 + a.R) {                  \
        case 9: return FN<1, 1>(__VA_ARGS__); \
        case 10: return FN<1, 2>(__VA_ARGS__); \
        case 11: return FN<1, 3>(__VA_ARGS__); \
        case 12: return FN<1, 4>(__VA_ARGS__); \
        case 17: return FN<2, 1>(__VA_ARGS__); \
        case 18: return FN<2, 2>(__VA_ARGS__); \
        case 19: return FN<2, 3>(__VA_ARGS__); \
        case 20: return FN<2, 4>(__VA_ARGS__); \
        case 25: return FN<3, 1>(__VA_ARGS__); \
        case 26: return FN<3, 2>(__VA_ARGS__); \
        case 27: return FN<3, 3>(__VA_ARGS__); \
        case 28: return FN<3, 4>(__VA_ARGS__); \
        case 33: return FN<4, 1>(__VA_ARGS__); \
        case 34: return FN<4, 2>(__VA_ARGS__); \
        case 35: return FN<4, 3>(__VA_ARGS__); \
        case 36: return FN<4, 4>(__VA_ARGS__); \
        default: return DEF;                  \
    }
#define JSP_DISPATCH_WR(FN, ...) JSP_DISPATCH_WR_OR(hipErrorInvalidValue, FN, __VA_ARGS__)

hipError_t launch_tally(const TallyArgs& a, hipStream_t s) { JSP_DISPATCH_WR(launch_tally_wr, a, s) }

size_t tally_wave_lds_bytes(uint32_t /*nc*/, uint32_t nv) {
    return sizeof(uint32_t) * (size_t)kTallyWaves * nv * kWaveTileRows;
}

hipError_t launch_tally_wave(const TallyArgs& a, const uint4* tiles, uint32_t n_tiles, uint32_t n_leaves, uint32_t grid,
                             hipStream_t s) {
    JSP_DISPATCH_WR(launch_tally_wave_wr, a, tiles, n_tiles, n_leaves, grid, s)
}

hipError_t launch_fused(const TallyArgs& a, const FusedArgs& f, hipStream_t s) {
    JSP_DISPATCH_WR(launch_fused_wr, a, f, s)
}

hipError_t launch_compact(const TallyArgs& a, const CompactArgs& f, hipStream_t s) {
    JSP_DISPATCH_WR(launch_compact_wr, a, f, s)
}

template <int W, int R>
static hipError_t launch_service_wr(const TallyArgs& a, const ServiceArgs& v, hipStream_t s) {
    jsp_launch((place_service_kernel<W, R>), dim3((a.n_blocks + 1) * (v.spread > 1 ? v.spread : 1u)), dim3(kTallyThreads),
               service_lds_bytes(a.la, a.W, a.R, v.row_cache_words != 0), s, a, v);
    return hipGetLastError();
}

hipError_t launch_service(const TallyArgs& a, const ServiceArgs& v, hipStream_t s) {
    JSP_DISPATCH_WR(launch_service_wr, a, v, s)
}

size_t split_lds_bytes(uint32_t cpg, uint32_t la) {
    // + s_x: [0..16) seq and scan scratch, [16, 16 + 256) prefixes, then the tile's line words
    return sizeof(uint32_t) * ((size_t)tally_lds_words((int)cpg, (int)cpg + 1, (int)la) + 16 + kTallyThreads +
                               8 * ((size_t)cpg + 1) + 4);
}

uint32_t split_row_cache_words(uint32_t cpg, uint32_t la) { return (uint32_t)((split_lds_bytes(cpg, la) + 15) / 16 * 4); }

// the split tiles' ancestor words (split_emit anc): (kMaxLevels - 1) x 256
// words past the row copy, or past the tally carve without one
uint32_t split_anc_words(uint32_t cpg, uint32_t la, int W, int R, bool row_cache) {
    return split_row_cache_words(cpg, la) + (row_cache ? (uint32_t)(2 * W + 2 + R) * 4u * kTallyThreads : 0u);
}

size_t split_service_lds_bytes(uint32_t cpg, uint32_t la, int W, int R, bool row_cache) {
    return sizeof(uint32_t) * ((size_t)split_anc_words(cpg, la, W, R, row_cache) + (kMaxLevels - 1) * kTallyThreads);
}

template <int W, int R>
static hipError_t launch_split_service_wr(const TallyArgs& a, const SplitArgs& sp, const ServiceArgs& v,
                                          hipStream_t s) {
    jsp_launch((place_split_service_kernel<W, R>), dim3(a.n_blocks * sp.groups + 1), dim3(kTallyThreads),
               split_service_lds_bytes(sp.cpg, a.la, a.W, a.R, v.row_cache_words != 0), s, a, sp, v);
    return hipGetLastError();
}

hipError_t launch_split_service(const TallyArgs& a, const SplitArgs& sp, const ServiceArgs& v, hipStream_t s) {
    JSP_DISPATCH_WR(launch_split_service_wr, a, sp, v, s)
}

template <int W, int R>
static hipError_t launch_split_oneshot_wr(const TallyArgs& a, const SplitArgs& sp, const ServiceArgs& v,
                                          hipStream_t s) {
    jsp_launch((place_split_service_kernel<W, R>), dim3(a.n_blocks * sp.groups + (sp.cw_flag != nullptr ? 1u : 0u)),
               dim3(kTallyThreads),
               split_service_lds_bytes(sp.cpg, a.la, a.W, a.R, false), s, a, sp, v);
    return hipGetLastError();
}

hipError_t launch_split_oneshot(const TallyArgs& a, const SplitArgs& sp, const ServiceArgs& v, hipStream_t s) {
    if (v.oneshot == 0u || v.row_cache_words != 0u) return hipErrorInvalidValue;
    JSP_DISPATCH_WR(launch_split_oneshot_wr, a, sp, v, s)
}

template <int W, int R>
static hipError_t service_occupancy_wr(const TallyArgs&, int shape, size_t lds_bytes, int* blocks) {
    const void* fn = shape == 2 ? reinterpret_cast<const void*>(&place_service_kernel<W, R>)
                                : reinterpret_cast<const void*>(&place_split_service_kernel<W, R>);
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, fn, kTallyThreads, lds_bytes);
}

hipError_t service_occupancy(const TallyArgs& a, int shape, size_t lds_bytes, int* blocks_per_cu) {
    JSP_DISPATCH_WR(service_occupancy_wr, a, shape, lds_bytes, blocks_per_cu)
}

size_t compact_lds_bytes(uint32_t la) { return sizeof(uint32_t) * (tally_lds_words(1, 2, (int)la) + 4 + 2 * kTallyWaves + 8); }

uint32_t service_row_cache_words(uint32_t la) { return (uint32_t)((compact_lds_bytes(la) + 15) / 16 * 4); }

size_t service_lds_bytes(uint32_t la, int W, int R, bool row_cache) {
    // + the dispatcher's words past the compaction's (service_dispatch s_p: 8 + kMailboxPayload after s_x[16])
    if (!row_cache) return compact_lds_bytes(la) + sizeof(uint32_t) * (8 + kMailboxPayload + 2);
    return sizeof(uint32_t) * service_row_cache_words(la) + (size_t)(2 * W + 2 + R) * 16 * kTallyThreads;
}


size_t fused_lds_bytes(uint32_t t_words, uint32_t feas_words, uint32_t nc, uint32_t nv, uint32_t la,
                       uint32_t topo_words, uint32_t fscr_words) {
    const size_t tail = (size_t)(t_words + kFusedWinWords64 + feas_words) * 8 +
                        sizeof(uint32_t) * (assign_small_words(kTallyThreads) + topo_words + kFusedStage) +
                        (fscr_words ? (size_t)fscr_words * 8 + 8 : 0);
    const size_t head = sizeof(uint32_t) * (tally_lds_words((int)nc, (int)nv, (int)la) + 4);
    return ((tail > head ? tail : head) + 15) & ~size_t(15);
}

uint32_t fused_scratch_words(uint32_t K, const uint32_t* D, const uint32_t* class_level, uint32_t C) {
    if (K < 2) return 0;
    uint64_t w = 0;
    for (uint32_t c = 0; c < C; ++c)
        if (class_level[c] + 1 < K) w += D[class_level[c]];
    if (w == 0) return 0;
    for (uint32_t k = 0; k + 1 < K; ++k) w += (D[k] + 63) / 64;
    return w <= kFusedScrMax ? (uint32_t)w : 0u;
}

AssignPlan plan_assign(uint32_t t_words, uint32_t feas_words, uint32_t topo_words) {
    AssignPlan p{};
    size_t used = (size_t)(t_words + kAssignWinWords64) * 8 + sizeof(uint32_t) * assign_small_words(kAssignThreads);
    if (used > kLdsBytes) return p;  // lds_bytes 0: does not fit
    if (topo_words > 0 && used + sizeof(uint32_t) * topo_words <= kLdsBytes) {
        p.topo_in_lds = 1;
        used += sizeof(uint32_t) * topo_words;
    }
    if (used + (size_t)feas_words * 8 + sizeof(uint32_t) * kMinStage <= kLdsBytes) {
        p.feas_in_lds = 1;
        used += (size_t)feas_words * 8;
    }
    size_t st = (kLdsBytes - used) / sizeof(uint32_t);
    if (st > kMaxStage) st = kMaxStage;
    st &= ~size_t(63);
    if (st < 64) return AssignPlan{};
    p.stage_cap = (uint32_t)st;
    p.lds_bytes = used + sizeof(uint32_t) * st;
    return p;
}

// u32 copy between device and host-mapped memory (the device path's host
// walk: runs and feasibility out, assign[] back), through jsp_launch so the
// call's stop event rides on it like on every other launch.
__global__ __launch_bounds__(256) void copy_u32_kernel(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                                       uint32_t n) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) dst[i] = src[i];
}

hipError_t launch_copy_wait(const uint32_t* flag, uint32_t tag, const uint32_t* src, uint32_t* dst, uint32_t n,
                            uint32_t* err, uint32_t err_tag, unsigned long long ticks, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint32_t blocks = (n + 255) / 256 < 64u ? (n + 255) / 256 : 64u;
    jsp_launch(copy_wait_kernel, dim3(blocks), dim3(256), 0, s, flag, tag, src, dst, n, err, err_tag, ticks);
    return hipGetLastError();
}

// one word to host-mapped memory, system scope: a completion tag behind the
// stream's earlier kernels
__global__ void tag_kernel(uint32_t* __restrict__ dst, uint32_t v) {
    if (threadIdx.x == 0) __hip_atomic_store(dst, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_tag(uint32_t* dst, uint32_t v, hipStream_t s) {
    jsp_launch(tag_kernel, dim3(1), dim3(64), 0, s, dst, v);
    return hipGetLastError();
}

hipError_t launch_copy_u32(const uint32_t* src, uint32_t* dst, uint32_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint32_t blocks = (n + 255) / 256 < 512u ? (n + 255) / 256 : 512u;
    jsp_launch(copy_u32_kernel, dim3(blocks), dim3(256), 0, s, src, dst, n);
    return hipGetLastError();
}

hipError_t launch_feas(const uint32_t* cap, const uint32_t* occ, uint32_t ld, const DevClass* cls, uint32_t C,
                       const uint32_t* word_off, uint32_t total_words, const TopoDev& topo, uint64_t* feas,
                       hipStream_t s) {
    if (total_words == 0) return hipSuccess;
    const uint32_t blocks = (total_words + 3) / 4;
    jsp_launch(feas_kernel, dim3(blocks), dim3(256), 0, s, cap, occ, ld, cls, C, word_off, topo, feas);
    return hipGetLastError();
}

hipError_t launch_assign(const uint64_t* feas, const uint32_t* word_off, const DevClass* cls, uint32_t C,
                         const TopoDev& topo, uint32_t t_words, uint32_t feas_words, const uint32_t* run_class,
                         const uint32_t* run_len, uint32_t n_runs, uint32_t J, int32_t* assign, uint32_t* stats,
                         uint32_t* rec_count, AssignRec* recs, hipStream_t s, const WaitErr& we) {
    const uint32_t topo_words = topo.K > 1 ? topo_table_words(topo.K, topo.D) : 0u;
    const AssignPlan p = plan_assign(t_words, feas_words, topo_words);
    if (p.lds_bytes == 0) return hipErrorInvalidValue;
    jsp_launch(assign_kernel, dim3(1), dim3(kAssignThreads), p.lds_bytes, s, feas, word_off, cls, C, topo,
                       run_class, run_len, n_runs, J, assign, stats, feas_words, p.feas_in_lds, p.topo_in_lds,
                       topo_words, p.stage_cap, recs, rec_count, we);
    if (hipError_t e = hipGetLastError(); e != hipSuccess || recs == nullptr || J == 0) return e;
    // Records never outnumber the placed jobs (each taken domain is in one
    // record), nor the feasibility words plus one per run (a run's records are
    // distinct words of its class; the next run of the class may share one).
    const uint64_t wb = (uint64_t)feas_words + n_runs;
    const uint32_t bound = wb < J ? (uint32_t)wb : J;
    const uint32_t rpw = kExpandRpw;
    const uint32_t waves = (bound + rpw - 1) / rpw;
    jsp_launch(expand_kernel, dim3((waves + 3) / 4), dim3(256), 0, s, recs, rec_count, bound, rpw, assign);
    return hipGetLastError();
}

// the level walker's shape for nw words: (words per thread, threads). Up to
// 256 words, 256 threads with one word each; above, 1024 threads with one or
// two words each (four waves per SIMD hide each other's latency in the
// per-run chain)
static void level_shape(uint32_t nw, uint32_t* wpt, uint32_t* nt) {
    *wpt = 0;
    *nt = 256;
    if (nw <= 256) *wpt = 1;
    else if (nw <= 1024) { *wpt = 1; *nt = 1024; }
    else if (nw <= 2048) { *wpt = 2; *nt = 1024; }
}

size_t level_walk_lds_bytes(uint32_t C, uint32_t nw) {
    uint32_t wpt, nt;
    level_shape(nw, &wpt, &nt);
    return wpt ? (size_t)C * nt * wpt * 8u : 0u;
}

hipError_t launch_assign_level(const uint64_t* feas, uint32_t C, uint32_t nw, const uint32_t* run_class,
                               const uint32_t* run_len, uint32_t n_runs, uint32_t J, int32_t* assign, uint32_t* stats,
                               uint32_t* rec_count, AssignRec* recs, hipStream_t s, unsigned long long* ready,
                               uint32_t epoch, const WaitErr& we) {
    uint32_t wpt, nt;
    level_shape(nw, &wpt, &nt);
    const size_t lds = level_walk_lds_bytes(C, nw);
    if (wpt == 0 || nw == 0 || n_runs > kLevelMaxRuns || recs == nullptr || ready == nullptr || lds > 128u * 1024u)
        return hipErrorInvalidValue;
    // records: one per (run, word) that gives domains away; a class's runs
    // take its words in order, so at most its words plus one per run
    const uint64_t wb = (uint64_t)C * nw + n_runs;
    const uint32_t bound = wb < J ? (uint32_t)wb : J;
    const uint32_t rpw = kExpandRpw;
    const uint32_t waves = (bound + rpw - 1) / rpw;
    // one launch: the walker plus the expanders behind it (none for J = 0)
    unsigned long long* rd = J > 0 ? ready : nullptr;
    const uint32_t wpb = nt / 64;  // expander waves per workgroup
    const dim3 g(rd ? 1u + (waves + wpb - 1) / wpb : 1u), b(nt);
#define JSP_LEVEL_LAUNCH(W_, N_) \
    jsp_launch((assign_level_kernel<W_, N_>), g, b, (uint32_t)lds, s, feas, C, nw, run_class, run_len, n_runs, assign, \
               stats, rec_count, recs, rd, epoch, bound, rpw, we)
    if (nt == 1024) {
        if (wpt == 1) JSP_LEVEL_LAUNCH(1, 1024);
        else JSP_LEVEL_LAUNCH(2, 1024);
    } else {
        JSP_LEVEL_LAUNCH(1, 256);
    }
#undef JSP_LEVEL_LAUNCH
    return hipGetLastError();
}

hipError_t launch_resolve(const int32_t* rows, const uint32_t* levels, uint32_t n, uint32_t n_rows,
                          const uint32_t* leaf_start, uint32_t n_leaves, uint32_t leaf_base, const TopoDev& topo,
                          int32_t* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    jsp_launch(resolve_kernel, dim3((n + 255) / 256), dim3(256), 0, s, rows, levels, n, n_rows, leaf_start,
                       n_leaves, leaf_base, topo, out);
    return hipGetLastError();
}

hipError_t launch_audit(const int32_t* leader_rows, const uint32_t* levels, const uint32_t* foff,
                        const int32_t* fdom, uint32_t n_jobs, uint32_t n_rows, const uint32_t* leaf_start,
                        uint32_t n_leaves, uint32_t leaf_base, const TopoDev& topo, uint32_t* bad, hipStream_t s) {
    if (n_jobs == 0) return hipSuccess;
    jsp_launch(audit_kernel, dim3((n_jobs + 3) / 4), dim3(256), 0, s, leader_rows, levels, foff, fdom,
                       n_jobs, n_rows, leaf_start, n_leaves, leaf_base, topo, bad);
    return hipGetLastError();
}

hipError_t launch_add_u32(uint32_t* dst, const uint32_t* src, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const size_t blocks = std::min<size_t>(1024, (n / 4 + 255) / 256 + 1);
    jsp_launch(add_u32_kernel, dim3((unsigned)blocks), dim3(256), 0, s, dst, src, n);
    return hipGetLastError();
}

hipError_t launch_link_probe(const uint32_t* req, uint32_t* ack, uint32_t n, uint64_t wait_ticks, hipStream_t s) {
    jsp_launch(link_probe_kernel, dim3(1), dim3(256), 0, s, req, ack, n, wait_ticks);
    return hipGetLastError();
}

hipError_t launch_empty(uint32_t grid, hipStream_t s) {
    jsp_launch(empty_kernel, dim3(grid), dim3(256), 0, s);
    return hipGetLastError();
}

hipError_t launch_scrub(const void* p, size_t bytes, uint32_t* sink, hipStream_t s) {
    if (bytes < 16) return hipSuccess;
    jsp_launch(scrub_kernel, dim3(4096), dim3(256), 0, s, static_cast<const uint4*>(p), bytes / 16, sink);
    return hipGetLastError();
}

hipError_t launch_patch(const PatchArgs& a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    jsp_launch(patch_kernel, dim3((a.n + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace jsp

#ifdef JSP_STAMPS
extern "C" int jsp_debug_stamps(unsigned long long* out, unsigned n) {
    if (n > 4096 * 8) n = 4096 * 8;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(jsp::jsp_dbg), n * sizeof(unsigned long long)) == hipSuccess ? 0 : -2;
}
extern "C" int jsp_debug_clear() {
    static unsigned long long zero[4096 * 8];
    return hipMemcpyToSymbol(HIP_SYMBOL(jsp::jsp_dbg), zero, sizeof zero) == hipSuccess ? 0 : -2;
}
#endif
