// jsp_kernels.hip — gfx950 kernels of the exclusive-topology placement engine.
//
// Three kernels make one placement (SURVEY.md §8a rows A8 then A7):
//   tally_kernel   HBM-streaming predicate + per-(class, leaf) capacity tally.
//                  One workgroup owns a contiguous run of whole leaves, so every
//                  leaf sum is finished inside one workgroup: no global atomics,
//                  no memset, bit-exact integer sums written exactly once.
//   feas_kernel    per-(class, domain) feasibility bitmap at the class's level
//                  (wave64 ballot -> one 64-bit word per wave).
//   assign_kernel  single-workgroup lowest-index 1:1 assignment over same-class
//                  job runs: block-wide popcount prefix over bitmap words gives
//                  the k-th available domain to the k-th job of the run.
// Plus two small gather kernels for the webhook / reconciler batch paths
// (A5 follower pinning, A9 placement audit).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jsp_internal.h"

namespace jsp {

// ----------------------------------------------------------------- helpers
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    return x;
}

// floor(free / req) clamped to `pods`, exact for every uint32 input: the
// float quotient is only an estimate, corrected by one step either way.
__device__ __forceinline__ uint32_t fit_count(uint32_t free, uint32_t req, float rcp, uint32_t pods) {
    if ((uint64_t)req * pods <= (uint64_t)free) return pods;
    uint32_t q = (uint32_t)((float)free * rcp);
    if ((uint64_t)q * req > (uint64_t)free) q -= 1;
    else if ((uint64_t)(q + 1) * req <= (uint64_t)free) q += 1;
    return q < pods ? q : pods;
}

// ----------------------------------------------------------------- A8 tally
// Rows of the workgroup: [leaf_start[l0], leaf_start[l1]) for leaves
// [blk_leaf[b], blk_leaf[b+1]). Each thread holds 4 consecutive rows (16-B
// column loads; a wave streams 1 KiB per column instruction). Per class the
// workgroup computes an inclusive prefix over its rows; a leaf's sum is
// prefix(last row) - prefix(before first row), folded into acc[c][leaf] with
// two LDS atomics placed at the leaf's first and last rows.
template <int W, int R>
__global__ __launch_bounds__(kTallyThreads) void tally_kernel(
    const uint64_t* __restrict__ labels, const uint32_t* __restrict__ taints,
    const uint32_t* __restrict__ freer, const int32_t* __restrict__ excl, uint32_t npad,
    const uint32_t* __restrict__ leaf_start, const uint32_t* __restrict__ blk_leaf,
    const DevClass* __restrict__ cls, uint32_t c0, uint32_t nc, int do_occ,
    uint32_t* __restrict__ cap_out, uint32_t* __restrict__ occ_out, uint32_t ld, uint32_t leaf_base) {
    __shared__ int16_t s_start[kChunkRows];
    __shared__ int16_t s_end[kChunkRows];
    __shared__ uint32_t s_acc[(kTallyClasses + 1) * kMaxBlkLeaves];
    __shared__ uint32_t s_wsum[(kTallyClasses + 1) * kTallyWaves];
    __shared__ uint32_t s_carry[kTallyClasses + 1];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t l0 = blk_leaf[blockIdx.x], l1 = blk_leaf[blockIdx.x + 1];
    const uint32_t nl = l1 - l0;
    const uint32_t r0 = leaf_start[l0], r1 = leaf_start[l1];
    const int nv = (int)nc + do_occ;

    for (int i = tid; i < nv * kMaxBlkLeaves; i += kTallyThreads) s_acc[i] = 0;
    if (tid < nv) s_carry[tid] = 0;

    for (uint32_t base = r0 & ~3u; base < r1; base += kChunkRows) {
        for (int i = tid; i < kChunkRows; i += kTallyThreads) { s_start[i] = -1; s_end[i] = -1; }
        __syncthreads();
        for (uint32_t li = tid; li < nl; li += kTallyThreads) {
            uint32_t s = leaf_start[l0 + li], e = leaf_start[l0 + li + 1];
            if (s < e) {
                if (s >= base && s < base + kChunkRows) s_start[s - base] = (int16_t)li;
                if (e - 1 >= base && e - 1 < base + kChunkRows) s_end[e - 1 - base] = (int16_t)li;
            }
        }
        __syncthreads();

        const uint32_t row = base + 4u * tid;
        const bool any = (row < r1) && (row + 3 >= r0) && (row < npad);
        uint64_t lab[W][4];
        uint32_t tn[4], fr[R][4];
        int32_t ex[4];
        bool valid[4];
        int16_t ms[4], me[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            valid[i] = any && (row + i >= r0) && (row + i < r1);
            ms[i] = -1;
            me[i] = -1;
        }
        if (any) {
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const ulonglong2* p = reinterpret_cast<const ulonglong2*>(labels + (size_t)w * npad + row);
                ulonglong2 a = p[0], b = p[1];
                lab[w][0] = a.x; lab[w][1] = a.y; lab[w][2] = b.x; lab[w][3] = b.y;
            }
            uint4 t4 = *reinterpret_cast<const uint4*>(taints + row);
            tn[0] = t4.x; tn[1] = t4.y; tn[2] = t4.z; tn[3] = t4.w;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                uint4 f4 = *reinterpret_cast<const uint4*>(freer + (size_t)r * npad + row);
                fr[r][0] = f4.x; fr[r][1] = f4.y; fr[r][2] = f4.z; fr[r][3] = f4.w;
            }
            int4 e4 = *reinterpret_cast<const int4*>(excl + row);
            ex[0] = e4.x; ex[1] = e4.y; ex[2] = e4.z; ex[3] = e4.w;
            const uint32_t o = 4u * tid;
#pragma unroll
            for (int i = 0; i < 4; ++i) { ms[i] = s_start[o + i]; me[i] = s_end[o + i]; }
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
#pragma unroll
                for (int w = 0; w < W; ++w) lab[w][i] = 0;
#pragma unroll
                for (int r = 0; r < R; ++r) fr[r][i] = 0;
                tn[i] = 0;
                ex[i] = -1;
            }
        }
        bool has_bnd = false;
#pragma unroll
        for (int i = 0; i < 4; ++i) has_bnd = has_bnd || ms[i] >= 0 || me[i] >= 0;

        // pass 1: per-value wave scans; boundary rows fold their in-wave prefix
        for (int c = 0; c < nv; ++c) {
            uint32_t v[4];
            if (c < (int)nc) {
                const DevClass& k = cls[c0 + c];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    bool ok = valid[i];
#pragma unroll
                    for (int w = 0; w < W; ++w)
                        ok = ok && ((lab[w][i] & k.req[w]) == k.req[w]) && ((lab[w][i] & k.forbid[w]) == 0);
                    ok = ok && ((tn[i] & ~k.tol) == 0);
                    uint32_t cap = k.pods;
#pragma unroll
                    for (int r = 0; r < R; ++r)
                        if (k.res[r] != 0) {
                            uint32_t q = fit_count(fr[r][i], k.res[r], k.rcp[r], k.pods);
                            cap = q < cap ? q : cap;
                        }
                    v[i] = ok ? cap : 0u;
                }
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = (valid[i] && ex[i] != -1) ? 1u : 0u;
            }
            const uint32_t p0 = v[0], p1 = p0 + v[1], p2 = p1 + v[2], p3 = p2 + v[3];
            const uint32_t incl = wave_incl_scan(p3, lane);
            const uint32_t wex = incl - p3;  // exclusive prefix of this lane inside the wave
            if (lane == 63) s_wsum[c * kTallyWaves + wid] = incl;
            if (has_bnd) {
                const uint32_t pex[4] = {0u, p0, p1, p2};
                const uint32_t pin[4] = {p0, p1, p2, p3};
                uint32_t* acc = s_acc + c * kMaxBlkLeaves;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    if (ms[i] >= 0) atomicSub(&acc[ms[i]], wex + pex[i]);
                    if (me[i] >= 0) atomicAdd(&acc[me[i]], wex + pin[i]);
                }
            }
        }
        __syncthreads();
        // pass 2: add the workgroup-level offset (earlier waves + earlier chunks)
        if (has_bnd) {
            for (int c = 0; c < nv; ++c) {
                uint32_t off = s_carry[c];
                for (int w = 0; w < wid; ++w) off += s_wsum[c * kTallyWaves + w];
                uint32_t* acc = s_acc + c * kMaxBlkLeaves;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    if (ms[i] >= 0) atomicSub(&acc[ms[i]], off);
                    if (me[i] >= 0) atomicAdd(&acc[me[i]], off);
                }
            }
        }
        __syncthreads();
        if (tid < nv) {
            uint32_t t = s_carry[tid];
            for (int w = 0; w < kTallyWaves; ++w) t += s_wsum[tid * kTallyWaves + w];
            s_carry[tid] = t;
        }
        // the next chunk's first barrier orders this update before any read
    }
    __syncthreads();
    for (uint32_t li = tid; li < nl; li += kTallyThreads) {
        const uint32_t leaf = leaf_base + l0 + li;
        for (int c = 0; c < (int)nc; ++c) cap_out[(size_t)(c0 + c) * ld + leaf] = s_acc[c * kMaxBlkLeaves + li];
        if (do_occ) occ_out[leaf] = s_acc[nc * kMaxBlkLeaves + li];
    }
}

// ----------------------------------------------------------------- feasibility bitmap
// One wave per 64-domain word of one class. Bit d of class c's bitmap:
// capsum(c, d) >= pods[c] && occsum(d) == 0 over the leaves of d at level[c].
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
    const uint32_t w = gw - word_off[c];
    const uint32_t k = cls[c].level;
    const uint32_t d = w * 64 + lane;
    bool ok = false;
    if (d < topo.D[k]) {
        uint32_t a = d, b = d + 1;
        if (k + 1 < topo.K) { a = topo.fl[k][d]; b = topo.fl[k][d + 1]; }
        uint64_t cs = 0, os = 0;
        const uint32_t* cp = cap + (size_t)c * ld;
        for (uint32_t leaf = a; leaf < b; ++leaf) { cs += cp[leaf]; os += occ[leaf]; }
        ok = (cs >= cls[c].pods) && (os == 0);
    }
    const uint64_t word = __ballot(ok);
    if (lane == 0) feas[gw] = word;
}

// ----------------------------------------------------------------- A7 assignment
// Single workgroup of kAssignThreads. Jobs are walked in global order as runs
// of equal class; within a run the jobs take the first `len` available
// domains (feasible for the class, not yet taken) at or after the class's
// cursor, found with a block-wide prefix sum of word popcounts. Taking a
// domain marks it, its ancestors and its descendants taken (LDS bitmaps).
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

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t* s_w, uint32_t* total, int tid) {
    const int lane = tid & 63, wid = tid >> 6;
    const uint32_t incl = wave_incl_scan(x, lane);
    if (lane == 63) s_w[wid] = incl;
    __syncthreads();
    if (wid == 0) {
        uint32_t v = lane < kAssignWaves ? s_w[lane] : 0u;
        uint32_t s = wave_incl_scan(v, lane);
        if (lane < kAssignWaves) s_w[kAssignWaves + lane] = s - v;  // exclusive
        if (lane == kAssignWaves - 1) s_w[2 * kAssignWaves] = s;
    }
    __syncthreads();
    *total = s_w[2 * kAssignWaves];
    return s_w[kAssignWaves + wid] + incl - x;
}

__global__ __launch_bounds__(kAssignThreads) void assign_kernel(
    const uint64_t* __restrict__ feas, const uint32_t* __restrict__ word_off,
    const DevClass* __restrict__ cls, uint32_t C, TopoDev topo, const uint32_t* __restrict__ t_off,
    const uint32_t* __restrict__ job_class, uint32_t J, int32_t* __restrict__ assign,
    uint32_t* __restrict__ stats) {
    extern __shared__ __attribute__((aligned(16))) uint64_t s_taken[];  // all levels, t_off[k] words each
    __shared__ uint32_t s_cursor[kMaxClasses];
    __shared__ uint32_t s_w[2 * kAssignWaves + 4];
    __shared__ uint32_t s_runend, s_newcur;

    const int tid = threadIdx.x;
    for (uint32_t i = tid; i < t_off[topo.K]; i += kAssignThreads) s_taken[i] = 0;
    for (uint32_t i = tid; i < C; i += kAssignThreads) s_cursor[i] = 0;
    __syncthreads();

    uint32_t runs = 0, placed = 0;
    uint32_t j0 = 0;
    while (j0 < J) {
        const uint32_t c = job_class[j0];
        // ---- end of the same-class run starting at j0
        if (tid == 0) s_runend = J;
        __syncthreads();
        for (uint32_t base = j0 + 1; base < J; base += kAssignThreads) {
            const uint32_t j = base + tid;
            if (j < J && job_class[j] != c) atomicMin(&s_runend, j);
            __syncthreads();
            if (s_runend != J) break;
        }
        const uint32_t runend = s_runend;
        ++runs;
        const uint32_t k = cls[c].level;
        const uint32_t D = topo.D[k];
        const uint32_t nw = (D + 63) >> 6;
        uint64_t* Tk = s_taken + t_off[k];
        const uint64_t* F = feas + word_off[c];
        uint32_t need = runend - j0;
        uint32_t jpos = j0;
        uint32_t cur = s_cursor[c];
        while (need > 0 && cur < D) {
            const uint32_t w = (cur >> 6) + tid;
            uint64_t bits = 0;
            if (w < nw) {
                bits = F[w] & ~Tk[w];
                if (w == (cur >> 6)) bits &= ~0ull << (cur & 63);
            }
            uint32_t total;
            const uint32_t pre = block_excl_scan((uint32_t)__popcll(bits), s_w, &total, tid);
            if (tid == 0) s_newcur = ((cur >> 6) + kAssignThreads) * 64u;
            __syncthreads();
            if (bits && pre < need) {
                uint32_t r = pre;
                uint64_t took = 0;
                while (bits && r < need) {
                    const uint32_t b = __builtin_ctzll(bits);
                    bits &= bits - 1;
                    const uint32_t d = w * 64 + b;
                    assign[jpos + r] = (int32_t)d;
                    took |= 1ull << b;
                    // ancestors
                    uint32_t dd = d;
                    for (int kk = (int)k - 1; kk >= 0; --kk) {
                        dd = (uint32_t)topo.par[kk + 1][dd];
                        lds_set_bit(s_taken + t_off[kk], dd);
                    }
                    // descendants
                    uint32_t lo = d, hi = d + 1;
                    for (uint32_t kk = k + 1; kk < topo.K; ++kk) {
                        lo = topo.cs[kk - 1][lo];
                        hi = topo.cs[kk - 1][hi];
                        lds_set_range(s_taken + t_off[kk], lo, hi);
                    }
                    ++r;
                    if (r == need) s_newcur = d + 1;
                }
                atomicOr(reinterpret_cast<unsigned long long*>(&Tk[w]), (unsigned long long)took);
            }
            __syncthreads();
            const uint32_t used = total < need ? total : need;
            need -= used;
            jpos += used;
            placed += used;
            cur = s_newcur < D ? s_newcur : D;
            __syncthreads();
        }
        for (uint32_t j = jpos + tid; j < runend; j += kAssignThreads) assign[j] = -1;
        if (tid == 0) s_cursor[c] = cur;
        __syncthreads();
        j0 = runend;
    }
    if (tid == 0 && stats != nullptr) { stats[0] = runs; stats[1] = placed; }
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
    // leaf: last l with leaf_start[l] <= row (leaf_start has n_leaves+1 entries)
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
__global__ void patch_kernel(const uint32_t* __restrict__ rows, uint32_t n, uint32_t npad, uint32_t W, uint32_t R,
                             const uint64_t* __restrict__ dlab, const uint32_t* __restrict__ dtaint,
                             const uint32_t* __restrict__ dfree, const int32_t* __restrict__ dexcl,
                             uint64_t* __restrict__ labels, uint32_t* __restrict__ taints,
                             uint32_t* __restrict__ freer, int32_t* __restrict__ excl) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t row = rows[i];
    if (dlab)
        for (uint32_t w = 0; w < W; ++w) labels[(size_t)w * npad + row] = dlab[(size_t)w * n + i];
    if (dtaint) taints[row] = dtaint[i];
    if (dfree)
        for (uint32_t r = 0; r < R; ++r) freer[(size_t)r * npad + row] = dfree[(size_t)r * n + i];
    if (dexcl) excl[row] = dexcl[i];
}

hipError_t launch_patch(const uint32_t* rows, uint32_t n, uint32_t npad, uint32_t W, uint32_t R,
                        const uint64_t* dlab, const uint32_t* dtaint, const uint32_t* dfree, const int32_t* dexcl,
                        uint64_t* labels, uint32_t* taints, uint32_t* freer, int32_t* excl, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(patch_kernel, dim3((n + 255) / 256), dim3(256), 0, s, rows, n, npad, W, R, dlab, dtaint,
                       dfree, dexcl, labels, taints, freer, excl);
    return hipGetLastError();
}

// ----------------------------------------------------------------- launchers
template <int W, int R>
static hipError_t launch_tally_wr(const TallyArgs& a, hipStream_t s) {
    hipLaunchKernelGGL((tally_kernel<W, R>), dim3(a.n_blocks), dim3(kTallyThreads), 0, s, a.labels, a.taints,
                       a.freer, a.excl, a.npad, a.leaf_start, a.blk_leaf, a.cls, a.c0, a.nc, a.do_occ,
                       a.cap_out, a.occ_out, a.ld, a.leaf_base);
    return hipGetLastError();
}

template <int W>
static hipError_t launch_tally_w(const TallyArgs& a, hipStream_t s) {
    switch (a.R) {
        case 1: return launch_tally_wr<W, 1>(a, s);
        case 2: return launch_tally_wr<W, 2>(a, s);
        case 3: return launch_tally_wr<W, 3>(a, s);
        default: return launch_tally_wr<W, 4>(a, s);
    }
}

hipError_t launch_tally(const TallyArgs& a, hipStream_t s) {
    switch (a.W) {
        case 1: return launch_tally_w<1>(a, s);
        case 2: return launch_tally_w<2>(a, s);
        case 3: return launch_tally_w<3>(a, s);
        default: return launch_tally_w<4>(a, s);
    }
}

hipError_t launch_feas(const uint32_t* cap, const uint32_t* occ, uint32_t ld, const DevClass* cls, uint32_t C,
                       const uint32_t* word_off, uint32_t total_words, const TopoDev& topo, uint64_t* feas,
                       hipStream_t s) {
    if (total_words == 0) return hipSuccess;
    const uint32_t blocks = (total_words + 3) / 4;
    hipLaunchKernelGGL(feas_kernel, dim3(blocks), dim3(256), 0, s, cap, occ, ld, cls, C, word_off, topo, feas);
    return hipGetLastError();
}

hipError_t launch_assign(const uint64_t* feas, const uint32_t* word_off, const DevClass* cls, uint32_t C,
                         const TopoDev& topo, const uint32_t* t_off, uint32_t t_words, const uint32_t* job_class,
                         uint32_t J, int32_t* assign, uint32_t* stats, hipStream_t s) {
    hipLaunchKernelGGL(assign_kernel, dim3(1), dim3(kAssignThreads), (size_t)t_words * 8, s, feas, word_off, cls,
                       C, topo, t_off, job_class, J, assign, stats);
    return hipGetLastError();
}

hipError_t launch_resolve(const int32_t* rows, const uint32_t* levels, uint32_t n, uint32_t n_rows,
                          const uint32_t* leaf_start, uint32_t n_leaves, uint32_t leaf_base, const TopoDev& topo,
                          int32_t* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(resolve_kernel, dim3((n + 255) / 256), dim3(256), 0, s, rows, levels, n, n_rows, leaf_start,
                       n_leaves, leaf_base, topo, out);
    return hipGetLastError();
}

hipError_t launch_audit(const int32_t* leader_rows, const uint32_t* levels, const uint32_t* foff,
                        const int32_t* fdom, uint32_t n_jobs, uint32_t n_rows, const uint32_t* leaf_start,
                        uint32_t n_leaves, uint32_t leaf_base, const TopoDev& topo, uint32_t* bad, hipStream_t s) {
    if (n_jobs == 0) return hipSuccess;
    hipLaunchKernelGGL(audit_kernel, dim3((n_jobs + 3) / 4), dim3(256), 0, s, leader_rows, levels, foff, fdom,
                       n_jobs, n_rows, leaf_start, n_leaves, leaf_base, topo, bad);
    return hipGetLastError();
}

}  // namespace jsp
