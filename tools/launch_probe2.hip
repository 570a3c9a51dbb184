// launch_probe2.hip — what the host-API placement path pays besides the
// kernel body: launch + completion seen through host completion words, by
// kernel argument size, grid oversubscription and how the output reaches
// host memory. Diagnostic only.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

struct Big {
    unsigned long long w[32];  // 256 B, like TallyArgs + CompactArgs
};

__global__ void k_small(unsigned* done, unsigned seq) {
    if (threadIdx.x == 0 && blockIdx.x == 0) __hip_atomic_store(done, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_big(Big b, unsigned* done, unsigned seq) {
    if (threadIdx.x == 0 && blockIdx.x == 0)
        __hip_atomic_store(done, seq + (unsigned)(b.w[31] & 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// tiles from a ticket; tile t writes n ints of out[] (host or device) then done[t]
template <int MODE>  // 0: system-scope stores to host, 1: plain stores + system release, 2: out in device memory
__global__ void k_tiles(unsigned long long* ticket, unsigned long long base, int tiles, int n, int* out, unsigned* done,
                        unsigned seq) {
    extern __shared__ unsigned lds_dyn[];
    __shared__ unsigned lds[1];
    if (threadIdx.x == 0)
        lds[0] = (unsigned)(__hip_atomic_fetch_add(ticket, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - base);
    __syncthreads();
    const unsigned t = lds[0];
    if ((int)t >= tiles) return;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        if (MODE == 0) __hip_atomic_store(out + t * n + i, (int)seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        else out[t * n + i] = (int)seq;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        if (MODE == 1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(done + t, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static unsigned g_seq = 1;
template <class L>
static void measure(const char* name, L launch, unsigned* done, int words, int reps = 1500) {
    std::vector<double> v, lv;
    unsigned& seq = g_seq;
    for (int i = 0; i < reps; ++i) {
        ++seq;
        double t0 = now_us();
        launch(seq);
        double t1 = now_us();
        for (int w = 0; w < words; ++w)
            while (__atomic_load_n(done + w, __ATOMIC_ACQUIRE) != seq) {
                if (now_us() - t0 > 2e6) {
                    printf("%s: TIMEOUT rep %d word %d value %u want %u\n", name, i, w, done[w], seq);
                    fflush(stdout);
                    exit(3);
                }
            }
        double t2 = now_us();
        if (i >= 100) {
            v.push_back(t2 - t0);
            lv.push_back(t1 - t0);
        }
    }
    std::sort(v.begin(), v.end());
    std::sort(lv.begin(), lv.end());
    fflush(stdout);
    printf("%-58s total p50 %6.2f us p90 %6.2f | launch call p50 %5.2f\n", name, v[v.size() / 2], v[v.size() * 9 / 10],
           lv[lv.size() / 2]);
    fflush(stdout);
}

int main() {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    unsigned* done;
    int* hout;
    int* dout;
    unsigned long long* ticket;
    hipHostMalloc(reinterpret_cast<void**>(&done), 4096, hipHostMallocMapped | hipHostMallocCoherent);
    hipHostMalloc(reinterpret_cast<void**>(&hout), 1 << 20, hipHostMallocMapped | hipHostMallocCoherent);
    hipMalloc(&dout, 1 << 20);
    hipMalloc(&ticket, 64);
    hipMemset(ticket, 0, 64);
    hipDeviceSynchronize();
    unsigned long long draws = 0;
    Big b{};
    measure("1 WG, small args", [&](unsigned q) { hipLaunchKernelGGL(k_small, dim3(1), dim3(256), 0, s, done, q); },
            done, 1);
    measure("1 WG, 256-B by-value args", [&](unsigned q) { hipLaunchKernelGGL(k_big, dim3(1), dim3(256), 0, s, b, done, q); },
            done, 1);
    for (int grid : {15, 79}) {
        for (int lds : {0, 24 * 1024}) {
            char name[128];
            snprintf(name, sizeof name, "grid %d lds %dK: 15 tiles x 66 ints, sys stores", grid, lds / 1024);
            measure(name, [&](unsigned q) {
                hipLaunchKernelGGL(k_tiles<0>, dim3(grid), dim3(256), lds, s, ticket, draws, 15, 66, hout, done, q);
                draws += grid;
            }, done, 15);
        }
    }
    measure("grid 79 lds 24K: plain stores + system release", [&](unsigned q) {
        hipLaunchKernelGGL(k_tiles<1>, dim3(79), dim3(256), 24 * 1024, s, ticket, draws, 15, 66, hout, done, q);
        draws += 79;
    }, done, 15);
    measure("grid 79 lds 24K: output to device memory, flag to host", [&](unsigned q) {
        hipLaunchKernelGGL(k_tiles<2>, dim3(79), dim3(256), 24 * 1024, s, ticket, draws, 15, 66, dout, done, q);
        draws += 79;
    }, done, 15);
    measure("grid 79 lds 24K: 1 tile only", [&](unsigned q) {
        hipLaunchKernelGGL(k_tiles<0>, dim3(79), dim3(256), 24 * 1024, s, ticket, draws, 1, 66, hout, done, q);
        draws += 79;
    }, done, 1);
    hipStreamSynchronize(s);
    return 0;
}
