// stop_anatomy.hip -- where the resident service's stop goes (DESIGN.md §11
// item 3). A persistent kernel shaped like the service (workgroup 0 polls a
// pinned host word, the others poll a device bell it rings, s_sleep between
// polls) is stopped the way jsp_engine_service_stop stops it: the host stores
// the stop word and polls hipStreamQuery. Per grid size and per amount of
// device memory the kernel dirtied first, the host times
//   seen   : stop word -> workgroup 0's "leaving" word back in host memory
//   end    : that word -> hipStreamQuery reports the kernel complete
// against an empty kernel's launch -> complete on the same stream.
// Diagnostic only.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void k_empty() {}

__global__ void k_park(unsigned* host, unsigned long long* bell, unsigned* ready, unsigned gen, uint4* dirty,
                       unsigned dirty_vec) {
    __shared__ unsigned s_go;
    if (threadIdx.x == 0) __hip_atomic_store(ready + blockIdx.x, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) {
            while (__hip_atomic_load(host, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != gen)
                __builtin_amdgcn_s_sleep(1);
            __hip_atomic_store(bell, (unsigned long long)gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    } else if (threadIdx.x == 0) {
        while (__hip_atomic_load(bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gen) __builtin_amdgcn_s_sleep(1);
    }
    __syncthreads();
    // device memory this workgroup dirtied while it lived (its share)
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < dirty_vec; i += gridDim.x * blockDim.x)
        dirty[i] = make_uint4(gen, i, gen, i);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        s_go = 1;
        __hip_atomic_store(host + 16, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double med(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}
static double p90(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() * 9 / 10];
}

int main() {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    unsigned* host;
    hipHostMalloc(reinterpret_cast<void**>(&host), 256, hipHostMallocMapped | hipHostMallocCoherent);
    std::fill(host, host + 64, 0u);
    unsigned* ready;
    hipHostMalloc(reinterpret_cast<void**>(&ready), 4096 * 4, hipHostMallocMapped | hipHostMallocCoherent);
    std::fill(ready, ready + 4096, 0u);
    unsigned long long* bell;
    hipMalloc(&bell, 128);
    hipMemset(bell, 0, 128);
    uint4* dirty;
    const unsigned max_vec = (64u << 20) / 16;
    hipMalloc(&dirty, (size_t)max_vec * 16);
    hipDeviceSynchronize();
    const int n = 60;
    {
        std::vector<double> a;
        for (int i = 0; i < n + 10; ++i) {
            const double t0 = now_us();
            hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
            while (hipStreamQuery(s) == hipErrorNotReady) {
            }
            if (i >= 10) a.push_back(now_us() - t0);
        }
        printf("empty kernel launch -> hipStreamQuery done: p50 %6.2f us p90 %6.2f\n", med(a), p90(a));
    }
    unsigned gen = 0;
    for (unsigned grid : {1u, 33u, 264u}) {
        for (unsigned mb : {0u, 1u, 16u}) {
            const unsigned dv = (mb << 20) / 16;
            std::vector<double> seen, end, tot, sync;
            for (int i = 0; i < n + 5; ++i) {
                ++gen;
                hipLaunchKernelGGL(k_park, dim3(grid), dim3(256), 0, s, host, bell, ready, gen, dirty, dv);
                for (unsigned b = 0; b < grid; ++b)
                    while (__atomic_load_n(ready + b, __ATOMIC_ACQUIRE) != gen) {
                    }
                // let it poll for a while, as the service does between requests
                const double tw = now_us();
                while (now_us() - tw < 200.0) {
                }
                const double t0 = now_us();
                __atomic_store_n(host, gen, __ATOMIC_RELEASE);
                while (__atomic_load_n(host + 16, __ATOMIC_ACQUIRE) != gen) {
                }
                const double t1 = now_us();
                while (hipStreamQuery(s) == hipErrorNotReady) {
                }
                const double t2 = now_us();
                hipDeviceSynchronize();
                const double t3 = now_us();
                if (i >= 5) {
                    seen.push_back(t1 - t0);
                    end.push_back(t2 - t1);
                    tot.push_back(t2 - t0);
                    sync.push_back(t3 - t2);
                }
            }
            printf("grid %3u dirty %2u MB: stop->leaving word p50 %6.2f | leaving->complete p50 %6.2f p90 %6.2f | "
                   "total p50 %6.2f p90 %6.2f | device sync after %5.2f us\n",
                   grid, mb, med(seen), med(end), p90(end), med(tot), p90(tot), med(sync));
        }
    }
    // how the host waits for the stopped kernel (grid 33, nothing dirtied):
    // 0 poll hipStreamQuery, 1 hipStreamSynchronize, 2 hipDeviceSynchronize,
    // 3 the leaving word then hipDeviceSynchronize, 4 hipEventSynchronize on
    // an event recorded behind the kernel at launch
    hipEvent_t ev;
    hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    const char* names[] = {"poll hipStreamQuery", "hipStreamSynchronize", "hipDeviceSynchronize",
                           "leaving word + hipDeviceSynchronize", "hipEventSynchronize (event behind it)"};
    for (int mode = 0; mode < 5; ++mode) {
        std::vector<double> tot;
        for (int i = 0; i < n + 5; ++i) {
            ++gen;
            hipLaunchKernelGGL(k_park, dim3(33), dim3(256), 0, s, host, bell, ready, gen, dirty, 0u);
            if (mode == 4) hipEventRecord(ev, s);
            for (unsigned b = 0; b < 33; ++b)
                while (__atomic_load_n(ready + b, __ATOMIC_ACQUIRE) != gen) {
                }
            const double tw = now_us();
            while (now_us() - tw < 200.0) {
            }
            const double t0 = now_us();
            __atomic_store_n(host, gen, __ATOMIC_RELEASE);
            if (mode == 0) {
                while (hipStreamQuery(s) == hipErrorNotReady) {
                }
            } else if (mode == 1) {
                hipStreamSynchronize(s);
            } else if (mode == 2) {
                hipDeviceSynchronize();
            } else if (mode == 3) {
                while (__atomic_load_n(host + 16, __ATOMIC_ACQUIRE) != gen) {
                }
                hipDeviceSynchronize();
            } else {
                hipEventSynchronize(ev);
            }
            const double t1 = now_us();
            hipDeviceSynchronize();
            if (i >= 5) tot.push_back(t1 - t0);
        }
        printf("stop word -> %-40s p50 %6.2f us p90 %6.2f\n", names[mode], med(tot), p90(tot));
    }
    return 0;
}
