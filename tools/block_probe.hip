// block_probe.hip — which HIP host calls wait for a kernel that stays
// resident on another stream (the placement service), and how fast a launch
// answers after the GPU sat idle with and without a one-wave keeper kernel
// resident (diagnostic).
//
// keeper: one wave polls a host-mapped stop word with s_sleep and leaves on
// it or after max_ticks of the 100 MHz clock (every run ends by itself).
// Output: one JSON line per measurement series.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

__global__ void keeper(const uint32_t* stop, unsigned long long max_ticks, uint32_t sleep_mode) {
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = wall_clock64();
    while (true) {
        if (__hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) break;
        if (wall_clock64() - t0 > max_ticks) break;
        if (sleep_mode == 0) __builtin_amdgcn_s_sleep(127);
        else __builtin_amdgcn_s_sleep(8);
    }
}

__global__ void tiny(uint32_t* p) {
    if (threadIdx.x == 0) p[blockIdx.x] += 1;
}

using clk = std::chrono::steady_clock;
static double us_since(clk::time_point t0) {
    return std::chrono::duration<double, std::micro>(clk::now() - t0).count();
}

struct Keeper {
    uint32_t* stop = nullptr;
    hipStream_t s = nullptr;
    bool on = false;
    void start(unsigned long long ticks, uint32_t mode = 0) {
        if (!stop) CK(hipHostMalloc(&stop, 64, hipHostMallocMapped | hipHostMallocCoherent));
        if (!s) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        __atomic_store_n(stop, 0u, __ATOMIC_RELEASE);
        hipLaunchKernelGGL(keeper, dim3(1), dim3(64), 0, s, stop, ticks, mode);
        CK(hipGetLastError());
        on = true;
        std::this_thread::sleep_for(std::chrono::milliseconds(2));
    }
    void halt() {
        if (!on) return;
        __atomic_store_n(stop, 1u, __ATOMIC_RELEASE);
        CK(hipStreamSynchronize(s));
        on = false;
    }
};

static std::string pct(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    char b[128];
    std::snprintf(b, sizeof b, "{\"p50\": %.1f, \"max\": %.1f}", v[v.size() / 2], v.back());
    return b;
}

int main(int argc, char** argv) {
    const int trials = argc > 1 ? std::atoi(argv[1]) : 15;
    CK(hipSetDevice(0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint32_t* d = nullptr;
    CK(hipMalloc(&d, 4096));
    CK(hipMemset(d, 0, 4096));
    CK(hipDeviceSynchronize());
    Keeper k;

    // 1. host calls made while a kernel stays resident on another stream:
    // a call that waits for it returns only when the keeper leaves (1 s).
    // Every call is made once before (first-use costs: blit kernels, staging).
    {
        std::vector<char> host(1 << 20, 1);
        {
            void* w = nullptr;
            CK(hipMalloc(&w, 1 << 20));
            CK(hipMemcpyAsync(w, host.data(), 65536, hipMemcpyHostToDevice, s));
            CK(hipMemcpyAsync(host.data(), w, 65536, hipMemcpyDeviceToHost, s));
            CK(hipMemsetAsync(w, 0, 65536, s));
            CK(hipStreamSynchronize(s));
            CK(hipFree(w));
        }
        k.start(100000000ull);  // 1 s
        std::printf("{\"blocking\": {");
        auto timed = [&](const char* name, auto fn, bool last = false) {
            const auto t0 = clk::now();
            fn();
            std::printf("\"%s\": %.1f%s", name, us_since(t0), last ? "" : ", ");
            std::fflush(stdout);
        };
        void* a = nullptr;
        void* h = nullptr;
        timed("hipMalloc_1MiB", [&] { CK(hipMalloc(&a, 1 << 20)); });
        timed("hipMemcpyAsync_pageable_64KiB_sync", [&] {
            CK(hipMemcpyAsync(a, host.data(), 65536, hipMemcpyHostToDevice, s));
            CK(hipStreamSynchronize(s));
        });
        timed("hipMemcpyAsync_pageable_D2H_64KiB_sync", [&] {
            CK(hipMemcpyAsync(host.data(), a, 65536, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
        });
        timed("hipMemsetAsync_64KiB_sync", [&] {
            CK(hipMemsetAsync(a, 0, 65536, s));
            CK(hipStreamSynchronize(s));
        });
        timed("kernel_and_stream_sync", [&] {
            hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d);
            CK(hipStreamSynchronize(s));
        });
        timed("hipHostMalloc_1MiB", [&] { CK(hipHostMalloc(&h, 1 << 20, hipHostMallocMapped | hipHostMallocCoherent)); });
        timed("hipFree_1MiB", [&] { CK(hipFree(a)); });
        const bool still = k.on && __atomic_load_n(k.stop, __ATOMIC_ACQUIRE) == 0 &&
                           hipStreamQuery(k.s) == hipErrorNotReady;
        timed("hipHostFree_1MiB", [&] { CK(hipHostFree(h)); });
        const bool still2 = hipStreamQuery(k.s) == hipErrorNotReady;
        std::printf("\"keeper_alive_after_hipFree\": %s, \"keeper_alive_after_hipHostFree\": %s}}\n",
                    still ? "true" : "false", still2 ? "true" : "false");
        std::fflush(stdout);
        k.halt();
    }

    // 2. tiny launch + synchronize after an idle gap, without / with a keeper
    const double gaps_ms[] = {0.1, 1.0, 5.0, 20.0, 60.0, 200.0};
    for (int mode = 0; mode < 3; ++mode) {
        if (mode == 1) k.start(3000000000ull, 0);  // 30 s, s_sleep 127
        if (mode == 2) k.start(3000000000ull, 1);  // 30 s, s_sleep 8
        std::printf("{\"%s\": {", mode == 0 ? "launch_idle" : mode == 1 ? "launch_with_keeper_sleep127"
                                                                          : "launch_with_keeper_sleep8");
        for (int gi = 0; gi < 6; ++gi) {
            std::vector<double> v;
            for (int t = 0; t < trials; ++t) {
                std::this_thread::sleep_for(std::chrono::microseconds((long)(gaps_ms[gi] * 1000)));
                const auto t0 = clk::now();
                hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d);
                CK(hipStreamSynchronize(s));
                v.push_back(us_since(t0));
            }
            std::printf("\"%gms\": %s%s", gaps_ms[gi], pct(v).c_str(), gi == 5 ? "" : ", ");
            std::fflush(stdout);
        }
        std::printf("}}\n");
        std::fflush(stdout);
        k.halt();
    }
    // 3. the launch call alone (host wall of hipLaunchKernel, no wait) after an idle gap
    {
        std::printf("{\"launch_call_only\": {");
        for (int gi = 0; gi < 6; ++gi) {
            std::vector<double> v;
            for (int t = 0; t < trials; ++t) {
                std::this_thread::sleep_for(std::chrono::microseconds((long)(gaps_ms[gi] * 1000)));
                const auto t0 = clk::now();
                hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d);
                v.push_back(us_since(t0));
                CK(hipStreamSynchronize(s));
            }
            std::printf("\"%gms\": %s%s", gaps_ms[gi], pct(v).c_str(), gi == 5 ? "" : ", ");
            std::fflush(stdout);
        }
        std::printf("}}\n");
    }
    CK(hipFree(d));
    return 0;
}
