// stream_ceiling.hip — the achievable HBM streaming rate on this MI355X at the
// byte counts the placement kernels move (cfg2 compaction 0.43 MB, cfg4 tally
// 29-31 MB), as the ceiling the roofline fractions in DESIGN.md are read
// against. Diagnostic only (make tools/diag/stream_ceiling), not the product.
//
// For each size it times, with HIP events around ONE launch:
//   read   — every byte read once with 16-B loads, XOR-folded per workgroup,
//            one word written per workgroup (what a tally does at best);
//   copy   — read + write of the same byte count split in halves;
// both "cold" (before each launch a separate kernel reads a 512 MiB buffer,
// which evicts the 256 MiB Infinity Cache and every XCD's L2 without leaving
// dirty lines behind) and "warm" (the same launch repeated back to back).
// Grid shape follows the tally: 256 threads, 16 KiB per workgroup (4 x 16 B
// per thread), so the launch has the tally's workgroup count at each size.
// Prints one JSON line.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

constexpr int kThreads = 256;
constexpr int kVecPerThread = 4;                                  // 4 x 16 B per thread
constexpr size_t kBlockBytes = (size_t)kThreads * kVecPerThread * 16;  // 16 KiB

__global__ __launch_bounds__(kThreads) void read_kernel(const uint4* __restrict__ src, size_t n_vec,
                                                        unsigned* __restrict__ out) {
    const size_t base = (size_t)blockIdx.x * kThreads * kVecPerThread + threadIdx.x;
    uint4 v[kVecPerThread];
#pragma unroll
    for (int i = 0; i < kVecPerThread; ++i) {
        const size_t k = base + (size_t)i * kThreads;
        v[i] = k < n_vec ? src[k] : make_uint4(0, 0, 0, 0);
    }
    unsigned x = 0;
#pragma unroll
    for (int i = 0; i < kVecPerThread; ++i) x ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
    for (int o = 32; o > 0; o >>= 1) x ^= __shfl_xor(x, o, 64);
    if ((threadIdx.x & 63) == 0 && x == 0x9e3779b9u) out[blockIdx.x] = x;  // keeps the loads live
}

__global__ __launch_bounds__(kThreads) void copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                        size_t n_vec) {
    const size_t base = (size_t)blockIdx.x * kThreads * kVecPerThread + threadIdx.x;
    uint4 v[kVecPerThread];
#pragma unroll
    for (int i = 0; i < kVecPerThread; ++i) {
        const size_t k = base + (size_t)i * kThreads;
        if (k < n_vec) v[i] = src[k];
    }
#pragma unroll
    for (int i = 0; i < kVecPerThread; ++i) {
        const size_t k = base + (size_t)i * kThreads;
        if (k < n_vec) dst[k] = v[i];
    }
}

// cache scrub: read 512 MiB (no stores of its lines)
__global__ __launch_bounds__(kThreads) void scrub_kernel(const uint4* __restrict__ p, size_t n_vec,
                                                         unsigned* __restrict__ out) {
    unsigned x = 0;
    for (size_t k = (size_t)blockIdx.x * kThreads + threadIdx.x; k < n_vec; k += (size_t)gridDim.x * kThreads) {
        const uint4 v = p[k];
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x9e3779b9u) out[0] = x;
}

int main() {
    const size_t sizes[] = {427964, 4u << 20, 30560128, 64u << 20, 256u << 20};
    const size_t max_bytes = 256u << 20;
    const size_t scrub_bytes = 512u << 20;
    uint4 *src, *dst, *scrub;
    unsigned* out;
    CK(hipMalloc(&src, max_bytes));
    CK(hipMalloc(&dst, max_bytes));
    CK(hipMalloc(&scrub, scrub_bytes));
    CK(hipMalloc(&out, 1 << 20));
    CK(hipMemset(src, 1, max_bytes));
    CK(hipMemset(dst, 0, max_bytes));
    CK(hipMemset(scrub, 2, scrub_bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto scrub_once = [&]() {
        hipLaunchKernelGGL(scrub_kernel, dim3(4096), dim3(kThreads), 0, 0, scrub, scrub_bytes / 16, out);
    };
    auto time_us = [&](auto launch, bool cold, int reps) {
        std::vector<float> t;
        for (int r = 0; r < reps; ++r) {
            if (cold) scrub_once();
            CK(hipEventRecord(a, 0));
            launch();
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            t.push_back(ms * 1000.f);
        }
        std::sort(t.begin(), t.end());
        return t[t.size() / 2];
    };
    std::printf("{\"probe\": \"stream_ceiling\", \"unit\": \"us / GB/s\", \"results\": [");
    bool first = true;
    for (size_t bytes : sizes) {
        const size_t nv = bytes / 16;
        const unsigned grid_r = (unsigned)((bytes + kBlockBytes - 1) / kBlockBytes);
        const size_t nv_c = bytes / 32;  // copy: half read, half written
        const unsigned grid_c = (unsigned)((bytes / 2 + kBlockBytes - 1) / kBlockBytes);
        auto rd = [&]() { hipLaunchKernelGGL(read_kernel, dim3(grid_r), dim3(kThreads), 0, 0, src, nv, out); };
        auto cp = [&]() { hipLaunchKernelGGL(copy_kernel, dim3(grid_c), dim3(kThreads), 0, 0, src, dst, nv_c); };
        for (int w = 0; w < 5; ++w) { rd(); cp(); }
        CK(hipDeviceSynchronize());
        const float rc = time_us(rd, true, 21), rw = time_us(rd, false, 21);
        const float cc = time_us(cp, true, 21), cw = time_us(cp, false, 21);
        auto gbs = [&](float us) { return (double)bytes / (us * 1e-6) / 1e9; };
        std::printf("%s{\"bytes\": %zu, \"workgroups\": %u, \"read_cold_us\": %.2f, \"read_cold_gbs\": %.1f, "
                    "\"read_warm_us\": %.2f, \"read_warm_gbs\": %.1f, \"copy_cold_us\": %.2f, \"copy_cold_gbs\": %.1f, "
                    "\"copy_warm_us\": %.2f, \"copy_warm_gbs\": %.1f}",
                    first ? "" : ", ", bytes, grid_r, rc, gbs(rc), rw, gbs(rw), cc, gbs(cc), cw, gbs(cw));
        first = false;
    }
    std::printf("]}\n");
    CK(hipGetLastError());
    return 0;
}
