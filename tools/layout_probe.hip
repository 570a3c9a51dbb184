// layout_probe.hip — does the snapshot's column layout set the tally's cold
// time? Diagnostic only (make tools/bin/layout_probe), not the product.
//
// 1,048,576 rows of the engine's row format (W = 1 label word, R = 3 free
// resources: 28 B per row), read once by a tally-shaped grid (256-thread
// workgroups, 4 consecutive rows per thread, 16-B loads per column), values
// XOR-folded, one word written per workgroup:
//   soa    the engine's layout: one column per allocation, npad rows each
//   tile   tile-major: per 256-row tile its columns back to back (7 KB)
//   flat   a contiguous read of the same byte count (the streaming ceiling)
// Cold = a 512 MiB scrub read before each launch; warm = back to back.
// HIP events around one launch (median of 21) and around 200 launches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
            std::exit(1);                                                      \
        }                                                                      \
    } while (0)

constexpr int kThreads = 256;
constexpr unsigned kRows = 1u << 20;
constexpr unsigned kNpad = kRows + 64;
constexpr unsigned kTileRows = 256;
constexpr unsigned kTileBytes = kTileRows * 28;  // labels 8 + taints 4 + free 12 + excl 4

struct Soa {
    const unsigned long long* labels;
    const unsigned* taints;
    const unsigned* freer;
    const int* excl;
};

__device__ __forceinline__ unsigned fold4(uint4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

__global__ __launch_bounds__(kThreads) void soa_kernel(Soa s, unsigned* out) {
    const unsigned row = blockIdx.x * 1024u + 4u * threadIdx.x;
    unsigned x = 0;
    if (row < kRows) {
        const uint4* l = reinterpret_cast<const uint4*>(s.labels + row);
        x ^= fold4(l[0]) ^ fold4(l[1]);
        x ^= fold4(*reinterpret_cast<const uint4*>(s.taints + row));
#pragma unroll
        for (int r = 0; r < 3; ++r) x ^= fold4(*reinterpret_cast<const uint4*>(s.freer + (size_t)r * kNpad + row));
        x ^= fold4(*reinterpret_cast<const uint4*>(s.excl + row));
    }
    for (int o = 32; o > 0; o >>= 1) x ^= __shfl_xor(x, o, 64);
    if (threadIdx.x == 0 && x == 0x9e3779b9u) out[blockIdx.x] = x;
}

// tile-major: tile t = row / 256 at t * kTileBytes: labels[256] u64, taints[256],
// free[3][256], excl[256]
__global__ __launch_bounds__(kThreads) void tile_kernel(const unsigned char* base, unsigned* out) {
    const unsigned row = blockIdx.x * 1024u + 4u * threadIdx.x;
    unsigned x = 0;
    if (row < kRows) {
        const unsigned char* t = base + (size_t)(row / kTileRows) * kTileBytes;
        const unsigned i = row % kTileRows;
        const uint4* l = reinterpret_cast<const uint4*>(t + 8 * i);
        x ^= fold4(l[0]) ^ fold4(l[1]);
        x ^= fold4(*reinterpret_cast<const uint4*>(t + 2048 + 4 * i));
#pragma unroll
        for (int r = 0; r < 3; ++r) x ^= fold4(*reinterpret_cast<const uint4*>(t + 3072 + 1024 * r + 4 * i));
        x ^= fold4(*reinterpret_cast<const uint4*>(t + 6144 + 4 * i));
    }
    for (int o = 32; o > 0; o >>= 1) x ^= __shfl_xor(x, o, 64);
    if (threadIdx.x == 0 && x == 0x9e3779b9u) out[blockIdx.x] = x;
}

// the same bytes as one stream: 7 x 16 B per thread, consecutive per instruction
__global__ __launch_bounds__(kThreads) void flat_kernel(const uint4* p, unsigned* out) {
    const size_t b = (size_t)blockIdx.x * kThreads * 7;
    unsigned x = 0;
#pragma unroll
    for (int i = 0; i < 7; ++i) x ^= fold4(p[b + (size_t)i * kThreads + threadIdx.x]);
    for (int o = 32; o > 0; o >>= 1) x ^= __shfl_xor(x, o, 64);
    if (threadIdx.x == 0 && x == 0x9e3779b9u) out[blockIdx.x] = x;
}

__global__ void scrub_kernel(const uint4* p, size_t n, unsigned* out) {
    unsigned x = 0;
    for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (size_t)gridDim.x * blockDim.x)
        x ^= fold4(p[k]);
    if (x == 0x9e3779b9u) out[0] = x;
}

int main() {
    unsigned long long* labels;
    unsigned *taints, *freer, *out;
    int* excl;
    unsigned char* tiles;
    uint4 *flat, *scrub;
    const size_t scrub_bytes = 512u << 20;
    CK(hipMalloc(&labels, (size_t)kNpad * 8));
    CK(hipMalloc(&taints, (size_t)kNpad * 4));
    CK(hipMalloc(&freer, (size_t)kNpad * 12));
    CK(hipMalloc(&excl, (size_t)kNpad * 4));
    CK(hipMalloc(&tiles, (size_t)(kRows / kTileRows) * kTileBytes));
    CK(hipMalloc(&flat, (size_t)kRows * 28));
    CK(hipMalloc(&scrub, scrub_bytes));
    CK(hipMalloc(&out, 1 << 20));
    CK(hipMemset(labels, 1, (size_t)kNpad * 8));
    CK(hipMemset(taints, 2, (size_t)kNpad * 4));
    CK(hipMemset(freer, 3, (size_t)kNpad * 12));
    CK(hipMemset(excl, 4, (size_t)kNpad * 4));
    CK(hipMemset(tiles, 5, (size_t)(kRows / kTileRows) * kTileBytes));
    CK(hipMemset(flat, 6, (size_t)kRows * 28));
    CK(hipMemset(scrub, 7, scrub_bytes));
    Soa s{labels, taints, freer, excl};
    const unsigned grid = kRows / 1024;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto time_one = [&](auto launch, bool cold) {
        std::vector<float> t;
        for (int r = 0; r < 21; ++r) {
            if (cold) hipLaunchKernelGGL(scrub_kernel, dim3(4096), dim3(256), 0, 0, scrub, scrub_bytes / 16, out);
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
    auto time_loop = [&](auto launch) {
        for (int r = 0; r < 10; ++r) launch();
        CK(hipEventRecord(a, 0));
        for (int r = 0; r < 200; ++r) launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms * 1000.f / 200;
    };
    auto soa = [&]() { hipLaunchKernelGGL(soa_kernel, dim3(grid), dim3(kThreads), 0, 0, s, out); };
    auto tile = [&]() { hipLaunchKernelGGL(tile_kernel, dim3(grid), dim3(kThreads), 0, 0, tiles, out); };
    auto fl = [&]() { hipLaunchKernelGGL(flat_kernel, dim3(grid), dim3(kThreads), 0, 0, flat, out); };
    const double bytes = (double)kRows * 28;
    std::printf("{\"probe\": \"layout\", \"rows\": %u, \"bytes\": %.0f, \"results\": {", kRows, bytes);
    const char* names[3] = {"soa", "tile", "flat"};
    for (int k = 0; k < 3; ++k) {
        float cold, warm, loop;
        if (k == 0) { cold = time_one(soa, true); warm = time_one(soa, false); loop = time_loop(soa); }
        else if (k == 1) { cold = time_one(tile, true); warm = time_one(tile, false); loop = time_loop(tile); }
        else { cold = time_one(fl, true); warm = time_one(fl, false); loop = time_loop(fl); }
        std::printf("%s\"%s\": {\"cold_us\": %.2f, \"warm_us\": %.2f, \"loop_us\": %.2f, \"cold_gbs\": %.0f, \"loop_gbs\": %.0f}",
                    k ? ", " : "", names[k], cold, warm, loop, bytes / cold / 1e3, bytes / loop / 1e3);
    }
    std::printf("}}\n");
    CK(hipGetLastError());
    return 0;
}
