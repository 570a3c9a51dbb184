// dispatch_probe.hip — measures when each workgroup of a small grid starts
// (s_memrealtime, 100 MHz) relative to the first, for several kernel shapes.
// Diagnostic only: explains the launch-latency floor of the single-launch
// placement kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

__global__ void probe_plain(unsigned long long* t) {
    if (threadIdx.x == 0) t[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
}

__global__ void probe_lds(unsigned long long* t) {
    extern __shared__ unsigned int lds[];
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (threadIdx.x == 0) t[blockIdx.x] = __builtin_amdgcn_s_memrealtime() + (lds[5] == 12345);
}

__global__ void probe_busy(unsigned long long* t, const unsigned* src, unsigned* dst) {
    if (threadIdx.x == 0) t[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    unsigned v = src[blockIdx.x * blockDim.x + threadIdx.x];
    for (int i = 0; i < 2000; ++i) v = v * 1664525u + 1013904223u;
    dst[blockIdx.x * blockDim.x + threadIdx.x] = v;
}

template <class F>
void run(const char* name, int grid, int block, size_t lds, F launch, unsigned long long* d_t) {
    std::vector<std::vector<double>> rows;
    for (int rep = 0; rep < 60; ++rep) {
        hipMemset(d_t, 0, 64 * sizeof(unsigned long long));
        launch(grid, block, lds);
        hipDeviceSynchronize();
        std::vector<unsigned long long> t(grid);
        hipMemcpy(t.data(), d_t, grid * sizeof(unsigned long long), hipMemcpyDeviceToHost);
        unsigned long long t0 = *std::min_element(t.begin(), t.end());
        std::vector<double> r(grid);
        for (int b = 0; b < grid; ++b) r[b] = (t[b] - t0) * 10.0;
        if (rep >= 10) rows.push_back(r);
    }
    printf("%-28s grid=%3d block=%4d lds=%6zu : median start ns per workgroup:", name, grid, block, lds);
    for (int b = 0; b < grid; ++b) {
        std::vector<double> v;
        for (auto& r : rows) v.push_back(r[b]);
        std::sort(v.begin(), v.end());
        printf(" %.0f", v[v.size() / 2]);
    }
    printf("\n");
}

int main() {
    unsigned long long* d_t;
    unsigned *src, *dst;
    hipMalloc(&d_t, 64 * sizeof(unsigned long long));
    hipMalloc(&src, 64 * 1024 * 4);
    hipMalloc(&dst, 64 * 1024 * 4);
    hipMemset(src, 1, 64 * 1024 * 4);
    for (int grid : {8, 16, 32}) {
        run("plain", grid, 256, 0, [&](int g, int b, size_t l) { hipLaunchKernelGGL(probe_plain, dim3(g), dim3(b), l, 0, d_t); }, d_t);
        run("plain-64thr", grid, 64, 0, [&](int g, int b, size_t l) { hipLaunchKernelGGL(probe_plain, dim3(g), dim3(b), l, 0, d_t); }, d_t);
        run("lds-16KiB", grid, 256, 16384, [&](int g, int b, size_t l) { hipLaunchKernelGGL(probe_lds, dim3(g), dim3(b), l, 0, d_t); }, d_t);
        run("busy", grid, 256, 0, [&](int g, int b, size_t l) { hipLaunchKernelGGL(probe_busy, dim3(g), dim3(b), l, 0, d_t, src, dst); }, d_t);
    }
    // back-to-back launches without host sync between them (the bench's situation)
    for (int rep = 0; rep < 3; ++rep) {
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        hipEventRecord(a, 0);
        for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(probe_plain, dim3(16), dim3(256), 0, 0, d_t);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        printf("200 back-to-back 16x256 trivial launches: %.2f us per launch\n", ms * 1000 / 200);
    }
    return 0;
}
