// launch_probe.hip — host-API latency floor on MI355X: how long one kernel
// launch takes from the host call to the host seeing its result, by the way
// the host learns of completion. Diagnostic only: it prices the fixed part of
// jsp_place's host-API latency.
//   sync     : hipLaunchKernel + hipStreamSynchronize
//   event    : hipLaunchKernel + hipEventRecord + hipEventSynchronize
//   flag     : kernel stores a sequence number to pinned host memory (vector
//              store, system scope); the host spins on it
//   launch   : host time of the hipLaunchKernel call alone
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void k_empty(int* p) {
    if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] = 1;
}

__global__ void k_flag(volatile unsigned* flag, unsigned seq) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        __hip_atomic_store(const_cast<unsigned*>(flag), seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void report(const char* name, std::vector<double>& v) {
    std::sort(v.begin(), v.end());
    printf("%-34s p50 %7.2f us  p10 %7.2f  p90 %7.2f  p99 %7.2f\n", name, v[v.size() / 2], v[v.size() / 10],
           v[v.size() * 9 / 10], v[v.size() * 99 / 100]);
}

int main() {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    int* d;
    hipMalloc(&d, 64);
    unsigned* flag;
    hipHostMalloc(reinterpret_cast<void**>(&flag), 64, hipHostMallocMapped | hipHostMallocCoherent);
    *flag = 0;
    hipEvent_t ev;
    hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    const int n = 2000;
    for (int grid : {1, 16}) {
        std::vector<double> a, b, c, e;
        for (int i = 0; i < n; ++i) {
            double t0 = now_us();
            hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, s, d);
            double t1 = now_us();
            hipStreamSynchronize(s);
            double t2 = now_us();
            if (i > 100) { a.push_back(t2 - t0); e.push_back(t1 - t0); }
        }
        for (int i = 0; i < n; ++i) {
            double t0 = now_us();
            hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, s, d);
            hipEventRecord(ev, s);
            hipEventSynchronize(ev);
            double t2 = now_us();
            if (i > 100) b.push_back(t2 - t0);
        }
        for (int i = 0; i < n; ++i) {
            const unsigned seq = (unsigned)i + 1 + (grid << 20);
            double t0 = now_us();
            hipLaunchKernelGGL(k_flag, dim3(grid), dim3(256), 0, s, flag, seq);
            while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
            }
            double t2 = now_us();
            if (i > 100) c.push_back(t2 - t0);
        }
        hipStreamSynchronize(s);
        printf("grid %d:\n", grid);
        report("  launch call only", e);
        report("  launch + hipStreamSynchronize", a);
        report("  launch + event sync", b);
        report("  launch + host spin on mapped flag", c);
    }
    return 0;
}
