// mailbox_probe.hip — where should the resident service's request word live?
// A one-wave persistent kernel answers a host ping-pong: the host writes seq i
// into the request word, the kernel polls it (system-scope loads) and writes
// an ack word in pinned host memory, the host spins on the ack. Round trip
// p50/p90 for a request word in
//   host: pinned host memory (what the service uses now; the device polls
//         across PCIe),
//   bar:  fine-grained device memory the CPU may write through the BAR
//         (hsa_amd_agents_allow_access; absent on hosts without a large BAR),
// plus the host-side cost of the request write itself. Diagnostic only.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            printf("{\"error\": \"%s: %s\"}\n", #x, hipGetErrorString(e_));        \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

// wave w (of `pollers`) polls its own request word and answers in its own ack
// word, so `pollers` loads are in flight at staggered times; the host takes
// the first ack. Every wave gives up (err word) after 200 ms without a
// request, so the grid always drains.
__global__ void pingpong(const unsigned* req, unsigned* ack, unsigned* err, unsigned n) {
    const unsigned w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (unsigned k = 0; k < w; ++k) __builtin_amdgcn_s_sleep(12);  // ~1/4 of a PCIe round trip apart
    for (unsigned i = 1; i <= n; ++i) {
        const unsigned long long t0 = wall_clock64();
        while (__hip_atomic_load(req + w * 16u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < i) {
            if (wall_clock64() - t0 > 20000000ull) {
                if (lane == 0) __hip_atomic_store(err + w * 16u, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                return;
            }
        }
        if (lane == 0) __hip_atomic_store(ack + w * 16u, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static hsa_agent_t g_cpu{}, g_gpu{};
static hsa_status_t find_agents(hsa_agent_t a, void*) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_CPU && g_cpu.handle == 0) g_cpu = a;
    if (t == HSA_DEVICE_TYPE_GPU && g_gpu.handle == 0) g_gpu = a;
    return HSA_STATUS_SUCCESS;
}

// request words for `pollers` lanes, 64 B apart; every one gets the same seq
static void post(unsigned* req, unsigned pollers, unsigned v) {
    for (unsigned p = 0; p < pollers; ++p) __atomic_store_n(req + p * 16u, v, __ATOMIC_RELEASE);
    __atomic_thread_fence(__ATOMIC_SEQ_CST);  // drain the write-combining buffer toward the device
}

static void run(const char* name, unsigned* req, unsigned* ack, unsigned* err, unsigned pollers, bool last) {
    const unsigned n = 3000;
    for (unsigned p = 0; p < pollers; ++p) __atomic_store_n(req + p * 16u, 0u, __ATOMIC_RELEASE);
    for (unsigned p = 0; p < pollers; ++p) {
        __atomic_store_n(ack + p * 16u, 0u, __ATOMIC_RELEASE);
        __atomic_store_n(err + p * 16u, 0u, __ATOMIC_RELEASE);
    }
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    hipLaunchKernelGGL(pingpong, dim3(1), dim3(64 * pollers), 0, 0, req, ack, err, n);
    std::vector<double> rt, wr;
    bool ok = true;
    for (unsigned i = 1; i <= n && ok; ++i) {
        const double t0 = now_us();
        post(req, pollers, i);
        const double t1 = now_us();
        for (bool seen = false; !seen;) {
            for (unsigned p = 0; p < pollers; ++p) seen |= __atomic_load_n(ack + p * 16u, __ATOMIC_ACQUIRE) == i;
            if (!seen && (__atomic_load_n(err, __ATOMIC_ACQUIRE) != 0 || now_us() - t0 > 1e6)) {
                ok = false;
                break;
            }
        }
        const double t2 = now_us();
        if (i > 200) {
            rt.push_back(t2 - t0);
            wr.push_back(t1 - t0);
        }
        // a host-side gap like the placement calls' (the host does work between requests)
        const double g = now_us();
        while (now_us() - g < 5.0) {
        }
    }
    // a request the kernel no longer waits for cannot strand it: it stops after n
    // or on its own 200 ms timeout
    CK(hipDeviceSynchronize());
    if (!ok) {
        printf("  \"%s\": {\"error\": \"no ack (err word %u)\"}%s\n", name, *err, last ? "" : ",");
        return;
    }
    std::sort(rt.begin(), rt.end());
    std::sort(wr.begin(), wr.end());
    const size_t m = rt.size();
    printf("  \"%s\": {\"rt_p50_us\": %.3f, \"rt_p90_us\": %.3f, \"rt_p99_us\": %.3f, \"post_p50_us\": %.3f}%s\n", name,
           rt[m / 2], rt[m * 9 / 10], rt[m * 99 / 100], wr[m / 2], last ? "" : ",");
    fflush(stdout);
}

int main() {
    CK(hipSetDevice(0));
    unsigned *hreq, *ack, *err;
    CK(hipHostMalloc(reinterpret_cast<void**>(&hreq), 4096, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostMalloc(reinterpret_cast<void**>(&ack), 4096, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostMalloc(reinterpret_cast<void**>(&err), 4096, hipHostMallocMapped | hipHostMallocCoherent));
    hsa_iterate_agents(find_agents, nullptr);
    // device memory the CPU may touch: the GPU's fine-grained pool, opened to the CPU agent
    unsigned* dreq = nullptr;
    const char* bar_note = "ok";
    CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&dreq), 4096, hipDeviceMallocFinegrained));
    if (g_cpu.handle == 0) {
        bar_note = "no CPU agent";
        dreq = nullptr;
    } else if (hsa_amd_agents_allow_access(1, &g_cpu, nullptr, dreq) != HSA_STATUS_SUCCESS) {
        bar_note = "hsa_amd_agents_allow_access refused (no large BAR?)";
        dreq = nullptr;
    }
    printf("{\n  \"bar_mailbox\": \"%s\",\n", bar_note);
    run("host_1poller", hreq, ack, err, 1, false);
    run("host_4pollers", hreq, ack, err, 4, dreq == nullptr);
    if (dreq) {
        run("bar_1poller", dreq, ack, err, 1, false);
        run("bar_4pollers", dreq, ack, err, 4, true);
    }
    printf("}\n");
    return 0;
}
