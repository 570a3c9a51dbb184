// valu_rate.hip -- issue cost of the VALU instructions the tally's capacity
// step can use, on gfx950 (diagnostic only): shader cycles (s_memtime) per
// wave64 instruction over a dependent-free unrolled loop, 1 and 2 waves per
// SIMD. Prints one JSON line.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
            std::exit(1);                                                      \
        }                                                                      \
    } while (0)

constexpr int kIters = 256;

template <int OP>
__global__ void rate_kernel(const unsigned* __restrict__ in, unsigned* __restrict__ out, unsigned long long* cyc) {
    unsigned a0 = in[threadIdx.x], a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
             a7 = a0 + 7;
    const unsigned m = in[1024];
    double d0 = a0, d1 = a1, d2 = a2, d3 = a3, d4 = a4, d5 = a5, d6 = a6, d7 = a7;
    const double r = 1.0 / (double)(m | 1);
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < kIters; ++i) {
        if (OP == 0) {  // v_add_u32
            a0 += m; a1 += m; a2 += m; a3 += m; a4 += m; a5 += m; a6 += m; a7 += m;
        } else if (OP == 1) {  // v_mul_hi_u32
            a0 = __umulhi(a0, m); a1 = __umulhi(a1, m); a2 = __umulhi(a2, m); a3 = __umulhi(a3, m);
            a4 = __umulhi(a4, m); a5 = __umulhi(a5, m); a6 = __umulhi(a6, m); a7 = __umulhi(a7, m);
        } else if (OP == 2) {  // v_mul_f64
            d0 *= r; d1 *= r; d2 *= r; d3 *= r; d4 *= r; d5 *= r; d6 *= r; d7 *= r;
        } else if (OP == 3) {  // v_cvt_f64_u32 + v_cvt_u32_f64 pairs
            a0 = (unsigned)(double)a0 + m; a1 = (unsigned)(double)a1 + m; a2 = (unsigned)(double)a2 + m;
            a3 = (unsigned)(double)a3 + m; a4 = (unsigned)(double)a4 + m; a5 = (unsigned)(double)a5 + m;
            a6 = (unsigned)(double)a6 + m; a7 = (unsigned)(double)a7 + m;
        } else if (OP == 4) {  // v_mul_hi_u32_u24
            a0 = a0;
        } else if (OP == 5) {  // v_mul_lo_u32
            a0 *= m; a1 *= m; a2 *= m; a3 *= m; a4 *= m; a5 *= m; a6 *= m; a7 *= m;
        } else if (OP == 6) {  // v_cvt_f32_u32 + v_mul_f32 + v_cvt_u32_f32
            const float rf = (float)r;
            a0 = (unsigned)((float)a0 * rf) + m; a1 = (unsigned)((float)a1 * rf) + m;
            a2 = (unsigned)((float)a2 * rf) + m; a3 = (unsigned)((float)a3 * rf) + m;
            a4 = (unsigned)((float)a4 * rf) + m; a5 = (unsigned)((float)a5 * rf) + m;
            a6 = (unsigned)((float)a6 * rf) + m; a7 = (unsigned)((float)a7 * rf) + m;
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] =
        a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (unsigned)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7);
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    unsigned *in, *out;
    unsigned long long* cyc;
    CK(hipMalloc(&in, 4096 * 4));
    CK(hipMalloc(&out, 1 << 24));
    CK(hipMalloc(&cyc, 1 << 16));
    CK(hipMemset(in, 7, 4096 * 4));
    const char* names[] = {"v_add_u32", "v_mul_hi_u32", "v_mul_f64", "cvt_f64_u32+cvt_u32_f64+add", "unused",
                           "v_mul_lo_u32", "cvt_f32_u32+mul_f32+cvt_u32_f32+add"};
    const int per_iter[] = {8, 8, 8, 24, 0, 8, 32};
    std::printf("{\"probe\": \"valu_rate\", \"unit\": \"shader cycles per wave64 instruction\", \"results\": [");
    bool first = true;
    for (int op : {0, 1, 2, 3, 5, 6}) {
        for (int wps : {1, 2}) {
            // one workgroup of 64*4*wps threads per CU: wps waves on each SIMD
            const int threads = 256 * wps;
            unsigned long long h[256];
            auto run = [&]() {
                switch (op) {
                    case 0: hipLaunchKernelGGL(rate_kernel<0>, dim3(256), dim3(threads), 0, 0, in, out, cyc); break;
                    case 1: hipLaunchKernelGGL(rate_kernel<1>, dim3(256), dim3(threads), 0, 0, in, out, cyc); break;
                    case 2: hipLaunchKernelGGL(rate_kernel<2>, dim3(256), dim3(threads), 0, 0, in, out, cyc); break;
                    case 3: hipLaunchKernelGGL(rate_kernel<3>, dim3(256), dim3(threads), 0, 0, in, out, cyc); break;
                    case 5: hipLaunchKernelGGL(rate_kernel<5>, dim3(256), dim3(threads), 0, 0, in, out, cyc); break;
                    case 6: hipLaunchKernelGGL(rate_kernel<6>, dim3(256), dim3(threads), 0, 0, in, out, cyc); break;
                }
            };
            run();
            run();
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost));
            double s = 0;
            for (int i = 0; i < 256; ++i) s += (double)h[i];
            const double per = s / 256 / kIters / per_iter[op];
            std::printf("%s{\"op\": \"%s\", \"waves_per_simd\": %d, \"cycles\": %.2f}", first ? "" : ", ", names[op], wps,
                        per);
            first = false;
        }
    }
    std::printf("]}\n");
    return 0;
}
