// exec_lanes.hip -- VALU cost against the number of active lanes (see exec_half.hip): is a
// wave64 v_fma_f32 with few exec lanes slower to ISSUE (SIMD busy longer: more waves per SIMD
// do not help) or only slower to COMPLETE (latency: more independent chains / waves hide it)?
// Sweeps active lanes {64, 32, 16, 8, 1} x independent chains per wave {16, 4, 1} x waves per
// SIMD {1, 4, 8} (≤ 64 VGPRs, so 8 waves fit).  One JSON line per point: cycles per
// wave-instruction per SIMD (in-kernel clock) and per wave.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define FMA1(a) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a) : "v"(m), "v"(k))

template <int CH>
__global__ void __launch_bounds__(256) fma_lanes(float* out, int iters, unsigned long long mask,
                                                 unsigned long long* stamps) {
    const int lane = threadIdx.x & 63;
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    float m = 0.999f + 1e-7f * threadIdx.x, k = 1e-3f;
    float a[16];
#pragma unroll
    for (int c = 0; c < 16; c++) a[c] = threadIdx.x + c;
    if ((mask >> lane) & 1ull) {
        for (int i = 0; i < iters; i++) {
            // 32 instructions per iteration over CH independent chains
#pragma unroll
            for (int j = 0; j < 32; j++) FMA1(a[j % CH]);
        }
    }
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
        stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; c++) s += a[c];
    if (s == 12345.678f) out[blockIdx.x * 256 + threadIdx.x] = s;
}

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
            return 1;                                                            \
        }                                                                        \
    } while (0)

template <int CH>
int run(int cus, int wps, int lanes, int iters, float* out, unsigned long long* stamps, unsigned long long* hst) {
    const unsigned long long mask = lanes >= 64 ? ~0ull : ((1ull << lanes) - 1);
    const int grid = cus * wps;   // 256-thread workgroups: one wave per SIMD each
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int rep = 0; rep < 4; rep++) {
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(fma_lanes<CH>, dim3(grid), dim3(256), 0, 0, out, iters, mask, stamps);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    CK(hipMemcpy(hst, stamps, sizeof(unsigned long long) * 2 * (size_t)grid, hipMemcpyDeviceToHost));
    double mhz = 0;
    for (int b = 0; b < grid; b++) mhz += hst[2 * b + 1] ? 100.0 * (double)hst[2 * b] / (double)hst[2 * b + 1] : 0.0;
    mhz /= grid;
    const double per_wave = (double)iters * 32;
    const double cyc_simd = (double)cus * 4 * mhz * 1e6 * best * 1e-3 / (per_wave * grid * 4);
    printf("{\"lanes\": %d, \"chains\": %d, \"waves_per_simd\": %d, \"kernel_ms\": %.4f, \"clock_mhz\": %.0f, "
           "\"cycles_per_inst_per_simd\": %.3f, \"cycles_per_inst_per_wave\": %.3f}\n",
           lanes, CH, wps, best, mhz, cyc_simd, cyc_simd * wps);
    fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return 0;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 4000;
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    float* out = nullptr;
    unsigned long long* stamps = nullptr;
    CK(hipMalloc(&out, sizeof(float) * (size_t)cus * 8 * 256));
    CK(hipMalloc(&stamps, sizeof(unsigned long long) * 2 * (size_t)cus * 8));
    unsigned long long* hst = (unsigned long long*)malloc(sizeof(unsigned long long) * 2 * (size_t)cus * 8);
    hipLaunchKernelGGL(fma_lanes<16>, dim3(cus * 4), dim3(256), 0, 0, out, iters, ~0ull, stamps);   // clock ramp
    CK(hipDeviceSynchronize());
    const int lanes_list[] = {64, 32, 16, 8, 1};
    const int wps_list[] = {1, 4, 8};
    for (int wps : wps_list)
        for (int lanes : lanes_list) {
            if (run<16>(cus, wps, lanes, iters, out, stamps, hst)) return 1;
            if (run<4>(cus, wps, lanes, iters, out, stamps, hst)) return 1;
            if (run<1>(cus, wps, lanes, iters, out, stamps, hst)) return 1;
        }
    return 0;
}
