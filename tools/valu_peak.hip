// valu_peak.hip — the VALU issue ceiling the render kernel's roofline is priced
// against (bench.py roofline.bound "valu").  MI355X_MICROARCH.md:54,473 give a
// wave64 v_fma_f32 2 cycles per SIMD-32 (4 for one wave alone); this measures
// it: every CU runs W waves per SIMD, each wave issues a known number of
// independent v_fma_f32 (inline asm, so the count is exact), and the kernel's
// wall time and its in-kernel clock (s_memtime / s_memrealtime at 100 MHz) give
// wave-instructions per second and cycles per wave-instruction per SIMD.
//
// Usage: valu_peak [iters]   -> one JSON line per waves-per-SIMD setting.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define FMA8(a, b, c, d, e, f, g, h)                                                                      \
    asm volatile(                                                                                        \
        "v_fma_f32 %0, %0, %8, %9\n\tv_fma_f32 %1, %1, %8, %9\n\tv_fma_f32 %2, %2, %8, %9\n\t"           \
        "v_fma_f32 %3, %3, %8, %9\n\tv_fma_f32 %4, %4, %8, %9\n\tv_fma_f32 %5, %5, %8, %9\n\t"           \
        "v_fma_f32 %6, %6, %8, %9\n\tv_fma_f32 %7, %7, %8, %9"                                             \
        : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h)                       \
        : "v"(m), "v"(k))

constexpr int kFmaPerIter = 32;

template <int BLOCK, int MINW>
__global__ void __launch_bounds__(BLOCK, MINW) valu_fma(float* out, int iters, unsigned long long* stamps) {
    float m = 0.999f + 1e-7f * threadIdx.x, k = 1e-3f;
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
          a7 = a0 + 7;
    float b0 = a0 * 2, b1 = b0 + 1, b2 = b0 + 2, b3 = b0 + 3, b4 = b0 + 4, b5 = b0 + 5, b6 = b0 + 6, b7 = b0 + 7;
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (int i = 0; i < iters; i++) {
        FMA8(a0, a1, a2, a3, a4, a5, a6, a7);
        FMA8(b0, b1, b2, b3, b4, b5, b6, b7);
        FMA8(a0, a1, a2, a3, a4, a5, a6, a7);
        FMA8(b0, b1, b2, b3, b4, b5, b6, b7);
    }
    if (threadIdx.x == 0) {
        unsigned long long t1 = __builtin_amdgcn_s_memtime();
        unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
        // stamps: their own buffer (never an output value)
        stamps[2 * blockIdx.x] = t1 - t0;
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
    float s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + b0 + b1 + b2 + b3 + b4 + b5 + b6 + b7;
    if (s == 12345.678f) out[blockIdx.x * BLOCK + threadIdx.x] = s;   // keeps the chains live
}

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
            return 1;                                                            \
        }                                                                        \
    } while (0)

template <int BLOCK, int MINW>
int run(int wps, int iters, int cus, float* out, unsigned long long* stamps) {
    // wps waves per SIMD = wps * 4 waves per CU = (wps * 256 / BLOCK) workgroups per CU
    const int per_cu = wps * 256 / BLOCK;
    const int grid = cus * per_cu;
    auto kern = valu_fma<BLOCK, MINW>;
    int occ = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, BLOCK, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(BLOCK), 0, 0, out, iters / 8, stamps);   // warm-up (clock ramp)
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    double clk_mhz = 0.0;
    for (int rep = 0; rep < 5; rep++) {
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(kern, dim3(grid), dim3(BLOCK), 0, 0, out, iters, stamps);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) {
            best = ms;
            unsigned long long* h = (unsigned long long*)malloc(sizeof(unsigned long long) * 2 * grid);
            CK(hipMemcpy(h, stamps, sizeof(unsigned long long) * 2 * grid, hipMemcpyDeviceToHost));
            // median over workgroups of (shader cycles / 100 MHz ticks)
            double* r = (double*)malloc(sizeof(double) * grid);
            for (int b = 0; b < grid; b++) r[b] = h[2 * b + 1] ? 100.0 * (double)h[2 * b] / (double)h[2 * b + 1] : 0.0;
            for (int i = 1; i < grid; i++)
                for (int j = i; j > 0 && r[j - 1] > r[j]; j--) {
                    double t = r[j]; r[j] = r[j - 1]; r[j - 1] = t;
                }
            clk_mhz = r[grid / 2];
            free(r);
            free(h);
        }
    }
    const double waves = (double)grid * (BLOCK / 64);
    const double insts = waves * (double)iters * kFmaPerIter;
    const double s = best * 1e-3;
    const double rate = insts / s;                 // wave-instructions per second, whole chip
    const double simds = (double)cus * 4.0;
    const double cyc_meas = simds * clk_mhz * 1e6 * s / insts;   // cycles per wave-instruction per SIMD
    const double cyc_24 = simds * 2.4e9 * s / insts;
    printf("{\"waves_per_simd\": %d, \"block\": %d, \"grid\": %d, \"occupancy_blocks_per_cu\": %d, \"cus\": %d, "
           "\"v_fma_f32_per_wave\": %.0f, \"wave_instructions\": %.6e, \"kernel_ms\": %.4f, "
           "\"wave_inst_per_s\": %.6e, \"clock_mhz_in_kernel\": %.1f, \"cycles_per_wave_inst_per_simd\": %.4f, "
           "\"cycles_per_wave_inst_per_simd_at_2400mhz\": %.4f}\n",
           wps, BLOCK, grid, occ, cus, (double)iters * kFmaPerIter, insts, best, rate, clk_mhz, cyc_meas, cyc_24);
    fflush(stdout);
    return 0;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20000;
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    float* out = nullptr;
    unsigned long long* stamps = nullptr;
    CK(hipMalloc(&out, sizeof(float) * (size_t)cus * 2048));
    CK(hipMalloc(&stamps, sizeof(unsigned long long) * 2 * (size_t)cus * 32));
    // 1 wave per SIMD (the guide's "one wave alone" row), 2 and 4 (the render kernel's occupancy)
    if (run<256, 1>(1, iters, cus, out, stamps)) return 1;
    if (run<512, 2>(2, iters, cus, out, stamps)) return 1;
    if (run<512, 4>(4, iters, cus, out, stamps)) return 1;
    CK(hipFree(out));
    CK(hipFree(stamps));
    return 0;
}
