// exec_ops.hip -- per instruction kind, the SIMD cycles of a wave64 instruction against the
// number of active exec lanes (exec_lanes.hip found v_fma_f32 at <= 8 lanes ~4.5x dearer
// than at >= 24).  4 waves per SIMD, 16 independent chains, lanes 64 / 32 / 24 / 16 / 12 /
// 10 / 9 / 8 / 4 / 1 (contiguous from lane 0).  Kinds: v_fma_f32, v_add_f32, v_mul_f32,
// v_max_f32, v_cndmask_b32, v_add_u32, v_pk_mul_f32, v_sqrt_f32 (transcendental), v_mov_b32.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

template <int OP>
__device__ __forceinline__ void op1(float& a, float m, float k) {
    if constexpr (OP == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a) : "v"(m), "v"(k));
    if constexpr (OP == 1) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a) : "v"(k));
    if constexpr (OP == 2) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a) : "v"(m));
    if constexpr (OP == 3) asm volatile("v_max_f32 %0, %0, %1" : "+v"(a) : "v"(k));
    if constexpr (OP == 4) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a) : "v"(k));
    if constexpr (OP == 5) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(k));
    if constexpr (OP == 6) asm volatile("v_sqrt_f32 %0, %0" : "+v"(a));
    if constexpr (OP == 7) asm volatile("v_mov_b32 %0, %1" : "=v"(a) : "v"(k));
}

template <int OP>
__global__ void __launch_bounds__(256) ops_lanes(float* out, int iters, unsigned long long mask,
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
#pragma unroll
            for (int j = 0; j < 32; j++) op1<OP>(a[j % 16], m, k);
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

template <int OP>
int run(const char* name, int cus, int lanes, int iters, float* out, unsigned long long* stamps,
        unsigned long long* hst) {
    const unsigned long long mask = lanes >= 64 ? ~0ull : ((1ull << lanes) - 1);
    const int wps = 4, grid = cus * wps;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(ops_lanes<OP>, dim3(grid), dim3(256), 0, 0, out, iters, mask, stamps);
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
    printf("{\"op\": \"%s\", \"lanes\": %d, \"kernel_ms\": %.4f, \"clock_mhz\": %.0f, \"cycles_per_inst_per_simd\": %.3f}\n",
           name, lanes, best, mhz, cyc_simd);
    fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return 0;
}

template <int OP>
int sweep(const char* name, int cus, int iters, float* out, unsigned long long* stamps, unsigned long long* hst) {
    const int lanes_list[] = {64, 32, 24, 16, 12, 10, 9, 8, 4, 1};
    for (int l : lanes_list)
        if (run<OP>(name, cus, l, iters, out, stamps, hst)) return 1;
    return 0;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    float* out = nullptr;
    unsigned long long* stamps = nullptr;
    CK(hipMalloc(&out, sizeof(float) * (size_t)cus * 4 * 256));
    CK(hipMalloc(&stamps, sizeof(unsigned long long) * 2 * (size_t)cus * 4));
    unsigned long long* hst = (unsigned long long*)malloc(sizeof(unsigned long long) * 2 * (size_t)cus * 4);
    hipLaunchKernelGGL(ops_lanes<0>, dim3(cus * 4), dim3(256), 0, 0, out, iters, ~0ull, stamps);   // clock ramp
    CK(hipDeviceSynchronize());
    if (sweep<0>("v_fma_f32", cus, iters, out, stamps, hst)) return 1;
    if (sweep<1>("v_add_f32", cus, iters, out, stamps, hst)) return 1;
    if (sweep<2>("v_mul_f32", cus, iters, out, stamps, hst)) return 1;
    if (sweep<3>("v_max_f32", cus, iters, out, stamps, hst)) return 1;
    if (sweep<4>("v_cndmask_b32", cus, iters, out, stamps, hst)) return 1;
    if (sweep<5>("v_add_u32", cus, iters, out, stamps, hst)) return 1;
    if (sweep<6>("v_sqrt_f32", cus, iters, out, stamps, hst)) return 1;
    if (sweep<7>("v_mov_b32", cus, iters, out, stamps, hst)) return 1;
    return 0;
}
