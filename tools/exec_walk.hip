// exec_walk.hip -- the exec-lane cost (exec_ops.hip) on a latency-bound loop shaped like the
// render kernel's node step: per step two ds_read_b128 at an address the previous step chose,
// 3 packed subtractions, 3 packed products, 10 min/max, a compare and a select of the next
// address.  4 waves per SIMD (1024-thread workgroups, 64 KB of LDS nodes), active lanes
// 64 / 32 / 16 / 9 / 8 / 4 / 1; prints ns per step per wave and the in-kernel clock.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const f4v lds_f4;

__device__ __forceinline__ float vmin(float a, float b) { float r; asm volatile("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }
__device__ __forceinline__ float vmax(float a, float b) { float r; asm volatile("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }

constexpr int NODES = 2048;   // 2048 x 32 B = 64 KB

__global__ void __launch_bounds__(1024, 2) walk(const float4* __restrict__ g, int steps, unsigned long long mask,
                                                unsigned* out, unsigned long long* stamps) {
    extern __shared__ float4 s[];
    for (int k = threadIdx.x; k < 2 * NODES; k += 1024) s[k] = g[k];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    uint32_t nx = (uint32_t)((threadIdx.x * 37) % NODES) * 32u;
    const float ox = 0.1f * lane, oy = 0.2f, oz = -0.3f;
    const float ix = 1.3f, iy = -0.7f, iz = 2.1f;
    if ((mask >> lane) & 1ull) {
        for (int i = 0; i < steps; i++) {
            const lds_f4* p = (const lds_f4*)(uintptr_t)nx;
            const f4v a = p[0], b = p[1];
            const f2v tx = (f2v{a.x, a.y} - f2v{ox, ox}) * f2v{ix, ix};
            const f2v ty = (f2v{a.z, a.w} - f2v{oy, oy}) * f2v{iy, iy};
            const f2v tz = (f2v{b.x, b.y} - f2v{oz, oz}) * f2v{iz, iz};
            float lo = vmax(vmax(vmax(0.001f, vmin(tx.x, tx.y)), vmin(ty.x, ty.y)), vmin(tz.x, tz.y));
            float hi = vmin(vmin(vmin(1e30f, vmax(tx.x, tx.y)), vmax(ty.x, ty.y)), vmax(tz.x, tz.y));
            nx = __float_as_uint(!(hi <= lo) ? b.z : b.w);
        }
    }
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
        stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
    if (nx == 0xFFFFFFFFu) out[blockIdx.x] = nx;
}

// the same step with the node halves swizzled across LDS banks: node k's two float4 are stored
// (h0, h1) for even k and (h1, h0) for odd k, so each of the step's two ds_read_b128 reads 16 B at
// a 32-B stride offset by 16 B on every other node (both bank halves) -- one address per half
__global__ void __launch_bounds__(1024, 2) walk_sw(const float4* __restrict__ g, int steps, unsigned long long mask,
                                                   unsigned* out, unsigned long long* stamps) {
    extern __shared__ float4 s[];
    for (int k = threadIdx.x; k < 2 * NODES; k += 1024) s[k ^ ((k >> 1) & 1)] = g[k];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    uint32_t nx = (uint32_t)((threadIdx.x * 37) % NODES) * 32u;
    const float ox = 0.1f * lane, oy = 0.2f, oz = -0.3f;
    const float ix = 1.3f, iy = -0.7f, iz = 2.1f;
    if ((mask >> lane) & 1ull) {
        for (int i = 0; i < steps; i++) {
            const uint32_t sw = (nx >> 1) & 16u;
            const f4v a = *(const lds_f4*)(uintptr_t)(nx + sw), b = *(const lds_f4*)(uintptr_t)(nx + (16u - sw));
            const f2v tx = (f2v{a.x, a.y} - f2v{ox, ox}) * f2v{ix, ix};
            const f2v ty = (f2v{a.z, a.w} - f2v{oy, oy}) * f2v{iy, iy};
            const f2v tz = (f2v{b.x, b.y} - f2v{oz, oz}) * f2v{iz, iz};
            float lo = vmax(vmax(vmax(0.001f, vmin(tx.x, tx.y)), vmin(ty.x, ty.y)), vmin(tz.x, tz.y));
            float hi = vmin(vmin(vmin(1e30f, vmax(tx.x, tx.y)), vmax(ty.x, ty.y)), vmax(tz.x, tz.y));
            nx = __float_as_uint(!(hi <= lo) ? b.z : b.w);
        }
    }
    if (nx == 0xFFFFFFFFu) out[blockIdx.x] = nx;
}

// the same step for two independent walks per lane (ILP 2)
__global__ void __launch_bounds__(1024, 1) walk2(const float4* __restrict__ g, int steps, unsigned long long mask,
                                                 unsigned* out, unsigned long long* stamps) {
    extern __shared__ float4 s[];
    for (int k = threadIdx.x; k < 2 * NODES; k += 1024) s[k] = g[k];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    uint32_t nx = (uint32_t)((threadIdx.x * 37) % NODES) * 32u, ny = (uint32_t)((threadIdx.x * 53 + 7) % NODES) * 32u;
    const float ox = 0.1f * lane, oy = 0.2f, oz = -0.3f;
    const float ix = 1.3f, iy = -0.7f, iz = 2.1f;
    const float px = -0.1f * lane, py = 0.4f, pz = 0.3f;
    const float jx = -0.8f, jy = 1.7f, jz = 0.9f;
    if ((mask >> lane) & 1ull) {
        for (int i = 0; i < steps / 2; i++) {
            const lds_f4* p = (const lds_f4*)(uintptr_t)nx;
            const lds_f4* q = (const lds_f4*)(uintptr_t)ny;
            const f4v a = p[0], b = p[1], c = q[0], e = q[1];
            const f2v tx = (f2v{a.x, a.y} - f2v{ox, ox}) * f2v{ix, ix};
            const f2v ty = (f2v{a.z, a.w} - f2v{oy, oy}) * f2v{iy, iy};
            const f2v tz = (f2v{b.x, b.y} - f2v{oz, oz}) * f2v{iz, iz};
            const f2v ux = (f2v{c.x, c.y} - f2v{px, px}) * f2v{jx, jx};
            const f2v uy = (f2v{c.z, c.w} - f2v{py, py}) * f2v{jy, jy};
            const f2v uz = (f2v{e.x, e.y} - f2v{pz, pz}) * f2v{jz, jz};
            float lo = vmax(vmax(vmax(0.001f, vmin(tx.x, tx.y)), vmin(ty.x, ty.y)), vmin(tz.x, tz.y));
            float hi = vmin(vmin(vmin(1e30f, vmax(tx.x, tx.y)), vmax(ty.x, ty.y)), vmax(tz.x, tz.y));
            float lo2 = vmax(vmax(vmax(0.001f, vmin(ux.x, ux.y)), vmin(uy.x, uy.y)), vmin(uz.x, uz.y));
            float hi2 = vmin(vmin(vmin(1e30f, vmax(ux.x, ux.y)), vmax(uy.x, uy.y)), vmax(uz.x, uz.y));
            nx = __float_as_uint(!(hi <= lo) ? b.z : b.w);
            ny = __float_as_uint(!(hi2 <= lo2) ? e.z : e.w);
        }
    }
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
        stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
    if ((nx ^ ny) == 0xFFFFFFFFu) out[blockIdx.x] = nx;
}

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
            return 1;                                                            \
        }                                                                        \
    } while (0)

int main(int argc, char** argv) {
    const int steps = argc > 1 ? atoi(argv[1]) : 4000;
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    // random boxes, successors pointing anywhere in the node array (byte offsets)
    float4* h = (float4*)malloc(sizeof(float4) * 2 * NODES);
    srand(7);
    auto rf = []() { return (float)rand() / RAND_MAX; };
    for (int k = 0; k < NODES; k++) {
        float x = rf() * 4 - 2, y = rf() * 4 - 2, z = rf() * 4 - 2, e = rf();
        h[2 * k] = make_float4(x, x + e, y, y + e);
        uint32_t s1 = (uint32_t)(rand() % NODES) * 32u, s2 = (uint32_t)(rand() % NODES) * 32u;
        float f1, f2;
        std::memcpy(&f1, &s1, 4);
        std::memcpy(&f2, &s2, 4);
        h[2 * k + 1] = make_float4(z, z + e, f1, f2);
    }
    float4* g = nullptr;
    unsigned* out = nullptr;
    unsigned long long* stamps = nullptr;
    CK(hipMalloc(&g, sizeof(float4) * 2 * NODES));
    CK(hipMemcpy(g, h, sizeof(float4) * 2 * NODES, hipMemcpyHostToDevice));
    CK(hipMalloc(&out, sizeof(unsigned) * cus));
    CK(hipMalloc(&stamps, sizeof(unsigned long long) * 2 * cus));
    unsigned long long* hs = (unsigned long long*)malloc(sizeof(unsigned long long) * 2 * cus);
    const size_t lds = sizeof(float4) * 2 * NODES;
    CK(hipFuncSetAttribute((const void*)walk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(walk, dim3(cus), dim3(1024), lds, 0, g, steps / 8, ~0ull, out, stamps);
    CK(hipDeviceSynchronize());
    CK(hipFuncSetAttribute((const void*)walk2, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    {
        // node steps per wave: one walk per lane vs two walks per lane (same total steps per lane)
        hipEvent_t a0, a1;
        CK(hipEventCreate(&a0));
        CK(hipEventCreate(&a1));
        for (int mode = 0; mode < 4; mode++) {
            float best = 1e30f;
            const unsigned long long msk = mode < 2 ? ~0ull : 0xFFFFFFFFull;
            for (int rep = 0; rep < 3; rep++) {
                CK(hipEventRecord(a0, 0));
                if (mode % 2 == 0)
                    hipLaunchKernelGGL(walk, dim3(cus), dim3(1024), lds, 0, g, steps, msk, out, stamps);
                else
                    hipLaunchKernelGGL(walk2, dim3(cus), dim3(1024), lds, 0, g, steps, msk, out, stamps);
                CK(hipEventRecord(a1, 0));
                CK(hipEventSynchronize(a1));
                float ms_ = 0;
                CK(hipEventElapsedTime(&ms_, a0, a1));
                if (ms_ < best) best = ms_;
            }
            printf("{\"walks_per_lane\": %d, \"lanes\": %d, \"steps_per_lane\": %d, \"kernel_ms\": %.4f}\n",
                   mode % 2 + 1, mode < 2 ? 64 : 32, steps, best);
            fflush(stdout);
        }
        CK(hipFuncSetAttribute((const void*)walk_sw, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        for (int mode = 0; mode < 6; mode++) {
            float best = 1e30f;
            const unsigned long long msk = (mode % 3 == 0) ? ~0ull : (mode % 3 == 1) ? 0xFFFFFFFFull : 0xFFFFull;
            for (int rep = 0; rep < 3; rep++) {
                CK(hipEventRecord(a0, 0));
                if (mode < 3)
                    hipLaunchKernelGGL(walk, dim3(cus), dim3(1024), lds, 0, g, steps, msk, out, stamps);
                else
                    hipLaunchKernelGGL(walk_sw, dim3(cus), dim3(1024), lds, 0, g, steps, msk, out, stamps);
                CK(hipEventRecord(a1, 0));
                CK(hipEventSynchronize(a1));
                float ms_ = 0;
                CK(hipEventElapsedTime(&ms_, a0, a1));
                if (ms_ < best) best = ms_;
            }
            printf("{\"swizzled\": %d, \"lanes\": %d, \"kernel_ms\": %.4f}\n", mode >= 3,
                   (mode % 3 == 0) ? 64 : (mode % 3 == 1) ? 32 : 16, best);
            fflush(stdout);
        }
        // 8 waves per SIMD: two 1024-thread workgroups per CU (2 x 64 KB of LDS), the same steps
        for (int mode = 0; mode < 2; mode++) {
            float best = 1e30f;
            const unsigned long long msk = mode == 0 ? ~0ull : 0xFFFFFFFFull;
            for (int rep = 0; rep < 3; rep++) {
                CK(hipEventRecord(a0, 0));
                hipLaunchKernelGGL(walk, dim3(2 * cus), dim3(1024), lds, 0, g, steps, msk, out, stamps);
                CK(hipEventRecord(a1, 0));
                CK(hipEventSynchronize(a1));
                float ms_ = 0;
                CK(hipEventElapsedTime(&ms_, a0, a1));
                if (ms_ < best) best = ms_;
            }
            printf("{\"waves_per_simd\": 8, \"lanes\": %d, \"steps_per_lane\": %d, \"kernel_ms\": %.4f, "
                   "\"note\": \"twice the waves of the rows above\"}\n", mode == 0 ? 64 : 32, steps, best);
            fflush(stdout);
        }
    }
    struct M { const char* name; unsigned long long mask; };
    const M ms[] = {{"64", ~0ull}, {"32", 0xFFFFFFFFull}, {"16", 0xFFFFull}, {"9", 0x1FFull}, {"8", 0xFFull},
                    {"4", 0xFull}, {"1", 1ull}, {"64again", ~0ull}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (const M& m : ms) {
        float best = 1e30f;
        for (int rep = 0; rep < 3; rep++) {
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(walk, dim3(cus), dim3(1024), lds, 0, g, steps, m.mask, out, stamps);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms_ = 0;
            CK(hipEventElapsedTime(&ms_, e0, e1));
            if (ms_ < best) best = ms_;
        }
        CK(hipMemcpy(hs, stamps, sizeof(unsigned long long) * 2 * cus, hipMemcpyDeviceToHost));
        double mhz = 0;
        for (int b = 0; b < cus; b++) mhz += hs[2 * b + 1] ? 100.0 * (double)hs[2 * b] / (double)hs[2 * b + 1] : 0.0;
        mhz /= cus;
        printf("{\"lanes\": \"%s\", \"kernel_ms\": %.4f, \"clock_mhz\": %.0f, \"cycles_per_step_per_wave\": %.1f}\n", m.name,
               best, mhz, best * 1e-3 * mhz * 1e6 / steps);
        fflush(stdout);
    }
    return 0;
}
