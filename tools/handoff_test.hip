// handoff_test.hip — checks the wave-to-wave hand-off that the render kernel's
// ordered chunks use (rt_kernel.hip wait_chunk / publish_chunk), in isolation:
// a persistent grid dequeues units (chunk-major: unit = chunk * tiles + tile),
// a unit k > 0 of a tile waits for unit k-1's flag, reads the tile's 64 float4,
// checks they hold k (a stale read shows as a smaller value), busy-works a
// variable time, writes k + 1 and publishes.  Poll / read flavours:
//   mode 0: relaxed agent atomic load poll (sc1), acquire fence, plain loads
//   mode 1: atomic fetch_add(0) poll (agent RMW), acquire fence, plain loads
//   mode 2: mode 1 + data read by relaxed agent atomic loads (sc1)
//   mode 3: mode 1 + data read by system-scope atomic loads (sc0 sc1)
// Every wait is bounded (s_memrealtime); stale reads and timeouts are counted.
// Usage: handoff_test  -> one JSON line per (mode, tiles).
#include <hip/hip_runtime.h>

#include <cstdio>

typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) float gf32;

struct Args {
    int tiles, chunks;
    unsigned* flags;   // per tile
    float4* data;      // tiles * 64
    int* counter;      // [0] next unit
    unsigned* stats;   // [0] stale, [1] timeouts, [2] units
};

template <int MODE>
__global__ void __launch_bounds__(512, 4) handoff(Args A) {
    const int lane = threadIdx.x & 63;
    unsigned stale = 0, timeouts = 0, units = 0;
    const int n_units = A.tiles * A.chunks;
    for (;;) {
        int unit = 0;
        if (lane == 0) unit = atomicAdd(A.counter, 1);
        unit = __shfl(unit, 0);
        if (unit >= n_units) break;
        const int k = unit / A.tiles, tile = unit - k * A.tiles;
        if (k > 0) {
            if (lane == 0) {
                const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                gu32* w = (gu32*)(A.flags + tile);
                for (;;) {
                    unsigned v = MODE == 0 ? __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                           : __hip_atomic_fetch_add(w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (v >= (unsigned)k) break;
                    __builtin_amdgcn_s_sleep(2);
                    if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {   // 0.2 s
                        timeouts++;
                        break;
                    }
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        float4* p = A.data + (size_t)tile * 64 + lane;
        float x;
        if (MODE == 2) x = __hip_atomic_load((gf32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else if (MODE == 3) x = __hip_atomic_load((gf32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        else x = p->x;
        if (x != (float)k) stale++;
        // variable busy work (a few to ~40 us), data-dependent so it is kept
        float acc = x;
        const int n = 2000 + ((tile * 7919 + k * 104729) % 16) * 1000;
        for (int i = 0; i < n; i++) acc = acc * 0.999999f + 1e-7f;
        float4 v = make_float4((float)(k + 1), acc, 0.0f, 0.0f);
        *p = v;
        if (k + 1 < A.chunks) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) __hip_atomic_store((gu32*)(A.flags + tile), (unsigned)(k + 1), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
        }
        units++;
    }
    // lane 0 counts per wave; sum the lanes' stale counts
    for (int o = 32; o > 0; o >>= 1) stale += __shfl_down(stale, o);
    if (lane == 0) {
        atomicAdd(A.stats + 0, stale);
        atomicAdd(A.stats + 1, timeouts);
        atomicAdd(A.stats + 2, units);
    }
}

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
            return 1;                                                            \
        }                                                                        \
    } while (0)

template <int MODE>
int run(int tiles, int chunks, int cus) {
    Args A;
    A.tiles = tiles;
    A.chunks = chunks;
    CK(hipMalloc(&A.flags, sizeof(unsigned) * tiles));
    CK(hipMalloc(&A.data, sizeof(float4) * 64 * (size_t)tiles));
    CK(hipMalloc(&A.counter, 64));
    CK(hipMalloc(&A.stats, 64));
    CK(hipMemset(A.flags, 0, sizeof(unsigned) * tiles));
    CK(hipMemset(A.data, 0, sizeof(float4) * 64 * (size_t)tiles));
    CK(hipMemset(A.counter, 0, 64));
    CK(hipMemset(A.stats, 0, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(handoff<MODE>, dim3(cus * 2), dim3(512), 0, 0, A);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    unsigned st[3];
    CK(hipMemcpy(st, A.stats, sizeof(st), hipMemcpyDeviceToHost));
    printf("{\"mode\": %d, \"tiles\": %d, \"chunks\": %d, \"units\": %u, \"stale_lane_reads\": %u, \"timeouts\": %u, "
           "\"ms\": %.3f}\n", MODE, tiles, chunks, st[2], st[0], st[1], ms);
    fflush(stdout);
    CK(hipFree(A.flags));
    CK(hipFree(A.data));
    CK(hipFree(A.counter));
    CK(hipFree(A.stats));
    return 0;
}

int main() {
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int tile_counts[3] = {15, 1000, 8192};
    for (int t : tile_counts) {
        if (run<0>(t, 32, cus)) return 1;
        if (run<1>(t, 32, cus)) return 1;
        if (run<2>(t, 32, cus)) return 1;
        if (run<3>(t, 32, cus)) return 1;
    }
    return 0;
}
