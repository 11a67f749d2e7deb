/*
 * rt_debug.h — test/diagnostic hooks exported by librtamd.so (not part of the
 * reference's interface; used by tests/ to check device-side pieces directly).
 */
#ifndef RT_DEBUG_H
#define RT_DEBUG_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Evaluate a GLSL built-in of rt_glsl.h on `device` (fn: 0 sin, 1 cos, 2 log,
 * 3 acos, 4 atan2(x, y), 5 fract, 6 sqrt). */
int rt_debug_eval_builtin(int device, int fn, const float* x, const float* y, float* out, int n);

/* Host-only: the threaded-BVH re-layout rt_upload_buffer(RT_BIND_BVH) builds
 * (32-byte rt_dnode records); out may be NULL to query the count. */
int rt_debug_threaded_bvh(const void* nodes, size_t nbytes, void* out, size_t out_cap, int* n_out);

/* Host-only: the exact near-first walk's tables (RT_KERNEL_VARIANT=60) for a
 * reference BVH upload plus its quad and box records: 8 octant layouts of
 * n_per_octant threaded rt_dnode records, one word per solid prim (spheres,
 * then quads, then boxes: reference rank << 16 | reference leaf node) and the
 * media slots in visit order (4 ints each: medium, leaf, tracker, flags).
 * Returns 1 when the walk is usable, 0 when every ray takes the exact walk. */
int rt_debug_fast_tables(const void* bvh, size_t nbytes, const void* quads, size_t qbytes, const void* boxes,
                         size_t bbytes, int n_spheres, void* nodes_out, size_t nodes_cap, int* n_per_octant,
                         unsigned int* info_out, size_t info_cap, int* slots_out, int* n_slots);

/* Host-only: the link-format copy of a reference BVH upload that the default
 * kernel stages in LDS (rt_device.h RT_LINK_*): per threaded node two float4
 * (box, hit / miss successor byte offsets), then the leaves' (types, prims)
 * as uint2.  *n_f4 = its float4 count, 0 when the BVH has too many nodes for
 * 16-bit offsets (the kernel then walks the threaded nodes). */
int rt_debug_link_nodes(const void* bvh, size_t nbytes, void* out, size_t out_cap, int* n_f4);

/* Diagnostic build of the render kernel with wave-level region timers and
 * active-lane counters (never used for timed numbers).  enable=1 switches the
 * context to it and zeroes the counters; read returns n <= 64 counters. */
struct rt_ctx;
int rt_debug_enable_stats(struct rt_ctx* ctx, int enable);
int rt_debug_read_stats(struct rt_ctx* ctx, unsigned long long* out, int n);

/* Number of visible HIP devices (0 when none). */
int rt_debug_device_count(void);

#ifdef __cplusplus
}
#endif

#endif
