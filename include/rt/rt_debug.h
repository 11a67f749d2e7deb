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
 * kernel walks (rt_device.h RT_LINK_*): the threaded nodes placed breadth-first,
 * two float4 each (box, hit / miss successor byte addresses), then the leaves'
 * (types | next address << 8, prims) as uint2.  *n_f4 = its float4 count, 0 when
 * there is no BVH. */
int rt_debug_link_nodes(const void* bvh, size_t nbytes, void* out, size_t out_cap, int* n_f4);
/* The same with the box pre-test nodes (option box_vnodes): vbox = 6 floats per box (its
 * pre-test bounds: xmin, xmax, ymin, ymax, zmin, zmax); *n_nodes = tree + pre-test nodes. */
int rt_debug_link_nodes_vbox(const void* bvh, size_t nbytes, const float* vbox, int n_box, void* out,
                             size_t out_cap, int* n_f4, int* n_nodes);
/* The link-format nodes of `bvh` as the walk of a context uses them: with rebuild != 0 the inner
 * nodes rebuilt over the leaf sequence (option rebuild, rt_capi.hip rebuild_inner), then the node
 * collapse of option collapse (plan_collapse) planned for camera `cam` (rt_camera_ubo, 28
 * floats) and a width x height image; drop (may be NULL) gets one byte per threaded node of that
 * tree (1 = left out), *n_dropped their count.  Host-side, no device needed
 * (tests/test_link_nodes.py replays the walk). */
int rt_debug_collapse_links(const void* bvh, size_t nbytes, const float cam[28], int width, int height, int rebuild,
                            void* out, size_t out_cap, int* n_f4, unsigned char* drop, size_t drop_cap,
                            int* n_dropped);

/* Host-only: the packed Perlin table rt_upload_texture keeps beside an R32F 6 x 256 texture
 * whose perm columns (3..5) hold whole numbers 0..255: 256 float4 (ranvec x, y, z; the three
 * perm entries as bytes 0, 1, 2 of the fourth word).  Returns 1 (table written to out when
 * out != NULL), 0 when the texture does not qualify (the kernel then reads it as uploaded). */
int rt_debug_perlin_pack(const float* texels, int w, int h, void* out, size_t out_cap);

/* Host-only: per mille of a reference BVH upload's leaves that hold two spheres; rt_render
 * takes the sphere-pair kernels at >= 500 (and when the boxes are not all canonical). */
int rt_debug_sphere_pair_leaves(const void* bvh, size_t nbytes, int* permille);

/* Host-only: rt_read_image's device de-interleave (deinterleave_kernel) with the same
 * row indexing (rt_device.h rt_gathered_row), on the host (tests compare it with
 * rt_deinterleave_rows). */
int rt_debug_deinterleave(const float* gathered, int width, int height, int world, int stripe_rows, float* out);

/* Host-only: the boxes' 48-byte records rt_upload_buffer(RT_BIND_BOXES) builds
 * (rt_capi.hip box_record: 3 float4 per box; float4[2].y = 1 for a compact record,
 * whose faces the kernel rebuilds from it) and how many are compact. */
int rt_debug_box_records(const void* boxes, size_t nbytes, void* out, size_t out_cap, int* n_compact);

/* Diagnostic build of the render kernel with wave-level region timers and
 * active-lane counters (never used for timed numbers).  enable=1 switches the
 * context to it and zeroes the counters; enable=2 also records the leaf census
 * (one record per wave leaf round: start cycle, cycles, workgroup | wave << 16 |
 * walking lanes << 24, slot 0's and slot 1's lanes per prim type as bytes: sphere,
 * quad, medium, box); read returns n <= 128 counters.  read_census copies the first
 * device's census (per resident wave its record count, then *cap records of 5 words
 * per wave); out may be NULL to query *needed (words), *waves and *cap.
 * The stats kernels exist only in the A/B build (librtamd_ab.so, built with
 * -DRT_AB_KNOBS); the release library returns RT_ERR_STATE. */
struct rt_ctx;
int rt_debug_enable_stats(struct rt_ctx* ctx, int enable);
int rt_debug_read_stats(struct rt_ctx* ctx, unsigned long long* out, int n);
int rt_debug_read_census(struct rt_ctx* ctx, unsigned int* out, size_t words, size_t* needed, int* waves, int* cap);
/* The stats twin's node-hit count (A/B experiments on the collapse plan, tools/collapse_hits_ab.py):
 * count_node_hits(ctx, 1) zeroes and arms it (0 frees it); read_node_hits gives, per link node of
 * the last launch's layout, the box tests that hit, then the walks begun at the root
 * (*n_out = nodes + 1 words; out may be NULL); set_collapse_hits plans the collapse from such counts
 * (per node of the walk's tree, breadth-first, as read with collapse and spine off) instead of the
 * camera grid (n = 0: the grid again). */
int rt_debug_count_node_hits(struct rt_ctx* ctx, int on);
int rt_debug_read_node_hits(struct rt_ctx* ctx, unsigned int* out, size_t words, size_t* n_out);
int rt_debug_set_collapse_hits(struct rt_ctx* ctx, const unsigned int* hits, size_t n, unsigned long long walks);

/* Number of visible HIP devices (0 when none). */
int rt_debug_device_count(void);

/* 1 when this library is the A/B build (-DRT_AB_KNOBS: kernel variants, stats
 * twins, non-exact ablations and the RT_* environment knobs), 0 for the release
 * library, whose output depends on nothing but its inputs. */
int rt_debug_ab_build(void);

/* Per-context options for tests and A/B runs, set by explicit calls (never read
 * from the environment by the release library).  Every option below 100 changes
 * only how the work is laid out or which exact form of a test runs, never a bit
 * of the image (tests/ compare each against the default).  Options >= 100 exist
 * in the A/B build only (the release library returns RT_ERR_INVALID_ARG). */
enum {
    RT_OPTION_BOX_PRETEST = 1,          /* box bounds pre-test (1)                          */
    RT_OPTION_FASTDIV = 2,              /* shared-reciprocal division where exact (1)       */
    RT_OPTION_SPH_LDS = 3,              /* leaf records staged in LDS (1)                   */
    RT_OPTION_BIG_WG = 4,               /* 1024-thread workgroups when records fit (1)      */
    RT_OPTION_CHUNK_TARGET = 5,         /* ordered units per resident wave; 0 = one per tile (16) */
    RT_OPTION_STAGED_CHUNK_TARGET = 6,  /* staged units per resident wave (48)              */
    RT_OPTION_STAGE_TILES = 7,          /* stage chunks below this many tiles per wave (2^20) */
    RT_OPTION_SM_BATCH = 8,             /* shading batch, lanes (64)                        */
    RT_OPTION_SM_FRAC = 9,              /* shading batch, 64ths of the walking lanes (0 =   
                                           by kernel: 50 compact-box kernels, else 56)      */
    RT_OPTION_WALK_FRAC = 10,           /* partial node walks, 64ths (0: by BVH size)       */
    RT_OPTION_WATCHDOG_MS = 11,         /* a wave that stores no sample for this long sets
                                           the fault word and leaves (120000); 0 = at once  */
    RT_OPTION_CHUNK_WAIT_MS = 12,       /* ordered-chunk wait bound (30000); 0 = at once    */
    RT_OPTION_LDS_NODE_CAP = 13,        /* bytes of BVH nodes staged in LDS; the rest is
                                           read from global memory (0 = as many as fit)     */
    RT_OPTION_COMPACT_BOXES = 14,       /* canonical boxes from 48-byte LDS records (1)     */
    RT_OPTION_SPINE = 15,               /* walks start past the root's right spine when its
                                           boxes surely hold the ray's origin (1)           */
    RT_OPTION_TL_LEAF_LDS = 16,         /* two-level walk: leaf records in LDS beside the
                                           top levels when they take <= half of it (1)      */
    RT_OPTION_PERLIN_PACKED = 17,       /* Perlin table staged as 256 float4 with packed
                                           perm bytes when its entries allow it (1)         */
    RT_OPTION_SPARSE_STAGE = 18,        /* staged chunks write only colours that are not
                                           exactly zero, plus a flag byte per sample (1)    */
    RT_OPTION_SPHERE_PAIRS = 19,        /* kernels testing a two-sphere leaf's spheres at
                                           once, when most leaves are such pairs (1); 2:
                                           always, compact-box kernels included            */
    RT_OPTION_LEAF_PREFETCH = 20,       /* compact-box kernels: each leaf slot's record loaded
                                           before the prim-type blocks when spheres, boxes
                                           and media are all staged in LDS (1)              */
    RT_OPTION_TL_SMALL_LDS = 21,        /* two-level walk: room is reserved beside the top
                                           levels for the sphere / compact box records that
                                           take at most 1/16 of it, and each table is staged
                                           whenever it fits after the nodes (1); 0: neither */
    RT_OPTION_SHADE_LDS = 22,           /* shading tables in LDS: sphere and compact box
                                           materials, texture descriptors, small texture
                                           slots (1)                                        */
    RT_OPTION_BOX_VNODES = 23,          /* compact-box kernels: each all-box leaf's box bounds
                                           pre-tests as nodes of the walk, the leaf stage
                                           testing only the boxes they pass (1)            */
    RT_OPTION_ZERO_DIR_END = 24,        /* a path whose next direction is vec3(0) (the no-
                                           light branch) ends in its shading pass with the
                                           miss colour its next bounce would give (1)       */
    RT_OPTION_COLLAPSE = 25,            /* the link walk leaves out the inner nodes whose
                                           tests a grid of camera rays says cost more than
                                           they save (rt_capi.hip plan_collapse) (1)        */
    RT_OPTION_REBUILD = 26,             /* the link walk's inner nodes rebuilt over the
                                           reference's leaf sequence (joined boxes: the same
                                           leaves, order and ray_t; rt_capi.hip
                                           rebuild_inner): 1 greedy surface-area splits,
                                           2 the least summed inner-box area (default); 0 off */
    RT_OPTION_TAIL_CHUNKS = 27,         /* staged launches end with this many one-frame
                                           chunks: the units claimed last are short (only
                                           the grouping of samples into units changes);
                                           -1 (default): 1 above 1024 BVH nodes, else 0  */
    RT_OPTION_KERNEL_VARIANT = 100,     /* A/B build: 0, 37, 30, 61 (+ stats twins)         */
    RT_OPTION_DEBUG_FLAGS = 101         /* A/B build: ablations, NOT exact                  */
};
int rt_debug_set_option(struct rt_ctx* ctx, int option, int value);
int rt_debug_get_option(struct rt_ctx* ctx, int option, int* value);

/* What the last rt_render launched on the context's first device (tests assert
 * that the intended path ran):
 *   out[0] launch shape (0 fast-lds, 1 fast-global, 2 link-lds, 3 meta-lds,
 *          4 meta-global, 5 link two-level: top nodes in LDS, the rest global)
 *   out[1] workgroup size          out[2] shared-reciprocal division on (1/0)
 *   out[3] box pre-test on (1/0)   out[4] dynamic LDS bytes
 *   out[5] BVH nodes staged in LDS out[6] box records: bit 0 compact tests, bit 1 in LDS
 *   out[7] staged chunks (1/0)     out[8] chunks per launch
 *   out[9] spine nodes a walk may skip (0 = off)
 *   out[10] sparse staging (1 = a flag byte per sample, only non-zero colours stored)
 *   out[11] sphere-pair kernel (1 = a two-sphere leaf's spheres tested at once)
 *   out[12] leaf record prefetch  out[13] shading tables in LDS (bits)  out[14] walk threshold
 *   out[15] the BVH the walk ran on: RT_BVH_REFERENCE (0) or RT_BVH_SAH (1, rt_set_bvh_mode)
 *   out[16] box pre-test nodes in the walk (option box_vnodes; 0 = none)
 *   out[17] inner nodes the walk leaves out (option collapse; 0 = none)
 *   out[18] the walk's inner nodes rebuilt over the leaf sequence (option rebuild; 1/0)
 * n <= 20 ints are written; returns RT_ERR_STATE before the first render. */
int rt_debug_last_launch(struct rt_ctx* ctx, int* out, int n);

/* The BVH the link walk of ctx uses, in the reference's node format (rt_bvh_node): the
 * uploaded one, or in RT_BVH_SAH mode the tree rt_set_bvh_mode builds (validated as by
 * rt_render).  out may be NULL to query *nbytes; returns RT_ERR_LIMIT if out_cap is short.
 * Tests feed it to the CPU oracle: the kernel on the SAH tree is bit-exact against the
 * oracle walking the same tree. */
int rt_debug_walk_bvh(struct rt_ctx* ctx, void* out, size_t out_cap, size_t* nbytes);

/* Context-free form of the RT_BVH_SAH build (no device needed): the SAH tree over the prims
 * of `bvh` (the reference's nodes), from the uploaded record bytes of the other bindings.
 * order: 0 the larger child (surface area) first, 1 the smaller first, 2 the child nearer
 * to eye[3] first (rt_set_bvh_mode's, with the camera position); prim_cost: the SAH cost of a
 * prim test in node steps (rt_set_bvh_mode's: 1). */
int rt_debug_build_sah_bvh(const void* spheres, size_t sph_bytes, const void* quads, size_t quad_bytes,
                           const void* media, size_t med_bytes, const void* boxes, size_t box_bytes,
                           const void* bvh, size_t bvh_bytes, int order, const float eye[3],
                           float prim_cost, void* out, size_t out_cap, size_t* nbytes);

#ifdef __cplusplus
}
#endif

#endif
