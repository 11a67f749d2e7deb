// rt_device.h — device-side scene layout and kernel arguments (internal to
// librtamd.so; not part of the C ABI).
//
// HBM layout per device (all replicated on every device):
//   nodes    : threaded BVH, right-first pre-order (see rt_bvh_thread.cpp), 32 B/node
//   spheres  : rt_sphere[] as uploaded (48 B AoS)
//   quads    : rt_quad[]   as uploaded (80 B AoS)
//   boxes    : rt_box[]    as uploaded (480 B AoS)
//   dquads   : per quad RT_DFACE_F4 float4: plane (n, d), A = (q_a, q_b, u_a, u_b),
//              B = (v_a, v_b, delta, axis case) — the intersection-only face record
//   dboxes   : per box RT_DBOX_F4 float4: the 6 planes, then the 6 (A, B) pairs, then the
//              canonical planes (s_i, w_i) x 6 in 3 float4 (boxes_canon, below), then the
//              box's bounds (xmin, xmax, ymin, ymax), (zmin, zmax, 0, 0) (box_margin)
//   media    : rt_medium[] as uploaded (20 B)
//   lights   : int32 packed ids
//   textures : RGB8 expanded to RGBA8 (4 B/texel, aligned), RGBA8, R32F
//   image    : float4 [padded_local_rows][W], stripe-compacted rows
//   tile_done: uint32 [tiles] chunks published per 8x8 tile (ordered-chunk launches)
//   samples  : float4 [frames][local_rows*W] per-frame colours (staged-chunk launches; sparse: only
//              the colours that are not exactly zero are written)
//   sflags   : uint8 [frames][local_rows*W] sparse staging: 1 where the colour was written
//   wbuf     : float4 [resident waves][2][chunk_frames][64] per-wave sample colours of the
//              units in flight (pooled units, ordered / one-chunk launches)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt/rt_types.h"

#define RT_MAX_FRAMES_PER_LAUNCH 512
#define RT_NODE_END 0xFFFFu
#define RT_DFACE_F4 3    // float4 per dquads record
#define RT_DBOX_F4 23    // float4 per dboxes record
#define RT_BOXC_F4 3     // float4 per compact box record (canonical boxes, box_test_compact)
// LDS per 512-thread workgroup (2 workgroups per CU share 160 KiB): what the
// launch shape stages (at most RT_LDS_DYN_BYTES), then the lanes' running-mean
// slots (RT_LDS_ACC_BYTES), all in the dynamic region (no static LDS)
#define RT_LDS_ACC_BYTES (512 * 16)
#define RT_LDS_DYN_BYTES (80 * 1024 - RT_LDS_ACC_BYTES)   // link nodes + Perlin + media, or variant 61's tree + stacks
// the pooled link-walk kernel as one 1024-thread workgroup per CU (16 waves, 4 per SIMD, the
// same as two workgroups of 512): one copy of the nodes per CU leaves room for the leaf
// tests' sphere and box records.  The release kernels have no static LDS and take all 160 KB; the
// stats twins (A/B library) keep 10 KB for their static counters (RT_LDS_BIG_STATS_BYTES), so their
// plan may leave out the last table (rt_capi.hip: the LDS plan by variant)
#define RT_LDS_BIG_BYTES (160 * 1024)
#define RT_LDS_BIG_STATS_BYTES (150 * 1024)
// the leaf census record (stats twin): start cycle, cycles, workgroup | wave << 16 | walking lanes << 24,
// slot 0's lanes per prim type (sphere, quad, medium, box: a byte each), slot 1's
#define RT_CENSUS_WORDS 5
#define RT_STATS_N 128   // counters rt_debug_read_stats can read (the kernels' ST_N <= 80)
#define RT_LDS_NODE_BYTES (64 * 1024)   // threaded (meta-word) nodes in LDS when they fit

// Threaded BVH node.  Traversal from node 0: on an AABB hit an inner node
// continues at index+1 (its RIGHT child, which the reference visits first
// because it pushes left then right, compute.glsl:259-260); a leaf tests its
// two prims (left then right, compute.glsl:247-256) and continues at `skip`;
// on a miss continue at `skip`.  skip == RT_NODE_END ends the walk.  This
// visits exactly the node sequence of the reference's int stack[64] walk.
struct rt_dnode {
    float xmin, xmax, ymin, ymax, zmin, zmax;
    uint32_t meta;    // bits 0-15 skip, 16-19 left type (0 = inner node), 20-23 right type
    uint32_t prims;   // bits 0-15 left index, 16-31 right index
};
static_assert(sizeof(rt_dnode) == 32, "device node is 32 B");

// Link format of the same nodes (the default walk): word 6 / 7 of a node are the
// successors on a box hit / miss as byte addresses into the node array, so the
// node loop is one select.  A hit leaf's successor leaves the loop:
// RT_LINK_LEAF | leaf ordinal; the end of the walk is RT_LINK_END (both have the
// sign bit set).  Leaf j's record (uint2, after the nodes) is (types | next << 8,
// prims): the prim types in bits 0-7 (left, right), then the address the walk
// continues at after the leaf's tests (its skip node; RT_LINK_NEXT_END = end).
// Nodes are placed breadth-first (the root's level first): when the whole array
// does not fit LDS, the first lds_node_f4 / 2 nodes -- the top levels every ray
// walks -- are staged in LDS and an address at or past them reads global memory
// (the two-level walk).  Up to 65535 nodes (the reference's 16-bit indices).
#define RT_LINK_LEAF 0x80000000u
#define RT_LINK_END 0xFFFFFFFFu
#define RT_LINK_NEXT_END 0xFFFFFFu
#define RT_LINK_MAX_NODES 65535
// In a leaf record's type byte: slot 0's box was pre-tested by a node of the walk (option box_vnodes,
// rt_capi.hip build_links), so the leaf stage skips its bounds pre-test
#define RT_LINK_PRETESTED 8u

struct rt_dtex {
    const void* data;   // RGBA8 (uint32) or R32F
    int w, h;
    int is_float;       // 1 = R32F
    int pad;
};

struct rt_kernel_args {
    const rt_dnode* nodes;
    const rt_sphere* spheres;
    const rt_quad* quads;
    const rt_box* boxes;
    const float4* dquads;
    const float4* dboxes;
    const float4* dboxc;         // per box RT_BOXC_F4 float4: the compact record (box_test_compact)
    const rt_medium* media;
    const int32_t* lights;
    int n_nodes, lights_count;
    int uv_always;       // a medium samples an image texture: keep sphere uv current (Q9)
    int variant;         // kernel structure variant (A/B; 0 = default)
    rt_dtex tex[8];
    rt_camera_ubo cam;
    float background[3];
    int max_depth;
    float sqrt_spp, recip_sqrt_spp;
    // image / partition
    float* image;        // float4 rows, local-compact
    int width, height;
    int local_rows;
    int rank, world, stripe_rows;
    int first_frame, n_frames;
    unsigned long long* stats;   // diagnostic counters (stats variant only)
    unsigned* census;            // stats twin, leaf census (rt_debug_enable_stats(ctx, 2)): per resident wave its
                                 // record count, then census_cap records of RT_CENSUS_WORDS words per wave
    int census_cap, census_waves;
    unsigned* node_hits;         // stats twin, node-hit count (rt_debug_count_node_hits): per link node the box tests
                                 // that hit, then (word n_nodes) the walks begun at the root
    int* tile_counter;           // persistent kernel: next work unit (zeroed per launch)
    // work split: unit = chunk * n_tiles + tile, chunk = frames [c*chunk_frames, ...) (ordered chunks);
    // staged launches may end with tail_chunks chunks of one frame each (option tail_chunks): chunk
    // c >= n_chunks - tail_chunks holds frame n_frames - (n_chunks - c)
    int n_chunks, chunk_frames, tail_chunks;
    unsigned* tile_done;         // ordered chunks: per tile, the chunks published so far (zeroed per launch)
    float4* samples;             // staged chunks: per-frame colours [n_frames][n_pixels]; nullptr = ordered / one chunk
    uint8_t* sflags;             // sparse staging (render_stream): per sample [n_frames][n_pixels] 1 when its colour
                                 // is not (+0, +0, +0) and was stored in `samples`, else 0; nullptr = dense
    size_t n_pixels;             // local_rows * width
    unsigned* fault;             // set when an ordered-chunk wait times out (rt_sync reports it)
    float4* wbuf;                // pooled units, ordered / one chunk: per resident wave 2 x 64 x chunk_frames colours
    int wbuf_waves;              // waves wbuf has slots for (the launch's grid never exceeds it)
    int sm_batch;                // render_sm: shade once this many lanes' walks ended,
    int sm_frac;                 // or this many 64ths of the lanes with a walk (or none runs)
    int walk_frac;               // render_sm: a round's node walk stops once this many 64ths of its lanes
                                 // hold a leaf or ended (64: all of them)
    int box_vnodes;              // the links carry box pre-test nodes (leaf records marked RT_LINK_PRETESTED)
    int zero_dir_end;            // render_stream: a path whose next direction is vec3(0) ends with its miss
                                 // colour in the same shading pass (option zero_dir_end)
    int leaf_pf;                 // BOXC kernels: the leaf stage prefetches each slot's record (spheres, boxes
                                 // and media all staged in LDS; rt_kernel.hip leaf_prims_t)
    int debug_flags;             // ablation switches for attribution runs (RT_DEBUG_FLAGS; 0 = exact)
    int boxes_canon;             // every box has Box.java's axis-aligned face layout (normal of face i
                                 // along axis z, x, z, x, y, y): planes read as (s_i, w_i)
    int fastdiv;                 // the scene's records are in the shared-reciprocal division regime
    float box_margin;            // > 0: box tests start with a slab test of the box's bounds
                                 // grown by this margin (2^-13 of the scene's extent), which no face
                                 // the exact test accepts can lie outside; 0: no pre-test
    int perlin_slot;             // texture slot staged in LDS for Perlin noise (R32F, 6 x 256), or -1
    int perlin_lds;              // its float4 offset in the dynamic LDS (after the nodes), or -1
    int perlin_packed;           // 1: LDS holds the packed table perlin_pk (256 float4), not the texture
    const float4* perlin_pk;     // the packed Perlin table (rt_capi.hip rt_upload_texture), or nullptr
    int n_media;
    int media_sph;               // every medium's boundary is a sphere (or there is none): RT_OPT_STD kernels
    int media_lds;               // float4 offset of the media records + sphere boundaries in LDS (3 float4
                                 // per medium, after the Perlin table), or -1
    int sph_lds;                 // float4 offset of the spheres' intersection halves (A, B) in LDS, or -1
    int n_sph_lds;               // spheres staged there
    int n_box_lds;               // boxes whose compact records are staged (all of them)
    // shading tables in LDS (option shade_lds; rt_kernel.hip shade / texture_color), each -1 when absent:
    int sph_mat_lds;             // per sphere its third float4 (emission, material)
    int box_mat_lds;             // per compact box (quads[0] emission, material); texture id and the
                                 // faces' zero-sign bits ride in its compact record (rt_capi.hip compact_box)
    int tex_lds;                 // 8 int4 per texture slot: (w, h, is_float, float4 offset of its texels or -1)
    int tex_lds_off[8];          // host side of the same offsets (the staging loop reads them)
    int block;                   // the render kernel's workgroup size: 512, or 1024 (one per CU) when the
                                 // records above fit its LDS (RT_LDS_BIG_BYTES)
    int acc_lds;                 // float4 offset of the lanes' running-mean slots (after everything staged)
    // exact near-first walk (variant 61; tables from rt_capi.hip build_fast)
    const uint32_t* finfo;       // per solid prim (finfo_base[type] + index): reference rank << 16 | reference leaf
    int fast_ok;
    int finfo_base[8];
    int fm_n;                    // media slots in the reference's visit order
    int fm_medium[4], fm_leaf[4], fm_track[4], fm_flags[4];   // flags: 1 same leaf as the previous slot, 2 solid first
    int fl_n;                    // trackers: the closest solid ranked before a constrained media slot
    int fl_medium[2], fl_rank[2];
    // the SAH tree as two-child nodes for the stack walk (FastTables::inner2/leaves2)
    const float4* f2inner;       // 4 float4 per inner node: left box, right box, refs + tracker bits
    const uint2* f2leaves;       // (meta, prims) per leaf
    int n_f2inner, n_f2leaves, f2depth;
    // the reference's threaded BVH with explicit successors (variant 0/37; rt_capi.hip build_links)
    const float4* lnodes;        // 2 float4 per node, then the leaves' (types | next << 8, prims) as uint2
    int n_lnode_f4;              // float4 of the whole array; 0 = not available (no BVH)
    int lds_node_f4;             // float4 of nodes staged in LDS (from address 0): all 2 * n_nodes, or
                                 // the top levels (two-level walk: addresses past them read lnodes)
    int leaf_lds;                // float4 offset of the leaf records in LDS, or -1 (read from lnodes)
    int lds_end_f4;              // float4 end of everything the link-format shapes stage in LDS
    int box_cmp_lds;             // float4 offset of the boxes' 48-byte records in LDS (RT_BOXC_F4 each), or
                                 // -1 (read from dboxc)
    int box_all_cmp;             // every box's record is compact (box_test_compact); else the full box test
    int sph_pairs;               // most leaves hold two spheres: the kernels that test such a leaf's two at once
    // the spine (rt_capi.hip plan_spine): every walk starts with the root and its right children
    // 1 .. spine_len-1; a ray whose origin lies in all their boxes, away from the faces by more than
    // 0.00125 x its largest direction component, hits every one of them, so its walk starts at
    // spine_start (the last one's hit successor).  spine_len 0: off.
    int spine_len;
    uint32_t spine_start;
    float spine_lo[3], spine_hi[3];   // the boxes' intersection, shrunk by 2^-18 of its largest coordinate
    // bounds of the device-side waits, in ticks of the 100 MHz real-time clock (s_memrealtime)
    unsigned long long watchdog_ticks;     // render_stream: no sample stored by the wave for this long
                                           // -> fault word 2, the wave leaves (checked on its first pass
                                           // and every 256th; 0 = at the first check)
    unsigned long long chunk_wait_ticks;   // ordered chunks: wait for the previous chunk -> fault word 1
    float rand_factors[RT_MAX_FRAMES_PER_LAUNCH];
};

// What rt_launch_render launched (rt_debug_last_launch)
enum { RT_LI_SHAPE = 0, RT_LI_BLOCK, RT_LI_FASTDIV, RT_LI_PRETEST, RT_LI_LDS, RT_LI_LDS_NODES, RT_LI_COMPACT,
       RT_LI_STAGED, RT_LI_CHUNKS, RT_LI_SPINE, RT_LI_SPARSE, RT_LI_SPAIR, RT_LI_LEAF_PF, RT_LI_SHADE_LDS, RT_LI_WALK_FRAC, RT_LI_BVH_MODE, RT_LI_VNODES, RT_LI_COLLAPSED, RT_LI_REBUILT, RT_LI_N = 20 };

#ifdef RT_AB_KNOBS
// A/B library only (rt_kernel_variants.hip): the structures the release library does not ship
#define RT_FAST_STACK 16   // the near-first walk's per-lane stack (shorts in LDS)
enum { RT_AB_SHAPE_FAST_LDS = 0, RT_AB_SHAPE_FAST_GLOBAL, RT_AB_SHAPE_LINK_PIXEL, RT_AB_SHAPE_META_LDS,
       RT_AB_SHAPE_META_GLOBAL };
int rt_launch_render_ab(int shape, rt_kernel_args& a, const rt_kernel_args* d, size_t lds, bool stats, void* stream);
#endif
// launcher implemented in rt_kernel.hip
int rt_resident_waves(void);   // waves a render launch keeps resident on the current device (its grid, at most)
// sets a.acc_lds; info (may be NULL): RT_LI_* of the launch
int rt_launch_render(rt_kernel_args& a, rt_kernel_args* dargs, void* stream, int* info);
// Row y of the image in the gathered stripe blocks [world][padded_rows][W]: rank k = s % world
// of its stripe s = y / stripe_rows, local row (s / world) * stripe_rows + y % stripe_rows
// (rt_set_partition).  Shared by deinterleave_kernel and rt_debug_deinterleave.
__host__ __device__ inline void rt_gathered_row(int y, int world, int stripe_rows, int* k, int* lr) {
    const int s = y / stripe_rows;
    *k = s % world;
    *lr = (s / world) * stripe_rows + y % stripe_rows;
}
// gathered stripe blocks [world][padded_rows][W] float4 -> [H][W] float4 (device 0 of a gather)
int rt_launch_deinterleave(const void* gathered, void* out, int width, int height, int world, int stripe_rows,
                           int padded_rows, void* stream);
// debug: evaluate GLSL built-ins on device (tests)
int rt_launch_eval_builtin(int fn, const float* dx, const float* dy, float* dout, int n, void* stream);
