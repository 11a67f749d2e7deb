// rt_capi.hip — implementation of include/rt/rt.h (the drop-in C ABI).
//
// Host-side responsibilities that the reference's Java/GL layer had:
// buffer/texture upload (BufferObject.uploadData, Texture.putData), uniforms
// (ShaderProgram.setUniform*), dispatch (RaytraceExecutor.raytrace), readback
// (glGetTexImage) and timing (QueryTimer).  Plus the MI355X-specific parts:
// the threaded-BVH re-layout, RGB8->RGBA8 texture expansion, stripe
// partitioning across devices/processes and caller-owned device images.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include <dlfcn.h>
#include <rccl/rccl.h>   // types only: librccl (~570 MB) is dlopen'ed by the first gather that uses it

#include "rt/rt.h"
#include "rt/rt_debug.h"
#include "rt/rt_types.h"
#include "rt_device.h"
#include "bvh_sah.h"

namespace {

// RCCL, loaded on first use (rt_comm_*, multi-device rt_read_image).  Not linked: a
// single-device context never pays for loading it.
struct Rccl {
    bool tried = false, ok = false;
    void* h = nullptr;
    decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
    decltype(&ncclCommInitRank) CommInitRank = nullptr;
    decltype(&ncclCommInitAll) CommInitAll = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclCommAbort) CommAbort = nullptr;   // optional: an error inside a group aborts
    decltype(&ncclSend) Send = nullptr;
    decltype(&ncclRecv) Recv = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
    // optional: a non-blocking communicator (rt_comm_init), so that no RCCL call can hold the
    // host past the context's deadline (rt_comm_set_timeout)
    decltype(&ncclCommInitRankConfig) CommInitRankConfig = nullptr;
    decltype(&ncclCommGetAsyncError) CommGetAsyncError = nullptr;
};
Rccl& rccl() {
    static Rccl r;
    if (!r.tried) {
        r.tried = true;
        r.h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!r.h) r.h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
        if (r.h) {
#define RT_SYM(F) r.F = reinterpret_cast<decltype(r.F)>(dlsym(r.h, "nccl" #F))
            RT_SYM(GetUniqueId); RT_SYM(CommInitRank); RT_SYM(CommInitAll); RT_SYM(CommDestroy); RT_SYM(Send);
            RT_SYM(Recv); RT_SYM(GroupStart); RT_SYM(GroupEnd); RT_SYM(GetErrorString); RT_SYM(CommAbort);
            RT_SYM(CommInitRankConfig); RT_SYM(CommGetAsyncError);
#undef RT_SYM
            r.ok = r.GetUniqueId && r.CommInitRank && r.CommInitAll && r.CommDestroy && r.Send && r.Recv &&
                   r.GroupStart && r.GroupEnd && r.GetErrorString;
        }
    }
    return r;
}

struct DevBuf {
    void* ptr = nullptr;
    size_t bytes = 0;
};

struct Device {
    int id = 0;
    hipStream_t stream = nullptr;
    bool own_stream = true;
    hipEvent_t ev_start = nullptr, ev_stop = nullptr;
    bool timed = false;
    DevBuf nodes, spheres, quads, boxes, media, lights, tex[8];
    DevBuf dquads, dboxes;   // intersection-only face records (rt_device.h)
    DevBuf dboxc;            // compact canonical box records (RT_BOXC_F4 per box)
    DevBuf perlin_pk;        // the Perlin table re-laid out (rt_kernel.hip perlin_noise_pk), when it qualifies
    DevBuf image;            // internal image
    DevBuf args;             // rt_kernel_args slot in device memory
    DevBuf stats;            // diagnostic counters (rt_debug_enable_stats)
    DevBuf census;           // the stats twin's leaf census (rt_debug_enable_stats(ctx, 2))
    DevBuf node_hits;        // the stats twin's node-hit count (rt_debug_count_node_hits)
    int census_cap = 0, census_waves = 0;
    DevBuf counter;          // persistent-kernel work-unit counter [0] and fault word [1]
    DevBuf tile_done;        // ordered chunks: chunks published per 8x8 tile
    DevBuf samples;          // staged chunks: per-frame colours [frames][local pixels]
    DevBuf sflags;           // sparse staging: per staged sample, 1 where its colour was stored
    DevBuf wbuf;             // pooled units (ordered / one chunk): per resident wave 64 x chunk_frames colours
    DevBuf finfo;            // exact near-first walk tables (variant 61)
    DevBuf f2inner, f2leaves;
    DevBuf links;            // link-format BVH (variant 0/37)
    int fast_gen = -1;       // rt_ctx::fast_gen these copies belong to
    static constexpr int kRing = 8;
    rt_kernel_args* ring = nullptr;   // pinned host staging slots for async arg uploads
    hipEvent_t ring_ev[kRing] = {};
    int ring_pos = 0;
    float* image_ptr = nullptr;  // active image (internal or bound)
    bool image_bound = false;
    int rank = 0, world = 1;     // stripe assignment of this device
    int local_rows = 0, padded_rows = 0;
    ncclComm_t comm = nullptr;   // RCCL communicator of a device gather (rank = this device's slot / process rank)
    DevBuf gather, full;         // device 0 / rank 0: the gathered stripe blocks, the de-interleaved image
};

// Tables of the exact near-first walk (build_fast below; rt_kernel.hip trace_fast).
struct FastTables {
    bool ok = false;
    std::vector<rt_dnode> nodes;   // 8 octant layouts x n_per threaded nodes
    int n_per = 0;
    std::vector<uint32_t> info;    // per solid prim: reference rank << 16 | reference leaf node
    int base[8] = {0};             // info offset by model type
    int fm_n = 0, fm_medium[4] = {0}, fm_leaf[4] = {0}, fm_track[4] = {0}, fm_flags[4] = {0};
    int fl_n = 0, fl_medium[2] = {0}, fl_rank[2] = {0};
    // the same tree as two-child nodes for the stack walk (variant 61): per inner node 4 float4 =
    // left box, right box, (left ref, right ref, tracker bits left | right << 8, 0); a ref >= 0 is an
    // inner node, ~ref a leaf; a leaf is (meta, prims) as in rt_dnode (types and indices, no skip)
    std::vector<float4> inner2;
    std::vector<uint2> leaves2;
    int depth = 0;   // levels of the tree (the stack walk holds at most depth - 1 entries)
};

}  // namespace

struct rt_ctx {
    std::vector<Device> devs;
    std::string err;
    // host copies of what the kernel needs
    std::vector<uint8_t> host_buf[6];
    bool uploaded[6] = {false, false, false, false, false, false};
    int tex_format[8] = {0}, tex_w[8] = {0}, tex_h[8] = {0};
    rt_camera_ubo cam{};
    bool have_cam = false;
    int max_depth = 5;
    float background[3] = {0, 0, 0};
    float sqrt_spp = 1.0f, recip_sqrt_spp = 1.0f;
    int width = 0, height = 0;
    int proc_rank = 0, proc_world = 1, stripe_rows = 16;
    int n_dnodes = 0;
    std::vector<rt_dnode> dnodes;   // host copy of the threaded BVH (fast-walk tables are built from it)
    // the BVH the link walk runs on (rt_set_bvh_mode): the uploaded one (RT_BVH_REFERENCE), or the
    // binned-SAH tree built from its prims at validation (RT_BVH_SAH, non-parity fast mode, bvh_sah.h)
    int bvh_mode = RT_BVH_REFERENCE;
    int n_link_nodes = 0;
    std::vector<uint8_t> sah_bvh;   // the SAH tree in the reference's node format (rt_debug_walk_bvh)
    std::vector<rt_dnode> walk_dn;  // threaded nodes of the BVH the link walk uses (reference or SAH)
    // the links the launch walks: c->links, or (option box_vnodes) the same with every all-box leaf's
    // box pre-tests as nodes of the walk (build_links with vbox); rebuilt when the margin changes
    std::vector<float4> walk_links;
    int n_walk_nodes = 0;
    bool walk_v = false;
    float walk_v_margin = -1.0f;
    bool walk_stale = true;
    std::vector<float4> boxc_host;  // the compact box records (host copy of Device::dboxc)
    bool box_vnodes = true;         // option box_vnodes
    bool zero_dir_end = true;       // option zero_dir_end (rt_kernel.hip render_stream)
    bool collapse = true;           // option collapse: the walk leaves out inner nodes (plan_collapse)
    int rebuild = 2;                // option rebuild: the walk's inner nodes rebuilt over its leaves (rebuild_inner mode)
    bool walk_r = false;            // walk_links were built on the rebuilt inner nodes
    int walk_rmode = 0;             // ... of this mode
    std::vector<rt_dnode> rb_dn;    // rebuild_inner(walk_dn, rb_mode), kept across camera moves
    int rb_mode = -1;               // -1: not built for the current walk_dn
    bool walk_c = false;            // walk_links were built with a collapse plan ...
    rt_camera_ubo walk_cam{};       // ... for this camera and image size
    int walk_w = 0, walk_h = 0;
    int n_dropped = 0;              // inner nodes the walk leaves out
    int n_rebuilt = 0;              // nodes of the rebuilt tree (0: the tree as uploaded / built)
    int n_vnodes = 0;               // box pre-test nodes in walk_links
    FastTables fast;
    std::vector<float4> links;   // build_links(dnodes), empty when unavailable
    int fast_gen = 0;
    bool spec_ok = false;   // every child box lies inside its parent's (the near-first walk needs it)
    int debug_flags = 0;    // env RT_DEBUG_FLAGS: ablation runs only (bit 0: Perlin -> 0.5)
    bool uv_always = false;
    bool boxes_canon = false;   // every box has Box.java's axis-aligned face layout (dboxes[18..20])
    bool fd_ok[6] = {true, true, true, true, true, true};   // per binding: records in the fast-division regime
    bool fd_cam = true;
    bool boxes_cond = false;   // every box face's 2-D Cramer system is well conditioned (box pre-test)
    float scene_extent = -1.0f;   // max |coordinate| over records and camera (< 0: not computed)
    bool validated = false;
    uint64_t last_ns = 0;
    int variant = 0;   // kernel structure variant (env RT_KERNEL_VARIANT; A/B only)
    int variant_no_stats = -1;   // the variant active before rt_debug_enable_stats(c, 1), restored by (c, 0)
    // the collapse plan from measured node hits (rt_debug_set_collapse_hits): per node of the walk's
    // tree in its breadth-first link order, the box tests that hit, and the walks begun at the root
    std::vector<int64_t> inj_hits;
    int64_t inj_walks = 0;
    // Work split: aim for chunk_target work units per resident wave (env
    // RT_CHUNK_TARGET; 0 = one chunk per tile), staged_chunk_target when staged
    // (RT_STAGED_CHUNK_TARGET).  With at least stage_tiles tiles
    // per resident wave (env RT_STAGE_TILES) the chunks are ordered (the running
    // mean is handed from wave to wave, rt_kernel.hip wait_chunk); with fewer, a
    // tile's frames would be one long serial chain, so the chunks run in parallel,
    // stage their per-frame colours (at most sample_budget bytes) and fold_kernel
    // applies the running mean in frame order.  The default stage_tiles stages
    // every chunked launch: with render_stream that measured fastest at N = 1 too
    // (scene 8 -5% against ordered chunks).
    int chunk_target = 16;          // ordered chunks (RT_CHUNK_TARGET)
    int staged_chunk_target = 48;   // staged chunks (RT_STAGED_CHUNK_TARGET)
    int tail_chunks = -1;           // option tail_chunks: staged launches end with this many one-frame chunks
                                    // (-1: tail_chunks_for the tree)
    int stage_tiles = 1 << 20;      // in effect always staged (the measured best with render_stream)
    bool fastdiv = true;   // shared-reciprocal divisions where exact (env RT_FASTDIV=0 disables; A/B)
    bool box_pretest = true;   // the canonical box tests' bounds pre-test (env RT_BOX_PRETEST=0 disables; A/B)
    int sm_batch = 64;   // render_stream's shading batch (env RT_SM_BATCH) ...
    int sm_frac = 0;     // ... or fraction of the lanes with a walk, in 64ths (env RT_SM_FRAC); 0 = by kernel:
                         // 50 for the compact-box kernels (scene 8 1080p -1.1%, 4K -1.6% against 56), 56 else
                         // (scene 6 +1.4% at 52; profiles/r03_sm_frac_knobs.log)
    bool shade_lds = true;       // shading tables in LDS (sphere / box materials, small textures; option):
                                 // scenes 8 / 0 / 6 -0.3 / -1.0 / -1.2% (profiles/r04_shade_lds_ab_s*.log)
    bool tl_small_lds = true;    // two-level walk: small sphere / box tables staged beside the top levels (option)
    bool leaf_prefetch = true;   // leaf records prefetched before the type blocks when all are in LDS (option)
    int walk_frac = 0;   // render_stream: node walks stop at this fraction of lanes ready, in 64ths (env RT_WALK_FRAC);
                         // 0 = by BVH size: 8 up to 64 nodes, 32 up to 1024, 48 above (walk_frac_for)
    bool big_wg = true;    // 1024-thread workgroups with sphere + box records in LDS when they fit (env RT_BIG_WG=0: A/B)
    bool sph_lds = true;   // sphere records' first two float4 in LDS when they fit (env RT_SPH_LDS=0 disables; A/B)
    bool compact_boxes = true;   // boxes' compact records when every box has one (box_test_compact; option 0: A/B)
    bool spine = true;           // walks start past the spine when they hit it for sure (plan_spine)
    int lds_node_cap = 0;        // bytes of BVH nodes staged in LDS, 0 = as many as fit (tests: force the two-level walk)
    bool tl_leaf_lds = true;     // two-level walk: the leaf records in LDS beside the top levels (when they fit)
    int perlin_pk_slot = -1;     // texture slot whose Perlin table has its packed copy (Device::perlin_pk)
    bool sparse_stage = true;    // staged chunks store only the colours that are not exactly zero (option)
    int sphere_pairs = 1;        // the sphere-pair kernels when most leaves hold two spheres (option; 2: always,
                                 // compact-box kernels included)
    int pair_leaves = -1;        // per mille of the link-format leaves that hold two spheres (< 0: not counted)
    bool perlin_pk = true;       // stage the packed Perlin table (option; else the texture as uploaded)
    int n_boxc_ok = 0;           // boxes whose compact record reproduces their faces
    unsigned long long watchdog_ticks = 120ull * 100000000ull;     // render_stream progress bound (100 MHz ticks)
    unsigned long long chunk_wait_ticks = 30ull * 100000000ull;    // ordered-chunk wait bound
    size_t sample_budget = (size_t)32 << 30;   // staged colours per launch, at most (and at most half the free memory)
    int last_launch[RT_LI_N] = {0};
    bool launched = false;
    // gathers (rt_read_image of a multi-device context, rt_gather_image): RT_GATHER_*
    int gather_path = -1;
    bool comm_tried = false;     // ncclCommInitAll of a multi-device context attempted
    bool proc_comm = false;      // rt_comm_init: one rank of a multi-process communicator
    bool comm_nonblocking = false;   // ... made non-blocking (ncclConfig_t.blocking = 0)
    int comm_timeout_ms = 120000;    // rt_comm_set_timeout: deadline of rt_comm_init / rt_gather_image (0: none)
};

namespace {

int set_err(rt_ctx* c, int code, const std::string& m) {
    if (c) c->err = m;
    return code;
}

#define HIPCHK(ctx, call)                                                                           \
    do {                                                                                            \
        hipError_t e_ = (call);                                                                     \
        if (e_ != hipSuccess)                                                                       \
            return set_err(ctx, RT_ERR_DEVICE, std::string(#call) + ": " + hipGetErrorString(e_));   \
    } while (0)

// Every host<->device transfer and fill is ordered on the device's render stream
// (which may be non-blocking or caller-owned) and completed before returning, so
// it can neither overlap a queued render nor race the next one.
int h2d(rt_ctx* c, Device& d, void* dst, const void* src, size_t n) {
    if (!n) return RT_OK;
    HIPCHK(c, hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, d.stream));
    HIPCHK(c, hipStreamSynchronize(d.stream));
    return RT_OK;
}
int d2h(rt_ctx* c, Device& d, void* dst, const void* src, size_t n) {
    if (!n) return RT_OK;
    HIPCHK(c, hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, d.stream));
    HIPCHK(c, hipStreamSynchronize(d.stream));
    return RT_OK;
}

int dev_alloc_copy(rt_ctx* c, Device& d, DevBuf& b, const void* src, size_t n) {
    HIPCHK(c, hipSetDevice(d.id));
    HIPCHK(c, hipStreamSynchronize(d.stream));
    if (b.ptr && b.bytes < n) {
        HIPCHK(c, hipFree(b.ptr));
        b.ptr = nullptr;
        b.bytes = 0;
    }
    if (!b.ptr && n > 0) {
        HIPCHK(c, hipMalloc(&b.ptr, n));
        b.bytes = n;
    }
    return h2d(c, d, b.ptr, src, n);
}

void dev_free(DevBuf& b) {
    if (b.ptr) (void)hipFree(b.ptr);
    b.ptr = nullptr;
    b.bytes = 0;
}

int local_rows_of(int h, int rank, int world, int stripe) {
    if (h <= 0 || world <= 0 || stripe <= 0) return 0;
    int n = 0;
    int n_stripes = (h + stripe - 1) / stripe;
    for (int s = rank; s < n_stripes; s += world) n += std::min(stripe, h - s * stripe);
    return n;
}

int padded_rows_of(int h, int world, int stripe) {
    int n_stripes = (h + stripe - 1) / stripe;
    return ((n_stripes + world - 1) / world) * stripe;
}

// Re-lay the reference's pre-order BVH (BVHNode.java:13-56) as a threaded
// array in the reference traversal's own visiting order (right child first).
int thread_bvh(rt_ctx* c, const rt_bvh_node* in, int n, std::vector<rt_dnode>& out) {
    out.clear();
    if (n == 0) return RT_OK;
    struct Item { int src; int depth; };
    // Explicit DFS producing right-first pre-order; skip links patched after.
    std::vector<int> order_src;
    std::vector<int> skip_parent;   // for each emitted node: index of the emitted node whose skip it inherits (-1 = END)
    struct Frame { int src; int inherit_skip_from_emitted; int left_sibling_src; int depth; };
    // Iterative: emit node, then (if inner) process right subtree whose skip = first node of left subtree,
    // then left subtree whose skip = this node's skip.
    // We compute skip by a second pass: skip(node) = next emitted node after its subtree.
    std::vector<int> subtree_end;   // emitted index one past this node's subtree
    std::vector<int> stack_src, stack_depth, stack_emitted;
    // recursive lambda with explicit stack to avoid deep recursion
    struct Work { int src; int depth; int phase; int emitted; };
    std::vector<Work> st;
    st.push_back({0, 1, 0, -1});
    const size_t kMaxNodes = (size_t)RT_MAX_RECORDS;
    while (!st.empty()) {
        Work& w = st.back();
        if (w.phase == 0) {
            if (w.src < 0 || w.src >= n) return set_err(c, RT_ERR_INVALID_ARG, "BVH child index out of range");
            if (w.depth > RT_MAX_BVH_DEPTH) return set_err(c, RT_ERR_LIMIT, "BVH deeper than the reference's stack[64]");
            if (order_src.size() >= kMaxNodes) return set_err(c, RT_ERR_LIMIT, "threaded BVH exceeds 65535 nodes");
            w.emitted = (int)order_src.size();
            order_src.push_back(w.src);
            subtree_end.push_back(0);
            const rt_bvh_node& nd = in[w.src];
            int lt = nd.left_id & 0xFFFF;
            if (lt != 0) {
                subtree_end[w.emitted] = w.emitted + 1;
                st.pop_back();
                continue;
            }
            w.phase = 1;
            int right = (nd.right_id >> 16) & 0xFFFF;
            int depth = w.depth;
            st.push_back({right, depth + 1, 0, -1});
        } else if (w.phase == 1) {
            w.phase = 2;
            const rt_bvh_node& nd = in[w.src];
            int left = (nd.left_id >> 16) & 0xFFFF;
            int depth = w.depth;
            st.push_back({left, depth + 1, 0, -1});
        } else {
            subtree_end[w.emitted] = (int)order_src.size();
            st.pop_back();
        }
    }
    int m = (int)order_src.size();
    out.resize(m);
    for (int k = 0; k < m; k++) {
        const rt_bvh_node& nd = in[order_src[k]];
        rt_dnode& d = out[k];
        d.xmin = nd.xmin; d.xmax = nd.xmax; d.ymin = nd.ymin; d.ymax = nd.ymax; d.zmin = nd.zmin; d.zmax = nd.zmax;
        int e = subtree_end[k];
        uint32_t skip = (e >= m) ? RT_NODE_END : (uint32_t)e;
        uint32_t lt = (uint32_t)(nd.left_id & 0xFFFF), rt = (uint32_t)(nd.right_id & 0xFFFF);
        if (lt != 0) {
            if (lt > 15 || rt > 15 || rt == 0) return set_err(c, RT_ERR_INVALID_ARG, "BVH leaf with bad model type");
            // A singleton leaf lists one prim twice (BVHNode.java:33-34).
            // Re-testing a sphere cannot hit (strict root test against the t it set);
            // a quad/box re-hit at equal t rebuilds the same record (same face: the
            // last interior face of minimal t).  Only a medium's second test matters
            // (its own rand() draw), so for the others slot 2 is marked empty (type 0).
            if (lt == rt && nd.left_id == nd.right_id && lt != RT_MODEL_CONSTANT_MEDIUM) rt = 0;
            d.meta = skip | (lt << 16) | (rt << 20);
            d.prims = (uint32_t)((nd.left_id >> 16) & 0xFFFF) | ((uint32_t)((nd.right_id >> 16) & 0xFFFF) << 16);
        } else {
            d.meta = skip;
            d.prims = 0;
        }
    }
    return RT_OK;
}

// Every inner node's two children (right = k+1, left = skip of k+1) lie inside
// its box.  The reference's builder guarantees it (a node's box is the padded
// join of its children's, AABB.java:15-66); uploaded bytes are checked anyway
// because the speculative walk (rt_kernel.hip, Trace) relies on it.
bool boxes_nest(const std::vector<rt_dnode>& dn) {
    const int m = (int)dn.size();
    auto inside = [](const rt_dnode& c, const rt_dnode& p) {
        return c.xmin >= p.xmin && c.xmax <= p.xmax && c.ymin >= p.ymin && c.ymax <= p.ymax && c.zmin >= p.zmin &&
               c.zmax <= p.zmax;
    };
    for (int k = 0; k < m; k++) {
        if ((dn[k].meta & 0xF0000u) != 0) continue;   // leaf
        if (k + 1 >= m) return false;
        uint32_t l = dn[k + 1].meta & 0xFFFFu;
        if (l == RT_NODE_END || (int)l >= m) return false;
        if (!inside(dn[k + 1], dn[k]) || !inside(dn[l], dn[k])) return false;
    }
    return true;
}

// The threaded BVH in link format (rt_device.h RT_LINK_*; rt_kernel.hip link_walk):
// the same nodes and boxes, placed breadth-first (node k's children in the threaded
// array are its right child k + 1 and its left child skip(k + 1)), each with its
// successor addresses: on a box hit an inner node continues at its right child (the
// reference pushes left then right and pops right first, compute.glsl:259-260), a leaf
// leaves the loop with its ordinal; on a miss both continue at the threaded skip node.
// Leaf j's record follows the nodes: (prim types | the skip node's address << 8,
// prims), in threaded order.  The walk therefore visits the threaded walk's node
// sequence (tests/test_link_nodes.py), and the top levels every ray walks sit at the
// lowest addresses, the part a two-level launch stages in LDS.  Empty when there is
// no BVH or it has more nodes than 16-bit indices address.
std::vector<float4> build_links(const std::vector<rt_dnode>& dn, const std::vector<float>* vbox = nullptr,
                                int* n_nodes_out = nullptr, const std::vector<uint8_t>* drop = nullptr) {
    std::vector<float4> out;
    const size_t n = dn.size();
    if (n_nodes_out) *n_nodes_out = 0;
    if (n == 0 || n > RT_LINK_MAX_NODES) return out;
    auto is_leaf = [&](size_t k) { return (dn[k].meta & 0xF0000u) != 0; };
    // Node collapse (plan_collapse): a link that leads to a left-out inner node leads to its first
    // child (threaded k + 1) instead, repeatedly; the left-out nodes get no place (the kept nodes keep
    // their breadth-first order, so a two-level launch's LDS prefix holds only reachable nodes).
    const bool dropping = drop && drop->size() == n && !(*drop)[0];
    auto kept = [&](uint32_t k) {
        while (dropping && k < n && (*drop)[k] && !is_leaf(k)) k++;
        return k;
    };
    std::vector<uint32_t> pos(n, 0xFFFFFFFFu), order;
    order.reserve(n);
    order.push_back(0);
    for (size_t h = 0; h < order.size(); h++) {
        const uint32_t k = order[h];
        if (pos[k] != 0xFFFFFFFFu || order.size() > n) return std::vector<float4>();
        pos[k] = (uint32_t)h;
        if (is_leaf(k)) continue;
        const uint32_t l = k + 1 < n ? (dn[k + 1].meta & 0xFFFFu) : RT_NODE_END;
        if (k + 1 >= n || l == RT_NODE_END || l >= n) return std::vector<float4>();
        order.push_back(k + 1);
        order.push_back(l);
    }
    if (order.size() != n) return out;
    size_t nk = n;   // the tree's nodes that get a place
    if (dropping) {
        nk = 0;
        for (size_t h = 0; h < n; h++) {
            const uint32_t k = order[h];
            pos[k] = ((*drop)[k] && !is_leaf(k)) ? 0xFFFFFFFFu : (uint32_t)nk++;
        }
    }
    // Box pre-tests as nodes (vbox: 6 floats per box, its bounds grown by the pre-test's margin,
    // rt_kernel.hip leaf_prims_t): a leaf of one or two boxes becomes a chain of one node per box
    // whose hit leads to that box's own leaf record -- the box tested alone, marked pre-tested
    // (RT_LINK_PRETESTED) -- and whose miss (or the record's continuation) leads to the next box's
    // node, after the last one to the leaf's skip node.  The walk meets the boxes in the same
    // order, each node test is the pre-test itself (the same slab function on the same floats
    // under the same ray_t), and a box whose pre-test misses is one the exact test rejects, so
    // every lane tests the same boxes with the same results -- only the pre-test moves from the
    // leaf stage into the walk.  The chain nodes follow the tree's nodes.
    const size_t nbox = vbox ? vbox->size() / 6 : 0;
    std::vector<uint32_t> vfirst(n, 0xFFFFFFFFu);   // leaf k's first chain node (0xFFFFFFFF: not expanded)
    size_t nv = 0;
    for (size_t k = 0; k < n && vbox; k++) {
        if (!is_leaf(k)) continue;
        const uint32_t t0 = (dn[k].meta >> 16) & 0xFu, t1 = (dn[k].meta >> 20) & 0xFu;
        const uint32_t p0 = dn[k].prims & 0xFFFFu, p1 = dn[k].prims >> 16;
        if (t0 != RT_MODEL_BOX || (t1 != RT_MODEL_BOX && t1 != 0) || p0 >= nbox || (t1 && p1 >= nbox)) continue;
        vfirst[k] = (uint32_t)(nk + nv);
        nv += t1 ? 2 : 1;
    }
    const size_t N = nk + nv;
    if (N > RT_LINK_MAX_NODES) return build_links(dn, nullptr, n_nodes_out, drop);
    size_t nl = 0;
    for (size_t k = 0; k < n; k++)
        if (is_leaf(k)) nl += vfirst[k] == 0xFFFFFFFFu ? 1 : (((dn[k].meta >> 20) & 0xFu) ? 2 : 1);
    out.assign(2 * N + (nl + 1) / 2, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    uint2* leaves = reinterpret_cast<uint2*>(out.data() + 2 * N);
    auto f = [](uint32_t u) {
        float x;
        std::memcpy(&x, &u, 4);
        return x;
    };
    auto put = [&](size_t at, float x0, float x1, float y0, float y1, float z0, float z1, uint32_t hit, uint32_t miss) {
        out[2 * at] = make_float4(x0, x1, y0, y1);
        out[2 * at + 1] = make_float4(z0, z1, f(hit), f(miss));
    };
    uint32_t li = 0;
    for (size_t k = 0; k < n; k++) {
        const rt_dnode& d = dn[k];
        if (pos[k] == 0xFFFFFFFFu) continue;   // left out (collapse)
        const uint32_t skip = d.meta & 0xFFFFu;
        const uint32_t skip_at = skip == RT_NODE_END ? RT_LINK_END : 32u * pos[kept(skip)];
        const uint32_t next_end = skip == RT_NODE_END ? RT_LINK_NEXT_END : skip_at;
        uint32_t hit;
        if (is_leaf(k) && vfirst[k] != 0xFFFFFFFFu) {
            const uint32_t v0 = vfirst[k];
            const bool two = ((d.meta >> 20) & 0xFu) != 0;
            hit = 32u * v0;
            for (int j = 0; j < (two ? 2 : 1); j++) {
                const uint32_t b = j ? d.prims >> 16 : d.prims & 0xFFFFu;
                const float* g = vbox->data() + 6 * (size_t)b;
                const bool last = !two || j == 1;
                const uint32_t cont = last ? skip_at : 32u * (v0 + 1);
                put(v0 + j, g[0], g[1], g[2], g[3], g[4], g[5], RT_LINK_LEAF | li, cont);
                leaves[li++] = make_uint2((RT_MODEL_BOX | RT_LINK_PRETESTED) | (last ? next_end : cont) << 8, b);
            }
        } else if (is_leaf(k)) {
            hit = RT_LINK_LEAF | li;
            leaves[li++] = make_uint2(((d.meta >> 16) & 0xFFu) | next_end << 8, d.prims);
        } else {
            hit = 32u * pos[kept((uint32_t)k + 1)];
        }
        put(pos[k], d.xmin, d.xmax, d.ymin, d.ymax, d.zmin, d.zmax, hit, skip_at);
    }
    if (n_nodes_out) *n_nodes_out = (int)N;
    return out;
}

// Small trees (up to RT_SMALL_TREE nodes: the Cornell boxes' 7) keep their nodes: there the camera's
// rays are few of the walks (paths bounce inside the box) and their counts mislead -- scenes 6 / 7
// measured +7.7 / +13.8% with the grid's choice, while scene 0 (511 nodes) -8.8%, scene 8 -5.6%
// (profiles/r05_j_opts_s*.log).
#define RT_SMALL_TREE 64

// Inner-node rebuild (option rebuild): the walk's leaves tested, their order and each test's
// ray_t do not depend on the inner nodes above them, as long as every inner box holds the leaf
// boxes below it.  A leaf node whose box test hits (under the ray_t of its turn) has every
// ancestor's test hit too -- an ancestor is tested earlier, under a ray_t.max at least as large,
// and the slab test is monotone in the box and in ray_t.max (plan_collapse below) -- so it is
// tested in any such tree; one whose test misses has its prims tested in none.  The leaves' own
// boxes and their order (the reference's walk order, the threaded array's) decide everything.  So
// the inner nodes are rebuilt over the reference's leaf sequence: each range of consecutive leaves
// split where the surface-area cost of its two parts, area x leaves, is least, a node's box the
// exact join (min / max) of its leaves' boxes.  The reference's builder splits at the median along
// a random axis (BVHNode.java:13-56); over scene 8's leaf order this tree takes a camera ray
// through 35% fewer node tests (tools/node_collapse_study.py).  Leaves and their records are
// unchanged.  Empty when the uploaded tree's boxes do not nest (the reference's walk
// then prunes leaves at a missed ancestor that the rebuilt tree would reach -- the ABI accepts any
// BVH bytes, so this is checked, as plan_collapse does), when a leaf box is flat or inverted
// (plan_collapse's condition), when the tree has fewer than 3 leaves, or when the host memory
// for the plan cannot be had.
std::vector<rt_dnode> rebuild_inner_impl(const std::vector<rt_dnode>& dn, int mode);
std::vector<rt_dnode> rebuild_inner(const std::vector<rt_dnode>& dn, int mode = 1) {
    if (dn.size() <= RT_SMALL_TREE || dn.size() > RT_LINK_MAX_NODES || !boxes_nest(dn)) return {};
    try {
        return rebuild_inner_impl(dn, mode);
    } catch (const std::bad_alloc&) {   // the walk keeps the uploaded tree
        return {};
    }
}

// The dynamic programme's ranges: up to RT_REBUILD_DP_LEAVES leaves (3 m x m doubles + an m x m
// split table: 28 MB at 1024; scene 8 has 897 leaves), greedy splits above.
#define RT_REBUILD_DP_LEAVES 1024

std::vector<rt_dnode> rebuild_inner_impl(const std::vector<rt_dnode>& dn, int mode) {
    std::vector<rt_dnode> out;
    const size_t n = dn.size();
    std::vector<uint32_t> L;
    for (size_t k = 0; k < n; k++) {
        const rt_dnode& d = dn[k];
        if ((d.meta & 0xF0000u) == 0) continue;
        if (!(d.xmin < d.xmax && d.ymin < d.ymax && d.zmin < d.zmax)) return out;
        L.push_back((uint32_t)k);
    }
    const size_t m = L.size();
    if (m < 3 || 2 * m - 1 > RT_LINK_MAX_NODES) return out;
    auto join = [](rt_dnode& a, const rt_dnode& b) {
        a.xmin = std::min(a.xmin, b.xmin); a.xmax = std::max(a.xmax, b.xmax);
        a.ymin = std::min(a.ymin, b.ymin); a.ymax = std::max(a.ymax, b.ymax);
        a.zmin = std::min(a.zmin, b.zmin); a.zmax = std::max(a.zmax, b.zmax);
    };
    auto area = [](const rt_dnode& b) {
        const double dx = (double)b.xmax - b.xmin, dy = (double)b.ymax - b.ymin, dz = (double)b.zmax - b.zmin;
        return dx * dy + dy * dz + dz * dx;
    };
    out.resize(2 * m - 1);
    std::vector<rt_dnode> pre(m), suf(m);
    // mode 2 (up to RT_REBUILD_DP_LEAVES leaves): the split points of the tree whose inner boxes'
    // areas sum least, by a dynamic programme over the ranges; otherwise each range split greedily
    std::vector<uint32_t> split;
    if (mode == 2 && m <= RT_REBUILD_DP_LEAVES) {
        std::vector<double> A(m * m), C(m * m, 0.0), CT(m * m, 0.0);   // CT[j * m + i] = C[i * m + j]
        for (size_t i = 0; i < m; i++) {
            rt_dnode b = dn[L[i]];
            for (size_t j = i; j < m; j++) {
                if (j > i) join(b, dn[L[j]]);
                A[i * m + j] = area(b);
            }
        }
        split.assign(m * m, 0);
        for (size_t len = 2; len <= m; len++) {
            for (size_t i = 0; i + len <= m; i++) {
                const size_t j = i + len - 1;
                double best = INFINITY;
                uint32_t bk = (uint32_t)i;
                const double* row = &C[i * m];
                const double* col = &CT[j * m + 1];   // col[k] = C[(k + 1) * m + j]
                // Knuth's window: the best split of [i, j] between those of [i, j - 1] and [i + 1, j]
                // (exact when the costs satisfy the quadrangle inequality; any split is exact for the
                // walk, so a window that misses the optimum only costs node tests): O(leaves^2)
                size_t k0 = i, k1 = j - 1;
                if (len > 2) {
                    k0 = std::max<size_t>(i, split[i * m + j - 1]);
                    k1 = std::min<size_t>(j - 1, split[(i + 1) * m + j]);
                    if (k0 > k1) {
                        k0 = i;
                        k1 = j - 1;
                    }
                }
                for (size_t k = k0; k <= k1; k++) {
                    const double c = row[k] + col[k];
                    if (c < best) {
                        best = c;
                        bk = (uint32_t)k;
                    }
                }
                C[i * m + j] = CT[j * m + i] = A[i * m + j] + best;
                split[i * m + j] = bk;
            }
        }
    }
    // pre-order emission: (range, slot); a node's first child follows it, its skip is the slot
    // after its subtree (2 x leaves - 1 slots), RT_NODE_END past the last
    struct Item { uint32_t i, j, at; };
    std::vector<Item> st{{0u, (uint32_t)m, 0u}};
    while (!st.empty()) {
        const Item it = st.back();
        st.pop_back();
        const uint32_t cnt = it.j - it.i, end = it.at + 2 * cnt - 1;
        const uint32_t skip = end >= 2 * m - 1 ? RT_NODE_END : end;
        if (cnt == 1) {
            rt_dnode d = dn[L[it.i]];
            d.meta = (d.meta & ~0xFFFFu) | skip;
            out[it.at] = d;
            continue;
        }
        for (uint32_t t = 0; t < cnt; t++) {
            pre[t] = dn[L[it.i + t]];
            if (t) join(pre[t], pre[t - 1]);
        }
        for (uint32_t t = cnt; t-- > 0;) {
            suf[t] = dn[L[it.i + t]];
            if (t + 1 < cnt) join(suf[t], suf[t + 1]);
        }
        uint32_t best = 1;
        double best_c = INFINITY;
        if (!split.empty()) {
            best = split[(size_t)it.i * m + (it.j - 1)] - it.i + 1;
            best_c = 0.0;
        }
        for (uint32_t s = 1; s < cnt && split.empty(); s++) {
            const double cst = area(pre[s - 1]) * s + area(suf[s]) * (cnt - s);
            if (cst < best_c) {
                best_c = cst;
                best = s;
            }
        }
        rt_dnode d = pre[cnt - 1];
        d.meta = skip;   // inner: no prim types
        d.prims = 0;
        out[it.at] = d;
        const uint32_t first_at = it.at + 1, second_at = it.at + 1 + (2 * best - 1);
        st.push_back({it.i + best, it.j, second_at});
        st.push_back({it.i, it.i + best, first_at});
    }
    return out;
}

// Node collapse (option collapse): which inner nodes the link walk leaves out.  When every node's
// box holds its children's (boxes_nest) and no box is flat, a walk that skips an inner node's test
// and tests its children where it stood tests the same leaves in the same order under the same
// ray_t: where the reference's test of the node misses, its children's tests miss too -- per axis
// the slab values are monotone in the plane coordinates (rounding is monotone; with a component
// of 1/dir infinite the fast form passes an axis only for o strictly inside the slab, the exact
// form (rt_kernel_common.h slab) only for o inside or on it, both monotone under nesting) and the
// interval test is monotone in ray_t.max, which only shrinks between a node and its later
// children -- and so on down to the leaf nodes, which are always kept.  Only the number of node
// tests changes: leaving node N out saves its V(N) tests and costs each child V(N) - H(N) more,
// where H(N), the tests of N that hit, does not depend on the other choices and V(N) = H of N's
// nearest kept ancestor.  H is counted over a 128 x 72 grid of the camera's rays (pixel centres,
// ray_t [0.001, inf), boxes only: the host traces no prims) and the least-tests choice for those
// counts taken by a dynamic programme over the tree; the root stays (the walk starts there).
// tools/node_collapse_study.py: on scene 8 this grid's choice cuts the node tests of the
// reference's own walks by 11.5% beyond the spine (the best choice for the walks themselves: 16%).
std::vector<uint8_t> plan_from_hits(const std::vector<rt_dnode>& dn, const std::vector<int64_t>& H, int64_t walks);
std::vector<uint8_t> plan_collapse(const std::vector<rt_dnode>& dn, const rt_camera_ubo& cam, int width, int height) {
    const size_t n = dn.size();
    std::vector<uint8_t> drop(n, 0);
    if (n <= RT_SMALL_TREE || n > RT_LINK_MAX_NODES || width <= 0 || height <= 0 || !boxes_nest(dn)) return drop;
    for (const rt_dnode& d : dn)
        if (!(d.xmin < d.xmax && d.ymin < d.ymax && d.zmin < d.zmax)) return drop;
    auto is_leaf = [&](size_t k) { return (dn[k].meta & 0xF0000u) != 0; };
    const int gx = 128, gy = 72;
    std::vector<int64_t> H(n, 0);
    for (int j = 0; j < gy; j++) {
        for (int i = 0; i < gx; i++) {
            const float px = ((float)i + 0.5f) * (float)width / (float)gx;
            const float py = ((float)j + 0.5f) * (float)height / (float)gy;
            float o[3], inv[3];
            for (int k = 0; k < 3; k++) {
                o[k] = cam.camera_pos[k];
                inv[k] = 1.0f / (cam.up_left[k] + cam.pixel_delta_u[k] * px + cam.pixel_delta_v[k] * py - o[k]);
            }
            uint32_t k = 0;
            while (k < n) {
                const rt_dnode& b = dn[k];
                const float lo3[3] = {b.xmin, b.ymin, b.zmin}, hi3[3] = {b.xmax, b.ymax, b.zmax};
                float lo = 0.001f, hi = INFINITY;
                for (int a = 0; a < 3; a++) {
                    const float t0 = (lo3[a] - o[a]) * inv[a], t1 = (hi3[a] - o[a]) * inv[a];
                    lo = std::fmax(lo, std::fmin(t0, t1));
                    hi = std::fmin(hi, std::fmax(t0, t1));
                }
                const uint32_t skip = b.meta & 0xFFFFu;
                if (!(hi <= lo)) {
                    H[k]++;
                    k = is_leaf(k) ? skip : k + 1;
                } else {
                    k = skip;
                }
                if (k == RT_NODE_END) break;
            }
        }
    }
    return plan_from_hits(dn, H, (int64_t)gx * gy);
}

// The collapse's dynamic programme for given hit counts H (per node of dn) over `walks` walks
// begun at the root (plan_collapse's grid, or counts measured on the walks themselves by the stats
// twin, rt_debug_set_collapse_hits).
std::vector<uint8_t> plan_from_hits(const std::vector<rt_dnode>& dn, const std::vector<int64_t>& H, int64_t walks) {
    const size_t n = dn.size();
    std::vector<uint8_t> drop(n, 0);
    if (H.size() != n || n <= RT_SMALL_TREE || n > RT_LINK_MAX_NODES || !boxes_nest(dn)) return drop;
    for (const rt_dnode& d : dn)
        if (!(d.xmin < d.xmax && d.ymin < d.ymax && d.zmin < d.zmax)) return drop;
    auto is_leaf = [&](size_t k) { return (dn[k].meta & 0xF0000u) != 0; };
    // cost(k, v): the fewest tests of k's subtree when k's place is reached v times
    std::map<std::pair<uint32_t, int64_t>, std::pair<int64_t, bool>> memo;
    std::function<std::pair<int64_t, bool>(uint32_t, int64_t)> cost = [&](uint32_t k, int64_t v) {
        if (is_leaf(k)) return std::make_pair(v, false);
        const auto key = std::make_pair(k, v);
        auto it = memo.find(key);
        if (it != memo.end()) return it->second;
        const uint32_t r = k + 1, l = dn[k + 1].meta & 0xFFFFu;
        const int64_t keep = v + cost(r, H[k]).first + cost(l, H[k]).first;
        std::pair<int64_t, bool> best(keep, false);
        if (k != 0) {
            const int64_t out = cost(r, v).first + cost(l, v).first;
            if (out < keep) best = std::make_pair(out, true);
        }
        memo.emplace(key, best);
        return best;
    };
    std::vector<std::pair<uint32_t, int64_t>> st{{0u, walks}};
    while (!st.empty()) {
        const auto [k, v] = st.back();
        st.pop_back();
        if (is_leaf(k)) continue;
        const bool out = cost(k, v).second;
        drop[k] = out ? 1 : 0;
        const uint32_t r = k + 1, l = dn[k + 1].meta & 0xFFFFu;
        st.push_back({r, out ? v : H[k]});
        st.push_back({l, out ? v : H[k]});
    }
    return drop;
}

// The default walk round threshold (option walk_frac 0): a round's node walk stops once this
// many 64ths of its lanes hold a leaf or ended.  Measured per scene (round 4,
// profiles/r04_knobs*_s*.log; the default was 48 for every scene): the 7-node Cornell boxes
// want short rounds (scene 6: 8..16 -6%, scene 7: 8 -8.6%, 16 -2.5%), scene 0's 511 nodes 32..36
// (-1.3%), scene 8's 1793 nodes 48..52 (44: +0.4%); a two-level launch takes 32 (LDS plan below).
// Rounds only regroup which lanes walk and
// test leaves together: every lane's node and prim sequence is unchanged (bit-identical).
int walk_frac_for(int n_nodes) { return n_nodes <= RT_SMALL_TREE ? 8 : n_nodes <= 1024 ? 32 : 48; }

// The default number of one-frame chunks that end a staged launch (option tail_chunks -1): the units
// the grid claims last are then 64 samples, so its waves finish closer together.  Measured (round 6,
// profiles/r06_l_opts_s*.log, r06_m_opts_s*.log): scene 8 (1793 nodes) -0.9% with one (+0.6% with 4,
// +3.5% with 8: a short unit's claim and set-up cost more than the imbalance), scene 0 (511 nodes)
// +0.4%, scene 6 +0.2%; so one above 1024 nodes, none otherwise.  Only the grouping of samples into
// units changes (bit-identical; tests/test_gpu_fullsize.py gates 0 and 7 at 1080p).
int tail_chunks_for(int n_nodes) { return n_nodes > 1024 ? 1 : 0; }

// The spine of the link-format walk (rt_kernel.hip spine_entry): every walk starts at the
// root and, while it hits, goes on to the right child (compute.glsl:259-260), so its first
// steps are the chain root, right child, its right child, ... down to the first leaf.  In
// scenes with one huge object (scene 8's fog boundary, r 5000; scene 0's ground, r 1000)
// the builder's sort puts it in the right-most leaf, and every box on the chain contains
// it: for a ray starting inside all of them they are hits, tested on every walk (11 of
// scene 8's ~41 node steps per walk).  Picks the longest prefix of the chain whose boxes'
// intersection holds the camera and >= 3/4 of the leaf boxes' centres (where later walks
// start), at least 3 nodes; its last node's hit successor is where such a walk starts.
void plan_spine(const std::vector<float4>& L, int n_nodes, const rt_camera_ubo& cam, bool on,
                rt_kernel_args& a) {
    a.spine_len = 0;
    a.spine_start = 0;
    for (int k = 0; k < 3; k++) a.spine_lo[k] = a.spine_hi[k] = 0.0f;
    if (!on || n_nodes <= 0 || L.size() < 2 * (size_t)n_nodes) return;
    auto bits = [](float f) {
        uint32_t u;
        std::memcpy(&u, &f, 4);
        return u;
    };
    std::vector<float> cx;   // leaf box centres, x y z
    for (int i = 0; i < n_nodes; i++) {
        if ((bits(L[2 * i + 1].z) & RT_LINK_LEAF) == 0) continue;
        cx.push_back(0.5f * (L[2 * i].x + L[2 * i].y));
        cx.push_back(0.5f * (L[2 * i].z + L[2 * i].w));
        cx.push_back(0.5f * (L[2 * i + 1].x + L[2 * i + 1].y));
    }
    const size_t n_leaf = cx.size() / 3;
    if (n_leaf == 0) return;
    float lo[3] = {-INFINITY, -INFINITY, -INFINITY}, hi[3] = {INFINITY, INFINITY, INFINITY};
    uint32_t at = 0;
    for (int len = 1; len <= n_nodes; len++) {
        const float4 b0 = L[2 * (at / 32)], b1 = L[2 * (at / 32) + 1];
        const float blo[3] = {b0.x, b0.z, b1.x}, bhi[3] = {b0.y, b0.w, b1.y};
        for (int k = 0; k < 3; k++) {
            lo[k] = std::max(lo[k], blo[k]);
            hi[k] = std::min(hi[k], bhi[k]);
        }
        float big = 0.0f;
        bool finite = true;
        for (int k = 0; k < 3; k++) {
            finite = finite && std::isfinite(lo[k]) && std::isfinite(hi[k]);
            big = std::max(big, std::max(std::fabs(lo[k]), std::fabs(hi[k])));
        }
        if (!finite) break;
        const float sh = std::ldexp(big, -18);
        float slo[3], shi[3];
        bool ok = true;
        for (int k = 0; k < 3; k++) {
            slo[k] = lo[k] + sh;
            shi[k] = hi[k] - sh;
            ok = ok && slo[k] < shi[k] && slo[k] < cam.camera_pos[k] && cam.camera_pos[k] < shi[k];
        }
        if (!ok) break;   // the intersection only shrinks along the chain
        size_t in = 0;
        for (size_t j = 0; j < n_leaf; j++)
            in += cx[3 * j] > slo[0] && cx[3 * j] < shi[0] && cx[3 * j + 1] > slo[1] && cx[3 * j + 1] < shi[1] &&
                  cx[3 * j + 2] > slo[2] && cx[3 * j + 2] < shi[2];
        if (4 * in < 3 * n_leaf) break;
        const uint32_t hit = bits(b1.z);
        if (len >= 3) {
            a.spine_len = len;
            a.spine_start = hit;
            for (int k = 0; k < 3; k++) {
                a.spine_lo[k] = slo[k];
                a.spine_hi[k] = shi[k];
            }
        }
        if (hit & RT_LINK_LEAF) break;   // the chain's leaf: the walk leaves with it
        if (hit / 32 >= (uint32_t)n_nodes) break;
        at = hit;
    }
}

// ---- exact near-first walk (variant 60; rt_kernel.hip trace_fast) -------------
// Built from the reference's threaded BVH (thread_bvh):
//  * a SAH tree over the BVH's solid prims (sphere / quad / box), each item
//    bounded by its REFERENCE LEAF box, so every SAH box contains the leaf
//    boxes below it (joins are exact min/max); binned SAH, <= 2 prims a leaf;
//  * that tree laid out 8 times as a threaded pre-order with the near child
//    first for each ray-direction octant (a negative direction on the split
//    axis visits the upper child first): the stackless walk, ordered;
//  * per solid prim its reference rank (2 * leaf ordinal + slot: the order in
//    which the reference tests prims) and its reference leaf node;
//  * the media slots in the reference order; a slot with solids ranked before
//    it gets a tracker k (the closest such solid is its ray_t.max), and meta
//    bit 24 + k marks the SAH subtrees holding solids ranked before it.
// Eligibility (ok): every quad / box face is axis-aligned, so plane hits are
// exact to a few ulps (the kernel's windows rely on it); <= 4 media slots,
// <= 2 trackers, every index in range.  The caller adds the box nesting and
// the no-image-texture-on-media conditions.
struct FastItem {
    float lo[3], hi[3], c[3];
    int type, idx, rank;
};
struct FastNode {
    float lo[3], hi[3];
    int kid[2];
    int axis, first, count, min_rank;
};

int fast_build_node(std::vector<FastItem>& it, int b, int e, std::vector<FastNode>& T) {
    FastNode nd;
    float clo[3], chi[3];
    for (int k = 0; k < 3; k++) {
        nd.lo[k] = clo[k] = INFINITY;
        nd.hi[k] = chi[k] = -INFINITY;
    }
    nd.kid[0] = nd.kid[1] = -1;
    nd.axis = 0;
    nd.first = b;
    nd.count = e - b;
    nd.min_rank = INT_MAX;
    for (int i = b; i < e; i++) {
        for (int k = 0; k < 3; k++) {
            nd.lo[k] = std::min(nd.lo[k], it[i].lo[k]);
            nd.hi[k] = std::max(nd.hi[k], it[i].hi[k]);
            clo[k] = std::min(clo[k], it[i].c[k]);
            chi[k] = std::max(chi[k], it[i].c[k]);
        }
        nd.min_rank = std::min(nd.min_rank, it[i].rank);
    }
    const int id = (int)T.size();
    T.push_back(nd);
    if (e - b <= 2) return id;
    constexpr int NB = 16;
    auto area = [](const float* lo, const float* hi) {
        float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        return dx * dy + dy * dz + dz * dx;
    };
    auto bin_of = [&](const FastItem& q, int ax) {   // a non-finite centroid (uploaded NaN / inf) to an end bin
        const float f = (q.c[ax] - clo[ax]) / (chi[ax] - clo[ax]) * NB;
        return f >= (float)NB ? NB - 1 : (f >= 0.0f ? (int)f : 0);
    };
    float best = INFINITY;
    int bax = -1, bsplit = 0;
    for (int ax = 0; ax < 3; ax++) {
        if (!(chi[ax] - clo[ax] > 0.0f)) continue;
        int cnt[NB] = {0};
        float blo[NB][3], bhi[NB][3];
        for (int s = 0; s < NB; s++)
            for (int k = 0; k < 3; k++) {
                blo[s][k] = INFINITY;
                bhi[s][k] = -INFINITY;
            }
        for (int i = b; i < e; i++) {
            const int s = bin_of(it[i], ax);
            cnt[s]++;
            for (int k = 0; k < 3; k++) {
                blo[s][k] = std::min(blo[s][k], it[i].lo[k]);
                bhi[s][k] = std::max(bhi[s][k], it[i].hi[k]);
            }
        }
        float lA[NB], llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        int lN[NB], n = 0;
        for (int s = 0; s < NB; s++) {
            n += cnt[s];
            for (int k = 0; k < 3; k++) {
                llo[k] = std::min(llo[k], blo[s][k]);
                lhi[k] = std::max(lhi[k], bhi[s][k]);
            }
            lN[s] = n;
            lA[s] = n ? area(llo, lhi) : 0.0f;
        }
        float rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        int rn = 0;
        for (int s = NB - 1; s >= 1; s--) {   // bins < s left, >= s right
            rn += cnt[s];
            for (int k = 0; k < 3; k++) {
                rlo[k] = std::min(rlo[k], blo[s][k]);
                rhi[k] = std::max(rhi[k], bhi[s][k]);
            }
            const int ln = lN[s - 1];
            if (ln == 0 || rn == 0) continue;
            const float cost = lA[s - 1] * ln + area(rlo, rhi) * rn;
            if (cost < best) {
                best = cost;
                bax = ax;
                bsplit = s;
            }
        }
    }
    int mid = b;
    if (bax >= 0) {
        auto pm = std::partition(it.begin() + b, it.begin() + e,
                                 [&](const FastItem& q) { return bin_of(q, bax) < bsplit; });
        mid = (int)(pm - it.begin());
    }
    if (mid == b || mid == e) {   // coincident centroids: halve the range along the widest axis
        int ax = 0;
        for (int k = 1; k < 3; k++)
            if (chi[k] - clo[k] > chi[ax] - clo[ax]) ax = k;
        mid = (b + e) / 2;
        std::nth_element(it.begin() + b, it.begin() + mid, it.begin() + e,
                         [ax](const FastItem& x, const FastItem& y) { return x.c[ax] < y.c[ax]; });
        bax = ax;
    }
    const int l = fast_build_node(it, b, mid, T);
    const int r = fast_build_node(it, mid, e, T);
    T[id].kid[0] = l;
    T[id].kid[1] = r;
    T[id].axis = bax;
    return id;
}

void fast_emit(const std::vector<FastNode>& T, const std::vector<FastItem>& it, int n, int oct, const FastTables& F,
               std::vector<rt_dnode>& out) {
    const int k = (int)out.size();
    out.emplace_back();
    const FastNode& s = T[n];
    rt_dnode d;
    d.xmin = s.lo[0]; d.xmax = s.hi[0];
    d.ymin = s.lo[1]; d.ymax = s.hi[1];
    d.zmin = s.lo[2]; d.zmax = s.hi[2];
    uint32_t bits = 0;
    d.prims = 0;
    for (int t = 0; t < F.fl_n; t++)
        if (s.min_rank < F.fl_rank[t]) bits |= 1u << (24 + t);
    if (s.kid[0] < 0) {
        for (int j = 0; j < s.count; j++) {
            const FastItem& q = it[s.first + j];
            bits |= (uint32_t)q.type << (16 + 4 * j);
            d.prims |= (uint32_t)q.idx << (16 * j);
        }
    } else {
        const int f = (oct >> s.axis) & 1;
        fast_emit(T, it, s.kid[f], oct, F, out);
        fast_emit(T, it, s.kid[1 - f], oct, F, out);
    }
    d.meta = bits | (uint32_t)out.size();   // skip = end of this subtree (END patched by the caller)
    out[k] = d;
}

// Two-child layout of tree T (FastTables::inner2 / leaves2).  Returns false when
// a reference does not fit the 16-bit stack entries.
int fast_ref(const std::vector<FastNode>& T, const std::vector<FastItem>& it, int n, FastTables& F, int depth);
bool fast_two_child(const std::vector<FastNode>& T, const std::vector<FastItem>& it, FastTables& F) {
    F.inner2.clear();
    F.leaves2.clear();
    F.depth = 0;
    fast_ref(T, it, 0, F, 1);
    return F.inner2.size() / 4 < 32768 && F.leaves2.size() <= 32768;
}
int fast_ref(const std::vector<FastNode>& T, const std::vector<FastItem>& it, int n, FastTables& F, int depth) {
    const FastNode& s = T[n];
    F.depth = std::max(F.depth, depth);
    if (s.kid[0] < 0) {
        uint2 lf = make_uint2(0u, 0u);
        for (int j = 0; j < s.count; j++) {
            lf.x |= (uint32_t)it[s.first + j].type << (16 + 4 * j);
            lf.y |= (uint32_t)it[s.first + j].idx << (16 * j);
        }
        F.leaves2.push_back(lf);
        return ~(int)(F.leaves2.size() - 1);
    }
    const int k = (int)(F.inner2.size() / 4);
    F.inner2.resize(F.inner2.size() + 4);
    const int rl = fast_ref(T, it, s.kid[0], F, depth + 1);
    const int rr = fast_ref(T, it, s.kid[1], F, depth + 1);
    const FastNode& L = T[s.kid[0]];
    const FastNode& R = T[s.kid[1]];
    uint32_t bits = 0;
    for (int t = 0; t < F.fl_n; t++) {
        if (L.min_rank < F.fl_rank[t]) bits |= 1u << t;
        if (R.min_rank < F.fl_rank[t]) bits |= 1u << (8 + t);
    }
    float4* o = &F.inner2[4 * (size_t)k];
    o[0] = make_float4(L.lo[0], L.hi[0], L.lo[1], L.hi[1]);
    o[1] = make_float4(L.lo[2], L.hi[2], R.lo[0], R.hi[0]);
    o[2] = make_float4(R.lo[1], R.hi[1], R.lo[2], R.hi[2]);
    float a, b, c;
    std::memcpy(&a, &rl, 4);
    std::memcpy(&b, &rr, 4);
    std::memcpy(&c, &bits, 4);
    o[3] = make_float4(a, b, c, 0.0f);
    return k;
}

FastTables build_fast(const std::vector<rt_dnode>& dn, size_t ns, const rt_quad* quads, size_t nq, const rt_box* boxes,
                      size_t nb) {
    FastTables F;
    auto aligned = [](const rt_quad& q) {
        return (q.normal[0] == 0.0f) + (q.normal[1] == 0.0f) + (q.normal[2] == 0.0f) == 2;
    };
    for (size_t i = 0; i < nq; i++)
        if (!aligned(quads[i])) return F;
    for (size_t i = 0; i < nb; i++)
        for (int f = 0; f < 6; f++)
            if (!aligned(boxes[i].quads[f])) return F;
    F.info.assign(ns + nq + nb, 0xFFFFFFFFu);
    F.base[RT_MODEL_SPHERE] = 0;
    F.base[RT_MODEL_QUAD] = (int)ns;
    F.base[RT_MODEL_BOX] = (int)(ns + nq);
    const size_t count[8] = {0, ns, nq, 0, nb, 0, 0, 0};
    std::vector<FastItem> items;
    int rank = 0;
    bool solid_seen = false;
    for (int k = 0; k < (int)dn.size(); k++) {
        const rt_dnode& nd = dn[k];
        if ((nd.meta & 0xF0000u) == 0) continue;   // inner node
        int prev = 0;
        for (int s = 0; s < 2; s++, rank++) {
            const int ty = (int)((nd.meta >> (16 + 4 * s)) & 0xFu), ix = (int)((nd.prims >> (16 * s)) & 0xFFFFu);
            const bool solid = ty == RT_MODEL_SPHERE || ty == RT_MODEL_QUAD || ty == RT_MODEL_BOX;
            if (solid) {
                if ((size_t)ix >= count[ty] || rank > 0xFFFF) return F;
                uint32_t& w = F.info[F.base[ty] + ix];
                if (w == 0xFFFFFFFFu) {   // a prim listed twice keeps its first (earliest) slot
                    w = ((uint32_t)rank << 16) | (uint32_t)k;
                    FastItem q;
                    q.lo[0] = nd.xmin; q.lo[1] = nd.ymin; q.lo[2] = nd.zmin;
                    q.hi[0] = nd.xmax; q.hi[1] = nd.ymax; q.hi[2] = nd.zmax;
                    for (int a = 0; a < 3; a++) q.c[a] = 0.5f * (q.lo[a] + q.hi[a]);
                    q.type = ty;
                    q.idx = ix;
                    q.rank = rank;
                    items.push_back(q);
                }
                solid_seen = true;
            } else if (ty == RT_MODEL_CONSTANT_MEDIUM) {
                if (F.fm_n == 4) return F;
                int tr = -1;
                if (solid_seen) {
                    if (F.fl_n == 2) return F;
                    tr = F.fl_n++;
                    F.fl_medium[tr] = ix;
                    F.fl_rank[tr] = rank;
                }
                const int j = F.fm_n++;
                F.fm_medium[j] = ix;
                F.fm_leaf[j] = k;
                F.fm_track[j] = tr;
                const bool prev_solid = prev == RT_MODEL_SPHERE || prev == RT_MODEL_QUAD || prev == RT_MODEL_BOX;
                F.fm_flags[j] = (s == 1 && prev == RT_MODEL_CONSTANT_MEDIUM ? 1 : 0) | (s == 1 && prev_solid ? 2 : 0);
            }
            prev = ty;
        }
    }
    if (!items.empty()) {
        std::vector<FastNode> T;
        T.reserve(2 * items.size());
        fast_build_node(items, 0, (int)items.size(), T);
        for (int oct = 0; oct < 8; oct++) {
            std::vector<rt_dnode> out;
            fast_emit(T, items, 0, oct, F, out);
            if (out.size() >= RT_NODE_END) return F;
            for (rt_dnode& d : out)
                if ((d.meta & 0xFFFFu) == out.size()) d.meta = (d.meta & ~0xFFFFu) | RT_NODE_END;
            F.n_per = (int)out.size();
            F.nodes.insert(F.nodes.end(), out.begin(), out.end());
        }
        if (!fast_two_child(T, items, F)) return F;   // the same tree for the stack walk (variant 61)
    }
    F.ok = true;
    return F;
}

// Intersection-only record of one quad face (rt_device.h, RT_DFACE_F4): the
// plane (normal, d) and the 2-D Cramer system of hit_quad (hitting.glsl:90-122)
// with its axis pair and delta precomputed by the same float expressions.
void face_record(const rt_quad& q, float4 out[3]) {
    const float* u = q.u;
    const float* v = q.v;
    float delta;
    int a, b, cs;
    if ((delta = u[0] * v[1] - u[1] * v[0]) != 0.0f) { a = 0; b = 1; cs = 0; }
    else if ((delta = u[0] * v[2] - u[2] * v[0]) != 0.0f) { a = 0; b = 2; cs = 1; }
    else { delta = u[1] * v[2] - u[2] * v[1]; a = 1; b = 2; cs = 2; }
    float csf;
    std::memcpy(&csf, &cs, 4);
    out[0] = make_float4(q.normal[0], q.normal[1], q.normal[2], q.d);
    out[1] = make_float4(q.q[a], q.q[b], u[a], u[b]);
    out[2] = make_float4(v[a], v[b], delta, csf);
}

// The compact record of a box with Box.java's axis-aligned layout (rt_kernel.hip
// box_test_compact, rt_device.h RT_BOXC_F4): its corners mn / mx as its faces' q carry
// them (Box.java:32-37) and its faces' normal components along z, x, y.  The kernel
// rebuilds every value its canonical test reads from these with the operations below;
// the record is kept (out[2].y = 1) only when each rebuilt value equals the one the
// uploaded faces give (face_record, the canonical planes), else the box takes the
// full record path.  Float equality: the sign of a zero is the one freedom, and no
// result depends on it (box_test_compact).
bool compact_box(const rt_quad* Q, float4 out[3]) {
    const float mnx = Q[0].q[0], mny = Q[0].q[1], mxz = Q[0].q[2], mxx = Q[1].q[0], mnz = Q[2].q[2],
                mxy = Q[4].q[1];
    const float sz = Q[0].normal[2], sx = Q[1].normal[0], sy = Q[4].normal[1];
    out[0] = make_float4(mnx, mny, mnz, mxx);
    out[1] = make_float4(mxy, mxz, sz, sx);
    // z: quads[0]'s texture id, w: the sign bits of each face normal's two zero components
    // (bits 2i, 2i+1: components (axis+1)%3, (axis+2)%3 of face i), so the shading can rebuild
    // every face normal's exact bits from the record (rt_kernel.hip boxc_normal)
    uint32_t zmask = 0;
    {
        static const int kAxS[6] = {2, 0, 2, 0, 1, 1};
        for (int i = 0; i < 6; i++)
            for (int j = 1; j <= 2; j++)
                if (std::signbit(Q[i].normal[(kAxS[i] + j) % 3])) zmask |= 1u << (2 * i + j - 1);
    }
    float texf, zmf;
    std::memcpy(&texf, &Q[0].texture_id, 4);
    std::memcpy(&zmf, &zmask, 4);
    out[2] = make_float4(sy, 0.0f, texf, zmf);
    static const int kAx[6] = {2, 0, 2, 0, 1, 1};   // Box.java:32-37 face order: normals along z, x, z, x, y, y
    const float sv[6] = {sz, sx, -sz, -sx, sy, -sy};
    const float qk[6] = {mxz, mxx, mnz, mnx, mxy, mny};
    const float DX = mxx - mnx, DY = mxy - mny, DZ = mxz - mnz;
    auto cs = [](int c) {
        float x;
        std::memcpy(&x, &c, 4);
        return x;
    };
    // box_test_compact's per-face systems (boxc_face)
    const float4 A[6] = {make_float4(mnx, mny, DX, 0.0f), make_float4(mny, mxz, 0.0f, -DZ),
                         make_float4(mxx, mny, -DX, 0.0f), make_float4(mny, mnz, 0.0f, DZ),
                         make_float4(mnx, mxz, DX, 0.0f), make_float4(mnx, mnz, DX, 0.0f)};
    const float4 B[6] = {make_float4(0.0f, DY, DX * DY, cs(0)), make_float4(DY, 0.0f, DZ * DY, cs(2)),
                         make_float4(0.0f, DY, -(DX * DY), cs(0)), make_float4(DY, 0.0f, -(DZ * DY), cs(2)),
                         make_float4(0.0f, -DZ, -(DX * DZ), cs(1)), make_float4(0.0f, DZ, DX * DZ, cs(1))};
    auto same = [](float4 a, float4 b) { return a.x == b.x && a.y == b.y && a.z == b.z && a.w == b.w; };
    for (int i = 0; i < 6; i++) {
        const rt_quad& q = Q[i];
        const int ax = kAx[i];
        for (int k = 0; k < 3; k++)
            if (!std::isfinite(q.normal[k]) || !std::isfinite(q.q[k]) || !std::isfinite(q.u[k]) || !std::isfinite(q.v[k]))
                return false;
        // the canonical plane: normal (s_i along its axis, zeros elsewhere), d = s_i * q_k
        if (q.normal[ax] != sv[i] || sv[i] == 0.0f || q.normal[(ax + 1) % 3] != 0.0f || q.normal[(ax + 2) % 3] != 0.0f)
            return false;
        if (q.d != sv[i] * qk[i]) return false;
        float4 f[3];
        face_record(q, f);
        uint32_t c0, c1;
        std::memcpy(&c0, &f[2].w, 4);
        std::memcpy(&c1, &B[i].w, 4);
        if (!same(f[1], A[i]) || f[2].x != B[i].x || f[2].y != B[i].y || f[2].z != B[i].z || c0 != c1) return false;
    }
    out[2].y = 1.0f;
    return true;
}

// A box's bounds (dboxes[21..22]): min / max over its faces' corners, rounded to float.
void box_bounds(const rt_quad* Q, float4 out[2]) {
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = 0; i < 6; i++)
        for (int k = 0; k < 3; k++)
            for (int cu = 0; cu < 2; cu++)
                for (int cv = 0; cv < 2; cv++) {
                    const double x = (double)Q[i].q[k] + cu * (double)Q[i].u[k] + cv * (double)Q[i].v[k];
                    lo[k] = std::min(lo[k], x);
                    hi[k] = std::max(hi[k], x);
                }
    out[0] = make_float4((float)lo[0], (float)hi[0], (float)lo[1], (float)hi[1]);
    out[1] = make_float4((float)lo[2], (float)hi[2], 0.0f, 0.0f);
}

// A box's 48-byte record (rt_kernel.hip leaf_prims_t): compact (compact_box) or, when its
// faces cannot be rebuilt from one, just its bounds (dboxes[21..22]) for the pre-test.
bool box_record(const rt_quad* Q, const float4 bounds[2], float4 rb[RT_BOXC_F4]) {
    if (compact_box(Q, rb)) return true;
    rb[0] = make_float4(bounds[0].x, bounds[0].z, bounds[1].x, bounds[0].y);
    rb[1] = make_float4(bounds[0].w, bounds[1].y, 0.0f, 0.0f);
    rb[2] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    return false;
}

// The scene side of the shared-reciprocal division regime (rt_kernel.hip rcp_nr /
// div_nr): coordinates within 2^20 (so are the rays' origins and directions: hit
// points, camera rays, scatter and light-sampling directions), a face's delta
// normal within [2^-60, 2^20].
bool fd_coord(float x) { return std::fabs(x) <= 1048576.0f; }
bool fd_face(const float4 f[3]) {
    const float ad = std::fabs(f[2].z);
    return fd_coord(f[0].w) && fd_coord(f[1].x) && fd_coord(f[1].y) && fd_coord(f[1].z) && fd_coord(f[1].w) &&
           fd_coord(f[2].x) && fd_coord(f[2].y) && ad >= 0x1p-60f && ad <= 0x1p20f;
}

// Max |coordinate| a ray origin or hit point can have: every record's reach (sphere
// centre + motion + radius, quad / box corners) and the camera block.
float scene_extent(const rt_ctx* c) {
    double b = 0.0;
    const auto& S = c->host_buf[RT_BIND_SPHERES];
    for (size_t k = 0; k < S.size() / sizeof(rt_sphere); k++) {
        const rt_sphere& sp = ((const rt_sphere*)S.data())[k];
        for (int i = 0; i < 3; i++)
            b = std::max(b, std::fabs((double)sp.center1[i]) + std::fabs((double)sp.center_vec[i]) +
                                std::fabs((double)sp.radius));
    }
    for (int bind : {RT_BIND_QUADS, RT_BIND_BOXES}) {
        const auto& Q = c->host_buf[bind];
        for (size_t k = 0; k < Q.size() / sizeof(rt_quad); k++) {
            const rt_quad& q = ((const rt_quad*)Q.data())[k];
            for (int i = 0; i < 3; i++)
                b = std::max(b, std::fabs((double)q.q[i]) + std::fabs((double)q.u[i]) + std::fabs((double)q.v[i]));
        }
    }
    const float* cam = (const float*)&c->cam;
    for (int i = 0; i < 28; i++) b = std::max(b, std::fabs((double)cam[i]));
    return b < 1e30 ? (float)b : INFINITY;
}

// The fast mode's tree (bvh_sah.h) over the uploaded BVH's prims; child order: the one nearer the
// camera first.
int build_sah(rt_ctx* c, std::vector<rt_bvh_node>& out) {
    rt_sah::Input in;
    in.sph = (const rt_sphere*)c->host_buf[RT_BIND_SPHERES].data();
    in.n_sph = c->host_buf[RT_BIND_SPHERES].size() / sizeof(rt_sphere);
    in.quad = (const rt_quad*)c->host_buf[RT_BIND_QUADS].data();
    in.n_quad = c->host_buf[RT_BIND_QUADS].size() / sizeof(rt_quad);
    in.med = (const rt_medium*)c->host_buf[RT_BIND_MEDIA].data();
    in.n_med = c->host_buf[RT_BIND_MEDIA].size() / sizeof(rt_medium);
    in.box = (const rt_box*)c->host_buf[RT_BIND_BOXES].data();
    in.n_box = c->host_buf[RT_BIND_BOXES].size() / sizeof(rt_box);
    in.ref = (const rt_bvh_node*)c->host_buf[RT_BIND_BVH].data();
    in.n_ref = c->host_buf[RT_BIND_BVH].size() / sizeof(rt_bvh_node);
    rt_sah::Builder b(in, 2, c->cam.camera_pos);
    if (!b.build(out)) return set_err(c, RT_ERR_INVALID_ARG, "SAH BVH: the uploaded BVH's prims cannot be rebuilt");
    if (out.size() > RT_MAX_RECORDS) return set_err(c, RT_ERR_LIMIT, "SAH BVH exceeds 65535 nodes");
    return RT_OK;
}

int validate(rt_ctx* c) {
    if (c->validated) return RT_OK;
    size_t ns = c->host_buf[RT_BIND_SPHERES].size() / sizeof(rt_sphere);
    size_t nq = c->host_buf[RT_BIND_QUADS].size() / sizeof(rt_quad);
    size_t nb = c->host_buf[RT_BIND_BOXES].size() / sizeof(rt_box);
    size_t nm = c->host_buf[RT_BIND_MEDIA].size() / sizeof(rt_medium);
    auto check_ref = [&](int type, int idx) -> bool {
        switch (type) {
            case RT_MODEL_SPHERE: return (size_t)idx < ns;
            case RT_MODEL_QUAD: return (size_t)idx < nq;
            case RT_MODEL_BOX: return (size_t)idx < nb;
            case RT_MODEL_CONSTANT_MEDIUM: return (size_t)idx < nm;
            default: return true;   // unknown types never hit (hit_model returns false)
        }
    };
    const rt_bvh_node* nodes = (const rt_bvh_node*)c->host_buf[RT_BIND_BVH].data();
    size_t nn = c->host_buf[RT_BIND_BVH].size() / sizeof(rt_bvh_node);
    for (size_t i = 0; i < nn; i++) {
        int lt = nodes[i].left_id & 0xFFFF;
        if (lt == 0) continue;
        if (!check_ref(lt, (nodes[i].left_id >> 16) & 0xFFFF) || !check_ref(nodes[i].right_id & 0xFFFF, (nodes[i].right_id >> 16) & 0xFFFF))
            return set_err(c, RT_ERR_INVALID_ARG, "BVH leaf references a missing record");
    }
    const rt_medium* media = (const rt_medium*)c->host_buf[RT_BIND_MEDIA].data();
    c->uv_always = false;
    for (size_t i = 0; i < nm; i++) {
        int bt = media[i].boundary_type;
        if (bt == RT_MODEL_CONSTANT_MEDIUM) return set_err(c, RT_ERR_INVALID_ARG, "medium boundary cannot be a medium");
        if (!check_ref(bt, media[i].boundary_idx) || media[i].boundary_idx < 0)
            return set_err(c, RT_ERR_INVALID_ARG, "medium boundary references a missing record");
        if (((media[i].texture_id >> 28) & 0xF) == RT_TEXTYPE_IMAGE) c->uv_always = true;
    }
    const std::vector<uint8_t>& L = c->host_buf[RT_BIND_LIGHTS];
    if (L.size() >= 4) {
        int32_t count;
        std::memcpy(&count, L.data(), 4);
        if (count < 0 || (size_t)(count + 1) * 4 > L.size()) return set_err(c, RT_ERR_INVALID_ARG, "lights count exceeds buffer");
        for (int i = 0; i < count; i++) {
            int32_t p;
            std::memcpy(&p, L.data() + 4 + 4 * i, 4);
            int t = (p >> 16) & 0xFFFF, ix = p & 0xFFFF;
            if ((t == RT_MODEL_SPHERE || t == RT_MODEL_QUAD) && !check_ref(t, ix))
                return set_err(c, RT_ERR_INVALID_ARG, "light references a missing record");
        }
    }
    // exact near-first walk tables (variant 60): rebuilt after every upload
    const std::vector<uint8_t>& QB = c->host_buf[RT_BIND_QUADS];
    const std::vector<uint8_t>& BB = c->host_buf[RT_BIND_BOXES];
    c->fast = build_fast(c->dnodes, ns, (const rt_quad*)QB.data(), nq, (const rt_box*)BB.data(), nb);
    c->fast.ok = c->fast.ok && c->spec_ok && !c->uv_always;
    if (c->bvh_mode == RT_BVH_SAH) {
        std::vector<rt_bvh_node> sah;
        int r = build_sah(c, sah);
        if (r) return r;
        std::vector<rt_dnode> dn;
        r = thread_bvh(c, sah.data(), (int)sah.size(), dn);
        if (r) return r;
        c->links = build_links(dn);
        c->n_link_nodes = (int)dn.size();
        c->sah_bvh.assign((const uint8_t*)sah.data(), (const uint8_t*)(sah.data() + sah.size()));
        c->walk_dn.swap(dn);
    } else {
        c->links = build_links(c->dnodes);
        c->n_link_nodes = c->n_dnodes;
        c->sah_bvh.clear();
        c->walk_dn = c->dnodes;
    }
    c->walk_stale = true;
    c->pair_leaves = -1;
    c->fast_gen++;
    c->validated = true;
    return RT_OK;
}

int alloc_image(rt_ctx* c, Device& d) {
    HIPCHK(c, hipSetDevice(d.id));
    HIPCHK(c, hipStreamSynchronize(d.stream));
    d.local_rows = local_rows_of(c->height, d.rank, d.world, c->stripe_rows);
    d.padded_rows = padded_rows_of(c->height, d.world, c->stripe_rows);
    size_t bytes = (size_t)d.padded_rows * c->width * 16;
    dev_free(d.image);
    if (bytes) {
        HIPCHK(c, hipMalloc(&d.image.ptr, bytes));
        d.image.bytes = bytes;
        HIPCHK(c, hipMemsetAsync(d.image.ptr, 0, bytes, d.stream));
        HIPCHK(c, hipStreamSynchronize(d.stream));
    }
    d.image_ptr = (float*)d.image.ptr;
    d.image_bound = false;
    return RT_OK;
}

int ensure(rt_ctx* c, Device& d, DevBuf& b, size_t n) {
    if (b.bytes >= n) return RT_OK;
    dev_free(b);
    HIPCHK(c, hipSetDevice(d.id));
    HIPCHK(c, hipMalloc(&b.ptr, n));
    b.bytes = n;
    return RT_OK;
}

#define NCCLCHK(ctx, call)                                                                               \
    do {                                                                                                 \
        ncclResult_t e_ = (call);                                                                        \
        if (e_ != ncclSuccess)                                                                           \
            return set_err(ctx, RT_ERR_DEVICE, std::string(#call) + ": " + rccl().GetErrorString(e_));    \
    } while (0)

// Runs the calls between ncclGroupStart and ncclGroupEnd and closes the group whatever they
// return, so a failed Send / Recv / copy does not leave a group open on this thread (later
// RCCL calls would be queued into it).  The body's error wins over GroupEnd's.  On an error the
// context's communicators are then aborted (ncclCommAbort): the group may have
// submitted a Send whose Recv was never queued (or the reverse), and a later stream
// synchronisation would wait on that unmatched peer forever; aborting frees the queued work and
// the next gather needs rt_comm_init (one process per GPU) or a fresh ncclCommInitAll.
void abort_comms(rt_ctx* c);
template <class F>
int group_body(rt_ctx* c, F&& body) {
    const int r = body();
    ncclResult_t e = rccl().GroupEnd();
    if (e == ncclInProgress && c->comm_nonblocking) e = ncclSuccess;   // completed by comm_wait
    if (r || e != ncclSuccess) abort_comms(c);
    if (r) return r;
    if (e != ncclSuccess) return set_err(c, RT_ERR_DEVICE, std::string("ncclGroupEnd: ") + rccl().GetErrorString(e));
    return RT_OK;
}

// Frees the context's communicators and whatever they still have queued: ncclCommAbort, or
// ncclCommDestroy where the library lacks it (a communicator is never just dropped).
void abort_comms(rt_ctx* c) {
    for (Device& d : c->devs) {
        if (!d.comm) continue;
        if (rccl().CommAbort) (void)rccl().CommAbort(d.comm);
        else (void)rccl().CommDestroy(d.comm);
        d.comm = nullptr;
    }
    c->proc_comm = false;
    c->comm_nonblocking = false;
    c->comm_tried = false;   // a multi-device context makes its communicators again on the next gather
}

// Deadlines of the one-process-per-GPU exchange.  A peer that never joins
// (ncclCommInitRank) or never posts its matching Send / Recv would otherwise hold the host
// forever; with a deadline the call returns RT_ERR_TIMEOUT after aborting the communicator,
// which also ends its queued kernels, and the caller falls back or reports.
using Clock = std::chrono::steady_clock;
Clock::time_point comm_deadline(const rt_ctx* c) {
    return c->comm_timeout_ms > 0 ? Clock::now() + std::chrono::milliseconds(c->comm_timeout_ms)
                                  : Clock::time_point::max();
}

int comm_timeout(rt_ctx* c, const std::string& what) {
    abort_comms(c);
    return set_err(c, RT_ERR_TIMEOUT, what + ": no completion within " + std::to_string(c->comm_timeout_ms) +
                                          " ms (the communicator was aborted; rt_comm_init again)");
}

// The state of a non-blocking communicator's last operation: RT_OK once it is no longer
// ncclInProgress, RT_ERR_DEVICE (communicator aborted) on an asynchronous error, RT_ERR_TIMEOUT
// past the deadline.  A blocking communicator has nothing to wait for.
int comm_wait(rt_ctx* c, ncclComm_t comm, Clock::time_point deadline, const char* what) {
    if (!c->comm_nonblocking || !rccl().CommGetAsyncError) return RT_OK;
    for (;;) {
        ncclResult_t st = ncclSuccess;
        const ncclResult_t e = rccl().CommGetAsyncError(comm, &st);
        if (e != ncclSuccess) st = e;
        if (st == ncclSuccess) return RT_OK;
        if (st != ncclInProgress) {
            abort_comms(c);
            return set_err(c, RT_ERR_DEVICE, std::string(what) + ": " + rccl().GetErrorString(st));
        }
        if (Clock::now() >= deadline) return comm_timeout(c, what);
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}

// hipStreamSynchronize with the deadline: polls the stream (and the communicator's asynchronous
// error) instead of blocking in the runtime.
int stream_wait(rt_ctx* c, Device& d, Clock::time_point deadline, const char* what) {
    for (;;) {
        const hipError_t e = hipStreamQuery(d.stream);
        if (e == hipSuccess) return RT_OK;
        if (e != hipErrorNotReady) {
            abort_comms(c);
            return set_err(c, RT_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
        }
        if (d.comm && c->comm_nonblocking && rccl().CommGetAsyncError) {
            ncclResult_t st = ncclSuccess;
            if (rccl().CommGetAsyncError(d.comm, &st) == ncclSuccess && st != ncclSuccess && st != ncclInProgress) {
                abort_comms(c);
                return set_err(c, RT_ERR_DEVICE, std::string(what) + ": " + rccl().GetErrorString(st));
            }
        }
        if (Clock::now() >= deadline) return comm_timeout(c, what);
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}

// Multi-device context: device k's stripe block (local_rows x W, in its padded slot) into
// device 0's gather buffer, then the de-interleave kernel into device 0's full image.
// RCCL (ncclCommInitAll over the context's devices, one ncclSend per device k > 0 and the
// matching ncclRecv on device 0, grouped) when the device ids are distinct and RCCL
// loads; peer copies otherwise (several slots on one device: RCCL allows one rank per
// device).  The renders were synchronised by the caller.
int device_gather(rt_ctx* c) {
    const int ndev = (int)c->devs.size();
    const int padded = padded_rows_of(c->height, ndev, c->stripe_rows);
    const size_t slot = (size_t)padded * c->width * 16;
    Device& d0 = c->devs[0];
    if (ensure(c, d0, d0.gather, slot * ndev) || ensure(c, d0, d0.full, (size_t)c->height * c->width * 16))
        return RT_ERR_DEVICE;
    if (!c->comm_tried) {
        c->comm_tried = true;
        bool distinct = true;
        for (int i = 0; i < ndev; i++)
            for (int j = 0; j < i; j++) distinct = distinct && c->devs[i].id != c->devs[j].id;
        if (distinct && rccl().ok) {
            std::vector<ncclComm_t> comms(ndev, nullptr);
            std::vector<int> ids(ndev);
            for (int k = 0; k < ndev; k++) ids[k] = c->devs[k].id;
            if (rccl().CommInitAll(comms.data(), ndev, ids.data()) == ncclSuccess)
                for (int k = 0; k < ndev; k++) c->devs[k].comm = comms[k];
        }
    }
    if (d0.comm) {
        NCCLCHK(c, rccl().GroupStart());
        // the group is closed on every path: an error inside it is returned after GroupEnd
        int in_group = group_body(c, [&]() -> int {
            for (int k = 0; k < ndev; k++) {
                Device& d = c->devs[k];
                const size_t n = (size_t)d.local_rows * c->width * 4;   // floats of the block
                char* dst = (char*)d0.gather.ptr + slot * k;
                HIPCHK(c, hipSetDevice(d.id));
                if (k == 0) {
                    HIPCHK(c, hipMemcpyAsync(dst, d.image_ptr, n * 4, hipMemcpyDeviceToDevice, d0.stream));
                } else if (n) {
                    NCCLCHK(c, rccl().Send(d.image_ptr, n, ncclFloat, 0, d.comm, d.stream));
                    NCCLCHK(c, rccl().Recv(dst, n, ncclFloat, k, d0.comm, d0.stream));
                }
            }
            return RT_OK;
        });
        if (in_group) return in_group;
        for (Device& d : c->devs) {
            HIPCHK(c, hipSetDevice(d.id));
            HIPCHK(c, hipStreamSynchronize(d.stream));
        }
        c->gather_path = RT_GATHER_RCCL;
    } else {
        HIPCHK(c, hipSetDevice(d0.id));
        for (int k = 0; k < ndev; k++) {
            Device& d = c->devs[k];
            HIPCHK(c, hipMemcpyPeerAsync((char*)d0.gather.ptr + slot * k, d0.id, d.image_ptr, d.id,
                                         (size_t)d.local_rows * c->width * 16, d0.stream));
        }
        c->gather_path = RT_GATHER_PEER;
    }
    HIPCHK(c, hipSetDevice(d0.id));
    if (rt_launch_deinterleave(d0.gather.ptr, d0.full.ptr, c->width, c->height, ndev, c->stripe_rows, padded,
                               d0.stream))
        return set_err(c, RT_ERR_DEVICE, "de-interleave kernel launch failed");
    HIPCHK(c, hipStreamSynchronize(d0.stream));
    return RT_OK;
}

}  // namespace

extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }

// ---- one process per GPU: RCCL behind the ABI (rt.h rt_comm_*) ----------------
int rt_comm_unique_id(void* id_out) {
    if (!id_out) return RT_ERR_INVALID_ARG;
    if (!rccl().ok) return RT_ERR_DEVICE;
    ncclUniqueId id;
    if (rccl().GetUniqueId(&id) != ncclSuccess) return RT_ERR_DEVICE;
    static_assert(sizeof(ncclUniqueId) == RT_COMM_ID_BYTES, "ncclUniqueId is 128 bytes");
    std::memcpy(id_out, &id, sizeof(id));
    return RT_OK;
}

int rt_comm_init(rt_ctx* c, const void* id, int rank, int world) {
    if (!c || !id) return RT_ERR_INVALID_ARG;
    if (c->devs.size() != 1) return set_err(c, RT_ERR_STATE, "rt_comm_init needs a 1-device context");
    if (world != c->proc_world || rank != c->proc_rank)
        return set_err(c, RT_ERR_STATE, "rt_comm_init: rank / world differ from rt_set_partition's");
    if (!rccl().ok) return set_err(c, RT_ERR_DEVICE, "RCCL (librccl.so) could not be loaded");
    Device& d = c->devs[0];
    HIPCHK(c, hipSetDevice(d.id));
    if (d.comm) {
        (void)rccl().CommDestroy(d.comm);
        d.comm = nullptr;
    }
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    const Clock::time_point deadline = comm_deadline(c);
    if (rccl().CommInitRankConfig && rccl().CommGetAsyncError && rccl().CommAbort) {
        // non-blocking: ncclCommInitRankConfig returns at once and the init is polled against the
        // deadline, so a rank that never joins cannot hold this one
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.blocking = 0;
        const ncclResult_t e = rccl().CommInitRankConfig(&d.comm, world, uid, rank, &cfg);
        if (e != ncclSuccess && e != ncclInProgress) {
            if (d.comm) (void)rccl().CommAbort(d.comm);
            d.comm = nullptr;
            return set_err(c, RT_ERR_DEVICE, std::string("ncclCommInitRankConfig: ") + rccl().GetErrorString(e));
        }
        c->comm_nonblocking = true;
        c->proc_comm = true;
        const int r = comm_wait(c, d.comm, deadline, "ncclCommInitRankConfig");
        if (r) return r;
    } else {
        NCCLCHK(c, rccl().CommInitRank(&d.comm, world, uid, rank));
        c->comm_nonblocking = false;
        c->proc_comm = true;
    }
    return RT_OK;
}

int rt_comm_set_timeout(rt_ctx* c, int timeout_ms) {
    if (!c) return RT_ERR_INVALID_ARG;
    if (timeout_ms < 0) return set_err(c, RT_ERR_INVALID_ARG, "rt_comm_set_timeout: negative timeout");
    c->comm_timeout_ms = timeout_ms;
    return RT_OK;
}

int rt_comm_abort(rt_ctx* c) {
    if (!c) return RT_ERR_INVALID_ARG;
    abort_comms(c);
    return RT_OK;
}

int rt_gather_image(rt_ctx* c, float* rgba) {
    if (!c) return RT_ERR_INVALID_ARG;
    if (c->width <= 0) return set_err(c, RT_ERR_STATE, "no image");
    if (c->devs.size() != 1) {   // a multi-device context gathers in rt_read_image
        if (!rgba) return set_err(c, RT_ERR_INVALID_ARG, "NULL image");
        return rt_read_image(c, rgba);
    }
    Device& d = c->devs[0];
    if (!c->proc_comm || !d.comm) return set_err(c, RT_ERR_STATE, "rt_comm_init before rt_gather_image");
    if (c->proc_rank == 0 && !rgba) return set_err(c, RT_ERR_INVALID_ARG, "rank 0 needs the output image");
    int r = rt_sync(c);
    if (r) return r;
    HIPCHK(c, hipSetDevice(d.id));
    const int world = c->proc_world;
    // every wait below ends by the context's deadline (rt_comm_set_timeout): on a non-blocking
    // communicator the enqueue is polled (comm_wait), and the stream is polled, not synchronised
    const Clock::time_point deadline = comm_deadline(c);
    // rank k sends its local_rows x W block (a bound image holds no more); rank 0 receives
    // it into slot k of the padded gather buffer
    const size_t slot = (size_t)d.padded_rows * c->width * 16;
    if (c->proc_rank == 0) {
        if (ensure(c, d, d.gather, slot * world) || ensure(c, d, d.full, (size_t)c->height * c->width * 16))
            return RT_ERR_DEVICE;
        NCCLCHK(c, rccl().GroupStart());
        int in_group = group_body(c, [&]() -> int {
            HIPCHK(c, hipMemcpyAsync(d.gather.ptr, d.image_ptr, (size_t)d.local_rows * c->width * 16,
                                     hipMemcpyDeviceToDevice, d.stream));
            for (int k = 1; k < world; k++) {
                const size_t nk = (size_t)local_rows_of(c->height, k, world, c->stripe_rows) * c->width * 4;
                if (nk)
                    NCCLCHK(c, rccl().Recv((char*)d.gather.ptr + slot * k, nk, ncclFloat, k, d.comm, d.stream));
            }
            return RT_OK;
        });
        if (in_group) return in_group;
        if ((r = comm_wait(c, d.comm, deadline, "ncclRecv group"))) return r;
        if (rt_launch_deinterleave(d.gather.ptr, d.full.ptr, c->width, c->height, world, c->stripe_rows,
                                   d.padded_rows, d.stream))
            return set_err(c, RT_ERR_DEVICE, "de-interleave kernel launch failed");
        if ((r = stream_wait(c, d, deadline, "ncclRecv"))) return r;
        if ((r = d2h(c, d, rgba, d.full.ptr, (size_t)c->height * c->width * 16))) return r;
    } else {
        const size_t n = (size_t)d.local_rows * c->width * 4;
        if (n) {
            ncclResult_t e = rccl().Send(d.image_ptr, n, ncclFloat, 0, d.comm, d.stream);
            if (e == ncclInProgress && c->comm_nonblocking) e = ncclSuccess;
            if (e != ncclSuccess) {   // a failed Send frees the communicator too
                abort_comms(c);
                return set_err(c, RT_ERR_DEVICE, std::string("ncclSend: ") + rccl().GetErrorString(e));
            }
            if ((r = comm_wait(c, d.comm, deadline, "ncclSend"))) return r;
        }
        if ((r = stream_wait(c, d, deadline, "ncclSend"))) return r;
    }
    c->gather_path = RT_GATHER_RCCL;
    return RT_OK;
}

int rt_gather_path(rt_ctx* c) { return c ? c->gather_path : RT_ERR_INVALID_ARG; }

// Failure of the last context-less call (rt_create) on this thread; rt_last_error(NULL).
namespace { thread_local std::string g_create_err; }

int rt_create(int n_devices, const int* device_ids, rt_ctx** out) {
    auto fail = [](int code, const char* msg) { g_create_err = msg; return code; };
    if (!out) return fail(RT_ERR_INVALID_ARG, "rt_create: NULL out");
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return fail(RT_ERR_DEVICE, "rt_create: no HIP device");
    // Explicit ids may repeat (several stripe slots on one device); without ids, devices 0..n-1.
    if (n_devices <= 0 || n_devices > 64 || (!device_ids && n_devices > count))
        return fail(RT_ERR_INVALID_ARG, "rt_create: bad device count");
    rt_ctx* c = new rt_ctx();
#ifdef RT_AB_KNOBS
    // A/B build only: the structure variants and knobs from the environment (tools/ab_variants.py).
    // The release library reads no environment: its output depends on its inputs alone.
    if (const char* v = std::getenv("RT_KERNEL_VARIANT")) {
        // 0 (default), 37, 30, 61 and their stats twins 39, 38, 31, 69
        // (rt_kernel.hip rt_launch_render); anything else is the default
        const int want = std::atoi(v);
        c->variant = (want == 30 || want == 31 || want == 37 || want == 38 || want == 39 || want == 61 || want == 69)
                         ? want
                         : 0;
    }
    if (const char* v = std::getenv("RT_CHUNK_TARGET")) c->chunk_target = std::max(0, std::atoi(v));
    if (const char* v = std::getenv("RT_STAGE_TILES")) c->stage_tiles = std::max(0, std::atoi(v));
    if (const char* v = std::getenv("RT_STAGED_CHUNK_TARGET")) c->staged_chunk_target = std::max(1, std::atoi(v));
    if (const char* v = std::getenv("RT_FASTDIV")) c->fastdiv = std::atoi(v) != 0;
    if (const char* v = std::getenv("RT_BOX_PRETEST")) c->box_pretest = std::atoi(v) != 0;
    if (const char* v = std::getenv("RT_SM_BATCH")) c->sm_batch = std::max(1, std::min(64, std::atoi(v)));
    if (const char* v = std::getenv("RT_SM_FRAC")) c->sm_frac = std::max(1, std::min(64, std::atoi(v)));
    if (const char* v = std::getenv("RT_WALK_FRAC")) c->walk_frac = std::max(1, std::min(64, std::atoi(v)));
    if (const char* v = std::getenv("RT_SPH_LDS")) c->sph_lds = std::atoi(v) != 0;
    if (const char* v = std::getenv("RT_BIG_WG")) c->big_wg = std::atoi(v) != 0;
    if (const char* v = std::getenv("RT_COMPACT_BOXES")) c->compact_boxes = std::atoi(v) != 0;
    if (const char* v = std::getenv("RT_LDS_NODE_CAP")) c->lds_node_cap = std::max(0, std::atoi(v));
    if (const char* v = std::getenv("RT_DEBUG_FLAGS")) c->debug_flags = std::atoi(v);
#endif
    c->devs.resize(n_devices);
    for (int i = 0; i < n_devices; i++) {
        Device& d = c->devs[i];
        d.id = device_ids ? device_ids[i] : i;
        if (d.id < 0 || d.id >= count) { delete c; return fail(RT_ERR_INVALID_ARG, "rt_create: device id out of range"); }
        d.rank = i;
        d.world = n_devices;
        if (hipSetDevice(d.id) != hipSuccess || hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreate(&d.ev_start) != hipSuccess || hipEventCreate(&d.ev_stop) != hipSuccess) {
            delete c;
            return fail(RT_ERR_DEVICE, "rt_create: stream/event creation failed");
        }
    }
    g_create_err.clear();
    *out = c;
    return RT_OK;
}

int rt_destroy(rt_ctx* c) {
    if (!c) return RT_ERR_INVALID_ARG;
    for (Device& d : c->devs) {
        (void)hipSetDevice(d.id);
        (void)hipStreamSynchronize(d.stream);
        dev_free(d.nodes); dev_free(d.spheres); dev_free(d.quads); dev_free(d.boxes); dev_free(d.media);
        dev_free(d.lights); dev_free(d.image); dev_free(d.args); dev_free(d.stats); dev_free(d.census); dev_free(d.counter);
        dev_free(d.tile_done); dev_free(d.samples); dev_free(d.wbuf); dev_free(d.dquads); dev_free(d.dboxes);
        dev_free(d.finfo); dev_free(d.f2inner); dev_free(d.f2leaves); dev_free(d.links); dev_free(d.dboxc);
        dev_free(d.gather); dev_free(d.full); dev_free(d.perlin_pk); dev_free(d.sflags);
        if (d.comm && rccl().ok) (void)rccl().CommDestroy(d.comm);
        if (d.ring) (void)hipHostFree(d.ring);
        for (auto& e : d.ring_ev)
            if (e) (void)hipEventDestroy(e);
        for (auto& t : d.tex) dev_free(t);
        if (d.ev_start) (void)hipEventDestroy(d.ev_start);
        if (d.ev_stop) (void)hipEventDestroy(d.ev_stop);
        if (d.own_stream && d.stream) (void)hipStreamDestroy(d.stream);
    }
    delete c;
    return RT_OK;
}

const char* rt_last_error(rt_ctx* c) { return c ? c->err.c_str() : g_create_err.c_str(); }

int rt_upload_buffer(rt_ctx* c, int binding, const void* bytes, size_t nbytes) {
    if (!c) return RT_ERR_INVALID_ARG;
    if (binding < 0 || binding > 5) return set_err(c, RT_ERR_INVALID_ARG, "binding must be 0..5");
    if (nbytes && !bytes) return set_err(c, RT_ERR_INVALID_ARG, "NULL bytes");
    static const size_t rec[6] = {sizeof(rt_sphere), sizeof(rt_bvh_node), sizeof(rt_quad), sizeof(rt_medium),
                                  sizeof(rt_box), 4};
    if (nbytes % rec[binding]) return set_err(c, RT_ERR_INVALID_ARG, "size is not a multiple of the std430 record size");
    if (binding != RT_BIND_LIGHTS && nbytes / rec[binding] > RT_MAX_RECORDS)
        return set_err(c, RT_ERR_LIMIT, "more than 65535 records");
    if (binding == RT_BIND_LIGHTS && nbytes < 4) return set_err(c, RT_ERR_INVALID_ARG, "lights buffer needs the count word");
    std::vector<uint8_t> dev_bytes;
    const void* src = bytes;
    size_t n = nbytes;
    // Thread the incoming BVH before anything of the context changes: a rejected
    // BVH leaves the previous one (host copy, threaded nodes, device buffers) intact.
    std::vector<rt_dnode> dn;
    if (binding == RT_BIND_BVH) {
        int r = thread_bvh(c, (const rt_bvh_node*)bytes, (int)(nbytes / sizeof(rt_bvh_node)), dn);
        if (r) return r;
        dev_bytes.assign((uint8_t*)dn.data(), (uint8_t*)dn.data() + dn.size() * sizeof(rt_dnode));
        src = dev_bytes.data();
        n = dev_bytes.size();
    }
    std::vector<uint8_t>& H = c->host_buf[binding];
    H.assign((const uint8_t*)bytes, (const uint8_t*)bytes + nbytes);
    c->uploaded[binding] = true;
    c->validated = false;
    c->scene_extent = -1.0f;
    if (binding == RT_BIND_BVH) {
        c->n_dnodes = (int)dn.size();
        c->spec_ok = boxes_nest(dn);
        c->dnodes.swap(dn);
        c->inj_hits.clear();   // measured node hits belong to the previous tree
        c->inj_walks = 0;
    }
    std::vector<float4> faces;   // intersection-only copy of quads / box sides
    std::vector<float4> boxc;    // compact canonical box records
    int n_cmp = 0;
    if (binding == RT_BIND_QUADS || binding == RT_BIND_BOXES) {
        const rt_quad* qs = (const rt_quad*)bytes;
        size_t nq = nbytes / sizeof(rt_quad);   // a box is 6 consecutive quads
        faces.resize(binding == RT_BIND_QUADS ? nq * RT_DFACE_F4 : (nq / 6) * RT_DBOX_F4);
        bool fd = true;
        if (binding == RT_BIND_QUADS) {
            for (size_t k = 0; k < nq; k++) {
                face_record(qs[k], &faces[k * RT_DFACE_F4]);
                fd = fd && fd_face(&faces[k * RT_DFACE_F4]);
            }
        } else {
            // per box: the 6 planes first, then the 6 (A, B) pairs, then the canonical
            // planes (RT_DBOX_F4 float4)
            c->boxes_canon = true;
            c->boxes_cond = true;
            boxc.assign((nq / 6) * RT_BOXC_F4, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
            for (size_t bx = 0; bx < nq / 6; bx++) {
                float4* o = &faces[bx * RT_DBOX_F4];
                float sw[12];
                for (int i = 0; i < 6; i++) {
                    const rt_quad& Q = qs[bx * 6 + i];
                    // the face test solves alpha, beta on the reference's axis pair (face_record);
                    // |delta| >= half of |u_a v_b| + |u_b v_a| bounds how far a point it accepts
                    // can lie outside the face (a few ulps of the scene's extent)
                    const float* u = Q.u;
                    const float* v = Q.v;
                    int ka = 1, kb = 2;
                    if (u[0] * v[1] - u[1] * v[0] != 0.0f) { ka = 0; kb = 1; }
                    else if (u[0] * v[2] - u[2] * v[0] != 0.0f) { ka = 0; kb = 2; }
                    const double t1 = (double)u[ka] * v[kb], t2 = (double)u[kb] * v[ka];
                    if (!(std::fabs(t1 - t2) >= 0.5 * (std::fabs(t1) + std::fabs(t2))) || t1 == t2)
                        c->boxes_cond = false;
                }
                box_bounds(qs + bx * 6, o + 21);
                for (int i = 0; i < 6; i++) {
                    float4 f[3];
                    face_record(qs[bx * 6 + i], f);
                    fd = fd && fd_face(f);
                    o[i] = f[0];
                    o[6 + 2 * i] = f[1];
                    o[7 + 2 * i] = f[2];
                    // Box.java:32-37 face order: normals along z, x, z, x, y, y
                    static const int kAx[6] = {2, 0, 2, 0, 1, 1};
                    const float* n = qs[bx * 6 + i].normal;
                    const int ax = kAx[i];
                    if (n[ax] == 0.0f || n[(ax + 1) % 3] != 0.0f || n[(ax + 2) % 3] != 0.0f) c->boxes_canon = false;
                    sw[2 * i] = n[ax];
                    sw[2 * i + 1] = qs[bx * 6 + i].d;
                }
                o[18] = make_float4(sw[0], sw[1], sw[2], sw[3]);
                o[19] = make_float4(sw[4], sw[5], sw[6], sw[7]);
                o[20] = make_float4(sw[8], sw[9], sw[10], sw[11]);
                n_cmp += box_record(qs + bx * 6, o + 21, &boxc[bx * RT_BOXC_F4]);
                // the canonical test shares one reciprocal per axis: opposite faces' normals negated
                if (sw[4] != -sw[0] || sw[6] != -sw[2] || sw[10] != -sw[8]) fd = false;
            }
        }
        c->fd_ok[binding] = fd;
        if (binding == RT_BIND_BOXES) {
            c->n_boxc_ok = n_cmp;
            c->boxc_host = boxc;
        }
    }
    if (binding == RT_BIND_SPHERES) {
        const rt_sphere* sp = (const rt_sphere*)bytes;
        bool fd = true;
        const float L = 524288.0f;   // center1 + center_vec * time within 2^20
        for (size_t k = 0; k < nbytes / sizeof(rt_sphere); k++)
            for (int i = 0; i < 3; i++)
                fd = fd && std::fabs(sp[k].center1[i]) <= L && std::fabs(sp[k].center_vec[i]) <= L &&
                     std::fabs(sp[k].radius) <= L;
        c->fd_ok[binding] = fd;
    }
    if (binding == RT_BIND_LIGHTS) {
        src = (const uint8_t*)bytes + 4;
        n = nbytes - 4;
    }
    for (Device& d : c->devs) {
        DevBuf* b = nullptr;
        switch (binding) {
            case RT_BIND_SPHERES: b = &d.spheres; break;
            case RT_BIND_BVH: b = &d.nodes; break;
            case RT_BIND_QUADS: b = &d.quads; break;
            case RT_BIND_MEDIA: b = &d.media; break;
            case RT_BIND_BOXES: b = &d.boxes; break;
            default: b = &d.lights; break;
        }
        int r = dev_alloc_copy(c, d, *b, src, n);
        if (r) return r;
        if (binding == RT_BIND_QUADS || binding == RT_BIND_BOXES) {
            r = dev_alloc_copy(c, d, binding == RT_BIND_QUADS ? d.dquads : d.dboxes, faces.data(),
                               faces.size() * sizeof(float4));
            if (r) return r;
        }
        if (binding == RT_BIND_BOXES) {
            r = dev_alloc_copy(c, d, d.dboxc, boxc.data(), boxc.size() * sizeof(float4));
            if (r) return r;
        }
    }
    return RT_OK;
}

// The packed Perlin table (rt_kernel.hip perlin_noise_pk): 256 float4 (ranvec x y z, perm x |
// perm y << 8 | perm z << 16) from an R32F 6 x 256 texture whose perm columns hold whole
// numbers 0..255; false (and pk empty) for any other texture.
bool perlin_pack(const float* t, int w, int h, std::vector<float4>& pk) {
    pk.clear();
    if (!t || w != 6 || h != 256) return false;
    pk.resize(256);
    for (int r = 0; r < 256; r++) {
        uint32_t packed = 0;
        for (int k = 0; k < 3; k++) {
            const float v = t[r * 6 + 3 + k];
            if (!(v >= 0.0f && v <= 255.0f && v == std::floor(v))) {
                pk.clear();
                return false;
            }
            packed |= (uint32_t)v << (8 * k);
        }
        float pf;
        std::memcpy(&pf, &packed, 4);
        pk[r] = make_float4(t[r * 6], t[r * 6 + 1], t[r * 6 + 2], pf);
    }
    return true;
}

// Per mille of the link-format leaves (build_links) that hold two spheres: the sphere-pair
// kernels' criterion (rt_render: at least 500).
int pair_leaves_permille(const std::vector<float4>& L, int n_nodes) {
    size_t n = 0, pairs = 0;
    const size_t nf4 = 2 * (size_t)n_nodes;
    for (int i = 0; i < n_nodes && L.size() > nf4; i++) {
        uint32_t hs;
        std::memcpy(&hs, &L[2 * (size_t)i + 1].z, 4);
        if (!(hs & RT_LINK_LEAF)) continue;
        const size_t ord = hs & 0x7FFFFFFFu;
        if (nf4 + ord / 2 >= L.size()) continue;
        uint32_t w[4];
        std::memcpy(w, &L[nf4 + ord / 2], 16);
        n++;
        pairs += (w[2 * (ord % 2)] & 0xFFu) == (uint32_t)(RT_MODEL_SPHERE | (RT_MODEL_SPHERE << 4));
    }
    return n ? (int)(1000 * pairs / n) : 0;
}

int rt_upload_texture(rt_ctx* c, int slot, int format, int w, int h, const void* texels) {
    if (!c) return RT_ERR_INVALID_ARG;
    if (slot < 0 || slot >= RT_MAX_TEXTURES) return set_err(c, RT_ERR_LIMIT, "texture slot must be 0..7");
    if (w <= 0 || h <= 0 || !texels) return set_err(c, RT_ERR_INVALID_ARG, "bad texture size or NULL texels");
    if ((size_t)w * h > (size_t)1 << 28) return set_err(c, RT_ERR_LIMIT, "texture too large");
    size_t n = (size_t)w * h;
    std::vector<uint32_t> rgba;
    const void* src = texels;
    size_t bytes = n * 4;
    if (format == RT_TEX_RGB8) {
        rgba.resize(n);
        const uint8_t* p = (const uint8_t*)texels;
        for (size_t i = 0; i < n; i++)
            rgba[i] = (uint32_t)p[3 * i] | ((uint32_t)p[3 * i + 1] << 8) | ((uint32_t)p[3 * i + 2] << 16) | 0xFF000000u;
        src = rgba.data();
    } else if (format != RT_TEX_RGBA8 && format != RT_TEX_R32F) {
        return set_err(c, RT_ERR_INVALID_ARG, "unknown texture format");
    }
    // A Perlin table (texture.glsl:38-77: R32F, 6 x 256, columns ranvec x y z, perm x y z) whose
    // perm entries are whole numbers 0..255 is also kept as 256 float4 (ranvec x y z, the three
    // perm entries packed as bytes 0 / 1 / 2 of the fourth word): the kernel's noise then reads
    // one float4 per lattice corner and needs no float-to-int conversions or bounds checks
    // (every index is & 255 or an xor of bytes), the same values as the reference's texelFetch +
    // int() of the texture (rt_kernel.hip perlin_noise_pk).
    std::vector<float4> pk;
    if (format == RT_TEX_R32F && !perlin_pack((const float*)texels, w, h, pk)) pk.clear();
    for (Device& d : c->devs) {
        int r = dev_alloc_copy(c, d, d.tex[slot], src, bytes);
        if (r) return r;
        if (!pk.empty()) {
            r = dev_alloc_copy(c, d, d.perlin_pk, pk.data(), pk.size() * sizeof(float4));
            if (r) return r;
        }
    }
    if (!pk.empty()) c->perlin_pk_slot = slot;
    else if (c->perlin_pk_slot == slot) c->perlin_pk_slot = -1;
    c->tex_format[slot] = format;
    c->tex_w[slot] = w;
    c->tex_h[slot] = h;
    return RT_OK;
}

int rt_set_camera(rt_ctx* c, const float ubo[28]) {
    if (!c || !ubo) return set_err(c, RT_ERR_INVALID_ARG, "NULL camera");
    std::memcpy(&c->cam, ubo, sizeof(rt_camera_ubo));
    c->have_cam = true;
    c->scene_extent = -1.0f;
    c->fd_cam = true;   // the camera's points and vectors within the fast-division regime's 2^20
    for (int i = 0; i < 28; i++) c->fd_cam = c->fd_cam && fd_coord(ubo[i]);
    if (c->bvh_mode == RT_BVH_SAH) c->validated = false;   // the SAH tree orders children by the camera
    return RT_OK;
}

int rt_set_params(rt_ctx* c, int max_depth, const float background[3], float sqrt_spp, float recip_sqrt_spp) {
    if (!c || !background) return set_err(c, RT_ERR_INVALID_ARG, "NULL background");
    if (max_depth < 0) return set_err(c, RT_ERR_INVALID_ARG, "max_depth must be >= 0");
    c->max_depth = max_depth;
    std::memcpy(c->background, background, 12);
    c->sqrt_spp = sqrt_spp;
    c->recip_sqrt_spp = recip_sqrt_spp;
    return RT_OK;
}

int rt_set_partition(rt_ctx* c, int rank, int world, int stripe_rows) {
    if (!c) return RT_ERR_INVALID_ARG;
    if (world < 1 || rank < 0 || rank >= world || stripe_rows < 1) return set_err(c, RT_ERR_INVALID_ARG, "bad partition");
    if (world > 1 && c->devs.size() != 1) return set_err(c, RT_ERR_STATE, "process partition needs a 1-device context");
    c->proc_rank = rank;
    c->proc_world = world;
    c->stripe_rows = stripe_rows;
    if (c->devs.size() == 1) {
        c->devs[0].rank = rank;
        c->devs[0].world = world;
    }
    if (c->width > 0) return rt_resize(c, c->width, c->height);
    return RT_OK;
}

int rt_local_rows(int height, int rank, int world, int stripe_rows) { return local_rows_of(height, rank, world, stripe_rows); }
int rt_padded_local_rows(int height, int world, int stripe_rows) {
    if (height <= 0 || world <= 0 || stripe_rows <= 0) return 0;
    return padded_rows_of(height, world, stripe_rows);
}

int rt_resize(rt_ctx* c, int w, int h) {
    if (!c) return RT_ERR_INVALID_ARG;
    if (w <= 0 || h <= 0 || w > RT_MAX_IMAGE_DIM || h > RT_MAX_IMAGE_DIM || (size_t)w * h > ((size_t)1 << 30))
        return set_err(c, RT_ERR_INVALID_ARG, "bad image size");
    c->width = w;
    c->height = h;
    for (Device& d : c->devs) {
        int r = alloc_image(c, d);
        if (r) return r;
    }
    return RT_OK;
}

int rt_bind_device_image(rt_ctx* c, void* ptr, size_t nbytes) {
    if (!c) return RT_ERR_INVALID_ARG;
    if (c->devs.size() != 1) return set_err(c, RT_ERR_STATE, "device image binding needs a 1-device context");
    Device& d = c->devs[0];
    if (c->width <= 0) return set_err(c, RT_ERR_STATE, "rt_resize first");
    if (!ptr) {
        d.image_ptr = (float*)d.image.ptr;
        d.image_bound = false;
        return RT_OK;
    }
    if (nbytes < (size_t)d.local_rows * c->width * 16) return set_err(c, RT_ERR_INVALID_ARG, "device image too small");
    d.image_ptr = (float*)ptr;
    d.image_bound = true;
    return RT_OK;
}

int rt_set_stream(rt_ctx* c, void* stream) {
    if (!c) return RT_ERR_INVALID_ARG;
    if (c->devs.size() != 1) return set_err(c, RT_ERR_STATE, "stream binding needs a 1-device context");
    Device& d = c->devs[0];
    HIPCHK(c, hipSetDevice(d.id));
    if (d.own_stream && d.stream) HIPCHK(c, hipStreamSynchronize(d.stream));
    if (!stream) {
        if (!d.own_stream) {
            HIPCHK(c, hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
            d.own_stream = true;
        }
        return RT_OK;
    }
    if (d.own_stream && d.stream) HIPCHK(c, hipStreamDestroy(d.stream));
    d.stream = (hipStream_t)stream;
    d.own_stream = false;
    return RT_OK;
}

int rt_render(rt_ctx* c, int first_frame, int n_frames, const float* rand_factors) {
    if (!c) return RT_ERR_INVALID_ARG;
    if (first_frame < 1 || n_frames < 0 || (n_frames > 0 && !rand_factors))
        return set_err(c, RT_ERR_INVALID_ARG, "first_frame >= 1, n_frames >= 0, rand_factors required");
    if (c->width <= 0) return set_err(c, RT_ERR_STATE, "rt_resize before rt_render");
    if (!c->have_cam) return set_err(c, RT_ERR_STATE, "rt_set_camera before rt_render");
    if (!c->uploaded[RT_BIND_BVH]) return set_err(c, RT_ERR_STATE, "no BVH uploaded");
    // u_rand_factor is (float)Math.random() in the reference (RaytraceExecutor.java:124-127).
    // rand() adds 0.001 to it per call (random.glsl:2-7): a NaN / inf, or a value so large
    // that the addition no longer changes it, would freeze rand() and keep a rejection
    // loop (random.glsl:19-24, 40-45) spinning on the device forever
    for (int i = 0; i < n_frames; i++)
        if (!(std::fabs(rand_factors[i]) <= RT_MAX_RAND_FACTOR))
            return set_err(c, RT_ERR_INVALID_ARG, "rand_factors must be finite with |value| <= 1024");
    int r = validate(c);
    if (r) return r;
    rt_kernel_args a;
    std::memset(&a, 0, sizeof(a));
    if (c->bvh_mode == RT_BVH_SAH && c->variant != 0 && c->variant != 39)
        return set_err(c, RT_ERR_STATE, "the SAH BVH runs on the default kernel structure only");
    a.watchdog_ticks = c->watchdog_ticks;
    a.chunk_wait_ticks = c->chunk_wait_ticks;
    int32_t lc = 0;
    if (c->host_buf[RT_BIND_LIGHTS].size() >= 4) std::memcpy(&lc, c->host_buf[RT_BIND_LIGHTS].data(), 4);
    a.lights_count = lc;
    a.uv_always = c->uv_always;
    a.boxes_canon = c->boxes_canon ? 1 : 0;
    // Box pre-test (rt_kernel.hip leaf_prims_t): a face the exact test accepts lies, with
    // the ray's point at its t, within ~2^-20 of the scene's extent of the box's bounds
    // (the face tests' rounding, amplified at most 2x by a well-conditioned 2-D solve:
    // boxes_cond); the kernel's slab test of the bounds grown by 2^-13 of that extent
    // cannot miss it.
    if (c->scene_extent < 0.0f) c->scene_extent = scene_extent(c);
    a.box_margin = (c->boxes_cond && c->box_pretest && c->scene_extent <= 0x1p60f)
                       ? std::max(c->scene_extent, 1.0f) * 0x1p-13f
                       : 0.0f;
    a.fastdiv = (c->fastdiv && c->fd_cam && c->fd_ok[RT_BIND_SPHERES] && c->fd_ok[RT_BIND_QUADS] &&
                 c->fd_ok[RT_BIND_BOXES])
                    ? 1
                    : 0;
    a.variant = c->variant;
    a.zero_dir_end = c->zero_dir_end ? 1 : 0;
    a.sm_batch = c->sm_batch;
    a.walk_frac = c->walk_frac ? c->walk_frac : walk_frac_for(c->n_link_nodes);   // by the tree, not the pre-test nodes
    const FastTables& F = c->fast;
    a.fast_ok = F.ok ? 1 : 0;
    a.n_f2inner = (int)(F.inner2.size() / 4);
    a.n_f2leaves = (int)F.leaves2.size();
    a.f2depth = F.depth;
    std::memcpy(a.finfo_base, F.base, sizeof(a.finfo_base));
    a.fm_n = F.fm_n;
    std::memcpy(a.fm_medium, F.fm_medium, sizeof(a.fm_medium));
    std::memcpy(a.fm_leaf, F.fm_leaf, sizeof(a.fm_leaf));
    std::memcpy(a.fm_track, F.fm_track, sizeof(a.fm_track));
    std::memcpy(a.fm_flags, F.fm_flags, sizeof(a.fm_flags));
    a.fl_n = F.fl_n;
    std::memcpy(a.fl_medium, F.fl_medium, sizeof(a.fl_medium));
    std::memcpy(a.fl_rank, F.fl_rank, sizeof(a.fl_rank));
    a.debug_flags = c->debug_flags;
    // the links the launch walks: with the box pre-test nodes (option box_vnodes) when every box has a
    // compact record and the pre-test is on (its margin is the nodes' growth: rebuilt when it changes)
    {
        const size_t nb = c->host_buf[RT_BIND_BOXES].size() / sizeof(rt_box);
        const bool all_cmp = c->compact_boxes && nb > 0 && c->n_boxc_ok == (int)nb;
        const bool use_v = c->box_vnodes && all_cmp && a.box_margin > 0.0f && (c->variant == 0 || c->variant == 39) &&
                           c->boxc_host.size() == nb * RT_BOXC_F4;
        // node collapse (plan_collapse): planned for the camera, so rebuilt when it or the image size changes
        const bool use_c = c->collapse && (c->variant == 0 || c->variant == 39) && c->have_cam;
        const bool cam_moved = use_c && (std::memcmp(&c->walk_cam, &c->cam, sizeof(rt_camera_ubo)) != 0 ||
                                         c->walk_w != c->width || c->walk_h != c->height);
        const bool use_r = c->rebuild > 0 && (c->variant == 0 || c->variant == 39);
        if (c->walk_stale || use_v != c->walk_v || (use_v && a.box_margin != c->walk_v_margin) ||
            use_c != c->walk_c || cam_moved || use_r != c->walk_r || c->rebuild != c->walk_rmode) {
            if (c->walk_stale) c->rb_mode = -1;   // a new walk_dn (validate)
            if (use_r && c->rb_mode != c->rebuild) {
                c->rb_dn = rebuild_inner(c->walk_dn, c->rebuild);
                c->rb_mode = c->rebuild;
            }
            static const std::vector<rt_dnode> none;
            const std::vector<rt_dnode>& rb = use_r ? c->rb_dn : none;
            const std::vector<rt_dnode>& wdn = rb.empty() ? c->walk_dn : rb;
            std::vector<uint8_t> drop;
            if (use_c) {
                try {
                    if (!c->inj_hits.empty() && c->inj_hits.size() >= wdn.size()) {
                        // measured hits, given per link node (breadth-first): back to dn's order
                        std::vector<uint32_t> order{0u};
                        for (size_t q = 0; q < order.size() && order.size() <= wdn.size(); q++) {
                            const uint32_t k = order[q];
                            if ((wdn[k].meta & 0xF0000u) != 0 || k + 1 >= wdn.size()) continue;
                            order.push_back(k + 1);
                            order.push_back(wdn[k + 1].meta & 0xFFFFu);
                        }
                        std::vector<int64_t> H(wdn.size(), 0);
                        if (order.size() == wdn.size())
                            for (size_t q = 0; q < order.size(); q++)
                                if (order[q] < wdn.size()) H[order[q]] = c->inj_hits[q];
                        drop = plan_from_hits(wdn, H, c->inj_walks);
                    } else {
                        drop = plan_collapse(wdn, c->cam, c->width, c->height);
                    }
                } catch (const std::bad_alloc&) {   // no plan: the walk keeps every node
                    drop.clear();
                }
            }
            c->n_dropped = 0;
            for (uint8_t x : drop) c->n_dropped += x;
            const std::vector<uint8_t>* dp = c->n_dropped ? &drop : nullptr;
            if (use_v) {
                // the kernel's pre-test bounds (leaf_prims_t): compact record c0 = (mn.x, mn.y, mn.z,
                // mx.x), c1 = (mx.y, mx.z, ..), each grown by the margin with the same float operations
                const float m = a.box_margin;
                std::vector<float> vb(6 * nb);
                for (size_t b = 0; b < nb; b++) {
                    const float4 c0 = c->boxc_host[b * RT_BOXC_F4], c1 = c->boxc_host[b * RT_BOXC_F4 + 1];
                    const float g[6] = {c0.x - m, c0.w + m, c0.y - m, c1.x + m, c0.z - m, c1.y + m};
                    std::memcpy(&vb[6 * b], g, sizeof(g));
                }
                int nn = 0;
                c->walk_links = build_links(wdn, &vb, &nn, dp);
                c->n_walk_nodes = nn;
                c->n_vnodes = std::max(0, nn - ((int)wdn.size() - (dp ? c->n_dropped : 0)));
            } else if (dp || !rb.empty()) {
                int nn = 0;
                c->walk_links = build_links(wdn, nullptr, &nn, dp);
                c->n_walk_nodes = nn;
            } else {
                c->walk_links = c->links;
                c->n_walk_nodes = c->n_link_nodes;
            }
            if (!use_v) c->n_vnodes = 0;
            c->walk_c = use_c;
            c->walk_r = use_r;
            c->walk_rmode = c->rebuild;
            c->n_rebuilt = rb.empty() ? 0 : (int)rb.size();
            c->walk_cam = c->cam;
            c->walk_w = c->width;
            c->walk_h = c->height;
            c->walk_v = use_v;
            c->walk_v_margin = use_v ? a.box_margin : -1.0f;
            c->walk_stale = false;
            c->pair_leaves = -1;
            c->fast_gen++;   // re-upload the links (rt_render's device loop)
        }
        a.box_vnodes = c->walk_v && c->n_vnodes > 0 ? 1 : 0;
    }
    a.n_nodes = c->n_walk_nodes;
    a.n_lnode_f4 = (int)c->walk_links.size();
    plan_spine(c->walk_links, c->n_walk_nodes, c->cam, c->spine, a);
    // LDS plan of the link-format shapes (rt_kernel.hip rt_launch_render): from address 0 the
    // nodes, then the leaf records, the Perlin table (6 x 256 R32F), the media records with
    // their sphere boundaries, the spheres' intersection halves (A, B) and the canonical
    // boxes' compact records -- each when it fits.  512-thread workgroups (2 per CU,
    // RT_LDS_DYN_BYTES each) when everything fits them, else one of 1024 threads per CU
    // (RT_LDS_BIG_BYTES); when not even the nodes and leaves fit that, the two-level walk:
    // the top levels (breadth-first prefix) in LDS, the rest of the nodes and the leaf
    // records in global memory.  The A/B structures 37 (one pixel per lane: 512 threads,
    // the lanes' running means after what is staged) and 61 (its own tree) plan below too.
    const bool fast_walk = c->variant == 61 || c->variant == 69;
    const bool pooled = c->variant == 0 || c->variant == 39;
    const int n_sph = (int)(c->host_buf[RT_BIND_SPHERES].size() / sizeof(rt_sphere));
    const int n_box = (int)(c->host_buf[RT_BIND_BOXES].size() / sizeof(rt_box));
    const int n_med = (int)(c->host_buf[RT_BIND_MEDIA].size() / sizeof(rt_medium));
    a.n_media = n_med;
    a.media_sph = 1;
    for (int k = 0; k < n_med; k++) {
        rt_medium m;
        std::memcpy(&m, c->host_buf[RT_BIND_MEDIA].data() + k * sizeof(rt_medium), sizeof m);
        if (m.boundary_type != RT_MODEL_SPHERE) a.media_sph = 0;
    }
    a.n_sph_lds = n_sph;
    a.n_box_lds = n_box;
    a.box_all_cmp = (c->compact_boxes && n_box > 0 && c->n_boxc_ok == n_box) ? 1 : 0;
    // the sphere-pair kernels (rt_kernel.hip leaf_prims_t SPAIR) for a BVH whose leaves are mostly
    // two spheres (scene 0: 485 spheres); measured slower where they are not
    if (c->pair_leaves < 0) c->pair_leaves = pair_leaves_permille(c->walk_links, c->n_walk_nodes);
    // option sphere_pairs = 2: the pair kernels whatever the share, compact-box kernels included
    a.sph_pairs = c->sphere_pairs == 2 ? 2 : (c->sphere_pairs && c->pair_leaves >= 500) ? 1 : 0;
    // the shading batch threshold by kernel: 50/64 of the walking lanes in the compact-box kernels, 52 in
    // the sphere-pair kernels (round 6, on their branchless walk: scene 0 -0.4%, twice,
    // profiles/r06_ag_opts_s0.log, r06_ah_opts_s0.log), 56 otherwise
    a.sm_frac = c->sm_frac ? c->sm_frac : (a.box_all_cmp ? 50 : (a.sph_pairs == 1 ? 52 : 56));
    a.perlin_slot = -1;
    for (int t = 0; t < RT_MAX_TEXTURES && a.perlin_slot < 0; t++)
        if (c->tex_format[t] == RT_TEX_R32F && c->tex_w[t] == 6) a.perlin_slot = t;
    {
        const size_t node_f4 = 2 * (size_t)c->n_walk_nodes;
        const size_t leaf_f4 = (size_t)a.n_lnode_f4 > node_f4 ? (size_t)a.n_lnode_f4 - node_f4 : 0;
        a.perlin_packed = (a.perlin_slot >= 0 && a.perlin_slot == c->perlin_pk_slot && c->perlin_pk) ? 1 : 0;
        // the Perlin table is staged in its packed form only (else its noise reads the texture)
        const size_t perlin_f4 = a.perlin_packed ? 256 : 0;
        const size_t media_f4 = (n_med > 0 && n_med <= 64) ? 3 * (size_t)n_med : 0;
        const size_t sph_f4 = (c->sph_lds && pooled) ? 2 * (size_t)n_sph : 0;
        const size_t box_f4 = (size_t)RT_BOXC_F4 * n_box;   // every box's record (bounds; compact faces)
        const bool stats_twin = c->variant == 39;   // static LDS counters beside the dynamic region
        const size_t cap_s = RT_LDS_DYN_BYTES / 16,
                     cap_b = (stats_twin ? RT_LDS_BIG_STATS_BYTES : RT_LDS_BIG_BYTES) / 16;
        const size_t ess = node_f4 + leaf_f4 + perlin_f4 + media_f4;   // what every walk and shade reads
        const size_t all = ess + sph_f4 + box_f4;
        const size_t node_cap = c->lds_node_cap > 0 ? (size_t)c->lds_node_cap / 32 * 2 : node_f4;
        const bool big_ok = c->big_wg && pooled;
        // A/B: threaded meta-word nodes (variant 30, or 37 when the link nodes do not fit 512 threads)
        const bool meta = !fast_walk && !pooled && (c->variant == 30 || c->variant == 31 || ess > cap_s);
        size_t cap;
        bool tl = false;
        if (fast_walk) {
            cap = 0;   // variant 61 stages its own tree (rt_launch_render)
        } else if (meta) {
            cap = cap_s;
        } else if (node_cap < node_f4 && pooled) {
            tl = true;
            cap = cap_b;
        } else if (all <= cap_s || (ess <= cap_s && !(big_ok && all <= cap_b))) {
            cap = cap_s;
        } else if (big_ok && ess <= cap_b) {
            cap = cap_b;
        } else {
            tl = pooled;
            cap = tl ? cap_b : cap_s;
        }
        a.block = cap == cap_b ? 1024 : 512;
        // the two-level walk's rounds: 32 (its walks wait on global nodes; 16 / 24 / 32 / 48 / 64 on
        // the 4000-sphere cloud at a 32 KB cap and the 9000-sphere cloud: 32 best, -1.7% against 48,
        // profiles/r04_bvh_walk_frac_*.log)
        if (tl && !c->walk_frac) a.walk_frac = 32;
        size_t at = 0;
        a.lds_node_f4 = 0;
        a.leaf_lds = -1;
        a.perlin_lds = a.media_lds = a.sph_lds = a.box_cmp_lds = -1;
        a.sph_mat_lds = a.box_mat_lds = a.tex_lds = -1;
        for (int t = 0; t < 8; t++) a.tex_lds_off[t] = -1;
        if (meta) {
            at = node_f4;   // the threaded nodes (32 B each) from address 0 (rt_launch_render: META_LDS)
        } else if (!fast_walk && a.n_lnode_f4 > 0) {
            if (tl) {
                // the top levels, then the leaf records (8 B per leaf, read on every leaf visit) when
                // they take at most half of the room, then the small tables the shading reads; room
                // is reserved for the sphere / compact box records that take at most 1/16 of it (a
                // few nodes' worth), and each table is staged below whenever it still fits (option
                // tl_small_lds; a larger table can fit after a node cap -- tests/test_gpu_adversarial.py
                // forces both layouts)
                const size_t room0 = cap - perlin_f4 - media_f4;
                const size_t rsv = (c->tl_small_lds && sph_f4 && 16 * sph_f4 <= room0 ? sph_f4 : 0) +
                                   (c->tl_small_lds && box_f4 && 16 * box_f4 <= room0 ? box_f4 : 0);
                const size_t room = room0 - rsv;
                const size_t lf_f4 = (c->tl_leaf_lds && 2 * leaf_f4 <= room) ? leaf_f4 : 0;
                a.lds_node_f4 = (int)(std::min(std::min(node_f4, node_cap), room - lf_f4) & ~(size_t)1);
                at = (size_t)a.lds_node_f4;
                if (lf_f4) {
                    a.leaf_lds = (int)at;
                    at += lf_f4;
                }
            } else {
                a.lds_node_f4 = (int)node_f4;
                a.leaf_lds = (int)node_f4;
                at = node_f4 + leaf_f4;
            }
        }
        if (!fast_walk) {
            if (perlin_f4 && at + perlin_f4 <= cap) { a.perlin_lds = (int)at; at += perlin_f4; }
            if (media_f4 && at + media_f4 <= cap) { a.media_lds = (int)at; at += media_f4; }
            if (!tl || c->tl_small_lds) {
                if (sph_f4 && at + sph_f4 <= cap) { a.sph_lds = (int)at; at += sph_f4; }
                if (box_f4 && at + box_f4 <= cap) { a.box_cmp_lds = (int)at; at += box_f4; }
            }
            // the shading tables (option shade_lds): every sphere's third float4, every compact
            // box's (emission, material), the texture slots' descriptors and the texels of the
            // small slots (at most 1024 words: the solid and checker colour tables), each when
            // it fits -- so a hit's material, texture and colour need no global read
            if (c->shade_lds && pooled && !tl) {
                if (a.sph_lds >= 0 && at + (size_t)n_sph <= cap) { a.sph_mat_lds = (int)at; at += (size_t)n_sph; }
                if (a.box_cmp_lds >= 0 && a.box_all_cmp && at + (size_t)n_box <= cap) {
                    a.box_mat_lds = (int)at;
                    at += (size_t)n_box;
                }
                size_t need = 8;
                for (int t = 0; t < 8; t++) {
                    const size_t words = (size_t)c->tex_w[t] * (size_t)c->tex_h[t];
                    if (c->tex_w[t] > 0 && c->tex_h[t] > 0 && words <= 1024) need += (words + 3) / 4;
                }
                if (at + need <= cap) {
                    a.tex_lds = (int)at;
                    size_t off = at + 8;
                    for (int t = 0; t < 8; t++) {
                        const size_t words = (size_t)c->tex_w[t] * (size_t)c->tex_h[t];
                        a.tex_lds_off[t] = -1;
                        if (c->tex_w[t] > 0 && c->tex_h[t] > 0 && words <= 1024) {
                            a.tex_lds_off[t] = (int)off;
                            off += (words + 3) / 4;
                        }
                    }
                    at = off;
                }
            }
        }
        a.lds_end_f4 = (int)at;
        // the leaf stage's record prefetch reads 3 float4 at any of these tables' offsets: every
        // table it can index is staged (and a sphere's 3rd float4 stays inside the staged region)
        a.leaf_pf = (c->leaf_prefetch && a.sph_lds >= 0 && a.box_cmp_lds >= 0 &&
                     (n_med == 0 || a.media_lds >= 0) && a.box_cmp_lds > a.sph_lds) ? 1 : 0;
    }
    a.cam = c->cam;
    std::memcpy(a.background, c->background, 12);
    a.max_depth = c->max_depth;
    a.sqrt_spp = c->sqrt_spp;
    a.recip_sqrt_spp = c->recip_sqrt_spp;
    a.width = c->width;
    a.height = c->height;
    a.stripe_rows = c->stripe_rows;
    uint64_t max_ns = 0;
    for (Device& d : c->devs) {
        HIPCHK(c, hipSetDevice(d.id));
        a.nodes = (const rt_dnode*)d.nodes.ptr;
        a.spheres = (const rt_sphere*)d.spheres.ptr;
        a.quads = (const rt_quad*)d.quads.ptr;
        a.boxes = (const rt_box*)d.boxes.ptr;
        a.dquads = (const float4*)d.dquads.ptr;
        a.dboxes = (const float4*)d.dboxes.ptr;
        a.dboxc = (const float4*)d.dboxc.ptr;
        a.perlin_pk = a.perlin_packed ? (const float4*)d.perlin_pk.ptr : nullptr;
        a.media = (const rt_medium*)d.media.ptr;
        a.lights = (const int32_t*)d.lights.ptr;
        for (int t = 0; t < 8; t++) {
            a.tex[t].data = d.tex[t].ptr;
            a.tex[t].w = c->tex_w[t];
            a.tex[t].h = c->tex_h[t];
            a.tex[t].is_float = c->tex_format[t] == RT_TEX_R32F;
        }
        a.image = d.image_ptr;
        a.stats = (unsigned long long*)d.stats.ptr;
        a.census = (unsigned*)d.census.ptr;
        a.census_cap = d.census_cap;
        a.node_hits = (unsigned*)d.node_hits.ptr;
        a.census_waves = d.census_waves;
        a.local_rows = d.local_rows;
        a.rank = d.rank;
        a.world = d.world;
        if (!d.args.ptr) {
            HIPCHK(c, hipMalloc(&d.counter.ptr, 256));
            d.counter.bytes = 256;
            HIPCHK(c, hipMemsetAsync(d.counter.ptr, 0, 256, d.stream));
            HIPCHK(c, hipMalloc(&d.args.ptr, sizeof(rt_kernel_args)));
            d.args.bytes = sizeof(rt_kernel_args);
            HIPCHK(c, hipHostMalloc((void**)&d.ring, sizeof(rt_kernel_args) * Device::kRing, hipHostMallocDefault));
            for (auto& e : d.ring_ev) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        }
        a.tile_counter = (int*)d.counter.ptr;
        if (d.fast_gen != c->fast_gen) {
            int rf = dev_alloc_copy(c, d, d.finfo, F.info.data(), F.info.size() * sizeof(uint32_t));
            if (!rf) rf = dev_alloc_copy(c, d, d.f2inner, F.inner2.data(), F.inner2.size() * sizeof(float4));
            if (!rf) rf = dev_alloc_copy(c, d, d.f2leaves, F.leaves2.data(), F.leaves2.size() * sizeof(uint2));
            if (!rf) rf = dev_alloc_copy(c, d, d.links, c->walk_links.data(), c->walk_links.size() * sizeof(float4));
            if (rf) return rf;
            d.fast_gen = c->fast_gen;
        }
        a.finfo = (const uint32_t*)d.finfo.ptr;
        a.f2inner = (const float4*)d.f2inner.ptr;
        a.f2leaves = (const uint2*)d.f2leaves.ptr;
        a.lnodes = (const float4*)d.links.ptr;
        // Frames per launch and the unit split.  Units = tiles x chunks; with too
        // few tiles per resident wave (small images, N-GPU stripes) the frames
        // are split into ordered chunks so the dynamic schedule has enough units
        // to balance (rt_kernel.hip wait_chunk / publish_chunk).
        const int n_tiles = ((c->width + 7) / 8) * ((d.local_rows + 7) / 8);
        int per_launch = RT_MAX_FRAMES_PER_LAUNCH;
        int chunks_wanted = 1;
        const long long waves = rt_resident_waves();
        const bool few_tiles = (long long)n_tiles < (long long)c->stage_tiles * waves;
        if (c->chunk_target > 0 && n_tiles > 0) {
            const long long target = few_tiles ? c->staged_chunk_target : c->chunk_target;
            chunks_wanted = (int)std::min<long long>(RT_MAX_FRAMES_PER_LAUNCH, (target * waves + n_tiles - 1) / n_tiles);
        }
        const bool staged = chunks_wanted > 1 && few_tiles;
        const size_t n_pixels = (size_t)d.local_rows * c->width;
        if (staged) {
            // staged colours per launch: at most sample_budget and half the device's free memory
            // (what this context already holds counts as free), and at most 2^31 samples (the
            // kernel's 32-bit sample index)
            size_t budget = c->sample_budget;
            size_t free_b = 0, total_b = 0;
            if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) budget = std::min(budget, (free_b + d.samples.bytes) / 2);
            const size_t per_frame = n_pixels * sizeof(float4);
            size_t frames = std::min<size_t>(RT_MAX_FRAMES_PER_LAUNCH, budget / per_frame);
            frames = std::min<size_t>(frames, ((size_t)1 << 31) / std::max<size_t>(n_pixels, 1));
            per_launch = (int)std::max<size_t>(1, frames);
        }
        {   // equal launches: no short last launch that the whole grid waits on
            const int n_launch = (std::max(n_frames, 1) + per_launch - 1) / per_launch;
            per_launch = (std::max(n_frames, 1) + n_launch - 1) / n_launch;
        }
        if (staged) {
            const size_t per_frame = n_pixels * sizeof(float4);
            const size_t need = per_frame * (size_t)std::min(per_launch, std::max(n_frames, 1));
            if (d.samples.bytes < need) {
                dev_free(d.samples);
                HIPCHK(c, hipMalloc(&d.samples.ptr, need));
                d.samples.bytes = need;
            }
        }
        a.samples = staged ? (float4*)d.samples.ptr : nullptr;
        a.n_pixels = n_pixels;
        if (!staged && chunks_wanted > 1 && d.tile_done.bytes < sizeof(unsigned) * (size_t)n_tiles) {
            dev_free(d.tile_done);
            HIPCHK(c, hipMalloc(&d.tile_done.ptr, sizeof(unsigned) * (size_t)n_tiles));
            d.tile_done.bytes = sizeof(unsigned) * (size_t)n_tiles;
        }
        a.tile_done = (unsigned*)d.tile_done.ptr;
        a.fault = (unsigned*)d.counter.ptr + 1;
        HIPCHK(c, hipEventRecord(d.ev_start, d.stream));
        for (int f0 = 0; f0 < n_frames; f0 += per_launch) {
            int nf = std::min(per_launch, n_frames - f0);
            a.first_frame = first_frame + f0;
            a.n_frames = nf;
            a.n_chunks = std::max(1, std::min(chunks_wanted, nf));
            a.chunk_frames = (nf + a.n_chunks - 1) / a.n_chunks;
            a.n_chunks = (nf + a.chunk_frames - 1) / a.chunk_frames;
            if (a.n_chunks == 1) a.samples = nullptr;   // one chunk: the running mean in place
            else if (staged) a.samples = (float4*)d.samples.ptr;
            // staged: the last frames as one-frame chunks (the units claimed last are then short,
            // so the grid's waves finish close together); the chunks before keep their size
            a.tail_chunks = 0;
            const int tail = c->tail_chunks >= 0 ? c->tail_chunks : tail_chunks_for(c->n_link_nodes);
            if (a.samples && tail > 0 && a.n_chunks > 1 && (c->variant == 0 || c->variant == 39)) {
                const int tc = std::min(tail, nf - 1);
                const int nm = nf - tc;
                const int cm = (nm + a.chunk_frames - 1) / a.chunk_frames;
                a.n_chunks = cm + tc;
                a.tail_chunks = tc;
            }
            // Sparse staging (render_stream): most samples' colours are exactly zero (scene 8: 96%:
            // a path that ends without reaching the light), so each sample writes a flag byte and
            // only the others their 16-byte colour; fold_kernel reads a clear flag as the zero
            // colour.  (A per-(chunk, pixel) bit word set by atomics measured slower: scene 6 +2.5%.)
            a.sflags = nullptr;
            if (a.samples && c->sparse_stage && (c->variant == 0 || c->variant == 39)) {
                const size_t need = n_pixels * (size_t)std::min(per_launch, std::max(n_frames, 1));
                if (d.sflags.bytes < need) {
                    dev_free(d.sflags);
                    HIPCHK(c, hipMalloc(&d.sflags.ptr, need));
                    d.sflags.bytes = need;
                }
                a.sflags = (uint8_t*)d.sflags.ptr;
            }
            a.wbuf = nullptr;
            a.wbuf_waves = 0;
            if (!a.samples && (c->variant == 0 || c->variant == 39)) {
                // pooled units fold per wave; two slots per wave (render_stream keeps two units in flight)
                const size_t need = (size_t)waves * 2 * 64 * (size_t)a.chunk_frames * sizeof(float4);
                if (d.wbuf.bytes < need) {
                    dev_free(d.wbuf);
                    HIPCHK(c, hipMalloc(&d.wbuf.ptr, need));
                    d.wbuf.bytes = need;
                }
                a.wbuf = (float4*)d.wbuf.ptr;
                a.wbuf_waves = (int)waves;
            }
            std::memcpy(a.rand_factors, rand_factors + f0, sizeof(float) * nf);
            int slot = d.ring_pos++ % Device::kRing;
            HIPCHK(c, hipEventSynchronize(d.ring_ev[slot]));   // the copy that last used this slot is done
            d.ring[slot] = a;
            if (rt_launch_render(d.ring[slot], (rt_kernel_args*)d.args.ptr, d.stream,
                                 &d == &c->devs[0] ? c->last_launch : nullptr))
                return set_err(c, RT_ERR_DEVICE, std::string("kernel launch failed: ") +
                                                     hipGetErrorString(hipGetLastError()));
            HIPCHK(c, hipEventRecord(d.ring_ev[slot], d.stream));
            if (&d == &c->devs[0]) {
                c->last_launch[RT_LI_BVH_MODE] = c->bvh_mode;
                c->last_launch[RT_LI_VNODES] = a.box_vnodes ? c->n_vnodes : 0;
                c->last_launch[RT_LI_COLLAPSED] = c->walk_c ? c->n_dropped : 0;
                c->last_launch[RT_LI_REBUILT] = c->n_rebuilt > 0 ? 1 : 0;
            }
        }
        HIPCHK(c, hipEventRecord(d.ev_stop, d.stream));
        d.timed = true;
        c->launched = c->launched || n_frames > 0;
    }
    (void)max_ns;
    return RT_OK;
}

int rt_sync(rt_ctx* c) {
    if (!c) return RT_ERR_INVALID_ARG;
    for (Device& d : c->devs) {
        HIPCHK(c, hipSetDevice(d.id));
        HIPCHK(c, hipStreamSynchronize(d.stream));
        if (d.counter.ptr) {   // fault word: an ordered-chunk wait timed out (never expected)
            unsigned fault = 0;
            HIPCHK(c, hipMemcpy(&fault, (unsigned*)d.counter.ptr + 1, sizeof(unsigned), hipMemcpyDeviceToHost));
            if (fault) {
                HIPCHK(c, hipMemset((unsigned*)d.counter.ptr + 1, 0, sizeof(unsigned)));
                return set_err(c, RT_ERR_DEVICE, fault == 2 ? "render kernel: a wave stored no sample within its progress bound (watchdog)"
                                                            : "render kernel: ordered-chunk wait timed out");
            }
        }
    }
    return RT_OK;
}

int rt_last_render_ns(rt_ctx* c, uint64_t* ns) {
    if (!c || !ns) return RT_ERR_INVALID_ARG;
    double mx = 0;
    for (Device& d : c->devs) {
        if (!d.timed) continue;
        HIPCHK(c, hipSetDevice(d.id));
        HIPCHK(c, hipEventSynchronize(d.ev_stop));
        float ms = 0;
        HIPCHK(c, hipEventElapsedTime(&ms, d.ev_start, d.ev_stop));
        mx = std::max(mx, (double)ms);
    }
    *ns = (uint64_t)(mx * 1e6);
    c->last_ns = *ns;
    return RT_OK;
}

int rt_render_done(rt_ctx* c, uint64_t* ns) {
    if (!c || !ns) return RT_ERR_INVALID_ARG;
    double mx = 0;
    for (Device& d : c->devs) {
        if (!d.timed) continue;
        HIPCHK(c, hipSetDevice(d.id));
        const hipError_t q = hipEventQuery(d.ev_stop);
        if (q == hipErrorNotReady) return 0;
        if (q != hipSuccess) return set_err(c, RT_ERR_DEVICE, std::string("hipEventQuery: ") + hipGetErrorString(q));
        float ms = 0;
        HIPCHK(c, hipEventElapsedTime(&ms, d.ev_start, d.ev_stop));
        mx = std::max(mx, (double)ms);
    }
    *ns = (uint64_t)(mx * 1e6);
    return 1;
}

int rt_read_image(rt_ctx* c, float* rgba) {
    if (!c || !rgba) return RT_ERR_INVALID_ARG;
    if (c->width <= 0) return set_err(c, RT_ERR_STATE, "no image");
    int r = rt_sync(c);
    if (r) return r;
    if (c->devs.size() == 1) {
        Device& d = c->devs[0];
        HIPCHK(c, hipSetDevice(d.id));
        return d2h(c, d, rgba, d.image_ptr, (size_t)d.local_rows * c->width * 16);
    }
    // multi-device context: the stripe blocks gathered on device 0 (RCCL when the devices
    // are distinct and RCCL loads, else peer copies), de-interleaved there, one copy out
    if (device_gather(c) == RT_OK) {
        Device& d0 = c->devs[0];
        HIPCHK(c, hipSetDevice(d0.id));
        return d2h(c, d0, rgba, d0.full.ptr, (size_t)c->height * c->width * 16);
    }
    // last resort: every block to the host, de-interleaved there
    int ndev = (int)c->devs.size();
    int padded = padded_rows_of(c->height, ndev, c->stripe_rows);
    std::vector<float> g((size_t)ndev * padded * c->width * 4, 0.0f);
    for (int k = 0; k < ndev; k++) {
        Device& d = c->devs[k];
        HIPCHK(c, hipSetDevice(d.id));
        int r2 = d2h(c, d, g.data() + (size_t)k * padded * c->width * 4, d.image_ptr,
                     (size_t)d.local_rows * c->width * 16);
        if (r2) return r2;
    }
    c->gather_path = RT_GATHER_HOST;
    return rt_deinterleave_rows(g.data(), c->width, c->height, ndev, c->stripe_rows, rgba);
}

int rt_write_image(rt_ctx* c, const float* rgba) {
    if (!c || !rgba) return RT_ERR_INVALID_ARG;
    if (c->width <= 0) return set_err(c, RT_ERR_STATE, "no image");
    int r = rt_sync(c);
    if (r) return r;
    for (Device& d : c->devs) {
        HIPCHK(c, hipSetDevice(d.id));
        std::vector<float> local((size_t)d.local_rows * c->width * 4);
        // pick this device's rows from the (process-local) image
        if (c->devs.size() == 1) {
            int r2 = h2d(c, d, d.image_ptr, rgba, local.size() * 4);
            if (r2) return r2;
            continue;
        }
        int n_stripes = (c->height + c->stripe_rows - 1) / c->stripe_rows;
        size_t lr = 0;
        for (int s = d.rank; s < n_stripes; s += d.world)
            for (int y = s * c->stripe_rows; y < std::min(c->height, (s + 1) * c->stripe_rows); y++, lr++)
                std::memcpy(&local[lr * c->width * 4], rgba + (size_t)y * c->width * 4, (size_t)c->width * 16);
        int r2 = h2d(c, d, d.image_ptr, local.data(), local.size() * 4);
        if (r2) return r2;
    }
    return RT_OK;
}

int rt_deinterleave_rows(const float* gathered, int width, int height, int world, int stripe_rows, float* out) {
    if (!gathered || !out || width <= 0 || height <= 0 || world < 1 || stripe_rows < 1) return RT_ERR_INVALID_ARG;
    int padded = padded_rows_of(height, world, stripe_rows);
    int n_stripes = (height + stripe_rows - 1) / stripe_rows;
    for (int k = 0; k < world; k++) {
        size_t lr = 0;
        for (int s = k; s < n_stripes; s += world)
            for (int y = s * stripe_rows; y < std::min(height, (s + 1) * stripe_rows); y++, lr++)
                std::memcpy(out + (size_t)y * width * 4, gathered + ((size_t)k * padded + lr) * width * 4,
                            (size_t)width * 16);
    }
    return RT_OK;
}

float rt_frame_rand_factor(uint64_t seed, uint64_t frame_index) {
    uint64_t z = seed + (frame_index + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z ^= z >> 31;
    return (float)(uint32_t)(z >> 40) / 16777216.0f;
}

// ---- debug / test hooks (rt_debug.h)
int rt_debug_eval_builtin(int device, int fn, const float* x, const float* y, float* out, int n) {
    if (!x || !out || n < 0) return RT_ERR_INVALID_ARG;
    if (n == 0) return RT_OK;
    if (hipSetDevice(device) != hipSuccess) return RT_ERR_DEVICE;
    float *dx = nullptr, *dy = nullptr, *dout = nullptr;
    size_t b = (size_t)n * 4;
    int rc = RT_OK;
    if (hipMalloc(&dx, b) != hipSuccess || hipMalloc(&dout, b) != hipSuccess || (y && hipMalloc(&dy, b) != hipSuccess))
        rc = RT_ERR_DEVICE;
    if (!rc && hipMemcpy(dx, x, b, hipMemcpyHostToDevice) != hipSuccess) rc = RT_ERR_DEVICE;
    if (!rc && y && hipMemcpy(dy, y, b, hipMemcpyHostToDevice) != hipSuccess) rc = RT_ERR_DEVICE;
    if (!rc && rt_launch_eval_builtin(fn, dx, dy, dout, n, nullptr)) rc = RT_ERR_DEVICE;
    if (!rc && hipMemcpy(out, dout, b, hipMemcpyDeviceToHost) != hipSuccess) rc = RT_ERR_DEVICE;
    if (dx) (void)hipFree(dx);
    if (dy) (void)hipFree(dy);
    if (dout) (void)hipFree(dout);
    return rc;
}

int rt_debug_threaded_bvh(const void* nodes, size_t nbytes, void* out, size_t out_cap, int* n_out) {
    if (!nodes || !n_out || nbytes % sizeof(rt_bvh_node)) return RT_ERR_INVALID_ARG;
    std::vector<rt_dnode> dn;
    rt_ctx tmp;
    int r = thread_bvh(&tmp, (const rt_bvh_node*)nodes, (int)(nbytes / sizeof(rt_bvh_node)), dn);
    if (r) return r;
    *n_out = (int)dn.size();
    if (out) {
        if (out_cap < dn.size() * sizeof(rt_dnode)) return RT_ERR_INVALID_ARG;
        if (!dn.empty()) std::memcpy(out, dn.data(), dn.size() * sizeof(rt_dnode));
    }
    return RT_OK;
}

int rt_debug_deinterleave(const float* gathered, int width, int height, int world, int stripe_rows, float* out) {
    if (!gathered || !out || width <= 0 || height <= 0 || world < 1 || stripe_rows < 1) return RT_ERR_INVALID_ARG;
    const int padded = padded_rows_of(height, world, stripe_rows);
    for (int y = 0; y < height; y++) {   // deinterleave_kernel's indexing, one row at a time
        int k, lr;
        rt_gathered_row(y, world, stripe_rows, &k, &lr);
        std::memcpy(out + (size_t)y * width * 4, gathered + ((size_t)k * padded + lr) * width * 4, (size_t)width * 16);
    }
    return RT_OK;
}

int rt_debug_box_records(const void* boxes, size_t nbytes, void* out, size_t out_cap, int* n_compact) {
    if (!boxes || !n_compact || nbytes % sizeof(rt_box)) return RT_ERR_INVALID_ARG;
    const size_t nb = nbytes / sizeof(rt_box);
    if (out && out_cap < nb * RT_BOXC_F4 * sizeof(float4)) return RT_ERR_INVALID_ARG;
    // the upload's own path (rt_upload_buffer(RT_BIND_BOXES))
    std::vector<float4> recs(nb * RT_BOXC_F4);
    int n = 0;
    const rt_quad* qs = (const rt_quad*)boxes;
    for (size_t bx = 0; bx < nb; bx++) {
        float4 b[2];
        box_bounds(qs + 6 * bx, b);
        n += box_record(qs + 6 * bx, b, &recs[bx * RT_BOXC_F4]);
    }
    *n_compact = n;
    if (out && !recs.empty()) std::memcpy(out, recs.data(), recs.size() * sizeof(float4));
    return RT_OK;
}

int rt_debug_link_nodes_vbox(const void* bvh, size_t nbytes, const float* vbox, int n_box, void* out,
                             size_t out_cap, int* n_f4, int* n_nodes) {
    if (!bvh || !n_f4 || !n_nodes || nbytes % sizeof(rt_bvh_node) || n_box < 0 || (n_box && !vbox))
        return RT_ERR_INVALID_ARG;
    std::vector<rt_dnode> dn;
    rt_ctx tmp;
    int r = thread_bvh(&tmp, (const rt_bvh_node*)bvh, (int)(nbytes / sizeof(rt_bvh_node)), dn);
    if (r) return r;
    const std::vector<float> vb(vbox, vbox + 6 * (size_t)n_box);
    const std::vector<float4> L = build_links(dn, &vb, n_nodes);
    *n_f4 = (int)L.size();
    if (out) {
        if (out_cap < L.size() * sizeof(float4)) return RT_ERR_INVALID_ARG;
        if (!L.empty()) std::memcpy(out, L.data(), L.size() * sizeof(float4));
    }
    return RT_OK;
}

int rt_debug_collapse_links(const void* bvh, size_t nbytes, const float cam[28], int width, int height, int rebuild,
                            void* out, size_t out_cap, int* n_f4, uint8_t* drop, size_t drop_cap, int* n_dropped) {
    if (!bvh || !cam || !n_f4 || !n_dropped || nbytes % sizeof(rt_bvh_node)) return RT_ERR_INVALID_ARG;
    std::vector<rt_dnode> dn;
    rt_ctx tmp;
    int r = thread_bvh(&tmp, (const rt_bvh_node*)bvh, (int)(nbytes / sizeof(rt_bvh_node)), dn);
    if (r) return r;
    if (rebuild) {
        std::vector<rt_dnode> rb = rebuild_inner(dn, rebuild);
        if (!rb.empty()) dn.swap(rb);
    }
    rt_camera_ubo cu;
    std::memcpy(&cu, cam, sizeof(cu));
    const std::vector<uint8_t> d = plan_collapse(dn, cu, width, height);
    int nd = 0;
    for (uint8_t x : d) nd += x;
    *n_dropped = nd;
    int nn = 0;
    const std::vector<float4> L = build_links(dn, nullptr, &nn, &d);
    *n_f4 = (int)L.size();
    if (out) {
        if (out_cap < L.size() * sizeof(float4)) return RT_ERR_INVALID_ARG;
        if (!L.empty()) std::memcpy(out, L.data(), L.size() * sizeof(float4));
    }
    if (drop) {
        if (drop_cap < d.size()) return RT_ERR_INVALID_ARG;
        if (!d.empty()) std::memcpy(drop, d.data(), d.size());
    }
    return RT_OK;
}

int rt_debug_link_nodes(const void* bvh, size_t nbytes, void* out, size_t out_cap, int* n_f4) {
    if (!bvh || !n_f4 || nbytes % sizeof(rt_bvh_node)) return RT_ERR_INVALID_ARG;
    std::vector<rt_dnode> dn;
    rt_ctx tmp;
    int r = thread_bvh(&tmp, (const rt_bvh_node*)bvh, (int)(nbytes / sizeof(rt_bvh_node)), dn);
    if (r) return r;
    const std::vector<float4> L = build_links(dn);
    *n_f4 = (int)L.size();
    if (out) {
        if (out_cap < L.size() * sizeof(float4)) return RT_ERR_INVALID_ARG;
        if (!L.empty()) std::memcpy(out, L.data(), L.size() * sizeof(float4));
    }
    return RT_OK;
}

int rt_debug_perlin_pack(const float* texels, int w, int h, void* out, size_t out_cap) {
    if (!texels || w <= 0 || h <= 0) return RT_ERR_INVALID_ARG;
    std::vector<float4> pk;
    if (!perlin_pack(texels, w, h, pk)) return 0;
    if (out) {
        if (out_cap < pk.size() * sizeof(float4)) return RT_ERR_INVALID_ARG;
        if (!pk.empty()) std::memcpy(out, pk.data(), pk.size() * sizeof(float4));
    }
    return 1;
}

int rt_debug_sphere_pair_leaves(const void* bvh, size_t nbytes, int* permille) {
    if (!bvh || !permille || nbytes % sizeof(rt_bvh_node)) return RT_ERR_INVALID_ARG;
    std::vector<rt_dnode> dn;
    rt_ctx tmp;
    int r = thread_bvh(&tmp, (const rt_bvh_node*)bvh, (int)(nbytes / sizeof(rt_bvh_node)), dn);
    if (r) return r;
    *permille = pair_leaves_permille(build_links(dn), (int)dn.size());
    return RT_OK;
}

int rt_debug_fast_tables(const void* bvh, size_t nbytes, const void* quads, size_t qbytes, const void* boxes,
                         size_t bbytes, int n_spheres, void* nodes_out, size_t nodes_cap, int* n_per_octant,
                         uint32_t* info_out, size_t info_cap, int* slots_out, int* n_slots) {
    if (!bvh || nbytes % sizeof(rt_bvh_node) || qbytes % sizeof(rt_quad) || bbytes % sizeof(rt_box) || n_spheres < 0 ||
        !n_per_octant || !n_slots || (qbytes && !quads) || (bbytes && !boxes))
        return RT_ERR_INVALID_ARG;
    std::vector<rt_dnode> dn;
    rt_ctx tmp;
    int r = thread_bvh(&tmp, (const rt_bvh_node*)bvh, (int)(nbytes / sizeof(rt_bvh_node)), dn);
    if (r) return r;
    FastTables F = build_fast(dn, (size_t)n_spheres, (const rt_quad*)quads, qbytes / sizeof(rt_quad),
                              (const rt_box*)boxes, bbytes / sizeof(rt_box));
    *n_per_octant = F.n_per;
    *n_slots = F.fm_n;
    if (nodes_out) {
        if (nodes_cap < F.nodes.size() * sizeof(rt_dnode)) return RT_ERR_INVALID_ARG;
        if (!F.nodes.empty()) std::memcpy(nodes_out, F.nodes.data(), F.nodes.size() * sizeof(rt_dnode));
    }
    if (info_out) {
        if (info_cap < F.info.size() * sizeof(uint32_t)) return RT_ERR_INVALID_ARG;
        if (!F.info.empty()) std::memcpy(info_out, F.info.data(), F.info.size() * sizeof(uint32_t));
    }
    if (slots_out)
        for (int j = 0; j < F.fm_n; j++) {
            slots_out[4 * j + 0] = F.fm_medium[j];
            slots_out[4 * j + 1] = F.fm_leaf[j];
            slots_out[4 * j + 2] = F.fm_track[j];
            slots_out[4 * j + 3] = F.fm_flags[j];
        }
    return (F.ok && boxes_nest(dn)) ? 1 : 0;
}

// The stats twin (region timers + lane counters) of a launch variant: 61 -> 69, 30 -> 31, 37 -> 38, 0 -> 39.
static int stats_twin(int v) {
    if (v == 61 || v == 69) return 69;
    if (v == 30 || v == 31) return 31;
    if (v == 37 || v == 38) return 38;
    return 39;
}

// Leaf census records per resident wave (rt_debug_enable_stats(ctx, 2); tools/leaf_census.py)
#define RT_CENSUS_CAP 2048

int rt_debug_enable_stats(rt_ctx* c, int on) {
    if (!c || on < 0 || on > 2) return RT_ERR_INVALID_ARG;
#ifndef RT_AB_KNOBS
    if (on) return set_err(c, RT_ERR_STATE, "the stats kernels are in the A/B build (librtamd_ab.so)");
#endif
    for (Device& d : c->devs) {
        HIPCHK(c, hipSetDevice(d.id));
        HIPCHK(c, hipStreamSynchronize(d.stream));
        if (on && !d.stats.ptr) {
            HIPCHK(c, hipMalloc(&d.stats.ptr, RT_STATS_N * sizeof(unsigned long long)));
            d.stats.bytes = RT_STATS_N * sizeof(unsigned long long);
        }
        if (d.stats.ptr) HIPCHK(c, hipMemsetAsync(d.stats.ptr, 0, d.stats.bytes, d.stream));
        if (on == 2 && !d.census.ptr) {
            const int waves = rt_resident_waves();
            const size_t bytes = ((size_t)waves + (size_t)waves * RT_CENSUS_CAP * RT_CENSUS_WORDS) * sizeof(unsigned);
            HIPCHK(c, hipMalloc(&d.census.ptr, bytes));
            d.census.bytes = bytes;
            d.census_cap = RT_CENSUS_CAP;
            d.census_waves = waves;
        }
        if (on != 2 && d.census.ptr) {
            dev_free(d.census);
            d.census_cap = d.census_waves = 0;
        }
        if (d.census.ptr) HIPCHK(c, hipMemsetAsync(d.census.ptr, 0, d.census.bytes, d.stream));
        HIPCHK(c, hipStreamSynchronize(d.stream));
    }
    if (on) {
        if (c->variant_no_stats < 0) c->variant_no_stats = c->variant;
        c->variant = stats_twin(c->variant_no_stats);
    } else if (c->variant_no_stats >= 0) {
        c->variant = c->variant_no_stats;
        c->variant_no_stats = -1;
    }
    return RT_OK;
}

int rt_debug_read_census(rt_ctx* c, unsigned* out, size_t words, size_t* needed, int* waves, int* cap) {
    if (!c || c->devs.empty()) return RT_ERR_INVALID_ARG;
    Device& d = c->devs[0];
    const size_t n = d.census.bytes / sizeof(unsigned);
    if (needed) *needed = n;
    if (waves) *waves = d.census_waves;
    if (cap) *cap = d.census_cap;
    if (!out) return RT_OK;
    if (words < n) return set_err(c, RT_ERR_LIMIT, "census buffer too small");
    if (!n) return RT_OK;
    HIPCHK(c, hipSetDevice(d.id));
    return d2h(c, d, out, d.census.ptr, d.census.bytes);
}

// The stats twin's node-hit count (tools/collapse_hits_ab.py): on = 1 allocates and zeroes one word
// per possible link node plus the walk count; the stats twin's launches then add to it.
int rt_debug_count_node_hits(rt_ctx* c, int on) {
    if (!c) return RT_ERR_INVALID_ARG;
    for (Device& d : c->devs) {
        HIPCHK(c, hipSetDevice(d.id));
        HIPCHK(c, hipStreamSynchronize(d.stream));
        if (!on) {
            dev_free(d.node_hits);
            continue;
        }
        const size_t bytes = ((size_t)2 * RT_LINK_MAX_NODES + 1) * sizeof(unsigned);
        if (!d.node_hits.ptr) {
            HIPCHK(c, hipMalloc(&d.node_hits.ptr, bytes));
            d.node_hits.bytes = bytes;
        }
        HIPCHK(c, hipMemset(d.node_hits.ptr, 0, d.node_hits.bytes));
    }
    return RT_OK;
}

// Per link node (the last launch's layout, n_walk_nodes of them) its hits, summed over the devices,
// then the walks begun at the root: n_out = n_walk_nodes + 1 words.
int rt_debug_read_node_hits(rt_ctx* c, unsigned* out, size_t words, size_t* n_out) {
    if (!c || c->devs.empty()) return RT_ERR_INVALID_ARG;
    const size_t n = (size_t)c->n_walk_nodes + 1;
    if (n_out) *n_out = n;
    if (!out) return RT_OK;
    if (words < n) return set_err(c, RT_ERR_LIMIT, "node-hit buffer too small");
    std::memset(out, 0, n * sizeof(unsigned));
    std::vector<unsigned> tmp(n);
    for (Device& d : c->devs) {
        if (!d.node_hits.ptr) return set_err(c, RT_ERR_STATE, "rt_debug_count_node_hits(ctx, 1) first");
        HIPCHK(c, hipSetDevice(d.id));
        HIPCHK(c, hipStreamSynchronize(d.stream));
        HIPCHK(c, hipMemcpy(tmp.data(), d.node_hits.ptr, (n - 1) * sizeof(unsigned), hipMemcpyDeviceToHost));
        HIPCHK(c, hipMemcpy(&tmp[n - 1], (unsigned*)d.node_hits.ptr + (n - 1), sizeof(unsigned), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < n; i++) out[i] += tmp[i];
    }
    return RT_OK;
}

// The collapse planned from measured hits (rt_debug_read_node_hits of an uncollapsed walk over the same
// tree, spine off) instead of the camera grid; n = 0 goes back to the grid.  Exact either way.
int rt_debug_set_collapse_hits(rt_ctx* c, const unsigned* hits, size_t n, unsigned long long walks) {
    if (!c || (n && !hits)) return RT_ERR_INVALID_ARG;
    c->inj_hits.assign(hits, hits + n);
    c->inj_walks = (int64_t)walks;
    c->walk_stale = true;
    return RT_OK;
}

int rt_debug_read_stats(rt_ctx* c, unsigned long long* out, int n) {
    if (!c || !out || n <= 0 || n > RT_STATS_N) return RT_ERR_INVALID_ARG;
    std::memset(out, 0, sizeof(unsigned long long) * n);
    for (Device& d : c->devs) {
        if (!d.stats.ptr) continue;
        HIPCHK(c, hipSetDevice(d.id));
        std::vector<unsigned long long> tmp(n);
        int r = d2h(c, d, tmp.data(), d.stats.ptr, sizeof(unsigned long long) * n);
        if (r) return r;
        for (int i = 0; i < n; i++) out[i] += tmp[i];
    }
    return RT_OK;
}

int rt_debug_ab_build(void) {
#ifdef RT_AB_KNOBS
    return 1;
#else
    return 0;
#endif
}

int rt_debug_set_option(rt_ctx* c, int option, int v) {
    if (!c) return RT_ERR_INVALID_ARG;
    auto bad = [&]() { return set_err(c, RT_ERR_INVALID_ARG, "option value out of range"); };
    switch (option) {
        case RT_OPTION_BOX_PRETEST: c->box_pretest = v != 0; break;
        case RT_OPTION_FASTDIV: c->fastdiv = v != 0; break;
        case RT_OPTION_SPH_LDS: c->sph_lds = v != 0; break;
        case RT_OPTION_BIG_WG: c->big_wg = v != 0; break;
        case RT_OPTION_COMPACT_BOXES: c->compact_boxes = v != 0; break;
        case RT_OPTION_SPINE: c->spine = v != 0; break;
        case RT_OPTION_TL_LEAF_LDS: c->tl_leaf_lds = v != 0; break;
        case RT_OPTION_PERLIN_PACKED: c->perlin_pk = v != 0; break;
        case RT_OPTION_SPARSE_STAGE: c->sparse_stage = v != 0; break;
        case RT_OPTION_SPHERE_PAIRS: if (v < 0 || v > 2) return bad(); c->sphere_pairs = v; break;
        case RT_OPTION_LEAF_PREFETCH: c->leaf_prefetch = v != 0; break;
        case RT_OPTION_TL_SMALL_LDS: c->tl_small_lds = v != 0; break;
        case RT_OPTION_SHADE_LDS: c->shade_lds = v != 0; break;
        case RT_OPTION_BOX_VNODES: c->box_vnodes = v != 0; break;
        case RT_OPTION_ZERO_DIR_END: c->zero_dir_end = v != 0; break;
        case RT_OPTION_COLLAPSE: c->collapse = v != 0; break;
        case RT_OPTION_REBUILD: if (v < 0 || v > 2) return bad(); c->rebuild = v; break;
        case RT_OPTION_CHUNK_TARGET: if (v < 0) return bad(); c->chunk_target = v; break;
        case RT_OPTION_STAGED_CHUNK_TARGET: if (v < 1) return bad(); c->staged_chunk_target = v; break;
        case RT_OPTION_STAGE_TILES: if (v < 0) return bad(); c->stage_tiles = v; break;
        case RT_OPTION_SM_BATCH: if (v < 1 || v > 64) return bad(); c->sm_batch = v; break;
        case RT_OPTION_SM_FRAC: if (v < 0 || v > 64) return bad(); c->sm_frac = v; break;
        case RT_OPTION_WALK_FRAC: if (v < 0 || v > 64) return bad(); c->walk_frac = v; break;
        case RT_OPTION_WATCHDOG_MS: if (v < 0) return bad(); c->watchdog_ticks = (unsigned long long)v * 100000ull; break;
        case RT_OPTION_CHUNK_WAIT_MS: if (v < 0) return bad(); c->chunk_wait_ticks = (unsigned long long)v * 100000ull; break;
        case RT_OPTION_LDS_NODE_CAP: if (v < 0) return bad(); c->lds_node_cap = v; break;
        case RT_OPTION_TAIL_CHUNKS: if (v < -1 || v > RT_MAX_FRAMES_PER_LAUNCH) return bad(); c->tail_chunks = v; break;
#ifdef RT_AB_KNOBS
        case RT_OPTION_KERNEL_VARIANT:
            if (!(v == 0 || v == 30 || v == 31 || v == 37 || v == 38 || v == 39 || v == 61 || v == 69)) return bad();
            c->variant = v;
            break;
        case RT_OPTION_DEBUG_FLAGS: c->debug_flags = v; break;
#endif
        default: return set_err(c, RT_ERR_INVALID_ARG, "unknown option (A/B options need librtamd_ab.so)");
    }
    return RT_OK;
}

int rt_debug_get_option(rt_ctx* c, int option, int* v) {
    if (!c || !v) return RT_ERR_INVALID_ARG;
    switch (option) {
        case RT_OPTION_BOX_PRETEST: *v = c->box_pretest; break;
        case RT_OPTION_FASTDIV: *v = c->fastdiv; break;
        case RT_OPTION_SPH_LDS: *v = c->sph_lds; break;
        case RT_OPTION_BIG_WG: *v = c->big_wg; break;
        case RT_OPTION_COMPACT_BOXES: *v = c->compact_boxes; break;
        case RT_OPTION_SPINE: *v = c->spine; break;
        case RT_OPTION_TL_LEAF_LDS: *v = c->tl_leaf_lds; break;
        case RT_OPTION_PERLIN_PACKED: *v = c->perlin_pk; break;
        case RT_OPTION_SPARSE_STAGE: *v = c->sparse_stage; break;
        case RT_OPTION_SPHERE_PAIRS: *v = c->sphere_pairs; break;
        case RT_OPTION_LEAF_PREFETCH: *v = c->leaf_prefetch; break;
        case RT_OPTION_TL_SMALL_LDS: *v = c->tl_small_lds; break;
        case RT_OPTION_SHADE_LDS: *v = c->shade_lds; break;
        case RT_OPTION_BOX_VNODES: *v = c->box_vnodes; break;
        case RT_OPTION_ZERO_DIR_END: *v = c->zero_dir_end; break;
        case RT_OPTION_COLLAPSE: *v = c->collapse; break;
        case RT_OPTION_REBUILD: *v = c->rebuild; break;
        case RT_OPTION_CHUNK_TARGET: *v = c->chunk_target; break;
        case RT_OPTION_STAGED_CHUNK_TARGET: *v = c->staged_chunk_target; break;
        case RT_OPTION_STAGE_TILES: *v = c->stage_tiles; break;
        case RT_OPTION_SM_BATCH: *v = c->sm_batch; break;
        case RT_OPTION_SM_FRAC: *v = c->sm_frac; break;
        case RT_OPTION_WALK_FRAC: *v = c->walk_frac; break;
        case RT_OPTION_WATCHDOG_MS: *v = (int)std::min<unsigned long long>(INT_MAX, c->watchdog_ticks / 100000ull); break;
        case RT_OPTION_CHUNK_WAIT_MS: *v = (int)std::min<unsigned long long>(INT_MAX, c->chunk_wait_ticks / 100000ull); break;
        case RT_OPTION_LDS_NODE_CAP: *v = c->lds_node_cap; break;
        case RT_OPTION_TAIL_CHUNKS: *v = c->tail_chunks; break;
#ifdef RT_AB_KNOBS
        case RT_OPTION_KERNEL_VARIANT: *v = c->variant; break;
        case RT_OPTION_DEBUG_FLAGS: *v = c->debug_flags; break;
#endif
        default: return set_err(c, RT_ERR_INVALID_ARG, "unknown option (A/B options need librtamd_ab.so)");
    }
    return RT_OK;
}

int rt_set_bvh_mode(rt_ctx* c, int mode) {
    if (!c) return RT_ERR_INVALID_ARG;
    if (mode != RT_BVH_REFERENCE && mode != RT_BVH_SAH) return set_err(c, RT_ERR_INVALID_ARG, "bad BVH mode");
    if (mode != c->bvh_mode) {
        c->bvh_mode = mode;
        c->validated = false;   // validate() rebuilds the links (and a new fast_gen re-uploads them)
    }
    return RT_OK;
}

int rt_debug_walk_bvh(rt_ctx* c, void* out, size_t out_cap, size_t* nbytes) {
    if (!c || !nbytes) return RT_ERR_INVALID_ARG;
    if (!c->uploaded[RT_BIND_BVH]) return set_err(c, RT_ERR_STATE, "no BVH uploaded");
    int r = validate(c);
    if (r) return r;
    const std::vector<uint8_t>& B = c->bvh_mode == RT_BVH_SAH ? c->sah_bvh : c->host_buf[RT_BIND_BVH];
    *nbytes = B.size();
    if (!out) return RT_OK;
    if (out_cap < B.size()) return set_err(c, RT_ERR_LIMIT, "buffer too small");
    if (!B.empty()) std::memcpy(out, B.data(), B.size());
    return RT_OK;
}

int rt_debug_build_sah_bvh(const void* spheres, size_t sph_bytes, const void* quads, size_t quad_bytes,
                           const void* media, size_t med_bytes, const void* boxes, size_t box_bytes,
                           const void* bvh, size_t bvh_bytes, int order, const float eye[3],
                           float prim_cost, void* out, size_t out_cap, size_t* nbytes) {
    if (!nbytes || (bvh_bytes && !bvh) || order < 0 || order > 2 || !(prim_cost > 0.0f)) return RT_ERR_INVALID_ARG;
    rt_sah::Input in;
    in.sph = (const rt_sphere*)spheres;
    in.n_sph = spheres ? sph_bytes / sizeof(rt_sphere) : 0;
    in.quad = (const rt_quad*)quads;
    in.n_quad = quads ? quad_bytes / sizeof(rt_quad) : 0;
    in.med = (const rt_medium*)media;
    in.n_med = media ? med_bytes / sizeof(rt_medium) : 0;
    in.box = (const rt_box*)boxes;
    in.n_box = boxes ? box_bytes / sizeof(rt_box) : 0;
    in.ref = (const rt_bvh_node*)bvh;
    in.n_ref = bvh_bytes / sizeof(rt_bvh_node);
    std::vector<rt_bvh_node> t;
    rt_sah::Builder b(in, order, eye, prim_cost);
    if (!b.build(t)) return RT_ERR_INVALID_ARG;
    *nbytes = t.size() * sizeof(rt_bvh_node);
    if (!out) return RT_OK;
    if (out_cap < *nbytes) return RT_ERR_LIMIT;
    std::memcpy(out, t.data(), *nbytes);
    return RT_OK;
}

int rt_debug_last_launch(rt_ctx* c, int* out, int n) {
    if (!c || !out || n < 0 || n > RT_LI_N) return RT_ERR_INVALID_ARG;
    if (!c->launched) return set_err(c, RT_ERR_STATE, "no render launched yet");
    std::memcpy(out, c->last_launch, sizeof(int) * (size_t)n);
    return RT_OK;
}

int rt_debug_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

}  // extern "C"
