// rt_kernel.hip — the MI355X (gfx950) path-tracing kernel.
//
// Semantics: the reference's per-invocation compute shader
// (S/raytrace/compute.glsl:345-358 + S/utils/*.glsl), bit-exact with the CPU
// oracle given the shared GLSL built-in definitions (include/rt/rt_glsl.h) and
// -ffp-contract=off.  Structure (MI355X-first; every change value-preserving):
//   * persistent grid: each workgroup stages the threaded BVH in LDS once and
//     each wave pulls units (8x8 pixel tile x a chunk of the launch's frames)
//     from a device-wide counter;
//   * the wave's lanes share the unit's samples (render_pool): a lane whose
//     path ended takes the next unclaimed (pixel, frame); the colours are
//     folded into the RGBA32F running mean (compute.glsl:355) per pixel in
//     frame order at the end of the unit, so the image is read/written once
//     per unit (variant 37: a lane owns one pixel and regenerates only its own
//     frames);
//   * stackless walk of a threaded BVH (rt_dnode) visiting the reference's node
//     sequence (stack pops, right child first) without the int stack[64];
//   * lean hit record during the walk (t, type, index, box face, uv source);
//     p, normal and front face are rebuilt once for the closest hit with the
//     reference's own expressions, and set_material_properties
//     (compute.glsl:197-224) / texture_color run once per bounce, only when
//     the value is used;
//   * per-ray constants hoisted (1/dir, dot(dir,dir)); a box's six face planes
//     are divided independently before the sequential acceptance; a medium's
//     two boundary hits share one quadratic.
// rand() consumption order is identical to the reference.
#include "rt_kernel_common.h"

namespace {

// Walks and shading in batches (RT_OPT_SM, link-format walk): every lane is
// FRESH (needs a sample), TRACE (its walk is running), HIT (walk done, to be
// shaded) or BEGIN (a new walk, set up in the next pass).  The wave runs rounds
// of node walk + leaf tests for its TRACE lanes until P.sm_batch lanes are HIT,
// or P.sm_frac/64 of the lanes with a walk, or none is tracing, then shades the
// HIT lanes together; lanes whose path goes on start their next walk, the others
// store their sample and claim the next.  So a lane whose walk ended early does
// not wait for the wave's longest walk: it is shaded with the next batch while
// the other lanes' walks continue from where they stopped (the walk position nx,
// ray_t.max and the hit record are the lane's own, so each walk is the
// reference's, as in trace()).  FD (P.fastdiv): the rounds' leaf tests use the
// shared-reciprocal divisions (one form of the leaf code per kernel keeps the hot
// loop's registers).
#define RT_SM_FRESH 0
#define RT_SM_TRACE 1
#define RT_SM_HIT 2
#define RT_SM_BEGIN 4
//
// The batched walks over a stream of units (RT_OPT_STREAM): when the wave's current unit
// has no unclaimed samples left, the wave claims its next unit and its free lanes
// take that unit's samples while the other lanes finish the previous unit's paths
// (before, they idled through the unit's tail: 8.5% of lane-rounds on scene 8).
// Ordered / one-chunk launches keep up to two units in flight, each with its slot
// of wbuf (2 per wave); a unit is folded into the image once all its samples are
// stored, oldest first, so a wave only ever waits (wait_chunk) for units claimed
// before its oldest one and the waits cannot form a cycle.  Staged launches store
// straight to P.samples and need no slots.  A lane's sample is its pixel (fx, fy),
// its slot `up` and its colour's place `dst` (slot offset frame-in-chunk * 64 +
// pixel slot, or the staged index).
struct UnitGeo {
    int chunk, tile, tx0, ly0, wt, ht, f0, f1;
    uint32_t total;
};
__device__ __forceinline__ UnitGeo unit_geo(const KP& P, int u, int n_tiles, int tiles_x) {
    UnitGeo g;
    g.chunk = u / n_tiles;
    g.tile = u - g.chunk * n_tiles;
    g.tx0 = (g.tile % tiles_x) * 8;
    g.ly0 = (g.tile / tiles_x) * 8;
    g.wt = min(8, P.width - g.tx0);
    g.ht = min(8, P.local_rows - g.ly0);
    // the grid's last units are the tail chunks' (units are claimed chunk by chunk): one frame each,
    // so waves finish within a short unit of each other
    const int c_main = P.n_chunks - P.tail_chunks;
    if (g.chunk < c_main) {
        g.f0 = g.chunk * P.chunk_frames;
        g.f1 = min(P.n_frames - P.tail_chunks, g.f0 + P.chunk_frames);
    } else {
        g.f0 = P.n_frames - (P.n_chunks - g.chunk);
        g.f1 = g.f0 + 1;
    }
    g.total = (uint32_t)(g.wt * g.ht * (g.f1 - g.f0));
    return g;
}
// Where a new walk (tmin 0.001, tmax infinite) starts: the root, or past the spine (KP spine_*)
// when the ray hits each of its boxes for sure.  Per axis k of such a box [lo, hi] with
// lo + m < o_k < hi - m, m = 0.00125 max|d| (> 0 for a walked ray): the far slab distance is
// (hi - o_k) / |d_k| >= m / |d_k| (1 - 3 ulp) > 0.001 (d_k = +-0: +inf, and no 0 * inf since
// o_k != lo, hi), the near one is negative, so the reference's slab loop (hitting.glsl:55-76) keeps
// ray_t = (0.001, min far) and reports a hit.  The host's 2^-18 shrink of the box covers the
// rounding of lo + m and hi - m.  Non-finite o or d: the root.
__device__ __forceinline__ uint32_t spine_entry(const KP& P, const v3& o, const v3& d) {
    if (P.spine_len == 0) return 0u;
    const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    const bool fin = ax <= __FLT_MAX__ && ay <= __FLT_MAX__ && az <= __FLT_MAX__;
    const float m = 0.00125f * fmaxf(ax, fmaxf(ay, az));
    const bool in = fin && o.x > P.spine_lo[0] + m && o.x < P.spine_hi[0] - m && o.y > P.spine_lo[1] + m &&
                    o.y < P.spine_hi[1] - m && o.z > P.spine_lo[2] + m && o.z < P.spine_hi[2] - m;
    return in ? P.spine_start : 0u;
}

template <bool STATS, int OPT, bool FD>
__device__ __forceinline__ void render_stream(const KP& P, const float4* __restrict__ nodes, int gwave,
                                              unsigned long long* st) {
    constexpr bool TL = (OPT & RT_OPT_TL) != 0;
    constexpr bool BOXC = (OPT & RT_OPT_BOXC) != 0;
    const int lane = threadIdx.x & 63;
    constexpr bool STD = (OPT & RT_OPT_STD) != 0;
    const bool staged = STD || P.samples != nullptr;
    const bool sparse = STD || P.sflags != nullptr;   // (staged launches)
    const int tiles_x = (P.width + 7) >> 3;
    const int n_tiles = tiles_x * ((P.local_rows + 7) >> 3);
    const int n_units = n_tiles * P.n_chunks;
    const uint32_t slot_f4 = 64u * (uint32_t)P.chunk_frames;
    float4* const wbase = staged ? nullptr : P.wbuf + (size_t)gwave * 2 * slot_f4;
    const rt_camera_ubo& C = P.cam;
    NodeSrc ns;
    ns.base = reinterpret_cast<const char*>(nodes);
    ns.gnodes = reinterpret_cast<const char*>(P.lnodes);
    ns.lim = (uint32_t)P.lds_node_f4 * 16u;
    ns.hits = STATS ? P.node_hits : nullptr;
    // the leaf records: LDS after the staged nodes, or (two-level walk, when they did not fit
    // beside its nodes) global memory after the node array
    const bool gleaf = TL && P.leaf_lds < 0;   // wave-uniform
    const uint2* __restrict__ leaves = reinterpret_cast<const uint2*>(nodes + (P.leaf_lds >= 0 ? P.leaf_lds : 0));
    const uint2* __restrict__ gleaves = reinterpret_cast<const uint2*>(P.lnodes + 2 * P.n_nodes);
    const int batch = P.sm_batch;
    // wave-uniform: the units in the two slots (-1 = free) and their stored samples;
    // the pool: its unit, slot and next unclaimed sample
    int unit0 = -1, unit1 = -1;
    uint32_t done0 = 0, done1 = 0;
    int cur = 1;
    uint32_t next = 0, total_cur = 0;
    bool no_more = false;
    UnitGeo gc = unit_geo(P, 0, n_tiles, tiles_x);   // the pool unit's geometry
    // per lane
    int up = 0;
    uint32_t dst = 0;
    float fx = 0.0f, fy = 0.0f;
    Path S;
    Hit h;
    bool has = false;
    float tmax = RT_INFINITY, a = 0.0f;
    v3 inv = mk3s(0.0f);
    uint32_t nx = RT_LINK_END;
    int status = RT_SM_FRESH;
    // a progress watchdog: on its first pass and every 256th, a wave that has stored no
    // sample since the previous check more than P.watchdog_ticks ago (120 s by default)
    // sets the fault word (rt_sync reports it) and leaves, so a bug cannot keep the grid
    // resident; a long launch that keeps storing samples never trips it
    unsigned long long t_prog = __builtin_amdgcn_s_memrealtime();
    uint32_t stored = 0, stored_seen = 0;   // wave-uniform: samples this wave stored
    uint32_t pass = 0;
    // the stats twin's pass-part timers (ST_PASS_CYC ... ST_PTAIL_CYC): tq = the current part's start
    unsigned long long tq = 0, tq0 = 0;
#define RT_ST_PART(slot)                                  \
    if (STATS) {                                          \
        const unsigned long long tn_ = clock64();         \
        st_add(st, (slot), tn_ - tq);                     \
        tq = tn_;                                         \
    }
    for (;;) {
        if (STATS) {
            tq0 = tq = clock64();
            st_add(st, ST_PASS_IT, 1ull);
        }
        if ((pass++ & 255u) == 0) {
            const unsigned long long now = __builtin_amdgcn_s_memrealtime();
            if (now - t_prog >= P.watchdog_ticks) {
                __hip_atomic_store((gu32*)P.fault, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            if (stored != stored_seen) {
                stored_seen = stored;
                t_prog = now;
            }
        }
        RT_ST_PART(ST_WATCH_CYC)
        // fold the units whose samples are all stored, oldest first (ordered / one chunk)
        if (!staged) {
#pragma unroll 1
            for (int k = 0; k < 2; k++) {
                const bool l0 = unit0 >= 0, l1 = unit1 >= 0;
                if (!l0 && !l1) break;
                const int p = (l0 && (!l1 || unit0 < unit1)) ? 0 : 1;
                const UnitGeo g = unit_geo(P, p ? unit1 : unit0, n_tiles, tiles_x);
                if ((p == cur && next < g.total) || (p ? done1 : done0) < g.total) break;
                // all of the unit's colours are in slot p: fold them per pixel in frame order
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                if (g.chunk > 0) wait_chunk(P, g.tile, g.chunk);
                if ((lane & 7) < g.wt && (lane >> 3) < g.ht) {
                    const float4* ws = wbase + (size_t)p * slot_f4;
                    float4* px = reinterpret_cast<float4*>(P.image) + (size_t)(g.ly0 + (lane >> 3)) * P.width +
                                 g.tx0 + (lane & 7);
                    float4 prev = *px;
                    for (int f = g.f0; f < g.f1; f++) {
                        const float4 c4 = ws[(f - g.f0) * 64 + lane];
                        const int fcnt = P.first_frame + f;
                        const float n1 = (float)(fcnt - 1), n = (float)fcnt;
                        prev.x = (prev.x * n1 + c4.x) / n;
                        prev.y = (prev.y * n1 + c4.y) / n;
                        prev.z = (prev.z * n1 + c4.z) / n;
                        prev.w = 1.0f;
                    }
                    *px = prev;
                }
                if (g.chunk + 1 < P.n_chunks) publish_chunk(P, g.tile, g.chunk);
                if (p) {
                    unit1 = -1;
                    done1 = 0;
                } else {
                    unit0 = -1;
                    done0 = 0;
                }
            }
        }
        RT_ST_PART(ST_FOLD_CYC)
        // claim samples for the FRESH lanes (compute.glsl:345-350); a new unit when the
        // pool's unit has none left
        bool fin = false;   // a sample stored in this pass (max_depth 0)
        for (;;) {
            if (STATS) st_add(st, ST_CLAIM_IT, 1ull);
            const unsigned long long need = __ballot(status == RT_SM_FRESH);
            if (need == 0) break;
            if (next >= total_cur) {
                if (no_more) break;
                const int o = staged ? 0 : cur ^ 1;
                if (!staged && (o ? unit1 : unit0) >= 0) break;   // both slots in use: the FRESH lanes wait
                int u = 0;
                unsigned long long ta = STATS ? clock64() : 0;
                if (lane == 0) u = atomicAdd(P.tile_counter, 1);
                u = __builtin_amdgcn_readfirstlane(__shfl(u, 0));
                if (STATS) {
                    st_add(st, ST_ATOM_CYC, clock64() - ta);
                    st_add(st, ST_UNIT_IT, 1ull);
                }
                if (u >= n_units) {
                    no_more = true;
                    break;
                }
                if (!staged) {
                    if (o) unit1 = u;
                    else unit0 = u;
                }
                cur = o;
                gc = unit_geo(P, u, n_tiles, tiles_x);
                total_cur = gc.total;
                next = 0;
                continue;
            }
            if (status == RT_SM_FRESH) {
                const uint32_t s = next + __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
                if (s < total_cur) {
                    // sample s of the pool unit: frame-in-chunk, then pixel (shifts for a full tile)
                    uint32_t fl, py, px;
                    if (gc.wt == 8 && gc.ht == 8) {
                        fl = s >> 6;
                        py = (s >> 3) & 7u;
                        px = s & 7u;
                    } else {
                        const uint32_t nv = (uint32_t)(gc.wt * gc.ht);
                        fl = s / nv;
                        const uint32_t pp = s - fl * nv;
                        py = pp / (uint32_t)gc.wt;
                        px = pp - py * (uint32_t)gc.wt;
                    }
                    const int lr = gc.ly0 + (int)py, x = gc.tx0 + (int)px;
                    const int y = P.world == 1 ? lr
                                               : ((lr / P.stripe_rows) * P.world + P.rank) * P.stripe_rows +
                                                     lr % P.stripe_rows;
                    const int f = gc.f0 + (int)fl;
                    up = cur;
                    dst = staged ? (uint32_t)f * (uint32_t)P.n_pixels + (uint32_t)lr * (uint32_t)P.width + (uint32_t)x
                                 : fl * 64u + py * 8u + px;
                    fx = (float)x;
                    fy = (float)y;
                    unsigned long long t0 = STATS ? clock64() : 0;
                    if (STATS) st_lanes(st, ST_START_IT, ST_START_LN);
                    const v3 pbase = add3(add3(ld3(C.up_left), scale3(ld3(C.pixel_delta_u), fx)),
                                          scale3(ld3(C.pixel_delta_v), fy));
                    start_path(P, S, P.first_frame + f, P.rand_factors[f], fx, fy, pbase);
                    if (STATS) st_add(st, ST_START_CYC, clock64() - t0);
                    if (P.max_depth <= 0) {   // the loop never runs: final_color vec3(0)
                        const float4 z4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                        if (staged) {
                            if (sparse) P.sflags[dst] = 0;   // sparse: a zero colour is its clear flag
                            else P.samples[dst] = z4;
                        } else {
                            wbase[(size_t)up * slot_f4 + dst] = z4;
                        }
                        fin = true;
                    } else {
                        status = RT_SM_BEGIN;
                    }
                }
            }
            next = min(next + (uint32_t)__popcll(need), total_cur);
            if (__ballot(fin)) break;   // count these before claiming more (below)
        }
        RT_ST_PART(ST_CLAIM_CYC)
        // a new walk (bounce(): depth, a zero direction hits nothing, compute.glsl:226-229)
        if (status == RT_SM_BEGIN) {
            S.depth++;
            h.t = 0.0f; h.tif = 0;
            h.uv_kind_idx = 0; h.uv_a = 0.0f; h.uv_b = 0.0f;
            has = false;
            tmax = RT_INFINITY;
            nx = spine_entry(P, S.o, S.d);
            const bool dir_zero = (S.d.x == 0.0f) && (S.d.y == 0.0f) && (S.d.z == 0.0f);
            status = (dir_zero || P.n_nodes == 0) ? RT_SM_HIT : RT_SM_TRACE;
            if (STATS) st_lanes(st, ST_TRACE_IT, ST_TRACE_LN);
            // the walk's per-ray constants, kept while it runs (a resumed walk has them)
            inv = mk3(1.0f / S.d.x, 1.0f / S.d.y, 1.0f / S.d.z);
            a = g_dot(S.d, S.d);
            if (STATS && P.node_hits) {   // the walks begun at the root (rt_debug_count_node_hits)
                const unsigned long long m = __ballot(status == RT_SM_TRACE && nx == 0u);
                if (m && first_active_lane()) atomicAdd(&P.node_hits[P.n_nodes], (unsigned)__popcll(m));
            }
        }
        // rounds of node walk + leaf tests (trace()), at wave priority 1: their dependent LDS
        // chains then issue as soon as their data is back, and the shading's long VALU runs (at
        // priority 0) fill the gaps -- scene 8 -3.1%, scene 0 -2.1%, scenes 6 / 7 -0.4 / -1.2%
        // (profiles/r04_setprio_combined_lib_ab.log; the walk alone at 1: scene 6 +0.6%)
        RT_ST_PART(ST_BEGIN_CYC)
        __builtin_amdgcn_s_setprio(1);
        for (;;) {
            unsigned long long th = STATS ? clock64() : 0;
            const unsigned long long tr = __ballot(status == RT_SM_TRACE);
            const int n_hit = __popcll(__ballot(status == RT_SM_HIT));
            if (STATS && tr) st_pred(st, status == RT_SM_FRESH, ST_RET_IT, ST_RET_LN);
            if (tr == 0 || n_hit >= batch || n_hit * 64 >= P.sm_frac * (n_hit + __popcll(tr))) break;
            const bool lane_exact = (inv.x == -INFINITY) || (inv.y == -INFINITY) || (inv.z == -INFINITY);
            const bool wave_exact = __ballot(status == RT_SM_TRACE && lane_exact) != 0;
            if (STATS) st_add(st, ST_RHEAD_CYC, clock64() - th);
            if (status == RT_SM_TRACE) {
                if (STATS) st_lanes(st, ST_ROUND_IT, ST_ROUND_LN);
                unsigned long long t0 = STATS ? clock64() : 0;
                if (P.walk_frac >= 64) {
                    nx = wave_exact ? link_walk<true, STATS, TL>(ns, nx, S.o, inv, 0.001f, tmax, st)
                                    : link_walk<false, STATS, TL>(ns, nx, S.o, inv, 0.001f, tmax, st);
                } else {
                    const int needw = (__popcll(__ballot(1)) * P.walk_frac + 63) >> 6;
                    nx = wave_exact ? link_walk_part<true, STATS, TL>(ns, nx, S.o, inv, 0.001f, tmax, needw, st)
                                    : link_walk_part<false, STATS, TL, (BOXC || (RT_BL_SPAIR && (OPT & RT_OPT_SPAIR) != 0)) && STD>(ns, nx, S.o, inv, 0.001f, tmax,
                                                                                    needw, st);
                }
                if (STATS) st_add(st, ST_NODE_CYC, clock64() - t0);
                if ((int)nx >= 0) {
                    // still walking: the next round goes on from nx
                } else if (nx == RT_LINK_END) {
                    status = RT_SM_HIT;
                } else {
                    unsigned long long t1 = STATS ? clock64() : 0;
                    if (STATS) st_lanes(st, ST_LEAF_IT, ST_LEAF_LN);
                    uint2 lf;
                    if (gleaf) lf = ldg_u2(gleaves + (nx & 0x7FFFFFFFu));
                    else lf = leaves[nx & 0x7FFFFFFFu];
                    leaf_prims_t<STATS, FD, BOXC, (OPT & RT_OPT_SPAIR) != 0, STD>(P, lf.x << 16, lf.y, S.o, S.d, inv, a,
                                                                             S.time, 0.001f, tmax, S.rf,
                                                  fx, fy, h, has, st);
                    if (STATS) {
                        const unsigned long long t2 = clock64();
                        st_add(st, ST_LEAF_CYC, t2 - t1);
                        if (P.census) census_leaf(P, gwave, lf.x, t1, t2, __popcll(tr), st);
                    }
                    nx = lf.x >> 8;   // the leaf's skip node
                    if (nx == RT_LINK_NEXT_END) status = RT_SM_HIT;
                }
            }
        }
        __builtin_amdgcn_s_setprio(0);
        RT_ST_PART(ST_ROUNDS_CYC)
        // shade the HIT lanes together
        if (status == RT_SM_HIT) {
            unsigned long long ts = STATS ? clock64() : 0;
            if (STATS) st_lanes(st, ST_SHADE_IT, ST_SHADE_LN);
            v3 cur3;
            h.t = tmax;   // the accepted hit's t (unused on a miss)
            bool done = after_trace<BOXC, STATS, STD>(P, S, h, has, fx, fy, cur3, st);
            if (!done && S.depth >= P.max_depth) {   // the loop is exhausted: final_color stays vec3(0)
                cur3 = mk3s(0.0f);
                done = true;
            } else if (!done && P.zero_dir_end && S.d.x == 0.0f && S.d.y == 0.0f && S.d.z == 0.0f) {
                // a zero direction (the no-light mixture branch, SURVEY App. A Q1: an isotropic
                // scatter goes on along vec3(0)): the next bounce hits nothing and draws no rand()
                // (bounce(), compute.glsl:226-229, 308-309), so its miss colour -- acc x background
                // with the acc of now -- is the path's colour; taken here instead of one more pass
                cur3 = mul3(S.acc, mk3(P.background[0], P.background[1], P.background[2]));
                done = true;
            }
            if (done) {
                const float4 c4 = make_float4(cur3.x, cur3.y, cur3.z, 0.0f);
                if (staged) {
                    // sparse staging (P.sflags): every sample writes one flag byte, and only a colour
                    // that is not exactly (+0, +0, +0) is stored; fold_kernel reads a clear flag as
                    // that zero colour -- the same values, so the same running mean
                    if (sparse) {
                        const bool nz = (__float_as_uint(cur3.x) | __float_as_uint(cur3.y) | __float_as_uint(cur3.z)) != 0u;
                        P.sflags[dst] = nz ? 1 : 0;
                        if (nz) P.samples[dst] = c4;
                    } else {
                        P.samples[dst] = c4;
                    }
                } else {
                    wbase[(size_t)up * slot_f4 + dst] = c4;
                }
                fin = true;
                status = RT_SM_FRESH;
            } else {
                status = RT_SM_BEGIN;
            }
            if (STATS) st_add(st, ST_SHADE_CYC, clock64() - ts);
        }
        RT_ST_PART(ST_SHBLK_CYC)
        // the samples stored in this pass, per slot
        const unsigned long long f_all = __ballot(fin), f_one = __ballot(fin && up == 1);
        done0 += (uint32_t)__popcll(f_all & ~f_one);
        done1 += (uint32_t)__popcll(f_one);
        stored += (uint32_t)__popcll(f_all);
        // the end: no unit left to claim, every lane idle, every slot folded
        if (STATS) {
            RT_ST_PART(ST_PTAIL_CYC)
            st_add(st, ST_PASS_CYC, tq - tq0);
        }
        if (no_more && __ballot(status != RT_SM_FRESH) == 0 && (staged || (unit0 < 0 && unit1 < 0))) break;
    }
#undef RT_ST_PART
}

// Persistent kernel: one resident grid; each workgroup stages the link-format BVH, the Perlin
// table, the media, sphere and box records and the shading tables in LDS once (stage_lds), then
// each wave streams over work units taken from a device-wide counter (render_stream; one
// returning atomic per unit) until the counter passes the last unit -- a condition every wave
// reaches.  STATS: the region-timer twin (A/B library only).
template <int MINW, bool STATS, int BLOCK, int OPT>
__global__ void __launch_bounds__(BLOCK, MINW) render_persistent(const KP* __restrict__ Pp) {
    const KP& P = *Pp;
    extern __shared__ float4 s_nodes[];
    __shared__ unsigned long long s_stats[STATS ? BLOCK / 64 : 1][STATS ? ST_N : 1];
    const int tid = threadIdx.x;
    unsigned long long* st = nullptr;
    unsigned long long t_begin = 0;
    if (STATS) {
        for (int k = tid; k < (BLOCK / 64) * ST_N; k += BLOCK) (&s_stats[0][0])[k] = 0;
        st = s_stats[tid / 64];
    }
    stage_lds<true, BLOCK>(P, s_nodes, tid);
    __syncthreads();
    if (STATS) t_begin = clock64();
    render_stream<STATS, OPT, (OPT & RT_OPT_FD) != 0>(P, s_nodes, (int)blockIdx.x * (BLOCK / 64) + (tid >> 6), st);
    if (STATS) {
        st_add(st, ST_TOTAL, clock64() - t_begin);
        const int gw = (int)blockIdx.x * (BLOCK / 64) + (tid >> 6);
        if (P.census && (tid & 63) == 0 && gw < P.census_waves) P.census[gw] = (unsigned)st[ST_CEN_N];
        __syncthreads();
        if (tid < ST_N) {
            unsigned long long v = 0;
            for (int w = 0; w < BLOCK / 64; w++) v += s_stats[w][tid];
            atomicAdd(P.stats + tid, v);
        }
    }
}

// Staged-chunk epilogue: the running mean of compute.glsl:355 over the launch's
// frames, in frame order, per pixel: (prev*(n-1)+cur)/n -- the operations the
// ordered path applies in LDS, so the same bits.
__global__ void __launch_bounds__(256) fold_kernel(const KP* __restrict__ Pp) {
    const KP& P = *Pp;
    const size_t pix = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (pix >= P.n_pixels) return;
    float4* px = reinterpret_cast<float4*>(P.image) + pix;
    float4 prev = *px;
    const float4* s = P.samples + pix;
    if (P.sflags) {   // sparse staging: a clear flag is the colour (+0, +0, +0), never stored
        // eight frames at a time: their flags, then the set ones' colours, all loads issued
        // before the eight folds (which stay in frame order)
        const uint8_t* fl = P.sflags + pix;
        int f = 0;
        for (; f + 8 <= P.n_frames; f += 8) {
            uint32_t fb[8];
            float4 cur[8];
#pragma unroll
            for (int k = 0; k < 8; k++) fb[k] = fl[(size_t)(f + k) * P.n_pixels];
#pragma unroll
            for (int k = 0; k < 8; k++)
                cur[k] = fb[k] ? s[(size_t)(f + k) * P.n_pixels] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const int fc = P.first_frame + f + k;
                const float n1 = (float)(fc - 1), n = (float)fc;
                prev.x = (prev.x * n1 + cur[k].x) / n;
                prev.y = (prev.y * n1 + cur[k].y) / n;
                prev.z = (prev.z * n1 + cur[k].z) / n;
                prev.w = 1.0f;
            }
        }
        for (; f < P.n_frames; f++) {
            const float4 cur = fl[(size_t)f * P.n_pixels] ? s[(size_t)f * P.n_pixels] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            const int fc = P.first_frame + f;
            const float n1 = (float)(fc - 1), n = (float)fc;
            prev.x = (prev.x * n1 + cur.x) / n;
            prev.y = (prev.y * n1 + cur.y) / n;
            prev.z = (prev.z * n1 + cur.z) / n;
            prev.w = 1.0f;
        }
    } else {
        for (int f = 0; f < P.n_frames; f++) {
            const float4 cur = s[(size_t)f * P.n_pixels];
            const int fc = P.first_frame + f;
            const float n1 = (float)(fc - 1), n = (float)fc;
            prev.x = (prev.x * n1 + cur.x) / n;
            prev.y = (prev.y * n1 + cur.y) / n;
            prev.z = (prev.z * n1 + cur.z) / n;
            prev.w = 1.0f;
        }
    }
    *px = prev;
}

// Gathered stripe blocks [world][padded_rows][W] float4 -> the image [H][W] (row 0 = top):
// row y belongs to stripe s = y / stripe_rows, rendered by rank s % world as its local row
// (s / world) * stripe_rows + y % stripe_rows (rt_set_partition).  One thread per pixel,
// coalesced along the row on both sides.
__global__ void __launch_bounds__(256) deinterleave_kernel(const float4* __restrict__ g, float4* __restrict__ out,
                                                           int width, int height, int world, int stripe_rows,
                                                           int padded_rows) {
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= width || y >= height) return;
    int k, lr;
    rt_gathered_row(y, world, stripe_rows, &k, &lr);
    out[(size_t)y * width + x] = g[((size_t)k * padded_rows + lr) * width + x];
}

__global__ void eval_builtin_kernel(int fn, const float* __restrict__ x, const float* __restrict__ y,
                                    float* __restrict__ out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float r = 0.0f;
    switch (fn) {
        case 0: r = g_sin(x[i]); break;
        case 1: r = g_cos(x[i]); break;
        case 2: r = g_log(x[i]); break;
        case 3: r = g_acos(x[i]); break;
        case 4: r = g_atan2(x[i], y ? y[i] : 1.0f); break;
        case 5: r = g_fract(x[i]); break;
        case 6: r = sqrtf(x[i]); break;
        case 7: r = g_inversesqrt(x[i]); break;
        // the leaf tests' division forms (rcp_nr / div_nr) against the compiler's '/'
        case 100: r = x[i] / y[i]; break;
        case 101: r = div_nr(x[i], y[i], rcp_nr(y[i])); break;
        case 102: r = div_nr(x[i], y[i], -rcp_nr(-y[i])); break;   // an opposite face's shared reciprocal
        default: break;
    }
    out[i] = r;
}

}  // namespace


int rt_resident_waves(void) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    return cus * 2 * (512 / 64);   // every shape: at most 2 workgroups of 512 per CU (launch_persistent)
}

int rt_launch_render(rt_kernel_args& a, rt_kernel_args* dargs, void* stream, int* info) {
    if (a.local_rows <= 0 || a.width <= 0 || a.n_frames <= 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    // The release library has one kernel structure (tests/test_gpu_*.py pin it to the oracle):
    // pooled samples streamed over units with walks and shading in batches (render_stream) over
    // link-format nodes staged in LDS with the Perlin table, media, sphere and box records the
    // host placed after them (a.lds_end_f4), 4 waves per SIMD, as 2 x 512 or 1 x 1024 threads
    // per CU (a.block); when the nodes do not fit (a.lds_node_f4 < 2 n_nodes) the two-level
    // walk reads the nodes below the staged top levels from global memory (1024 threads).
    // Each in a shared-reciprocal division form (a.fastdiv) and the plain one.
    // The A/B build (RT_AB_KNOBS) adds the other structures, all bit-identical
    // (RT_OPTION_KERNEL_VARIANT): 37 the link walk with one pixel per lane (the round-1
    // default), 30 threaded meta-word nodes (LDS when they fit, else global), 61 the exact
    // near-first stack walk, and the region-timer stats twins 39 / 38 / 31 / 69.
    enum { FAST_LDS, FAST_GLOBAL, LINK_LDS, META_LDS, META_GLOBAL, LINK_TL } shape = LINK_LDS;
    size_t staged = (size_t)a.lds_end_f4 * 16;
    bool stats = false, pool = true;
    const bool tl = a.n_lnode_f4 > 0 && a.lds_node_f4 < 2 * a.n_nodes;
    if (tl) shape = LINK_TL;
#ifdef RT_AB_KNOBS
    stats = a.variant == 38 || a.variant == 31 || a.variant == 69 || a.variant == 39;
    pool = a.variant == 0 || a.variant == 39;
    if (a.variant == 61 || a.variant == 69) {
        const size_t stack_b = (size_t)RT_FAST_STACK * 512 * sizeof(short);
        const size_t tree_b = (size_t)a.n_f2inner * 64 + (size_t)((a.n_f2leaves + 1) / 2) * 16;
        shape = tree_b + stack_b <= RT_LDS_DYN_BYTES ? FAST_LDS : FAST_GLOBAL;
        staged = shape == FAST_LDS ? tree_b + stack_b : stack_b;
    } else if (a.variant == 30 || a.variant == 31 || (!pool && tl)) {
        // threaded meta-word nodes, then what the host placed after the link-format nodes
        const size_t lds_t = (size_t)a.n_nodes * sizeof(rt_dnode);
        staged = std::max(lds_t, staged);
        shape = (lds_t <= RT_LDS_NODE_BYTES && staged <= RT_LDS_DYN_BYTES) ? META_LDS : META_GLOBAL;
    }
    if (shape == FAST_LDS || shape == FAST_GLOBAL || shape == META_GLOBAL) {   // nothing else staged
        if (shape == META_GLOBAL) staged = 0;
        a.perlin_lds = a.media_lds = a.sph_lds = a.box_cmp_lds = -1;
        a.sph_mat_lds = a.box_mat_lds = a.tex_lds = -1;
    }
#endif
    if ((shape == LINK_LDS || shape == LINK_TL) && staged > (a.block == 1024 ? RT_LDS_BIG_BYTES : RT_LDS_DYN_BYTES))
        return -1;
    if (shape == LINK_TL && (a.block != 1024 || !pool)) return -1;
    if (pool && !a.samples && !a.wbuf) return -1;   // pooled ordered / one-chunk units need the per-wave slots
    // the leaf record prefetch reads only tables that are staged (the A/B shapes above may drop them)
    a.leaf_pf = (a.leaf_pf && a.box_all_cmp && a.sph_lds >= 0 && a.box_cmp_lds > a.sph_lds &&
                 (a.n_media == 0 || a.media_lds >= 0)) ? 1 : 0;
    // the one-pixel-per-lane kernels (A/B) keep the lanes' running means in LDS after what is staged
    a.acc_lds = (int)(staged / 16);
    const size_t lds = staged + (pool ? 0 : RT_LDS_ACC_BYTES);
    if (info) {
        info[RT_LI_SHAPE] = (int)shape;
        info[RT_LI_BLOCK] = (shape == LINK_LDS || shape == LINK_TL) ? a.block : 512;
        info[RT_LI_FASTDIV] = a.fastdiv;
        info[RT_LI_PRETEST] = a.box_margin > 0.0f;
        info[RT_LI_LDS] = (int)lds;
        info[RT_LI_LDS_NODES] = (shape == LINK_LDS || shape == LINK_TL) ? a.lds_node_f4 / 2 : 0;
        info[RT_LI_COMPACT] = a.box_all_cmp + 2 * (a.box_cmp_lds >= 0);
        info[RT_LI_STAGED] = a.samples != nullptr;
        info[RT_LI_CHUNKS] = a.n_chunks;
        info[RT_LI_SPINE] = pool ? a.spine_len : 0;
        info[RT_LI_SPARSE] = a.samples && a.sflags ? 1 : 0;
        info[RT_LI_SPAIR] = (pool && shape == LINK_LDS && a.sph_lds >= 0 &&
                             ((a.sph_pairs && !a.box_all_cmp) || (a.sph_pairs == 2 && a.fastdiv))) ? 1 : 0;
        info[RT_LI_LEAF_PF] = (pool && (shape == LINK_LDS || shape == LINK_TL)) ? a.leaf_pf : 0;
        info[RT_LI_WALK_FRAC] = a.walk_frac;
        info[RT_LI_SHADE_LDS] = (a.sph_mat_lds >= 0) + 2 * (a.box_mat_lds >= 0) + 4 * (a.tex_lds >= 0);
    }
    // Arguments live in device memory: the by-value kernarg struct would be copied
    // to scratch as soon as a non-inlined device function takes its address.
    // `a` is a pinned staging slot; same-stream ordering makes one device slot
    // safe to reuse per launch.
    if (hipMemcpyAsync(dargs, &a, sizeof(a), hipMemcpyHostToDevice, st) != hipSuccess) return -1;
    const rt_kernel_args* d = (const rt_kernel_args*)dargs;
    // the work-unit counter, then (ordered chunks) the tiles' published chunk counts
    const int n_tiles = ((a.width + 7) / 8) * ((a.local_rows + 7) / 8);
    if (hipMemsetAsync(a.tile_counter, 0, sizeof(int), st) != hipSuccess) return -1;
    if (a.n_chunks > 1 && !a.samples &&
        hipMemsetAsync(a.tile_done, 0, sizeof(unsigned) * (size_t)n_tiles, st) != hipSuccess)
        return -1;

    constexpr int SM = RT_OPT_POOL | RT_OPT_SM | RT_OPT_STREAM;
    // the instantiations: <MINW, STATS, BLOCK, OPT> (stats twins in the A/B build only)
#ifdef RT_AB_KNOBS
#define RT_KERNEL(BLOCK, OPT)                                                                            \
    (stats ? launch_persistent(render_persistent<4, true, BLOCK, OPT>, BLOCK, lds, a, d, st)                \
           : launch_persistent(render_persistent<4, false, BLOCK, OPT>, BLOCK, lds, a, d, st))
#else
#define RT_KERNEL(BLOCK, OPT) launch_persistent(render_persistent<4, false, BLOCK, OPT>, BLOCK, lds, a, d, st)
#endif
    int rc = -1;
    // the default launch's configuration (RT_OPT_STD) holds: the kernels with it compiled in
    const bool std_cfg = a.samples && a.sflags && a.media_sph &&
                         (a.n_sph_lds == 0 || (a.sph_lds >= 0 && a.sph_mat_lds >= 0)) &&
                         (a.n_media == 0 || a.media_lds >= 0) && (a.n_box_lds == 0 || a.box_cmp_lds >= 0) &&
                         (!a.box_all_cmp || (a.leaf_pf && a.box_mat_lds >= 0)) && a.tex_lds >= 0;
    // the link shapes x (shared-reciprocal division | plain) x (compact boxes | full box records)
#define RT_LINK4(BLOCK, OPT)                                                                                 \
    (a.fastdiv ? (a.box_all_cmp ? (std_cfg ? RT_KERNEL(BLOCK, (OPT) | RT_OPT_FD | RT_OPT_BOXC | RT_OPT_STD)            \
                                           : RT_KERNEL(BLOCK, (OPT) | RT_OPT_FD | RT_OPT_BOXC))                         \
                                : (std_cfg ? RT_KERNEL(BLOCK, (OPT) | RT_OPT_FD | RT_OPT_STD)                            \
                                           : RT_KERNEL(BLOCK, (OPT) | RT_OPT_FD)))                                      \
               : (a.box_all_cmp ? RT_KERNEL(BLOCK, (OPT) | RT_OPT_BOXC) : RT_KERNEL(BLOCK, (OPT))))
    // ... and, for a scene whose leaves are mostly sphere pairs (a.sph_pairs), without compact boxes
#define RT_LINK4S(BLOCK, OPT)                                                                                 \
    ((a.sph_pairs == 2 && a.box_all_cmp && a.fastdiv) ? RT_KERNEL(BLOCK, (OPT) | RT_OPT_FD | RT_OPT_BOXC | RT_OPT_SPAIR) : \
    (a.sph_pairs && !a.box_all_cmp)                                                                          \
         ? (a.fastdiv ? (std_cfg ? RT_KERNEL(BLOCK, (OPT) | RT_OPT_FD | RT_OPT_SPAIR | RT_OPT_STD)                      \
                                 : RT_KERNEL(BLOCK, (OPT) | RT_OPT_FD | RT_OPT_SPAIR))                                \
                      : RT_KERNEL(BLOCK, (OPT) | RT_OPT_SPAIR))                                                       \
         : RT_LINK4(BLOCK, OPT))
    switch (shape) {
        case LINK_LDS:
            if (!pool) {
#ifdef RT_AB_KNOBS
                rc = rt_launch_render_ab(RT_AB_SHAPE_LINK_PIXEL, a, d, lds, stats, st);
#endif
            } else if (a.block == 1024) {
                rc = RT_LINK4S(1024, SM);
            } else {
                rc = RT_LINK4S(512, SM);
            }
            break;
        case LINK_TL: rc = RT_LINK4(1024, SM | RT_OPT_TL); break;
#ifdef RT_AB_KNOBS
        case FAST_LDS: rc = rt_launch_render_ab(RT_AB_SHAPE_FAST_LDS, a, d, lds, stats, st); break;
        case FAST_GLOBAL: rc = rt_launch_render_ab(RT_AB_SHAPE_FAST_GLOBAL, a, d, lds, stats, st); break;
        case META_LDS: rc = rt_launch_render_ab(RT_AB_SHAPE_META_LDS, a, d, lds, stats, st); break;
        case META_GLOBAL: rc = rt_launch_render_ab(RT_AB_SHAPE_META_GLOBAL, a, d, lds, stats, st); break;
#endif
        default: break;
    }
#undef RT_KERNEL
#undef RT_LINK4
#undef RT_LINK4S
    if (rc) return rc;
    if (a.samples) {   // staged chunks: the running mean over the launch's frames
        const unsigned blocks = (unsigned)((a.n_pixels + 255) / 256);
        hipLaunchKernelGGL(fold_kernel, dim3(blocks), dim3(256), 0, st, d);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int rt_launch_deinterleave(const void* gathered, void* out, int width, int height, int world, int stripe_rows,
                           int padded_rows, void* stream) {
    if (width <= 0 || height <= 0) return 0;
    hipLaunchKernelGGL(deinterleave_kernel, dim3((unsigned)((width + 255) / 256), (unsigned)height), dim3(256), 0,
                       (hipStream_t)stream, (const float4*)gathered, (float4*)out, width, height, world, stripe_rows,
                       padded_rows);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int rt_launch_eval_builtin(int fn, const float* dx, const float* dy, float* dout, int n, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(eval_builtin_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, fn, dx, dy, dout,
                       n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
