// rt_kernel_variants.hip -- A/B library only (librtamd_ab.so, -DRT_AB_KNOBS): the kernel structures the
// release library does not ship, each bit-identical to it (tests/test_gpu_boundary.py,
// tests/test_gpu_fast.py): 37 the link walk with one pixel per lane (the round-1 default), 30 the
// threaded meta-word nodes (LDS when they fit, else global), 61 the exact near-first stack walk
// over a SAH tree with the reference walk as its fallback, and their region-timer stats twins
// 38 / 31 / 69.  The release structure (render_stream) and its stats twin 39 are rt_kernel.hip's.
// rt_launch_render (rt_kernel.hip) calls rt_launch_render_ab for these shapes.
#ifndef RT_AB_KNOBS
#error "rt_kernel_variants.hip is the A/B library's translation unit (-DRT_AB_KNOBS)"
#endif
#include "rt_kernel_common.h"

namespace {

// compute.glsl:226-266 over the threaded BVH.  Each lane's node sequence is the
// reference's; only the interleaving of a wave's lanes differs: lanes advance
// through inner/missed nodes until each holds a hit leaf (or is done), then the
// leaves are tested together ("while-while").  LINK (variant 0/37): link-format
// nodes; otherwise (variant 30) the threaded nodes with their meta word.  Both
// use the branch-free node step with the NaN-exact min/max slab test.
template <bool LINK, bool STATS, int OPT>
__device__ __forceinline__ bool trace(const KP& P, const float4* __restrict__ nodes, v3 o, v3 d, float time,
                                      float& rf, float px, float py, Hit& h, unsigned long long* st) {
    if (P.n_nodes == 0) return false;
    float tmin = 0.001f, tmax = RT_INFINITY;
    v3 inv = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    float a = g_dot(d, d);
    bool has = false;
    uint32_t i = 0;
    // rays that need the exact slab (see aabb_fast); wave-uniform fast path otherwise
    const bool lane_exact = (inv.x == -INFINITY) || (inv.y == -INFINITY) || (inv.z == -INFINITY);
    const bool wave_exact = __ballot(lane_exact) != 0;   // uniform
    if (LINK) {
        // link-format nodes (rt_device.h RT_LINK_*): the successor is one select
        // between the node's hit and miss words; a hit leaf or the end leaves
        // the loop (sign bit)
        NodeSrc ns;
        ns.base = reinterpret_cast<const char*>(nodes);
        ns.gnodes = nullptr;
        ns.lim = 0;
        ns.hits = nullptr;
        const uint2* __restrict__ leaves = reinterpret_cast<const uint2*>(nodes + P.leaf_lds);
        uint32_t nx = 0u;
        if (STATS) st_lanes(st, ST_TRACE_IT, ST_TRACE_LN);
        for (;;) {
            if (STATS) st_lanes(st, ST_ROUND_IT, ST_ROUND_LN);
            unsigned long long t0 = STATS ? clock64() : 0;
            nx = wave_exact ? link_walk<true, STATS>(ns, nx, o, inv, tmin, tmax, st)
                            : link_walk<false, STATS>(ns, nx, o, inv, tmin, tmax, st);
            if (STATS) st_add(st, ST_NODE_CYC, clock64() - t0);
            if (nx == RT_LINK_END) break;
            unsigned long long t1 = STATS ? clock64() : 0;
            if (STATS) st_lanes(st, ST_LEAF_IT, ST_LEAF_LN);
            const uint2 lf = leaves[nx & 0x7FFFFFFFu];
            leaf_prims_t<STATS, false>(P, lf.x << 16, lf.y, o, d, inv, a, time, tmin, tmax, rf, px, py, h, has, st);
            if (STATS) st_add(st, ST_LEAF_CYC, clock64() - t1);
            nx = lf.x >> 8;
            if (nx == RT_LINK_NEXT_END) break;
        }
        return has;
    }
    // threaded nodes with the meta word: a hit inner node continues at i+1 (its
    // right child), anything else at the skip link; a hit leaf leaves the loop
    // with its prims pending.
    for (;;) {
        uint32_t meta = 0, prims = 0;
        bool leaf = false;
        unsigned long long t0 = STATS ? clock64() : 0;
        if (i != RT_NODE_END) {
            for (;;) {
                if (STATS) st_lanes(st, ST_NODE_IT, ST_NODE_LN);
                float4 n0 = nodes[2 * i], n1 = nodes[2 * i + 1];
                meta = __float_as_uint(n1.z);
                prims = __float_as_uint(n1.w);
                bool hitn;
                if (!wave_exact) {
                    hitn = aabb_fast(n0, n1, o, inv, tmin, tmax);
                } else {
                    float lo = tmin, hi = tmax;
                    slab(n0.x, n0.y, o.x, inv.x, lo, hi);
                    slab(n0.z, n0.w, o.y, inv.y, lo, hi);
                    slab(n1.x, n1.y, o.z, inv.z, lo, hi);
                    hitn = !(hi <= lo);
                }
                bool inner = (meta & 0xF0000u) == 0;
                i = (hitn && inner) ? i + 1 : (meta & 0xFFFFu);
                leaf = hitn && !inner;
                if (leaf || i == RT_NODE_END) break;
            }
        }
        if (STATS) st_add(st, ST_NODE_CYC, clock64() - t0);
        if (!leaf) break;
        unsigned long long t1 = STATS ? clock64() : 0;
        if (STATS) st_lanes(st, ST_LEAF_IT, ST_LEAF_LN);
        leaf_prims_t<STATS, false>(P, meta, prims, o, d, inv, a, time, tmin, tmax, rf, px, py, h, has, st);
        if (STATS) st_add(st, ST_LEAF_CYC, clock64() - t1);
    }
    return has;
}

// ===========================================================================
// Exact near-first walk (variant 61).  The reference walks its own median-split
// BVH in a fixed right-first order (compute.glsl:226-266) and keeps the LAST
// hit it accepts.  For a ray with a finite origin and no -inf/NaN in 1/dir this walk
// returns the same hit from a SAH tree over the BVH's solid prims, visited
// near child first (rt_capi.hip build_fast), and replays the media slots in
// the reference order:
//  * solids have no side effects, so the reference's hit is the closest one
//    among the solid prims it VISITS (its acceptance tests are the same
//    functions), and media draw rand() only in their own slots;
//  * every SAH box contains the reference leaf boxes of the prims below it
//    (joins of exactly those boxes) and rounding is monotone, so an SAH node's
//    slab interval contains theirs: pruning at fprune(best), far above the
//    error of a hit t against its box entry, skips no leaf whose prim could be
//    the reference's closest hit;
//  * the closest solid p is the reference's iff the reference visits p's leaf
//    L(p).  With no other hit within fwin(best), the reference's ray_t.max at
//    L(p) exceeds fwin(best); the reference's boxes nest (boxes_nest), so L(p)
//    passing at fwin(best) means every test on the way to it passes;
//  * a medium slot sees ray_t.max = min(closest solid ranked before it — the
//    tracker, checked like p —, earlier medium hits); its leaf test is exact
//    at that value, or a lower bound of it when only passing matters;
//  * anything inside the windows (near ties, a medium hit next to the closest
//    solid, a medium t above ray_t.max, a failed leaf check) returns a nonzero
//    reason and the caller takes the exact walk with the rand() state restored.
// Windows: fwin for ties and the acceptance check (2^-14 relative + 1e-4),
// fprune for pruning (2^-7 relative + 2e-3).  The host enables the walk only
// when every quad/box face is axis-aligned (plane hits exact to a few ulps),
// the boxes nest and no medium samples an image texture (uv never goes stale).
__device__ __forceinline__ float fwin(float t) { return t * (1.0f + 6.103515625e-05f) + 1.0e-4f; }
__device__ __forceinline__ float fprune(float t) { return t * (1.0f + 7.8125e-03f) + 2.0e-3f; }
__device__ __forceinline__ bool fnear(float x, float y) { return x <= fwin(y) && y <= fwin(x); }
__device__ __forceinline__ float fmin2(float x, float y) { return x < y ? x : y; }
__device__ __forceinline__ float fmax2(float x, float y) { return x > y ? x : y; }
// aabb_fast that also returns the entry distance (near-child-first ordering)
__device__ __forceinline__ bool aabb_lo(float xmn, float xmx, float ymn, float ymx, float zmn, float zmx, v3 o, v3 inv,
                                       float tmin, float tmax, float& lo_out) {
    float t0x = (xmn - o.x) * inv.x, t1x = (xmx - o.x) * inv.x;
    float t0y = (ymn - o.y) * inv.y, t1y = (ymx - o.y) * inv.y;
    float t0z = (zmn - o.z) * inv.z, t1z = (zmx - o.z) * inv.z;
    float lo = v_max(v_max3(tmin, v_min(t0x, t1x), v_min(t0y, t1y)), v_min(t0z, t1z));
    float hi = v_min(v_min3(tmax, v_max(t0x, t1x), v_max(t0y, t1y)), v_max(t0z, t1z));
    lo_out = lo;
    return !(hi <= lo);
}

// The stack walk's tables and this lane's stack (variant 61): two-child nodes
// and leaves (LDS when they fit), stack entry e at stack[e * stride].
struct FastCtx {
    const float4* inner;
    const uint2* leaves;
    short* stack;
    int stride;
};

__device__ __forceinline__ bool ref_leaf_hit(const float4* __restrict__ rn, uint32_t k, v3 o, v3 inv, float tmax) {
    return aabb_fast(rn[2 * k], rn[2 * k + 1], o, inv, 0.001f, tmax);
}

// Two-child nodes, near child first by entry distance, per-lane stack (fc).
template <bool STATS = false>
__device__ __forceinline__ int trace_fast(const KP& P, const float4* __restrict__ rn, const FastCtx& fc, v3 o, v3 d,
                                          float time, float& rf, float px, float py, Hit& h, bool& has,
                                          unsigned long long* st = nullptr) {
    const v3 inv = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    // +inf (a +0 direction component, common: rand() is coarse, so -1 + 2*rand() hits 0) keeps the
    // fast slab test equal to the reference's and monotone in the box; -inf and NaN do not
    if (!(inv.x > -INFINITY && inv.y > -INFINITY && inv.z > -INFINITY)) return 1;
    if (!(fabsf(o.x) < INFINITY && fabsf(o.y) < INFINITY && fabsf(o.z) < INFINITY)) return 8;
    if (!(fabsf(d.x) < INFINITY && fabsf(d.y) < INFINITY && fabsf(d.z) < INFINITY)) return 1;
    const float a = g_dot(d, d);
    const float tmin = 0.001f;
    unsigned long long c_pre = STATS ? clock64() : 0;
    // trackers: boundary of the constrained slot's medium (its exit bounds the
    // solids that can be its ray_t.max) and the closest / second closest solid
    // ranked before the slot
    float t1_0 = 0.0f, t2_0 = 0.0f, t1_1 = 0.0f, t2_1 = 0.0f;
    const bool tb0 = P.fl_n > 0 && medium_bounds(P, P.media[P.fl_medium[0]], o, d, a, time, t1_0, t2_0);
    const bool tb1 = P.fl_n > 1 && medium_bounds(P, P.media[P.fl_medium[1]], o, d, a, time, t1_1, t2_1);
    float lt0 = RT_INFINITY, lt0b = RT_INFINITY, lt1 = RT_INFINITY, lt1b = RT_INFINITY;
    uint32_t ll0 = 0u, ll1 = 0u;
    float pb0 = tb0 ? fprune(t2_0) : -RT_INFINITY;
    float pb1 = tb1 ? fprune(t2_1) : -RT_INFINITY;
    if (STATS) st_add(st, ST_FAST_PRE_CYC, clock64() - c_pre);
    float best = RT_INFINITY, second = RT_INFINITY, pb = RT_INFINITY;
    int bty = 0, bix = 0, bface = 0;
    float bal = 0.0f, bbe = 0.0f;
    uint32_t n_steps = 0, n_tests = 0;   // diagnostics (P.stats)
    // the two prims of a leaf: every hit updates the closest / second closest
    // and the trackers, and tightens the pruning bounds
    auto leaf_test = [&](uint32_t meta, uint32_t prims) {
#pragma unroll 1
        for (int s = 0; s < 2; s++) {
            const int ty = (int)((meta >> (16 + 4 * s)) & 0xFu);
            const int ix = (int)((prims >> (16 * s)) & 0xFFFFu);
            float t = 0.0f, al = 0.0f, be = 0.0f;
            int face = 0;
            bool hit = false;
            n_tests += ty != 0;
            if (ty == RT_MODEL_SPHERE)
                hit = sphere_t(reinterpret_cast<const float4*>(P.spheres + ix), time, o, d, a, tmin, RT_INFINITY, t);
            else if (ty == RT_MODEL_QUAD)
                hit = quad_test(P.dquads + RT_DFACE_F4 * ix, o, d, tmin, RT_INFINITY, t, al, be);
            else if (ty == RT_MODEL_BOX)
                hit = box_test(P.dboxes + RT_DBOX_F4 * ix, o, d, tmin, RT_INFINITY, t, face, al, be);
            if (!hit) continue;
            if (t < best) {
                second = best;
                best = t;
                bty = ty; bix = ix; bface = face; bal = al; bbe = be;
                pb = fprune(best);
            } else if (t < second) {
                second = t;
            }
            if (P.fl_n > 0) {
                const uint32_t w = P.finfo[P.finfo_base[ty] + ix];
                const int rank = (int)(w >> 16);
                if (rank < P.fl_rank[0]) {
                    if (t < lt0) { lt0b = lt0; lt0 = t; ll0 = w & 0xFFFFu; }
                    else if (t < lt0b) lt0b = t;
                    if (tb0) pb0 = fprune(fmin2(lt0, t2_0));
                }
                if (P.fl_n > 1 && rank < P.fl_rank[1]) {
                    if (t < lt1) { lt1b = lt1; lt1 = t; ll1 = w & 0xFFFFu; }
                    else if (t < lt1b) lt1b = t;
                    if (tb1) pb1 = fprune(fmin2(lt1, t2_1));
                }
            }
        }
    };
    {
        constexpr int EMPTY = -0x40000000;   // refs are 16-bit: never a node
        int n = P.n_f2inner > 0 ? 0 : (P.n_f2leaves > 0 ? ~0 : EMPTY);
        int sp = 0;
        for (;;) {
            unsigned long long c0 = STATS ? clock64() : 0;
            while (n >= 0) {   // inner node: test both children, descend into the nearer
                if (STATS) st_lanes(st, ST_NODE_IT, ST_NODE_LN);
                n_steps++;
                const float4 A = fc.inner[4 * n], B = fc.inner[4 * n + 1], C = fc.inner[4 * n + 2];
                const float4 D = fc.inner[4 * n + 3];
                const int rl = __float_as_int(D.x), rr = __float_as_int(D.y);
                const uint32_t tb = __float_as_uint(D.z);
                float bl = pb, br = pb;
                if (tb & 0x001u) bl = fmax2(bl, pb0);
                if (tb & 0x002u) bl = fmax2(bl, pb1);
                if (tb & 0x100u) br = fmax2(br, pb0);
                if (tb & 0x200u) br = fmax2(br, pb1);
                float lol = 0.0f, lor = 0.0f;
                const bool hl = aabb_lo(A.x, A.y, A.z, A.w, B.x, B.y, o, inv, tmin, bl, lol);
                const bool hr = aabb_lo(B.z, B.w, C.x, C.y, C.z, C.w, o, inv, tmin, br, lor);
                if (hl && hr) {
                    if (sp == RT_FAST_STACK) return 9;   // deeper than the stack: the exact walk
                    const bool lfirst = lol <= lor;
                    fc.stack[sp * fc.stride] = (short)(lfirst ? rr : rl);
                    sp++;
                    n = lfirst ? rl : rr;
                } else if (hl || hr) {
                    n = hl ? rl : rr;
                } else {
                    n = sp > 0 ? (int)fc.stack[--sp * fc.stride] : EMPTY;
                }
            }
            if (STATS) st_add(st, ST_NODE_CYC, clock64() - c0);
            if (n == EMPTY) break;
            unsigned long long c1 = STATS ? clock64() : 0;
            if (STATS) st_lanes(st, ST_LEAF_IT, ST_LEAF_LN);
            const uint2 lf = fc.leaves[~n];
            leaf_test(lf.x, lf.y);
            if (STATS) st_add(st, ST_LEAF_CYC, clock64() - c1);
            n = sp > 0 ? (int)fc.stack[--sp * fc.stride] : EMPTY;
        }
    }
    if (STATS) {
        atomicAdd(st + ST_FAST_STEPS, (unsigned long long)n_steps);
        atomicAdd(st + ST_FAST_TESTS, (unsigned long long)n_tests);
    }
    unsigned long long c_post = STATS ? clock64() : 0;
    if (best < RT_INFINITY) {
        if (second <= fwin(best)) return 2;
        if (!ref_leaf_hit(rn, P.finfo[P.finfo_base[bty] + bix] & 0xFFFFu, o, inv, fwin(best))) return 3;
    }
    // media slots in the reference order
    float cur = RT_INFINITY;   // ray_t.max after the media hits so far
    int med = -1, pvis = 2;
#pragma unroll 1
    for (int j = 0; j < P.fm_n; j++) {
        const int mi = P.fm_medium[j], k = P.fm_track[j], flags = P.fm_flags[j];
        const rt_medium m = P.media[mi];
        float t1 = 0.0f, t2 = 0.0f;
        bool bnd;
        if (k == 0) { bnd = tb0; t1 = t1_0; t2 = t2_0; }
        else if (k == 1) { bnd = tb1; t1 = t1_1; t2 = t2_1; }
        else bnd = medium_bounds(P, m, o, d, a, time, t1, t2);
        float R = RT_INFINITY, Tl = cur;
        bool exact = k < 0;   // Tl is the reference's ray_t.max at the slot's leaf, not just a lower bound
        bool verified = false;
        if (k >= 0 && bnd) {
            const float l = k ? lt1 : lt0, lb = k ? lt1b : lt0b;
            if (l < t2) {
                // the closest solid ranked before the slot is its ray_t.max: one the reference accepts
                if (lb <= fwin(l) || fnear(cur, l)) return 4;
                if (!ref_leaf_hit(rn, k ? ll1 : ll0, o, inv, fwin(l))) return 5;
                R = l;
                verified = true;
            }
            // The reference's ray_t.max at the leaf is min(cur, closest accepted solid ranked before
            // the leaf) >= min(cur, l, t2): an earlier-ranked solid below min(l, t2) would be l.  It
            // equals Tl when cur is the smaller one, or when l is verified and no solid precedes the
            // medium inside its own leaf.
            Tl = fmin2(cur, fmin2(l, t2));
            exact = (cur <= fmin2(l, t2)) || (verified && !(flags & 2));
        }
        const float tmax_at = fmin2(cur, R);
        // the clamped interval [max(t1, tmin), min(t2, ray_t.max)] is empty whatever ray_t.max is:
        // hit_constant_medium returns before rand() whether or not the leaf is visited
        const bool no_draw = bnd && !((t1 < tmin ? tmin : t1) < t2);
        int vis;   // the slot's leaf is visited: 1 yes, 0 no, 2 unknown
        if (flags & 1) vis = pvis;
        else if (!bnd) vis = 2;
        else if (ref_leaf_hit(rn, (uint32_t)P.fm_leaf[j], o, inv, Tl)) vis = 1;
        else vis = (exact && !(flags & 2)) ? 0 : 2;
        pvis = vis;
        if (!bnd || vis == 0 || no_draw) continue;   // hit_constant_medium returns before rand()
        if (vis == 2) return 6;
        float tm;
        if (!medium_tail(m.neg_inv_density, t1, t2, a, tmin, tmax_at, rf, px, py, tm)) continue;
        if (!(tm <= tmax_at) || fnear(tm, best)) return 7;
        cur = tm;
        med = mi;
    }
    if (med >= 0 && cur < best) {
        h.t = cur; h.tif = RT_MODEL_CONSTANT_MEDIUM | (med << 16);
        h.uv_kind_idx = 0;
        has = true;
    } else if (best < RT_INFINITY) {
        h.t = best; h.tif = bty | (bface << 4) | (bix << 16);
        h.uv_kind_idx = (bty == RT_MODEL_SPHERE) ? ((1 << 16) | bix) : (2 << 16);
        h.uv_a = (bty == RT_MODEL_SPHERE) ? best : bal;
        h.uv_b = bbe;
        has = true;
    } else {
        has = false;
    }
    if (STATS) st_add(st, ST_FAST_POST_CYC, clock64() - c_post);
    return 0;
}

// Diagnostic counters of the near-first walk (stats builds; st = the wave's LDS counters).
__device__ __forceinline__ void fast_count(unsigned long long* st, int why) {
    const unsigned long long all = __ballot(1), fb = __ballot(why != 0);
    if (first_active_lane()) {
        atomicAdd(st + ST_FAST_TRACES, (unsigned long long)__popcll(all));
        atomicAdd(st + ST_FAST_EXACT, (unsigned long long)__popcll(fb));
    }
    if (why) atomicAdd(st + ST_FAST_WHY + why - 1, 1ull);   // reasons 1..9
}

// One iteration of ray_color's loop (compute.glsl:304-340).
template <bool LINK, bool STATS, bool FAST, int OPT>
__device__ __forceinline__ bool bounce(const KP& P, const float4* __restrict__ nodes, const FastCtx& fc, Path& S,
                                       float px, float py, v3& result, unsigned long long* st) {
    if (S.depth >= P.max_depth) {   // loop exhausted: final_color stays vec3(0)
        result = mk3s(0.0f);
        return true;
    }
    S.depth++;
    v3 d = S.d;
    Hit h;
    h.t = 0.0f; h.tif = 0;
    h.uv_kind_idx = 0; h.uv_a = 0.0f; h.uv_b = 0.0f;
    // A zero direction (Q1 isotropic corner) can hit nothing and consumes no rand().
    bool dir_zero = (d.x == 0.0f) && (d.y == 0.0f) && (d.z == 0.0f);
    bool hit = false;
    if (dir_zero) {
    } else if (FAST && P.fast_ok) {
        const float rf0 = S.rf;
        bool fh = false;
        const int why = trace_fast<STATS>(P, nodes, fc, S.o, d, S.time, S.rf, px, py, h, fh, st);
        if (STATS) fast_count(st, why);
        if (why == 0) {
            hit = fh;
        } else {   // the exact walk, from the same rand() state
            unsigned long long c_ex = STATS ? clock64() : 0;
            S.rf = rf0;
            hit = trace<LINK, STATS, OPT>(P, nodes, S.o, d, S.time, S.rf, px, py, h, st);
            if (STATS) st_add(st, ST_FAST_EXACT_CYC, clock64() - c_ex);
        }
    } else {
        hit = trace<LINK, STATS, OPT>(P, nodes, S.o, d, S.time, S.rf, px, py, h, st);
    }
    unsigned long long ts = STATS ? clock64() : 0;
    if (STATS) st_lanes(st, ST_SHADE_IT, ST_SHADE_LN);
    const bool done = after_trace(P, S, h, hit, px, py, result);
    if (STATS) st_add(st, ST_SHADE_CYC, clock64() - ts);
    return done;
}

// compute.glsl:345-358 for frames [f0, f1) of the launch, for the pixel at
// column x of local (stripe-compacted) row lr, with the running mean
// (compute.glsl:355) kept in the lane's LDS slot `acc` between frames (not in
// registers: the four floats would be live across the whole bounce loop, which
// costs spills at 128 VGPRs).  Path regeneration: a lane whose path ended
// starts its next frame at once; each pixel still runs its frames in order, and
// the mean is applied per frame in the reference's order.
template <bool LINK, bool STATS, bool FAST, int OPT>
__device__ __forceinline__ void render_pixel(const KP& P, const float4* __restrict__ nodes, const FastCtx& fc, int x,
                                             int lr, int f0, int f1, float4* acc, unsigned long long* st) {
    const uint32_t pix = (uint32_t)lr * (uint32_t)P.width + (uint32_t)x;   // local pixel index (staged chunks)
    int gstripe = (lr / P.stripe_rows) * P.world + P.rank;
    int y = gstripe * P.stripe_rows + lr % P.stripe_rows;
    const rt_camera_ubo& C = P.cam;
    float fx = (float)x, fy = (float)y;
    // get_norm_coord (compute.glsl:268-283) before its jitter term: per pixel
    v3 base = add3(add3(ld3(C.up_left), scale3(ld3(C.pixel_delta_u), fx)), scale3(ld3(C.pixel_delta_v), fy));
    Path S;
    int f = f0;
    bool fresh = true;
    for (;;) {
        if (fresh) {
            if (f >= f1) break;
            unsigned long long t0 = STATS ? clock64() : 0;
            if (STATS) st_lanes(st, ST_START_IT, ST_START_LN);
            start_path(P, S, P.first_frame + f, P.rand_factors[f], fx, fy, base);
            if (STATS) st_add(st, ST_START_CYC, clock64() - t0);
            fresh = false;
        }
        v3 cur;
        if (bounce<LINK, STATS, FAST, OPT>(P, nodes, fc, S, fx, fy, cur, st)) {
            if (P.samples) {   // staged chunks: fold_kernel applies the running mean in frame order
                P.samples[(size_t)f * P.n_pixels + pix] = make_float4(cur.x, cur.y, cur.z, 0.0f);
            } else {
                int fc = P.first_frame + f;
                float n1 = (float)(fc - 1), n = (float)fc;
                float4 prev = *acc;
                prev.x = (prev.x * n1 + cur.x) / n;
                prev.y = (prev.y * n1 + cur.y) / n;
                prev.z = (prev.z * n1 + cur.z) / n;
                prev.w = 1.0f;
                *acc = prev;
            }
            f++;
            fresh = true;
        }
    }
}

// Pooled unit (variant 0): the wave's 64 lanes share the unit's samples -- the
// tile's nv valid pixels x its kf frames, sample s = frame-in-chunk * nv + pixel
// -- instead of each lane owning one pixel.  A lane whose path ends takes the
// next unclaimed sample (one ballot per loop iteration: the lanes needing work
// get consecutive indices by mbcnt), so no lane idles while the wave still has
// samples, whichever pixels' paths run long.  A sample's bits depend only on
// its pixel and frame (random.glsl:2-7), not on the lane that runs it.  Colours
// go to `out` by (frame-in-chunk, pixel slot = py * 8 + px): the unit's per-wave
// slot (ordered / one chunk; the caller folds them in frame order) or, for
// staged chunks, straight to P.samples.
// Sample s of a pooled unit (frame-in-chunk * nv + pixel) to the wave's slot (by
// frame-in-chunk and the pixel's slot py * 8 + px) or, staged, to P.samples.
__device__ __forceinline__ void store_sample(const KP& P, float4* wslot, uint32_t s, uint32_t nv, int wt, int tx0,
                                             int ly0, int f0, v3 cur) {
    const uint32_t fl = s / nv, p = s - fl * nv;
    const uint32_t py = p / (uint32_t)wt, px = p - py * (uint32_t)wt;
    const float4 c4 = make_float4(cur.x, cur.y, cur.z, 0.0f);
    if (wslot)
        wslot[fl * 64u + py * 8u + px] = c4;
    else
        P.samples[(size_t)(f0 + (int)fl) * P.n_pixels + (uint32_t)(ly0 + (int)py) * (uint32_t)P.width +
                  (uint32_t)(tx0 + (int)px)] = c4;
}

template <bool LINK, bool STATS, bool FAST, int OPT>
__device__ __forceinline__ void render_pool(const KP& P, const float4* __restrict__ nodes, const FastCtx& fc,
                                            int tx0, int ly0, int wt, int ht, int f0, int kf, float4* wslot,
                                            unsigned long long* st) {
    const uint32_t nv = (uint32_t)(wt * ht), total = nv * (uint32_t)kf;
    const rt_camera_ubo& C = P.cam;
    uint32_t next = 0;   // first unclaimed sample (the same in every lane)
    uint32_t s = 0;
    float fx = 0.0f, fy = 0.0f;
    Path S;
    bool fresh = true;
    for (;;) {
        const unsigned long long need = __ballot(fresh);
        if (fresh)
            s = next + __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
        next += (uint32_t)__popcll(need);
        if (fresh) {
            if (s >= total) break;
            const uint32_t fl = s / nv, p = s - fl * nv;
            const int lr = ly0 + (int)(p / (uint32_t)wt), x = tx0 + (int)(p % (uint32_t)wt);
            const int y = ((lr / P.stripe_rows) * P.world + P.rank) * P.stripe_rows + lr % P.stripe_rows;
            fx = (float)x;
            fy = (float)y;
            unsigned long long t0 = STATS ? clock64() : 0;
            if (STATS) st_lanes(st, ST_START_IT, ST_START_LN);
            // get_norm_coord (compute.glsl:268-283) before its jitter term
            const v3 base =
                add3(add3(ld3(C.up_left), scale3(ld3(C.pixel_delta_u), fx)), scale3(ld3(C.pixel_delta_v), fy));
            const int f = f0 + (int)fl;
            start_path(P, S, P.first_frame + f, P.rand_factors[f], fx, fy, base);
            if (STATS) st_add(st, ST_START_CYC, clock64() - t0);
            fresh = false;
        }
        v3 cur;
        if (bounce<LINK, STATS, FAST, OPT>(P, nodes, fc, S, fx, fy, cur, st)) {
            store_sample(P, wslot, s, nv, wt, tx0, ly0, f0, cur);
            fresh = true;
        }
    }
}

// Persistent kernel: one resident grid; each workgroup stages the BVH (link
// format, 57 KB for scene 8), the Perlin table and the media records in LDS
// once, then each wave repeatedly takes the next work unit from a device-wide
// counter (one returning atomic per unit) until the counter passes the last
// unit — a condition every wave reaches.
//   LINK: link-format node loop (variant 0/37) vs threaded meta nodes (30);
//   LDSN: the nodes are staged in LDS (else read from global memory);
//   FAST: the exact near-first stack walk (variant 61) with the reference walk
//         as its fallback.
template <bool LINK, int MINW, bool STATS, bool LDSN, int BLOCK, bool FAST, int OPT = 0>
__global__ void __launch_bounds__(BLOCK, MINW) render_persistent_ab(const KP* __restrict__ Pp) {
    const KP& P = *Pp;
    extern __shared__ float4 s_nodes[];
    __shared__ unsigned long long s_stats[STATS ? BLOCK / 64 : 1][STATS ? ST_N : 1];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    unsigned long long* st = nullptr;
    unsigned long long t_begin = 0;
    if (STATS) {
        for (int k = tid; k < (BLOCK / 64) * ST_N; k += BLOCK) (&s_stats[0][0])[k] = 0;
        st = s_stats[tid / 64];
    }
    // FAST keeps its two-child tree + stack in LDS (the reference nodes stay in
    // global memory: leaf checks and the rare exact walk); otherwise LDSN stages
    // the reference's nodes, then the Perlin table and the media records
    FastCtx fc;
    fc.inner = P.f2inner;
    fc.leaves = P.f2leaves;
    fc.stack = nullptr;
    fc.stride = BLOCK;
    if (FAST) {
        const int n4 = 4 * P.n_f2inner, nl4 = (P.n_f2leaves + 1) / 2;
        if (LDSN) {
            for (int k = tid; k < n4; k += BLOCK) s_nodes[k] = P.f2inner[k];
            const float4* gl = reinterpret_cast<const float4*>(P.f2leaves);
            for (int k = tid; k < P.n_f2leaves / 2; k += BLOCK) s_nodes[n4 + k] = gl[k];
            if ((P.n_f2leaves & 1) && tid == 0) {
                const uint2 last = P.f2leaves[P.n_f2leaves - 1];
                reinterpret_cast<uint2*>(s_nodes + n4)[P.n_f2leaves - 1] = last;
            }
            fc.inner = s_nodes;
            fc.leaves = reinterpret_cast<const uint2*>(s_nodes + n4);
            fc.stack = reinterpret_cast<short*>(s_nodes + n4 + nl4) + tid;
        } else {
            fc.stack = reinterpret_cast<short*>(s_nodes) + tid;
        }
    } else if (LDSN) {
        stage_lds<LINK, BLOCK>(P, s_nodes, tid);
    }
    // per lane: the pixel's running mean during a unit, after what this launch
    // shape stages (P.acc_lds, set by rt_launch_render with the LDS size)
    float4* s_acc = s_nodes + P.acc_lds;
    if (LDSN || STATS) __syncthreads();
    if (STATS) t_begin = clock64();
    const float4* __restrict__ rnodes = (LDSN && !FAST) ? s_nodes : reinterpret_cast<const float4*>(P.nodes);
    const int tiles_x = (P.width + 7) >> 3;
    const int n_tiles = tiles_x * ((P.local_rows + 7) >> 3);
    const int n_units = n_tiles * P.n_chunks;
    for (;;) {
        int unit = 0;
        if (lane == 0) unit = atomicAdd(P.tile_counter, 1);
        unit = __builtin_amdgcn_readfirstlane(__shfl(unit, 0));   // wave-uniform (scalar)
        if (unit >= n_units) break;
        const int chunk = unit / n_tiles, tile = unit - chunk * n_tiles;
        const int f0 = chunk * P.chunk_frames;
        const int f1 = min(P.n_frames, f0 + P.chunk_frames);
        const int x = (tile % tiles_x) * 8 + (lane & 7);
        const int lr = (tile / tiles_x) * 8 + (lane >> 3);
        const bool valid = x < P.width && lr < P.local_rows;   // lane 0 (the tile's corner) always is
        const bool ordered = P.samples == nullptr;             // else staged: chunks independent
        if (OPT & RT_OPT_POOL) {
            const int tx0 = x - (lane & 7), ly0 = lr - (lane >> 3);
            float4* wslot =
                ordered ? P.wbuf + ((size_t)blockIdx.x * (BLOCK / 64) + (tid >> 6)) * 64 * P.chunk_frames : nullptr;
            render_pool<LINK, STATS, FAST, OPT>(P, rnodes, fc, tx0, ly0, min(8, P.width - tx0),
                                                min(8, P.local_rows - ly0), f0, f1 - f0, wslot, st);
            if (!ordered) continue;
            // the unit's colours, written by any lane of this wave, folded by the pixel's lane
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            if (chunk > 0) wait_chunk(P, tile, chunk);
            if (valid) {
                float4* px = reinterpret_cast<float4*>(P.image) + (size_t)lr * P.width + x;
                float4 prev = *px;
                for (int f = f0; f < f1; f++) {
                    const float4 cur = wslot[(f - f0) * 64 + lane];
                    const int fcnt = P.first_frame + f;
                    const float n1 = (float)(fcnt - 1), n = (float)fcnt;
                    prev.x = (prev.x * n1 + cur.x) / n;
                    prev.y = (prev.y * n1 + cur.y) / n;
                    prev.z = (prev.z * n1 + cur.z) / n;
                    prev.w = 1.0f;
                }
                *px = prev;
            }
            if (chunk + 1 < P.n_chunks) publish_chunk(P, tile, chunk);
            continue;
        }
        if (ordered && chunk > 0) wait_chunk(P, tile, chunk);
        if (valid) {
            float4* px = reinterpret_cast<float4*>(P.image) + (size_t)lr * P.width + x;
            if (ordered) s_acc[tid] = *px;
            render_pixel<LINK, STATS, FAST, OPT>(P, rnodes, fc, x, lr, f0, f1, s_acc + tid, st);
            if (ordered) *px = s_acc[tid];
        }
        if (ordered && chunk + 1 < P.n_chunks) publish_chunk(P, tile, chunk);
    }
    if (STATS) {
        st_add(st, ST_TOTAL, clock64() - t_begin);
        __syncthreads();
        if (tid < ST_N) {
            unsigned long long v = 0;
            for (int w = 0; w < BLOCK / 64; w++) v += s_stats[w][tid];
            atomicAdd(P.stats + tid, v);
        }
    }
}


}  // namespace

int rt_launch_render_ab(int shape, rt_kernel_args& a, const rt_kernel_args* d, size_t lds, bool stats, void* stream) {
    hipStream_t st = (hipStream_t)stream;
#define RT_KERNEL(LINK, LDSN, BLOCK, FAST, OPT)                                                                     \
    (stats ? launch_persistent(render_persistent_ab<LINK, 4, true, LDSN, BLOCK, FAST, OPT>, BLOCK, lds, a, d, st)  \
           : launch_persistent(render_persistent_ab<LINK, 4, false, LDSN, BLOCK, FAST, OPT>, BLOCK, lds, a, d, st))
    switch (shape) {
        case RT_AB_SHAPE_FAST_LDS: return RT_KERNEL(false, true, 512, true, 0);
        case RT_AB_SHAPE_FAST_GLOBAL: return RT_KERNEL(false, false, 512, true, 0);
        case RT_AB_SHAPE_LINK_PIXEL: return RT_KERNEL(true, true, 512, false, 0);
        case RT_AB_SHAPE_META_LDS: return RT_KERNEL(false, true, 512, false, 0);
        case RT_AB_SHAPE_META_GLOBAL: return RT_KERNEL(false, false, 512, false, 0);
        default: return -1;
    }
#undef RT_KERNEL
}
