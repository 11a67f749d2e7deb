// rt_kernel_common.h -- the device code both kernel translation units share (included once per
// TU, inside its anonymous namespace): the GLSL restatement's primitives, leaf tests, link walks,
// textures, sampling and shading, the ordered-chunk hand-off, the LDS staging and the persistent
// launcher.  rt_kernel.hip builds the release structure on it (render_stream);
// (rt_kernel_variants.hip, A/B library only, -DRT_AB_KNOBS) the other structures (one pixel per lane, threaded meta-word
// nodes, the exact near-first walk) and their stats twins.  rand() consumption order is identical
// to the reference.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "rt/rt_glsl.h"
#include "rt_device.h"


namespace {

typedef rt_kernel_args KP;

// OPT bits of the kernel templates
// the branchless walk (link_walk_part BL) in the sphere-pair STD kernels too (scene 0: -0.8%,
// profiles/r06_ae_bl_spair_lib_ab.log); the compact-box STD kernels always
#ifndef RT_BL_SPAIR
#define RT_BL_SPAIR 1
#endif
#define RT_OPT_POOL 1   // pooled units (render_pool): without it a lane owns a pixel (variant 37)
#define RT_OPT_SM 2     // with RT_OPT_POOL and the link walk: walks and shading in batches (render_stream)
#define RT_OPT_FD 4     // with RT_OPT_SM: the scene is in the shared-reciprocal division regime (P.fastdiv)
#define RT_OPT_STREAM 8 // with RT_OPT_SM: the wave streams over units (render_stream) instead of one at a time
#define RT_OPT_TL 16    // with RT_OPT_STREAM: two-level walk (top levels in LDS, the rest of the nodes global)
#define RT_OPT_BOXC 32  // with RT_OPT_STREAM: every box has a compact record (box_test_compact), no full box test
#define RT_OPT_SPAIR 64 // with RT_OPT_STREAM: leaves of two spheres tested at once (leaf_prims_t; most leaves are)
#define RT_OPT_STD 128  // the default launch's configuration, compiled in (rt_launch_render std_config takes these
                        // kernels when it holds): staged chunks with sparse staging (P.samples, P.sflags), every
                        // medium bounded by a sphere (P.media_sph; no out-of-line boundary call), the leaf and
                        // shading tables in LDS (spheres, media, box records, sphere materials, texture
                        // descriptors) and with RT_OPT_BOXC the compact boxes' materials and the leaf record
                        // prefetch (P.leaf_pf: the leaf stage holds only the prefetched forms).  Fewer wave-uniform
                        // flags live through the rounds: the C3 kernel 128 -> 117 VGPRs, SGPR spills 34 -> 0

// The kernels' dynamic LDS (render_persistent stages the BVH there, then the
// Perlin table and the media records when P.perlin_lds / P.media_lds >= 0).
extern __shared__ float4 rt_dyn_lds[];

__device__ __forceinline__ v3 f3(float4 v) { return mk3(v.x, v.y, v.z); }

// Scene records through global-address-space loads (global_load, not flat): the
// record pointers come from the argument block, so the compiler cannot infer
// their address space; flat loads also count against the LDS counter, which makes
// the walk's LDS reads wait on them.
typedef float f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const f4v g_f4v;
typedef __attribute__((address_space(1))) const float g_f;
typedef __attribute__((address_space(3))) const float lds_f;
__device__ __forceinline__ float4 ldg(const float4* p) {
    const f4v v = *(const g_f4v*)p;
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ int ldg_i(const int* p) { return *(__attribute__((address_space(1))) const int*)p; }
// The same loads through the constant address space: with a uniform address (a record every lane
// reads, e.g. the lights' in lights_pdf_value) the compiler issues a scalar load (s_load, the
// scalar cache, no vector registers); with a divergent one an ordinary vector load.
typedef __attribute__((address_space(4))) const f4v c_f4v;
__device__ __forceinline__ float4 ldc(const float4* p) {
    const f4v v = *(const c_f4v*)p;
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ int ldc_i(const int* p) { return *(__attribute__((address_space(4))) const int*)p; }
typedef unsigned u2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint2 ldg_u2(const uint2* p) {
    const u2v v = *(__attribute__((address_space(1))) const u2v*)p;
    return make_uint2(v.x, v.y);
}

// ---- diagnostic statistics (stats variants only; never in a timed build) ----
// Wave-level: the first active lane adds into the wave's LDS counters, so a
// region is charged once per wave execution whatever its EXEC mask.
enum {
    ST_TOTAL = 0, ST_START_CYC, ST_START_IT, ST_START_LN, ST_NODE_CYC, ST_NODE_IT, ST_NODE_LN, ST_LEAF_CYC,
    ST_LEAF_IT, ST_LEAF_LN, ST_SPH_LN, ST_QUAD_LN, ST_BOX_LN, ST_MED_LN, ST_SHADE_CYC, ST_SHADE_IT, ST_SHADE_LN,
    ST_SPH_IT, ST_QUAD_IT, ST_BOX_IT, ST_MED_IT,
    // near-first walk (variants 60/61): traces, those that took the exact walk (and why: 9 reasons),
    // node steps and prim tests
    ST_FAST_TRACES, ST_FAST_EXACT, ST_FAST_WHY, ST_FAST_STEPS = ST_FAST_WHY + 9, ST_FAST_TESTS,
    ST_FAST_PRE_CYC, ST_FAST_POST_CYC, ST_FAST_EXACT_CYC,
    // leaf stage by prim type: wave-cycles from the slot's start to the end of that type's test
    // (the types run one after another in this order, so each includes the ones before it)
    ST_SPH_CYC, ST_QUAD_CYC, ST_BOX_CYC, ST_MED_CYC,
    // link walk: traces begun (wave calls, lanes), and rounds of its node-walk + leaf loop with the
    // lanes whose trace is still running (the rest wait for the wave's longest trace)
    ST_TRACE_IT, ST_TRACE_LN, ST_ROUND_IT, ST_ROUND_LN,
    // render_stream rounds: lanes of the wave idle (no sample to claim: the tail of the launch)
    ST_RET_IT, ST_RET_LN,
    // wave executions with 1..8 active lanes (a wave64 VALU instruction with <= 8 exec lanes
    // occupies the SIMD 1.4-5x longer than with >= 9 in a register-only loop: tools/exec_ops.hip):
    // the leaf slots' type blocks and the node steps
    ST_SPH_SM, ST_QUAD_SM, ST_BOX_SM, ST_MED_SM, ST_NODE_SM,
    // shading (round 5): wave-cycles of its parts -- the hit record, the material's scatter, the
    // mixture pdf, the texture lookups -- and the material blocks' executions and lanes
    ST_SH_HIT_CYC, ST_SH_SCAT_CYC, ST_SH_MIX_CYC, ST_SH_TEX_CYC, ST_SH_LAM_IT, ST_SH_LAM_LN, ST_SH_ISO_IT,
    ST_SH_ISO_LN, ST_SH_MET_IT, ST_SH_MET_LN, ST_SH_DIE_IT, ST_SH_DIE_LN,
    // render_stream's scheduling (round 6): passes of its loop and the wave-cycles
    // of each part of a pass -- the watchdog check, the unit folds, the claim loop (which holds
    // START), its iterations, units claimed and the unit counter's atomic, the new walks' set-up,
    // the rounds (which hold NODE and LEAF) and their loop heads, the shading block (SHADE's
    // first-lane timer runs inside it) and the pass tail; the leaf census' per-wave record count
    ST_PASS_IT, ST_PASS_CYC, ST_WATCH_CYC, ST_FOLD_CYC, ST_CLAIM_CYC, ST_CLAIM_IT, ST_UNIT_IT, ST_ATOM_CYC,
    ST_BEGIN_CYC, ST_ROUNDS_CYC, ST_RHEAD_CYC, ST_SHBLK_CYC, ST_PTAIL_CYC, ST_CEN_N, ST_N
};
// 16 waves x ST_N x 8 B of static LDS in a 1024-thread stats twin: <= 10 KB (RT_LDS_BIG_STATS_BYTES)
static_assert(ST_N <= 80, "the stats twins' static counters fit 10 KB per 1024-thread workgroup");
__device__ __forceinline__ bool first_active_lane() {
    unsigned long long m = __ballot(1);
    return (unsigned)__lane_id() == (unsigned)(__ffsll((long long)m) - 1);
}
__device__ __forceinline__ void st_add(unsigned long long* st, int slot, unsigned long long v) {
    if (first_active_lane()) atomicAdd(&st[slot], v);
}
__device__ __forceinline__ void st_lanes(unsigned long long* st, int it_slot, int ln_slot) {
    unsigned long long m = __ballot(1);
    if (first_active_lane()) {
        atomicAdd(&st[it_slot], 1ull);
        atomicAdd(&st[ln_slot], (unsigned long long)__popcll(m));
    }
}
__device__ __forceinline__ void st_pred(unsigned long long* st, bool pred, int it_slot, int ln_slot) {
    unsigned long long m = __ballot(pred);
    if (m && first_active_lane()) {
        atomicAdd(&st[it_slot], 1ull);
        atomicAdd(&st[ln_slot], (unsigned long long)__popcll(m));
    }
}

// The leaf census (stats twin with P.census): one record per wave leaf round -- when it started,
// how long it took, which wave, how many lanes were walking, and per prim type how many lanes
// hold a slot-0 / slot-1 test -- so tools/leaf_census.py can count what a workgroup-wide queue
// per prim type could have pooled.  Called by the lanes at a leaf (the first one writes).
__device__ __forceinline__ void census_leaf(const KP& P, int gwave, uint32_t types, unsigned long long t0,
                                            unsigned long long t1, int walking, unsigned long long* st) {
    const uint32_t a = types & 7u, b = (types >> 4) & 0xFu;
    uint32_t s0 = 0, s1 = 0;
#pragma unroll
    for (int k = 1; k <= 4; k++) {
        s0 |= (uint32_t)__popcll(__ballot(a == (uint32_t)k)) << (8 * (k - 1));
        s1 |= (uint32_t)__popcll(__ballot(b == (uint32_t)k)) << (8 * (k - 1));
    }
    if (first_active_lane()) {
        const unsigned long long i = atomicAdd(&st[ST_CEN_N], 1ull);
        if (gwave < P.census_waves && i < (unsigned long long)P.census_cap) {
            unsigned* r = P.census + P.census_waves + ((size_t)gwave * P.census_cap + i) * RT_CENSUS_WORDS;
            r[0] = (unsigned)t0;
            r[1] = (unsigned)(t1 - t0);
            r[2] = (unsigned)blockIdx.x | ((unsigned)(threadIdx.x >> 6) << 16) | ((unsigned)walking << 24);
            r[3] = s0;
            r[4] = s1;
        }
    }
}

__device__ __forceinline__ void st_small(unsigned long long* st, bool pred, int slot) {
    const int n = __popcll(__ballot(pred));
    if (n > 0 && n <= 8 && first_active_lane()) atomicAdd(&st[slot], 1ull);
}

// ------------------------------------------------------------------ rand()
// random.glsl:2-7; `rf` is the invocation's running rand_factor.
__device__ __forceinline__ float rnd(float& rf, float px, float py) {
    rf += 0.001f;
    v2 co;
    co.x = px + rf;
    co.y = py + rf;
    v2 k = {12.9898f, 78.233f};
    return g_fract(g_sin(g_dot2(co, k)) * 43758.5453123f);
}

// Source of hit_record.uv (compute.glsl:62): the last successful sphere or quad
// hit of the sample (it persists across bounces; media do not write it).
struct UvSrc {
    int kind_idx;   // kind in bits 16.. (0 none, 1 sphere, 2 quad), sphere index in bits 0..15
    float a, b, c;  // sphere: hit point p; quad: (alpha, beta)
};

// Closest hit of one walk.
struct Hit {
    float t;
    int tif;            // prim type | box face << 4 | prim index << 16 (one register)
    int uv_kind_idx;    // uv written during this walk (kind 0 = none)
    float uv_a, uv_b;   // sphere: t of that hit; quad: (alpha, beta)
};

// ------------------------------------------------------- shared-reciprocal division
// The compiler's f32 division num / den is: v_div_scale of den and of num, v_rcp,
// two refinement fmas (the reciprocal r), q0 = num * r, e2 = num - den * q0,
// q1 = q0 + e2 * r, e3 = num - den * q1, v_div_fmas (q1 + e3 * r), v_div_fixup.
// v_div_scale returns its operand unchanged (and v_div_fmas is that plain fma)
// unless num or den is zero or denormal, 1/den or num/den would be denormal, or
// the exponents are 96 or more apart; v_div_fixup returns q itself unless an
// input is zero, inf or NaN or the quotient over/underflows.  Outside those
// cases rcp_nr + div_nr below are the same operations, so the same bits, and r
// depends on den alone: quotients with one denominator share it (3 + 5 VALU
// instead of 11 each).  Callers use them only where every quotient they keep is
// in that regime (below); tests/test_gpu_parity.py compares both forms bit for bit.
__device__ __forceinline__ float rcp_nr(float den) {
    const float r0 = __builtin_amdgcn_rcpf(den);
    return fmaf(fmaf(-den, r0, 1.0f), r0, r0);
}
__device__ __forceinline__ float div_nr(float num, float den, float r) {
    const float q0 = num * r;
    const float q1 = fmaf(fmaf(-den, q0, num), r, q0);
    return fmaf(fmaf(-den, q1, num), r, q1);
}
// Where the leaf tests use them (FD kernels, P.fastdiv: the camera and every record
// within 2^20, faces' delta in [2^-60, 2^20]), every kept quotient is in that
// regime: a box or quad plane divides by a denominator of at least 1e-8 (smaller
// ones skip the face) and at most the scene's size, and a numerator so small that
// the quotient would be below tmin = 0.001 is rejected either way; a sphere root
// divides by dot(dir, dir), checked >= 2^-60 per wave (else '/'), which bounds the
// exponent gap by ~52; alpha and beta fall back to '/' for a numerator below
// 2^-100 (a tiny alpha >= 0 is kept).
// ------------------------------------------------------------- primitives
// hitting.glsl:17-38 — the root only.  fd: the roots as div_nr with ra =
// rcp_nr(a), unless a lane's a = dot(dir, dir) is below 2^-60.
__device__ __forceinline__ bool sphere_t_ab(float4 A, float4 B, float time, v3 o, v3 d, float a, float tmin,
                                            float tmax, float& t, bool fd = false, float ra = 0.0f) {
    v3 center = add3(f3(A), scale3(f3(B), time));
    v3 oc = sub3(o, center);
    float half_b = g_dot(oc, d);
    float c = g_dot(oc, oc) - B.w * B.w;
    float disc = half_b * half_b - a * c;
    if (disc < 0.0f) return false;
    float sq = sqrtf(disc);
    fd = fd && __ballot(!(a >= 0x1p-60f)) == 0;
    float root = fd ? div_nr(-half_b - sq, a, ra) : (-half_b - sq) / a;
    if (!(tmin < root && root < tmax)) {
        root = fd ? div_nr(-half_b + sq, a, ra) : (-half_b + sq) / a;
        if (!(tmin < root && root < tmax)) return false;
    }
    t = root;
    return true;
}
// sphere_t_ab's quadratic with both roots, (-b - sq) / a and (-b + sq) / a, whatever ray_t is
// (false when the discriminant is negative); the division form as sphere_t_ab chooses it.
__device__ __forceinline__ bool sphere_roots(float4 A, float4 B, float time, v3 o, v3 d, float a, float& lo, float& hi,
                                             bool fd) {
    v3 center = add3(f3(A), scale3(f3(B), time));
    v3 oc = sub3(o, center);
    float half_b = g_dot(oc, d);
    float c = g_dot(oc, oc) - B.w * B.w;
    float disc = half_b * half_b - a * c;
    if (disc < 0.0f) return false;
    float sq = sqrtf(disc);
    fd = fd && __ballot(!(a >= 0x1p-60f)) == 0;
    const float ra = fd ? rcp_nr(a) : 0.0f;
    lo = fd ? div_nr(-half_b - sq, a, ra) : (-half_b - sq) / a;
    hi = fd ? div_nr(-half_b + sq, a, ra) : (-half_b + sq) / a;
    return true;
}
__device__ __forceinline__ bool sphere_t(const float4* __restrict__ sp, float time, v3 o, v3 d, float a, float tmin,
                                         float tmax, float& t, bool fd = false, float ra = 0.0f) {
    return sphere_t_ab(ldg(sp), ldg(sp + 1), time, o, d, a, tmin, tmax, t, fd, ra);
}

// hitting.glsl:103-124 on an intersection-only face record (rt_device.h):
// A = (q_a, q_b, u_a, u_b), B = (v_a, v_b, delta, axis case).  The host chose
// the reference's first non-degenerate projection (xy, xz, else yz) and
// computed delta with the reference's expression, so alpha/beta here are the
// reference's values: intersection = o + dir*t, ph = intersection - q, then the
// 2-D Cramer quotients on the chosen pair of axes.
// fd: alpha and beta share delta's reciprocal (delta within [2^-60, 2^20], host
// check) unless a lane's numerator is below 2^-100 in magnitude (or zero), the
// one case where a kept value (0 <= alpha <= 1) could leave the regime.
__device__ __forceinline__ bool face_interior(float4 A, float4 B, v3 o, v3 d, float t, float& alpha, float& beta,
                                              bool fd = false) {
    const int cs = __float_as_int(B.w);
    float oa = (cs == 2) ? o.y : o.x, da = (cs == 2) ? d.y : d.x;
    float ob = (cs == 0) ? o.y : o.z, db = (cs == 0) ? d.y : d.z;
    float pa = (oa + da * t) - A.x;
    float pb = (ob + db * t) - A.y;
    const float na = pa * B.y - pb * B.x, nb = pb * A.z - pa * A.w;
    if (fd && __ballot(!(fabsf(na) >= 0x1p-100f && fabsf(nb) >= 0x1p-100f)) == 0) {
        const float r = rcp_nr(B.z);
        alpha = div_nr(na, B.z, r);
        beta = div_nr(nb, B.z, r);
    } else {
        alpha = na / B.z;
        beta = nb / B.z;
    }
    return (0.0f <= alpha && alpha <= 1.0f) && (0.0f <= beta && beta <= 1.0f);
}

// hitting.glsl:90-133 without the record writes; f = dquads record.
// Q0, Q1 = the record's first two float4 (loaded by the caller).
__device__ __forceinline__ bool quad_test_ab(const float4* __restrict__ f, float4 Q0, float4 Q1, v3 o, v3 d,
                                             float tmin, float tmax, float& t, float& alpha, float& beta,
                                             bool fd = false, bool uniform = false) {
    const float4 Q2 = uniform ? ldc(f + 2) : ldg(f + 2);
    v3 n = f3(Q0);
    float denom = g_dot(n, d);
    if (fabsf(denom) < 1e-8f) return false;
    const float num = Q0.w - g_dot(n, o);
    float tt = fd ? div_nr(num, denom, rcp_nr(denom)) : num / denom;
    if (!(tmin <= tt && tt <= tmax)) return false;
    if (!face_interior(Q1, Q2, o, d, tt, alpha, beta, fd)) return false;
    t = tt;
    return true;
}
__device__ __forceinline__ bool quad_test(const float4* __restrict__ f, v3 o, v3 d, float tmin, float tmax, float& t,
                                          float& alpha, float& beta, bool fd = false) {
    return quad_test_ab(f, ldg(f), ldg(f + 1), o, d, tmin, tmax, t, alpha, beta, fd);
}

// hitting.glsl:135-146; fb = dboxes record.  The six faces' plane parameters
// t_i do not depend on the shrinking ray_t.max, so they are divided
// independently (ILP); faces are then accepted in the reference order with the
// reference's sequential test tmin <= t_i <= current max, and only those reach
// the interior test — the same tests on the same values, so the same result.
__device__ __forceinline__ bool box_test(const float4* __restrict__ fb, v3 o, v3 d, float tmin, float tmax, float& t,
                                         int& face, float& alpha, float& beta, bool fd = false) {
    bool has = false;
    // two halves of three faces: fewer live registers than six at once
#pragma unroll
    for (int h = 0; h < 6; h += 3) {
        float ti[3];
        unsigned cand = 0;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            float4 pl = ldg(fb + h + k);
            v3 n = f3(pl);
            float denom = g_dot(n, d);
            ti[k] = (pl.w - g_dot(n, o)) / denom;   // unused when |denom| < 1e-8
            if (!(fabsf(denom) < 1e-8f) && (tmin <= ti[k] && ti[k] <= tmax)) cand |= 1u << k;
        }
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const int i = h + k;
            if ((cand >> k) & 1u) {
                float al, be;
                if (ti[k] <= tmax && face_interior(ldg(fb + 6 + 2 * i), ldg(fb + 7 + 2 * i), o, d, ti[k], al, be, fd)) {
                    tmax = ti[k];
                    t = ti[k];
                    face = i;
                    alpha = al;
                    beta = be;
                    has = true;
                }
            }
        }
    }
    return has;
}

// The canonical box test from a compact record (RT_BOXC_F4 float4, rt_capi.hip compact_box):
// c0 = (mn.x, mn.y, mn.z, mx.x), c1 = (mx.y, mx.z, s_z, s_x), c2 = (s_y, ok, 0, 0) -- the box's
// corners (Box.java:19-37 builds its six faces from them) and its faces' normal components.
// Everything the face tests read is rebuilt with the builder's own float operations:
// the edges DX = mx.x - mn.x (Box.java's dx, dy, dz), the planes (s_i, s_i * q_k) with the
// opposite faces' normals negated, and each face's 2-D system (A, B) on the reference's axis
// pair with its delta.  The host rebuilds the same values with the same operations and keeps
// a box's record (ok = 1) only when they equal the uploaded faces' records (float equality:
// a zero's sign is the only freedom, and it cannot reach a result: it only makes a zero
// plane numerator, alpha or beta a zero of the other sign, which every test and the uv's
// texture lookup treat alike).  So the test reads 48 B of LDS instead of 80 B of LDS plus up
// to 192 B of face systems from global memory.
template <int I>
__device__ __forceinline__ void boxc_face(float mnx, float mny, float mnz, float mxx, float mxz, float DX, float DY,
                                          float DZ, float4& A, float4& B) {
    // faces of Box.java:32-37: q, u, v of side I (face_record's axis pair and delta expression)
    if (I == 0) { A = make_float4(mnx, mny, DX, 0.0f); B = make_float4(0.0f, DY, DX * DY, __int_as_float(0)); }
    if (I == 1) { A = make_float4(mny, mxz, 0.0f, -DZ); B = make_float4(DY, 0.0f, DZ * DY, __int_as_float(2)); }
    if (I == 2) { A = make_float4(mxx, mny, -DX, 0.0f); B = make_float4(0.0f, DY, -(DX * DY), __int_as_float(0)); }
    if (I == 3) { A = make_float4(mny, mnz, 0.0f, DZ); B = make_float4(DY, 0.0f, -(DZ * DY), __int_as_float(2)); }
    if (I == 4) { A = make_float4(mnx, mxz, DX, 0.0f); B = make_float4(0.0f, -DZ, -(DX * DZ), __int_as_float(1)); }
    if (I == 5) { A = make_float4(mnx, mnz, DX, 0.0f); B = make_float4(0.0f, DZ, DX * DZ, __int_as_float(1)); }
}
__device__ __forceinline__ bool box_test_compact(float4 c0, float4 c1, float4 c2, v3 o, v3 d, float tmin, float tmax,
                                                 float& t, int& face, float& alpha, float& beta, bool fd = false) {
    const float mnx = c0.x, mny = c0.y, mnz = c0.z, mxx = c0.w, mxy = c1.x, mxz = c1.y;
    const float sz = c1.z, sx = c1.w, sy = c2.x;
    // faces in the reference's order (hitting.glsl:135-146): each face's plane t, then its
    // interior test when tmin <= t <= the current ray_t.max (fd: rcp_nr / div_nr per face;
    // sharing one reciprocal per axis kept it live across the next faces' tests: more spills)
    bool has = false;
#define RT_BOXC_FACE(I, S, Q, DK, OK)                                                           \
    {                                                                                                      \
        const float s_ = (S), den = s_ * (DK);                                                             \
        float ti;                                                                                          \
        if (fd) {                                                                                          \
            ti = div_nr(s_ * (Q) - s_ * (OK), den, rcp_nr(den));                                           \
        } else {                                                                                           \
            ti = (s_ * (Q) - s_ * (OK)) / den;                                                             \
        }                                                                                                  \
        if (!(fabsf(den) < 1e-8f) && (tmin <= ti && ti <= tmax)) {                                         \
            float4 A, B;                                                                                   \
            boxc_face<I>(mnx, mny, mnz, mxx, mxz, mxx - mnx, mxy - mny, mxz - mnz, A, B);                  \
            float al, be;                                                                                  \
            if (face_interior(A, B, o, d, ti, al, be, fd)) {                                               \
                tmax = ti;                                                                                 \
                t = ti;                                                                                    \
                face = I;                                                                                  \
                alpha = al;                                                                                \
                beta = be;                                                                                 \
                has = true;                                                                                \
            }                                                                                              \
        }                                                                                                  \
    }
    RT_BOXC_FACE(0, sz, mxz, d.z, o.z)
    RT_BOXC_FACE(1, sx, mxx, d.x, o.x)
    RT_BOXC_FACE(2, -sz, mnz, d.z, o.z)
    RT_BOXC_FACE(3, -sx, mnx, d.x, o.x)
    RT_BOXC_FACE(4, sy, mxy, d.y, o.y)
    RT_BOXC_FACE(5, -sy, mny, d.y, o.y)
#undef RT_BOXC_FACE
    return has;
}

// hitting.glsl:148-160 for a medium boundary (only rec.t is read, :165-178).
// Out of line: only quad/box boundaries (scene 7) come here.
__device__ __noinline__ bool boundary_t(const KP& P, int idx, int type, v3 o, v3 d, float a, float time, float tmin,
                                           float tmax, float& t) {
    float al, be;
    int face;
    if (type == RT_MODEL_SPHERE)
        return sphere_t(reinterpret_cast<const float4*>(P.spheres + idx), time, o, d, a, tmin, tmax, t);
    if (type == RT_MODEL_QUAD) return quad_test(P.dquads + RT_DFACE_F4 * idx, o, d, tmin, tmax, t, al, be);
    if (type == RT_MODEL_BOX) return box_test(P.dboxes + RT_DBOX_F4 * idx, o, d, tmin, tmax, t, face, al, be);
    return false;
}

// hitting.glsl:165-168 for a sphere boundary (A, B = the sphere's first two float4).
// Both boundary hit_sphere calls (:165, :168) see the same ray and sphere: the
// quadratic and both roots are computed once, then each call's root selection
// is applied to its own interval.
// fd: the two roots share rcp_nr(a) (the sphere roots' regime, sphere_t_ab: the wave falls back
// to '/' when a lane's a = dot(dir, dir) is below 2^-60).
__device__ __forceinline__ bool sphere_bounds(float4 A, float4 B, v3 o, v3 d, float a, float time, float& t1,
                                              float& t2, bool fd = false) {
    {
        v3 center = add3(f3(A), scale3(f3(B), time));
        v3 oc = sub3(o, center);
        float half_b = g_dot(oc, d);
        float c = g_dot(oc, oc) - B.w * B.w;
        float disc = half_b * half_b - a * c;
        // without branches: disc < 0 makes sq and both roots NaN, and every test below fails
        // as the early return did (t1 / t2 are not read on false).  All lanes take the ballot
        // now; it only chooses between div_nr and '/', which give the same bits in its regime.
        float sq = sqrtf(disc);
        fd = fd && __ballot(!(a >= 0x1p-60f)) == 0;
        const float ra = fd ? rcp_nr(a) : 0.0f;
        float r_lo = fd ? div_nr(-half_b - sq, a, ra) : (-half_b - sq) / a;
        float r_hi = fd ? div_nr(-half_b + sq, a, ra) : (-half_b + sq) / a;
        const bool lo_in = -RT_INFINITY < r_lo && r_lo < RT_INFINITY;
        const bool hi_in = -RT_INFINITY < r_hi && r_hi < RT_INFINITY;
        t1 = lo_in ? r_lo : r_hi;
        const float lo2 = t1 + 0.0001f;
        const bool lo_2 = lo2 < r_lo && r_lo < RT_INFINITY;
        const bool hi_2 = lo2 < r_hi && r_hi < RT_INFINITY;
        t2 = lo_2 ? r_lo : r_hi;
        return !(disc < 0.0f) && (lo_in || hi_in) && (lo_2 || hi_2);
    }
}

// hitting.glsl:165-168 — the medium's two boundary hits (no rand() yet).
__device__ __forceinline__ bool medium_bounds(const KP& P, const rt_medium& m, v3 o, v3 d, float a, float time,
                                              float& t1, float& t2) {
    if (m.boundary_type == RT_MODEL_SPHERE) {
        const float4* sp = reinterpret_cast<const float4*>(P.spheres + m.boundary_idx);
        return sphere_bounds(sp[0], sp[1], o, d, a, time, t1, t2);
    }
    if (!boundary_t(P, m.boundary_idx, m.boundary_type, o, d, a, time, -RT_INFINITY, RT_INFINITY, t1)) return false;
    return boundary_t(P, m.boundary_idx, m.boundary_type, o, d, a, time, t1 + 0.0001f, RT_INFINITY, t2);
}

// hitting.glsl:169-192 — clamp to ray_t, draw the distance; returns the hit t.
__device__ __forceinline__ bool medium_tail(float neg_inv_density, float t1, float t2, float a, float tmin, float tmax,
                                            float& rf, float px, float py, float& t) {
    if (t1 < tmin) t1 = tmin;
    if (t2 > tmax) t2 = tmax;
    if (t1 >= t2) return false;
    if (t1 < 0.0f) t1 = 0.0f;
    float len = sqrtf(a);   // length(ray.dir); a == dot(dir, dir)
    float inside = (t2 - t1) * len;
    float hd = neg_inv_density * g_log(rnd(rf, px, py));
    if (hd > inside) return false;
    t = t1 + hd / len;
    return true;
}

// medium_test on the medium's LDS record already loaded (R0 = boundary idx, type, -1/density, phase;
// R1, R2 = its sphere boundary's A, B when the boundary is a sphere): the same operations.
template <bool FD = false, bool MSPH = false>
__device__ __forceinline__ bool medium_test_rec(const KP& P, float4 R0, float4 R1, float4 R2, v3 o, v3 d, float a,
                                                float time, float tmin, float tmax, float& rf, float px, float py,
                                                float& t) {
    float t1, t2;
    rt_medium m;
    m.boundary_idx = __float_as_int(R0.x);
    m.boundary_type = __float_as_int(R0.y);
    m.neg_inv_density = R0.z;
    m.phase_material = __float_as_int(R0.w);
    m.texture_id = 0;
    if (MSPH || m.boundary_type == RT_MODEL_SPHERE) {   // MSPH: every medium's boundary is a sphere
        if (!sphere_bounds(R1, R2, o, d, a, time, t1, t2, FD)) return false;
    } else if (!medium_bounds(P, m, o, d, a, time, t1, t2)) {
        return false;
    }
    return medium_tail(m.neg_inv_density, t1, t2, a, tmin, tmax, rf, px, py, t);
}

// hitting.glsl:162-193 — returns the hit distance t.
template <bool FD = false, bool STD = false>
__device__ __forceinline__ bool medium_test(const KP& P, int idx, v3 o, v3 d, float a, float time, float tmin,
                                            float tmax, float& rf, float px, float py, float& t) {
    float t1, t2;
    rt_medium m;
    if (STD || P.media_lds >= 0) {   // the record and its sphere boundary from LDS (render_persistent)
        const float4* r = rt_dyn_lds + P.media_lds + 3 * idx;
        const float4 R0 = r[0];
        m.boundary_idx = __float_as_int(R0.x);
        m.boundary_type = __float_as_int(R0.y);
        m.neg_inv_density = R0.z;
        m.phase_material = __float_as_int(R0.w);
        m.texture_id = 0;
        if (STD || m.boundary_type == RT_MODEL_SPHERE) {
            if (!sphere_bounds(r[1], r[2], o, d, a, time, t1, t2, FD)) return false;
        } else if (!medium_bounds(P, m, o, d, a, time, t1, t2)) {
            return false;
        }
    } else {
        m = P.media[idx];
        if (!medium_bounds(P, m, o, d, a, time, t1, t2)) return false;
    }
    return medium_tail(m.neg_inv_density, t1, t2, a, tmin, tmax, rf, px, py, t);
}

// hitting.glsl:55-76 for one axis (branch-free; the same assignments)
__device__ __forceinline__ void slab(float mn, float mx, float o, float inv, float& lo, float& hi) {
    float t0 = (mn - o) * inv;
    float t1 = (mx - o) * inv;
    bool ord = t0 < t1;
    float a = ord ? t0 : t1;
    float b = ord ? t1 : t0;
    lo = (a > lo) ? a : lo;
    hi = (b < hi) ? b : hi;
}

// hit_aabb (hitting.glsl:55-76) with NaN-ignoring min/max: the reference's
// per-axis swap + conditional updates are lo = max({tmin} U near_i), hi =
// min({tmax} U far_i) over the non-NaN candidates, and v_min/v_max (IEEE
// minNum/maxNum) ignore a NaN operand.  A slab value is NaN only when
// inv = +-inf (dir component +-0 or denormal-small) and the origin lies on the
// slab plane; with inv = +inf the reference's asymmetric NaN handling still
// equals min/max, with inv = -inf it does not, so rays with an inv component
// of -inf take the exact path (slab()).  Signed zeros differ only where
// hi <= lo holds either way (lo >= tmin = 0.001 > 0).
// The instructions themselves: the compiler wraps fminf/fmaxf operands in
// canonicalizing moves (sNaN quieting), which our operands never need (their
// only NaNs are quiet 0*inf products).
__device__ __forceinline__ float v_min(float a, float b) {
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float v_max(float a, float b) {
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float v_min3(float a, float b, float c) {
    float r;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float v_max3(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ bool aabb_fast(float4 n0, float4 n1, v3 o, v3 inv, float tmin, float tmax) {
    float t0x = (n0.x - o.x) * inv.x, t1x = (n0.y - o.x) * inv.x;
    float t0y = (n0.z - o.y) * inv.y, t1y = (n0.w - o.y) * inv.y;
    float t0z = (n1.x - o.z) * inv.z, t1z = (n1.y - o.z) * inv.z;
    float lo = v_max(v_max3(tmin, v_min(t0x, t1x), v_min(t0y, t1y)), v_min(t0z, t1z));
    float hi = v_min(v_min3(tmax, v_max(t0x, t1x), v_max(t0y, t1y)), v_max(t0z, t1z));
    return !(hi <= lo);
}

// aabb_fast with the six slab subtractions and products as packed pairs
// (v_pk_add_f32 / v_pk_mul_f32: the same IEEE roundings, half the issue).
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ bool aabb_pk(float4 n0, float4 n1, v3 o, v3 inv, float tmin, float tmax) {
    const f2v tx = (f2v{n0.x, n0.y} - f2v{o.x, o.x}) * f2v{inv.x, inv.x};
    const f2v ty = (f2v{n0.z, n0.w} - f2v{o.y, o.y}) * f2v{inv.y, inv.y};
    const f2v tz = (f2v{n1.x, n1.y} - f2v{o.z, o.z}) * f2v{inv.z, inv.z};
    float lo = v_max(v_max3(tmin, v_min(tx.x, tx.y), v_min(ty.x, ty.y)), v_min(tz.x, tz.y));
    float hi = v_min(v_min3(tmax, v_max(tx.x, tx.y), v_max(ty.x, ty.y)), v_max(tz.x, tz.y));
    return !(hi <= lo);
}

// The two prims of a leaf (compute.glsl:247-256), left then right.
// FD: the shared-reciprocal divisions (rcp_nr / div_nr; FD kernels only).
template <bool STATS, bool FD, bool BOXC = false, bool SPAIR = false, bool STD = false>
__device__ __forceinline__ void leaf_prims_t(const KP& P, uint32_t meta, uint32_t prims, v3 o, v3 d, v3 inv, float a,
                                             float time, float tmin, float& tmax, float& rf, float px, float py, Hit& h,
                                             bool& has, unsigned long long* st) {
    constexpr bool fd = FD;
    // A leaf of two spheres (the sphere cluster's leaves; a singleton sphere leaf tests its sphere
    // twice, Q7): both quadratics and all four roots at once, then the reference's selection of
    // each sphere in turn (hitting.glsl:28-34) under the ray_t.max the first one leaves.  A root
    // does not depend on ray_t, so this is sphere_t_ab twice in order: the same values, the same
    // hits, the two records' loads and dependent chains overlapped.
    // Only in the SPAIR kernels (scenes whose leaves are mostly sphere pairs, rt_capi.hip): where
    // most lanes hold other leaves, the extra block costs more than it saves (scene 8 +1%, and
    // the code alone scene 6 +1.3%); scene 0 -6.1%.
    if (SPAIR && !STATS && (STD || P.sph_lds >= 0) && ((meta >> 16) & 0xFFu) == (RT_MODEL_SPHERE | (RT_MODEL_SPHERE << 4))) {
        const int i0 = (int)(prims & 0xFFFFu), i1 = (int)(prims >> 16);
        const float4* r0 = rt_dyn_lds + P.sph_lds + 2 * i0;
        const float4* r1 = rt_dyn_lds + P.sph_lds + 2 * i1;
        const float4 A0 = r0[0], B0 = r0[1], A1 = r1[0], B1 = r1[1];
        float lo0, hi0, lo1, hi1;
        const bool ok0 = sphere_roots(A0, B0, time, o, d, a, lo0, hi0, fd);
        const bool ok1 = sphere_roots(A1, B1, time, o, d, a, lo1, hi1, fd);
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const bool ok = k ? ok1 : ok0;
            const int ix = k ? i1 : i0;
            float root = k ? lo1 : lo0;
            bool hit = ok && tmin < root && root < tmax;
            if (ok && !hit) {
                root = k ? hi1 : hi0;
                hit = tmin < root && root < tmax;
            }
            if (hit) {
                h.uv_kind_idx = (1 << 16) | ix;
                h.uv_a = root;
                has = true;
                tmax = root;
                h.t = root;
                h.tif = RT_MODEL_SPHERE | (ix << 16);
            }
        }
        return;
    }
    // finite origin and direction: the canonical box planes equal the reference's dot products
    const bool fin = fabsf(o.x) < INFINITY && fabsf(o.y) < INFINITY && fabsf(o.z) < INFINITY &&
                     fabsf(d.x) < INFINITY && fabsf(d.y) < INFINITY && fabsf(d.z) < INFINITY;
    // both slots unrolled (the second slot's record loads can start during the first's tests):
    // scenes 8 / 0 / 6 -0.4 / -1.2 / -1.1%, no spills at 125 VGPRs (profiles/r03_leaf_unroll_lib_ab.log)
#pragma unroll
    for (int s = 0; s < 2; s++) {
        int ty = (int)((meta >> (16 + 4 * s)) & 0xFu);
        int ix = (int)((prims >> (16 * s)) & 0xFFFFu);
        // a box whose bounds pre-test already ran as a node of the walk (P.box_vnodes, rt_capi.hip
        // build_links; its leaf record's RT_LINK_PRETESTED bit): the same test, not repeated
        bool pretested = false;
        if (s == 0 && BOXC) {
            pretested = (ty & RT_LINK_PRETESTED) != 0;
            ty &= 7;
        }
        // the second slot is empty in every lane of the wave (singleton leaves, the pre-tested boxes'
        // records): nothing to test, its record loads skipped (wave-uniform)
        if (BOXC && s == 1 && __ballot(ty != 0) == 0) break;
        if (STATS) {
            st_pred(st, ty == RT_MODEL_SPHERE, ST_SPH_IT, ST_SPH_LN);
            st_pred(st, ty == RT_MODEL_QUAD, ST_QUAD_IT, ST_QUAD_LN);
            st_pred(st, ty == RT_MODEL_BOX, ST_BOX_IT, ST_BOX_LN);
            st_pred(st, ty == RT_MODEL_CONSTANT_MEDIUM, ST_MED_IT, ST_MED_LN);
            st_small(st, ty == RT_MODEL_SPHERE, ST_SPH_SM);
            st_small(st, ty == RT_MODEL_QUAD, ST_QUAD_SM);
            st_small(st, ty == RT_MODEL_BOX, ST_BOX_SM);
            st_small(st, ty == RT_MODEL_CONSTANT_MEDIUM, ST_MED_SM);
        }
        float t = 0.0f, al = 0.0f, be = 0.0f;
        int face = 0;
        bool hit = false;
        // Record prefetch (BOXC kernels whose sphere, box and medium records are all in LDS,
        // P.leaf_pf): the slot's record -- a sphere's (A, B), a box's compact record, a medium's
        // record and sphere boundary, each 3 float4 from its table's offset -- is loaded once for
        // every lane before the type blocks, so the blocks do not each wait on their own LDS
        // round trip.  (A sphere's third float4 is its successor's A, or the next table's first:
        // in LDS, unused.)  The same values reach the same tests.
        // STD kernels (RT_OPT_STD): known on, the other forms compiled out
        const bool pf = BOXC && (STD || P.leaf_pf);   // wave-uniform
        float4 q0, q1, q2;
        if (pf) {
            const int off = ty == RT_MODEL_SPHERE ? P.sph_lds + 2 * ix
                          : ty == RT_MODEL_BOX ? P.box_cmp_lds + RT_BOXC_F4 * ix
                          : ty == RT_MODEL_CONSTANT_MEDIUM ? P.media_lds + 3 * ix : 0;
            const float4* r = rt_dyn_lds + off;
            q0 = r[0];
            q1 = r[1];
            q2 = r[2];
        }
        unsigned long long c0 = STATS ? clock64() : 0;
        if (ty == RT_MODEL_SPHERE) {
            if (pf) {
                hit = sphere_t_ab(q0, q1, time, o, d, a, tmin, tmax, t, fd, fd ? rcp_nr(a) : 0.0f);
            } else if (STD || P.sph_lds >= 0) {   // the record's intersection half from LDS (render_persistent)
                const float4* r = rt_dyn_lds + P.sph_lds + 2 * ix;
                hit = sphere_t_ab(r[0], r[1], time, o, d, a, tmin, tmax, t, fd, fd ? rcp_nr(a) : 0.0f);
            } else {
                hit = sphere_t(reinterpret_cast<const float4*>(P.spheres + ix), time, o, d, a, tmin, tmax, t, fd,
                               fd ? rcp_nr(a) : 0.0f);
            }
            if (hit) { h.uv_kind_idx = (1 << 16) | ix; h.uv_a = t; }
            if (STATS) st_add(st, ST_SPH_CYC, clock64() - c0);
        } else if (ty == RT_MODEL_QUAD) {
            hit = quad_test(P.dquads + RT_DFACE_F4 * ix, o, d, tmin, tmax, t, al, be, fd);
            if (hit) { h.uv_kind_idx = 2 << 16; h.uv_a = al; h.uv_b = be; }
            if (STATS) st_add(st, ST_QUAD_CYC, clock64() - c0);
        } else if (ty == RT_MODEL_BOX) {
            // the box's 48-byte record (rt_capi.hip compact_box), from LDS when staged: its bounds
            // for the pre-test, and -- every box of the scene having Box.java's axis-aligned
            // layout (BOXC) -- everything its faces' tests read (box_test_compact); otherwise the
            // faces' full records (box_test).  A canonical face is never hit by a ray with a
            // non-finite origin or direction, in the reference's form or the compact one (its
            // plane t or its alpha / beta is then inf or NaN), so BOXC needs no finiteness check.
            float4 r0, r1, r2;
            if (pf) {
                r0 = q0;
                r1 = q1;
                r2 = q2;
            } else if (STD || P.box_cmp_lds >= 0) {
                const float4* cr = rt_dyn_lds + P.box_cmp_lds + RT_BOXC_F4 * ix;
                r0 = cr[0];
                r1 = cr[1];
                r2 = cr[2];
            } else {
                const float4* cr = P.dboxc + RT_BOXC_F4 * ix;
                r0 = ldg(cr);
                r1 = ldg(cr + 1);
                r2 = ldg(cr + 2);
            }
            bool maybe = true;
            if (P.box_margin > 0.0f && (BOXC || fin) && !pretested) {
                // the box's bounds grown by box_margin (rt_device.h): a ray that misses them
                // misses every face the exact test below would accept
                const float m = P.box_margin;
                maybe = aabb_pk(make_float4(r0.x - m, r0.w + m, r0.y - m, r1.x + m),
                                make_float4(r0.z - m, r1.y + m, 0.0f, 0.0f), o, inv, tmin, tmax);
            }
            if (maybe) {
                if constexpr (BOXC)
                    hit = box_test_compact(r0, r1, r2, o, d, tmin, tmax, t, face, al, be, fd);
                else
                    hit = box_test(P.dboxes + RT_DBOX_F4 * ix, o, d, tmin, tmax, t, face, al, be, fd);
            }
            if (hit) { h.uv_kind_idx = 2 << 16; h.uv_a = al; h.uv_b = be; }
            if (STATS) st_add(st, ST_BOX_CYC, clock64() - c0);
        } else if (ty == RT_MODEL_CONSTANT_MEDIUM) {
            hit = pf ? medium_test_rec<FD, STD>(P, q0, q1, q2, o, d, a, time, tmin, tmax, rf, px, py, t)
                     : medium_test<FD, STD>(P, ix, o, d, a, time, tmin, tmax, rf, px, py, t);
            if (STATS) st_add(st, ST_MED_CYC, clock64() - c0);
        }
        if (hit) {
            has = true;
            tmax = t;
            h.t = t; h.tif = ty | (face << 4) | (ix << 16);
        }
    }
}


// The link-format node loop from byte offset nx until a hit leaf or the end of
// the walk (sign bit).  EXACT: the reference's per-axis slab (a -inf in 1/dir);
// otherwise the NaN-ignoring min/max form.  The choice is wave-uniform and made
// once per walk, outside the loop (3.6 % faster on scene 8 than testing it per
// node step).  Reading both successors while the node is tested (to hide the
// dependent LDS read) measured 9 % slower: its extra VALU outweigh the hidden latency.
// Node reads: an LDS address is the node's byte offset plus the dynamic region's
// base, which is 0 in a kernel without static LDS (every non-stats build), so
// the offset is the address itself (no add per step).
typedef __attribute__((address_space(3))) const f4v lds_f4;
// Where the walk reads its nodes: LDS from `base` (the dynamic region) and, in the
// two-level walk (TL), global memory `gnodes` for addresses at or past `lim`.
struct NodeSrc {
    const char* base;
    const char* gnodes;
    uint32_t lim;
    unsigned* hits;   // stats twin: per link node the tests that hit (P.node_hits), else null
};
// The stats twin's node-hit count (rt_debug_count_node_hits; the collapse plan's H(N) measured on the
// walks themselves): the lanes at the wave's first lane's node add with one atomic, the others one each.
__device__ __forceinline__ void count_node_hit(unsigned* hits, uint32_t nx, bool hit) {
    const uint32_t n0 = __builtin_amdgcn_readfirstlane(nx);
    const unsigned long long hm = __ballot(hit && nx == n0);
    if (hm && first_active_lane()) atomicAdd(&hits[n0 >> 5], (unsigned)__popcll(hm));
    if (hit && nx != n0) atomicAdd(&hits[nx >> 5], 1u);
}
template <bool STATS, bool TL>
__device__ __forceinline__ void load_node(const NodeSrc& ns, uint32_t nx, float4& n0, float4& n1) {
    if (TL && nx >= ns.lim) {   // below the LDS-staged top levels: the node array in global memory
        const float4* g = reinterpret_cast<const float4*>(ns.gnodes + nx);
        n0 = ldg(g);
        n1 = ldg(g + 1);
    } else if (STATS) {   // static LDS (the stats counters) precedes the dynamic region
        n0 = *reinterpret_cast<const float4*>(ns.base + nx);
        n1 = *reinterpret_cast<const float4*>(ns.base + nx + 16);
    } else {
        const lds_f4* p = (const lds_f4*)(uintptr_t)nx;
        const f4v a = p[0], b = p[1];
        n0 = make_float4(a.x, a.y, a.z, a.w);
        n1 = make_float4(b.x, b.y, b.z, b.w);
    }
}
template <bool EXACT, bool STATS, bool TL = false>
__device__ __forceinline__ uint32_t link_walk(const NodeSrc& ns, uint32_t nx, v3 o, v3 inv, float tmin, float tmax,
                                              unsigned long long* st) {
    while ((int)nx >= 0) {
        if (STATS) st_lanes(st, ST_NODE_IT, ST_NODE_LN);
        float4 n0, n1;
        load_node<STATS, TL>(ns, nx, n0, n1);
        bool hit;
        if (!EXACT) {
            hit = aabb_pk(n0, n1, o, inv, tmin, tmax);
        } else {
            float lo = tmin, hi = tmax;
            slab(n0.x, n0.y, o.x, inv.x, lo, hi);
            slab(n0.z, n0.w, o.y, inv.y, lo, hi);
            slab(n1.x, n1.y, o.z, inv.z, lo, hi);
            hit = !(hi <= lo);
        }
        if (STATS && ns.hits) count_node_hit(ns.hits, nx, hit);
        nx = __float_as_uint(hit ? n1.z : n1.w);
    }
    return nx;
}

// link_walk for a wave's walking lanes that stops once `need` of them hold a hit
// leaf or have ended (the others keep their position nx >= 0 and go on in the
// next round): the wave does not step its last walkers alone while the lanes
// waiting at a leaf idle.  Checked every third step (every second: scene 6 +2.7%, scenes 0 / 8 +0.6..0.8%;
// round 4, under the per-BVH walk thresholds, every 2nd / 4th: scenes 6 / 7 +9..15%, 0 / 8 -0.1..+1.2%,
// profiles/r04_walk_check_interval_lib_ab.log).
// BL (the compact-box and sphere-pair STD kernels, scenes 8 and 0): every lane takes every step -- a lane that holds a leaf
// or ended reads the root and keeps its position -- so a step has no exec-mask branch (its
// s_and_saveexec / s_cbranch / exec restore): the same node sequence per walking lane.  Scene 8
// -0.4% (with the stop check every 2 steps, RT_BL_STEPS, another -0.2..-0.3%), scene 0 -0.8% (with it);
// scene 6's kernel (a 7-node tree: short walks) +1.8%, so there it stays off
// (profiles/r06_x_node_branchless_lib_ab.log, r06_ae_bl_spair_lib_ab.log; round 3: -0.5 / -0.2 / +1.7%).
// the BL walk's steps between the partial walk's stop checks: 2 (scene 8 -0.2% at 1080p, -0.3% at
// 4K against 3; 1 +1.8%, 4 +0.8%: profiles/r06_ab_bl_steps{,_4k}_lib_ab.log, r06_aa_lib_ab.log)
#ifndef RT_BL_STEPS
#define RT_BL_STEPS 2
#endif
template <bool EXACT, bool STATS, bool TL = false, bool BL = false>
__device__ __forceinline__ uint32_t link_walk_part(const NodeSrc& ns, uint32_t nx, v3 o, v3 inv, float tmin,
                                                   float tmax, int need, unsigned long long* st) {
    for (;;) {
#pragma unroll
        for (int k = 0; k < (BL ? RT_BL_STEPS : 3); k++) {
            if constexpr (BL && !STATS && !EXACT && !TL) {
                const bool w = (int)nx >= 0;
                float4 n0, n1;
                load_node<STATS, TL>(ns, w ? nx : 0u, n0, n1);
                const bool hit = aabb_pk(n0, n1, o, inv, tmin, tmax);
                const uint32_t nn = __float_as_uint(hit ? n1.z : n1.w);
                nx = w ? nn : nx;
                continue;
            }
            if ((int)nx >= 0) {
                if (STATS) {
                    st_lanes(st, ST_NODE_IT, ST_NODE_LN);
                    st_small(st, true, ST_NODE_SM);
                }
                float4 n0, n1;
                load_node<STATS, TL>(ns, nx, n0, n1);
                bool hit;
                if (!EXACT) {
                    hit = aabb_pk(n0, n1, o, inv, tmin, tmax);
                } else {
                    float lo = tmin, hi = tmax;
                    slab(n0.x, n0.y, o.x, inv.x, lo, hi);
                    slab(n0.z, n0.w, o.y, inv.y, lo, hi);
                    slab(n1.x, n1.y, o.z, inv.z, lo, hi);
                    hit = !(hi <= lo);
                }
                if (STATS && ns.hits) count_node_hit(ns.hits, nx, hit);
                nx = __float_as_uint(hit ? n1.z : n1.w);
            }
        }
        const unsigned long long walking = __ballot((int)nx >= 0);
        if (walking == 0 || __popcll(__ballot(1) & ~walking) >= need) break;
    }
    return nx;
}

// ---------------------------------------------------------------- textures
// rt_unorm8 (c / 255.0f, correctly rounded) without the division: one
// reciprocal-refinement step, q = c*r, q' = fma(fma(-q, 255, c), r, q) with
// r = RN(1/255).  Equal to c / 255.0f for every byte c (exhaustive check in
// tests/test_oracle.py::test_unorm8_refinement_is_exact).
__device__ __forceinline__ float unorm8_fast(uint32_t c) {
    const float r = 1.0f / 255.0f;
    float x = (float)c;
    float q = x * r;
    return fmaf(fmaf(-q, 255.0f, x), r, q);
}

__device__ __forceinline__ void texel(const rt_dtex& T, int x, int y, float out[3]) {
    out[0] = out[1] = out[2] = 0.0f;
    if (!T.data || x < 0 || y < 0 || x >= T.w || y >= T.h) return;
    int i = y * T.w + x;
    if (T.is_float) {
        out[0] = ((g_f*)T.data)[i];
    } else {
        uint32_t c = ((__attribute__((address_space(1))) const uint32_t*)T.data)[i];
        out[0] = unorm8_fast(c & 0xFFu);
        out[1] = unorm8_fast((c >> 8) & 0xFFu);
        out[2] = unorm8_fast((c >> 16) & 0xFFu);
    }
}
// texel() at an (x, y) the caller has clamped into the image of a texture with data, without
// branches: a float texel and an RGBA8 texel are both one 32-bit word at the same index, so one
// load serves either and the format selects the conversion
__device__ __forceinline__ void texel_in(const rt_dtex& T, int x, int y, float out[3]) {
    const uint32_t c = ((__attribute__((address_space(1))) const uint32_t*)T.data)[y * T.w + x];
    out[0] = T.is_float ? __uint_as_float(c) : unorm8_fast(c & 0xFFu);
    out[1] = T.is_float ? 0.0f : unorm8_fast((c >> 8) & 0xFFu);
    out[2] = T.is_float ? 0.0f : unorm8_fast((c >> 16) & 0xFFu);
}
// texel() of slot `slot` through the LDS shading table when it is staged (P.tex_lds: the slot's
// (w, h, is_float, texel offset); the same words as the texture), else from global memory
template <bool STD = false>
__device__ __forceinline__ void texel_slot(const KP& P, int slot, int x, int y, float out[3]) {
    if (STD || P.tex_lds >= 0) {
        const float4 dsc = rt_dyn_lds[P.tex_lds + slot];
        const int w = __float_as_int(dsc.x), h = __float_as_int(dsc.y), off = __float_as_int(dsc.w);
        if (off >= 0) {
            out[0] = out[1] = out[2] = 0.0f;
            if (x < 0 || y < 0 || x >= w || y >= h) return;
            const uint32_t c = reinterpret_cast<const uint32_t*>(rt_dyn_lds + off)[y * w + x];
            if (__float_as_int(dsc.z)) {
                out[0] = __uint_as_float(c);
            } else {
                out[0] = unorm8_fast(c & 0xFFu);
                out[1] = unorm8_fast((c >> 8) & 0xFFu);
                out[2] = unorm8_fast((c >> 16) & 0xFFu);
            }
            return;
        }
    }
    texel(P.tex[slot], x, y, out);
}
__device__ __forceinline__ float texel_r(const rt_dtex& T, int x, int y) {
    float t[3];
    texel(T, x, y, t);
    return t[0];
}

// texel_r of an R32F table: the LDS copy (ds_read) or the texture in global memory
template <bool LDS>
__device__ __forceinline__ float table_r(const float* tab, int w, int h, int x, int y) {
    if (!tab || x < 0 || y < 0 || x >= w || y >= h) return 0.0f;
    return LDS ? ((lds_f*)tab)[y * w + x] : ((g_f*)tab)[y * w + x];
}

// texture.glsl:38-77 with perlin_interp (19-36) fused; Hermite applied twice (Q6)
template <bool LDS>
__device__ __forceinline__ float perlin_noise(const float* tab, int tw, int th, v3 p) {
    float u = p.x - floorf(p.x);
    float v = p.y - floorf(p.y);
    float w = p.z - floorf(p.z);
    u = u * u * (3.0f - 2.0f * u);
    v = v * v * (3.0f - 2.0f * v);
    w = w * w * (3.0f - 2.0f * w);
    int i = rt_f2i(floorf(p.x));
    int j = rt_f2i(floorf(p.y));
    int k = rt_f2i(floorf(p.z));
    float uu = u * u * (3.0f - 2.0f * u);
    float vv = v * v * (3.0f - 2.0f * v);
    float ww = w * w * (3.0f - 2.0f * w);
    float accum = 0.0f;
#pragma unroll
    for (int di = 0; di < 2; di++) {
        int px = rt_f2i(table_r<LDS>(tab, tw, th, 3, (i + di) & 255));
#pragma unroll
        for (int dj = 0; dj < 2; dj++) {
            int py = rt_f2i(table_r<LDS>(tab, tw, th, 4, (j + dj) & 255));
#pragma unroll
            for (int dk = 0; dk < 2; dk++) {
                int pz = rt_f2i(table_r<LDS>(tab, tw, th, 5, (k + dk) & 255));
                int idx = px ^ py ^ pz;
                v3 c = mk3(table_r<LDS>(tab, tw, th, 0, idx), table_r<LDS>(tab, tw, th, 1, idx), table_r<LDS>(tab, tw, th, 2, idx));
                v3 wv = mk3(u - (float)di, v - (float)dj, w - (float)dk);
                float fi = (float)di, fj = (float)dj, fk = (float)dk;
                accum += (fi * uu + (1.0f - fi) * (1.0f - uu)) * (fj * vv + (1.0f - fj) * (1.0f - vv)) *
                         (fk * ww + (1.0f - fk) * (1.0f - ww)) * g_dot(c, wv);
            }
        }
    }
    return accum;
}

// perlin_noise on the packed table (rt_capi.hip rt_upload_texture: row r = (ranvec r, perm_x r |
// perm_y r << 8 | perm_z r << 16), the host having checked that every perm entry is a whole
// number 0..255): the same lattice corners, vectors and float operations in the same order; a
// perm value is its byte instead of int(texel), and no index can leave the table (& 255, or an
// xor of bytes), so no bounds check.  One ds_read per corner vector, one per perm entry.
__device__ __forceinline__ float perlin_noise_pk(const float4* tab, v3 p) {
    float u = p.x - floorf(p.x);
    float v = p.y - floorf(p.y);
    float w = p.z - floorf(p.z);
    u = u * u * (3.0f - 2.0f * u);
    v = v * v * (3.0f - 2.0f * v);
    w = w * w * (3.0f - 2.0f * w);
    int i = rt_f2i(floorf(p.x));
    int j = rt_f2i(floorf(p.y));
    int k = rt_f2i(floorf(p.z));
    float uu = u * u * (3.0f - 2.0f * u);
    float vv = v * v * (3.0f - 2.0f * v);
    float ww = w * w * (3.0f - 2.0f * w);
    // the reference's corner weight fi * uu + (1 - fi) * (1 - uu) (texture.glsl:30-33) for fi = 0
    // and 1: uu is a fade of a value in [0, 1], so finite and >= +0 (or NaN, which both forms
    // propagate), hence 0 * uu = +0, 1 * x = x and x + (+0) = x: the weights are exactly
    // 1 - uu and uu (likewise vv, ww)
    const lds_f* t = (const lds_f*)tab;
    float accum = 0.0f;
#pragma unroll
    for (int di = 0; di < 2; di++) {
        const uint32_t px = __float_as_uint(t[4 * ((i + di) & 255) + 3]) & 0xFFu;
#pragma unroll
        for (int dj = 0; dj < 2; dj++) {
            const uint32_t py = (__float_as_uint(t[4 * ((j + dj) & 255) + 3]) >> 8) & 0xFFu;
#pragma unroll
            for (int dk = 0; dk < 2; dk++) {
                const uint32_t pz = (__float_as_uint(t[4 * ((k + dk) & 255) + 3]) >> 16) & 0xFFu;
                const uint32_t idx = px ^ py ^ pz;
                const f4v cv = ((const lds_f4*)tab)[idx];
                v3 c = mk3(cv.x, cv.y, cv.z);
                v3 wv = mk3(u - (float)di, v - (float)dj, w - (float)dk);
                accum += (di ? uu : 1.0f - uu) * (dj ? vv : 1.0f - vv) * (dk ? ww : 1.0f - ww) * g_dot(c, wv);
            }
        }
    }
    return accum;
}

// noise_turb's seven octaves (texture.glsl:79-90) over the packed LDS table at float4 offset
// `at` (inline, or as the out-of-line perlin_turb_lds) / over the texture in global memory
// (out of line).  A call keeps the noise's registers off the walk and shading code around
// it; which form a kernel uses is measured (texture_color).
__device__ __forceinline__ float perlin_turb_lds_in(int at, float px, float py, float pz) {
    const float4* tab = rt_dyn_lds + at;
    float accum = 0.0f, weight = 1.0f;
    v3 q = mk3(px, py, pz);
#pragma unroll 1
    for (int o = 0; o < 7; o++) {
        accum += weight * perlin_noise_pk(tab, q);
        weight *= 0.5f;
        q = scale3(q, 2.0f);
    }
    return accum;
}
__device__ __noinline__ float perlin_turb_lds(int at, float px, float py, float pz) {
    return perlin_turb_lds_in(at, px, py, pz);
}
__device__ __noinline__ float perlin_turb_global(const float* tab, int tw, int th, float px, float py, float pz) {
    float accum = 0.0f, weight = 1.0f;
    v3 q = mk3(px, py, pz);
#pragma unroll 1
    for (int o = 0; o < 7; o++) {
        accum += weight * perlin_noise<false>(tab, tw, th, q);
        weight *= 0.5f;
        q = scale3(q, 2.0f);
    }
    return accum;
}

// texture.glsl:96-110
__device__ __forceinline__ v2 sphere_uv(v3 p) {
    p = g_normalize(p);
    float theta = g_acos(-p.y);
    float phi = g_atan2(-p.z, p.x) + RT_PI;
    v2 r = {phi / (2.0f * RT_PI), theta / RT_PI};
    return r;
}

template <bool STD = false>
__device__ __forceinline__ v2 resolve_uv(const KP& P, const UvSrc& s, float time) {
    int kind = s.kind_idx >> 16;
    if (kind == 2) { v2 r = {s.a, s.b}; return r; }
    if (kind == 1) {
        const int si = s.kind_idx & 0xFFFF;
        float4 A, B;
        if (STD || P.sph_mat_lds >= 0) {   // the shading tables are on: the sphere's (A, B) from LDS
            A = rt_dyn_lds[P.sph_lds + 2 * si];
            B = rt_dyn_lds[P.sph_lds + 2 * si + 1];
        } else {
            const float4* sp = reinterpret_cast<const float4*>(P.spheres + si);
            A = ldg(sp);
            B = ldg(sp + 1);
        }
        v3 center = add3(f3(A), scale3(f3(B), time));
        return sphere_uv(sub3(mk3(s.a, s.b, s.c), center));
    }
    v2 z = {0.0f, 0.0f};
    return z;
}

// texture.glsl:112-132
template <bool PK_INLINE = false, bool STD = false>
__device__ __forceinline__ v3 texture_color(const KP& P, v3 p, int id, const UvSrc& uvs, float time) {
#ifdef RT_AB_KNOBS
    if (P.debug_flags & 4) return mk3s(0.5f);   // ablation only (A/B build): every texture a constant, never exact
#endif
    int detail_i = id & 0xFFF;
    int index = (id >> 12) & 0xFFFF;
    int type = (id >> 28) & 0xF;
    const rt_dtex& T = P.tex[index & 7];
    float t[3];
    if (type == RT_TEXTYPE_SOLID) {
        texel_slot<STD>(P, index & 7, detail_i, 0, t);
        return mk3(t[0], t[1], t[2]);
    }
    if (type == RT_TEXTYPE_CHECKER) {   // :6-17
        int pix = detail_i * 3;
        texel_slot<STD>(P, index & 7, pix + 2, 0, t);
        float scale = t[0];
        float inv_scale = 1.0f / scale;
        v3 q = scale3(p, inv_scale);
        int s = rt_f2i(q.x) + rt_f2i(q.y) + rt_f2i(q.z);
        texel_slot<STD>(P, index & 7, (s % 2 == 0) ? pix : pix + 1, 0, t);
        return mk3(t[0], t[1], t[2]);
    }
    if (type == RT_TEXTYPE_PERLIN) {    // :79-94
#ifdef RT_AB_KNOBS
        if (P.debug_flags & 1) return mk3s(0.5f);   // ablation only (A/B build, RT_DEBUG_FLAGS), never exact
#endif
        float scale = ((float)detail_i / 4095.0f) * 100.0f;
        const bool lds = P.perlin_lds >= 0 && (index & 7) == P.perlin_slot;
        // PK_INLINE (the compact-box kernels, scene 8): the packed noise inline, -0.8% against the call;
        // the other kernels call it (inline it cost them 6 more spilled VGPRs, scene 6 +1.1%)
        const float accum = lds ? (PK_INLINE ? perlin_turb_lds_in(P.perlin_lds, p.x, p.y, p.z)
                                             : perlin_turb_lds(P.perlin_lds, p.x, p.y, p.z))
                                : perlin_turb_global(reinterpret_cast<const float*>(T.is_float ? T.data : nullptr),
                                                     T.w, T.h, p.x, p.y, p.z);
        float s = 1.0f + g_sin(scale * p.z + 10.0f * fabsf(accum));
        return mk3s(0.5f * s);
    }
    if (type == RT_TEXTYPE_IMAGE) {     // texture2D: GL_LINEAR, CLAMP_TO_EDGE
#ifdef RT_AB_KNOBS
        if (P.debug_flags & 2) return mk3s(0.5f);   // ablation only (A/B build, RT_DEBUG_FLAGS), never exact
#endif
        if (!T.data || T.w <= 0 || T.h <= 0) return mk3s(0.0f);
        v2 uv = resolve_uv<STD>(P, uvs, time);
        float x = uv.x * (float)T.w - 0.5f;
        float y = uv.y * (float)T.h - 0.5f;
        float fx = floorf(x), fy = floorf(y);
        float a = x - fx, b = y - fy;
        int x0 = rt_f2i(fx), y0 = rt_f2i(fy);
        int x1 = x0 >= T.w - 1 ? T.w - 1 : x0 + 1;
        int y1 = y0 >= T.h - 1 ? T.h - 1 : y0 + 1;
        x1 = x1 < 0 ? 0 : x1;
        y1 = y1 < 0 ? 0 : y1;
        x0 = x0 < 0 ? 0 : (x0 > T.w - 1 ? T.w - 1 : x0);
        y0 = y0 < 0 ? 0 : (y0 > T.h - 1 ? T.h - 1 : y0);
        float t00[3], t10[3], t01[3], t11[3];
        texel_in(T, x0, y0, t00); texel_in(T, x1, y0, t10); texel_in(T, x0, y1, t01); texel_in(T, x1, y1, t11);
        float r[3];
#pragma unroll
        for (int c = 0; c < 3; c++)
            r[c] = (t00[c] * (1.0f - a) + t10[c] * a) * (1.0f - b) + (t01[c] * (1.0f - a) + t11[c] * a) * b;
        return mk3(r[0], r[1], r[2]);
    }
    return mk3s(0.0f);
}

// ------------------------------------------------------------- sampling
// math.glsl:3-12
__device__ __forceinline__ v3 transform_onb(v3 vec, v3 normal) {
    v3 w = g_normalize(normal);
    v3 a = (fabsf(w.x) > 0.9f) ? mk3(0.0f, 1.0f, 0.0f) : mk3(1.0f, 0.0f, 0.0f);
    v3 v = g_normalize(g_cross(w, a));
    v3 u = g_cross(w, v);
    return g_mat3_mul(u, v, w, vec);
}

// random.glsl:40-49
__device__ __forceinline__ v3 rand_unit_vec(float& rf, float px, float py) {
    v3 p;
    for (;;) {
        float x = -1.0f + rnd(rf, px, py) * 2.0f;
        float y = -1.0f + rnd(rf, px, py) * 2.0f;
        float z = -1.0f + rnd(rf, px, py) * 2.0f;
        p = mk3(x, y, z);
#ifdef RT_ABL_UNITVEC1   // ablation (A/B builds only, not exact): the first candidate, no rejection
        break;
#endif
        if (g_dot(p, p) < 1.0f) break;
    }
    return g_normalize(p);
}

// pdf.glsl:11-24
// idx is the same in every lane (lights_pdf_value's loop): the records by scalar loads (ldc)
__device__ __forceinline__ float sphere_light_pdf(const KP& P, int idx, v3 o, v3 d, float time) {
    const float4* sp = reinterpret_cast<const float4*>(P.spheres + idx);
    const float4 A = ldc(sp), B = ldc(sp + 1);
    float t;
    if (!sphere_t_ab(A, B, time, o, d, g_dot(d, d), 0.001f, RT_INFINITY, t)) return 0.0f;
    v3 pc = sub3(f3(A), o);
    float d2 = g_dot(pc, pc);
    float ctm = sqrtf(1.0f - B.w * B.w / d2);
    float solid = 2.0f * RT_PI * (1.0f - ctm);
    return 1.0f / solid;
}

// pdf.glsl:41-51
__device__ __forceinline__ float quad_light_pdf(const KP& P, int idx, v3 o, v3 d) {
    const float4* q = reinterpret_cast<const float4*>(P.quads + idx);
    const float4* f = P.dquads + RT_DFACE_F4 * idx;
    float t, al, be;
    if (!quad_test_ab(f, ldc(f), ldc(f + 1), o, d, 0.001f, RT_INFINITY, t, al, be, false, true)) return 0.0f;
    v3 n = f3(ldc(q));
    bool front = g_dot(d, n) < 0.0f;
    v3 normal = front ? n : neg3(n);
    float d2 = t * t * g_dot(d, d);
    float cosine = fabsf(g_dot(d, normal) / g_length(d));
    return d2 / (cosine * ldc(q + 3).w);
}

// pdf.glsl:58-81
__device__ __forceinline__ float lights_pdf_value(const KP& P, v3 o, v3 d, float time) {
    float weight = 1.0f / (float)P.lights_count;
    float sum = 0.0f;
    for (int i = 0; i < P.lights_count; i++) {
        int packed = ldc_i(P.lights + i);   // the same in every lane: a scalar load
        int type = (packed >> 16) & 0xFFFF, idx = packed & 0xFFFF;
        float pdf = 0.0f;
        if (type == RT_MODEL_SPHERE) pdf = sphere_light_pdf(P, idx, o, d, time);
        else if (type == RT_MODEL_QUAD) pdf = quad_light_pdf(P, idx, o, d);
        sum += weight * pdf;
    }
    return sum;
}

// pdf.glsl:83-96 (+ random.glsl:71-80, pdf.glsl:26-30, :53-56); no light -> vec3(0) (Q1)
__device__ __forceinline__ v3 lights_random(const KP& P, v3 o, float& rf, float px, float py) {
    float r = 0.0f + rnd(rf, px, py) * ((float)(P.lights_count - 1 + 1) - 0.0f);
    int li = rt_f2i(floorf(r));
    if (li < 0 || li >= P.lights_count) return mk3s(0.0f);
    int packed = ldg_i(P.lights + li);
    int type = (packed >> 16) & 0xFFFF, idx = packed & 0xFFFF;
    if (type == RT_MODEL_SPHERE) {
        const float4* sp = reinterpret_cast<const float4*>(P.spheres + idx);
        float4 A = ldg(sp), B = ldg(sp + 1);
        v3 dir = sub3(f3(A), o);
        float d2 = g_dot(dir, dir);
        float r1 = rnd(rf, px, py);
        float r2 = rnd(rf, px, py);
        float z = 1.0f + r2 * (sqrtf(1.0f - B.w * B.w / d2) - 1.0f);
        float phi = 2.0f * RT_PI * r1;
        float s, c;
        g_sincos(phi, &s, &c);
        float x = c * sqrtf(1.0f - z * z);
        float y = s * sqrtf(1.0f - z * z);
        return transform_onb(mk3(x, y, z), dir);
    }
    if (type == RT_MODEL_QUAD) {
        const float4* q = reinterpret_cast<const float4*>(P.quads + idx);
        float4 Q1 = ldg(q + 1), Q2 = ldg(q + 2), Q3 = ldg(q + 3);
        float r1 = rnd(rf, px, py);
        v3 p = add3(f3(Q1), scale3(f3(Q2), r1));
        float r2 = rnd(rf, px, py);
        p = add3(p, scale3(f3(Q3), r2));
        return sub3(p, o);
    }
    return mk3s(0.0f);
}

// ------------------------------------------------------------- ray_color
// Per-lane path state carried between bounces (ray_color's locals).
struct Path {
    v3 o, d, acc;
    float time, rf;
    UvSrc uvs;
    int depth;
};

// The shading half of ray_color's loop body (compute.glsl:310-339) for a hit.
// Returns true when the path ended, with its color in `result`.
// STD (RT_OPT_STD kernels): the shading tables are staged -- every sphere's, and with PK_INLINE (the
// compact-box kernels) every box's; the texture descriptors
template <bool PK_INLINE = false, bool STATS = false, bool STD = false>
__device__ __forceinline__ bool shade(const KP& P, Path& S, const Hit& h, float px, float py, v3& result,
                                      unsigned long long* st = nullptr) {
    unsigned long long c0 = STATS ? clock64() : 0;
    v3 d = S.d;
    // hit_record of the closest hit: p = ray.o + ray.dir*t (hitting.glsl:39,104,188)
    v3 p = add3(S.o, scale3(d, h.t));
    v3 normal;
    bool front;
    int material, tex_id;
    v3 emis = mk3s(0.0f);
    const int h_type = h.tif & 0xF, h_face = (h.tif >> 4) & 0x7, h_idx = (int)((unsigned)h.tif >> 16);
    if (h_type == RT_MODEL_SPHERE) {   // hitting.glsl:40-42 + compute.glsl:199-204
        const float4* sp = reinterpret_cast<const float4*>(P.spheres + h_idx);
        float4 A, B, C;
        if (STD || P.sph_mat_lds >= 0) {   // the shading tables: the whole record from LDS
            A = rt_dyn_lds[P.sph_lds + 2 * h_idx];
            B = rt_dyn_lds[P.sph_lds + 2 * h_idx + 1];
            C = rt_dyn_lds[P.sph_mat_lds + h_idx];
        } else {
            A = ldg(sp);
            B = ldg(sp + 1);
            C = ldg(sp + 2);
        }
        v3 center = add3(f3(A), scale3(f3(B), S.time));
        v3 on = divs3(sub3(p, center), B.w);
        front = g_dot(d, on) < 0.0f;
        normal = front ? on : neg3(on);
        material = __float_as_int(C.w);
        tex_id = __float_as_int(A.w);
        if (front) emis = f3(C);
    } else if (h_type == RT_MODEL_CONSTANT_MEDIUM) {   // hitting.glsl:189-190 + compute.glsl:211-216
        normal = mk3(1.0f, 0.0f, 0.0f);
        front = true;
        material = ldg_i(&P.media[h_idx].phase_material);
        tex_id = ldg_i(&P.media[h_idx].texture_id);
    } else if (h_type == RT_MODEL_BOX && (STD ? PK_INLINE : P.box_mat_lds >= 0)) {
        // a compact box from the shading tables: face h_face's normal rebuilt bit for bit from the
        // compact record (canonical axis and value, the zero components' signs in c2.w), material,
        // texture and emission of quads[0] (compute.glsl:217-221)
        const float4* cr = rt_dyn_lds + P.box_cmp_lds + RT_BOXC_F4 * h_idx;
        const float4 c1 = cr[1], c2 = cr[2];
        const float4 bm = rt_dyn_lds[P.box_mat_lds + h_idx];
        const float sval = h_face == 0 ? c1.z : h_face == 1 ? c1.w : h_face == 2 ? -c1.z
                         : h_face == 3 ? -c1.w : h_face == 4 ? c2.x : -c2.x;
        const int ax = (h_face == 0 || h_face == 2) ? 2 : (h_face == 1 || h_face == 3) ? 0 : 1;
        const uint32_t zm = (uint32_t)__float_as_int(c2.w) >> (2 * h_face);
        const float z1 = __uint_as_float((zm & 1u) << 31), z2 = __uint_as_float(((zm >> 1) & 1u) << 31);
        // components (ax+1)%3 and (ax+2)%3 are the zeros
        v3 n = ax == 0 ? mk3(sval, z1, z2) : ax == 1 ? mk3(z2, sval, z1) : mk3(z1, z2, sval);
        front = g_dot(d, n) < 0.0f;
        normal = front ? n : neg3(n);
        material = __float_as_int(bm.w);
        tex_id = __float_as_int(c2.z);
        if (front) emis = mk3(bm.x, bm.y, bm.z);
    } else {   // quad, or box face h_face (material from quads[0], compute.glsl:217-221)
        const float4* q0 = (h_type == RT_MODEL_QUAD) ? reinterpret_cast<const float4*>(P.quads + h_idx)
                                                    : reinterpret_cast<const float4*>(P.boxes + h_idx);
        v3 n = f3(ldg(q0 + 5 * h_face));
        front = g_dot(d, n) < 0.0f;
        normal = front ? n : neg3(n);
        material = __float_as_int(ldg(q0 + 1).w);
        tex_id = __float_as_int(ldg(q0 + 2).w);
        if (front) emis = f3(ldg(q0 + 4));
    }
    // A solid texture's colour (texture_color's first case) read here, before the scatter, so that its
    // two dependent LDS reads overlap the scatter's arithmetic; the same texel, so the same value.
    // Not in the compact-box kernels (PK_INLINE, scene 8): there +0.5%, scene 6 -1.5%, scene 0 -0.7%
    // (profiles/r05_u_lib_ab.log).
    const bool solid_tex = !PK_INLINE && ((tex_id >> 28) & 0xF) == RT_TEXTYPE_SOLID;
    float sc[3] = {0.0f, 0.0f, 0.0f};
    if (solid_tex) texel_slot<STD>(P, (tex_id >> 12) & 7, tex_id & 0xFFF, 0, sc);
    // scatter (scatter.glsl:43-98)
    int mid = (material >> 16) & 0xFFFF;
    bool skip_pdf = false, should = false;
    if (STATS) {
        const unsigned long long c1 = clock64();
        st_add(st, ST_SH_HIT_CYC, c1 - c0);
        c0 = c1;
        st_pred(st, mid == RT_MAT_LAMBERTIAN, ST_SH_LAM_IT, ST_SH_LAM_LN);
        st_pred(st, mid == RT_MAT_ISOTROPIC, ST_SH_ISO_IT, ST_SH_ISO_LN);
        st_pred(st, mid == RT_MAT_METAL, ST_SH_MET_IT, ST_SH_MET_LN);
        st_pred(st, mid == RT_MAT_DIELECTRIC, ST_SH_DIE_IT, ST_SH_DIE_LN);
    }
    if (mid == RT_MAT_DIFFUSE_LIGHT) {
        result = mul3(S.acc, emis);
        return true;
    }
    float& rf = S.rf;
    if (mid == RT_MAT_LAMBERTIAN) {
        float r1 = rnd(rf, px, py);
        float r2 = rnd(rf, px, py);
        float phi = 2.0f * RT_PI * r1;
        float s, c;
        g_sincos(phi, &s, &c);
        v3 cd = mk3(c * sqrtf(r2), s * sqrtf(r2), sqrtf(1.0f - r2));
        d = transform_onb(cd, normal);
        should = true;
    } else if (mid == RT_MAT_METAL) {
        float fuzz = (float)(material & 0xFFFF) / 65535.0f;
        d = g_reflect(d, normal);
        v3 n = g_normalize(d);
        d = add3(n, scale3(rand_unit_vec(rf, px, py), fuzz));
        should = g_dot(d, normal) > 0.0f;
        skip_pdf = true;
    } else if (mid == RT_MAT_DIELECTRIC) {
        float nior = (float)(material & 0xFFFF) / 65535.0f;
        float eta = g_mix(1.0f, 2.5f, nior);
        if (front) eta = 1.0f / eta;
        d = g_normalize(d);
        float cos_t = g_min(g_dot(neg3(d), normal), 1.0f);
        float sin_t = sqrtf(1.0f - cos_t * cos_t);
        bool refl = eta * sin_t > 1.0f;
        if (!refl) {
            float r0 = (1.0f - eta) / (1.0f + eta);
            r0 = r0 * r0;
            float rr = r0 + (1.0f - r0) * g_pow5(1.0f - cos_t);
            refl = rr > rnd(rf, px, py);
        }
        d = refl ? g_reflect(d, normal) : g_refract(d, normal, eta);
        should = true;
        skip_pdf = true;
    } else if (mid == RT_MAT_ISOTROPIC) {
        d = rand_unit_vec(rf, px, py);
        should = true;
    }
    if ((fabsf(d.x) < 1e-8f) && (fabsf(d.y) < 1e-8f) && (fabsf(d.z) < 1e-8f)) d = normal;
    if (STATS) {
        const unsigned long long c1 = clock64();
        st_add(st, ST_SH_SCAT_CYC, c1 - c0);
        c0 = c1;
    }
    if (!should) {
        result = mul3(S.acc, emis);
        return true;
    }
    S.o = p;
    if (skip_pdf) {
        S.acc = mul3(S.acc, solid_tex ? mk3(sc[0], sc[1], sc[2]) : texture_color<PK_INLINE, STD>(P, p, tex_id, S.uvs, S.time));
        S.d = d;
        if (STATS) st_add(st, ST_SH_TEX_CYC, clock64() - c0);
        return false;
    }
    if (rnd(rf, px, py) < 0.5f) d = lights_random(P, p, rf, px, py);
    float lpdf = (P.lights_count > 0) ? lights_pdf_value(P, p, d, S.time) : 0.0f;
    float mpdf;
    // cosine_pdf_value (pdf.glsl:32-35): max(0, normalize(cos)/PI) with the scalar
    // normalize = cos/|cos| in {+1, -1, NaN}: 1/PI exactly when 0 < cos < inf, else 0
    if (mid == RT_MAT_LAMBERTIAN) {
        float cs = g_dot(d, normal);
        mpdf = (cs > 0.0f && cs < INFINITY) ? 1.0f / RT_PI : 0.0f;
    }
    else if (mid == RT_MAT_ISOTROPIC) mpdf = 1.0f / (4.0f * RT_PI);
    else mpdf = 0.0f;
    float pdf = 0.5f * lpdf + 0.5f * mpdf;
    if (pdf == 0.0f) {
        result = mul3(S.acc, emis);
        return true;
    }
    float spdf;
    if (mid == RT_MAT_LAMBERTIAN) spdf = g_max(0.0f, g_dot(normal, g_normalize(d)) / RT_PI);
    else if (mid == RT_MAT_ISOTROPIC) spdf = 1.0f / (4.0f * RT_PI);
    else spdf = 0.0f;
    if (STATS) {
        const unsigned long long c1 = clock64();
        st_add(st, ST_SH_MIX_CYC, c1 - c0);
        c0 = c1;
    }
    v3 att = solid_tex ? mk3(sc[0], sc[1], sc[2]) : texture_color<PK_INLINE, STD>(P, p, tex_id, S.uvs, S.time);
    if (STATS) st_add(st, ST_SH_TEX_CYC, clock64() - c0);
    S.acc = mul3(S.acc, divs3(scale3(att, spdf), pdf));
    S.d = d;
    return false;
}

// The rest of ray_color's loop body after the walk (compute.glsl:308-340): the
// uv the walk left (compute.glsl:62), the background on a miss, else shade().
template <bool PK_INLINE = false, bool STATS = false, bool STD = false>
__device__ __forceinline__ bool after_trace(const KP& P, Path& S, const Hit& h, bool hit, float px, float py,
                                            v3& result, unsigned long long* st = nullptr) {
    if (h.uv_kind_idx != 0) {
        bool sph = (h.uv_kind_idx >> 16) == 1;
        v3 up = add3(S.o, scale3(S.d, h.uv_a));   // the sphere hit's p (hitting.glsl:39)
        S.uvs.kind_idx = h.uv_kind_idx;
        S.uvs.a = sph ? up.x : h.uv_a;
        S.uvs.b = sph ? up.y : h.uv_b;
        S.uvs.c = sph ? up.z : S.uvs.c;
    }
    if (!hit) {
        result = mul3(S.acc, mk3(P.background[0], P.background[1], P.background[2]));
        return true;
    }
    return shade<PK_INLINE, STATS, STD>(P, S, h, px, py, result, st);
}

// Camera ray of frame `frame_count` (compute.glsl:345-350, random.glsl:19-30,82-100).
__device__ __forceinline__ void start_path(const KP& P, Path& S, int frame_count, float rf0, float fx, float fy,
                                           v3 base) {
    const rt_camera_ubo& C = P.cam;
    v3 du = ld3(C.pixel_delta_u), dv = ld3(C.pixel_delta_v), cpos = ld3(C.camera_pos);
    float rf = rf0;
    S.time = rnd(rf, fx, fy);
    float col = g_mod((float)frame_count, P.sqrt_spp);
    float layer = (float)frame_count / P.sqrt_spp;
    float base_x = (col + 0.5f) * P.recip_sqrt_spp;
    float base_y = (layer + 0.5f) * P.recip_sqrt_spp;
    float jx = (rnd(rf, fx, fy) - 0.5f) * P.recip_sqrt_spp;
    float jy = (rnd(rf, fx, fy) - 0.5f) * P.recip_sqrt_spp;
    float spx = base_x + jx - 0.5f;
    float spy = base_y + jy - 0.5f;
    v3 coord = add3(base, add3(scale3(du, spx), scale3(dv, spy)));
    v3 o = cpos;
    if (!(C.defocus_angle <= 0.0f)) {
        float dx, dy;
        for (;;) {
            dx = -1.0f + rnd(rf, fx, fy) * 2.0f;
            dy = -1.0f + rnd(rf, fx, fy) * 2.0f;
            v3 p = mk3(dx, dy, 0.0f);
            if (g_dot(p, p) < 1.0f) break;
        }
        o = add3(add3(cpos, scale3(ld3(C.defocus_disk_u), dx)), scale3(ld3(C.defocus_disk_v), dy));
    }
    S.rf = rf;
    S.o = o;
    S.d = sub3(coord, o);
    S.acc = mk3s(1.0f);
    S.depth = 0;
    S.uvs.kind_idx = 0; S.uvs.a = 0.0f; S.uvs.b = 0.0f; S.uvs.c = 0.0f;
}

// Ordered chunks (a launch over few tiles per resident wave, e.g. the stripe set
// of one of N GPUs): the work unit is one 8x8 tile x one chunk of the launch's
// frames, unit = chunk * n_tiles + tile, so chunk k of a tile is dequeued after
// chunk k-1.  The wave that takes chunk k > 0 waits until chunk k-1 of its tile
// is published, then continues that tile's running mean from the image: the
// reference's per-frame formula in frame order, so the same bits as one chunk.
// Publication follows the agent-scope release/acquire recipe of
// cdna_hip_programming.md §6 G16: the producing wave's plain image stores,
// vmcnt(0), release fence, vmcnt(0), then one relaxed agent-scope store of the
// tile's chunk count; the consumer polls that word relaxed (with s_sleep), then
// one acquire fence, then plain loads.  The unit it waits for was dequeued
// earlier by a running wave that waits only on earlier units, so the chain ends
// at chunk 0; the poll is still bounded (RT_CHUNK_WAIT_TICKS of the 100 MHz
// real-time clock, P.chunk_wait_ticks: 30 s by default) and a timeout sets
// P.fault, which rt_sync reports.
typedef __attribute__((address_space(1))) unsigned gu32;   // global (never flat) accesses to shared words
// tile and chunk are wave-uniform (readfirstlane): every lane polls / stores the
// same word with the same value, so there is no lane-divergent control flow here
__device__ __forceinline__ void wait_chunk(const KP& P, int tile, int chunk) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    gu32* w = (gu32*)(P.tile_done + tile);
    while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) <
           (unsigned)chunk) {
        __builtin_amdgcn_s_sleep(2);
        if (__builtin_amdgcn_s_memrealtime() - t0 >= P.chunk_wait_ticks) {
            __hip_atomic_store((gu32*)P.fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void publish_chunk(const KP& P, int tile, int chunk) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store((gu32*)(P.tile_done + tile), (unsigned)(chunk + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The link-format shapes' LDS staging (rt_capi.hip plans it; every workgroup once): the nodes
// (all, or the two-level walk's top levels; LINK = false: the threaded meta-word nodes of the A/B
// variant 30), the leaf records, the packed Perlin table, the media records with their sphere
// boundaries, the spheres' (A, B) halves, the boxes' compact records and the shading tables.
template <bool LINK, int BLOCK>
__device__ __forceinline__ void stage_lds(const KP& P, float4* s_nodes, int tid) {
    // link format: the nodes staged (all, or the two-level walk's top levels), then the leaf
    // records when they are staged too; meta format: the threaded nodes
    const float4* g = LINK ? P.lnodes : reinterpret_cast<const float4*>(P.nodes);
    const int nf4 = LINK ? P.lds_node_f4 : 2 * P.n_nodes;
    for (int k = tid; k < nf4; k += BLOCK) s_nodes[k] = g[k];
    if (LINK && P.leaf_lds >= 0)
        for (int k = tid; k < P.n_lnode_f4 - 2 * P.n_nodes; k += BLOCK)
            s_nodes[P.leaf_lds + k] = g[2 * P.n_nodes + k];
    if (P.perlin_lds >= 0)   // the packed Perlin table after the nodes (host-sized launch)
        for (int k = tid; k < 256; k += BLOCK) s_nodes[P.perlin_lds + k] = ldg(P.perlin_pk + k);
    if (P.media_lds >= 0) {   // per medium: (boundary idx, type, -1/density, phase), sphere A, B
        for (int k = tid; k < 3 * P.n_media; k += BLOCK) {
            const rt_medium& m = P.media[k / 3];
            float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (k % 3 == 0)
                v = make_float4(__int_as_float(m.boundary_idx), __int_as_float(m.boundary_type), m.neg_inv_density,
                                __int_as_float(m.phase_material));
            else if (m.boundary_type == RT_MODEL_SPHERE)
                v = reinterpret_cast<const float4*>(P.spheres + m.boundary_idx)[k % 3 - 1];
            s_nodes[P.media_lds + k] = v;
        }
    }
    if (P.sph_lds >= 0) {   // per sphere its first two float4 (center0 + texture, motion + radius)
        const float4* sp = reinterpret_cast<const float4*>(P.spheres);
        for (int k = tid; k < 2 * P.n_sph_lds; k += BLOCK) s_nodes[P.sph_lds + k] = ldg(sp + (k >> 1) * 3 + (k & 1));
    }
    if (P.box_cmp_lds >= 0)   // the boxes' compact records (box_test_compact)
        for (int k = tid; k < RT_BOXC_F4 * P.n_box_lds; k += BLOCK) s_nodes[P.box_cmp_lds + k] = ldg(P.dboxc + k);
    // the shading tables (P.sph_mat_lds / box_mat_lds / tex_lds, option shade_lds)
    if (P.sph_mat_lds >= 0) {   // per sphere its third float4: emission, material
        const float4* sp = reinterpret_cast<const float4*>(P.spheres);
        for (int k = tid; k < P.n_sph_lds; k += BLOCK) s_nodes[P.sph_mat_lds + k] = ldg(sp + 3 * k + 2);
    }
    if (P.box_mat_lds >= 0) {   // per box quads[0]'s emission and material
        for (int k = tid; k < P.n_box_lds; k += BLOCK) {
            const float4* q0 = reinterpret_cast<const float4*>(P.boxes + k);
            const float4 e = ldg(q0 + 4), m = ldg(q0 + 1);
            s_nodes[P.box_mat_lds + k] = make_float4(e.x, e.y, e.z, m.w);
        }
    }
    if (P.tex_lds >= 0) {   // per slot (w, h, is_float, texel offset), then the small slots' texels
        if (tid < 8) {
            const rt_dtex& T = P.tex[tid];
            const int off = T.data ? P.tex_lds_off[tid] : -1;
            s_nodes[P.tex_lds + tid] = make_float4(__int_as_float(T.data ? T.w : 0), __int_as_float(T.h),
                                                   __int_as_float(T.is_float), __int_as_float(off));
        }
        for (int t = 0; t < 8; t++) {
            const rt_dtex& T = P.tex[t];
            if (P.tex_lds_off[t] < 0 || !T.data) continue;
            const int words = T.w * T.h;
            const uint32_t* src = reinterpret_cast<const uint32_t*>(T.data);
            uint32_t* dst = reinterpret_cast<uint32_t*>(s_nodes + P.tex_lds_off[t]);
            for (int k = tid; k < words; k += BLOCK) dst[k] = src[k];
        }
    }
}

template <typename K>
int launch_persistent(K kernel, int block, size_t lds, const rt_kernel_args& a, const rt_kernel_args* d,
                      hipStream_t st) {
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
    if (lds > 64 * 1024 &&
        hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds) != hipSuccess)
        return -1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, lds) != hipSuccess || per_cu < 1)
        per_cu = 1;
    per_cu = per_cu > 2 ? 2 : per_cu;   // rt_resident_waves(): the per-wave buffers are sized for it
    if ((long long)cus * per_cu * (block / 64) > (long long)rt_resident_waves()) return -1;
    if (a.wbuf && (long long)cus * per_cu * (block / 64) > (long long)a.wbuf_waves) return -1;
    hipLaunchKernelGGL(kernel, dim3(cus * per_cu), dim3(block), lds, st, d);
    return 0;
}

}  // namespace
