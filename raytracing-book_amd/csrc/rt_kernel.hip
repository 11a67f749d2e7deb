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
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "rt/rt_glsl.h"
#include "rt_device.h"

namespace {

typedef rt_kernel_args KP;

// OPT bits of the kernel templates
#define RT_OPT_POOL 1   // pooled units (render_pool): without it a lane owns a pixel (variant 37)
#define RT_OPT_SM 2     // with RT_OPT_POOL and the link walk: walks and shading in batches (render_stream)
#define RT_OPT_FD 4     // with RT_OPT_SM: the scene is in the shared-reciprocal division regime (P.fastdiv)
#define RT_OPT_STREAM 8 // with RT_OPT_SM: the wave streams over units (render_stream) instead of one at a time
#define RT_OPT_TL 16    // with RT_OPT_STREAM: two-level walk (top levels in LDS, the rest of the nodes global)
#define RT_OPT_BOXC 32  // with RT_OPT_STREAM: every box has a compact record (box_test_compact), no full box test
#define RT_OPT_SPAIR 64 // with RT_OPT_STREAM: leaves of two spheres tested at once (leaf_prims_t; most leaves are)

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
    ST_SPH_SM, ST_QUAD_SM, ST_BOX_SM, ST_MED_SM, ST_NODE_SM, ST_N
};
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
                                             bool fd = false) {
    const float4 Q2 = ldg(f + 2);
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
template <bool FD = false>
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
    if (m.boundary_type == RT_MODEL_SPHERE) {
        if (!sphere_bounds(R1, R2, o, d, a, time, t1, t2, FD)) return false;
    } else if (!medium_bounds(P, m, o, d, a, time, t1, t2)) {
        return false;
    }
    return medium_tail(m.neg_inv_density, t1, t2, a, tmin, tmax, rf, px, py, t);
}

// hitting.glsl:162-193 — returns the hit distance t.
template <bool FD = false>
__device__ __forceinline__ bool medium_test(const KP& P, int idx, v3 o, v3 d, float a, float time, float tmin,
                                            float tmax, float& rf, float px, float py, float& t) {
    float t1, t2;
    rt_medium m;
    if (P.media_lds >= 0) {   // the record and its sphere boundary from LDS (render_persistent)
        const float4* r = rt_dyn_lds + P.media_lds + 3 * idx;
        const float4 R0 = r[0];
        m.boundary_idx = __float_as_int(R0.x);
        m.boundary_type = __float_as_int(R0.y);
        m.neg_inv_density = R0.z;
        m.phase_material = __float_as_int(R0.w);
        m.texture_id = 0;
        if (m.boundary_type == RT_MODEL_SPHERE) {
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
template <bool STATS, bool FD, bool BOXC = false, bool SPAIR = false>
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
    if (SPAIR && !STATS && P.sph_lds >= 0 && ((meta >> 16) & 0xFFu) == (RT_MODEL_SPHERE | (RT_MODEL_SPHERE << 4))) {
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
        const bool pf = BOXC && P.leaf_pf;   // wave-uniform
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
            } else if (P.sph_lds >= 0) {   // the record's intersection half from LDS (render_persistent)
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
            } else if (P.box_cmp_lds >= 0) {
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
            hit = pf ? medium_test_rec<FD>(P, q0, q1, q2, o, d, a, time, tmin, tmax, rf, px, py, t)
                     : medium_test<FD>(P, ix, o, d, a, time, tmin, tmax, rf, px, py, t);
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
};
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
template <bool EXACT, bool STATS, bool TL = false>
__device__ __forceinline__ uint32_t link_walk_part(const NodeSrc& ns, uint32_t nx, v3 o, v3 inv, float tmin,
                                                   float tmax, int need, unsigned long long* st) {
    for (;;) {
#pragma unroll
        for (int k = 0; k < 3; k++) {
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
                nx = __float_as_uint(hit ? n1.z : n1.w);
            }
        }
        const unsigned long long walking = __ballot((int)nx >= 0);
        if (walking == 0 || __popcll(__ballot(1) & ~walking) >= need) break;
    }
    return nx;
}

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
__device__ __forceinline__ void texel_slot(const KP& P, int slot, int x, int y, float out[3]) {
    if (P.tex_lds >= 0) {
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

__device__ __forceinline__ v2 resolve_uv(const KP& P, const UvSrc& s, float time) {
    int kind = s.kind_idx >> 16;
    if (kind == 2) { v2 r = {s.a, s.b}; return r; }
    if (kind == 1) {
        const int si = s.kind_idx & 0xFFFF;
        float4 A, B;
        if (P.sph_mat_lds >= 0) {   // the shading tables are on: the sphere's (A, B) from LDS
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
template <bool PK_INLINE = false>
__device__ __forceinline__ v3 texture_color(const KP& P, v3 p, int id, const UvSrc& uvs, float time) {
    int detail_i = id & 0xFFF;
    int index = (id >> 12) & 0xFFFF;
    int type = (id >> 28) & 0xF;
    const rt_dtex& T = P.tex[index & 7];
    float t[3];
    if (type == RT_TEXTYPE_SOLID) {
        texel_slot(P, index & 7, detail_i, 0, t);
        return mk3(t[0], t[1], t[2]);
    }
    if (type == RT_TEXTYPE_CHECKER) {   // :6-17
        int pix = detail_i * 3;
        texel_slot(P, index & 7, pix + 2, 0, t);
        float scale = t[0];
        float inv_scale = 1.0f / scale;
        v3 q = scale3(p, inv_scale);
        int s = rt_f2i(q.x) + rt_f2i(q.y) + rt_f2i(q.z);
        texel_slot(P, index & 7, (s % 2 == 0) ? pix : pix + 1, 0, t);
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
        v2 uv = resolve_uv(P, uvs, time);
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
        if (g_dot(p, p) < 1.0f) break;
    }
    return g_normalize(p);
}

// pdf.glsl:11-24
__device__ __forceinline__ float sphere_light_pdf(const KP& P, int idx, v3 o, v3 d, float time) {
    const float4* sp = reinterpret_cast<const float4*>(P.spheres + idx);
    float t;
    if (!sphere_t(sp, time, o, d, g_dot(d, d), 0.001f, RT_INFINITY, t)) return 0.0f;
    float4 A = ldg(sp), B = ldg(sp + 1);
    v3 pc = sub3(f3(A), o);
    float d2 = g_dot(pc, pc);
    float ctm = sqrtf(1.0f - B.w * B.w / d2);
    float solid = 2.0f * RT_PI * (1.0f - ctm);
    return 1.0f / solid;
}

// pdf.glsl:41-51
__device__ __forceinline__ float quad_light_pdf(const KP& P, int idx, v3 o, v3 d) {
    const float4* q = reinterpret_cast<const float4*>(P.quads + idx);
    float t, al, be;
    if (!quad_test(P.dquads + RT_DFACE_F4 * idx, o, d, 0.001f, RT_INFINITY, t, al, be)) return 0.0f;
    v3 n = f3(ldg(q));
    bool front = g_dot(d, n) < 0.0f;
    v3 normal = front ? n : neg3(n);
    float d2 = t * t * g_dot(d, d);
    float cosine = fabsf(g_dot(d, normal) / g_length(d));
    return d2 / (cosine * ldg(q + 3).w);
}

// pdf.glsl:58-81
__device__ __forceinline__ float lights_pdf_value(const KP& P, v3 o, v3 d, float time) {
    float weight = 1.0f / (float)P.lights_count;
    float sum = 0.0f;
    for (int i = 0; i < P.lights_count; i++) {
        int packed = ldg_i(P.lights + i);
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
#define RT_FAST_STACK 16
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
template <bool PK_INLINE = false>
__device__ __forceinline__ bool shade(const KP& P, Path& S, const Hit& h, float px, float py, v3& result) {
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
        if (P.sph_mat_lds >= 0) {   // the shading tables: the whole record from LDS
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
    } else if (h_type == RT_MODEL_BOX && P.box_mat_lds >= 0) {
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
    // scatter (scatter.glsl:43-98)
    int mid = (material >> 16) & 0xFFFF;
    bool skip_pdf = false, should = false;
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
    if (!should) {
        result = mul3(S.acc, emis);
        return true;
    }
    S.o = p;
    if (skip_pdf) {
        S.acc = mul3(S.acc, texture_color<PK_INLINE>(P, p, tex_id, S.uvs, S.time));
        S.d = d;
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
    v3 att = texture_color<PK_INLINE>(P, p, tex_id, S.uvs, S.time);
    S.acc = mul3(S.acc, divs3(scale3(att, spdf), pdf));
    S.d = d;
    return false;
}

// The rest of ray_color's loop body after the walk (compute.glsl:308-340): the
// uv the walk left (compute.glsl:62), the background on a miss, else shade().
template <bool PK_INLINE = false>
__device__ __forceinline__ bool after_trace(const KP& P, Path& S, const Hit& h, bool hit, float px, float py,
                                            v3& result) {
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
    return shade<PK_INLINE>(P, S, h, px, py, result);
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
    g.f0 = g.chunk * P.chunk_frames;
    g.f1 = min(P.n_frames, g.f0 + P.chunk_frames);
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
    const bool staged = P.samples != nullptr;
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
    for (;;) {
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
        // claim samples for the FRESH lanes (compute.glsl:345-350); a new unit when the
        // pool's unit has none left
        bool fin = false;   // a sample stored in this pass (max_depth 0)
        for (;;) {
            const unsigned long long need = __ballot(status == RT_SM_FRESH);
            if (need == 0) break;
            if (next >= total_cur) {
                if (no_more) break;
                const int o = staged ? 0 : cur ^ 1;
                if (!staged && (o ? unit1 : unit0) >= 0) break;   // both slots in use: the FRESH lanes wait
                int u = 0;
                if (lane == 0) u = atomicAdd(P.tile_counter, 1);
                u = __builtin_amdgcn_readfirstlane(__shfl(u, 0));
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
                            if (P.sflags) P.sflags[dst] = 0;   // sparse: a zero colour is its clear flag
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
        }
        // per-ray constants of every walk (new or resumed: the same values again)
        if (status == RT_SM_TRACE) {
            inv = mk3(1.0f / S.d.x, 1.0f / S.d.y, 1.0f / S.d.z);
            a = g_dot(S.d, S.d);
        }
        // rounds of node walk + leaf tests (trace()), at wave priority 1: their dependent LDS
        // chains then issue as soon as their data is back, and the shading's long VALU runs (at
        // priority 0) fill the gaps -- scene 8 -3.1%, scene 0 -2.1%, scenes 6 / 7 -0.4 / -1.2%
        // (profiles/r04_setprio_combined_lib_ab.log; the walk alone at 1: scene 6 +0.6%)
        __builtin_amdgcn_s_setprio(1);
        for (;;) {
            const unsigned long long tr = __ballot(status == RT_SM_TRACE);
            const int n_hit = __popcll(__ballot(status == RT_SM_HIT));
            if (STATS && tr) st_pred(st, status == RT_SM_FRESH, ST_RET_IT, ST_RET_LN);
            if (tr == 0 || n_hit >= batch || n_hit * 64 >= P.sm_frac * (n_hit + __popcll(tr))) break;
            const bool lane_exact = (inv.x == -INFINITY) || (inv.y == -INFINITY) || (inv.z == -INFINITY);
            const bool wave_exact = __ballot(status == RT_SM_TRACE && lane_exact) != 0;
            if (status == RT_SM_TRACE) {
                if (STATS) st_lanes(st, ST_ROUND_IT, ST_ROUND_LN);
                unsigned long long t0 = STATS ? clock64() : 0;
                if (P.walk_frac >= 64) {
                    nx = wave_exact ? link_walk<true, STATS, TL>(ns, nx, S.o, inv, 0.001f, tmax, st)
                                    : link_walk<false, STATS, TL>(ns, nx, S.o, inv, 0.001f, tmax, st);
                } else {
                    const int needw = (__popcll(__ballot(1)) * P.walk_frac + 63) >> 6;
                    nx = wave_exact ? link_walk_part<true, STATS, TL>(ns, nx, S.o, inv, 0.001f, tmax, needw, st)
                                    : link_walk_part<false, STATS, TL>(ns, nx, S.o, inv, 0.001f, tmax, needw, st);
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
                    leaf_prims_t<STATS, FD, BOXC, (OPT & RT_OPT_SPAIR) != 0>(P, lf.x << 16, lf.y, S.o, S.d, inv, a,
                                                                             S.time, 0.001f, tmax, S.rf,
                                                  fx, fy, h, has, st);
                    if (STATS) st_add(st, ST_LEAF_CYC, clock64() - t1);
                    nx = lf.x >> 8;   // the leaf's skip node
                    if (nx == RT_LINK_NEXT_END) status = RT_SM_HIT;
                }
            }
        }
        __builtin_amdgcn_s_setprio(0);
        // shade the HIT lanes together
        if (status == RT_SM_HIT) {
            unsigned long long ts = STATS ? clock64() : 0;
            if (STATS) st_lanes(st, ST_SHADE_IT, ST_SHADE_LN);
            v3 cur3;
            h.t = tmax;   // the accepted hit's t (unused on a miss)
            bool done = after_trace<BOXC>(P, S, h, has, fx, fy, cur3);
            if (!done && S.depth >= P.max_depth) {   // the loop is exhausted: final_color stays vec3(0)
                cur3 = mk3s(0.0f);
                done = true;
            }
            if (done) {
                const float4 c4 = make_float4(cur3.x, cur3.y, cur3.z, 0.0f);
                if (staged) {
                    // sparse staging (P.sflags): every sample writes one flag byte, and only a colour
                    // that is not exactly (+0, +0, +0) is stored; fold_kernel reads a clear flag as
                    // that zero colour -- the same values, so the same running mean
                    if (P.sflags) {
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
        // the samples stored in this pass, per slot
        const unsigned long long f_all = __ballot(fin), f_one = __ballot(fin && up == 1);
        done0 += (uint32_t)__popcll(f_all & ~f_one);
        done1 += (uint32_t)__popcll(f_one);
        stored += (uint32_t)__popcll(f_all);
        // the end: no unit left to claim, every lane idle, every slot folded
        if (no_more && __ballot(status != RT_SM_FRESH) == 0 && (staged || (unit0 < 0 && unit1 < 0))) break;
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
__global__ void __launch_bounds__(BLOCK, MINW) render_persistent(const KP* __restrict__ Pp) {
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
    // per lane: the pixel's running mean during a unit, after what this launch
    // shape stages (P.acc_lds, set by rt_launch_render with the LDS size)
    float4* s_acc = s_nodes + P.acc_lds;
    if (LDSN || STATS) __syncthreads();
    if (STATS) t_begin = clock64();
    const float4* __restrict__ rnodes = (LDSN && !FAST) ? s_nodes : reinterpret_cast<const float4*>(P.nodes);
    const int tiles_x = (P.width + 7) >> 3;
    const int n_tiles = tiles_x * ((P.local_rows + 7) >> 3);
    const int n_units = n_tiles * P.n_chunks;
    if constexpr (LINK && !FAST && (OPT & RT_OPT_SM) && (OPT & RT_OPT_STREAM)) {
        render_stream<STATS, OPT, (OPT & RT_OPT_FD) != 0>(P, rnodes, (int)blockIdx.x * (BLOCK / 64) + (tid >> 6), st);
    } else for (;;) {
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
        info[RT_LI_SPAIR] = (pool && shape == LINK_LDS && a.sph_pairs && !a.box_all_cmp && a.sph_lds >= 0) ? 1 : 0;
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
    // the instantiations: <LINK, MINW, STATS, LDSN, BLOCK, FAST, OPT>
#ifdef RT_AB_KNOBS
#define RT_KERNEL(LINK, LDSN, BLOCK, FAST, OPT)                                                                    \
    (stats ? launch_persistent(render_persistent<LINK, 4, true, LDSN, BLOCK, FAST, OPT>, BLOCK, lds, a, d, st)  \
           : launch_persistent(render_persistent<LINK, 4, false, LDSN, BLOCK, FAST, OPT>, BLOCK, lds, a, d, st))
#else
#define RT_KERNEL(LINK, LDSN, BLOCK, FAST, OPT) \
    launch_persistent(render_persistent<LINK, 4, false, LDSN, BLOCK, FAST, OPT>, BLOCK, lds, a, d, st)
#endif
    int rc = -1;
    // the link shapes x (shared-reciprocal division | plain) x (compact boxes | full box records)
#define RT_LINK4(BLOCK, OPT)                                                                              \
    (a.fastdiv ? (a.box_all_cmp ? RT_KERNEL(true, true, BLOCK, false, (OPT) | RT_OPT_FD | RT_OPT_BOXC)        \
                                : RT_KERNEL(true, true, BLOCK, false, (OPT) | RT_OPT_FD))                     \
               : (a.box_all_cmp ? RT_KERNEL(true, true, BLOCK, false, (OPT) | RT_OPT_BOXC)                    \
                                : RT_KERNEL(true, true, BLOCK, false, (OPT))))
    // ... and, for a scene whose leaves are mostly sphere pairs (a.sph_pairs), without compact boxes
#define RT_LINK4S(BLOCK, OPT)                                                                                 \
    ((a.sph_pairs && !a.box_all_cmp)                                                                         \
         ? (a.fastdiv ? RT_KERNEL(true, true, BLOCK, false, (OPT) | RT_OPT_FD | RT_OPT_SPAIR)                \
                      : RT_KERNEL(true, true, BLOCK, false, (OPT) | RT_OPT_SPAIR))                          \
         : RT_LINK4(BLOCK, OPT))
    switch (shape) {
        case LINK_LDS:
            if (!pool) {
#ifdef RT_AB_KNOBS
                rc = RT_KERNEL(true, true, 512, false, 0);
#endif
            } else if (a.block == 1024) {
                rc = RT_LINK4S(1024, SM);
            } else {
                rc = RT_LINK4S(512, SM);
            }
            break;
        case LINK_TL: rc = RT_LINK4(1024, SM | RT_OPT_TL); break;
#ifdef RT_AB_KNOBS
        case FAST_LDS: rc = RT_KERNEL(false, true, 512, true, 0); break;
        case FAST_GLOBAL: rc = RT_KERNEL(false, false, 512, true, 0); break;
        case META_LDS: rc = RT_KERNEL(false, true, 512, false, 0); break;
        case META_GLOBAL: rc = RT_KERNEL(false, false, 512, false, 0); break;
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
