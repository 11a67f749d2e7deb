// rt_kernel.hip — the MI355X (gfx950) path-tracing kernel.
//
// Semantics: the reference's per-invocation compute shader
// (S/raytrace/compute.glsl:345-358 + S/utils/*.glsl), bit-exact with the CPU
// oracle given the shared GLSL built-in definitions (include/rt/rt_glsl.h) and
// -ffp-contract=off.  Structure (MI355X-first, every change value-preserving):
//   * one work-item per pixel, 16x16 workgroups (4 waves of 16x4 pixels), and
//     ALL frames of a launch looped in-register: the RGBA32F running mean
//     (compute.glsl:355) is applied per frame exactly, but the image is read
//     and written once per launch instead of once per frame;
//   * stackless traversal of a threaded BVH (rt_dnode) that visits the
//     reference's node sequence (stack pops, right child first) without the
//     int stack[64] the GLSL keeps in scratch;
//   * per-ray constants hoisted: 1/dir per axis and dot(dir,dir) (identical
//     values, computed once instead of per node / per sphere);
//   * deferred shading: set_material_properties (compute.glsl:197-224) is
//     resolved once for the final closest hit, and texture_color (pure, no
//     rand()) only when the bounce actually uses the attenuation;
//   * sphere uv (acos/atan2) only when an image texture will read it.
// rand() consumption order is identical to the reference.
#include <hip/hip_runtime.h>

#include "rt/rt_glsl.h"
#include "rt_device.h"

namespace {

typedef rt_kernel_args KP;

struct Rng {
    float rf, px, py;
};

// random.glsl:2-7
__device__ __forceinline__ float rnd(Rng& g) {
    g.rf += 0.001f;
    v2 co;
    co.x = g.px + g.rf;
    co.y = g.py + g.rf;
    v2 k = {12.9898f, 78.233f};
    return g_fract(g_sin(g_dot2(co, k)) * 43758.5453123f);
}

struct HitRec {
    float t;
    v3 p, normal;
    bool front;
};

// Source of hit_record.uv (compute.glsl:62): last successful sphere or quad hit.
struct UvSrc {
    int kind;   // 0 none, 1 sphere (idx, p), 2 quad (a, b)
    int idx;
    v3 p;
    v2 ab;
};

__device__ __forceinline__ v3 f3(float4 v) { return mk3(v.x, v.y, v.z); }

// ------------------------------------------------------------- primitives
// hitting.glsl:17-47 — root only.  Callers that need the surface compute
// p = o + d*t, then (deferred to the final closest hit) the outward normal.
__device__ __forceinline__ bool sphere_t(const float4* __restrict__ sp, float time, v3 o, v3 d, float a, float tmin,
                                         float tmax, float& t) {
    float4 A = sp[0], B = sp[1];
    v3 center = add3(f3(A), scale3(f3(B), time));
    v3 oc = sub3(o, center);
    float half_b = g_dot(oc, d);
    float c = g_dot(oc, oc) - B.w * B.w;
    float disc = half_b * half_b - a * c;
    if (disc < 0.0f) return false;
    float sq = sqrtf(disc);
    float root = (-half_b - sq) / a;
    if (!(tmin < root && root < tmax)) {
        root = (-half_b + sq) / a;
        if (!(tmin < root && root < tmax)) return false;
    }
    t = root;
    return true;
}

// the rest of hit_sphere (hitting.glsl:39-42) for a hit at rec.p
__device__ __forceinline__ void sphere_surface(const float4* __restrict__ sp, float time, v3 d, HitRec& rec) {
    float4 A = sp[0], B = sp[1];
    v3 center = add3(f3(A), scale3(f3(B), time));
    v3 on = divs3(sub3(rec.p, center), B.w);
    rec.front = g_dot(d, on) < 0.0f;
    rec.normal = rec.front ? on : neg3(on);
}

// hitting.glsl:90-133
__device__ __forceinline__ bool quad_hit(const float4* __restrict__ q, v3 o, v3 d, float tmin, float tmax,
                                         HitRec& rec, v2& ab) {
    float4 Q0 = q[0];
    v3 n = f3(Q0);
    float denom = g_dot(n, d);
    if (fabsf(denom) < 1e-8f) return false;
    float t = (Q0.w - g_dot(n, o)) / denom;
    if (!(tmin <= t && t <= tmax)) return false;
    float4 Q1 = q[1], Q2 = q[2], Q3 = q[3];
    v3 inter = add3(o, scale3(d, t));
    v3 ph = sub3(inter, f3(Q1));
    v3 u = f3(Q2), v = f3(Q3);
    float delta, alpha, beta;
    if ((delta = u.x * v.y - u.y * v.x) != 0.0f) {
        alpha = (ph.x * v.y - ph.y * v.x) / delta;
        beta = (ph.y * u.x - ph.x * u.y) / delta;
    } else if ((delta = u.x * v.z - u.z * v.x) != 0.0f) {
        alpha = (ph.x * v.z - ph.z * v.x) / delta;
        beta = (ph.z * u.x - ph.x * u.z) / delta;
    } else {
        delta = u.y * v.z - u.z * v.y;
        alpha = (ph.y * v.z - ph.z * v.y) / delta;
        beta = (ph.z * u.y - ph.y * u.z) / delta;
    }
    if (!(0.0f <= alpha && alpha <= 1.0f) || !(0.0f <= beta && beta <= 1.0f)) return false;
    ab.x = alpha;
    ab.y = beta;
    rec.t = t;
    rec.p = inter;
    rec.front = g_dot(d, n) < 0.0f;
    rec.normal = rec.front ? n : neg3(n);
    return true;
}

// hitting.glsl:135-146
__device__ __forceinline__ bool box_hit(const float4* __restrict__ b, v3 o, v3 d, float tmin, float tmax, HitRec& rec,
                                        v2& ab) {
    bool has = false;
    for (int i = 0; i < 6; i++) {
        if (quad_hit(b + 5 * i, o, d, tmin, tmax, rec, ab)) {
            tmax = rec.t;
            has = true;
        }
    }
    return has;
}

// hitting.glsl:148-160 (the medium only reads rec.t of its boundary hits)
__device__ __forceinline__ bool boundary_t(const KP& P, int idx, int type, v3 o, v3 d, float a, float time, float tmin, float tmax,
                           float& t) {
    v2 ab;
    HitRec r;
    if (type == RT_MODEL_SPHERE)
        return sphere_t(reinterpret_cast<const float4*>(P.spheres + idx), time, o, d, a, tmin, tmax, t);
    bool h = false;
    if (type == RT_MODEL_QUAD) h = quad_hit(reinterpret_cast<const float4*>(P.quads + idx), o, d, tmin, tmax, r, ab);
    else if (type == RT_MODEL_BOX) h = box_hit(reinterpret_cast<const float4*>(P.boxes + idx), o, d, tmin, tmax, r, ab);
    if (h) t = r.t;
    return h;
}

// hitting.glsl:162-193
__device__ __forceinline__ bool medium_hit(const KP& P, int idx, v3 o, v3 d, float a, float time, float tmin, float tmax, Rng& g,
                           HitRec& rec) {
    const rt_medium m = P.media[idx];
    float t1, t2;
    if (!boundary_t(P, m.boundary_idx, m.boundary_type, o, d, a, time, -RT_INFINITY, RT_INFINITY, t1)) return false;
    if (!boundary_t(P, m.boundary_idx, m.boundary_type, o, d, a, time, t1 + 0.0001f, RT_INFINITY, t2)) return false;
    if (t1 < tmin) t1 = tmin;
    if (t2 > tmax) t2 = tmax;
    if (t1 >= t2) return false;
    if (t1 < 0.0f) t1 = 0.0f;
    float len = sqrtf(a);   // length(ray.dir); a == dot(dir, dir)
    float inside = (t2 - t1) * len;
    float hd = m.neg_inv_density * g_log(rnd(g));
    if (hd > inside) return false;
    rec.t = t1 + hd / len;
    rec.p = add3(o, scale3(d, rec.t));
    rec.normal = mk3(1.0f, 0.0f, 0.0f);
    rec.front = true;
    return true;
}

// hitting.glsl:55-76 for one axis (branch-free; same assignments)
__device__ __forceinline__ void slab(float mn, float mx, float o, float inv, float& lo, float& hi) {
    float t0 = (mn - o) * inv;
    float t1 = (mx - o) * inv;
    bool ord = t0 < t1;
    float a = ord ? t0 : t1;
    float b = ord ? t1 : t0;
    lo = (a > lo) ? a : lo;
    hi = (b < hi) ? b : hi;
}

// Test the two prims of a leaf (compute.glsl:247-256), left then right.
__device__ __forceinline__ void leaf_prims(const KP& P, uint32_t meta, uint32_t prims, v3 o, v3 d, float a, float time,
                                           float tmin, float& tmax, Rng& g, HitRec& rec, int& htype, int& hidx,
                                           UvSrc& uvs, bool& has) {
#pragma unroll
    for (int s = 0; s < 2; s++) {
        int ty = (int)((meta >> (16 + 4 * s)) & 0xFu);
        int ix = (int)((prims >> (16 * s)) & 0xFFFFu);
        if (ty == RT_MODEL_SPHERE) {
            float t;
            if (sphere_t(reinterpret_cast<const float4*>(P.spheres + ix), time, o, d, a, tmin, tmax, t)) {
                has = true; tmax = t; htype = ty; hidx = ix;
                rec.t = t;
                rec.p = add3(o, scale3(d, t));
                uvs.kind = 1; uvs.idx = ix; uvs.p = rec.p;
            }
        } else if (ty == RT_MODEL_QUAD) {
            v2 ab;
            if (quad_hit(reinterpret_cast<const float4*>(P.quads + ix), o, d, tmin, tmax, rec, ab)) {
                has = true; tmax = rec.t; htype = ty; hidx = ix;
                uvs.kind = 2; uvs.ab = ab;
            }
        } else if (ty == RT_MODEL_BOX) {
            v2 ab;
            if (box_hit(reinterpret_cast<const float4*>(P.boxes + ix), o, d, tmin, tmax, rec, ab)) {
                has = true; tmax = rec.t; htype = ty; hidx = ix;
                uvs.kind = 2; uvs.ab = ab;
            }
        } else if (ty == RT_MODEL_CONSTANT_MEDIUM) {
            if (medium_hit(P, ix, o, d, a, time, tmin, tmax, g, rec)) {
                has = true; tmax = rec.t; htype = ty; hidx = ix;
            }
        }
    }
}

// compute.glsl:226-266 over the threaded BVH.  The node sequence of every lane
// is the reference's; only how a wave interleaves its lanes differs:
//   WHILE_WHILE: lanes advance through inner/missed nodes until each holds a
//                hit leaf (or is done), then leaves are tested together;
//   else       : one node per iteration, leaf tests inline (if-if).
template <bool WHILE_WHILE>
__device__ __forceinline__ bool trace(const KP& P, v3 o, v3 d, float time, Rng& g, HitRec& rec, int& htype, int& hidx, UvSrc& uvs) {
    if (P.n_nodes == 0) return false;
    float tmin = 0.001f, tmax = RT_INFINITY;
    v3 inv = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    float a = g_dot(d, d);
    bool has = false;
    const float4* __restrict__ nodes = reinterpret_cast<const float4*>(P.nodes);
    uint32_t i = 0;
    if (WHILE_WHILE) {
        for (;;) {
            uint32_t meta = 0, prims = 0;
            bool leaf = false;
            while (i != RT_NODE_END) {
                float4 n0 = nodes[2 * i], n1 = nodes[2 * i + 1];
                meta = __float_as_uint(n1.z);
                prims = __float_as_uint(n1.w);
                float lo = tmin, hi = tmax;
                slab(n0.x, n0.y, o.x, inv.x, lo, hi);
                slab(n0.z, n0.w, o.y, inv.y, lo, hi);
                slab(n1.x, n1.y, o.z, inv.z, lo, hi);
                if (hi <= lo) { i = meta & 0xFFFFu; continue; }
                if (((meta >> 16) & 0xFu) == 0) { i = i + 1; continue; }
                leaf = true;
                break;
            }
            if (!leaf) break;
            leaf_prims(P, meta, prims, o, d, a, time, tmin, tmax, g, rec, htype, hidx, uvs, has);
            i = meta & 0xFFFFu;
        }
    } else {
        while (i != RT_NODE_END) {
            float4 n0 = nodes[2 * i], n1 = nodes[2 * i + 1];
            uint32_t meta = __float_as_uint(n1.z);
            uint32_t prims = __float_as_uint(n1.w);
            float lo = tmin, hi = tmax;
            slab(n0.x, n0.y, o.x, inv.x, lo, hi);
            slab(n0.z, n0.w, o.y, inv.y, lo, hi);
            slab(n1.x, n1.y, o.z, inv.z, lo, hi);
            uint32_t skip = meta & 0xFFFFu;
            if (hi <= lo) { i = skip; continue; }
            if (((meta >> 16) & 0xFu) == 0) { i = i + 1; continue; }
            leaf_prims(P, meta, prims, o, d, a, time, tmin, tmax, g, rec, htype, hidx, uvs, has);
            i = skip;
        }
    }
    if (has && htype == RT_MODEL_SPHERE)
        sphere_surface(reinterpret_cast<const float4*>(P.spheres + hidx), time, d, rec);
    return has;
}

// ---------------------------------------------------------------- textures
__device__ __forceinline__ void texel(const rt_dtex& T, int x, int y, float out[3]) {
    out[0] = out[1] = out[2] = 0.0f;
    if (!T.data || x < 0 || y < 0 || x >= T.w || y >= T.h) return;
    int i = y * T.w + x;
    if (T.is_float) {
        out[0] = reinterpret_cast<const float*>(T.data)[i];
    } else {
        uint32_t c = reinterpret_cast<const uint32_t*>(T.data)[i];
        out[0] = rt_unorm8(c & 0xFFu);
        out[1] = rt_unorm8((c >> 8) & 0xFFu);
        out[2] = rt_unorm8((c >> 16) & 0xFFu);
    }
}
__device__ __forceinline__ float texel_r(const rt_dtex& T, int x, int y) {
    float t[3];
    texel(T, x, y, t);
    return t[0];
}

// texture.glsl:38-77 (Perlin table: 6 x 256 R32F, row-major width 6)
__device__ __forceinline__ float perlin_noise(const rt_dtex& T, v3 p) {
    float u = p.x - floorf(p.x);
    float v = p.y - floorf(p.y);
    float w = p.z - floorf(p.z);
    u = u * u * (3.0f - 2.0f * u);
    v = v * v * (3.0f - 2.0f * v);
    w = w * w * (3.0f - 2.0f * w);
    int i = rt_f2i(floorf(p.x));
    int j = rt_f2i(floorf(p.y));
    int k = rt_f2i(floorf(p.z));
    // perlin_interp (texture.glsl:19-36), double Hermite as in the reference (Q6)
    float uu = u * u * (3.0f - 2.0f * u);
    float vv = v * v * (3.0f - 2.0f * v);
    float ww = w * w * (3.0f - 2.0f * w);
    float accum = 0.0f;
#pragma unroll
    for (int di = 0; di < 2; di++) {
        int px = rt_f2i(texel_r(T, 3, (i + di) & 255));
#pragma unroll
        for (int dj = 0; dj < 2; dj++) {
            int py = rt_f2i(texel_r(T, 4, (j + dj) & 255));
#pragma unroll
            for (int dk = 0; dk < 2; dk++) {
                int pz = rt_f2i(texel_r(T, 5, (k + dk) & 255));
                int idx = px ^ py ^ pz;
                v3 c = mk3(texel_r(T, 0, idx), texel_r(T, 1, idx), texel_r(T, 2, idx));
                v3 wv = mk3(u - (float)di, v - (float)dj, w - (float)dk);
                float fi = (float)di, fj = (float)dj, fk = (float)dk;
                accum += (fi * uu + (1.0f - fi) * (1.0f - uu)) * (fj * vv + (1.0f - fj) * (1.0f - vv)) *
                         (fk * ww + (1.0f - fk) * (1.0f - ww)) * g_dot(c, wv);
            }
        }
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
    if (s.kind == 2) return s.ab;
    if (s.kind == 1) {
        const float4* sp = reinterpret_cast<const float4*>(P.spheres + s.idx);
        float4 A = sp[0], B = sp[1];
        v3 center = add3(f3(A), scale3(f3(B), time));
        return sphere_uv(sub3(s.p, center));
    }
    v2 z = {0.0f, 0.0f};
    return z;
}

// texture.glsl:112-132
__device__ __forceinline__ v3 texture_color(const KP& P, v3 p, int id, const UvSrc& uvs, float time) {
    int detail_i = id & 0xFFF;
    int index = (id >> 12) & 0xFFFF;
    int type = (id >> 28) & 0xF;
    const rt_dtex& T = P.tex[index & 7];
    float t[3];
    if (type == RT_TEXTYPE_SOLID) {
        texel(T, detail_i, 0, t);
        return mk3(t[0], t[1], t[2]);
    }
    if (type == RT_TEXTYPE_CHECKER) {   // :6-17
        int pix = detail_i * 3;
        float scale = texel_r(T, pix + 2, 0);
        float inv_scale = 1.0f / scale;
        v3 q = scale3(p, inv_scale);
        int s = rt_f2i(q.x) + rt_f2i(q.y) + rt_f2i(q.z);
        texel(T, (s % 2 == 0) ? pix : pix + 1, 0, t);
        return mk3(t[0], t[1], t[2]);
    }
    if (type == RT_TEXTYPE_PERLIN) {    // :79-94
        float scale = ((float)detail_i / 4095.0f) * 100.0f;
        float accum = 0.0f, weight = 1.0f;
        v3 q = p;
        for (int o = 0; o < 7; o++) {
            accum += weight * perlin_noise(T, q);
            weight *= 0.5f;
            q = scale3(q, 2.0f);
        }
        float s = 1.0f + g_sin(scale * p.z + 10.0f * fabsf(accum));
        return mk3s(0.5f * s);
    }
    if (type == RT_TEXTYPE_IMAGE) {     // texture2D: GL_LINEAR, CLAMP_TO_EDGE
        if (!T.data || T.w <= 0 || T.h <= 0) return mk3s(0.0f);
        v2 uv = resolve_uv(P, uvs, time);
        float x = uv.x * (float)T.w - 0.5f;
        float y = uv.y * (float)T.h - 0.5f;
        float fx = floorf(x), fy = floorf(y);
        float a = x - fx, b = y - fy;
        int x0 = rt_f2i(fx), y0 = rt_f2i(fy);
        int x1 = x0 >= T.w - 1 ? T.w - 1 : x0 + 1;
        int y1 = y0 >= T.h - 1 ? T.h - 1 : y0 + 1;
        x1 = x1 < 0 ? 0 : x1; y1 = y1 < 0 ? 0 : y1;
        x0 = x0 < 0 ? 0 : (x0 > T.w - 1 ? T.w - 1 : x0);
        y0 = y0 < 0 ? 0 : (y0 > T.h - 1 ? T.h - 1 : y0);
        float t00[3], t10[3], t01[3], t11[3];
        texel(T, x0, y0, t00); texel(T, x1, y0, t10); texel(T, x0, y1, t01); texel(T, x1, y1, t11);
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
__device__ __forceinline__ v3 rand_unit_vec(Rng& g) {
    v3 p;
    for (;;) {
        float x = -1.0f + rnd(g) * 2.0f;
        float y = -1.0f + rnd(g) * 2.0f;
        float z = -1.0f + rnd(g) * 2.0f;
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
    float4 A = sp[0], B = sp[1];
    v3 pc = sub3(f3(A), o);
    float d2 = g_dot(pc, pc);
    float ctm = sqrtf(1.0f - B.w * B.w / d2);
    float solid = 2.0f * RT_PI * (1.0f - ctm);
    return 1.0f / solid;
}

// pdf.glsl:41-51
__device__ __forceinline__ float quad_light_pdf(const KP& P, int idx, v3 o, v3 d) {
    const float4* q = reinterpret_cast<const float4*>(P.quads + idx);
    HitRec r;
    v2 ab;
    if (!quad_hit(q, o, d, 0.001f, RT_INFINITY, r, ab)) return 0.0f;
    float d2 = r.t * r.t * g_dot(d, d);
    float cosine = fabsf(g_dot(d, r.normal) / g_length(d));
    return d2 / (cosine * q[3].w);
}

// pdf.glsl:58-81
__device__ __forceinline__ float lights_pdf_value(const KP& P, v3 o, v3 d, float time) {
    float weight = 1.0f / (float)P.lights_count;
    float sum = 0.0f;
    for (int i = 0; i < P.lights_count; i++) {
        int packed = P.lights[i];
        int type = (packed >> 16) & 0xFFFF, idx = packed & 0xFFFF;
        float pdf = 0.0f;
        if (type == RT_MODEL_SPHERE) pdf = sphere_light_pdf(P, idx, o, d, time);
        else if (type == RT_MODEL_QUAD) pdf = quad_light_pdf(P, idx, o, d);
        sum += weight * pdf;
    }
    return sum;
}

// pdf.glsl:83-96 (+ random.glsl:71-80, pdf.glsl:26-30, :53-56); no light -> vec3(0) (Q1)
__device__ __forceinline__ v3 lights_random(const KP& P, v3 o, Rng& g) {
    float r = 0.0f + rnd(g) * ((float)(P.lights_count - 1 + 1) - 0.0f);
    int li = rt_f2i(floorf(r));
    if (li < 0 || li >= P.lights_count) return mk3s(0.0f);
    int packed = P.lights[li];
    int type = (packed >> 16) & 0xFFFF, idx = packed & 0xFFFF;
    if (type == RT_MODEL_SPHERE) {
        const float4* sp = reinterpret_cast<const float4*>(P.spheres + idx);
        float4 A = sp[0], B = sp[1];
        v3 dir = sub3(f3(A), o);
        float d2 = g_dot(dir, dir);
        float r1 = rnd(g);
        float r2 = rnd(g);
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
        float4 Q1 = q[1], Q2 = q[2], Q3 = q[3];
        float r1 = rnd(g);
        v3 p = add3(f3(Q1), scale3(f3(Q2), r1));
        float r2 = rnd(g);
        p = add3(p, scale3(f3(Q3), r2));
        return sub3(p, o);
    }
    return mk3s(0.0f);
}

// ------------------------------------------------------------- ray_color
// Per-lane path state carried between bounces (ray_color's locals).
struct Path {
    v3 o, d, acc;
    float time;
    Rng g;
    HitRec rec;
    UvSrc uvs;
    int depth;
};

// One iteration of ray_color's loop (compute.glsl:304-340).  Returns true when
// the path ended, with its color in `result`.
template <bool WW>
__device__ __forceinline__ bool bounce(const KP& P, Path& S, v3& result) {
    if (S.depth >= P.max_depth) {   // loop exhausted: final_color stays vec3(0)
        result = mk3s(0.0f);
        return true;
    }
    S.depth++;
    int htype = 0, hidx = 0;
    v3 d = S.d;
    bool dir_zero = (d.x == 0.0f) && (d.y == 0.0f) && (d.z == 0.0f);
    // A zero direction (Q1 isotropic corner) can hit nothing and consumes no rand().
    if (dir_zero || !trace<WW>(P, S.o, d, S.time, S.g, S.rec, htype, hidx, S.uvs)) {
        result = mul3(S.acc, mk3(P.background[0], P.background[1], P.background[2]));
        return true;
    }
    const HitRec& rec = S.rec;
    // set_material_properties for the closest hit (compute.glsl:197-224)
    int material, tex_id;
    v3 emis = mk3s(0.0f);
    if (htype == RT_MODEL_SPHERE) {
        const float4* sp = reinterpret_cast<const float4*>(P.spheres + hidx);
        float4 A = sp[0], C = sp[2];
        material = __float_as_int(C.w);
        tex_id = __float_as_int(A.w);
        if (rec.front) emis = f3(C);
    } else if (htype == RT_MODEL_CONSTANT_MEDIUM) {
        material = P.media[hidx].phase_material;
        tex_id = P.media[hidx].texture_id;
    } else {
        const float4* q = (htype == RT_MODEL_QUAD) ? reinterpret_cast<const float4*>(P.quads + hidx)
                                                  : reinterpret_cast<const float4*>(P.boxes + hidx);
        material = __float_as_int(q[1].w);
        tex_id = __float_as_int(q[2].w);
        if (rec.front) emis = f3(q[4]);
    }
    // scatter (scatter.glsl:43-98)
    int mid = (material >> 16) & 0xFFFF;
    bool skip_pdf = false, should = false;
    if (mid == RT_MAT_DIFFUSE_LIGHT) {
        result = mul3(S.acc, emis);
        return true;
    }
    Rng& g = S.g;
    if (mid == RT_MAT_LAMBERTIAN) {
        float r1 = rnd(g);
        float r2 = rnd(g);
        float phi = 2.0f * RT_PI * r1;
        float s, c;
        g_sincos(phi, &s, &c);
        v3 cd = mk3(c * sqrtf(r2), s * sqrtf(r2), sqrtf(1.0f - r2));
        d = transform_onb(cd, rec.normal);
        should = true;
    } else if (mid == RT_MAT_METAL) {
        float fuzz = (float)(material & 0xFFFF) / 65535.0f;
        d = g_reflect(d, rec.normal);
        v3 n = g_normalize(d);
        d = add3(n, scale3(rand_unit_vec(g), fuzz));
        should = g_dot(d, rec.normal) > 0.0f;
        skip_pdf = true;
    } else if (mid == RT_MAT_DIELECTRIC) {
        float nior = (float)(material & 0xFFFF) / 65535.0f;
        float eta = g_mix(1.0f, 2.5f, nior);
        if (rec.front) eta = 1.0f / eta;
        d = g_normalize(d);
        float cos_t = g_min(g_dot(neg3(d), rec.normal), 1.0f);
        float sin_t = sqrtf(1.0f - cos_t * cos_t);
        bool refl = eta * sin_t > 1.0f;
        if (!refl) {
            float r0 = (1.0f - eta) / (1.0f + eta);
            r0 = r0 * r0;
            float rf = r0 + (1.0f - r0) * g_pow5(1.0f - cos_t);
            refl = rf > rnd(g);
        }
        d = refl ? g_reflect(d, rec.normal) : g_refract(d, rec.normal, eta);
        should = true;
        skip_pdf = true;
    } else if (mid == RT_MAT_ISOTROPIC) {
        d = rand_unit_vec(g);
        should = true;
    }
    if ((fabsf(d.x) < 1e-8f) && (fabsf(d.y) < 1e-8f) && (fabsf(d.z) < 1e-8f)) d = rec.normal;
    if (!should) {
        result = mul3(S.acc, emis);
        return true;
    }
    S.o = rec.p;
    if (skip_pdf) {
        S.acc = mul3(S.acc, texture_color(P, rec.p, tex_id, S.uvs, S.time));
        S.d = d;
        return false;
    }
    if (rnd(g) < 0.5f) d = lights_random(P, S.o, g);
    float lpdf = (P.lights_count > 0) ? lights_pdf_value(P, S.o, d, S.time) : 0.0f;
    float mpdf;
    if (mid == RT_MAT_LAMBERTIAN) mpdf = g_max(0.0f, g_normalize1(g_dot(d, rec.normal)) / RT_PI);
    else if (mid == RT_MAT_ISOTROPIC) mpdf = 1.0f / (4.0f * RT_PI);
    else mpdf = 0.0f;
    float pdf = 0.5f * lpdf + 0.5f * mpdf;
    if (pdf == 0.0f) {
        result = mul3(S.acc, emis);
        return true;
    }
    float spdf;
    if (mid == RT_MAT_LAMBERTIAN) spdf = g_max(0.0f, g_dot(rec.normal, g_normalize(d)) / RT_PI);
    else if (mid == RT_MAT_ISOTROPIC) spdf = 1.0f / (4.0f * RT_PI);
    else spdf = 0.0f;
    v3 att = texture_color(P, rec.p, tex_id, S.uvs, S.time);
    S.acc = mul3(S.acc, divs3(scale3(att, spdf), pdf));
    S.d = d;
    return false;
}

// Camera ray of frame `frame_count` (compute.glsl:345-350, random.glsl:19-30,82-100).
__device__ __forceinline__ void start_path(const KP& P, Path& S, int frame_count, float rf, float fx, float fy, v3 base) {
    const rt_camera_ubo& C = P.cam;
    v3 du = ld3(C.pixel_delta_u), dv = ld3(C.pixel_delta_v), cpos = ld3(C.camera_pos);
    Rng& g = S.g;
    g.rf = rf;
    g.px = fx;
    g.py = fy;
    S.time = rnd(g);
    float col = g_mod((float)frame_count, P.sqrt_spp);
    float layer = (float)frame_count / P.sqrt_spp;
    float base_x = (col + 0.5f) * P.recip_sqrt_spp;
    float base_y = (layer + 0.5f) * P.recip_sqrt_spp;
    float jx = (rnd(g) - 0.5f) * P.recip_sqrt_spp;
    float jy = (rnd(g) - 0.5f) * P.recip_sqrt_spp;
    float spx = base_x + jx - 0.5f;
    float spy = base_y + jy - 0.5f;
    v3 coord = add3(base, add3(scale3(du, spx), scale3(dv, spy)));
    v3 o = cpos;
    if (!(C.defocus_angle <= 0.0f)) {
        float dx, dy;
        for (;;) {
            dx = -1.0f + rnd(g) * 2.0f;
            dy = -1.0f + rnd(g) * 2.0f;
            v3 p = mk3(dx, dy, 0.0f);
            if (g_dot(p, p) < 1.0f) break;
        }
        o = add3(add3(cpos, scale3(ld3(C.defocus_disk_u), dx)), scale3(ld3(C.defocus_disk_v), dy));
    }
    S.o = o;
    S.d = sub3(coord, o);
    S.acc = mk3s(1.0f);
    S.depth = 0;
    S.rec.t = 0.0f; S.rec.p = mk3s(0.0f); S.rec.normal = mk3s(0.0f); S.rec.front = false;
    S.uvs.kind = 0; S.uvs.idx = 0; S.uvs.p = mk3s(0.0f); S.uvs.ab.x = 0.0f; S.uvs.ab.y = 0.0f;
}

// compute.glsl:345-358 for all frames of the launch.  Path regeneration: a lane
// whose path ended starts its next frame at once, so a wave never idles until
// its longest path of a frame is done; each pixel still runs its frames in order
// and applies the running mean per frame.
template <bool WW, int MINW>
__global__ void __launch_bounds__(256, MINW) render_kernel(const KP* __restrict__ Pp) {
    const KP& P = *Pp;
    int x = blockIdx.x * 16 + threadIdx.x;
    int lr = blockIdx.y * 16 + threadIdx.y;
    if (x >= P.width || lr >= P.local_rows) return;
    int gstripe = (lr / P.stripe_rows) * P.world + P.rank;
    int y = gstripe * P.stripe_rows + lr % P.stripe_rows;
    float4* px = reinterpret_cast<float4*>(P.image) + (size_t)lr * P.width + x;
    float4 prev = *px;
    const rt_camera_ubo& C = P.cam;
    float fx = (float)x, fy = (float)y;
    // get_norm_coord (compute.glsl:268-283) before its jitter term: per pixel
    v3 base = add3(add3(ld3(C.up_left), scale3(ld3(C.pixel_delta_u), fx)), scale3(ld3(C.pixel_delta_v), fy));
    Path S;
    int f = 0;
    bool fresh = true;
    for (;;) {
        if (fresh) {
            if (f >= P.n_frames) break;
            start_path(P, S, P.first_frame + f, P.rand_factors[f], fx, fy, base);
            fresh = false;
        }
        v3 cur;
        if (bounce<WW>(P, S, cur)) {
            int fc = P.first_frame + f;
            float n1 = (float)(fc - 1), n = (float)fc;
            prev.x = (prev.x * n1 + cur.x) / n;
            prev.y = (prev.y * n1 + cur.y) / n;
            prev.z = (prev.z * n1 + cur.z) / n;
            prev.w = 1.0f;
            f++;
            fresh = true;
        }
    }
    *px = prev;
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
        default: break;
    }
    out[i] = r;
}

}  // namespace

int rt_launch_render(const rt_kernel_args& a, rt_kernel_args* dargs, void* stream) {
    if (a.local_rows <= 0 || a.width <= 0 || a.n_frames <= 0) return 0;
    // Arguments live in device memory: the by-value kernarg struct would be copied
    // to scratch as soon as a non-inlined device function takes its address.
    // Same-stream ordering makes one slot per device safe to reuse per launch.
    if (hipMemcpyAsync(dargs, &a, sizeof(a), hipMemcpyHostToDevice, (hipStream_t)stream) != hipSuccess) return -1;
    dim3 block(16, 16);
    dim3 grid((a.width + 15) / 16, (a.local_rows + 15) / 16);
    // variant (A/B only): 0 while-while default occupancy, 1 if-if, 2/3 while-while
    // with >= 4 / >= 5 waves per SIMD, 4 if-if with >= 4 waves per SIMD.
    const rt_kernel_args* d = (const rt_kernel_args*)dargs;
    hipStream_t st = (hipStream_t)stream;
    switch (a.variant) {
        case 1: hipLaunchKernelGGL((render_kernel<false, 1>), grid, block, 0, st, d); break;
        case 2: hipLaunchKernelGGL((render_kernel<true, 4>), grid, block, 0, st, d); break;
        case 3: hipLaunchKernelGGL((render_kernel<true, 5>), grid, block, 0, st, d); break;
        case 4: hipLaunchKernelGGL((render_kernel<false, 4>), grid, block, 0, st, d); break;
        default: hipLaunchKernelGGL((render_kernel<true, 1>), grid, block, 0, st, d); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int rt_launch_eval_builtin(int fn, const float* dx, const float* dy, float* dout, int n, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(eval_builtin_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, fn, dx, dy, dout, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
