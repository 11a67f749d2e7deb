// scene_builder.cpp — C++ restatement of the reference's Java scene side:
// Scene.java (scenes 0-8), RaytraceModel.java (model lists, BVH build, std430
// packers), BVHNode/AABB/Sphere/Quad/Box/ConstantMedium/Camera.java,
// materials/{Material,Metal,...}.java, textures/{Texture,SolidTexture,...}.java, Color.java, Interval.java.
// Produces the exact bytes rt_upload_buffer/rt_upload_texture/rt_set_camera take.
#include "rt/rt_scene.h"
#include "rt/rt.h"
#include "rt/rt_types.h"
#include "java_compat.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace rts_detail {   // image_decode.cpp
int decode_image_file(const char* path, int* w, int* h, int* comps, std::vector<uint8_t>* px);
}

#ifndef RT_ASSET_DIR
#define RT_ASSET_DIR "assets"
#endif

namespace rtb {

static thread_local std::string g_err;
static int fail(int code, const std::string& msg) { g_err = msg; return code; }

// ------------------------------------------------------------ Interval/AABB
// Interval.java:3-41 (empty = [FLT_MAX, -FLT_MAX])
struct Interval {
    float min = 3.4028235e38f, max = -3.4028235e38f;
    float size() const { return max - min; }
    void set(float a, float b) { min = a; max = b; }
    void set_union(const Interval& a, const Interval& b) {
        min = std::min(a.min, b.min);
        max = std::max(a.max, b.max);
    }
    void expand(float delta) { float p = delta / 2; min = min - p; max = max + p; }
};

// AABB.java:9-66
struct AABB {
    Interval x, y, z;
    AABB() = default;
    AABB(const Vec3f& a, const Vec3f& b) {
        x.set(std::min(a.x, b.x), std::max(a.x, b.x));
        y.set(std::min(a.y, b.y), std::max(a.y, b.y));
        z.set(std::min(a.z, b.z), std::max(a.z, b.z));
        pad_to_minimums();
    }
    static AABB join(const AABB& a, const AABB& b) {
        AABB r; r.x.set_union(a.x, b.x); r.y.set_union(a.y, b.y); r.z.set_union(a.z, b.z); return r;
    }
    const Interval& axis(int n) const { return n == 1 ? y : (n == 2 ? z : x); }
    int longest_axis() const {
        if (x.size() > y.size()) return x.size() > z.size() ? 0 : 2;
        return y.size() > z.size() ? 1 : 2;
    }
    void pad_to_minimums() {
        const float delta = 0.001f;
        if (x.size() < delta) x.expand(delta);
        if (y.size() < delta) y.expand(delta);
        if (z.size() < delta) z.expand(delta);
    }
};

// ---------------------------------------------------------------- materials
// Material.java:34-44, Metal.java:28-35, Dielectric.java:20-29, DiffuseLight.java
struct Material {
    int id = RT_MAT_LAMBERTIAN;
    int texture_packed = 0;
    float fuzz = 0, ior = 1;
    Vec3f emit{0, 0, 0};
    int packed() const {
        int v = id << 16;
        if (id == RT_MAT_METAL) v |= java_f2i(fuzz * 65535.0f) & 0xFFFF;
        if (id == RT_MAT_DIELECTRIC) {
            float n = (ior - 1.0f) / (2.5f - 1.0f);
            v |= java_f2i(n * 65535.0f) & 0xFFFF;
        }
        return v;
    }
};

// ---------------------------------------------------------------- models
struct Model {
    int type = 0;            // RT_MODEL_*
    int index_in_list = 0;   // RaytraceModel.indexInList
    AABB bbox;
    Material mat;
    // sphere
    Vec3f center1, vec12; float radius = 0;
    // quad
    Vec3f q, u, v, normal; float d = 0, area = 0;
    // box
    Model* sides[6] = {};
    // medium
    Model* boundary = nullptr; float density = 0;
    // BVH node
    Model* left = nullptr; Model* right = nullptr;
};

// ---------------------------------------------------------------- textures
struct TexSlot {
    int kind = 0;           // RT_TEXTYPE_*
    int format = RT_TEX_RGB8;
    int w = 0, h = 0;
    std::vector<uint8_t> bytes;
    float perlin_scale = 0;
};

struct World;

// Scene state that the reference keeps in static fields (RaytraceModel,
// Texture.TEXTURES_IN_COMPUTE, SolidTexture/CheckerTexture lists).
struct World {
    std::vector<std::unique_ptr<Model>> pool;
    std::vector<Model*> all_models, spheres, quads, media, boxes, lights, bvh_nodes;
    std::vector<TexSlot> textures;
    int solid_slot = -1, checker_slot = -1;
    std::vector<AwtColor> solid_colors;
    std::vector<AwtColor> checker1, checker2;
    std::vector<float> checker_scales;
    int perlin_count = 0;
    uint64_t seed = 1;
    std::string asset_dir;
    std::string err;

    // camera (Camera.java:14-72)
    Vec3f look_from{0, 0, 0}, look_at{0, 0, -1}, vup{0, 1, 0};
    float vfov = 90, defocus_angle = 0, focus_dist = 10;
    Vec3f background{0, 0, 0};
    int img_w = 1, img_h = 1;
    float aspect = 1;
    rt_camera_ubo ubo{};

    Model* make() { pool.emplace_back(new Model()); return pool.back().get(); }

    // ---- Texture.getValue(type, index, int detail) (Texture.java:219-229)
    int tex_value(int type, int index, int detail) {
        return (type << 28) | (index << 12) | (detail & 0xFFF);
    }
    // Texture.getValue(type, index, float detail) (Texture.java:203-217)
    int tex_value_f(int type, int index, float detail) {
        int bits = java_f2i(detail * 4095);
        return (type << 28) | (index << 12) | (bits & 0xFFF);
    }
    // SolidTexture.init / registerColor (SolidTexture.java:26-45)
    void solid_init() {
        textures.push_back(TexSlot{});
        textures.back().kind = RT_TEXTYPE_SOLID;
        solid_slot = (int)textures.size() - 1;
    }
    int solid_register(const AwtColor& c) {
        solid_colors.push_back(c);
        return tex_value(RT_TEXTYPE_SOLID, solid_slot < 0 ? 0 : solid_slot, (int)solid_colors.size() - 1);
    }
    int solid_register(float r, float g, float b) { return solid_register(awt(r, g, b)); }
    AwtColor awt(float r, float g, float b) {
        if (!AwtColor::valid(r) || !AwtColor::valid(g) || !AwtColor::valid(b))
            throw std::runtime_error("Color parameter outside of expected range");
        AwtColor c; c.r = AwtColor::chan(r); c.g = AwtColor::chan(g); c.b = AwtColor::chan(b); return c;
    }
    // CheckerTexture.init / registerColor (CheckerTexture.java:23-44)
    void checker_init() {
        textures.push_back(TexSlot{});
        textures.back().kind = RT_TEXTYPE_CHECKER;
        checker_slot = (int)textures.size() - 1;
    }
    int checker_register(float r1, float g1, float b1, float r2, float g2, float b2, float scale) {
        // both colours are made (and may throw, as java.awt.Color does) before anything is registered
        const AwtColor a = awt(r1, g1, b1), b = awt(r2, g2, b2);
        checker1.push_back(a);
        checker2.push_back(b);
        checker_scales.push_back(scale);
        return tex_value(RT_TEXTYPE_CHECKER, checker_slot < 0 ? 0 : checker_slot, (int)checker1.size() - 1);
    }
    // PerlinNoiseTexture.create (PerlinNoiseTexture.java:59-107)
    int perlin_create(float scale) {
        JavaRandom rnd((int64_t)(seed + 2 + (uint64_t)perlin_count));
        perlin_count++;
        float vec[256][3];
        for (int i = 0; i < 256; i++) {
            vec[i][0] = rnd.next_float(-1, 1);
            vec[i][1] = rnd.next_float(-1, 1);
            vec[i][2] = rnd.next_float(-1, 1);
        }
        int perm[3][256];
        for (int a = 0; a < 3; a++) {
            for (int i = 0; i < 256; i++) perm[a][i] = i;
            // Collections.shuffle(list, rnd): for i=size..2: swap(i-1, nextInt(i))
            for (int i = 256; i > 1; i--) std::swap(perm[a][i - 1], perm[a][rnd.next_int(i)]);
        }
        TexSlot t;
        t.kind = RT_TEXTYPE_PERLIN; t.format = RT_TEX_R32F; t.w = 6; t.h = 256; t.perlin_scale = scale;
        t.bytes.resize(6 * 256 * 4);
        float* f = reinterpret_cast<float*>(t.bytes.data());
        for (int i = 0; i < 256; i++) {
            f[i * 6 + 0] = vec[i][0]; f[i * 6 + 1] = vec[i][1]; f[i * 6 + 2] = vec[i][2];
            f[i * 6 + 3] = (float)perm[0][i]; f[i * 6 + 4] = (float)perm[1][i]; f[i * 6 + 5] = (float)perm[2][i];
        }
        textures.push_back(std::move(t));
        int idx = (int)textures.size() - 1;
        // PerlinNoiseTexture.getDetail = scale/100 (float)
        return tex_value_f(RT_TEXTYPE_PERLIN, idx, scale / 100.0f);
    }
    // ImageTexture.create (ImageTexture.java:22-92): the file decoded as ImageIO + getRGB do it
    // (image_decode.cpp), then the loop's vertical flip and wrap shift.  A name without a '/'
    // A relative name is a resource of the asset directory (the reference's classpath
    // "textures/"), an absolute one a file; 3 components upload as GL_RGB, 4 as GL_RGBA.
    int image_create(const char* name, int shift_x, int shift_y) {
        std::string path = name[0] == '/' ? std::string(name) : asset_dir + "/" + name;
        int w = 0, h = 0, comps = 0;
        std::vector<uint8_t> src;
        rts_detail::decode_image_file(path.c_str(), &w, &h, &comps, &src);
        TexSlot t;
        t.kind = RT_TEXTYPE_IMAGE; t.format = comps == 4 ? RT_TEX_RGBA8 : RT_TEX_RGB8; t.w = w; t.h = h;
        t.bytes.resize(src.size());
        for (int y = 0; y < h; y++) {
            int sy = (h - 1 - (y - shift_y + h) % h);   // vertical flip + wrap shift
            for (int x = 0; x < w; x++) {
                int sx = (x - shift_x + w) % w;
                const uint8_t* p = &src[((size_t)sy * w + sx) * comps];
                uint8_t* q = &t.bytes[((size_t)y * w + x) * comps];
                for (int k = 0; k < comps; k++) q[k] = p[k];
            }
        }
        textures.push_back(std::move(t));
        return tex_value_f(RT_TEXTYPE_IMAGE, (int)textures.size() - 1, 0.0f);
    }
    void solid_put_data() {
        if (solid_slot < 0) return;
        TexSlot& t = textures[solid_slot];
        t.w = (int)solid_colors.size(); t.h = 1; t.format = RT_TEX_RGB8;
        t.bytes.clear();
        for (auto& c : solid_colors) { t.bytes.push_back((uint8_t)c.r); t.bytes.push_back((uint8_t)c.g); t.bytes.push_back((uint8_t)c.b); }
    }
    void checker_put_data() {
        if (checker_slot < 0) return;
        TexSlot& t = textures[checker_slot];
        t.w = (int)checker1.size() * 3; t.h = 1; t.format = RT_TEX_RGB8;
        t.bytes.clear();
        for (size_t i = 0; i < checker1.size(); i++) {
            const AwtColor &a = checker1[i], &b = checker2[i];
            t.bytes.push_back((uint8_t)a.r); t.bytes.push_back((uint8_t)a.g); t.bytes.push_back((uint8_t)a.b);
            t.bytes.push_back((uint8_t)b.r); t.bytes.push_back((uint8_t)b.g); t.bytes.push_back((uint8_t)b.b);
            t.bytes.push_back((uint8_t)(int8_t)java_f2i(checker_scales[i] * 255));  // (byte)(scale*255)
            t.bytes.push_back(0); t.bytes.push_back(0);
        }
    }

    // ---- materials
    Material lambertian(int tex) { Material m; m.id = RT_MAT_LAMBERTIAN; m.texture_packed = tex; return m; }
    Material metal(int tex, float fuzz) {
        if (fuzz < 0 || fuzz >= 1) throw std::invalid_argument("Fuzz value should always in range [0, 1).");
        Material m; m.id = RT_MAT_METAL; m.texture_packed = tex; m.fuzz = fuzz; return m;
    }
    Material dielectric(float ior) {
        Material m; m.id = RT_MAT_DIELECTRIC; m.texture_packed = solid_register(awt(1, 1, 1)); m.ior = ior; return m;
    }
    Material diffuse_light(float r, float g, float b) {
        Material m; m.id = RT_MAT_DIFFUSE_LIGHT; m.texture_packed = 0; m.emit = Vec3f(r, g, b); return m;
    }
    Material isotropic(int tex) { Material m; m.id = RT_MAT_ISOTROPIC; m.texture_packed = tex; return m; }

    // ---- models
    // Sphere.java:21-31
    Model* sphere(const Vec3f& c1, const Vec3f& c2, float r, const Material& m) {
        Model* s = make();
        s->type = RT_MODEL_SPHERE; s->mat = m; s->center1 = c1; s->vec12 = c2.sub(c1); s->radius = r;
        Vec3f rv(r);
        AABB b1(c1.sub(rv), c1.add(rv)), b2(c2.sub(rv), c2.add(rv));
        s->bbox = AABB::join(b1, b2);
        return s;
    }
    Model* sphere(const Vec3f& c, float r, const Material& m) { return sphere(c, c, r, m); }
    // Quad.java:23-41
    Model* quad(const Vec3f& q, const Vec3f& u, const Vec3f& v, const Material& m) {
        Model* s = make();
        s->type = RT_MODEL_QUAD; s->mat = m; s->q = q; s->u = u; s->v = v;
        Vec3f n = u.cross(v);
        s->area = n.length();
        s->normal = n.normalize();
        s->d = s->normal.dot(q);
        AABB d1(q, q.add(u).add(v)), d2(q.add(u), q.add(v));
        s->bbox = AABB::join(d1, d2);
        return s;
    }
    // Box.java:19-74
    Model* box(const Vec3f& a, const Vec3f& b, const Vec3f* translation, const Vec3f* rotation, const Material& m) {
        Model* s = make();
        s->type = RT_MODEL_BOX; s->mat = m;
        Vec3f mn(std::min(a.x, b.x), std::min(a.y, b.y), std::min(a.z, b.z));
        Vec3f mx(std::max(a.x, b.x), std::max(a.y, b.y), std::max(a.z, b.z));
        Vec3f dx(mx.x - mn.x, 0, 0), dy(0, mx.y - mn.y, 0), dz(0, 0, mx.z - mn.z);
        auto side = [&](Vec3f q, Vec3f u, Vec3f v) {
            if (rotation && translation) {
                Mat3f rm = Mat3f().rotate_x(rotation->x).rotate_y(rotation->y).rotate_z(rotation->z);
                q = rm.transform(q).add(*translation);
                u = rm.transform(u);
                v = rm.transform(v);
            }
            return quad(q, u, v, m);
        };
        s->sides[0] = side(Vec3f(mn.x, mn.y, mx.z), dx, dy);
        s->sides[1] = side(Vec3f(mx.x, mn.y, mx.z), dz.negate(), dy);
        s->sides[2] = side(Vec3f(mx.x, mn.y, mn.z), dx.negate(), dy);
        s->sides[3] = side(Vec3f(mn.x, mn.y, mn.z), dz, dy);
        s->sides[4] = side(Vec3f(mn.x, mx.y, mx.z), dx, dz.negate());
        s->sides[5] = side(Vec3f(mn.x, mn.y, mn.z), dx, dz);
        // Box.setBoundingBox: the loop's double increment leaves sides[4] U sides[5] (Q10)
        AABB bb;
        for (int i = 0; i < 6; i++) { bb = AABB::join(s->sides[i]->bbox, s->sides[i + 1]->bbox); i++; }
        s->bbox = bb;
        return s;
    }
    // ConstantMedium.java:12-20 (its constructor registers the boundary)
    Model* constant_medium(Model* boundary, float density, const Material& phase) {
        Model* s = make();
        s->type = RT_MODEL_CONSTANT_MEDIUM; s->mat = phase; s->boundary = boundary; s->density = density;
        add_model(boundary);
        s->bbox = boundary->bbox;
        return s;
    }
    // RaytraceModel.addModel (RaytraceModel.java:57-79)
    void add_model(Model* m) {
        switch (m->type) {
            case RT_MODEL_SPHERE: spheres.push_back(m); m->index_in_list = (int)spheres.size() - 1; break;
            case RT_MODEL_QUAD: quads.push_back(m); m->index_in_list = (int)quads.size() - 1; break;
            case RT_MODEL_BOX: boxes.push_back(m); m->index_in_list = (int)boxes.size() - 1; break;
            case RT_MODEL_CONSTANT_MEDIUM: {
                media.push_back(m); m->index_in_list = (int)media.size() - 1;
                auto it = std::find(all_models.begin(), all_models.end(), m->boundary);
                if (it != all_models.end()) all_models.erase(it);
                break;
            }
            default: throw std::runtime_error("Unknown model type.");
        }
        all_models.push_back(m);
    }
    void add_light(Model* m) { lights.push_back(m); }

    // BVHNode.java:13-45.  The Java comparator (boxCompare, :63-69) orders by
    // DESCENDING axis min and never returns 0; we sort with the equivalent
    // strict order stable on ties (TimSort's tie handling under an
    // inconsistent comparator is not reproduced).
    Model* bvh_build(std::vector<Model*>& objs, int start, int end) {
        Model* n = make();
        n->type = RT_MODEL_BVH_NODE;
        bvh_nodes.push_back(n);
        n->index_in_list = (int)bvh_nodes.size() - 1;
        AABB bb;
        for (int i = start; i < end; i++) bb = AABB::join(bb, objs[i]->bbox);
        n->bbox = bb;
        int axis = bb.longest_axis();
        int span = end - start;
        if (span == 1) {
            n->left = n->right = objs[start];
        } else if (span == 2) {
            n->left = objs[start]; n->right = objs[start + 1];
        } else {
            // a NaN bound (a degenerate model) sorts last: the reference's comparator is then
            // inconsistent (TimSort may throw), and std::stable_sort needs a strict weak order
            auto key = [axis](const Model* m) {
                const float v = m->bbox.axis(axis).min;
                return v != v ? -INFINITY : v;
            };
            std::stable_sort(objs.begin() + start, objs.begin() + end, [&key](const Model* a, const Model* b) {
                return key(a) > key(b);
            });
            int mid = start + span / 2;
            n->left = bvh_build(objs, start, mid);
            n->right = bvh_build(objs, mid, end);
        }
        return n;
    }

    // ---- camera (Camera.java:91-143)
    void set_image_size(int w, int h) { img_w = w; img_h = h; aspect = (float)w / (float)h; }
    void camera_calculate() {
        float theta = (float)to_radians((double)vfov);
        float h = (float)std::tan((double)(theta / 2.0f));
        float vh = 2.0f * h * focus_dist;
        float vw = vh * aspect;
        Vec3f w = look_from.sub(look_at).normalize();
        Vec3f u = vup.cross(w);   // not normalized, as in the reference
        Vec3f v = w.cross(u);
        Vec3f vu = u.mul(vw), vv = v.mul(-vh);
        Vec3f du = vu.div((float)img_w), dv = vv.div((float)img_h);
        Vec3f ul = look_from.sub(w.mul(focus_dist));
        ul = ul.sub(vu.div(2));
        ul = ul.sub(vv.div(2));
        float dr = (float)((double)focus_dist * std::tan(to_radians((double)(defocus_angle / 2))));
        Vec3f ddu = u.mul(dr), ddv = v.mul(dr);
        rt_camera_ubo c{};
        c.viewport_width = vw; c.viewport_height = vh; c.aspect_ratio = aspect; c.defocus_angle = defocus_angle;
        auto put = [](float* d, const Vec3f& s) { d[0] = s.x; d[1] = s.y; d[2] = s.z; };
        put(c.camera_pos, look_from); put(c.up_left, ul); put(c.pixel_delta_u, du); put(c.pixel_delta_v, dv);
        put(c.defocus_disk_u, ddu); put(c.defocus_disk_v, ddv);
        ubo = c;
    }
};

// ---------------------------------------------------------------- packers
static void put_vec(std::vector<uint8_t>& b, const Vec3f& v) {
    float f[3] = {v.x, v.y, v.z};
    b.insert(b.end(), (uint8_t*)f, (uint8_t*)f + 12);
}
static void put_f(std::vector<uint8_t>& b, float f) { b.insert(b.end(), (uint8_t*)&f, (uint8_t*)&f + 4); }
static void put_i(std::vector<uint8_t>& b, int32_t i) { b.insert(b.end(), (uint8_t*)&i, (uint8_t*)&i + 4); }

// Quad.putToBuffer (Quad.java:43-54)
static void pack_quad(std::vector<uint8_t>& b, const Model* q) {
    put_vec(b, q->normal); put_f(b, q->d); put_vec(b, q->q); put_i(b, q->mat.packed());
    put_vec(b, q->u); put_i(b, q->mat.texture_packed); put_vec(b, q->v); put_f(b, q->area);
    put_vec(b, q->mat.emit); put_f(b, 0.0f);
}

}  // namespace rtb

using namespace rtb;

struct rts_scene {
    int scene_id = 0;
    World world;
    std::vector<uint8_t> buf[6];
    rts_info info{};
    std::vector<Material> materials;   // custom scenes (rts_new): the builder's Material objects
    bool finished = false;
};

namespace rtb {

static int bvh_depth(const Model* n) {
    if (n->type != RT_MODEL_BVH_NODE) return 0;
    return 1 + std::max(bvh_depth(n->left), bvh_depth(n->right));
}

// RaytraceModel.putModelsToProgram (RaytraceModel.java:115-136)
static void put_models_to_program(rts_scene* s) {
    World& W = s->world;
    std::vector<uint8_t>& sp = s->buf[RT_BIND_SPHERES];
    for (Model* m : W.spheres) {  // Sphere.putToBuffer (Sphere.java:33-51)
        put_vec(sp, m->center1); put_i(sp, m->mat.texture_packed); put_vec(sp, m->vec12); put_f(sp, m->radius);
        put_vec(sp, m->mat.emit); put_i(sp, m->mat.packed());
    }
    for (Model* m : W.quads) pack_quad(s->buf[RT_BIND_QUADS], m);
    for (Model* m : W.boxes)
        for (int i = 0; i < 6; i++) pack_quad(s->buf[RT_BIND_BOXES], m->sides[i]);
    std::vector<uint8_t>& md = s->buf[RT_BIND_MEDIA];
    for (Model* m : W.media) {  // ConstantMedium.putToBuffer (:26-37)
        put_i(md, m->boundary->index_in_list); put_i(md, m->boundary->type);
        put_f(md, -1.0f / m->density); put_i(md, m->mat.packed()); put_i(md, m->mat.texture_packed);
    }
    std::vector<uint8_t>& lt = s->buf[RT_BIND_LIGHTS];
    put_i(lt, (int)W.lights.size());
    for (Model* m : W.lights) put_i(lt, (m->type << 16) | m->index_in_list);
    if (!W.all_models.empty()) {
        Model* root = W.bvh_build(W.all_models, 0, (int)W.all_models.size());
        s->info.bvh_depth = bvh_depth(root);
    }
    std::vector<uint8_t>& bn = s->buf[RT_BIND_BVH];
    for (Model* n : W.bvh_nodes) {  // BVHNode.putToBuffer (BVHNode.java:47-56)
        put_f(bn, n->bbox.x.min); put_f(bn, n->bbox.x.max); put_f(bn, n->bbox.y.min); put_f(bn, n->bbox.y.max);
        put_f(bn, n->bbox.z.min); put_f(bn, n->bbox.z.max);
        put_i(bn, (n->left->index_in_list << 16) | (n->left->type & 0xFFFF));
        put_i(bn, (n->right->index_in_list << 16) | (n->right->type & 0xFFFF));
    }
}

// ---------------------------------------------------------------- scenes
// Scene.java:43-105
static void scene_bouncing_spheres(World& W) {
    JavaRandom math_random((int64_t)W.seed);
    JavaRandom color_random((int64_t)(W.seed + 1));
    JavaRandom random((int64_t)(W.seed + 100));
    W.solid_init();
    W.checker_init();
    Material mat = W.lambertian(W.solid_register(0.5f, 0.5f, 0.5f));
    W.add_model(W.sphere(Vec3f(0, -1, 0), 0.5f, mat));
    Material ground = W.lambertian(W.checker_register(.2f, .3f, .1f, .9f, .9f, .9f, .32f));
    W.add_model(W.sphere(Vec3f(0, -1000, 0), 1000, ground));
    auto rand_color = [&]() { float r = color_random.next_float(); float g = color_random.next_float();
                              float b = color_random.next_float(); return Vec3f(r, g, b); };
    for (int a = -11; a < 11; a++) {
        for (int b = -11; b < 11; b++) {
            double choose = math_random.next_double();
            float cx = (float)((double)a + (double)0.9f * math_random.next_double());
            float cz = (float)((double)b + (double)0.9f * math_random.next_double());
            Vec3f center(cx, 0.2f, cz);
            if (center.sub(4, 0.2f, 0).length() > 0.9f) {
                if (choose < 0.8) {
                    Vec3f c1 = rand_color(), c2 = rand_color();
                    Vec3f alb(c1.x * c2.x, c1.y * c2.y, c1.z * c2.z);   // Color.mul
                    Material m = W.lambertian(W.solid_register(alb.x, alb.y, alb.z));
                    float dy = (float)(math_random.next_double() * (double)0.5f);
                    Vec3f center2 = center.add(Vec3f(0, dy, 0));
                    W.add_model(W.sphere(center, center2, 0.2f, m));
                } else if (choose < 0.95) {
                    float r = color_random.next_float(0.5f, 1), g = color_random.next_float(0.5f, 1),
                          bb = color_random.next_float(0.5f, 1);
                    float fuzz = random.next_float(0, 0.5f);
                    Material m = W.metal(W.solid_register(r, g, bb), fuzz);
                    W.add_model(W.sphere(center, 0.2f, m));
                } else {
                    Material m = W.dielectric(1.5f);
                    W.add_model(W.sphere(center, 0.2f, m));
                }
            }
        }
    }
    W.add_model(W.sphere(Vec3f(0, 1, 0), 1, W.dielectric(1.5f)));
    W.add_model(W.sphere(Vec3f(-4, 1, 0), 1, W.lambertian(W.solid_register(0.4f, 0.2f, 0.1f))));
    Material m3 = W.metal(W.solid_register(0.7f, 0.6f, 0.5f), 0);
    W.add_model(W.sphere(Vec3f(4, 1, 0), 1, m3));
    W.vfov = 20; W.look_from = Vec3f(13, 2, 3); W.look_at = Vec3f(0, 0, 0);
    W.defocus_angle = 0.6f; W.focus_dist = 10; W.background = Vec3f(0.70f, 0.80f, 1.00f);
}

// Scene.java:107-124
static void scene_checker_spheres(World& W) {
    W.checker_init();
    int c1 = W.checker_register(.2f, .3f, .1f, .9f, .9f, .9f, 0.32f);
    int c2 = W.checker_register(.5f, .2f, .1f, .9f, .9f, .9f, 0.32f);
    W.add_model(W.sphere(Vec3f(0, -10, 0), 10, W.lambertian(c1)));
    W.add_model(W.sphere(Vec3f(0, 10, 0), 10, W.lambertian(c2)));
    W.vfov = 20; W.look_from = Vec3f(13, 2, 3); W.look_at = Vec3f(0, 0, 0);
    W.defocus_angle = 0; W.background = Vec3f(0.70f, 0.80f, 1.00f);
}

// Scene.java:126-139
static void scene_earth(World& W) {
    int earth = W.image_create("earthmap.jpg", 0, 0);
    W.add_model(W.sphere(Vec3f(0, 0, 0), 2, W.lambertian(earth)));
    W.vfov = 20; W.look_from = Vec3f(0, 0, 12); W.look_at = Vec3f(0, 0, 0);
    W.defocus_angle = 0; W.background = Vec3f(0.70f, 0.80f, 1.00f);
}

// Scene.java:141-157
static void scene_perlin_spheres(World& W) {
    int p = W.perlin_create(4);
    W.add_model(W.sphere(Vec3f(0, -1000, 0), 1000, W.lambertian(p)));
    W.add_model(W.sphere(Vec3f(0, 2, 0), 2, W.lambertian(p)));
    W.vfov = 20; W.look_from = Vec3f(13, 2, 3); W.look_at = Vec3f(0, 0, 0);
    W.defocus_angle = 0; W.background = Vec3f(0.70f, 0.80f, 1.00f);
}

// Scene.java:159-182
static void scene_quads(World& W) {
    W.solid_init();
    Material red = W.lambertian(W.solid_register(1.0f, 0.2f, 0.2f));
    Material green = W.lambertian(W.solid_register(0.2f, 1.0f, 0.2f));
    Material blue = W.lambertian(W.solid_register(0.2f, 0.2f, 1.0f));
    Material orange = W.lambertian(W.solid_register(1.0f, 0.5f, 0.0f));
    Material teal = W.lambertian(W.solid_register(0.2f, 0.8f, 0.8f));
    W.add_model(W.quad(Vec3f(-3, -2, 5), Vec3f(0, 0, -4), Vec3f(0, 4, 0), red));
    W.add_model(W.quad(Vec3f(-2, -2, 0), Vec3f(4, 0, 0), Vec3f(0, 4, 0), green));
    W.add_model(W.quad(Vec3f(3, -2, 1), Vec3f(0, 0, 4), Vec3f(0, 4, 0), blue));
    W.add_model(W.quad(Vec3f(-2, 3, 1), Vec3f(4, 0, 0), Vec3f(0, 0, 4), orange));
    W.add_model(W.quad(Vec3f(-2, -3, 5), Vec3f(4, 0, 0), Vec3f(0, 0, -4), teal));
    W.vfov = 80; W.look_from = Vec3f(0, 0, 9); W.look_at = Vec3f(0, 0, 0);
    W.defocus_angle = 0; W.background = Vec3f(0.70f, 0.80f, 1.00f);
}

// Scene.java:184-210
static void scene_simple_light(World& W) {
    int p = W.perlin_create(4);
    W.add_model(W.sphere(Vec3f(0, -1000, 0), 1000, W.lambertian(p)));
    W.add_model(W.sphere(Vec3f(0, 2, 0), 2, W.lambertian(p)));
    Material light = W.diffuse_light(4, 4, 4);
    W.add_model(W.sphere(Vec3f(0, 7, 0), 2, light));
    W.add_model(W.quad(Vec3f(3, 1, -2), Vec3f(2, 0, 0), Vec3f(0, 2, 0), light));
    W.vfov = 20; W.look_from = Vec3f(26, 3, 6); W.look_at = Vec3f(0, 2, 0);
    W.defocus_angle = 0; W.background = Vec3f(0, 0, 0);
}

// Scene.java:212-249
static void scene_cornell_box(World& W) {
    W.solid_init();
    Material red = W.lambertian(W.solid_register(0.65f, 0.05f, 0.05f));
    Material white = W.lambertian(W.solid_register(0.73f, 0.73f, 0.73f));
    Material green = W.lambertian(W.solid_register(0.12f, 0.45f, 0.15f));
    Material light = W.diffuse_light(15, 15, 15);
    Model* light_quad = W.quad(Vec3f(343, 554, 332), Vec3f(-130, 0, 0), Vec3f(0, 0, -105), light);
    W.add_model(W.quad(Vec3f(555, 0, 0), Vec3f(0, 555, 0), Vec3f(0, 0, 555), green));
    W.add_model(W.quad(Vec3f(0, 0, 0), Vec3f(0, 555, 0), Vec3f(0, 0, 555), red));
    W.add_model(light_quad);
    W.add_light(light_quad);
    W.add_model(W.quad(Vec3f(0, 0, 0), Vec3f(555, 0, 0), Vec3f(0, 0, 555), white));
    W.add_model(W.quad(Vec3f(555, 555, 555), Vec3f(-555, 0, 0), Vec3f(0, 0, -555), white));
    W.add_model(W.quad(Vec3f(0, 0, 555), Vec3f(555, 0, 0), Vec3f(0, 555, 0), white));
    Vec3f t1(265, 0, 295), r1(0, (float)to_radians(15), 0);
    Model* box1 = W.box(Vec3f(0, 0, 0), Vec3f(165, 330, 165), &t1, &r1, white);
    Material glass = W.dielectric(1.5f);
    Model* glass_sphere = W.sphere(Vec3f(190, 90, 190), 90, glass);
    W.add_model(box1);
    W.add_model(glass_sphere);
    W.add_light(glass_sphere);
    W.vfov = 40; W.look_from = Vec3f(278, 278, -800); W.look_at = Vec3f(278, 278, 0);
    W.defocus_angle = 0; W.background = Vec3f(0, 0, 0);
}

// Scene.java:251-280
static void scene_cornell_smoke(World& W) {
    W.solid_init();
    Material red = W.lambertian(W.solid_register(0.65f, 0.05f, 0.05f));
    Material white = W.lambertian(W.solid_register(0.73f, 0.73f, 0.73f));
    Material green = W.lambertian(W.solid_register(0.12f, 0.45f, 0.15f));
    Material light = W.diffuse_light(7, 7, 7);
    W.add_model(W.quad(Vec3f(555, 0, 0), Vec3f(0, 555, 0), Vec3f(0, 0, 555), green));
    W.add_model(W.quad(Vec3f(0, 0, 0), Vec3f(0, 555, 0), Vec3f(0, 0, 555), red));
    W.add_model(W.quad(Vec3f(113, 554, 127), Vec3f(330, 0, 0), Vec3f(0, 0, 305), light));
    W.add_model(W.quad(Vec3f(0, 555, 0), Vec3f(555, 0, 0), Vec3f(0, 0, 555), white));
    W.add_model(W.quad(Vec3f(0, 0, 0), Vec3f(555, 0, 0), Vec3f(0, 0, 555), white));
    W.add_model(W.quad(Vec3f(0, 0, 555), Vec3f(555, 0, 0), Vec3f(0, 555, 0), white));
    Vec3f t1(265, 0, 295), r1(0, (float)to_radians(15), 0);
    Vec3f t2(130, 0, 65), r2(0, (float)to_radians(-18), 0);
    Model* box1 = W.box(Vec3f(0, 0, 0), Vec3f(165, 330, 165), &t1, &r1, white);
    Model* box2 = W.box(Vec3f(0, 0, 0), Vec3f(165, 165, 165), &t2, &r2, white);
    Material iso_black = W.isotropic(W.solid_register(0.0f, 0.0f, 0.0f));
    W.add_model(W.constant_medium(box1, 0.01f, iso_black));
    Material iso_white = W.isotropic(W.solid_register(1, 1, 1));
    W.add_model(W.constant_medium(box2, 0.01f, iso_white));
    W.vfov = 40; W.look_from = Vec3f(278, 278, -800); W.look_at = Vec3f(278, 278, 0);
    W.defocus_angle = 0; W.background = Vec3f(0, 0, 0);
}

// Scene.java:282-343 (Book 2 final scene)
static void scene_final(World& W) {
    JavaRandom math_random((int64_t)W.seed);
    W.solid_init();
    Material ground = W.lambertian(W.solid_register(0.48f, 0.83f, 0.53f));
    const int boxes_per_side = 20;
    for (int i = 0; i < boxes_per_side; i++) {
        for (int j = 0; j < boxes_per_side; j++) {
            float w = 100.0f;
            float x0 = -1000.0f + i * w;
            float z0 = -1000.0f + j * w;
            float y0 = 0.0f;
            float x1 = x0 + w;
            float y1 = (float)(1 + math_random.next_double() * 100);
            float z1 = z0 + w;
            W.add_model(W.box(Vec3f(x0, y0, z0), Vec3f(x1, y1, z1), nullptr, nullptr, ground));
        }
    }
    Material light = W.diffuse_light(7, 7, 7);
    W.add_model(W.quad(Vec3f(123, 554, 147), Vec3f(300, 0, 0), Vec3f(0, 0, 265), light));
    Vec3f center1(400, 400, 200);
    Vec3f center2 = center1.add(Vec3f(100, 0, 0));
    Material sphere_material = W.lambertian(W.solid_register(0.7f, 0.3f, 0.1f));
    W.add_model(W.sphere(center1, center2, 50, sphere_material));
    W.add_model(W.sphere(Vec3f(260, 150, 45), 50, W.dielectric(1.5f)));
    W.add_model(W.sphere(Vec3f(0, 150, 145), 50, W.metal(W.solid_register(0.8f, 0.8f, 0.9f), 0.999f)));
    Model* boundary = W.sphere(Vec3f(360, 150, 145), 70, W.dielectric(1.5f));
    W.add_model(boundary);
    Material iso1 = W.isotropic(W.solid_register(0.2f, 0.4f, 0.9f));
    W.add_model(W.constant_medium(boundary, 0.2f, iso1));
    boundary = W.sphere(Vec3f(0, 0, 0), 5000, W.dielectric(1.5f));
    Material iso2 = W.isotropic(W.solid_register(1, 1, 1));
    W.add_model(W.constant_medium(boundary, 0.0001f, iso2));
    Material earth = W.lambertian(W.image_create("earthmap.jpg", 100, 0));
    W.add_model(W.sphere(Vec3f(400, 200, 400), 100, earth));
    Material noise = W.lambertian(W.perlin_create(0.2f));
    W.add_model(W.sphere(Vec3f(220, 280, 300), 80, noise));
    Material white = W.lambertian(W.solid_register(0.73f, 0.73f, 0.73f));
    const int ns = 1000;
    for (int j = 0; j < ns; j++) {
        float cx = (float)(165 * math_random.next_double());
        float cy = (float)(165 * math_random.next_double());
        float cz = (float)(165 * math_random.next_double());
        Vec3f center = Vec3f(cx, cy, cz).add(-100, 270, 395);
        W.add_model(W.sphere(center, 10, white));
    }
    W.vfov = 40; W.look_from = Vec3f(478, 278, -600); W.look_at = Vec3f(278, 278, 0);
    W.defocus_angle = 0; W.background = Vec3f(0, 0, 0);
}

// Scene 9: build-defined "Book-1 three spheres" (not in Scene.java)
static void scene_three_spheres(World& W) {
    W.solid_init();
    W.add_model(W.sphere(Vec3f(0, -100.5f, -1), 100, W.lambertian(W.solid_register(0.8f, 0.8f, 0.0f))));
    W.add_model(W.sphere(Vec3f(0, 0, -1.2f), 0.5f, W.lambertian(W.solid_register(0.1f, 0.2f, 0.5f))));
    W.add_model(W.sphere(Vec3f(-1, 0, -1), 0.5f, W.dielectric(1.5f)));
    W.add_model(W.sphere(Vec3f(1, 0, -1), 0.5f, W.metal(W.solid_register(0.8f, 0.6f, 0.2f), 0.999f)));
    W.vfov = 20; W.look_from = Vec3f(-2, 2, 1); W.look_at = Vec3f(0, 0, -1);
    W.defocus_angle = 10.0f; W.focus_dist = 3.4f; W.background = Vec3f(0.70f, 0.80f, 1.00f);
}

static int max_stack_needed(const std::vector<uint8_t>& nodes) {
    // Simulate the reference traversal's stack growth with every AABB hit.
    size_t n = nodes.size() / sizeof(rt_bvh_node);
    if (n == 0) return 0;
    const rt_bvh_node* nd = reinterpret_cast<const rt_bvh_node*>(nodes.data());
    std::vector<int> stack{0};
    int mx = 1;
    while (!stack.empty()) {
        int i = stack.back(); stack.pop_back();
        if ((nd[i].left_id & 0xFFFF) == 0) {
            stack.push_back((nd[i].left_id >> 16) & 0xFFFF);
            stack.push_back((nd[i].right_id >> 16) & 0xFFFF);
            mx = std::max(mx, (int)stack.size());
        }
    }
    return mx;
}

static void fill_info(rts_scene* s, int width, int height) {
    World& W = s->world;
    rts_info& I = s->info;
    I.scene_id = s->scene_id; I.width = width; I.height = height;
    I.n_spheres = (int)W.spheres.size(); I.n_quads = (int)W.quads.size(); I.n_boxes = (int)W.boxes.size();
    I.n_media = (int)W.media.size(); I.n_lights = (int)W.lights.size(); I.n_bvh_nodes = (int)W.bvh_nodes.size();
    I.n_bvh_prims = (int)W.all_models.size();
    I.max_stack = max_stack_needed(s->buf[RT_BIND_BVH]);
    I.n_textures = (int)W.textures.size();
    I.background[0] = W.background.x; I.background[1] = W.background.y; I.background[2] = W.background.z;
}

}  // namespace rtb

extern "C" {

const char* rts_last_error(void) { return g_err.c_str(); }

int rts_build(int scene_id, int width, int height, uint64_t seed, const char* asset_dir, rts_scene** out) {
    if (!out) return fail(RT_ERR_INVALID_ARG, "out is NULL");
    *out = nullptr;
    if (scene_id < 0 || scene_id >= RTS_NUM_SCENES)
        return fail(RT_ERR_INVALID_ARG, "Invalid scene ID: " + std::to_string(scene_id));
    if (width <= 0 || height <= 0) return fail(RT_ERR_INVALID_ARG, "image size must be positive");
    std::unique_ptr<rts_scene> s(new rts_scene());
    s->scene_id = scene_id;
    World& W = s->world;
    W.seed = seed;
    W.asset_dir = asset_dir ? asset_dir : RT_ASSET_DIR;
    try {
        switch (scene_id) {
            case 0: scene_bouncing_spheres(W); break;
            case 1: scene_checker_spheres(W); break;
            case 2: scene_earth(W); break;
            case 3: scene_perlin_spheres(W); break;
            case 4: scene_quads(W); break;
            case 5: scene_simple_light(W); break;
            case 6: scene_cornell_box(W); break;
            case 7: scene_cornell_smoke(W); break;
            case 8: scene_final(W); break;
            case 9: scene_three_spheres(W); break;
        }
        put_models_to_program(s.get());
        W.solid_put_data();
        W.checker_put_data();
    } catch (const std::exception& e) {
        return fail(RT_ERR_INVALID_ARG, e.what());
    }
    if (W.textures.size() > RT_MAX_TEXTURES) return fail(RT_ERR_LIMIT, "more than 8 textures");
    if (W.spheres.size() > RT_MAX_RECORDS || W.quads.size() > RT_MAX_RECORDS || W.boxes.size() > RT_MAX_RECORDS ||
        W.media.size() > RT_MAX_RECORDS || W.bvh_nodes.size() > RT_MAX_RECORDS)
        return fail(RT_ERR_LIMIT, "more than 65535 records of one type");
    W.set_image_size(width, height);
    W.camera_calculate();
    fill_info(s.get(), width, height);
    s->finished = true;
    *out = s.release();
    return RT_OK;
}

void rts_free(rts_scene* s) { delete s; }

// ---- custom scenes: the reference's builder calls (Scene.java's statements) one by one
int rts_new(uint64_t seed, const char* asset_dir, rts_scene** out) {
    if (!out) return fail(RT_ERR_INVALID_ARG, "out is NULL");
    *out = nullptr;
    rts_scene* s = new rts_scene();
    s->scene_id = -1;
    s->world.seed = seed;
    s->world.asset_dir = asset_dir ? asset_dir : RT_ASSET_DIR;
    *out = s;
    return RT_OK;
}

}  // extern "C"

namespace {
template <typename F>
int guarded(rts_scene* s, F&& f) {
    if (!s) return fail(RT_ERR_INVALID_ARG, "NULL scene");
    if (s->finished) return fail(RT_ERR_STATE, "the scene was already finished (rts_finish)");
    try {
        return f();
    } catch (const std::exception& e) {
        return fail(RT_ERR_INVALID_ARG, e.what());
    }
}
Vec3f v3f(const float* p) { return Vec3f(p[0], p[1], p[2]); }
int model_of(rts_scene* s, int handle, Model** m) {
    if (handle < 0 || handle >= (int)s->world.pool.size()) return fail(RT_ERR_INVALID_ARG, "no such model handle");
    *m = s->world.pool[handle].get();
    if ((*m)->type == RT_MODEL_BVH_NODE) return fail(RT_ERR_INVALID_ARG, "no such model handle");
    return RT_OK;
}
int new_model(rts_scene* s, Model* m, int* handle) {
    // the pool's index of m (just created: a box's side quads follow it)
    int k = (int)s->world.pool.size() - 1;
    while (k >= 0 && s->world.pool[k].get() != m) k--;
    if (handle) *handle = k;
    return RT_OK;
}
int material_of(rts_scene* s, int handle, Material* m) {
    if (handle < 0 || handle >= (int)s->materials.size()) return fail(RT_ERR_INVALID_ARG, "no such material handle");
    *m = s->materials[handle];
    return RT_OK;
}
}  // namespace

extern "C" {

int rts_solid_texture(rts_scene* s, float r, float g, float b, int* tex) {
    return guarded(s, [&] {
        World& W = s->world;
        if (W.solid_slot < 0) W.solid_init();
        const int id = W.solid_register(r, g, b);
        if (tex) *tex = id;
        return (int)RT_OK;
    });
}

int rts_checker_texture(rts_scene* s, const float c1[3], const float c2[3], float scale, int* tex) {
    return guarded(s, [&] {
        if (!c1 || !c2) return fail(RT_ERR_INVALID_ARG, "NULL colour");
        World& W = s->world;
        if (W.checker_slot < 0) W.checker_init();
        const int id = W.checker_register(c1[0], c1[1], c1[2], c2[0], c2[1], c2[2], scale);
        if (tex) *tex = id;
        return (int)RT_OK;
    });
}

int rts_perlin_texture(rts_scene* s, float scale, int* tex) {
    return guarded(s, [&] {
        const int id = s->world.perlin_create(scale);
        if (tex) *tex = id;
        return (int)RT_OK;
    });
}

int rts_image_texture(rts_scene* s, const char* asset_name, int shift_x, int shift_y, int* tex) {
    return guarded(s, [&] {
        if (!asset_name) return fail(RT_ERR_INVALID_ARG, "NULL asset name");
        const int id = s->world.image_create(asset_name, shift_x, shift_y);
        if (tex) *tex = id;
        return (int)RT_OK;
    });
}

int rts_material(rts_scene* s, int kind, int texture, float param, const float emit[3], int* handle) {
    return guarded(s, [&] {
        World& W = s->world;
        Material m;
        switch (kind) {
            case RT_MAT_LAMBERTIAN: m = W.lambertian(texture); break;
            case RT_MAT_METAL: m = W.metal(texture, param); break;   // Metal.java:13: fuzz in [0, 1)
            case RT_MAT_DIELECTRIC:
                if (!(param >= 1.0f && param <= 2.5f))   // Dielectric.java:20-29 packs (ior - 1) / 1.5 in 16 bits
                    return fail(RT_ERR_INVALID_ARG, "dielectric IOR must be in [1, 2.5]");
                if (W.solid_slot < 0) W.solid_init();
                m = W.dielectric(param);
                break;
            case RT_MAT_DIFFUSE_LIGHT:
                if (!emit) return fail(RT_ERR_INVALID_ARG, "diffuse light needs an emission colour");
                m = W.diffuse_light(emit[0], emit[1], emit[2]);
                break;
            case RT_MAT_ISOTROPIC: m = W.isotropic(texture); break;
            default: return fail(RT_ERR_INVALID_ARG, "unknown material kind");
        }
        s->materials.push_back(m);
        if (handle) *handle = (int)s->materials.size() - 1;
        return (int)RT_OK;
    });
}

int rts_sphere(rts_scene* s, const float center1[3], const float center2[3], float radius, int material, int* handle) {
    return guarded(s, [&] {
        Material m;
        if (!center1) return fail(RT_ERR_INVALID_ARG, "NULL centre");
        if (int r = material_of(s, material, &m)) return r;
        Model* sp = s->world.sphere(v3f(center1), center2 ? v3f(center2) : v3f(center1), radius, m);
        return new_model(s, sp, handle);
    });
}

int rts_quad(rts_scene* s, const float q[3], const float u[3], const float v[3], int material, int* handle) {
    return guarded(s, [&] {
        Material m;
        if (!q || !u || !v) return fail(RT_ERR_INVALID_ARG, "NULL vector");
        if (int r = material_of(s, material, &m)) return r;
        return new_model(s, s->world.quad(v3f(q), v3f(u), v3f(v), m), handle);
    });
}

int rts_box(rts_scene* s, const float a[3], const float b[3], const float translation[3], const float rotation[3],
            int material, int* handle) {
    return guarded(s, [&] {
        Material m;
        if (!a || !b) return fail(RT_ERR_INVALID_ARG, "NULL corner");
        if ((translation == nullptr) != (rotation == nullptr))
            return fail(RT_ERR_INVALID_ARG, "Box.java takes translation and rotation together");
        if (int r = material_of(s, material, &m)) return r;
        Vec3f t, rot;
        if (translation) { t = v3f(translation); rot = v3f(rotation); }
        Model* bx = s->world.box(v3f(a), v3f(b), translation ? &t : nullptr, rotation ? &rot : nullptr, m);
        return new_model(s, bx, handle);
    });
}

int rts_constant_medium(rts_scene* s, int boundary, float density, int material, int* handle) {
    return guarded(s, [&] {
        Material m;
        Model* bnd = nullptr;
        if (int r = model_of(s, boundary, &bnd)) return r;
        if (bnd->type == RT_MODEL_CONSTANT_MEDIUM) return fail(RT_ERR_INVALID_ARG, "a medium cannot bound a medium");
        if (int r = material_of(s, material, &m)) return r;
        if (!(density > 0.0f)) return fail(RT_ERR_INVALID_ARG, "density must be positive");
        // ConstantMedium.java:12-20: the constructor registers its boundary with addModel
        return new_model(s, s->world.constant_medium(bnd, density, m), handle);
    });
}

int rts_add_model(rts_scene* s, int handle) {
    return guarded(s, [&] {
        Model* m = nullptr;
        if (int r = model_of(s, handle, &m)) return r;
        s->world.add_model(m);
        return (int)RT_OK;
    });
}

int rts_add_light(rts_scene* s, int handle) {
    return guarded(s, [&] {
        Model* m = nullptr;
        if (int r = model_of(s, handle, &m)) return r;
        if (m->type != RT_MODEL_SPHERE && m->type != RT_MODEL_QUAD)
            return fail(RT_ERR_INVALID_ARG, "lights are spheres or quads (pdf.glsl:58-96)");
        s->world.add_light(m);
        return (int)RT_OK;
    });
}

int rts_camera(rts_scene* s, const rts_camera_params* p) {
    return guarded(s, [&] {
        if (!p) return fail(RT_ERR_INVALID_ARG, "NULL camera");
        World& W = s->world;
        W.look_from = v3f(p->look_from);
        W.look_at = v3f(p->look_at);
        W.vup = v3f(p->vup);
        W.vfov = p->vfov;
        W.defocus_angle = p->defocus_angle;
        W.focus_dist = p->focus_dist;
        W.background = v3f(p->background);
        return (int)RT_OK;
    });
}

int rts_finish(rts_scene* s, int width, int height) {
    if (!s) return fail(RT_ERR_INVALID_ARG, "NULL scene");
    if (s->scene_id >= 0 || s->finished) return fail(RT_ERR_STATE, "only an unfinished rts_new scene can be finished");
    if (width <= 0 || height <= 0) return fail(RT_ERR_INVALID_ARG, "image size must be positive");
    World& W = s->world;
    try {
        put_models_to_program(s);
        W.solid_put_data();
        W.checker_put_data();
    } catch (const std::exception& e) {
        return fail(RT_ERR_INVALID_ARG, e.what());
    }
    if (W.textures.size() > RT_MAX_TEXTURES) return fail(RT_ERR_LIMIT, "more than 8 textures");
    if (W.spheres.size() > RT_MAX_RECORDS || W.quads.size() > RT_MAX_RECORDS || W.boxes.size() > RT_MAX_RECORDS ||
        W.media.size() > RT_MAX_RECORDS || W.bvh_nodes.size() > RT_MAX_RECORDS)
        return fail(RT_ERR_LIMIT, "more than 65535 records of one type");
    W.set_image_size(width, height);
    W.camera_calculate();
    fill_info(s, width, height);
    s->finished = true;
    return RT_OK;
}

int rts_get_info(const rts_scene* s, rts_info* info) {
    if (!s || !info) return fail(RT_ERR_INVALID_ARG, "NULL argument");
    *info = s->info;
    return RT_OK;
}

int rts_get_buffer(const rts_scene* s, int binding, const void** bytes, size_t* nbytes) {
    if (!s || !bytes || !nbytes) return fail(RT_ERR_INVALID_ARG, "NULL argument");
    if (binding < 0 || binding > 5) return fail(RT_ERR_INVALID_ARG, "binding out of range");
    *bytes = s->buf[binding].data();
    *nbytes = s->buf[binding].size();
    return RT_OK;
}

int rts_get_texture(const rts_scene* s, int slot, int* format, int* w, int* h, const void** texels, size_t* nbytes) {
    if (!s || !format || !w || !h || !texels || !nbytes) return fail(RT_ERR_INVALID_ARG, "NULL argument");
    if (slot < 0 || slot >= (int)s->world.textures.size()) return fail(RT_ERR_INVALID_ARG, "no such texture slot");
    const TexSlot& t = s->world.textures[slot];
    *format = t.format; *w = t.w; *h = t.h; *texels = t.bytes.data(); *nbytes = t.bytes.size();
    return RT_OK;
}

int rts_get_camera(const rts_scene* s, float ubo[28]) {
    if (!s || !ubo) return fail(RT_ERR_INVALID_ARG, "NULL argument");
    std::memcpy(ubo, &s->world.ubo, sizeof(rt_camera_ubo));
    return RT_OK;
}

int rts_set_image_size(rts_scene* s, int width, int height) {
    if (!s || width <= 0 || height <= 0) return fail(RT_ERR_INVALID_ARG, "bad size");
    s->world.set_image_size(width, height);
    s->world.camera_calculate();
    s->info.width = width; s->info.height = height;
    return RT_OK;
}

void rts_spp_uniforms(int spp, float* sqrt_spp, float* recip) {
    float s = (float)std::sqrt((double)spp);
    if (sqrt_spp) *sqrt_spp = s;
    if (recip) *recip = 1.0f / s;
}

int32_t rts_java_random_next_int(int64_t seed, int n_before) {
    JavaRandom r(seed); for (int i = 0; i < n_before; i++) r.next_int(); return r.next_int();
}
double rts_java_random_next_double(int64_t seed, int n_before) {
    JavaRandom r(seed); for (int i = 0; i < n_before; i++) r.next_double(); return r.next_double();
}
float rts_java_random_next_float(int64_t seed, int n_before) {
    JavaRandom r(seed); for (int i = 0; i < n_before; i++) r.next_float(); return r.next_float();
}
int32_t rts_java_random_next_int_bound(int64_t seed, int bound) { JavaRandom r(seed); return r.next_int(bound); }

}  // extern "C"
