/*
 * rt_scene.h — C ABI of the host scene builder (librtscene.so).
 *
 * A C++ restatement of the reference's Java host side that produces the exact
 * std430/std140 bytes the GLSL path consumed and rt.h now consumes:
 *   Scene.java:19-343 (scenes 0-8)  + build-defined scene 9
 *   RaytraceModel.java:57-246 (addModel/addLight, BVH build, packers)
 *   BVHNode.java:13-56, AABB.java, Sphere/Quad/Box/ConstantMedium.java
 *   Camera.java:91-143, materials/{Material,Metal,...}.java, textures/{Texture,SolidTexture,...}.java, Color.java
 * plus Texture.saveAsPNG (Texture.java:89-120) and the per-frame uniforms of
 * RaytraceExecutor (sqrt_spp, recip_sqrt_spp).
 *
 * The reference builds scenes from unseeded Math.random()/new Random(); this
 * builder substitutes java.util.Random-exact LCGs seeded from `seed`
 * (SURVEY §8d): Math.random -> Random(seed), Color.RANDOM -> Random(seed+1),
 * k-th Perlin texture -> Random(seed+2+k), scene0 fuzz -> Random(seed+100).
 */
#ifndef RT_SCENE_H
#define RT_SCENE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rts_scene rts_scene;

#define RTS_NUM_SCENES 10

typedef struct rts_info {
    int scene_id, width, height;
    int n_spheres, n_quads, n_boxes, n_media, n_lights, n_bvh_nodes;
    int n_bvh_prims;      /* models in the BVH list (ALL_MODELS)            */
    int bvh_depth;        /* levels, root = 1                               */
    int max_stack;        /* stack entries the reference traversal needs     */
    int n_textures;
    float background[3];
} rts_info;

/* Build scene `scene_id` (0..9) for a width x height image.  asset_dir holds
 * earthmap.jpg (scenes 2 and 8; the reference's textures/earthmap.jpg, decoded by
 * rts_decode_image); NULL = "<repo>/assets" resolved at build time.
 * Returns 0 or a negative rt.h error code. */
int rts_build(int scene_id, int width, int height, uint64_t seed,
              const char* asset_dir, rts_scene** out);
void rts_free(rts_scene* s);
const char* rts_last_error(void);

int rts_get_info(const rts_scene* s, rts_info* info);
/* Exact bytes for SSBO binding 0..5 (rt.h RT_BIND_*). */
int rts_get_buffer(const rts_scene* s, int binding, const void** bytes, size_t* nbytes);
/* Texture slot data as rt_upload_texture expects it. */
int rts_get_texture(const rts_scene* s, int slot, int* format, int* w, int* h,
                    const void** texels, size_t* nbytes);
int rts_get_camera(const rts_scene* s, float ubo[28]);

/* Re-aim the camera for a new image size (Scene.updateCamera). */
int rts_set_image_size(rts_scene* s, int width, int height);

/* ---- Custom scenes: the reference's builder calls one by one (Scene.java's
 * statements).  rts_new starts an empty world (RaytraceModel's and the texture
 * classes' static lists); textures and materials are objects the models share,
 * as in Java; rts_finish runs RaytraceModel.putModelsToProgram (BVH build and
 * packers), Solid/CheckerTexture.putDataToTexture and Camera.init, after which
 * the rts_get_* calls return the scene's bytes.  Handles are >= 0 ints; every
 * call returns 0 or a negative rt.h error code (message: rts_last_error). */
int rts_new(uint64_t seed, const char* asset_dir, rts_scene** out);
/* SolidTexture.registerColor / CheckerTexture(c1, c2, scale) / new PerlinNoiseTexture(scale)
 * / ImageTexture.create(asset, shift): *tex = the packed texture id (Texture.getValue). */
int rts_solid_texture(rts_scene* s, float r, float g, float b, int* tex);
int rts_checker_texture(rts_scene* s, const float c1[3], const float c2[3], float scale, int* tex);
int rts_perlin_texture(rts_scene* s, float scale, int* tex);
int rts_image_texture(rts_scene* s, const char* asset_name, int shift_x, int shift_y, int* tex);
/* new Lambertian(tex) / Metal(tex, fuzz = param) / Dielectric(ior = param) /
 * DiffuseLight(emit) / Isotropic(tex); kind = RT_MAT_*. */
int rts_material(rts_scene* s, int kind, int texture, float param, const float emit[3], int* material);
/* new Sphere(center1[, center2], r, mat) / Quad(q, u, v, mat) / Box(a, b, mat) or
 * Box(a, b, translation, rotation in radians, mat) / ConstantMedium(boundary, density, mat):
 * *model = the model's handle (not yet in the world). */
int rts_sphere(rts_scene* s, const float center1[3], const float center2[3], float radius, int material, int* model);
int rts_quad(rts_scene* s, const float q[3], const float u[3], const float v[3], int material, int* model);
int rts_box(rts_scene* s, const float a[3], const float b[3], const float translation[3], const float rotation[3],
            int material, int* model);
int rts_constant_medium(rts_scene* s, int boundary_model, float density, int material, int* model);
/* RaytraceModel.addModel / addLight (RaytraceModel.java:57-79). */
int rts_add_model(rts_scene* s, int model);
int rts_add_light(rts_scene* s, int model);
/* Camera.lookFrom/lookAt/vup/vfov/defocusAngle/focusDist and the background colour. */
typedef struct rts_camera_params {
    float look_from[3], look_at[3], vup[3];
    float vfov, defocus_angle, focus_dist;
    float background[3];
} rts_camera_params;
int rts_camera(rts_scene* s, const rts_camera_params* p);
int rts_finish(rts_scene* s, int width, int height);

/* RaytraceExecutor.setSamplePerPixel: sqrt_spp = (float)Math.sqrt(spp). */
void rts_spp_uniforms(int spp, float* sqrt_spp, float* recip_sqrt_spp);

/* Texture.saveAsPNG semantics: RGBA32F (row 0 = top) -> unorm8 (clamp, round)
 * -> (byte)(pow(b/255, 1/2.2)*255) -> RGB PNG.  rgb8_out (W*H*3) optional. */
int rts_tonemap_rgb8(const float* rgba, int width, int height, uint8_t* rgb8_out);
int rts_save_png(const float* rgba, int width, int height, const char* path);

/* ImageTexture.create's read (ImageTexture.java:22-85: ImageIO.read, then getRGB per
 * pixel): decode a JPEG (baseline / progressive, the IJG decoder's islow IDCT, fancy
 * upsampling and YCbCr tables), PNG (8-bit RGB / RGBA / palette) or P6 PPM file into
 * 8-bit R, G, B (, A) rows, row 0 = top (before ImageTexture's flip and shift).
 * *channels = 3 or 4 (BufferedImage's colour-model components); greyscale and other
 * component counts fail like the reference ("Unsupported image format").  pixels may be
 * NULL (size query); else it must hold width * height * channels bytes (capacity).
 * Message of a failure: rts_decode_last_error. */
int rts_decode_image(const char* path, int* width, int* height, int* channels, uint8_t* pixels,
                     size_t capacity);
const char* rts_decode_last_error(void);

/* java.util.Random known-answer hooks (tests). */
int32_t rts_java_random_next_int(int64_t seed, int n_calls_before);
double rts_java_random_next_double(int64_t seed, int n_calls_before);
float rts_java_random_next_float(int64_t seed, int n_calls_before);
int32_t rts_java_random_next_int_bound(int64_t seed, int bound);

#ifdef __cplusplus
}
#endif

#endif /* RT_SCENE_H */
