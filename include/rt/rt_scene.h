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
 * earthmap.ppm (scenes 2 and 8); NULL = "<repo>/assets" resolved at build time.
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

/* RaytraceExecutor.setSamplePerPixel: sqrt_spp = (float)Math.sqrt(spp). */
void rts_spp_uniforms(int spp, float* sqrt_spp, float* recip_sqrt_spp);

/* Texture.saveAsPNG semantics: RGBA32F (row 0 = top) -> unorm8 (clamp, round)
 * -> (byte)(pow(b/255, 1/2.2)*255) -> RGB PNG.  rgb8_out (W*H*3) optional. */
int rts_tonemap_rgb8(const float* rgba, int width, int height, uint8_t* rgb8_out);
int rts_save_png(const float* rgba, int width, int height, const char* path);

/* java.util.Random known-answer hooks (tests). */
int32_t rts_java_random_next_int(int64_t seed, int n_calls_before);
double rts_java_random_next_double(int64_t seed, int n_calls_before);
float rts_java_random_next_float(int64_t seed, int n_calls_before);
int32_t rts_java_random_next_int_bound(int64_t seed, int bound);

#ifdef __cplusplus
}
#endif

#endif /* RT_SCENE_H */
