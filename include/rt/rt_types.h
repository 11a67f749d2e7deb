/*
 * rt_types.h — byte layouts of the scene records exactly as the reference's
 * Java packers write them (little-endian, std430 SSBOs / std140 UBO), and
 * exactly as compute.glsl declares them.  These are the ABI records that
 * rt_upload_buffer() accepts.
 *
 *   Sphere         48 B  compute.glsl:65-80,  Sphere.java:33-51
 *   BVHNode        32 B  compute.glsl:117-125, BVHNode.java:47-56
 *   Quad           80 B  compute.glsl:82-92,  Quad.java:43-54
 *   ConstantMedium 20 B  compute.glsl:98-104, ConstantMedium.java:26-37
 *   Box           480 B  compute.glsl:94-96,  Box.java:56-59
 *   Lights        4+4n B compute.glsl:147-153, RaytraceModel.java:232-246
 *   Camera UBO    112 B  compute.glsl:31-42,  Camera.java:121-139 (std140)
 */
#ifndef RT_TYPES_H
#define RT_TYPES_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Model type ids (RaytraceModel.java:14-18) — low 16 bits of a packed id. */
enum { RT_MODEL_BVH_NODE = 0, RT_MODEL_SPHERE = 1, RT_MODEL_QUAD = 2,
       RT_MODEL_CONSTANT_MEDIUM = 3, RT_MODEL_BOX = 4 };

/* Material ids (Material.java:7-11) — high 16 bits of a packed material. */
enum { RT_MAT_LAMBERTIAN = 0, RT_MAT_METAL = 1, RT_MAT_DIELECTRIC = 2,
       RT_MAT_DIFFUSE_LIGHT = 3, RT_MAT_ISOTROPIC = 4 };

/* Texture type ids (Texture.java:20-24) — bits 28..31 of a packed texture id. */
enum { RT_TEXTYPE_DEFAULT = 0, RT_TEXTYPE_IMAGE = 1, RT_TEXTYPE_CHECKER = 2,
       RT_TEXTYPE_PERLIN = 3, RT_TEXTYPE_SOLID = 4 };

/* Texture formats accepted by rt_upload_texture (Texture.java ctor calls):
 *   RGB8  — SolidTexture / CheckerTexture / ImageTexture (GL_RGB8, GL_UNSIGNED_BYTE)
 *   RGBA8 — ImageTexture with 4 channels (ImageTexture.java:44-46)
 *   R32F  — PerlinNoiseTexture (GL_R32F, GL_FLOAT), PerlinNoiseTexture.java:41-43 */
enum { RT_TEX_RGB8 = 1, RT_TEX_RGBA8 = 2, RT_TEX_R32F = 3 };

typedef struct rt_sphere {
    float center1[3];
    int32_t texture_id;
    float center_vec[3];
    float radius;
    float emission[3];
    int32_t material;
} rt_sphere;

typedef struct rt_bvh_node {
    float xmin, xmax, ymin, ymax, zmin, zmax;
    int32_t left_id;   /* (index << 16) | model type */
    int32_t right_id;
} rt_bvh_node;

typedef struct rt_quad {
    float normal[3];
    float d;
    float q[3];
    int32_t material;
    float u[3];
    int32_t texture_id;
    float v[3];
    float area;
    float emission[3];
    float pad;
} rt_quad;

typedef struct rt_medium {
    int32_t boundary_idx;
    int32_t boundary_type;
    float neg_inv_density;
    int32_t phase_material;
    int32_t texture_id;
} rt_medium;

typedef struct rt_box {
    rt_quad quads[6];
} rt_box;

typedef struct rt_camera_ubo {
    float viewport_width, viewport_height, aspect_ratio, defocus_angle;
    float camera_pos[3];    float pad0;
    float up_left[3];       float pad1;
    float pixel_delta_u[3]; float pad2;
    float pixel_delta_v[3]; float pad3;
    float defocus_disk_u[3]; float pad4;
    float defocus_disk_v[3]; float pad5;
} rt_camera_ubo;

#ifdef __cplusplus
}
static_assert(sizeof(rt_sphere) == 48, "Sphere std430 record is 48 B");
static_assert(sizeof(rt_bvh_node) == 32, "BVHNode std430 record is 32 B");
static_assert(sizeof(rt_quad) == 80, "Quad std430 record is 80 B");
static_assert(sizeof(rt_medium) == 20, "ConstantMedium std430 record is 20 B");
static_assert(sizeof(rt_box) == 480, "Box std430 record is 480 B");
static_assert(sizeof(rt_camera_ubo) == 112, "Camera std140 block is 112 B");
#endif

#endif /* RT_TYPES_H */
