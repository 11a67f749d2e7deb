/*
 * rt_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's per-pixel kernel (compute.glsl +
 * utils/{hitting,scatter,pdf,random,texture,math,interval}.glsl) used as the parity checker for the HIP path and as the timed
 * CPU baseline in bench.py.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load liboracle.so.  The product library
 * (librtamd.so) never links or calls it.
 *
 * Parity status: the reference (Java + OpenGL GLSL) cannot run anywhere in this
 * pipeline (no JDK, no GL, Windows-only natives), and it ships no
 * tests or golden vectors.  The oracle is therefore pinned only by (a) the
 * get_sphere_uv known-answer table in texture.glsl:100-102, (b) the std430
 * layout comments of RaytraceModel.java:139-219 vs compute.glsl structs, and
 * (c) statistical agreement with the reference gallery render of scene 6;
 * everything else is "parity unpinned" against the reference itself.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_scene_desc {
    const void* buf[6];          /* SSBO bytes, rt.h RT_BIND_* order */
    size_t nbytes[6];
    int tex_format[8];           /* rt.h RT_TEX_*, 0 = unbound */
    int tex_w[8], tex_h[8];
    const void* tex[8];
    float camera[28];            /* std140 Camera block */
    int max_depth;
    float background[3];
    float sqrt_spp, recip_sqrt_spp;
} oracle_scene_desc;

/* Logical record traffic of the reference kernel. */
typedef struct oracle_counters {
    uint64_t samples;
    uint64_t bounces;            /* ray_color loop iterations            */
    uint64_t node_visits;        /* bvh_nodes[...] loads (32 B)          */
    uint64_t sphere_tests, quad_tests, box_tests, medium_tests;
    uint64_t rand_calls;
    uint64_t framebuffer_bytes;  /* 32 per sample                        */
    uint64_t node_bytes;
    uint64_t prim_bytes;         /* primitive records read by hit tests  */
    uint64_t material_bytes;     /* set_material_properties re-reads     */
    uint64_t texel_bytes;
    uint64_t light_bytes;
} oracle_counters;

/* Render n_frames frames (frame_count = first_frame + i, u_rand_factor =
 * rand_factors[i]) into the full-size W x H RGBA32F image `rgba` (row 0 = top),
 * touching only rows r with (r / stripe_rows) % world == rank.
 * nthreads = 0 -> all hardware threads.  counters may be NULL. */
int oracle_render(const oracle_scene_desc* d, int width, int height, float* rgba,
                  int first_frame, int n_frames, const float* rand_factors,
                  int rank, int world, int stripe_rows, int nthreads,
                  oracle_counters* counters);

/* Pin oracle_render's threads: worker i to CPU cpus[i % n] (n = 0: unpinned, the
 * default).  Used by bench.py's CPU baseline only. */
void oracle_set_thread_cpus(const int* cpus, int n);

/* Analysis hook: per-trace BVH node sequences for a pixel window
 * (records [pixel, frame, bounce, n, node...]); returns int32 count. */
long oracle_trace_log(const oracle_scene_desc* d, int width, int height, int x0, int x1, int y0, int y1,
                      int first_frame, int n_frames, const float* rand_factors, int32_t* out, long cap);

/* Known-answer hooks. */
void oracle_get_sphere_uv(float x, float y, float z, float* u, float* v);
/* n successive rand() values for an invocation at (px,py) with u_rand_factor f */
void oracle_rand_sequence(float px, float py, float f, int n, float* out);
/* GLSL built-ins as defined in include/rt/rt_glsl.h: fn 0 sin, 1 cos, 2 log,
 * 3 acos, 4 atan2(x, y2), 5 fract, 6 sqrt */
void oracle_eval_builtin(int fn, const float* x, const float* y2, float* out, int n);
/* Perlin noise_turb / perlin_noise_color for a 6x256 R32F table */
float oracle_perlin_turb(const float* table, float px, float py, float pz, int depth);
/* ray-primitive KATs: return 1 on hit and fill t / p / normal / front */
int oracle_hit_sphere(const void* sphere48, float time, const float o[3], const float dir[3],
                      float tmin, float tmax, float* t, float p[3], float n[3], int* front);
int oracle_hit_quad(const void* quad80, const float o[3], const float dir[3],
                    float tmin, float tmax, float* t, float p[3], float n[3], int* front);
int oracle_hit_aabb(const float box6[6], const float o[3], const float dir[3], float tmin, float tmax);

#ifdef __cplusplus
}
#endif

#endif
