/*
 * rt.h — drop-in C ABI of the MI355X path tracer (librtamd.so).
 *
 * It replaces the OpenGL binding contract that the reference's Java host drives
 * (SURVEY §8b).  Each entry point names the reference call it stands in for.
 * All calls return 0 (RT_OK) or a negative RT_ERR_* code; the message of the
 * last failure on a context is available from rt_last_error().  A context is
 * used by one host thread at a time (the reference's GL-context rule); callers
 * own every host buffer they pass (the library copies what it keeps).
 */
#ifndef RT_H
#define RT_H

#include <stddef.h>
#include <stdint.h>

#include "rt_types.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 1

enum {
    RT_OK = 0,
    RT_ERR_INVALID_ARG = -1,  /* bad pointer/size/enum, record size mismatch       */
    RT_ERR_DEVICE = -2,       /* HIP runtime failure                               */
    RT_ERR_STATE = -3,        /* call order (e.g. render before resize)            */
    RT_ERR_LIMIT = -4,        /* an implicit reference limit exceeded (SURVEY App.C)*/
    RT_ERR_NOMEM = -5,
    RT_ERR_TIMEOUT = -6       /* rt_comm_init / rt_gather_image: a peer did not complete in
                                 time (rt_comm_set_timeout); the communicator was aborted   */
};

/* SSBO binding points (compute.glsl:127-153, RaytraceModel.java:81-113) */
enum {
    RT_BIND_SPHERES = 0, RT_BIND_BVH = 1, RT_BIND_QUADS = 2,
    RT_BIND_MEDIA = 3, RT_BIND_BOXES = 4, RT_BIND_LIGHTS = 5
};


#define RT_MAX_TEXTURES 8        /* uniform sampler2D textures[8], compute.glsl:23 */
#define RT_MAX_RECORDS 65535     /* 16-bit indices in packed ids (App. C)          */
#define RT_MAX_BVH_DEPTH 64      /* int stack[64], compute.glsl:229                */
#define RT_MAX_IMAGE_DIM 65536   /* image width / height (pixel coordinates feed rand()) */
#define RT_MAX_RAND_FACTOR 1024.0f /* |u_rand_factor| (see rt_render)                */

typedef struct rt_ctx rt_ctx;

/* Create a context rendering on n_devices HIP devices (device_ids may be NULL
 * for 0..n-1; explicit ids may repeat, n <= 64).  Rows are split in
 * interleaved stripes over the device slots and gathered on device 0 by
 * rt_read_image (RCCL, see rt_comm_*); the result equals a 1-device render bit
 * for bit.
 * Replaces: Window.initGLFW/initShaderPrograms (Window.java:90-193). */
int rt_create(int n_devices, const int* device_ids, rt_ctx** out);
int rt_destroy(rt_ctx* ctx);
/* Message of the last failure on ctx; with ctx == NULL, of the last failed
 * rt_create on the calling thread. */
const char* rt_last_error(rt_ctx* ctx);
int rt_abi_version(void);

/* Upload one SSBO's exact std430 bytes (rt_types.h records; lights = int count
 * followed by count packed ints).  nbytes must be a multiple of the record size.
 * Replaces: RaytraceModel.put{Spheres,BVHNodes,Quads,ConstantMediums,Boxes,
 * Lights}ToProgram -> BufferObject.uploadData (RaytraceModel.java:138-246). */
int rt_upload_buffer(rt_ctx* ctx, int binding, const void* bytes, size_t nbytes);

/* Upload texture slot 0..7; rows tightly packed, row 0 first (glTexImage2D).
 * Sampling follows GL_LINEAR + CLAMP_TO_EDGE (Texture.java:74-77).
 * Replaces: Texture.putData (Texture.java:122-133). */
int rt_upload_texture(rt_ctx* ctx, int slot, int format, int w, int h, const void* texels);

/* The 28-float std140 camera block (rt_camera_ubo).
 * Replaces: Camera.putToShaderProgram UBO upload (Camera.java:121-139). */
int rt_set_camera(rt_ctx* ctx, const float ubo[28]);

/* Uniforms max_depth, background, sqrt_spp, recip_sqrt_spp.
 * Replaces: GuiRenderer.maxDepthUpdate, Camera.putToShaderProgram("background"),
 * RaytraceExecutor.setSamplePerPixel (RaytraceExecutor.java:50-56). */
int rt_set_params(rt_ctx* ctx, int max_depth, const float background[3],
                  float sqrt_spp, float recip_sqrt_spp);

/* (Re)allocate the RGBA32F accumulation image, zero-filled; 1 <= w, h <= RT_MAX_IMAGE_DIM.
 * Replaces: Texture.resize on the framebuffer callback (Window.java:116-129). */
int rt_resize(rt_ctx* ctx, int w, int h);

/* Run n_frames progressive frames.  Equal to n_frames x { frame_count =
 * first_frame+i; u_rand_factor = rand_factors[i]; glDispatchCompute;
 * glMemoryBarrier }.  Asynchronous on the context's stream(s).  Each rand
 * factor must be finite with |value| <= RT_MAX_RAND_FACTOR (the reference
 * passes (float)Math.random() in [0, 1); beyond, rand()'s +0.001 steps vanish).
 * Replaces: RaytraceExecutor.raytrace (RaytraceExecutor.java:100-142). */
int rt_render(rt_ctx* ctx, int first_frame, int n_frames, const float* rand_factors);

/* Wait for all queued renders. */
int rt_sync(rt_ctx* ctx);

/* Copy the accumulation image (W*H*4 floats, row 0 = top) to the host.
 * Replaces: glGetTexImage in Texture.saveAsPNG (Texture.java:93). */
int rt_read_image(rt_ctx* ctx, float* rgba);

/* Overwrite the accumulation image (resume a checkpointed accumulation). */
int rt_write_image(rt_ctx* ctx, const float* rgba);

/* Device time of the last rt_render call (max over devices), after completion.
 * Replaces: QueryTimer GL_TIME_ELAPSED (QueryTimer.java:24-50). */
int rt_last_render_ns(rt_ctx* ctx, uint64_t* ns);

/* Non-blocking: returns 1 with *ns (max over devices) once the last rt_render
 * call has finished on the device, 0 while it still runs (*ns untouched).
 * Replaces: the polling of finished QueryTimer results that feeds
 * lastDispatchTime on every raytrace() (RaytraceExecutor.java:106-115). */
int rt_render_done(rt_ctx* ctx, uint64_t* ns);

/* ---- MI355X-native extensions (no reference counterpart) ---------------- */

/* Multi-process partition (one process per GPU): this context renders only the
 * rows r with (r / stripe_rows) % world == rank.  Its image then holds
 * local_rows = rt_local_rows(...) rows, stripe-compacted; gather with
 * torch.distributed (RCCL) and rt_deinterleave_rows().  Must precede rt_resize. */
int rt_set_partition(rt_ctx* ctx, int rank, int world, int stripe_rows);
int rt_local_rows(int height, int rank, int world, int stripe_rows);
int rt_padded_local_rows(int height, int world, int stripe_rows);

/* Bind a caller-owned device buffer (>= W*local_rows*16 bytes, on the context's
 * single device) as the accumulation image instead of an internal one; pass
 * NULL to go back to the internal image.  Must follow rt_resize. */
int rt_bind_device_image(rt_ctx* ctx, void* device_ptr, size_t nbytes);

/* Use a caller-provided hipStream_t (e.g. torch's current stream); NULL = own. */
int rt_set_stream(rt_ctx* ctx, void* hip_stream);

/* ---- RCCL over xGMI behind the ABI (the partition's one exchange).
 * A context over several devices (rt_create(n > 1)) gathers in rt_read_image: each
 * device's stripe block to device 0 over RCCL (ncclCommInitAll; one ncclSend /
 * ncclRecv pair per device) when the device ids are distinct, else by peer copies,
 * then a de-interleave kernel on device 0 and one copy to the host.
 * One process per GPU: rank 0 makes a communicator id (RT_COMM_ID_BYTES bytes) that
 * the host hands to every rank by its own means (the reference has no transport);
 * each rank, after rt_set_partition(rank, world, ...), calls rt_comm_init; then
 * rt_gather_image sends every rank's stripe block to rank 0 over RCCL, where it is
 * de-interleaved on the device and copied out (rgba: W*H*4 floats on rank 0, NULL
 * elsewhere).  librccl.so is loaded on first use. */
#define RT_COMM_ID_BYTES 128
enum { RT_GATHER_HOST = 0, RT_GATHER_PEER = 1, RT_GATHER_RCCL = 2 };
int rt_comm_unique_id(void* id_out);
int rt_comm_init(rt_ctx* ctx, const void* id, int rank, int world);
int rt_gather_image(rt_ctx* ctx, float* rgba);
/* Deadline of rt_comm_init and rt_gather_image on this context, in ms (default 120000;
 * 0 = wait forever).  The communicator is made non-blocking (ncclConfig_t.blocking = 0)
 * where the library allows it, and every wait polls against the deadline: a rank that
 * never joins or never posts its Send / Recv makes the call return RT_ERR_TIMEOUT, with
 * the communicator aborted (its queued work freed), instead of holding the host. */
int rt_comm_set_timeout(rt_ctx* ctx, int timeout_ms);
/* Abort the context's communicator(s) (ncclCommAbort; ncclCommDestroy where absent) and
 * free their queued work.  A later gather needs rt_comm_init again. */
int rt_comm_abort(rt_ctx* ctx);
/* How the last gather ran: RT_GATHER_*, or -1 before any. */
int rt_gather_path(rt_ctx* ctx);

/* Host helper: scatter gathered stripe blocks [world][padded_rows][W][4] into a
 * full W x H image (row 0 = top). */
int rt_deinterleave_rows(const float* gathered, int width, int height, int world,
                         int stripe_rows, float* rgba_out);

/* ---- Non-parity fast mode -------------------------------
 * RT_BVH_REFERENCE (default): the walk runs on the uploaded BVH -- the reference's median
 * split (BVHNode.java:13-56) -- and every image is bit-identical to the reference semantics.
 * RT_BVH_SAH: the context rebuilds the BVH from the uploaded BVH's prims with a binned-SAH
 * builder (leaves of at most two prims; each medium keeps its reference leaf, so its test
 * multiplicity and hence its density are the reference's) and walks that.  Same kernel, same
 * leaf tests; far fewer node visits and prim tests.  NOT bit-exact against the reference
 * BVH: a medium's rand() draws fall at another point of the visit sequence, so images agree
 * statistically (tests/test_gpu_fast_bvh.py).  Takes effect at the next rt_render. */
enum { RT_BVH_REFERENCE = 0, RT_BVH_SAH = 1 };
int rt_set_bvh_mode(rt_ctx* ctx, int mode);

/* Per-frame u_rand_factor for frame index f (0-based) of a seeded render:
 * top 24 bits of splitmix64(seed, f) / 2^24, in [0,1).  Stands in for the
 * reference's (float)Math.random() per frame (RaytraceExecutor.java:124). */
float rt_frame_rand_factor(uint64_t seed, uint64_t frame_index);

#ifdef __cplusplus
}
#endif

#endif /* RT_H */
