package net.bowen.system;

import java.lang.foreign.Arena;
import java.lang.foreign.FunctionDescriptor;
import java.lang.foreign.Linker;
import java.lang.foreign.MemorySegment;
import java.lang.foreign.SymbolLookup;
import java.lang.invoke.MethodHandle;
import java.nio.ByteBuffer;

import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_BYTE;
import static java.lang.foreign.ValueLayout.JAVA_FLOAT;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;

/**
 * Panama FFM (JDK 22+) binding of include/rt/rt.h, the C ABI of librtamd.so, for the
 * reference's Java host.  Every method is one rt_* call; a non-zero status becomes an
 * {@link IllegalStateException} carrying rt_last_error.  The calls it replaces:
 * <ul>
 *   <li>{@link #uploadBuffer}: RaytraceModel.put*ToProgram / BufferObject.uploadData
 *       (RaytraceModel.java:115-246) -- the same std430 ByteBuffer the packers fill;</li>
 *   <li>{@link #uploadTexture}: Texture.putData / glTexImage2D (Texture.java:122-133);</li>
 *   <li>{@link #setCamera}: Camera.putToShaderProgram, the 28-float std140 block
 *       (Camera.java:121-143);</li>
 *   <li>{@link #setParams}: the max_depth / background / sqrt_spp uniforms
 *       (RaytraceExecutor.java:50-56, GuiRenderer.java:64-68);</li>
 *   <li>{@link #resize}: the RGBA32F image texture (Window.java:201-204);</li>
 *   <li>{@link #render}: frame_count / u_rand_factor + glDispatchCompute + glMemoryBarrier
 *       (RaytraceExecutor.java:100-142), n frames per call;</li>
 *   <li>{@link #readImage}: glGetTexImage in Texture.saveAsPNG (Texture.java:89-120);</li>
 *   <li>{@link #lastRenderNanos} / {@link #renderDoneNanos}: the GL_TIME_ELAPSED query
 *       (QueryTimer.java), waited for / polled.</li>
 * </ul>
 * Several GPUs: {@link #RtAmd(int...)} renders interleaved row stripes on each device and
 * {@link #readImage} gathers them on device 0 over RCCL; one process per GPU uses
 * {@link #setPartition}, {@link #commUniqueId} / {@link #commInit} and {@link #gatherImage}.
 *
 * <p>Native memory: the context's own arena holds nothing but the context handle; every
 * call allocates its arguments from a confined arena that closes when the call returns,
 * so a long progressive loop does not grow native memory (readImage copies the pixels
 * to the Java heap before its arena closes).  Like a GL context, one thread at a time.
 *
 * <p>Reviewed only: this image has no JDK.  The same contract is exercised from Python
 * (raytracing-book_amd/rtamd/_lib.py) by the tests.
 */
public final class RtAmd implements AutoCloseable {
    /** rt.h bindings (compute.glsl:127-153). */
    public static final int SPHERES = 0, BVH = 1, QUADS = 2, MEDIA = 3, BOXES = 4, LIGHTS = 5;
    /** rt.h texture formats. */
    public static final int TEX_RGB8 = 1, TEX_RGBA8 = 2, TEX_R32F = 3;
    /** rt.h RT_COMM_ID_BYTES. */
    public static final int COMM_ID_BYTES = 128;

    private static final Linker LINKER = Linker.nativeLinker();
    private static final SymbolLookup LIB = SymbolLookup.libraryLookup(
            System.getProperty("rtamd.library", "librtamd.so"), Arena.global());

    private static MethodHandle fn(String name, FunctionDescriptor fd) {
        return LINKER.downcallHandle(LIB.find(name).orElseThrow(
                () -> new UnsatisfiedLinkError("librtamd.so has no " + name)), fd);
    }

    private static final MethodHandle CREATE = fn("rt_create", FunctionDescriptor.of(JAVA_INT, JAVA_INT, ADDRESS, ADDRESS));
    private static final MethodHandle DESTROY = fn("rt_destroy", FunctionDescriptor.of(JAVA_INT, ADDRESS));
    private static final MethodHandle LAST_ERROR = fn("rt_last_error", FunctionDescriptor.of(ADDRESS, ADDRESS));
    private static final MethodHandle UPLOAD_BUFFER =
            fn("rt_upload_buffer", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, ADDRESS, JAVA_LONG));
    private static final MethodHandle UPLOAD_TEXTURE =
            fn("rt_upload_texture", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT, JAVA_INT, JAVA_INT, ADDRESS));
    private static final MethodHandle SET_CAMERA = fn("rt_set_camera", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));
    private static final MethodHandle SET_PARAMS =
            fn("rt_set_params", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, ADDRESS, JAVA_FLOAT, JAVA_FLOAT));
    private static final MethodHandle SET_PARTITION =
            fn("rt_set_partition", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT, JAVA_INT));
    private static final MethodHandle RESIZE = fn("rt_resize", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT));
    private static final MethodHandle SET_BVH_MODE = fn("rt_set_bvh_mode", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT));
    private static final MethodHandle RENDER = fn("rt_render", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT, ADDRESS));
    private static final MethodHandle SYNC = fn("rt_sync", FunctionDescriptor.of(JAVA_INT, ADDRESS));
    private static final MethodHandle READ_IMAGE = fn("rt_read_image", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));
    private static final MethodHandle LAST_NS = fn("rt_last_render_ns", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));
    private static final MethodHandle RENDER_DONE = fn("rt_render_done", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));
    private static final MethodHandle LOCAL_ROWS =
            fn("rt_local_rows", FunctionDescriptor.of(JAVA_INT, JAVA_INT, JAVA_INT, JAVA_INT, JAVA_INT));
    private static final MethodHandle COMM_UNIQUE_ID = fn("rt_comm_unique_id", FunctionDescriptor.of(JAVA_INT, ADDRESS));
    private static final MethodHandle COMM_INIT =
            fn("rt_comm_init", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_INT, JAVA_INT));
    private static final MethodHandle GATHER_IMAGE = fn("rt_gather_image", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));
    private static final MethodHandle GATHER_PATH = fn("rt_gather_path", FunctionDescriptor.of(JAVA_INT, ADDRESS));
    private static final MethodHandle COMM_SET_TIMEOUT =
            fn("rt_comm_set_timeout", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT));
    private static final MethodHandle COMM_ABORT = fn("rt_comm_abort", FunctionDescriptor.of(JAVA_INT, ADDRESS));

    private final MemorySegment ctx;
    private int width, height;
    private int rank = 0, world = 1, stripeRows = 16;

    /** rt_create on one device (RaytraceModel.initSSBOs + the GL context setup). */
    public RtAmd(int device) {
        this(new int[]{device});
    }

    /** rt_create over several devices: row stripes on each, gathered on the first by readImage. */
    public RtAmd(int... devices) {
        try (Arena a = Arena.ofConfined()) {
            MemorySegment ids = a.allocateFrom(JAVA_INT, devices);
            MemorySegment out = a.allocate(ADDRESS);
            check(call(() -> (int) CREATE.invokeExact(devices.length, ids, out)), MemorySegment.NULL);
            ctx = out.get(ADDRESS, 0);
        }
    }

    @FunctionalInterface
    private interface Native {
        int run() throws Throwable;
    }

    private static int call(Native n) {
        try {
            return n.run();
        } catch (RuntimeException | Error e) {
            throw e;
        } catch (Throwable t) {
            throw new IllegalStateException(t);
        }
    }

    private static void check(int rc, MemorySegment c) {
        if (rc >= 0) return;
        String msg;
        try {
            msg = ((MemorySegment) LAST_ERROR.invokeExact(c)).reinterpret(4096).getString(0);
        } catch (Throwable t) {
            msg = "(no message)";
        }
        throw new IllegalStateException("rt error " + rc + ": " + msg);
    }

    /** The packer's ByteBuffer as it stands: direct, native (little-endian) order; the library copies it. */
    public void uploadBuffer(int binding, ByteBuffer direct) {
        MemorySegment seg = MemorySegment.ofBuffer(direct);
        long n = direct.remaining();
        check(call(() -> (int) UPLOAD_BUFFER.invokeExact(ctx, binding, seg, n)), ctx);
    }

    /** Rows tightly packed, row 0 first (glTexImage2D); sampled with GL_LINEAR + CLAMP_TO_EDGE. */
    public void uploadTexture(int slot, int format, int w, int h, ByteBuffer direct) {
        MemorySegment seg = MemorySegment.ofBuffer(direct);
        check(call(() -> (int) UPLOAD_TEXTURE.invokeExact(ctx, slot, format, w, h, seg)), ctx);
    }

    /** The same from a Java array (a texture whose upload was deferred until its slot was known). */
    public void uploadTexture(int slot, int format, int w, int h, byte[] texels) {
        try (Arena a = Arena.ofConfined()) {
            MemorySegment seg = a.allocateFrom(JAVA_BYTE, texels);
            check(call(() -> (int) UPLOAD_TEXTURE.invokeExact(ctx, slot, format, w, h, seg)), ctx);
        }
    }

    public void setCamera(float[] std140Block28) {
        if (std140Block28.length != 28) throw new IllegalArgumentException("camera block is 28 floats");
        try (Arena a = Arena.ofConfined()) {
            MemorySegment seg = a.allocateFrom(JAVA_FLOAT, std140Block28);
            check(call(() -> (int) SET_CAMERA.invokeExact(ctx, seg)), ctx);
        }
    }

    /** RaytraceExecutor.setSamplePerPixel's uniforms: sqrt_spp = (float) Math.sqrt(spp), its reciprocal. */
    public void setParams(int maxDepth, float[] background, int samplePerPixel) {
        float sqrtSpp = (float) Math.sqrt(samplePerPixel);
        try (Arena a = Arena.ofConfined()) {
            MemorySegment bg = a.allocateFrom(JAVA_FLOAT, background);
            check(call(() -> (int) SET_PARAMS.invokeExact(ctx, maxDepth, bg, sqrtSpp, 1f / sqrtSpp)), ctx);
        }
    }

    /** rt_set_bvh_mode: RT_BVH_REFERENCE (0, the default, bit-exact) or RT_BVH_SAH (1, the non-parity
     *  fast mode: a binned-SAH tree over the same prims; statistically equal images, not bit-exact). */
    public static final int BVH_REFERENCE = 0, BVH_SAH = 1;

    public void setBvhMode(int mode) {
        check(call(() -> (int) SET_BVH_MODE.invokeExact(ctx, mode)), ctx);
    }

    /** One process per GPU: this process renders the stripes s with s % world == rank. */
    public void setPartition(int rank, int world, int stripeRows) {
        check(call(() -> (int) SET_PARTITION.invokeExact(ctx, rank, world, stripeRows)), ctx);
        this.rank = rank;
        this.world = world;
        this.stripeRows = stripeRows;
    }

    public void resize(int w, int h) {
        check(call(() -> (int) RESIZE.invokeExact(ctx, w, h)), ctx);
        width = w;
        height = h;
    }

    /** Frames firstFrame, firstFrame+1, ... (frame_count), one u_rand_factor each. */
    public void render(int firstFrame, float[] randFactors) {
        int n = randFactors.length;
        try (Arena a = Arena.ofConfined()) {
            MemorySegment rf = a.allocateFrom(JAVA_FLOAT, randFactors);
            check(call(() -> (int) RENDER.invokeExact(ctx, firstFrame, n, rf)), ctx);
        }
    }

    public void sync() {
        check(call(() -> (int) SYNC.invokeExact(ctx)), ctx);
    }

    /** Device time of the last rt_render call, after it finished (waits for it). */
    public long lastRenderNanos() {
        sync();
        try (Arena a = Arena.ofConfined()) {
            MemorySegment ns = a.allocate(JAVA_LONG);
            check(call(() -> (int) LAST_NS.invokeExact(ctx, ns)), ctx);
            return ns.get(JAVA_LONG, 0);
        }
    }

    /** Device time of the last rt_render call if it has finished, else -1 (never waits). */
    public long renderDoneNanos() {
        try (Arena a = Arena.ofConfined()) {
            MemorySegment ns = a.allocate(JAVA_LONG);
            int rc = call(() -> (int) RENDER_DONE.invokeExact(ctx, ns));
            check(rc, ctx);
            return rc == 1 ? ns.get(JAVA_LONG, 0) : -1L;
        }
    }

    /**
     * width * height * 4 floats, row 0 = top (what Texture.saveAsPNG reads back); for a
     * partitioned context (setPartition) only this process's rows, stripe-compacted.
     */
    public float[] readImage() {
        int rows = world > 1 ? call(() -> (int) LOCAL_ROWS.invokeExact(height, rank, world, stripeRows)) : height;
        try (Arena a = Arena.ofConfined()) {
            MemorySegment rgba = a.allocate(JAVA_FLOAT, (long) width * rows * 4);
            check(call(() -> (int) READ_IMAGE.invokeExact(ctx, rgba)), ctx);
            return rgba.toArray(JAVA_FLOAT);   // copied to the heap before the arena closes
        }
    }

    /** Rank 0 of a one-process-per-GPU render: a fresh RCCL communicator id to hand to every rank. */
    public static byte[] commUniqueId() {
        try (Arena a = Arena.ofConfined()) {
            MemorySegment id = a.allocate(COMM_ID_BYTES);
            int rc = call(() -> (int) COMM_UNIQUE_ID.invokeExact(id));
            if (rc != 0) throw new IllegalStateException("rt_comm_unique_id failed (" + rc + "): RCCL unavailable");
            return id.toArray(JAVA_BYTE);
        }
    }

    /** Joins the RCCL communicator (after setPartition with the same rank / world). */
    public void commInit(byte[] id, int rank, int world) {
        if (id.length != COMM_ID_BYTES) throw new IllegalArgumentException("communicator id is 128 bytes");
        try (Arena a = Arena.ofConfined()) {
            MemorySegment seg = a.allocateFrom(JAVA_BYTE, id);
            check(call(() -> (int) COMM_INIT.invokeExact(ctx, seg, rank, world)), ctx);
        }
    }

    /** Every rank's stripes to rank 0 over RCCL: the full image there, null on the other ranks. */
    public float[] gatherImage() {
        if (rank != 0) {
            check(call(() -> (int) GATHER_IMAGE.invokeExact(ctx, MemorySegment.NULL)), ctx);
            return null;
        }
        try (Arena a = Arena.ofConfined()) {
            MemorySegment rgba = a.allocate(JAVA_FLOAT, (long) width * height * 4);
            check(call(() -> (int) GATHER_IMAGE.invokeExact(ctx, rgba)), ctx);
            return rgba.toArray(JAVA_FLOAT);
        }
    }

    /** Deadline of commInit / gatherImage in ms (0 = none; default 120000): past it they throw with
     *  RT_ERR_TIMEOUT (-6) and the communicator aborted, instead of waiting on a peer forever. */
    public void commSetTimeout(int timeoutMs) {
        check(call(() -> (int) COMM_SET_TIMEOUT.invokeExact(ctx, timeoutMs)), ctx);
    }

    /** Aborts the communicator and frees its queued work; the next gather needs commInit. */
    public void commAbort() {
        check(call(() -> (int) COMM_ABORT.invokeExact(ctx)), ctx);
    }

    /** How the last gather ran: 0 host, 1 peer copies, 2 RCCL; -1 before any. */
    public int gatherPath() {
        return call(() -> (int) GATHER_PATH.invokeExact(ctx));
    }

    public int width() {
        return width;
    }

    public int height() {
        return height;
    }

    @Override
    public void close() {
        call(() -> (int) DESTROY.invokeExact(ctx));
    }
}
