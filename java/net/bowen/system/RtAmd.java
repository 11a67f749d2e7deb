package net.bowen.system;

import java.lang.foreign.Arena;
import java.lang.foreign.FunctionDescriptor;
import java.lang.foreign.Linker;
import java.lang.foreign.MemorySegment;
import java.lang.foreign.SymbolLookup;
import java.lang.invoke.MethodHandle;
import java.nio.ByteBuffer;

import static java.lang.foreign.ValueLayout.ADDRESS;
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
 *   <li>{@link #lastRenderNanos}: the GL_TIME_ELAPSED query (QueryTimer.java).</li>
 * </ul>
 * Reviewed only: this image has no JDK.  The same contract is exercised from Python
 * (raytracing-book_amd/rtamd/_lib.py) by the tests.
 */
public final class RtAmd implements AutoCloseable {
    /** rt.h bindings (compute.glsl:127-153). */
    public static final int SPHERES = 0, BVH = 1, QUADS = 2, MEDIA = 3, BOXES = 4, LIGHTS = 5;
    /** rt.h texture formats. */
    public static final int TEX_RGB8 = 1, TEX_RGBA8 = 2, TEX_R32F = 3;

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
    private static final MethodHandle RENDER = fn("rt_render", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT, ADDRESS));
    private static final MethodHandle SYNC = fn("rt_sync", FunctionDescriptor.of(JAVA_INT, ADDRESS));
    private static final MethodHandle READ_IMAGE = fn("rt_read_image", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));
    private static final MethodHandle LAST_NS = fn("rt_last_render_ns", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));

    private final Arena arena = Arena.ofConfined();
    private final MemorySegment ctx;
    private int width, height;

    /** rt_create on one device (RaytraceModel.initSSBOs + the GL context setup). */
    public RtAmd(int device) {
        MemorySegment ids = arena.allocateFrom(JAVA_INT, device);
        MemorySegment out = arena.allocate(ADDRESS);
        check(call(() -> (int) CREATE.invokeExact(1, ids, out)), MemorySegment.NULL);
        ctx = out.get(ADDRESS, 0);
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
        if (rc == 0) return;
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

    public void setCamera(float[] std140Block28) {
        if (std140Block28.length != 28) throw new IllegalArgumentException("camera block is 28 floats");
        MemorySegment seg = arena.allocateFrom(JAVA_FLOAT, std140Block28);
        check(call(() -> (int) SET_CAMERA.invokeExact(ctx, seg)), ctx);
    }

    /** RaytraceExecutor.setSamplePerPixel's uniforms: sqrt_spp = (float) Math.sqrt(spp), its reciprocal. */
    public void setParams(int maxDepth, float[] background, int samplePerPixel) {
        float sqrtSpp = (float) Math.sqrt(samplePerPixel);
        MemorySegment bg = arena.allocateFrom(JAVA_FLOAT, background);
        check(call(() -> (int) SET_PARAMS.invokeExact(ctx, maxDepth, bg, sqrtSpp, 1f / sqrtSpp)), ctx);
    }

    /** One process per GPU: this process renders the stripes s with s % world == rank. */
    public void setPartition(int rank, int world, int stripeRows) {
        check(call(() -> (int) SET_PARTITION.invokeExact(ctx, rank, world, stripeRows)), ctx);
    }

    public void resize(int w, int h) {
        check(call(() -> (int) RESIZE.invokeExact(ctx, w, h)), ctx);
        width = w;
        height = h;
    }

    /** Frames firstFrame, firstFrame+1, ... (frame_count), one u_rand_factor each. */
    public void render(int firstFrame, float[] randFactors) {
        MemorySegment rf = arena.allocateFrom(JAVA_FLOAT, randFactors);
        int n = randFactors.length;
        check(call(() -> (int) RENDER.invokeExact(ctx, firstFrame, n, rf)), ctx);
    }

    public void sync() {
        check(call(() -> (int) SYNC.invokeExact(ctx)), ctx);
    }

    /** Device time of the last rt_render call, after it finished. */
    public long lastRenderNanos() {
        MemorySegment ns = arena.allocate(JAVA_LONG);
        sync();
        check(call(() -> (int) LAST_NS.invokeExact(ctx, ns)), ctx);
        return ns.get(JAVA_LONG, 0);
    }

    /** width * height * 4 floats, row 0 = top (what Texture.saveAsPNG reads back). */
    public float[] readImage() {
        MemorySegment rgba = arena.allocate(JAVA_FLOAT, (long) width * height * 4);
        check(call(() -> (int) READ_IMAGE.invokeExact(ctx, rgba)), ctx);
        return rgba.toArray(JAVA_FLOAT);
    }

    @Override
    public void close() {
        call(() -> (int) DESTROY.invokeExact(ctx));
        arena.close();
    }
}
