package net.bowen.system;

import net.bowen.draw.textures.Texture;

import java.awt.image.BufferedImage;
import java.io.File;
import java.io.IOException;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.nio.FloatBuffer;
import java.util.IdentityHashMap;
import java.util.List;
import java.util.Map;

import javax.imageio.ImageIO;

import static org.lwjgl.opengl.GL43.GL_FLOAT;
import static org.lwjgl.opengl.GL43.GL_RED;
import static org.lwjgl.opengl.GL43.GL_RGB;
import static org.lwjgl.opengl.GL43.GL_RGBA;
import static org.lwjgl.opengl.GL43.GL_RGBA32F;
import static org.lwjgl.opengl.GL43.GL_UNSIGNED_BYTE;

/**
 * The process's rt.h context behind the reference's GL call sites (the drop-in of
 * java/patches/rtamd-dropin.patch).  Each static method is what one patched call site
 * calls instead of its GL upload:
 * <ul>
 *   <li>{@link #upload}: RaytraceModel.put{Spheres,Quads,Boxes,ConstantMediums,BVHNodes,
 *       Lights}ToProgram, where they called {@code xxxSSBO.uploadData(buffer, GL_STATIC_DRAW)}
 *       (RaytraceModel.java:138-246);</li>
 *   <li>{@link #putTexture} / {@link #uploadTextures}: Texture.putData's glTexImage2D
 *       (Texture.java:122-133) and Texture.putTextureIndices (Texture.java:238-247): a texture's
 *       slot is its index in TEXTURES_IN_COMPUTE, known only once the scene registered it (image
 *       and Perlin textures upload in their constructors, before), so the bytes are kept until
 *       putTextureIndices, where the reference binds the slots too;</li>
 *   <li>{@link #setCamera}: Camera.putToShaderProgram's UBO upload and background uniform
 *       (Camera.java:121-143);</li>
 *   <li>{@link #get} / {@link #saveAsPNG} / {@link #preview}: Window's executor, image
 *       texture, PNG output and display (Window.java:199-238, 250-281).</li>
 * </ul>
 * Device: system property {@code rtamd.device} (default 0).  Reviewed only: no JDK here.
 */
public final class RtAmdBackend {
    private static RtAmd rt;
    private static float[] background = {0f, 0f, 0f};
    // texture -> (format, width, height, bytes) until its compute slot is known
    private static final Map<Texture, Object[]> PENDING = new IdentityHashMap<>();

    private RtAmdBackend() {
    }

    /** The context (created on first use). */
    public static synchronized RtAmd get() {
        if (rt == null) rt = new RtAmd(Integer.getInteger("rtamd.device", 0));
        return rt;
    }

    /** RaytraceModel.put*ToProgram: the packer's flipped std430 buffer for SSBO binding 0..5. */
    public static void upload(int binding, ByteBuffer buffer) {
        get().uploadBuffer(binding, buffer);
    }

    /**
     * Texture.putData's arguments.  The RGBA32F accumulation / display texture is never a
     * scene texture (those are GL_RGB8 and GL_R32F, Texture.java:179-229): not kept.
     */
    public static synchronized void putTexture(Texture texture, int internalFormat, int format, int type, int width,
                                               int height, ByteBuffer data) {
        if (data == null || internalFormat == GL_RGBA32F) return;
        int rtFormat;
        if (format == GL_RGB && type == GL_UNSIGNED_BYTE) rtFormat = RtAmd.TEX_RGB8;
        else if (format == GL_RGBA && type == GL_UNSIGNED_BYTE) rtFormat = RtAmd.TEX_RGBA8;
        else if (format == GL_RED && type == GL_FLOAT) rtFormat = RtAmd.TEX_R32F;
        else throw new IllegalArgumentException("texture format not supported by rt.h: " + format + "/" + type);
        byte[] bytes = new byte[data.remaining()];
        data.duplicate().get(bytes);
        PENDING.put(texture, new Object[]{rtFormat, width, height, bytes});
    }

    /** Texture.putTextureIndices: every scene texture to its slot (its index in the list). */
    public static synchronized void uploadTextures(List<Texture> texturesInCompute) {
        if (texturesInCompute.size() > 8) throw new IllegalStateException("compute.glsl has 8 texture slots");
        for (int slot = 0; slot < texturesInCompute.size(); slot++) {
            Object[] t = PENDING.get(texturesInCompute.get(slot));
            if (t == null) continue;   // not uploaded yet: putData will be followed by another putTextureIndices
            get().uploadTexture(slot, (int) t[0], (int) t[1], (int) t[2], (byte[]) t[3]);
        }
    }

    /** Camera.putToShaderProgram: the flipped 28-float std140 block and the background colour. */
    public static synchronized void setCamera(FloatBuffer ubo, float[] rgb) {
        float[] block = new float[28];
        ubo.duplicate().get(block);
        get().setCamera(block);
        background = rgb.clone();
    }

    public static synchronized float[] background() {
        return background.clone();
    }

    /**
     * Texture.saveAsPNG on the accumulated image: glGetTexImage's conversion (clamp to [0, 1],
     * round to unorm8) then the reference's per-byte gamma, (byte)(pow(b / 255, 1 / 2.2) * 255),
     * row 0 at the top (Texture.java:89-120).
     */
    public static String saveAsPNG(String filename) {
        RtAmd r = get();
        float[] rgba = r.readImage();
        int w = r.width(), h = r.height();
        BufferedImage image = new BufferedImage(w, h, BufferedImage.TYPE_INT_RGB);
        for (int y = 0; y < h; y++) {
            for (int x = 0; x < w; x++) {
                int i = (x + w * y) * 4, rgb = 0;
                for (int c = 0; c < 3; c++) {
                    float v = rgba[i + c];
                    v = Float.isNaN(v) ? 0f : Math.min(1f, Math.max(0f, v));
                    int b = Math.round(v * 255f);
                    int corrected = (byte) ((float) Math.pow(b / 255.0, 1.0 / 2.2) * 255.0f) & 0xFF;
                    rgb = (rgb << 8) | corrected;
                }
                image.setRGB(x, y, rgb);
            }
        }
        File out = new File(filename);
        try {
            ImageIO.write(image, "png", out);
        } catch (IOException e) {
            throw new RuntimeException("Failed to save the image as PNG", e);
        }
        return out.getAbsolutePath();
    }

    /** The progressive image into the display texture (the window shows it as the GL path did). */
    public static void preview(Texture displayTexture) {
        RtAmd r = get();
        float[] rgba = r.readImage();
        ByteBuffer buf = ByteBuffer.allocateDirect(rgba.length * 4).order(ByteOrder.nativeOrder());
        buf.asFloatBuffer().put(rgba);
        displayTexture.putData(r.width(), r.height(), buf);
    }
}
