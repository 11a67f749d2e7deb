package net.bowen.system;

import java.util.ArrayList;
import java.util.List;
import java.util.concurrent.TimeUnit;

/**
 * The reference's RaytraceExecutor (RaytraceExecutor.java:16-157) over {@link RtAmd}
 * instead of OpenGL: the same public methods, the same per-frame uniforms
 * (frame_count = ++numSamples, u_rand_factor = (float) Math.random(), :124-127) and
 * the same completion bookkeeping, with the dispatch, the memory barrier and the
 * GL_TIME_ELAPSED query replaced by rt_render / rt_render_done / rt_last_render_ns.
 *
 * <p>Drop-in: Window.initRaytraceExecutor constructs this instead of
 * {@code new RaytraceExecutor(quadTexture, program)}; the frame loop
 * (Window.java:250-281) still calls {@link #raytrace()} once per frame and
 * {@link #sampleComplete()}.  {@link #raytrace(int)} queues n frames in one launch,
 * which is how the MI355X kernel is meant to be fed (one dispatch per vsync caps
 * the reference at the display rate, BASELINE.md section 1).
 *
 * <p>Reviewed only: this image has no JDK.
 */
public class RtAmdRaytraceExecutor {
    private final RtAmd rt;
    private final List<Runnable> completeListeners = new ArrayList<>();
    private int maxDepth = 5;
    private float[] background = {0f, 0f, 0f};

    private int numSamples;
    private long startMillis;
    private int finishTime = -1;
    private int lastDispatchTime;
    private boolean isSampleComplete;
    private int samplePerPixel;

    public RtAmdRaytraceExecutor(RtAmd rt) {
        this.rt = rt;
    }

    /** GuiRenderer.maxDepthUpdate / Camera.setBackground feed these; they travel with rt_set_params. */
    public void setMaxDepth(int maxDepth) {
        this.maxDepth = maxDepth;
        rt.setParams(maxDepth, background, samplePerPixel);
    }

    public void setBackground(float[] rgb) {
        this.background = rgb.clone();
        rt.setParams(maxDepth, background, samplePerPixel);
    }

    public void setSamplePerPixel(int samplePerPixel) {
        this.samplePerPixel = samplePerPixel;
        rt.setParams(maxDepth, background, samplePerPixel);   // sqrt_spp and its reciprocal
    }

    public void resetCompleteState() {
        isSampleComplete = false;
        numSamples = 0;
        finishTime = -1;
    }

    public int getNumSamples() {
        return numSamples;
    }

    public int getSamplePerPixel() {
        return samplePerPixel;
    }

    public int getFinishTime() {
        return finishTime;
    }

    public String getFinishTimeString() {
        long hours = TimeUnit.MILLISECONDS.toHours(finishTime);
        long minutes = TimeUnit.MILLISECONDS.toMinutes(finishTime) % 60;
        long seconds = TimeUnit.MILLISECONDS.toSeconds(finishTime) % 60;
        StringBuilder sb = new StringBuilder();
        if (hours > 0) sb.append(hours).append("hour ");
        if (minutes > 0) sb.append(minutes).append("minutes ");
        return sb.append(seconds).append('.').append(finishTime % 1000).append("seconds").toString();
    }

    /**
     * Milliseconds of the last finished rt_render call (the reference truncates its timer
     * query to int ms), refreshed by every raytrace() as the GUI status line expects.
     */
    public int getLastDispatchTime() {
        return lastDispatchTime;
    }

    public void addCompleteListener(Runnable l) {
        completeListeners.add(l);
    }

    /** One frame, as the reference's raytrace() (unclamped, like the reference's). */
    public void raytrace() {
        launch(1);
    }

    /**
     * Up to n frames in one launch: frame_count numSamples+1 .. numSamples+k, one
     * Math.random() each, where k = n clamped to the frames still missing from
     * samplePerPixel (when one is set).  The reference renders exactly samplePerPixel
     * frames, one raytrace() per loop iteration while !sampleComplete()
     * (RaytraceExecutor.java:100-156, Window.java:250-281), so a caller queueing
     * FRAMES_PER_DISPLAY frames at a time must not run past it: with spp 20 and 16 per
     * display the launches are 16 then 4 (rtamd/render.py and rt_main.cpp clamp the same way).
     * Returns the number of frames queued.
     */
    public int raytrace(int n) {
        return launch(clampFrames(n, numSamples, samplePerPixel));
    }

    /** The frames raytrace(n) queues after numSamples of samplePerPixel (0 = unbounded). */
    static int clampFrames(int n, int numSamples, int samplePerPixel) {
        if (samplePerPixel > 0) n = Math.min(n, samplePerPixel - numSamples);
        return Math.max(n, 0);
    }

    private int launch(int n) {
        if (n <= 0) return 0;
        if (numSamples == 0) startMillis = System.currentTimeMillis();
        // as the reference does with its finished QueryTimers (RaytraceExecutor.java:106-115): the
        // previous call's device time once it is available, never waiting for it
        if (numSamples > 0) {
            long ns = rt.renderDoneNanos();
            if (ns >= 0) lastDispatchTime = (int) (ns / 1_000_000L);
        }
        float[] factors = new float[n];
        for (int i = 0; i < n; i++) factors[i] = (float) Math.random();
        rt.render(numSamples + 1, factors);
        numSamples += n;
        return n;
    }

    public boolean sampleComplete() {
        if (!isSampleComplete && numSamples >= samplePerPixel) {
            isSampleComplete = true;
            lastDispatchTime = (int) (rt.lastRenderNanos() / 1_000_000L);   // waits for the device
            finishTime = (int) (System.currentTimeMillis() - startMillis);
            for (Runnable l : completeListeners) l.run();
        }
        return isSampleComplete;
    }
}
