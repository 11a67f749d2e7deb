// rt_main.cpp — `rtrender`, the command-line front end of the reference
// (src/main/java/net/bowen/Main.java:6-70) over the rt.h / rt_scene.h C ABIs.
//
// Same options, defaults and error behaviour as the reference's commons-cli
// parser:
//   -h,--help  -s,--scene <id>=0  -r,--resolution <W:H>=500:300
//   -spp,--sample-per-pixel <n>=20  -md,--max-depth <n>=5  -o,--output <png>
// A parse error prints the parser message and the help text and exits 1
// (Main.java:16-20); a non-integer value exits 1 with the message of the
// NumberFormatException Integer.parseInt throws; an unknown scene id exits 1
// with "Invalid scene ID: <id>" (Scene.java:29).
//
// Where the reference opens a window and dispatches one frame per vsync until
// samplePerPixel frames are done (Window.java:250-281, RaytraceExecutor.java:
// 100-156), rtrender queues the frames in batches of --frames-per-launch on the
// MI355X (rt_render), then runs the completion listeners of Window.java:213-233:
// "All samples have completed in ..." and, with -o, Texture.saveAsPNG.
//
// MI355X-only options (no reference counterpart): --seed (scene + per-frame
// factor seed; the reference uses the unseeded Math.random), --devices
// (comma-separated HIP device ids, rows striped across them), --frames-per-launch.
//
// Progressive preview, the headless form of the window loop
// (Window.java:250-281): --preview <png> rewrites that PNG with the running mean
// every --preview-every frames (drawResult: the image so far, through
// Texture.saveAsPNG) and prints GuiRenderer.draw's status lines
// (GuiRenderer.java:48-62): "Last raytrace took: <ms> ms." and
// "Sample: <n>/<spp>." (+ "Render completed in: ..." once complete).
#include "rt/rt.h"
#include "rt/rt_scene.h"

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <limits.h>
#include <stdlib.h>

namespace {

struct Opt {
    const char* shrt;
    const char* lng;
    bool has_arg;
    const char* desc;
};

// commons-cli Options in Main.getOptions order (Main.java:43-70)
enum { O_HELP, O_SCENE, O_RES, O_SPP, O_DEPTH, O_OUT, O_SEED, O_DEVICES, O_PER_LAUNCH, O_PREVIEW, O_PREVIEW_EVERY, O_N };
const Opt kOpts[O_N] = {
    {"h", "help", false, "print help message"},
    {"s", "scene", true, "scene ID"},
    {"r", "resolution", true, "screen resolution"},
    {"spp", "sample-per-pixel", true, "sample per pixel"},
    {"md", "max-depth", true, "max depth"},
    {"o", "output", true, "output file (must be a .png file)"},
    // MI355X extensions
    {nullptr, "seed", true, "scene and frame RNG seed (default 1)"},
    {nullptr, "devices", true, "comma-separated HIP device ids (default 0)"},
    {nullptr, "frames-per-launch", true, "frames per kernel launch (default 64)"},
    {nullptr, "preview", true, "progressive preview PNG, rewritten every --preview-every frames"},
    {nullptr, "preview-every", true, "frames between preview updates (default: --frames-per-launch)"},
};

// HelpFormatter.printHelp("OpenGL Ray Tracer", options): options sorted by key.
void print_help() {
    std::vector<std::string> left(O_N);
    size_t width = 0;
    for (int i = 0; i < O_N; i++) {
        std::string l = " ";
        l += kOpts[i].shrt ? std::string("-") + kOpts[i].shrt + "," : std::string("   ");
        l += std::string("--") + kOpts[i].lng;
        if (kOpts[i].has_arg) l += " <arg>";
        left[i] = l;
        width = std::max(width, l.size());
    }
    std::vector<int> order(O_N);
    for (int i = 0; i < O_N; i++) order[i] = i;
    auto key = [](int i) { return std::string(kOpts[i].shrt ? kOpts[i].shrt : kOpts[i].lng); };
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return key(a) < key(b); });
    std::printf("usage: OpenGL Ray Tracer\n");
    for (int i : order) std::printf("%-*s   %s\n", (int)width, left[i].c_str(), kOpts[i].desc);
}

[[noreturn]] void parse_fail(const std::string& msg) {
    std::printf("%s\n", msg.c_str());
    print_help();
    std::exit(1);
}

// The reference reports these as uncaught Java exceptions (exit status 1).
[[noreturn]] void uncaught(const char* cls, const std::string& msg) {
    std::fprintf(stderr, "Exception in thread \"main\" %s: %s\n", cls, msg.c_str());
    std::exit(1);
}

// Integer.parseInt: optional sign, decimal digits, 32-bit range.
int parse_int(const std::string& s) {
    bool ok = !s.empty();
    size_t i = (ok && (s[0] == '-' || s[0] == '+')) ? 1 : 0;
    if (i == s.size()) ok = false;
    long long v = 0;
    for (size_t k = i; ok && k < s.size(); k++) {
        if (s[k] < '0' || s[k] > '9') ok = false;
        else if ((v = v * 10 + (s[k] - '0')) > (long long)INT_MAX + 1) ok = false;
    }
    if (ok && s[0] == '-') v = -v;
    if (!ok || v > INT_MAX || v < INT_MIN) uncaught("java.lang.NumberFormatException", "For input string: \"" + s + "\"");
    return (int)v;
}

// RaytraceExecutor.getFinishTimeString (RaytraceExecutor.java:76-89)
std::string finish_time_string(int finish_ms) {
    long long ms = finish_ms;
    long long hours = ms / 3600000, minutes = (ms / 60000) % 60, seconds = (ms / 1000) % 60;
    std::string s;
    if (hours > 0) s += std::to_string(hours) + "hour ";
    if (minutes > 0) s += std::to_string(minutes) + "minutes ";
    s += std::to_string(seconds) + "." + std::to_string(finish_ms % 1000) + "seconds";
    return s;
}

[[noreturn]] void die(const char* what, const char* msg) {
    std::fprintf(stderr, "%s: %s\n", what, msg ? msg : "");
    std::exit(1);
}

}  // namespace

int main(int argc, char** argv) {
    // commons-cli DefaultParser: "-x v", "-xv" (value attached to a short
    // option), "--long v", "--long=v"; an unknown "-..." token is an error.
    std::string val[O_N];
    bool seen[O_N] = {};
    for (int i = 1; i < argc; i++) {
        std::string t = argv[i];
        if (t.size() < 2 || t[0] != '-') continue;   // stray arguments land in cmd.getArgs()
        int hit = -1;
        std::string attached;
        bool has_attached = false;
        if (t.rfind("--", 0) == 0) {
            std::string name = t.substr(2);
            size_t eq = name.find('=');
            if (eq != std::string::npos) {
                attached = name.substr(eq + 1);
                has_attached = true;
                name = name.substr(0, eq);
            }
            for (int k = 0; k < O_N; k++)
                if (name == kOpts[k].lng) hit = k;
        } else {
            std::string name = t.substr(1);
            for (int k = 0; k < O_N; k++)
                if (kOpts[k].shrt && name == kOpts[k].shrt) hit = k;
            if (hit < 0)   // "-s8": the longest value-taking short option that prefixes the token
                for (int k = 0; k < O_N; k++)
                    if (kOpts[k].shrt && kOpts[k].has_arg && name.rfind(kOpts[k].shrt, 0) == 0 &&
                        (hit < 0 || std::strlen(kOpts[k].shrt) > std::strlen(kOpts[hit].shrt))) {
                        hit = k;
                        attached = name.substr(std::strlen(kOpts[k].shrt));
                        has_attached = true;
                    }
        }
        if (hit < 0) parse_fail("Unrecognized option: " + t);
        seen[hit] = true;
        if (!kOpts[hit].has_arg) continue;
        if (has_attached) {
            val[hit] = attached;
        } else if (i + 1 < argc && !(argv[i + 1][0] == '-' && argv[i + 1][1] != '\0')) {
            val[hit] = argv[++i];
        } else {
            parse_fail(std::string("Missing argument for option: ") + (kOpts[hit].shrt ? kOpts[hit].shrt : kOpts[hit].lng));
        }
    }
    if (seen[O_HELP]) {
        print_help();
        return 0;
    }
    auto get = [&](int k, const char* def) { return seen[k] ? val[k] : std::string(def ? def : ""); };

    // Main.java:30-38
    std::string res = get(O_RES, "500:300");
    size_t colon = res.find(':');
    int width = parse_int(res.substr(0, colon));
    if (colon == std::string::npos)
        uncaught("java.lang.ArrayIndexOutOfBoundsException", "Index 1 out of bounds for length 1");
    size_t colon2 = res.find(':', colon + 1);
    int height = parse_int(res.substr(colon + 1, colon2 == std::string::npos ? std::string::npos : colon2 - colon - 1));
    int scene_id = parse_int(get(O_SCENE, "0"));
    int spp = parse_int(get(O_SPP, "20"));
    int max_depth = parse_int(get(O_DEPTH, "5"));
    std::string output = get(O_OUT, nullptr);
    long long seed = parse_int(get(O_SEED, "1"));
    int per_launch = parse_int(get(O_PER_LAUNCH, "64"));
    std::vector<int> devices;
    {
        std::string d = get(O_DEVICES, "0");
        size_t p = 0;
        while (p <= d.size()) {
            size_t q = d.find(',', p);
            if (q == std::string::npos) q = d.size();
            devices.push_back(parse_int(d.substr(p, q - p)));
            p = q + 1;
        }
    }
    // Scene.java:19-30; scene 9 is the build's Book-1 three-sphere scene
    if (scene_id < 0 || scene_id > 9)
        uncaught("java.lang.IllegalArgumentException", "Invalid scene ID: " + std::to_string(scene_id));
    if (width <= 0 || height <= 0) die("rtrender", "resolution must be positive");
    if (per_launch <= 0) die("rtrender", "--frames-per-launch must be positive");
    const std::string preview = get(O_PREVIEW, nullptr);
    const int preview_every = seen[O_PREVIEW_EVERY] ? parse_int(val[O_PREVIEW_EVERY]) : per_launch;
    if (preview_every <= 0) die("rtrender", "--preview-every must be positive");

    rts_scene* scene = nullptr;
    if (rts_build(scene_id, width, height, (uint64_t)seed, nullptr, &scene) != 0) die("rts_build", rts_last_error());
    rts_info info;
    rts_get_info(scene, &info);

    rt_ctx* ctx = nullptr;
    if (rt_create((int)devices.size(), devices.data(), &ctx) != 0) die("rt_create", rt_last_error(nullptr));
    auto chk = [&](int rc, const char* what) {
        if (rc != 0) die(what, rt_last_error(ctx));
    };
    // RaytraceModel.putModelsToProgram, Texture.putData, Camera.init
    for (int b = 0; b < 6; b++) {
        const void* p = nullptr;
        size_t n = 0;
        rts_get_buffer(scene, b, &p, &n);
        chk(rt_upload_buffer(ctx, b, p, n), "rt_upload_buffer");
    }
    for (int s = 0; s < info.n_textures; s++) {
        int fmt = 0, w = 0, h = 0;
        const void* p = nullptr;
        size_t n = 0;
        rts_get_texture(scene, s, &fmt, &w, &h, &p, &n);
        chk(rt_upload_texture(ctx, s, fmt, w, h, p), "rt_upload_texture");
    }
    float ubo[28];
    rts_get_camera(scene, ubo);
    chk(rt_set_camera(ctx, ubo), "rt_set_camera");
    float sqrt_spp, recip;
    rts_spp_uniforms(spp, &sqrt_spp, &recip);   // RaytraceExecutor.setSamplePerPixel
    chk(rt_set_params(ctx, max_depth, info.background, sqrt_spp, recip), "rt_set_params");
    chk(rt_resize(ctx, width, height), "rt_resize");

    // RaytraceExecutor.raytrace x samplePerPixel, batched per launch
    auto t0 = std::chrono::steady_clock::now();
    std::vector<float> rf((size_t)per_launch);
    uint64_t device_ns = 0;
    std::vector<float> rgba;
    for (int f0 = 0; f0 < spp;) {
        int n = std::min(per_launch, spp - f0);
        if (!preview.empty()) n = std::min(n, preview_every - f0 % preview_every);   // stop at the next preview
        for (int i = 0; i < n; i++) rf[i] = rt_frame_rand_factor((uint64_t)seed, (uint64_t)(f0 + i));
        chk(rt_render(ctx, f0 + 1, n, rf.data()), "rt_render");
        chk(rt_sync(ctx), "rt_sync");
        uint64_t ns = 0;
        chk(rt_last_render_ns(ctx, &ns), "rt_last_render_ns");
        device_ns += ns;
        f0 += n;
        if (!preview.empty() && (f0 % preview_every == 0 || f0 == spp)) {
            // one pass of the window loop: drawResult + GuiRenderer.draw
            rgba.resize((size_t)width * height * 4);
            chk(rt_read_image(ctx, rgba.data()), "rt_read_image");
            if (rts_save_png(rgba.data(), width, height, preview.c_str()) != 0)
                uncaught("java.lang.RuntimeException", "Failed to save texture as PNG");
            std::printf("Last raytrace took: %d ms.\n", (int)(ns / 1000000));
            std::printf("Sample: %d/%d.", f0, spp);
            if (f0 == spp) {
                const int ms = (int)std::chrono::duration_cast<std::chrono::milliseconds>(
                                   std::chrono::steady_clock::now() - t0).count();
                std::printf("Render completed in: %s.", finish_time_string(ms).c_str());
            }
            std::printf("\n");
            std::fflush(stdout);
        }
    }
    int finish_ms = (int)std::chrono::duration_cast<std::chrono::milliseconds>(
                        std::chrono::steady_clock::now() - t0).count();
    std::printf("All samples have completed in %s.\n", finish_time_string(finish_ms).c_str());
    if (device_ns > 0)
        std::printf("device time %.3f ms, %.1f Msamples/s (scene %d, %dx%d, %d spp, max_depth %d, %zu device(s))\n",
                    device_ns * 1e-6, (double)width * height * spp / (device_ns * 1e-9) * 1e-6, scene_id, width,
                    height, spp, max_depth, devices.size());

    if (!output.empty()) {   // Window.saveImage (Window.java:227-233)
        std::printf("Saving the result to %s...\n", output.c_str());
        std::vector<float> rgba((size_t)width * height * 4);
        chk(rt_read_image(ctx, rgba.data()), "rt_read_image");
        if (rts_save_png(rgba.data(), width, height, output.c_str()) != 0)
            uncaught("java.lang.RuntimeException", "Failed to save texture as PNG");
        char abs_path[PATH_MAX];
        const char* shown = realpath(output.c_str(), abs_path) ? abs_path : output.c_str();
        std::printf("A PNG file has been saved to: %s\n", shown);
    }
    rt_destroy(ctx);
    rts_free(scene);
    return 0;
}
