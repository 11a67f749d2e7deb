// host fuzz driver: random worlds through the scene builder's C API (rt_scene.h: the reference's
// Scene.java builder calls) -- random and non-finite parameters, bad handles, empty worlds -- then
// rts_finish (BVH build, packers, camera) and the getters.
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <random>
#include <vector>
#include "rt/rt_scene.h"
int main(int argc, char** argv) {
    std::mt19937 rng(std::atoi(argv[1]));
    const int iters = std::atoi(argv[2]);
    auto val = [&]() -> float {
        switch (rng() % 12) {
        case 0: return NAN;
        case 1: return INFINITY;
        case 2: return -INFINITY;
        case 3: return 0.0f;
        case 4: return 1e30f;
        default: return (float)((int)(rng() % 2001) - 1000) * 0.5f;
        }
    };
    int ok = 0, err = 0;
    for (int it = 0; it < iters; it++) {
        rts_scene* s = nullptr;
        if (rts_new(rng(), nullptr, &s)) return 3;
        std::vector<int> mats, models;
        int tex = 0, h = 0;
        for (int k = 0; k < 4; k++) {
            float c1[3] = {val(), val(), val()}, c2[3] = {val(), val(), val()};
            if (rts_solid_texture(s, val(), val(), val(), &tex) == 0) {
                const float emit[3] = {val(), val(), val()};
                if (rts_material(s, (int)(rng() % 6), rng() % 3 ? tex : (int)rng(), val(), emit, &h) == 0) mats.push_back(h);
            }
            if (rts_checker_texture(s, c1, c2, val(), &tex) == 0 && rts_material(s, 0, tex, 0.0f, c1, &h) == 0)
                mats.push_back(h);
            if (rng() % 3 == 0 && rts_perlin_texture(s, val(), &tex) == 0 && rts_material(s, 4, tex, 0.0f, c1, &h) == 0)
                mats.push_back(h);
        }
        const int n = (int)(rng() % 40);
        for (int k = 0; k < n; k++) {
            const int mat = mats.empty() || rng() % 10 == 0 ? (int)rng() % 100 : mats[rng() % mats.size()];
            float a[3] = {val(), val(), val()}, b[3] = {val(), val(), val()}, c[3] = {val(), val(), val()};
            float r[3] = {val(), val(), val()};
            int rc = 1;
            switch (rng() % 5) {
            case 0: rc = rts_sphere(s, a, rng() % 2 ? b : nullptr, val(), mat, &h); break;
            case 1: rc = rts_quad(s, a, b, c, mat, &h); break;
            case 2: rc = rts_box(s, a, b, rng() % 2 ? c : nullptr, rng() % 2 ? r : nullptr, mat, &h); break;
            case 3:
                if (!models.empty()) rc = rts_constant_medium(s, models[rng() % models.size()], val(), mat, &h);
                break;
            case 4: rc = rts_sphere(s, a, nullptr, (float)(rng() % 100) + 0.5f, mat, &h); break;
            }
            if (rc == 0) {
                models.push_back(h);
                if (rng() % 4) rts_add_model(s, rng() % 20 ? h : (int)rng());
                if (rng() % 8 == 0) rts_add_light(s, h);
            }
        }
        rts_camera_params cp{};
        for (int k = 0; k < 3; k++) {
            cp.look_from[k] = val();
            cp.look_at[k] = val();
            cp.vup[k] = val();
        }
        cp.vfov = val();
        cp.defocus_angle = val();
        cp.focus_dist = val();
        rts_camera(s, &cp);
        const int w = 1 + (int)(rng() % 64), hh = 1 + (int)(rng() % 64);
        int rc = rts_finish(s, w, hh);
        if (rc == 0) {
            rts_info info;
            rts_get_info(s, &info);
            for (int b = 0; b < 6; b++) {
                const void* p = nullptr;
                size_t nb = 0;
                rts_get_buffer(s, b, &p, &nb);
            }
            float ubo[28];
            rts_get_camera(s, ubo);
            rts_set_image_size(s, 1 + (int)(rng() % 100), 1 + (int)(rng() % 100));
        }
        (rc ? err : ok)++;
        rts_free(s);
    }
    std::printf("ok %d err %d\n", ok, err);
}
