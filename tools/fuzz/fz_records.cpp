// host fuzz driver: mutated scene records (boxes, spheres, quads, media, BVH) through the host-only
// C-ABI entries that build the compact box records, the fast (A/B) tables and the SAH BVH
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>
#include <string>
#include <vector>
#include "rt/rt_debug.h"
#include "rt/rt_types.h"
static std::vector<uint8_t> load(const std::string& p) {
    std::vector<uint8_t> b;
    FILE* f = std::fopen(p.c_str(), "rb");
    if (!f) return b;
    int ch;
    while ((ch = std::fgetc(f)) != EOF) b.push_back((uint8_t)ch);
    std::fclose(f);
    return b;
}
static void mutate(std::vector<uint8_t>& b, std::mt19937& rng, size_t rec) {
    if (b.empty()) return;
    const int muts = 1 + rng() % 8;
    for (int m = 0; m < muts; m++) {
        const size_t at = (rng() % b.size()) & ~(size_t)3;
        switch (rng() % 4) {
        case 0: b[at] = (uint8_t)rng(); break;
        case 1: { uint32_t v = rng() % 2048; std::memcpy(&b[at], &v, 4); break; }
        case 2: { float v = (float)((int)(rng() % 4000) - 2000) * 0.25f; std::memcpy(&b[at], &v, 4); break; }
        case 3: { const uint32_t s[4] = {0x7fc00000u, 0x7f800000u, 0xff800000u, 0x00000001u};
                  std::memcpy(&b[at], &s[rng() % 4], 4); break; }   // NaN, +-inf, a denormal
        }
    }
    if (rng() % 5 == 0 && b.size() > rec) b.resize((b.size() / rec - 1) * rec);
}
int main(int argc, char** argv) {
    const std::string dir = argv[1];
    const auto sph0 = load(dir + "/sph.bin"), quad0 = load(dir + "/quad.bin"), med0 = load(dir + "/med.bin"),
               box0 = load(dir + "/box.bin"), bvh0 = load(dir + "/bvh.bin");
    std::mt19937 rng(std::atoi(argv[2]));
    int ok = 0, err = 0;
    std::vector<uint8_t> out(64 << 20);
    std::vector<unsigned> info(1 << 20);
    std::vector<int> slots(4096);
    for (int it = 0; it < std::atoi(argv[3]); it++) {
        auto sph = sph0, quad = quad0, med = med0, box = box0, bvh = bvh0;
        const int which = rng() % 5;
        if (which == 0) mutate(sph, rng, sizeof(rt_sphere));
        if (which == 1) mutate(quad, rng, sizeof(rt_quad));
        if (which == 2) mutate(med, rng, sizeof(rt_medium));
        if (which == 3) mutate(box, rng, sizeof(rt_box));
        if (which == 4) mutate(bvh, rng, sizeof(rt_bvh_node));
        int nc = 0, nper = 0, nslot = 0;
        size_t nb = 0;
        int r = rt_debug_box_records(box.data(), box.size(), out.data(), out.size(), &nc);
        r |= rt_debug_fast_tables(bvh.data(), bvh.size(), quad.data(), quad.size(), box.data(), box.size(),
                                  (int)(sph.size() / sizeof(rt_sphere)), out.data(), out.size(), &nper, info.data(),
                                  info.size(), slots.data(), &nslot) < 0;
        const float eye[3] = {478.0f, 278.0f, -600.0f};
        r |= rt_debug_build_sah_bvh(sph.data(), sph.size(), quad.data(), quad.size(), med.data(), med.size(),
                                    box.data(), box.size(), bvh.data(), bvh.size(), (int)(rng() % 3), eye, 1.0f,
                                    out.data(), out.size(), &nb);
        (r ? err : ok)++;
    }
    std::printf("ok %d err %d\n", ok, err);
}
