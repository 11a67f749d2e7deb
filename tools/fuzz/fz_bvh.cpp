// host fuzz driver: random / mutated BVH node arrays through the C ABI's host-only debug entries
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>
#include <vector>
#include "rt/rt_debug.h"
#include "rt/rt_types.h"
int main(int argc, char** argv) {
    FILE* f = std::fopen(argv[1], "rb");
    std::vector<uint8_t> base;
    int ch;
    while ((ch = std::fgetc(f)) != EOF) base.push_back((uint8_t)ch);
    std::fclose(f);
    float cam[28];
    f = std::fopen(argv[2], "rb");
    if (std::fread(cam, 4, 28, f) != 28) return 2;
    std::fclose(f);
    std::mt19937 rng(std::atoi(argv[3]));
    const size_t rec = sizeof(rt_bvh_node);
    int ok = 0, err = 0;
    std::vector<uint8_t> out(64 << 20), drop(1 << 20);
    for (int it = 0; it < std::atoi(argv[4]); it++) {
        std::vector<uint8_t> b = base;
        const int muts = 1 + rng() % 12;
        for (int m = 0; m < muts; m++) {
            const size_t at = rng() % b.size();
            switch (rng() % 4) {
            case 0: b[at] = (uint8_t)rng(); break;                     // a byte
            case 1: { uint32_t v = rng() % 4096; std::memcpy(&b[at & ~(size_t)3], &v, 4); break; }   // an index-like word
            case 2: { float v = (float)((int)(rng() % 2000) - 1000); std::memcpy(&b[at & ~(size_t)3], &v, 4); break; }
            case 3: b.resize(std::max<size_t>(rec, (b.size() / rec - rng() % 4) * rec)); break;   // drop nodes
            }
        }
        int n = 0, nf = 0, nd = 0;
        int r1 = rt_debug_threaded_bvh(b.data(), b.size(), out.data(), out.size(), &n);
        int r2 = rt_debug_link_nodes(b.data(), b.size(), out.data(), out.size(), &nf);
        int r3 = rt_debug_collapse_links(b.data(), b.size(), cam, 96, 54, 1 + (int)(rng() % 2), out.data(), out.size(), &nf,
                                         drop.data(), drop.size(), &nd);
        ((r1 | r2 | r3) ? err : ok)++;
    }
    std::printf("ok %d err %d\n", ok, err);
}
