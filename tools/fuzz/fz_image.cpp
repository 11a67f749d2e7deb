#include <cstdio>
#include <cstdint>
#include <cstddef>
#include <vector>
extern "C" int rts_decode_image(const char*, int*, int*, int*, uint8_t*, size_t);
int main(int argc, char** argv) {
    int ok = 0, err = 0;
    for (int i = 1; i < argc; i++) {
        int w, h, c;
        if (rts_decode_image(argv[i], &w, &h, &c, nullptr, 0)) { err++; continue; }
        std::vector<uint8_t> px((size_t)w * h * c);
        if (rts_decode_image(argv[i], &w, &h, &c, px.data(), px.size())) err++; else ok++;
    }
    printf("ok %d err %d\n", ok, err);
}
