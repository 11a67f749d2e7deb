#!/bin/bash
# Compares the working tree's rt_glsl.h g_sincos / g_log with a previous revision's, bit for bit,
# on every 7th float bit pattern (~614 M inputs, ~2 min) and the edge values: a rewrite of a
# built-in (e.g. round 3's branch-free quadrant and special cases) must not change one result.
# usage: tools/glsl_equiv.sh [rev]   (default HEAD)
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" show "$REV:include/rt/rt_glsl.h" | sed 's/RT_GLSL_H/RT_GLSL_OLD_H/g' > "$TMP/old.h"
cat > "$TMP/chk.cpp" <<'CPP'
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include "rt/rt_glsl.h"
namespace old {
#include "old.h"
}
static uint32_t b(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static int same(float x) {
    float s1, c1, s2, c2;
    g_sincos(x, &s1, &c1);
    old::g_sincos(x, &s2, &c2);
    return b(s1) == b(s2) && b(c1) == b(c2) && b(g_log(x)) == b(old::g_log(x));
}
int main() {
    unsigned long long n = 0, bad = 0;
    for (uint64_t i = 0; i < (1ull << 32); i += 7) {
        float x; uint32_t u = (uint32_t)i; memcpy(&x, &u, 4);
        n++;
        if (!same(x) && bad++ < 5) printf("differs at 0x%08x\n", u);
    }
    const float edge[] = {2147483520.0f, 3.3732712e9f, 3.4028235e38f, -3.4028235e38f, INFINITY, -INFINITY,
                          NAN, 0.0f, -0.0f, 1e-45f, 1.1754942e-38f};
    for (float x : edge) { n++; if (!same(x) && bad++ < 5) printf("differs at %g\n", x); }
    printf("%llu inputs, %llu differ\n", n, bad);
    return bad != 0;
}
CPP
g++ -O2 -ffp-contract=off -I"$ROOT/include" -I"$TMP" -o "$TMP/chk" "$TMP/chk.cpp"
"$TMP/chk"
rm -rf "$TMP"
