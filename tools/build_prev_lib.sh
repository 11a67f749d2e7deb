#!/bin/bash
# Builds raytracing-book_amd/lib/prev/librtamd.so from a previous revision's kernel source
# and built-ins (default HEAD) and the working tree's C ABI, for tools/lib_ab.py.  The two kernels must
# share rt_device.h's argument layout.  usage: tools/build_prev_lib.sh [rev]
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/raytracing-book_amd
TMP=$(mktemp -d)
git -C "$ROOT" show "$REV:raytracing-book_amd/csrc/rt_kernel.hip" > "$TMP/rt_kernel.hip"
# the shared device code (round 5 on): found beside the kernel source before the working tree's
git -C "$ROOT" show "$REV:raytracing-book_amd/csrc/rt_kernel_common.h" > "$TMP/rt_kernel_common.h" 2>/dev/null || rm -f "$TMP/rt_kernel_common.h"
# the built-in definitions (rt_glsl.h) of that revision too: searched before the working tree's
mkdir -p "$TMP/include/rt"
git -C "$ROOT" show "$REV:include/rt/rt_glsl.h" > "$TMP/include/rt/rt_glsl.h"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -fPIC -Wno-unused-variable -Wno-unused-function"
INC="-I$TMP/include -I$ROOT/include -I$PKG/csrc -I$PKG/host"
/opt/rocm/bin/hipcc $FLAGS $INC -c -o "$TMP/k.o" "$TMP/rt_kernel.hip"
mkdir -p "$PKG/lib/prev"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$PKG/lib/prev/librtamd.so" "$TMP/k.o" "$PKG/build/obj/rt_capi.o"
rm -rf "$TMP"
echo "built $PKG/lib/prev/librtamd.so from $REV"
