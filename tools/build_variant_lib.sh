#!/bin/bash
# Builds raytracing-book_amd/lib/<tag>/librtamd.so from the working tree's kernel source with extra
# compiler definitions (ablations and A/B forms, e.g. -DRT_ABL_UNITVEC1) and the working tree's
# C ABI object, for tools/lib_ab.py.  usage: tools/build_variant_lib.sh <tag> <-Dflags...>
set -e
TAG=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/raytracing-book_amd
TMP=$(mktemp -d)
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -fPIC -Wno-unused-variable -Wno-unused-function"
INC="-I$ROOT/include -I$PKG/csrc -I$PKG/host"
/opt/rocm/bin/hipcc $FLAGS $INC "$@" -c -o "$TMP/k.o" "$PKG/csrc/rt_kernel.hip"
mkdir -p "$PKG/lib/$TAG"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$PKG/lib/$TAG/librtamd.so" "$TMP/k.o" "$PKG/build/obj/rt_capi.o"
rm -rf "$TMP"
echo "built $PKG/lib/$TAG/librtamd.so with $*"
