#!/bin/bash
# Run a command with raytracing-book_amd/lib/librtamd_$1.so in place of librtamd.so,
# then put the working tree's library back:  tools/ab_swap.sh prev python tools/ab_variants.py ...
tag=$1; shift
lib=$(cd "$(dirname "$0")/.." && pwd)/raytracing-book_amd/lib
cp "$lib/librtamd.so" "$lib/librtamd_cur.so"
cp "$lib/librtamd_$tag.so" "$lib/librtamd.so"
"$@"; rc=$?
cp "$lib/librtamd_cur.so" "$lib/librtamd.so"
exit $rc
