#!/bin/bash
# Build librtamd.so of git revision $1 into raytracing-book_amd/lib/librtamd_$2.so
# (A/B against the working tree: tools/ab_swap.sh swaps it in for one run).
set -e
rev=$1; tag=$2
repo=$(cd "$(dirname "$0")/.." && pwd)
wt=$(mktemp -d /tmp/rtwt.XXXX)
git -C "$repo" worktree add -q --detach "$wt" "$rev"
make -C "$wt/raytracing-book_amd" -j8 "$wt/raytracing-book_amd/lib/librtamd.so" >/dev/null
cp "$wt/raytracing-book_amd/lib/librtamd.so" "$repo/raytracing-book_amd/lib/librtamd_$tag.so"
git -C "$repo" worktree remove --force "$wt"
echo "built $rev -> raytracing-book_amd/lib/librtamd_$tag.so"
