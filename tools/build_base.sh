#!/bin/bash
# Build the library of another git revision into ab/libcvlite_<tag>.so for a same-box A/B
# (CVL_LIB=ab/libcvlite_<tag>.so selects it; ab/ is git-ignored and travels with gpurun).
# usage: tools/build_base.sh <rev> [tag]
set -e
rev=${1:-HEAD~1}; tag=${2:-base}
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" cv-lite-object-detection_amd/csrc include | tar -x -C "$tmp"
mkdir -p "$root/ab"
make -s -C "$tmp/cv-lite-object-detection_amd/csrc" -j8 OUT="$root/ab/libcvlite_$tag.so"
rm -rf "$tmp"
echo "built $root/ab/libcvlite_$tag.so from $rev"
