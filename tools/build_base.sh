#!/bin/bash
# build the library of a git revision (default HEAD) into ab/libcvlite_<name>.so for same-box A/B
# runs (CVL_LIB=ab/libcvlite_<name>.so): tools/build_base.sh <name> [rev]
set -e
name=${1:-base}; rev=${2:-HEAD}
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" worktree add -q --detach "$tmp" "$rev"
make -s -C "$tmp/cv-lite-object-detection_amd/csrc" -j8 OUT="$root/ab/libcvlite_$name.so"
git -C "$root" worktree remove --force "$tmp"
mkdir -p "$root/ab"; ls -la "$root/ab/libcvlite_$name.so"
