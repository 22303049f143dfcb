#!/bin/bash
# The measurement build of the library (make MEASURE=1: in-kernel stamps, ablation variants,
# cvl_debug_* exports, per-knob CVL_* tuning variables) into ab/libcvlite_measure.so.  The
# measurement tools (wgx_stamps.py, h64_stamps.py, stem_stamps.py, x32_*.py, p_*.py) load it via
# CVL_LIB; the product library (cvlite/libcvlite_hip.so) has none of that.
set -e
root=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$root/ab"
make -s -C "$root/cv-lite-object-detection_amd/csrc" -j8 MEASURE=1 BUILD=build_measure OUT="$root/ab/libcvlite_measure.so"
echo "built $root/ab/libcvlite_measure.so"
