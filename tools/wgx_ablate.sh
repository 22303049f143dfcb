#!/bin/bash
# What bounds the 2-D weight-gradient loop: stamped loops (measurement build) under CVL_WGX_ABLATE
# bits (1 no fragment reads, 2 DMA out of range: no memory traffic, 16 no MFMAs, combinations).
# usage: tools/wgx_ablate.sh <tag> [bits...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=${1:-wa}; shift
for ab in ${*:-0 1 2 16 3 17 18 19}; do
  CVL_WGX_ABLATE=$ab timeout -k 10 120 python -u tools/wgx_stamps.py > gpurun_out/${tag}_wgx_ab$ab.md 2> gpurun_out/${tag}_wgx_ab$ab.err || exit 1
  echo "== wgx ablate $ab"; grep "1x1 1024->256 @ 32x32\|1x1 64->256 @ 128x128\|3x3 256->256 @ 64x64 +9" gpurun_out/${tag}_wgx_ab$ab.md
done
