#!/bin/bash
# Where do the LDS-DMA conv loops spend their load segments?  Stamped weight-gradient phases under
# CVL_WGX_ABLATE = 0 (as built), 2 (DMA issued, out-of-range: no memory traffic), 4 (an L2-hot
# 256 KiB source window), 8 (no x traffic); the tower X32 under CVL_X_ABLATE = 0, 1 (no A traffic),
# 2 (no B traffic), 3 (neither), 32 (no DMA instructions).  Measurement library (tools/build_measure.sh).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=${1:-pm}
for ab in 0 2 4 8; do
  CVL_WGX_ABLATE=$ab timeout -k 10 120 python -u tools/wgx_stamps.py > gpurun_out/${tag}_wgx_ab$ab.md 2> gpurun_out/${tag}_wgx_ab$ab.err || exit 1
  echo "== wgx ablate $ab"; grep "1x1 1024->256 @ 32x32\|3x3 256->256 @ 64x64 +9" gpurun_out/${tag}_wgx_ab$ab.md
done
timeout -k 10 150 python -u tools/x32_probe.py 0 1 2 3 32 > gpurun_out/${tag}_x32.txt 2>&1 || exit 1
cat gpurun_out/${tag}_x32.txt
