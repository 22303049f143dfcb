#!/bin/bash
# A/B of the fused BN-backward first pass: bench (no CPU baseline) twice each, interleaved
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  CVL_NO_BNSUM_FUSE=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > gpurun_out/ab_off_$i.json 2>/dev/null || exit 1
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > gpurun_out/ab_on_$i.json 2>/dev/null || exit 1
  echo "off $(grep -o '"value": [0-9.]*' gpurun_out/ab_off_$i.json) on $(grep -o '"value": [0-9.]*' gpurun_out/ab_on_$i.json)"
done
