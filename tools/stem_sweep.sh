#!/bin/bash
# stem kernel timings (tools/stem_probe.py); the round-4 rows-per-workgroup sweep ran it once per
# CVL_STEM_RPW_F / CVL_STEM_RPW_W setting (knobs since folded into constants, stem.hip RPW_F / RPW_W)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for cfg in "8 8"; do
  set -- $cfg
  CVL_STEM_RPW_F=$1 CVL_STEM_RPW_W=$2 timeout -k 10 60 python -u tools/stem_probe.py >> gpurun_out/stem_sweep.txt 2>&1 || exit 1
done
cat gpurun_out/stem_sweep.txt
