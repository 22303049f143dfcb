#!/bin/bash
# LDS operand-staging rates on the GPU: LDS-DMA (mode 0) vs global->VGPR->ds_write (mode 1), L2-resident
# (8 MiB) and HBM-streamed (1 GiB) sources, 256 workgroups (one per CU): tools/ubench_ldsdma.sh <out>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=${1:-gpurun_out/ubench_ldsdma.txt}
: > "$out"
for f in 8 1024; do
  for m in 0 1; do
    timeout -k 10 60 ./tools/ubench_ldsdma $m 256 $f 1000 >> "$out" 2>&1 || exit $?
  done
done
cat "$out"
