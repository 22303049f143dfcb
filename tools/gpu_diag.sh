#!/bin/bash
# Diagnostics pass: backbone 3x3 PMC (tools/pmc_bb3.sh), per-launch conv and non-conv tables of one
# FCOS step.  usage: bash tools/gpu_diag.sh <tag>
set -o pipefail
TAG=${1:-diag}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/conv_table.py --out gpurun_out/${TAG}_conv_table.md > gpurun_out/${TAG}_conv_table.log 2>&1 || { tail -20 gpurun_out/${TAG}_conv_table.log; exit 1; }
head -12 gpurun_out/${TAG}_conv_table.md
timeout -k 10 300 python3 -u tools/op_table.py --out gpurun_out/${TAG}_op_table.md > gpurun_out/${TAG}_op_table.log 2>&1 || { tail -20 gpurun_out/${TAG}_op_table.log; exit 1; }
head -8 gpurun_out/${TAG}_op_table.md
bash tools/pmc_bb3.sh ${TAG}
