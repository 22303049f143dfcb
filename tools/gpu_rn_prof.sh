#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/rn_prof -o prof -- python3 bench.py --model retinanet --steps 10 --warmup 3 > gpurun_out/rn.json 2> gpurun_out/rn.err || { tail -20 gpurun_out/rn.err; exit 1; }
cat gpurun_out/rn.json
