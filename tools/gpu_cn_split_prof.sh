#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/cnsplit_prof -o prof -- python3 bench.py --model centernet --steps 10 --warmup 3 > gpurun_out/cnsplit.json 2> gpurun_out/cnsplit.err || { tail -20 gpurun_out/cnsplit.err; exit 1; }
cat gpurun_out/cnsplit.json
