#!/bin/bash
# rocprofv3 kernel-stats profile of the FCOS bench step.  usage: bash tools/gpu_prof2.sh <tag> [bench args]
set -o pipefail
TAG=${1:-prof}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err || { tail -30 gpurun_out/${TAG}_prof.err; exit 1; }
cat gpurun_out/${TAG}_prof_bench.json
