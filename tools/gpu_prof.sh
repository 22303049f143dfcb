#!/bin/bash
# rocprofv3 kernel-trace stats of one bench configuration: bash tools/gpu_prof.sh <tag> <bench args...>
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py --no-cpu-baseline "$@" > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err || { tail -30 gpurun_out/${TAG}_prof.err; exit 1; }
cat gpurun_out/${TAG}_prof_bench.json
