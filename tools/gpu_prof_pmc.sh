#!/bin/bash
# rocprofv3 kernel-stats profile of a short bench run + the PMC traffic passes of the bench's
# dominant kernel.  usage: bash tools/gpu_prof_pmc.sh <tag>
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err || { tail -30 gpurun_out/${TAG}_prof.err; exit 1; }
cut -c1-200 gpurun_out/${TAG}_prof_bench.json
bash tools/pmc_tower.sh
