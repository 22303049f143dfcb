#!/bin/bash
# tests given + rocprof of the FCOS bench, then one kernel's average: tools/gpu_kprof.sh <tag> <kernel substring> <pytest args>
set -o pipefail
TAG=$1; K=$2; shift 2
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest "$@" -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -20 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2>/dev/null || exit 1
grep -o '"value": [0-9.]*' gpurun_out/${TAG}_bench.json
grep "$K" gpurun_out/${TAG}_prof/prof_kernel_stats.csv | cut -c1-160
