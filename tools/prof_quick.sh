#!/bin/bash
# kernel stats of a short bench run: tools/prof_quick.sh <tag> [ENV=..]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=$1; shift
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/pq_$tag -o p -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/pq_$tag.json 2> gpurun_out/pq_$tag.err || { tail -5 gpurun_out/pq_$tag.err; exit 1; }
