#!/bin/bash
# kernel trace of conv_table.py under a planner setting: tools/wgx_prof.sh <tag> [ENV=..]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=$1; shift
env "$@" timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d gpurun_out/wgx_$tag -o p -- python3 tools/conv_table.py --iters 5 --out gpurun_out/wgx_$tag.md > /dev/null 2> gpurun_out/wgx_$tag.err || { tail -5 gpurun_out/wgx_$tag.err; exit 1; }
