#!/bin/bash
# conv_table.py wgrad rows under several wgrad_x planner settings: tools/wgx_sweep.sh "ENV=.." ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for st in "" "$@"; do
  echo "== $st"
  env $st timeout -k 10 200 python3 tools/conv_table.py --iters 10 --out gpurun_out/wgx.md > /dev/null 2> gpurun_out/wgx.err || { tail -5 gpurun_out/wgx.err; exit 1; }
  grep "wgrad" gpurun_out/wgx.md | head -24 | awk -F'|' '{printf "%-46s %-22s %6s\n", $3, $4, $6}'
done
