#!/bin/bash
# A/B of environment settings on the default bench (no CPU baseline), alternating, 2 rounds.
# usage: bash tools/bench_ab.sh "" "CVL_X=1" ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for rep in 1 2; do
  for st in "$@"; do
    env $st timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print('rep $rep %-40s %.1f img/s %.3f ms' % (sys.argv[1], d['value'], d['ms_per_step']))" "$st"
  done
done
