#!/bin/bash
# same-box A/B of env settings on the default bench line: tools/ab_env.sh <tag> "<ENV=V ...>" ["<ENV=V ...>" ...]
# (an empty string = the default); each setting runs twice, alternating, 30 timed steps
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=$1; shift
for r in 1 2; do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 120 python -u bench.py --steps 30 --runs 1 --no-cpu-baseline > gpurun_out/${tag}_${i}_${r}.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/${tag}_${i}_${r}.json').read().strip().splitlines()[-1]); print('%-40s run $r: %.1f img/s' % ('$e' or 'default', d['value']))"
  done
done
