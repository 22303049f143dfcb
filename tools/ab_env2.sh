#!/bin/bash
# A/B of one env setting on the FCOS and CenterNet bench lines: tools/ab_env2.sh VAR=VALUE
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in ${AB_MODELS:-centernet fcos}; do
  for i in 1 2; do
    a=$(timeout -k 10 300 python -u bench.py --model $m --no-cpu-baseline --steps 30 2>/dev/null | grep -o '"value": [0-9.]*') || exit 1
    b=$(env "$@" timeout -k 10 300 python -u bench.py --model $m --no-cpu-baseline --steps 30 2>/dev/null | grep -o '"value": [0-9.]*') || exit 1
    echo "$m base $a | $* $b"
  done
done
