#!/bin/bash
# Whole-step A/B of env settings over the three detector benches (FCOS headline, CenterNet, RetinaNet).
# usage: bash tools/ab_models.sh "<envA>" "<envB>" [rounds]   (env strings like "X=1 Y=2", or "-")
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A=$1; B=$2; N=${3:-1}
for i in $(seq $N); do
  for m in fcos centernet retinanet; do
    for E in "$A" "$B"; do
      [ "$E" = "-" ] && EV="" || EV="$E"
      env $EV timeout -k 10 200 python3 bench.py --model $m --no-cpu-baseline > gpurun_out/abm.json 2> gpurun_out/abm.err || { tail -5 gpurun_out/abm.err; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/abm.json')); print('$m', '[$E]', d['value'], 'img/s', d['ms_per_step'], 'ms')"
    done
  done
done
