#!/bin/bash
# Interleaved whole-step A/B of an env switch: bash tools/ab_env.sh <VAR> <valueA> <valueB> [rounds]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
V=$1; A=$2; B=$3; N=${4:-2}
for i in $(seq $N); do
  for val in $A $B; do
    env $V=$val timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$V=$val', d['value'], 'img/s', d['ms_per_step'], 'ms', d['roofline']['achieved'], 'TF', d['roofline']['kernel'][:40])"
  done
done
