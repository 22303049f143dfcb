#!/bin/bash
# Whole-step A/B of the conv dispatch knobs (cvl_env_* in csrc), interleaved over 2 rounds.
set -o pipefail
mkdir -p gpurun_out
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/kn_${tag}_$r.json 2>gpurun_out/kn_${tag}_$r.err || { tail -5 gpurun_out/kn_${tag}_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/kn_${tag}_$r.json')); print('$tag', $r, d['value'], d['roofline']['achieved'])"
}
for r in 1 2; do
  run def X=0
  if [ -n "$SWEEP_TILES" ]; then
    for t in $SWEEP_TILES; do run lmin$t CVL_CONV_L_MIN_TILES=$t; done
  fi
  for v in ${SWEEP_KSPLIT:-}; do   # entries MAXTILES:TARGET
    run ks_${v/:/_} CVL_KSPLIT_MAX_TILES=${v%%:*} CVL_KSPLIT_TARGET=${v##*:}
  done
  for v in ${SWEEP_ENV:-}; do run ${v%%=*} $v; done
done
