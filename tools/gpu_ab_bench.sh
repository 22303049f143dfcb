#!/bin/bash
# bench A/B in one box session: default vs CVL_CONV_NO_256=1 (interleaved, 2 rounds each)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_def_$r.json 2>/dev/null || exit 1
  CVL_CONV_NO_256=1 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_no256_$r.json 2>/dev/null || exit 1
done
for f in gpurun_out/ab_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['roofline']['achieved'])"; done
