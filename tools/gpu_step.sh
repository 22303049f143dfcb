#!/bin/bash
# full -m gpu suite + default bench (no CPU baseline) + per-launch conv table.  usage: gpu_step.sh <tag>
set -o pipefail
TAG=${1:-step}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/${TAG}_pytest.log | head -20; exit $rc; fi
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print('img/s', d['value'], 'ms', d['ms_per_step'], 'tower frac', d['roofline']['frac'], 'bb3', d['roofline']['backbone_3x3']['frac'])"
timeout -k 10 300 python3 -u tools/conv_table.py --out gpurun_out/${TAG}_conv_table.md > gpurun_out/${TAG}_conv_table.log 2>&1 || exit 1
head -4 gpurun_out/${TAG}_conv_table.md
