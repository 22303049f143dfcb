#!/bin/bash
# side bench lines (configs[3] CenterNet hourglass, configs[4] RetinaNet) + the smoke test: tools/gpu_side_bench.sh <tag>
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 bench.py --model centernet --steps 20 --warmup 5 > gpurun_out/${TAG}_cn.json 2> gpurun_out/${TAG}_cn.err || { tail -30 gpurun_out/${TAG}_cn.err; exit 1; }
cat gpurun_out/${TAG}_cn.json
timeout -k 10 300 python3 bench.py --model retinanet --steps 20 --warmup 5 > gpurun_out/${TAG}_rn.json 2> gpurun_out/${TAG}_rn.err || { tail -30 gpurun_out/${TAG}_rn.err; exit 1; }
cat gpurun_out/${TAG}_rn.json
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -30 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -3 gpurun_out/${TAG}_smoke.log
